/*
 * helpers_eval.h -- the device-only sample-stream and exact-correlator
 * helpers of dsp.h / analysis.h, one selected by `mode`, on a lane's private
 * int16 array, for their self-test (engine.hip k_helpers_eval,
 * melpe_helpers_eval_dev; tests/test_device_helpers.py checks the device
 * build and the host build against plain integer arithmetic).
 *
 * These are the parts of the codec whose gfx950 form differs from the host
 * form (v_perm_b32, v_alignbit, v_dot2_i32_i16, packed shifts) and whose
 * behaviour depends on the per-lane alignment of the stream start: buf + a
 * and buf + b may start on any int16.
 *
 * modes (o = the lane's output row):
 *   0  P16 stream of buf[a .. a+len): o[j] = sample j
 *   1  PairStream pairs of buf[a .. a+len) through ps_head<4> / ps_pairs4:
 *      o[2m], o[2m+1] = lo, hi of pair m, m < ceil(len / 2)
 *   2  P16C chunks from pair 1 (p16c_open / p16c_next4): pairs 1 .. 4G, G =
 *      ps_full_groups(s, 1), written as in mode 1; o[2] .. o[8G+1]
 *   3  xcorr_pairs<8, FpLags<8>, false>   (find_pitch's lag block), 8 sums
 *   4  xcorr_pairs<8, CpLags, true>        (corPeak's block, hi8/lo8 split)
 *   5  xcorr_pairs<11, FcLags11, true>     (frac_cor's eleven lags)
 *   6  xcorr_pairs<12, FpLags<12>, false>  (find_pitch's +-5 pass)
 *   7  fp_sums9                            (frac_pch's nine sums)
 *   8  sdot2 / sdot2_sat / pair_mid / pk_hi8 / pk_lo8 / perm_b32 (byte
 *      selects 0..7, as the codec uses it) of the dwords at buf + a,
 *      buf + b (a, b even) and c = len: o[0..5]
 */
#ifndef MELPE_HELPERS_EVAL_H
#define MELPE_HELPERS_EVAL_H

#include "codec.h"

namespace mlp {

#define HE_N 464	/* int16 per lane */
#define HE_OUT 512	/* int32 outputs per lane */

MD void he_pairs_out(int32_t *o, int m, uint32_t x)
{
	o[2 * m] = lo16(x);
	o[2 * m + 1] = hi16(x);
}

MD void he_eval(int mode, const int16_t *buf, int a, int b, int len, int32_t *o)
{
	const int16_t *pa = buf + a, *pb = buf + b;
	switch (mode) {
	case 0: {
		P16 r;
		int np = p16_open(r, pa, len), j = 0;
		for (int k = 0; k < np; k++, j += 2) {
			uint32_t x = p16_next(r);
			o[j] = lo16(x);
			o[j + 1] = hi16(x);
		}
		for (; j < len; j++)
			o[j] = pa[j];
		break;
	}
	case 1: {
		PairStream s;
		ps_open(s, pa, len);
		const int M = (len + 1) / 2;
		uint32_t h[4];
		ps_head<4>(s, h);
		for (int m = 0; m < 4 && m < M; m++)
			he_pairs_out(o, m, h[m]);
		for (int m0 = 4; m0 < M; m0 += 4) {
			uint32_t x[4];
			ps_pairs4(s, m0, x);
			for (int i = 0; i < 4 && m0 + i < M; i++)
				he_pairs_out(o, m0 + i, x[i]);
		}
		break;
	}
	case 2: {
		PairStream s;
		ps_open(s, pa, len);
		const int G = ps_full_groups(s, 1);
		if (G > 0) {
			P16C<MELPE_XC_PD> c;
			p16c_open(c, s, 1, G);
			for (int g = 0; g < G; g++) {
				uint32_t x[4];
				p16c_next4(c, x);
				for (int i = 0; i < 4; i++)
					he_pairs_out(o, 1 + 4 * g + i, x[i]);
			}
		}
		break;
	}
	case 3:
		xcorr_pairs<8, FpLags<8>, false>(pa, pb, len, o);
		break;
	case 4:
		xcorr_pairs<8, CpLags, true>(pa, pb, len, o);
		break;
	case 5:
		xcorr_pairs<11, FcLags11, true>(pa, pb, len, o);
		break;
	case 6:
		xcorr_pairs<12, FpLags<12>, false>(pa, pb, len, o);
		break;
	case 7:
		fp_sums9(pa, pb, len, o);
		break;
	default: {
		const u32_alias *wa = reinterpret_cast<const u32_alias *>(pa);
		const u32_alias *wb = reinterpret_cast<const u32_alias *>(pb);
		uint32_t x = wa[0], y = wb[0];
		o[0] = sdot2(x, y, len);
		o[1] = sdot2_sat(x, y, len);
		o[2] = (int32_t) pair_mid(x, y);
		o[3] = (int32_t) pk_hi8(x);
		o[4] = (int32_t) pk_lo8(x);
		o[5] = (int32_t) perm_b32(x, y, (uint32_t) len & 0x07070707u);	/* byte selects only */
		break;
	}
	}
}

}  // namespace mlp

#endif
