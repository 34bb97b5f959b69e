/*
 * npp_wave.h -- the noise pre-processor with one WAVEFRONT per channel
 * (device code only; k_npp.hip).
 *
 * Same algorithm and arithmetic as npp.h (melpe/npp.c), laid out for a
 * 64-lane wave instead of one lane:
 *  - the channel's NppState and all frame scratch live in LDS (NppWave,
 *    ~19 KB per wave), loaded from / stored to the channel's HBM record once
 *    per launch with coalesced dword copies;
 *  - every per-bin loop of the reference (129 bins) runs bin i on lane
 *    i % 64, through the very same per-bin functions npp.h's scalar loops
 *    call (npp_*_bin), so both builds share one arithmetic definition;
 *  - the 256-point complex FFT (melpe/fft_lib.c:115 cfft) runs its 128
 *    butterflies per stage across the lanes; the per-stage block-floating-
 *    point guard (max |x| over the block) is a wave max reduction;
 *  - sums over bins are wave reductions.  Each one is a sum the reference
 *    accumulates with saturating L_add, and each is proved saturation-free
 *    where it is defined (npp_spec_term, npp_bias_scalars, wv_enh_init), so
 *    the reduction order cannot change the result;
 *  - the two cross-bin scans whose order matters (the gain average with its
 *    running block-floating-point rescale, npp.c:1361-1389, and the
 *    comp_data_shift arg-max, :1391-1399): the average as an exact
 *    fixed-point sum over a prefix max of the exponents, the arg-max as a
 *    scan in reference order over the few bins that can win (wv_gain_scan).
 * Scalars of the state are computed redundantly by all lanes and written by
 * all lanes with identical values.  wsync() (the wave's own LDS ordering)
 * separates phases whose LDS data crosses lanes.
 */
#ifndef MELPE_NPP_WAVE_H
#define MELPE_NPP_WAVE_H

#include "npp.h"

namespace mlp {
namespace wv {

#define WV 64
#define LANE_LOOP(i, n) for (int i = lane; i < (n); i += WV)
/* the lane's bins i = lane + 64 t, t = 0..2, unrolled: per-bin values that
 * only the owning lane reads back can live in registers indexed by t */
#define BIN_LOOP(t, i) \
	_Pragma("unroll") for (int t = 0, i = lane; t < 3; t++, i += WV) if (i < NPP_NB)

/* The per-bin loops over the 129 bins: bin i on lane i % 64, three passes
 * unrolled (t = 0, 1, 2), the third on lane 0 alone.  Measured against
 * running bin 128 in wave-uniform control flow (its values on the scalar
 * unit, every lane taking part): 11.0 vs 11.2 ms per k_enc_npp launch at
 * 262,144 channels (profiles/r04_c_npp_*.json) -- the third vector pass
 * costs no more than the scalar code, so the simpler form stays. */
#define BIN_PASSES(t, i, ...) \
	_Pragma("unroll") for (int t = 0, i = lane; t < 3; t++, i += WV) if (i < NPP_NB) { \
		__VA_ARGS__ \
	}
__device__ __forceinline__ void wsync()
{
#if defined(MELPE_NPP_WG_WAVES) && MELPE_NPP_WG_WAVES > 1
	/* several channels' waves per workgroup, each on its own LDS image: the
	 * LDS serves one wave's instructions in order, so the wave's own
	 * accesses need only be kept in program order by the compiler */
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#else
	__syncthreads();
#endif
}

/* wave reductions, result uniform in every lane: DPP within each row of 16
 * lanes (quad swaps, half-row and row mirrors), then the four row results
 * combined through v_readlane (no LDS round trip).  All 64 lanes must be
 * active (callers sit in uniform control flow). */
#define DPP_QUAD_1032 0xB1
#define DPP_QUAD_2301 0x4E
#define DPP_ROW_HALF_MIRROR 0x141
#define DPP_ROW_MIRROR 0x140
template <int CTRL> __device__ __forceinline__ int dppmov(int v)
{
	return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}

__device__ __forceinline__ int wmax(int v)
{
	v = max(v, dppmov<DPP_QUAD_1032>(v));
	v = max(v, dppmov<DPP_QUAD_2301>(v));
	v = max(v, dppmov<DPP_ROW_HALF_MIRROR>(v));
	v = max(v, dppmov<DPP_ROW_MIRROR>(v));
	int a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
	int c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
	return max(max(a, b), max(c, d));
}

__device__ __forceinline__ int wsum(int v)
{
	v += dppmov<DPP_QUAD_1032>(v);
	v += dppmov<DPP_QUAD_2301>(v);
	v += dppmov<DPP_ROW_HALF_MIRROR>(v);
	v += dppmov<DPP_ROW_MIRROR>(v);
	return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
	       __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}

/* inclusive prefix max over the lanes (lane l gets the max of lanes 0..l):
 * row_shr 1, 2, 4, 8 inside each row of 16 lanes (max is idempotent, so
 * the overlapping windows are harmless), then row_bcast:15 (the end of rows
 * 0 and 2 into rows 1 and 3) and row_bcast:31 (the end of row 1 into rows 2
 * and 3).  Lanes without a source keep `old` = the identity. */
#define DPP_ROW_SHR(n) (0x110 + (n))
#define DPP_ROW_BCAST15 0x142
#define DPP_ROW_BCAST31 0x143
template <int CTRL, int RM> __device__ __forceinline__ int dpp_or(int old, int v)
{
	return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, 0xF, false);
}

__device__ __forceinline__ int wscan_max(int v)
{
	v = max(v, dpp_or<DPP_ROW_SHR(1), 0xF>(INT32_MIN, v));
	v = max(v, dpp_or<DPP_ROW_SHR(2), 0xF>(INT32_MIN, v));
	v = max(v, dpp_or<DPP_ROW_SHR(4), 0xF>(INT32_MIN, v));
	v = max(v, dpp_or<DPP_ROW_SHR(8), 0xF>(INT32_MIN, v));
	v = max(v, dpp_or<DPP_ROW_BCAST15, 0xA>(INT32_MIN, v));
	v = max(v, dpp_or<DPP_ROW_BCAST31, 0xC>(INT32_MIN, v));
	return v;
}

/* the same for floats (as bit patterns; -inf is the identity) */
__device__ __forceinline__ float wscan_maxf(float f)
{
	const int ni = (int) 0xff800000u;
	int v = __float_as_int(f);
	v = __float_as_int(fmaxf(__int_as_float(v), __int_as_float(dpp_or<DPP_ROW_SHR(1), 0xF>(ni, v))));
	v = __float_as_int(fmaxf(__int_as_float(v), __int_as_float(dpp_or<DPP_ROW_SHR(2), 0xF>(ni, v))));
	v = __float_as_int(fmaxf(__int_as_float(v), __int_as_float(dpp_or<DPP_ROW_SHR(4), 0xF>(ni, v))));
	v = __float_as_int(fmaxf(__int_as_float(v), __int_as_float(dpp_or<DPP_ROW_SHR(8), 0xF>(ni, v))));
	v = __float_as_int(fmaxf(__int_as_float(v), __int_as_float(dpp_or<DPP_ROW_BCAST15, 0xA>(ni, v))));
	v = __float_as_int(fmaxf(__int_as_float(v), __int_as_float(dpp_or<DPP_ROW_BCAST31, 0xC>(ni, v))));
	return __int_as_float(v);
}

/* value of bin i (0..128) held one bin per lane in r0 (bins 0..63), r1
 * (64..127), r2 (128, uniform) -- uniform i */
__device__ __forceinline__ int bin_at(int r0, int r1, int r2, int i)
{
	return i < 64 ? __builtin_amdgcn_readlane(r0, i)
		      : (i < 128 ? __builtin_amdgcn_readlane(r1, i - 64) : r2);
}

/* LDS image of one channel's NPP */
struct NppWave {
	union {
		NppScratchW w;	/* YY.., ybuf */
		/* wv_enh_init's temp_yy (the scratch is dead there); may_alias
		 * dwords, like the record copies */
		u32_alias ty_init[NPP_WIN + 2];
	};
	/* the channel's NppState up to its min-statistics memory (NPP_HOT_BYTES);
	 * that memory stays in the HBM record (the `m` view below) */
	u32_alias s_hot[NPP_HOT_BYTES / 4];	/* an NppState image, read as fields */
	int16_t GainD[NPP_NB];
	int16_t gk[NPP_NB], gks[NPP_NB];
	/* analysis frame / initial noise frame, then the synthesis frame (the
	 * analysis frame is dead once the forward FFT's input is built) */
	int16_t buf[NPP_WIN];
};

/* per-lane constants of the FFT and the analysis window, loaded once per
 * kernel: the twiddles of the lane's two butterflies in each of the six
 * twiddled stages (packed wr | wi << 16), and win[lane + 64 t] */
/* the LDS image as an NppState: only fields before NPP_HOT_BYTES are
 * touched through it */
MD NppState *wv_S(NppWave *W)
{
	return (NppState *) W->s_hot;
}

struct WvConst {
	int tw[6][2];
	int16_t win[4];
};

MD void wv_const_init(WvConst *k, int lane)
{
	const int16_t *wrt = g_der.wr, *wit = g_der.wi;
	int istep_idx = 128, st = 0;
	for (int mmax = 8; mmax < 512; mmax *= 2, st++) {
		istep_idx >>= 1;
		int half = mmax / 2;
		for (int t = 0; t < 2; t++) {
			int kk = (lane + WV * t) % half;
			int wr = SW_MAX_, wi = 0;
			if (kk) {
				wr = wrt[kk * istep_idx];
				wi = wit[kk * istep_idx];
			}
			k->tw[st][t] = (wr & 0xffff) | (wi << 16);
		}
	}
	const int16_t *win = TB(sqrt_tukey_256_180);
	for (int t = 0; t < 4; t++)
		k->win[t] = win[lane + WV * t];
}

/* cfft :115 for nn = 256 complex points (512 shorts) in LDS; returns the
 * number of halvings (dsp.h cfft: same stages, same guard scaling).  Each
 * stage's guard shift is applied as the stage loads its inputs, and each
 * stage takes the max |x| of the values it writes for the next guard. */
MD Word16 wv_cfft256(int16_t *d0, const WvConst *kc, int lane)
{
	PROF_SCOPE(30);
	/* bit-reversal permutation of the complex points (the reference's swap
	 * loop): the pair (k, rev k) is swapped by the lane owning the smaller
	 * index, so every point is read by exactly one lane */
	int m = 0;
	for (int t = 0; t < 4; t++) {
		int k = lane + WV * t;
		int r = (int) (__brev((unsigned) k) >> 24);
		if (r >= k) {
			int16_t a0 = d0[2 * k], a1 = d0[2 * k + 1];
			int16_t b0 = d0[2 * r], b1 = d0[2 * r + 1];
			m = max(m, max(max((int) abs_s(a0), (int) abs_s(a1)),
				       max((int) abs_s(b0), (int) abs_s(b1))));
			if (r > k) {
				d0[2 * k] = b0;
				d0[2 * k + 1] = b1;
				d0[2 * r] = a0;
				d0[2 * r + 1] = a1;
			}
		}
	}
	Word16 g = 0;
	Word16 sc = 0;
	if (wmax(m) > 16383) {
		g += 1;
		sc = 1;
	}
	wsync();
	m = 0;
	for (int t = 0; t < 2; t++) {	/* span-1 butterflies, i = 0, 4, ... */
		int i = 4 * (lane + WV * t);
		Word16 pr = shr(d0[i], sc), qr = shr(d0[i + 2], sc);
		Word16 pi = shr(d0[i + 1], sc), qi = shr(d0[i + 3], sc);
		Word16 o0 = add(pr, qr), o2 = sub(pr, qr), o1 = add(pi, qi), o3 = sub(pi, qi);
		d0[i] = o0;
		d0[i + 2] = o2;
		d0[i + 1] = o1;
		d0[i + 3] = o3;
		m = max(m, max(max((int) abs_s(o0), (int) abs_s(o1)),
			       max((int) abs_s(o2), (int) abs_s(o3))));
	}
	sc = 0;
	if (wmax(m) > 16383) {
		g += 1;
		sc = 1;
	}
	wsync();
	{	/* span-2 butterflies (twiddles 1 and -j), i = 0, 8, ... */
		int i = 8 * lane;
		int16_t v[8];
		for (int k = 0; k < 8; k++)
			v[k] = shr(d0[i + k], sc);
		int16_t o[8];
		o[0] = add(v[0], v[4]);
		o[4] = sub(v[0], v[4]);
		o[1] = add(v[1], v[5]);
		o[5] = sub(v[1], v[5]);
		o[2] = add(v[2], v[7]);
		o[6] = sub(v[2], v[7]);
		o[3] = sub(v[3], v[6]);
		o[7] = add(v[3], v[6]);
		m = 0;
		for (int k = 0; k < 8; k++) {
			d0[i + k] = o[k];
			m = max(m, (int) abs_s(o[k]));
		}
	}
	int16_t *d = d0 - 1;	/* 1-based view, as the reference */
	int st = 0;
#pragma unroll
	for (int mmax = 8; mmax < 512; mmax *= 2, st++) {
		Word16 mx = (Word16) wmax(m);
		sc = 0;
		if (mx > 16383) {
			g += 2;
			sc = 2;
		} else if (mx > 8191) {
			g += 1;
			sc = 1;
		}
		wsync();
		int istep = 2 * mmax;
		int half = mmax / 2;	/* twiddles per block */
		m = 0;
		for (int t = 0; t < 2; t++) {
			int b = lane + WV * t;	/* 128 butterflies */
			int k = b % half, blk = b / half;
			int i = 1 + 2 * k + blk * istep;
			int jj = i + mmax;
			Word16 wr = (Word16) (kc->tw[st][t] & 0xffff);
			Word16 wi = (Word16) (kc->tw[st][t] >> 16);
			Word16 pr = shr(d[i], sc), qr = shr(d[jj], sc);
			Word16 pi = shr(d[i + 1], sc), qi = shr(d[jj + 1], sc);
			Word32 tr = L_add(L_mult(wr, qr), L_mult(wi, qi));
			tr = L_add(tr, L_shl(0x80, 8));
			tr = L_shl(L_shr(tr, 16), 16);
			Word32 ti = L_sub(L_mult(wi, qr), L_mult(wr, qi));
			ti = L_add(ti, L_shl(0x80, 8));
			ti = L_shl(L_shr(ti, 16), 16);
			Word16 o0 = extract_h(L_add(L_deposit_h(pr), tr));
			Word16 o1 = extract_h(L_sub(L_deposit_h(pr), tr));
			Word16 o2 = extract_h(L_sub(L_deposit_h(pi), ti));
			Word16 o3 = extract_h(L_add(L_deposit_h(pi), ti));
			d[i] = o0;
			d[jj] = o1;
			d[i + 1] = o2;
			d[jj + 1] = o3;
			m = max(m, max(max((int) abs_s(o0), (int) abs_s(o1)),
				       max((int) abs_s(o2), (int) abs_s(o3))));
		}
	}
	wsync();
	return g;
}

/* fft_npp :270 */
MD Word16 wv_fft_npp(int16_t *d, Word16 dir, const WvConst *kc, int lane)
{
	Word16 g = wv_cfft256(d, kc, lane);
	if (dir < 0) {
		for (int n = 1 + lane; n < 128; n += WV) {
			int16_t t = d[2 * n];
			d[2 * n] = d[2 * (256 - n)];
			d[2 * (256 - n)] = t;
			t = d[2 * n + 1];
			d[2 * n + 1] = d[2 * (256 - n) + 1];
			d[2 * (256 - n) + 1] = t;
		}
		wsync();
	}
	return g;
}

/* yb[256..511] := conjugate mirror of yb[2..255] (npp.c:1150-1155, 1600-1605) */
MD void wv_mirror(int16_t *yb, int lane)
{
	LANE_LOOP(i, NPP_WIN / 2 - 1) {
		yb[NPP_WIN + 2 * i + 2] = yb[NPP_WIN - 2 * i - 2];
		yb[NPP_WIN + 2 * i + 3] = negate(yb[NPP_WIN - 2 * i - 1]);
	}
	wsync();
}

/* minstat_init :1164 */
MD void wv_minstat_init(NppState *s, NppState *m, int lane)
{
	LANE_LOOP(i, NPP_NB) {
		Word16 sp = mult(s->lambdaD[i], NOISE_BIAS);
		Word16 ls = s->lambdaD_shift[i];
		s->smoothedspect[i] = sp;
		for (int k = 0; k < NPP_NMINWIN; k++) {
			m->circb[k][i] = sp;
			m->circb_shift[k][i] = ls;
		}
		s->sm_shift[i] = ls;
		s->act_min[i] = sp;
		s->act_min_shift[i] = ls;
		m->act_min_sub[i] = sp;
		m->act_min_sub_shift[i] = ls;
		s->noisespect[i] = sp;
		s->noise_shift[i] = ls;
		s->var_sp_av[i] = mult(sp, 20066);
		s->av_shift[i] = add(ls, 1);
		Word32 L = L_mult(sp, sp);
		Word16 sh = norm_l(L);
		s->var_sp_2[i] = extract_h(L_shl(L, sh));
		s->av2_shift[i] = sub(shl(ls, 1), sub(sh, 1));
	}
	s->alphacorr = 29491;
}

/* enh_init :1023 -- initial noise estimate; `noise` (256, LDS) is consumed */
MD void wv_enh_init(NppWave *W, int16_t *noise, const WvConst *kc, int lane, NppState *m)
{
	NppState *s = wv_S(W);
	int16_t *yb = W->w.ybuf;
	u32_alias *ty = W->ty_init;
	int mx = 0;
#pragma unroll
	LANE_LOOP(i, NPP_WIN) {
		noise[i] = mult(kc->win[i >> 6], noise[i]);
		mx = max(mx, (int) abs_s(noise[i]));
	}
	mx = max(1, wmax(mx));
	Word16 sh = norm_s((Word16) mx);
	Word16 ash = sub(15, sh);
	LANE_LOOP(i, NPP_WIN + 1) {
		yb[2 * i] = (i < NPP_WIN) ? shl(noise[i], sh) : (int16_t) 0;
		yb[2 * i + 1] = 0;
	}
	wsync();
	Word16 g = wv_fft_npp(yb, 1, kc, lane);
	int Lm = INT32_MIN;
	LANE_LOOP(p, NPP_NB) {
		int i = 2 * p;
		Word32 v;
		if (p == 0 || p == NPP_NB - 1)
			v = L_shr(L_mult(yb[i], yb[i]), 1);
		else
			v = L_shr(L_add(L_mult(yb[i], yb[i]), L_mult(yb[i + 1], yb[i + 1])), 1);
		ty[i] = (uint32_t) v;
		ty[i + 1] = 0;
		Lm = max(Lm, (int) v);
		if (p != NPP_NB - 1)
			Lm = max(Lm, 0);	/* ty[i + 1] = 0 is in the max's range */
	}
	Word32 L = wmax(Lm);
	wsync();
	sh = norm_l(L);
	LANE_LOOP(i, NPP_WIN + 1)
		yb[i] = extract_h(L_shl((Word32) ty[i], sh));
	sh = sub(shl(add(ash, g), 1), add(sh, 7));
	wsync();
	wv_mirror(yb, lane);
	g = wv_fft_npp(yb, -1, kc, lane);
	sh = add(sh, g);
	sh = sub(sh, 8);
	mx = 0;
	LANE_LOOP(i, NPP_WIN) {
		noise[i] = yb[2 * i];
		mx = max(mx, (int) abs_s(noise[i]));
	}
	mx = wmax(mx);
	Word16 t = norm_s((Word16) mx);
	sh = sub(sh, t);
	const int16_t *wf = TB(wtr_front);
	LANE_LOOP(i, NPP_WIN) {	/* shl + smoothing_win (npp.c:486) */
		Word16 v = shl(noise[i], t);
		if (i >= 1 && i < 32)
			v = mult(v, wf[i]);
		else if (i >= NPP_WIN - 32 + 1)
			v = mult(v, wf[NPP_WIN - i]);
		else if (i >= 32)
			v = 0;
		noise[i] = v;
	}
	wsync();
	LANE_LOOP(i, NPP_WIN + 1) {
		yb[2 * i] = (i < NPP_WIN) ? noise[i] : (int16_t) 0;
		yb[2 * i + 1] = 0;
	}
	wsync();
	g = wv_fft_npp(yb, 1, kc, lane);
	Word16 nsh = add(sh, g);
	/* the noise power sum: every term is non-negative (yb clamped at 0)
	 * and 127 * 2^23.5 + 2 * 2^22.5 < 2^31, so the reference's L_add chain
	 * never saturates */
	int part = 0;
	LANE_LOOP(p, NPP_NB) {
		Word16 y = yb[2 * p];
		if (y < 0)
			y = 0;
		Word32 Ld = L_add(L_shl(L_mult(181, y), 7), 2);
		Word16 ns = norm_l(Ld);
		s->lambdaD[p] = extract_h(L_shl(Ld, ns));
		s->lambdaD_shift[p] = add(nsh, sub(1, ns));
		part += (p == 0 || p == NPP_NB - 1) ? L_shr(Ld, 8) : L_shr(Ld, 7);
	}
	L = wsum(part);
	sh = norm_l(L);
	s->n_pwr = extract_h(L_shl(L, sh));
	s->n_pwr_shift = sub(add(nsh, 1), sh);
	s->SN_LT = divide_s(14648, s->n_pwr);
	s->SN_LT_shift = sub(22, s->n_pwr_shift);
	wv_minstat_init(s, m, lane);
	wsync();
}

/* The gamma average with its running rescale and the gamma arg-max
 * (npp.c:1361-1399) over gk / gks (129 bins, LDS).  gk = divide_s(..) is in
 * [0, 32767] and the shifts are small, so the reference's saturating ops
 * reduce to plain integer ones: the running sum is at most 129 * 2^22 <
 * 2^31, a left-shifted term at most 2^22 (shift <= 7), sub() of two shifts
 * cannot saturate.
 *
 * The average in parallel.  Let a_j be bin j's exponent as the sum sees it
 * (gks, one lower for bins 0 and 128) and M_j = max(a_0..a_j) the running
 * shift.  Bin j adds term_j = gk_j << (7 - t) or >> (t - 7), t = M_j - a_j,
 * and each rise of the running shift by D floors the sum to sum >> D.
 * Since floor(floor(x / 2^p) + y) / 2^q) = floor((x + y 2^p) / 2^(p+q)) for
 * an integer y, the reference's sum is exactly
 *     floor( sum_j term_j / 2^(M_128 - M_j) ),
 * the terms taken relative to the final shift.  With every M_128 - M_j <=
 * 32 that is an exact fixed-point sum with 32 fraction bits: integer parts
 * (< 2^30 in all) and the 32-bit fractions as two 16-bit halves.  M_j is a
 * prefix max across the lanes (wscan_max); a wave whose exponents spread
 * wider runs the reference's serial scan (wv_gain_scan_serial).
 *
 * The arg-max stays a scan in reference order (its comparison truncates
 * the smaller-exponent mantissa, which makes it order-dependent), but only
 * over the bins that can be taken.  In values v = gk 2^gks: a bin is taken
 * only if v exceeds the current champion c; the champion only rises; and
 * every earlier bin i left behind satisfied v_i < v_c + 2^max(e_i, e_c).
 * So bin j can be taken only if v_j > max(v_0..v_(j-1)) - 2^E_j, E_j the
 * largest exponent up to j.  The test runs in floats (gk has 15 bits, so
 * v is exact; the threshold's rounding error is below 2^(E_j - 9), and the
 * float test uses 2^(E_j + 1), so it keeps a superset); a wave whose
 * exponents leave the float range scans every bin. */
MD void wv_gain_scan_serial(const int16_t *gk, const int16_t *gks, int lane, int *acc_out, int *sh_out,
			    int *mn_out, int *ms_out, bool sum)
{
	int gk0 = gk[lane], gk1 = gk[lane + 64], gk2 = gk[NPP_NB - 1];
	int gs0 = gks[lane], gs1 = gks[lane + 64], gs2 = gks[NPP_NB - 1];
	int acc, sh2;		/* L, sh of the reference */
	int mn, ms;		/* gmax, gmaxs */
	{
		int g = __builtin_amdgcn_readlane(gk0, 0), e = __builtin_amdgcn_readlane(gs0, 0);
		acc = g << 7;
		sh2 = e - 1;
		mn = g;
		ms = e;
	}
	/* one bin: branch-free (selects), shift counts clamped to 31 where the
	 * reference's saturating shift would give 0 (operands are >= 0) */
	auto shc = [](int k) { return k < 0 ? 0 : (k > 31 ? 31 : k); };
	auto step = [&](int g, int e, int ee) {
		/* cmp_shift(gmax, gmaxs, g, e) < 0 for non-negative mantissas:
		 * the value with the smaller exponent truncated to the larger */
		int d = ms - e;
		int a1 = d > 0 ? mn : mn >> shc(-d);
		int b1 = d > 0 ? g >> shc(d) : g;
		bool take = a1 < b1;
		mn = take ? g : mn;
		ms = take ? e : ms;
		if (sum) {
			int t = sh2 - ee;
			int n = t - 7;	/* L_shr(gk, t - 7), no saturation for t >= 1 */
			int term = n >= 0 ? g >> shc(n) : g << shc(-n);
			int accb = (acc >> shc(-t)) + (g << 7);
			acc = t > 0 ? acc + term : accb;
			sh2 = t > 0 ? sh2 : ee;
		}
	};
	#pragma unroll 2
	for (int i = 1; i < 64; i++) {
		int e = __builtin_amdgcn_readlane(gs0, i);
		step(__builtin_amdgcn_readlane(gk0, i), e, e);
	}
	#pragma unroll 2
	for (int i = 0; i < 64; i++) {
		int e = __builtin_amdgcn_readlane(gs1, i);
		step(__builtin_amdgcn_readlane(gk1, i), e, e);
	}
	step(gk2, gs2, gs2 - 1);
	*acc_out = acc;
	*sh_out = sh2;
	*mn_out = mn;
	*ms_out = ms;
}

MD void wv_gain_scan(const int16_t *gk, const int16_t *gks, int lane, Word16 *gav, Word16 *gavs,
		     Word16 *gmax, Word16 *gmaxs)
{
	const int g0 = gk[lane], g1 = gk[lane + 64], g2 = gk[NPP_NB - 1];
	const int e0 = gks[lane], e1 = gks[lane + 64], e2 = gks[NPP_NB - 1];
	/* ---- the average ---- */
	const int a0 = lane == 0 ? e0 - 1 : e0, a2 = e2 - 1;
	const int M0 = wscan_max(a0);
	const int M1 = max(__builtin_amdgcn_readlane(M0, 63), wscan_max(e1));
	const int M2 = max(__builtin_amdgcn_readlane(M1, 63), a2);	/* the final shift */
	const int dmax = M2 - __builtin_amdgcn_readlane(a0, 0);
	int acc, sh2, mn, ms;
	bool serial_sum = dmax > 32;
	if (!serial_sum) {
		auto term = [](int g, int t) { return t >= 7 ? g >> (t - 7 > 31 ? 31 : t - 7) : g << (7 - t); };
		const int t0 = term(g0, M0 - a0), t1 = term(g1, M1 - e1), t2 = term(g2, M2 - a2);
		const int d0 = M2 - M0, d1 = M2 - M1;	/* 0 .. 32 */
		auto ip = [](int t, int d) { return d >= 32 ? 0 : t >> d; };
		auto fp = [](int t, int d) {
			return d == 0 ? 0u : (uint32_t) ((uint64_t) (uint32_t) t << (32 - d));
		};
		const uint32_t f0 = fp(t0, d0), f1 = fp(t1, d1);
		const int si = wsum(ip(t0, d0) + ip(t1, d1)) + t2;
		const int slo = wsum((int) ((f0 & 0xffffu) + (f1 & 0xffffu)));
		const int shi = wsum((int) ((f0 >> 16) + (f1 >> 16)));
		acc = si + ((shi + (slo >> 16)) >> 16);
		sh2 = M2;
	}
	/* ---- the arg-max over the bins that can be taken ---- */
	const int emx = max(wmax(max(e0, e1)), e2), emn = min(-wmax(-min(e0, e1)), e2);
	if (serial_sum || emx > 100 || emn < -100) {
		int a, s2;
		wv_gain_scan_serial(gk, gks, lane, &a, &s2, &mn, &ms, serial_sum);
		if (serial_sum) {
			acc = a;
			sh2 = s2;
		}
	} else {
		const float v0 = ldexpf((float) g0, e0), v1 = ldexpf((float) g1, e1), v2 = ldexpf((float) g2, e2);
		const int E0 = wscan_max(e0);
		const int E1 = max(__builtin_amdgcn_readlane(E0, 63), wscan_max(e1));
		const int E2 = max(__builtin_amdgcn_readlane(E1, 63), e2);
		const float I0 = wscan_maxf(v0);
		const float I1 = fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(I0), 63)), wscan_maxf(v1));
		const float I2 = fmaxf(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(I1), 63)), v2);
		const bool c0 = v0 > I0 - ldexpf(1.0f, E0 + 1) && lane != 0;
		const bool c1 = v1 > I1 - ldexpf(1.0f, E1 + 1);
		const bool c2 = v2 > I2 - ldexpf(1.0f, E2 + 1);
		uint64_t m0 = __ballot(c0), m1 = __ballot(c1);
		mn = __builtin_amdgcn_readlane(g0, 0);
		ms = __builtin_amdgcn_readlane(e0, 0);
		auto shc = [](int k) { return k < 0 ? 0 : (k > 31 ? 31 : k); };
		auto step = [&](int g, int e) {
			int d = ms - e;
			int x = d > 0 ? mn : mn >> shc(-d);
			int y = d > 0 ? g >> shc(d) : g;
			bool take = x < y;
			mn = take ? g : mn;
			ms = take ? e : ms;
		};
		while (m0) {
			const int k = __builtin_ctzll(m0);
			m0 &= m0 - 1;
			step(__builtin_amdgcn_readlane(g0, k), __builtin_amdgcn_readlane(e0, k));
		}
		while (m1) {
			const int k = __builtin_ctzll(m1);
			m1 &= m1 - 1;
			step(__builtin_amdgcn_readlane(g1, k), __builtin_amdgcn_readlane(e1, k));
		}
		if (c2)
			step(g2, e2);
	}
	Word32 L = acc;
	if (L == 0)
		L = 1;
	Word16 t1 = norm_l(L);
	*gav = extract_h(L_shl(L, t1));
	*gavs = add(sub((Word16) sh2, t1), 2);
	*gmax = (Word16) mn;
	*gmaxs = (Word16) ms;
}

/* process_frame :1212 -- one 256-sample analysis/synthesis frame; in and
 * out are 256-sample LDS buffers */
MD void wv_process_frame(NppWave *W, NppState *m, const int16_t *in, int16_t *out, const WvConst *kc,
			 int lane)
{
	PROF_SCOPE(34);
	NppState *s = wv_S(W);
	NppScratchW *w = &W->w;
	int16_t *yb = w->ybuf;
	int16_t *GainD = W->GainD, *gk = W->gk, *gks = W->gks;
	Word16 sh, t, t1, t2, t3, t4;
	Word32 L;

	if (!s->pf_started) {
		LANE_LOOP(i, NPP_NB) {
			s->agal[i] = 0;
			s->agal_shift[i] = 0;
			s->ksi[i] = GM_MIN;
			s->ksi_shift[i] = 0;
			s->qk[i] = ENH_QK_MAX;
			s->Gain[i] = GM_MIN;
		}
		s->YY_LT = 0;
		s->YY_LT_shift = 0;
		s->SN_LT0 = s->SN_LT;
		s->SN_LT0_shift = s->SN_LT_shift;
		s->pf_started = 1;
	}
	LANE_LOOP(i, NPP_NB)
		GainD[i] = GM_MIN;
	if (s->enh_i < 50)
		s->enh_i = (int16_t) (s->enh_i + 1);

	int16_t *analy = W->buf;
	Word16 g, Ysh, YYavs;
	{
	PROF_SCOPE(60);
	int mx = 0;
#pragma unroll
	LANE_LOOP(i, NPP_WIN) {
		analy[i] = mult(kc->win[i >> 6], in[i]);
		mx = max(mx, (int) abs_s(analy[i]));
	}
	mx = max(1, wmax(mx));
	sh = norm_s((Word16) mx);
	Word16 ash = sub(15, sh);
	LANE_LOOP(i, NPP_WIN + 1) {
		yb[2 * i] = (i < NPP_WIN) ? shl(analy[i], sh) : (int16_t) 0;
		yb[2 * i + 1] = 0;
	}
	wsync();
	g = wv_fft_npp(yb, 1, kc, lane);
	Ysh = add(ash, g);
	YYavs = shl(Ysh, 1);
	}
	int maxs = SW_MIN_;
	int part = 0;
	/* |Y| of the lane's bins lane + 64 t: read back only by the same lane,
	 * so it stays in registers (BIN_LOOP) */
	int16_t ymag[3] = {0, 0, 0}, ymag_sh[3] = {0, 0, 0};
	{
	PROF_SCOPE(53);
	BIN_PASSES(t, i, {
		Word32 v;
		if (i == 0)
			v = L_mult(yb[0], yb[0]);
		else if (i == NPP_NB - 1)
			v = L_mult(yb[NPP_WIN], yb[NPP_WIN]);
		else
			v = L_add(L_mult(yb[2 * i], yb[2 * i]), L_mult(yb[2 * i + 1], yb[2 * i + 1]));
		if (v < 1)
			v = 1;
		Word16 n = norm_l(v);
		w->YY[i] = extract_h(L_shl(v, n));
		w->YY_shift[i] = sub(YYavs, n);
		maxs = max(maxs, (int) w->YY_shift[i]);
	})
	maxs = wmax(maxs);
	BIN_PASSES(t, i, {
		Word16 y = w->YY[i], ys = w->YY_shift[i];
		if (ys & 1) {
			y = shr(y, 1);
			ys = add(ys, 1);
		}
		ymag[t] = sqrt_Q15(y);
		ymag_sh[t] = shr(ys, 1);
		w->YY_shift[i] = sub(w->YY_shift[i], 8);
		/* maxs is taken before the -8 (npp.c:1300-1330) */
		Word32 st = npp_spec_term(w->YY, w->YY_shift, (Word16) maxs, i);
		part += st;
	})
	L = wsum(part);
	}
	if (L == 0)
		L = 1;
	t1 = norm_l(L);
	Word16 YY_av = extract_h(L_shl(L, t1));
	Word16 YY_av_shift = sub(add((Word16) maxs, 1), t1);

	/* smoothed_periodogram :511 */
	{
	PROF_SCOPE(36);
	maxs = SW_MIN_;
	BIN_PASSES(t, i, { maxs = max(maxs, (int) s->sm_shift[i]); })
	maxs = wmax(maxs);
	part = 0;
	BIN_PASSES(t, i, {
		Word32 st = npp_spec_term(s->smoothedspect, s->sm_shift, (Word16) maxs, i);
		part += st;
	})
	L = wsum(part);
	Word16 amin;
	Word16 anum = npp_sm_period_scalars(s, (Word16) maxs, L, YY_av, YY_av_shift, &amin);
	part = 0;
	{
	PROF_SCOPE(54);
	BIN_PASSES(t, i, {
		int16_t ns2, ns2sh, av;	/* bin i's, this lane's only */
		npp_sm_period_bin(s, w, anum, amin, i, ns2, ns2sh, av);
		npp_bias1_bin(s, w, i, av, ns2, ns2sh);
		part += w->var_rel[i];
	})
	}
	Word32 vsum = wsum(part);
	wsync();
	Word16 f1, f2;
	Word16 vsq = npp_bias_scalars(s, w, vsum, &f1, &f2);
	Word16 slope = npp_noise_slope(s);
	{
	PROF_SCOPE(55);
	BIN_PASSES(t, i, {
		int16_t bsp, bsh, bsub, bsubsh;	/* bin i's, this lane's only */
		npp_bias2_bin(s, w, bsp, bsh, bsub, bsubsh, vsq, f1, f2, i);
		npp_min_search_bin(s, m, bsp, bsh, bsub, bsubsh, slope, i);
		gk[i] = divide_s(shr(w->YY[i], 1), s->lambdaD[i]);
		gks[i] = sub(add(w->YY_shift[i], 1), s->lambdaD_shift[i]);
	})
	}
	wsync();
	npp_min_search_post(s);
	}

	Word16 gav, gavs, gmax, gmaxs;
	{
	PROF_SCOPE(37);
	wv_gain_scan(gk, gks, lane, &gav, &gavs, &gmax, &gmaxs);
	}
	bool nflag = false;
	if (cmp_shift(gmax, gmaxs, 18102, 6) < 0 && cmp_shift(gav, gavs, 23170, 1) < 0) {
		nflag = true;
		t1 = mult(s->n_pwr, 23170);
		t2 = add(s->n_pwr_shift, 2);
		if (cmp_shift(YY_av, YY_av_shift, t1, t2) > 0)
			nflag = false;
	}

	{
	PROF_SCOPE(38);
	if (s->enh_i == 1) {
		BIN_LOOP(t, i) {
			Word32 v = L_mult(ymag[t], GM_MIN);
			Word16 n = norm_l(v);
			s->agal[i] = extract_h(L_shl(v, n));
			s->agal_shift[i] = sub(ymag_sh[t], n);
		}
	} else {
		{
		PROF_SCOPE(56);
		BIN_PASSES(t, i, { npp_ksi_bin(s, gk, gks, i); })
		}
		t1 = mult(29491, s->Ksi_min_var);
		t2 = mult(3277, npp_ksi_min_adapt(nflag, GM_MIN, s->SN_LT, s->SN_LT_shift));
		Word16 kmv = add(t1, t2);
		s->Ksi_min_var = kmv;
		sh = norm_s(kmv);
		t1 = shl(kmv, sh);
		Word16 nsh = negate(sh);
		BIN_PASSES(t, i, {
			if (cmp_shift(s->ksi[i], s->ksi_shift[i], t1, nsh) < 0) {
				s->ksi[i] = t1;
				s->ksi_shift[i] = nsh;
			}
			s->qk[i] = ENH_QK_MAX;
		})
		if (!nflag) {
			if (cmp_shift(gav, gavs, 23170, 1) > 0) {
				L = L_mult(s->YY_LT, 32023);
				sh = norm_l(L);
				t1 = extract_h(L_shl(L, sh));
				t2 = sub(s->YY_LT_shift, sh);
				L = L_mult(YY_av, 745);
				sh = norm_l(L);
				t3 = extract_h(L_shl(L, sh));
				t4 = sub(YY_av_shift, sh);
				t1 = shr(t1, 1);
				t3 = shr(t3, 1);
				sh = sub(t2, t4);
				Word16 yl, yls;
				if (sh > 0) {
					yl = add(t1, shr(t3, sh));
					yls = t2;
				} else {
					yl = add(shl(t1, sh), t3);
					yls = t4;
				}
				yls = add(yls, 1);
				if (sub(yl, s->n_pwr) > 0) {
					yl = shr(yl, 1);
					yls = add(yls, 1);
				}
				s->YY_LT = yl;
				s->YY_LT_shift = yls;
				Word16 sn = divide_s(yl, s->n_pwr);
				Word16 sns = sub(yls, s->n_pwr_shift);
				if (cmp_shift(sn, sns, SW_MAX_, 0) < 0) {
					sn = s->SN_LT0;
					sns = s->SN_LT0_shift;
				} else {
					L = L_sub(L_deposit_h(sn), L_shr(L_deposit_h(SW_MAX_), sns));
					sh = norm_l(L);
					sn = extract_h(L_shl(L, sh));
					sns = sub(sns, sh);
				}
				s->SN_LT = sn;
				s->SN_LT_shift = sns;
				s->SN_LT0 = sn;
				s->SN_LT0_shift = sns;
			}
			bool first = !s->qk_started;
			PROF_SCOPE(57);
			BIN_PASSES(t, i, {
				npp_compute_qk_bin(s, s->qk, gk, gks, 19273, first, i);
				if (s->qk[i] > ENH_QK_MAX)
					s->qk[i] = ENH_QK_MAX;
				else if (s->qk[i] < ENH_QK_MIN)
					s->qk[i] = ENH_QK_MIN;
			})
			s->qk_started = 1;
		}
		PROF_SCOPE(58);
		BIN_PASSES(t, i, {
			int16_t vk, vksh;	/* bin i's, this lane's only */
			npp_gain_log_mmse_bin(s, vk, vksh, s->qk, s->Gain, gk, gks, i);
			GainD[i] = s->Gain[i];
			npp_gain_mod_bin(s, vk, vksh, s->qk, GainD, i);
			Word32 v = L_mult(GainD[i], ymag[t]);
			Word16 n = norm_l(v);
			s->agal[i] = extract_h(L_shl(v, n));
			s->agal_shift[i] = sub(ymag_sh[t], n);
		})
	}
	}
	wsync();
	{
	PROF_SCOPE(59);
	int lm = 0;
	Word32 tyr[5];	/* temp_yy of samples lane + 64 t, in registers */
#pragma unroll
	for (int t = 0; t < 5; t++) {
		int i = lane + WV * t;
		tyr[t] = 0;
		if (i < NPP_WIN + 2) {
			Word32 v = L_mult(yb[i], GainD[i / 2]);
			tyr[t] = v;
			lm = max(lm, (int) L_abs(v));
		}
	}
	Word32 Lmax = wmax(lm);
	sh = norm_l(Lmax);
#pragma unroll
	for (int t = 0; t < 5; t++) {
		int i = lane + WV * t;
		if (i < NPP_WIN + 2)
			yb[i] = extract_h(L_shl(tyr[t], sh));
	}
	sh = sub(Ysh, sh);
	wsync();
	wv_mirror(yb, lane);
	g = wv_fft_npp(yb, -1, kc, lane);
	sh = add(sh, g);
	sh = sub(sh, 8);
	Word16 osh = sub(sh, 15);
#pragma unroll
	LANE_LOOP(i, NPP_WIN)
		out[i] = mult(shl(yb[2 * i], osh), kc->win[i >> 6]);
	}
	/* noise power for the next frame (npp.c:1621-1635) */
	maxs = SW_MIN_;
	BIN_PASSES(t, i, { maxs = max(maxs, (int) s->lambdaD_shift[i]); })
	maxs = wmax(maxs);
	part = 0;
	BIN_PASSES(t, i, {
		Word32 st = npp_spec_term(s->lambdaD, s->lambdaD_shift, (Word16) maxs, i);
		part += st;
	})
	L = wsum(part);
	if (L == 0)
		L = 1;
	sh = norm_l(L);
	s->n_pwr = extract_h(L_shl(L, sh));
	s->n_pwr_shift = add(sub((Word16) maxs, sh), 1);
	wsync();
}

/* npp :170 -- 180 new samples from `x` (global memory), 180 enhanced
 * samples back to the same place.  `avail` = valid samples at x for the
 * first call's 256-sample read (npp.c:176-189); short reads see zeros. */
MD void wv_npp_frame(NppWave *W, NppState *m, int16_t *x, int avail, bool rate1200, const WvConst *kc,
		     int lane)
{
	PROF_SCOPE(0);
	NppState *s = wv_S(W);
	if (!s->started) {
		int16_t *noise = W->buf;
		LANE_LOOP(i, NPP_WIN) {
			int16_t v = 0;
			if (rate1200)
				v = i < avail ? x[i] : (int16_t) 0;
			else if (i >= NPP_OVL)
				v = x[i - NPP_OVL];
			noise[i] = v;
		}
		wsync();
		wv_enh_init(W, noise, kc, lane, m);
		LANE_LOOP(i, NPP_WIN)
			s->speech_in[i] = 0;
		s->started = 1;
		wsync();
	}
	LANE_LOOP(i, NPP_OVL)
		s->speech_in[i] = s->speech_in[NPP_HOP + i];
	wsync();	/* lanes below overwrite what lanes above read */
	LANE_LOOP(i, NPP_HOP)
		s->speech_in[NPP_OVL + i] = x[i];
	wsync();
	wv_process_frame(W, m, s->speech_in, W->buf, kc, lane);
	LANE_LOOP(i, NPP_OVL) {
		Word16 o = add(W->buf[i], s->overlap[i]);
		s->overlap[i] = W->buf[NPP_HOP + i];
		W->buf[i] = o;
	}
	wsync();
	LANE_LOOP(i, NPP_HOP)
		x[i] = W->buf[i];
	wsync();
}

/* HBM record <-> LDS image of a channel's NppState, dword copies */
MD void wv_state_in(NppWave *W, const NppState *g, int lane)
{
	PROF_SCOPE(35);
	const u32_alias *src = (const u32_alias *) g;	/* kern.h: may_alias dwords */
	u32_alias *dst = W->s_hot;
	LANE_LOOP(i, (int) (NPP_HOT_BYTES / 4))
		dst[i] = src[i];
	wsync();
}

MD void wv_state_out(NppState *g, const NppWave *W, int lane)
{
	PROF_SCOPE(35);
	wsync();
	const u32_alias *src = W->s_hot;
	u32_alias *dst = (u32_alias *) g;
	LANE_LOOP(i, (int) (NPP_HOT_BYTES / 4))
		dst[i] = src[i];
}

}  // namespace wv
}  // namespace mlp

#endif
