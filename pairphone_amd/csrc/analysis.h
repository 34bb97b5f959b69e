/*
 * analysis.h -- the MELPe analysis front end on one lane (= one channel):
 * DC removal, bandpass voicing, integer/fractional pitch, pitch tracking and
 * frame classification, LPC/LSF, gain, Fourier magnitudes, and the
 * superframe smoothing (sc_ana).
 *
 * Restates melpe/melp_ana.c, melpe/melp_sub.c (analysis part),
 * melpe/pit_lib.c, melpe/pitch.c, melpe/classify.c and melpe/fs_lib.c with
 * the reference's statics held in EncState.  Function names follow the
 * reference's; line numbers cite the reference file each one restates.
 */
#ifndef MELPE_ANALYSIS_H
#define MELPE_ANALYSIS_H

#include "state.h"

namespace mlp {

/* ------------------------------------------------------------------ */
/* melpe/melp_sub.c                                                   */
/* ------------------------------------------------------------------ */

/* dc_rmv :211 -- 3 double-precision biquads (NEW_DC_FILTER) */
MD void dc_rmv(const int16_t *in, int16_t *out, int16_t *din, int16_t *dhi,
	       int16_t *dlo, int n)
{
	PROF_SCOPE(33);
	iir3_d(in, out, TB(dc_den), TB(dc_num), din, dhi, dlo, n);
}

/* remove_dc's offset from the sample sum (an L_add chain of int16 over at
 * most PIT_COR_LEN terms: never clamps) */
MD Word16 remove_dc_off(Word32 sum, int16_t len)
{
	Word16 up = sub(15, norm_s(len));
	Word16 pdown = shl(1, sub(up, 1));
	sum = L_shr(sum, up);
	Word16 off = mult(extract_l(sum), divide_s(pdown, len));
	return shl(off, 1);
}

/* remove_dc :261 */
MN void remove_dc(const int16_t *in, int16_t *out, int16_t len)
{
	Word32 sum = 0;
	P16 r;
	int np = p16_open(r, in, len);
	int i = 0;
	#pragma unroll 4
	for (int k = 0; k < np; k++, i += 2) {
		uint32_t x = p16_next(r);
		sum = L_add(sum, L_deposit_l(lo16(x)));
		sum = L_add(sum, L_deposit_l(hi16(x)));
	}
	for (; i < len; i++)
		sum = L_add(sum, L_deposit_l(in[i]));
	const Word16 off = remove_dc_off(sum, len);
	v_batch(in, out, len, [off](int, int16_t x) { return sub(x, off); });
}

/* gain_ana :311 -- pitch-adaptive RMS in dB (Q8) */
MN Word16 gain_ana(const int16_t *sig, Word16 pitch, Word16 minlen, Word16 maxlen)
{
	PROF_SCOPE(23);
#if defined(MELPE_OPCOUNT)
	int16_t tb[PITCHMAX * 2 + 8];
#endif
	Word16 pq6 = shr(pitch, 1);
	Word16 tmin = shl(minlen, 6);
	Word16 fl = pq6;
	while (fl < tmin)
		fl = add(fl, pq6);
	Word16 len = shr(add(fl, 32), 6);
	if (len > maxlen)
		len = shr(len, 1);
	Word16 beg = negate(shr(len, 1));
	Word16 sc = 3;
#if defined(MELPE_OPCOUNT)
	v_equ_shr(tb, &sig[beg], sc, len);
	Word32 e = L_v_magsq(tb, len, 0, 1);
#else
	/* both energies straight from sig with the shift applied per sample
	 * (magsq_shr): the same L_mac chains as L_v_magsq over the shifted
	 * copies, without writing them */
	Word32 e = magsq_shr(&sig[beg], len, sc);
#endif
	if (e) {
		sc = sub(sc, shr(norm_l(e), 1));
		if (sc < 0)
			sc = 0;
	} else {
		sc = 0;
	}
	Word16 g, t1, t2;
#if defined(MELPE_OPCOUNT)
	if (sc)
		v_equ_shr(tb, &sig[beg], sc, len);
	else
		v_copy(tb, &sig[beg], len);
	e = L_v_magsq(tb, len, 0, 0);
#else
	e = L_shr(magsq_shr(&sig[beg], len, sc), 1);
#endif
	if (sc) {
		t1 = L_log10_fxp(e, 0);
		t2 = L_log10_fxp(L_deposit_l(len), 0);
		t1 = sub(t1, t2);
		t2 = extract_l(L_shr(L_mult(sc, 1233), 1));
		t1 = add(t1, t2);
		g = shl(mult(20480, t1), 1);
	} else {
		t1 = (e == 0) ? (Word16) -4096 : L_log10_fxp(e, 0);
		t2 = L_log10_fxp(L_deposit_l(len), 0);
		t1 = sub(t1, t2);
		g = shl(mult(20480, t1), 1);
	}
	return g < 0 ? 0 : g;
}

/* q_bpvc :555 -- returns uv_flag */
MD int16_t q_bpvc(int16_t *bpvc, int16_t *idx, int nb)
{
	Word16 k = 0;
	int16_t uv;
	if (bpvc[0] > BPTHRESH_Q14) {
		uv = 0;
		bpvc[0] = 16384;
		for (int i = 1; i < nb; i++) {
			k = shl(k, 1);
			if (bpvc[i] > BPTHRESH_Q14) {
				bpvc[i] = 16384;
				k |= 1;
			} else {
				bpvc[i] = 0;
			}
		}
		if (k == 1) {	/* INVALID_BPVC */
			bpvc[nb - 1] = 0;
			k = 0;
		}
	} else {
		uv = 1;
		k = 0;
		v_zero(bpvc, nb);
	}
	*idx = k;
	return uv;
}

/* q_bpvc_dec :595 */
MD void q_bpvc_dec(int16_t *bpvc, Word16 idx, int16_t uv, int nb)
{
	if (uv) {
		idx = 0;
		bpvc[0] = 0;
	} else {
		bpvc[0] = 16384;
	}
	if (idx == 1)
		idx = 0;
	for (int i = nb - 1; i > 0; i--) {
		bpvc[i] = (idx & 1) ? 16384 : 0;
		idx = shr(idx, 1);
	}
}

/* ------------------------------------------------------------------ */
/* melpe/pit_lib.c                                                    */
/* ------------------------------------------------------------------ */

/* Exact-path bookkeeping for the host build's tests: MELPE_NO_EXACT turns the
 * exact correlators off (every chain runs sequentially), MELPE_EXACT_STATS
 * counts the frac_pch / find_pitch calls that took each path. */
#if defined(MELPE_EXACT_STATS) && !defined(__HIP__)
extern "C" long melpe_exact_stats[6];
#define EXACT_STAT(i) (melpe_exact_stats[i]++)
#else
#define EXACT_STAT(i) ((void) 0)
#endif

/* p[i] = shr(p[i], sc) in place, returning sum y^2 saturated to 32 bits
 * (exact below 2^31 - 1, which is all the bound needs): dword pairs in
 * chunks of four, the next chunk loaded before this one is stored */
MD int32_t shr_energy_inplace(int16_t *p, int n, Word16 sc)
{
	int32_t e = 0;
	int i = 0;
	if (n > 0 && ((reinterpret_cast<uintptr_t>(p) >> 1) & 1)) {
		int16_t y = shr(p[0], sc);
		p[0] = y;
		e = (int32_t) y * y;
		i = 1;
	}
	u32_alias *w = reinterpret_cast<u32_alias *>(p + i);
	const int nd = (n - i) >> 1, G = nd >> 2;
	auto sh2 = [&](uint32_t v) {
		return (uint32_t) (uint16_t) shr(lo16(v), sc) | ((uint32_t) (uint16_t) shr(hi16(v), sc) << 16);
	};
	uint32_t cur[4];
	if (G > 0)
		for (int k = 0; k < 4; k++)
			cur[k] = w[k];
	#pragma unroll 1
	for (int g = 0; g < G; g++) {
		int gn = g + 1 < G ? g + 1 : g;
		uint32_t nxt[4];
		#pragma unroll
		for (int k = 0; k < 4; k++)
			nxt[k] = w[4 * gn + k];
		#pragma unroll
		for (int k = 0; k < 4; k++) {
			uint32_t y = sh2(cur[k]);
			w[4 * g + k] = y;
			e = sdot2_sat(y, y, e);
			cur[k] = nxt[k];
		}
	}
	for (int d = 4 * G; d < nd; d++) {
		uint32_t y = sh2(w[d]);
		w[d] = y;
		e = sdot2_sat(y, y, e);
	}
	for (int k = i + 2 * nd; k < n; k++) {
		int16_t y = shr(p[k], sc);
		p[k] = y;
		int64_t t = (int64_t) e + (int32_t) y * y;
		e = t > LW_MAX_ ? LW_MAX_ : (int32_t) t;
	}
	return e;
}

/* f_pitch_scale's second half, given the window's exact energy (the sum of
 * L_mult(x, x), in 64 bits): callers that produce the window can add its
 * energy up while they write it (bpvc_ana) */
MD Word16 f_pitch_scale_e(int16_t *out, const int16_t *in, int len, int64_t sum,
			     bool *exact = nullptr, int64_t extra = 0)
{
	Word16 sc = 0;
	/* Every term L_mult(x, x) is >= 0, so the reference's running margin
	 * test (:193-203) fails exactly when the running sum first exceeds
	 * LW_MAX, i.e. iff the whole 64-bit sum does; without it L_add never
	 * saturates and the sum is exact. */
	Word32 corr = (Word32) sum;
	if (sum > (int64_t) LW_MAX_) {
		int16_t tb[PITCH_FR + 8];
		sc = 5;
		v_equ_shr(tb, in, sc, len);
		corr = L_v_magsq(tb, len, 0, 1);
	}
	sc = sub(sc, shr(norm_l(corr), 1));
	if (!exact) {
		v_equ_shr(out, in, sc, len);
		return sc;
	}
	/* the output's own energy, sum of 2 y^2 without saturation: when it
	 * fits 32 bits no L_mac chain over these samples can clamp
	 * (sum |2ab| <= sum a^2 + b^2), which the exact correlators rely on */
	int64_t e2 = extra;
	if (out == in) {
		e2 += 2 * (int64_t) shr_energy_inplace(out, len, sc);
	} else {
		for (int i = 0; i < len; i++) {
			int16_t y = shr(in[i], sc);
			out[i] = y;
			e2 += 2 * (int64_t) ((int32_t) y * y);
		}
	}
#if defined(MELPE_NO_EXACT)
	*exact = false;
#else
	*exact = e2 <= (int64_t) LW_MAX_;
#endif
	return sc;
}

/* f_pitch_scale :178 -- scale so the energy fits, returns the shift */
MN Word16 f_pitch_scale(int16_t *out, const int16_t *in, int len, bool *exact = nullptr,
			int64_t extra = 0)
{
	Word16 sc = 0;
	Word32 corr;
	bool ovf;
#if defined(MELPE_OPCOUNT)
	/* census build: the reference's loop, op for op */
	{
		Word32 sum = 0, margin = LW_MAX_;
		ovf = false;
		for (int i = 0; i < len && !ovf; i++) {
			Word32 t = L_mult(in[i], in[i]);
			if (t <= margin) {
				sum = L_add(sum, t);
				margin = L_sub(margin, t);
			} else {
				ovf = true;
			}
		}
		corr = sum;
	}
#else
	/* the energy in one pass, no data-dependent exit (f_pitch_scale_e) */
	{
		int64_t sum = 0;
		P16 r;
		int np = p16_open(r, in, len);
		int i = 0;
		#pragma unroll 8
		for (int k = 0; k < np; k++, i += 2) {
			uint32_t x = p16_next(r);
			sum += L_mult(lo16(x), lo16(x));
			sum += L_mult(hi16(x), hi16(x));
		}
		for (; i < len; i++)
			sum += L_mult(in[i], in[i]);
		return f_pitch_scale_e(out, in, len, sum, exact, extra);
	}
#endif
	if (ovf) {
		int16_t tb[PITCH_FR + 8];
		sc = 5;
		v_equ_shr(tb, in, sc, len);
		corr = L_v_magsq(tb, len, 0, 1);
	}
	sc = sub(sc, shr(norm_l(corr), 1));
	v_equ_shr(out, in, sc, len);
	if (exact)
		*exact = false;
	(void) extra;
	return sc;
}

/* the 8 correlations of one lag block of find_pitch: lag n0+k (k = 0..7,
 * n0 even) reads sig[cb + a_k + j] * sig[cb + upper - n0 - 7 + 3 + b_k + j]
 * ... i.e. the a-offsets {0,1,1,2,2,3,3,4} and b-offsets {3,3,2,2,1,1,0,0}
 * relative to the block's two bases (cb_n = cb0 + (n + 1) / 2, lag
 * i_n = upper - n).  Each lag keeps its own saturating L_mac chain in j
 * order, so the result is the reference's per-lag L_v_inner; the block only
 * shares the sample loads (two per j instead of sixteen). */
MD void fp_corr8(const int16_t *pa, const int16_t *pb, int len, Word32 *out)
{
	Word32 acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	int16_t A0 = pa[0], A1 = pa[1], A2 = pa[2], A3 = pa[3];
	int16_t B0 = pb[0], B1 = pb[1], B2 = pb[2];
	auto step = [&](int16_t A4, int16_t B3) {
		acc[0] = L_mac(acc[0], A0, B3);
		acc[1] = L_mac(acc[1], A1, B3);
		acc[2] = L_mac(acc[2], A1, B2);
		acc[3] = L_mac(acc[3], A2, B2);
		acc[4] = L_mac(acc[4], A2, B1);
		acc[5] = L_mac(acc[5], A3, B1);
		acc[6] = L_mac(acc[6], A3, B0);
		acc[7] = L_mac(acc[7], A4, B0);
		A0 = A1;
		A1 = A2;
		A2 = A3;
		A3 = A4;
		B0 = B1;
		B1 = B2;
		B2 = B3;
	};
	/* the new samples pa[j + 4], pb[j + 3] two at a time (P16) */
	P16 ra, rb;
	int np = p16_open(ra, pa + 4, len), nb = p16_open(rb, pb + 3, len);
	np = np < nb ? np : nb;
	int j = 0;
	#pragma unroll 4
	for (int k = 0; k < np; k++, j += 2) {
		uint32_t x = p16_next(ra), y = p16_next(rb);
		step(lo16(x), lo16(y));
		step(hi16(x), hi16(y));
	}
	for (; j < len; j++)
		step(pa[j + 4], pb[j + 3]);
	for (int k = 0; k < 8; k++)
		out[k] = acc[k];
}

/* fp_corr8 for a block of K lags (K even or odd): lag n0 + k reads
 * pa[j + (k + 1) / 2] * pb[j + (k + 1) / 2 - k + BMAX], BMAX = (K - 1) - K / 2,
 * from the bases a = cb_n0 and b = cb_(n0+K-1) + i_(n0+K-1).  find_pitch's
 * +-5 lag searches are 11 lags or fewer: one pass of K = 12 covers them all
 * (the reads of the unused lags stay inside the window the real lags span). */
template <int K>
MD void fp_corrK(const int16_t *pa, const int16_t *pb, int len, Word32 *out)
{
	constexpr int NA = K / 2 + 1, BMAX = (K - 1) - K / 2;
	Word32 acc[K];
	int16_t A[NA], B[BMAX + 1];
	#pragma unroll
	for (int k = 0; k < K; k++)
		acc[k] = 0;
	#pragma unroll
	for (int q = 0; q < NA - 1; q++)
		A[q] = pa[q];
	#pragma unroll
	for (int q = 0; q < BMAX; q++)
		B[q] = pb[q];
	auto step = [&](int16_t an, int16_t bn) {
		A[NA - 1] = an;
		B[BMAX] = bn;
		#pragma unroll
		for (int k = 0; k < K; k++)
			acc[k] = L_mac(acc[k], A[(k + 1) / 2], B[(k + 1) / 2 - k + BMAX]);
		#pragma unroll
		for (int q = 0; q < NA - 1; q++)
			A[q] = A[q + 1];
		#pragma unroll
		for (int q = 0; q < BMAX; q++)
			B[q] = B[q + 1];
	};
	P16 ra, rb;
	int np = p16_open(ra, pa + NA - 1, len), nb = p16_open(rb, pb + BMAX, len);
	np = np < nb ? np : nb;
	int j = 0;
	#pragma unroll 2
	for (int k = 0; k < np; k++, j += 2) {
		uint32_t x = p16_next(ra), y = p16_next(rb);
		step(lo16(x), lo16(y));
		step(hi16(x), hi16(y));
	}
	for (; j < len; j++)
		step(pa[j + NA - 1], pb[j + BMAX]);
	#pragma unroll
	for (int k = 0; k < K; k++)
		out[k] = acc[k];
}

/* frac_pch's nine sums as exact plain sums (the caller's bound), on packed
 * pairs: a_j = pa[j], b_j = pb[j], j < len; in q[]: a.a, b.b, a.b, a.b+1,
 * a.b+2, b+1.b+2, b+1.b+1, b+2.b+2, b.b+1.  Reads pa[0 .. len), pb[0 .. len + 2). */
MD void fp_sums9(const int16_t *pa, const int16_t *pb, int len, int32_t *q)
{
	constexpr int PD = MELPE_XC_PD;
	int32_t acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
	const int T = len >> 1;
	int jt = 0;
	if (T >= 4) {
		PairStream sa, sb;
		ps_open(sa, pa, len);
		ps_open(sb, pb, len + 2);
		/* steps 4g .. 4g + 3: a pairs xa[st]; b pairs wb[st] (b_j),
		 * their mids (b_j+1) and wb[st + 1] (b_j+2) */
		uint32_t wb[5];
		ps_head<1>(sb, wb);
		auto group = [&](const uint32_t *xa, int nst) {
			#pragma unroll
			for (int st = 0; st < 4; st++) {
				uint32_t A = xa[st], b0 = wb[st], b2 = wb[st + 1];
				uint32_t b1 = pair_mid(b2, b0);
				int32_t d[9] = {sdot2(A, A, acc[0]), sdot2(b0, b0, acc[1]),
						 sdot2(A, b0, acc[2]), sdot2(A, b1, acc[3]),
						 sdot2(A, b2, acc[4]), sdot2(b1, b2, acc[5]),
						 sdot2(b1, b1, acc[6]), sdot2(b2, b2, acc[7]),
						 sdot2(b0, b1, acc[8])};
				#pragma unroll
				for (int k = 0; k < 9; k++)
					acc[k] = st < nst ? d[k] : acc[k];
			}
			wb[0] = wb[4];
		};
		int G = T >> 2, ga = ps_full_groups(sa, 0), gb = ps_full_groups(sb, 1);
		G = G < ga ? G : ga;
		G = G < gb ? G : gb;
		if (G > 0) {
			P16C<PD> ca, cb;
			p16c_open(ca, sa, 0, G);
			p16c_open(cb, sb, 1, G);
			#pragma unroll 1
			for (int g = 0; g < G; g++) {
				uint32_t xa[4];
				p16c_next4(ca, xa);
				p16c_next4(cb, &wb[1]);
				group(xa, 4);
			}
		}
		#pragma unroll 1
		for (int t = 4 * G; t < T; t += 4) {
			uint32_t xa[4];
			ps_pairs4(sa, t, xa);
			ps_pairs4(sb, 1 + t, &wb[1]);
			group(xa, T - t);
		}
		jt = 2 * T;
	}
	for (int j = jt; j < len; j++) {
		int a = pa[j], x0 = pb[j], x1 = pb[j + 1], x2 = pb[j + 2];
		acc[0] += a * a;
		acc[1] += x0 * x0;
		acc[2] += a * x0;
		acc[3] += a * x1;
		acc[4] += a * x2;
		acc[5] += x1 * x2;
		acc[6] += x1 * x1;
		acc[7] += x2 * x2;
		acc[8] += x0 * x1;
	}
	for (int k = 0; k < 9; k++)
		q[k] = acc[k];
}

/* find_pitch :240 -- normalised autocorrelation lag search, lags upper..lower */
/* lsh > 0 (exact only): sig holds the window before f_pitch_scale's left
 * shift by lsh, which the caller proved exact (see frac_pch) */
MN Word16 find_pitch(const int16_t *sig, Word16 *pcorr, Word16 lower, Word16 upper, Word16 len,
		     bool exact = false, int lsh = 0)
{
	PROF_SCOPE(2);
#if defined(MELPE_OPCOUNT)
	exact = false;
#endif
	EXACT_STAT(exact ? 1 : 0);
	Word16 ip = lower;
	Word32 max_num = 0, max_den = 1;
	Word16 cb = negate(shr(add(len, upper), 1));
	const Word16 cb0 = cb;
	/* exact: the caller's bound holds over sig[cb0 .. cb0 + upper + len),
	 * which every lag block below reads inside (also the unused lags of a
	 * last partial block), so each L_mac chain is the plain sum */
	Word32 c00, cTT;
	/* sums of the scaled samples: the plain sums times 4^lsh */
	const int32_t sm = 2 << (2 * lsh);
	const int qm = 1 << lsh;
	if (exact) {
		c00 = sm * magsq_pairs(&sig[cb], len);
		cTT = sm * magsq_pairs(&sig[cb + upper], len);
		OPC_ADD(OP_L_mac, 0);
	} else {
		c00 = L_v_magsq(&sig[cb], len, 0, 1);
		cTT = L_v_magsq(&sig[cb + upper], len, 0, 1);
	}
	Word32 blk[8];
	int nlags = upper - lower + 1;
#if !defined(MELPE_OPCOUNT)
	/* up to 12 lags (every +-5 search): all of them in one pass */
	Word32 blk12[12];
	const bool one = nlags <= 12;
	if (one) {
		if (exact) {
			int32_t raw[12];
			xcorr_pairs<12, FpLags<12>, false>(&sig[cb0], &sig[cb0 + 6 + upper - 11], len, raw);
			for (int k = 0; k < 12; k++)
				blk12[k] = sm * raw[k];
		} else {
			fp_corrK<12>(&sig[cb0], &sig[cb0 + 6 + upper - 11], len, blk12);
		}
	}
#else
	const bool one = false;
	Word32 *blk12 = blk;
#endif
	/* the energy updates' samples, loaded eight lags ahead: the c00 update
	 * of lag n0 + 2k reads sig[cb0 + n0/2 + k] (and + len), the cTT update
	 * of lag n0 + 2k + 1 sig[cb0 + upper - 1 - n0/2 - k] (and + len); each
	 * register queue moves up by one per update */
	int16_t qa[4], qal[4], qb[4], qbl[4];
	/* lag i = upper - n; k8 = n & 7 and (for the one-pass search) n itself
	 * are compile-time constants in the unrolled loops below, so blk[] and
	 * blk12[] stay in registers (indexed at run time they lived in the
	 * private segment: a store per block, a load and its wait per lag) */
	auto lag = [&](int n, int k8) __attribute__((always_inline)) {
		const Word16 i = upper - n;
		const bool even = (k8 & 1) == 0;
		Word32 corr;
		if (k8 == 0) {
			const int16_t *pa = &sig[cb0 + n / 2], *pb = &sig[cb0 + upper - 1 - n / 2];
			#pragma unroll
			for (int k = 0; k < 4; k++) {
				qa[k] = (int16_t) (pa[k] * qm);
				qal[k] = (int16_t) (pa[k + len] * qm);
				qb[k] = (int16_t) (pb[-k] * qm);
				qbl[k] = (int16_t) (pb[len - k] * qm);
			}
		}
		if (one) {
			corr = blk12[n < 12 ? n : 0];
		} else if (k8 == 0 && (exact || n + 8 <= nlags)) {
			/* the block's bases: a at cb_n0, b at cb_(n0+7) + i_(n0+7) */
			int c_n0 = cb0 + (n + 1) / 2;
			int b0 = cb0 + (n + 8) / 2 + upper - n - 7;
			if (exact) {
				int32_t raw[8];
				xcorr_pairs<8, FpLags<8>, false>(&sig[c_n0], &sig[b0], len, raw);
				for (int k = 0; k < 8; k++)
					blk[k] = sm * raw[k];
			} else {
				fp_corr8(&sig[c_n0], &sig[b0], len, blk);
			}
		}
		if (one) {
		} else if (exact || n < (nlags & ~7)) {
			corr = blk[k8];
			/* census: the reference's L_v_inner tail per lag */
			OPC_ADD(OP_add, 2);
			OPC_ADD(OP_sub, 1);
			OPC_ADD(OP_L_shl, 1);
		} else
			corr = L_v_inner(&sig[cb], &sig[cb + i], len, 0, 0, 1);
		Word16 s1a = norm_s(extract_h(c00));
		Word16 s1b = norm_s(extract_h(cTT));
		Word16 s = add(s1a, s1b);
		Word16 s2 = shr(s, 1);
		if (shl(s2, 1) != s)
			s1a = sub(s1a, 1);
		Word32 num;
		if (corr > 0) {
			Word16 sc = extract_h(L_shl(corr, s2));
			num = extract_h(L_mult(sc, sc));
		} else {
			num = 0;
		}
		Word32 den = extract_h(L_mult(extract_h(L_shl(c00, s1a)),
					      extract_h(L_shl(cTT, s1b))));
		if (den < 1)
			den = 1;
		if (L_mult(extract_l(num), extract_l(max_den)) >
		    L_mult(extract_l(max_num), extract_l(den))) {
			max_den = den;
			max_num = num;
			ip = i;
		}
		if (even) {
			c00 = L_msu(c00, qa[0], qa[0]);	/* sig[cb], sig[cb + len] */
			c00 = L_mac(c00, qal[0], qal[0]);
			cb = add(cb, 1);
			#pragma unroll
			for (int k = 0; k < 3; k++) {
				qa[k] = qa[k + 1];
				qal[k] = qal[k + 1];
			}
		} else {
			/* sig[cb + i - 1 + len], sig[cb + i - 1] */
			cTT = L_msu(cTT, qbl[0], qbl[0]);
			cTT = L_mac(cTT, qb[0], qb[0]);
			#pragma unroll
			for (int k = 0; k < 3; k++) {
				qb[k] = qb[k + 1];
				qbl[k] = qbl[k + 1];
			}
		}
	};
#if !defined(MELPE_OPCOUNT)
	if (one) {
		#pragma unroll
		for (int n = 0; n < 12; n++)
			if (n < nlags)
				lag(n, n & 7);
	} else {
		for (int n0 = 0; n0 < nlags; n0 += 8) {
			#pragma unroll
			for (int k8 = 0; k8 < 8; k8++)
				if (n0 + k8 < nlags)
					lag(n0 + k8, k8);
		}
	}
#else
	for (int n = 0; n < nlags; n++)
		lag(n, n & 7);
#endif
	(void) cb;
	*pcorr = shr(sqrt_fxp(divide_s(extract_l(max_num), extract_l(max_den)), 15), 1);
	return ip;
}

/* frac_pch :340 -- fractional pitch refinement and its correlation */
/* lsh > 0 (range 0 only): sig holds the window before its scaling by
 * f_pitch_scale, which the caller proved a plain left shift by lsh with no
 * saturation (bpvc_band_s); every sample is shifted as it is read, so the
 * scaled window is never written out */
MN Word16 frac_pch(const int16_t *sig, Word16 *pcorr, Word16 fpitch, Word16 range,
		   Word16 pmin, Word16 pmax, Word16 pmin_q7, Word16 pmax_q7, Word16 lmin,
		   bool exact = false, int lsh = 0)
{
	PROF_SCOPE(3);
#if defined(MELPE_OPCOUNT)
	exact = false;
#endif
#if defined(MELPE_DIAG_UNIFORM_PITCH)
	fpitch = 80 << 7;	/* diagnostics only: every lane at one lag (wrong output) */
#endif
	EXACT_STAT(exact ? 3 : 2);
	Word16 len, cb, ip, corr;
	if (range > 0) {
		ip = shift_r(fpitch, -7);
		Word16 lo = sub(ip, range), hi = add(ip, range);
		if (hi > pmax)
			hi = pmax;
		if (lo < pmin)
			lo = pmin;
		Word16 q = add(shr(ip, 1), shr(ip, 2));
		if (lo < q)
			lo = q;
		len = ip;
		if (len < lmin)
			len = lmin;
		fpitch = shl(find_pitch(sig, &corr, lo, hi, len, exact, lsh), 7);
	}
	ip = shift_r(fpitch, -7);
	if (ip >= pmax)
		ip = sub(pmax, 1);
	len = ip;
	if (len < lmin)
		len = lmin;
	cb = negate(shr(add(len, ip), 1));
	/* All nine sums of the reference's separate L_v_magsq / L_v_inner calls
	 * in one pass over the samples: a_j = sig[cb + j], b_j = sig[cb + ip -
	 * 1 + j].  Each sum keeps its own saturating L_mac chain in j order, so
	 * each equals the call it replaces; the candidates for both outcomes of
	 * the ip-1 test are formed (cTT of one outcome is cT1T1 of the other, and
	 * cTT of the ip-1 outcome is the len-prefix of the (len+2)-term magsq). */
	Word32 msq = 0, m2 = 0, cm1 = 0, c0 = 0, c1 = 0, tt1 = 0, tt = 0, t1t1 = 0, tt1m = 0;
	if (exact) {
		int32_t q[9];
		fp_sums9(&sig[cb], &sig[cb + ip - 1], len, q);
		/* the sums of the samples scaled up by 2^lsh: the plain sums times
		 * 4^lsh, exactly (the caller's bound holds for the scaled ones) */
		const int32_t m = 2 << (2 * lsh);
		msq = m * q[0];
		m2 = m * q[1];
		cm1 = m * q[2];
		c0 = m * q[3];
		c1 = m * q[4];
		tt1 = m * q[5];
		tt = m * q[6];
		t1t1 = m * q[7];
		tt1m = m * q[8];
	} else {
		const int16_t *pa = &sig[cb], *pb = &sig[cb + ip - 1];
		int16_t b0 = (int16_t) (pb[0] * (1 << lsh)), b1 = (int16_t) (pb[1] * (1 << lsh));
		auto step = [&](int16_t a, int16_t b2) {
			msq = L_mac(msq, a, a);
			m2 = L_mac(m2, b0, b0);
			cm1 = L_mac(cm1, a, b0);
			c0 = L_mac(c0, a, b1);
			c1 = L_mac(c1, a, b2);
			tt1 = L_mac(tt1, b1, b2);
			tt = L_mac(tt, b1, b1);
			t1t1 = L_mac(t1t1, b2, b2);
			tt1m = L_mac(tt1m, b0, b1);
			b0 = b1;
			b1 = b2;
		};
		/* a_j and b_(j+2) two at a time (P16) */
		P16 ra, rb;
		int np = p16_open(ra, pa, len), nb = p16_open(rb, pb + 2, len);
		np = np < nb ? np : nb;
		int j = 0;
		#pragma unroll 4
		for (int k = 0; k < np; k++, j += 2) {
			uint32_t x = pk_shl16(p16_next(ra), lsh), y = pk_shl16(p16_next(rb), lsh);
			step(lo16(x), lo16(y));
			step(hi16(x), hi16(y));
		}
		for (; j < len; j++)
			step((int16_t) (pa[j] * (1 << lsh)), (int16_t) (pb[j + 2] * (1 << lsh)));
	}
	/* census: the reference's two L_v_magsq and six L_v_inner calls */
	OPC_ADD(OP_L_mac, -len);
	OPC_ADD(OP_shl, 2);
	OPC_ADD(OP_sub, 10);
	OPC_ADD(OP_add, 12);
	OPC_ADD(OP_L_shl, 8);
	Word32 ttm = m2;	/* sum of b_j^2, j < len */
	{
		const int m = 1 << lsh;
		const int16_t u = (int16_t) (sig[cb + ip - 1 + len] * m), v = (int16_t) (sig[cb + ip + len] * m);
		m2 = L_mac(m2, u, u);
		m2 = L_mac(m2, v, v);
	}
	Word16 s1a = norm_s(extract_h(msq));
	Word16 s1b = norm_s(extract_h(m2));
	Word16 s = add(s1a, s1b);
	Word16 s2 = shr(s, 1);
	if (shl(s2, 1) != s)
		s1a = sub(s1a, 1);
	Word16 c00 = extract_h(L_shl(msq, s1a));
	Word16 c0T = extract_h(L_shl(c0, s2));
	Word16 c0T1 = extract_h(L_shl(c1, s2));
	Word16 c0Tm1 = extract_h(L_shl(cm1, s2));
	Word32 rTT1 = tt1, rTT = tt, rT1T1 = t1t1;
	if (c0Tm1 > c0T1) {
		c0T1 = c0T;
		c0T = c0Tm1;
		ip = sub(ip, 1);
		rTT1 = tt1m;
		rTT = ttm;
		rT1T1 = tt;
	}
	Word16 cTT1 = extract_h(L_shl(rTT1, s1b));
	Word16 cTT = extract_h(L_shl(rTT, s1b));
	Word16 cT1T1 = extract_h(L_shl(rT1T1, s1b));
	Word32 den = L_add(L_mult(c0T1, sub(shr(cTT, 1), shr(cTT1, 1))),
			   L_mult(c0T, sub(shr(cT1T1, 1), shr(cTT1, 1))));
	Word32 num = L_sub(L_shr(L_mult(c0T1, cTT), 1), L_shr(L_mult(c0T, cTT1), 1));
	Word16 frac;
	Word32 aden = L_abs(den);
	if (aden > 0) {
		if (L_abs(L_shr(num, 2)) > aden) {
			if ((num > 0 && den < 0) || (num < 0 && den > 0))
				frac = -8192;
			else
				frac = 16384;
		} else {
			frac = L_divider2(num, den, 2, 0);
		}
	} else {
		frac = 4096;
	}
	if (frac > 16384)
		frac = 16384;
	if (frac < -8192)
		frac = -8192;
	fpitch = add(shl(ip, 7), shr(frac, 6));
	if (fpitch > pmax_q7) {
		fpitch = pmax_q7;
		frac = shl(sub(fpitch, shl(ip, 7)), 6);
	}
	if (fpitch < pmin_q7) {
		fpitch = pmin_q7;
		frac = shl(sub(fpitch, shl(ip, 7)), 6);
	}
	Word16 f1 = sub(8192, frac);
	Word32 d1 = L_shr(L_mpy_ls(L_mult(cTT, f1), f1), 1);
	Word32 d2 = L_mpy_ls(L_mult(cTT1, f1), frac);
	Word32 d3 = L_shr(L_mpy_ls(L_mult(cT1T1, frac), frac), 1);
	den = L_mpy_ls(L_add(L_add(d1, d2), d3), c00);
	Word16 root = L_sqrt_fxp(den, 0);
	Word32 t = L_mac(L_mult(c0T, f1), c0T1, frac);
	corr = (t <= 0) ? (Word16) 0 : extract_h(t);
	if (corr < root)
		*pcorr = shr(divide_s(corr, root), 1);
	else if (root <= 0)
		*pcorr = 0;
	else
		*pcorr = 16384;
	return fpitch;
}

/* double_ver :151 */
MN void double_ver(const int16_t *sig, Word16 *pcorr, Word16 pitch, Word16 pmin, Word16 pmax,
		   Word16 pmin_q7, Word16 pmax_q7, Word16 lmin, bool exact)
{
	Word16 m = 1;
	while (extract_l(L_shr(L_mult(pitch, m), 1)) < 3840)
		m = add(m, 1);
	if (m > 1) {
		Word16 tp = extract_l(L_shr(L_mult(pitch, m), 1));
		Word16 c;
		frac_pch(sig, &c, tp, 0, pmin, pmax, pmin_q7, pmax_q7, lmin, exact);
		if (c < *pcorr)
			*pcorr = c;
	}
}

/* double_chk :84 -- pitch-halving check over multiples 8..2 */
MN Word16 double_chk(const int16_t *sig, Word16 *pcorr, Word16 pitch, Word16 pdouble,
		     Word16 pmin, Word16 pmax, Word16 pmin_q7, Word16 pmax_q7, Word16 lmin,
		     bool exact)
{
	pitch = frac_pch(sig, pcorr, pitch, 0, pmin, pmax, pmin_q7, pmax_q7, lmin, exact);
	Word16 thresh = extract_l(L_shr(L_mult(*pcorr, pdouble), 8));
	for (Word16 m = 8; m >= 2; m--) {
		Word16 t1 = 0;
		Word16 t2 = shl(m, 11);
		Word16 tp = pitch;
		while (tp > t2) {
			tp = shr(tp, 1);
			t1 = add(t1, 1);
		}
		t2 = divide_s(tp, t2);
		t1 = sub(4, t1);
		tp = shr(t2, t1);
		if (tp >= pmin_q7) {
			Word16 c;
			tp = frac_pch(sig, &c, tp, 0, pmin, pmax, pmin_q7, pmax_q7, lmin, exact);
			double_ver(sig, &c, tp, pmin, pmax, pmin_q7, pmax_q7, lmin, exact);
			if (c > thresh) {
				pitch = frac_pch(sig, pcorr, tp, 0, pmin, pmax, pmin_q7, pmax_q7, lmin,
						 exact);
				break;
			}
		}
	}
	double_ver(sig, pcorr, pitch, pmin, pmax, pmin_q7, pmax_q7, lmin, exact);
	return pitch;
}

/* p_avg_update :515 */
MD Word16 p_avg_update(EncAna *E, Word16 pitch, Word16 pcorr, Word16 pthresh)
{
	if (!E->pavg_started) {
		v_set(E->good_pitch, DEFAULT_PITCH_Q7, NF);
		E->pavg_started = 1;
	}
	if (pcorr > pthresh) {
		v_copy(E->good_pitch, &E->good_pitch[1], NF - 1);
		E->good_pitch[NF - 1] = pitch;
	} else {
		for (int i = 0; i < NF; i++)
			E->good_pitch[i] = add(mult(31129, E->good_pitch[i]), 320);
	}
	return median3(E->good_pitch);
}

/* pitch_ana :571 -- final pitch from the lowpassed residual, with the
 * speech fallback; pa_sigbuf is persistent (its tail 323..326 can be read
 * stale by double_chk) */
MN Word16 pitch_ana(EncAna *E, const int16_t *speech, const int16_t *resid, Word16 pest,
		    Word16 pavg, Word16 *pcorr2)
{
	PROF_SCOPE(7);
	int16_t *sb = E->pa_sigbuf;
	Word16 pcorr, pitch, t, t2;
	bool ex = false;
	if (!E->pana_started) {
		v_zero(E->lpres_delin, LPF_ORD);
		v_zero(E->lpres_delout, LPF_ORD);
		E->pana_started = 1;
	}
#if defined(MELPE_OPCOUNT)
	v_copy(&sb[2], &resid[-PITCHMAX], PITCH_FR);
	iir3_s(&sb[2], TB(lpf_den), TB(lpf_num), E->lpres_delin, E->lpres_delout, PITCH_FR,
	       FRAME);
	f_pitch_scale(&sb[2], &sb[2], PITCH_FR, &ex);
#else
	/* copy, lowpass (memories kept after FRAME samples) and the
	 * f_pitch_scale energy in one pass, as bpvc_ana's windows */
	{
		int64_t e = 0;
		auto acc = [&](int, int16_t y) { e += L_mult(y, y); };
		iir3_s_io(&resid[-PITCHMAX], &sb[2], TB(lpf_den), TB(lpf_num), E->lpres_delin,
			  E->lpres_delout, FRAME, acc);
		int16_t tin[2 * 3], tout[2 * 3];
		v_copy(tin, E->lpres_delin, 6);
		v_copy(tout, E->lpres_delout, 6);
		iir3_s_io(&resid[-PITCHMAX + FRAME], &sb[2 + FRAME], TB(lpf_den), TB(lpf_num), tin, tout,
			  PITCH_FR - FRAME, acc);
		/* double_chk below reads up to sb[LPF_ORD + PITCH_FR), past the
		 * scaled window: the persistent tail joins the bound */
		int64_t tail = 0;
		for (int i = 2 + PITCH_FR; i < LPF_ORD + PITCH_FR; i++)
			tail += 2 * (int64_t) ((int32_t) sb[i] * sb[i]);
		f_pitch_scale_e(&sb[2], &sb[2], PITCH_FR, e, &ex, tail);
	}
#endif
	t = frac_pch(&sb[2 + PITCH_FR / 2], &pcorr, pest, 5, PITCHMIN, PITCHMAX,
		     PITCHMIN_Q7, PITCHMAX_Q7, 160, ex);
#if !defined(MELPE_OPCOUNT)
	/* The reference's two double_chk calls (pit_lib.c:650 / :663) differ only in
	 * the threshold t2 and run on the same window, so lanes of both
	 * branches share one call site (a wave with both kinds of lanes would
	 * run the check twice). */
	const bool low = pcorr < 9831;
	if (low) {
		v_copy(&sb[LPF_ORD], &speech[-PITCHMAX], PITCH_FR);
		int64_t tail = 0;
		for (int i = 2 + PITCH_FR; i < LPF_ORD + PITCH_FR; i++)
			tail += 2 * (int64_t) ((int32_t) sb[i] * sb[i]);
		f_pitch_scale(&sb[2], &sb[2], PITCH_FR, &ex, tail);
		t = frac_pch(&sb[LPF_ORD + PITCH_FR / 2], &pcorr, pest, 0, PITCHMIN, PITCHMAX,
			     PITCHMIN_Q7, PITCHMAX_Q7, 160, ex);
	}
	if (low && pcorr < 9012) {
		pitch = pavg;
	} else {
		t2 = low ? ((t > 12800) ? 89 : 115) : ((t > 12800) ? 64 : 96);
		pitch = double_chk(&sb[LPF_ORD + PITCH_FR / 2], &pcorr, t, t2, PITCHMIN, PITCHMAX,
				   PITCHMIN_Q7, PITCHMAX_Q7, 160, ex);
	}
#else
	if (pcorr < 9831) {
		v_copy(&sb[LPF_ORD], &speech[-PITCHMAX], PITCH_FR);
		/* the frac_pch calls below read up to sb[LPF_ORD + PITCH_FR): past
		 * the scaled sb[2 .. 2 + PITCH_FR), four unscaled speech samples
		 * join the bound */
		int64_t tail = 0;
		for (int i = 2 + PITCH_FR; i < LPF_ORD + PITCH_FR; i++)
			tail += 2 * (int64_t) ((int32_t) sb[i] * sb[i]);
		f_pitch_scale(&sb[2], &sb[2], PITCH_FR, &ex, tail);
		t = frac_pch(&sb[LPF_ORD + PITCH_FR / 2], &pcorr, pest, 0, PITCHMIN, PITCHMAX,
			     PITCHMIN_Q7, PITCHMAX_Q7, 160, ex);
		if (pcorr < 9012) {
			pitch = pavg;
		} else {
			t2 = (t > 12800) ? 89 : 115;
			pitch = double_chk(&sb[LPF_ORD + PITCH_FR / 2], &pcorr, t, t2, PITCHMIN,
					   PITCHMAX, PITCHMIN_Q7, PITCHMAX_Q7, 160, ex);
		}
	} else {
		t2 = (t > 12800) ? 64 : 96;
		pitch = double_chk(&sb[LPF_ORD + PITCH_FR / 2], &pcorr, t, t2, PITCHMIN, PITCHMAX,
				   PITCHMIN_Q7, PITCHMAX_Q7, 160, ex);
	}
#endif
	if (pcorr < 9012)
		pitch = pavg;
	*pcorr2 = pcorr;
	return pitch;
}

/* ------------------------------------------------------------------ */
/* bpvc_ana, melpe/melp_sub.c:77 -- 5-band bandpass voicing           */
/* ------------------------------------------------------------------ */
/* bpvc_ana's first-call zeroing of the band memories (melp_sub.c:91-101) */
MD void bpvc_init_band(EncAna *E, int b)
{
	BandState *B = &E->band[b];
	v_zero(B->fsp, PITCH_FR - FRAME);
	v_zero(B->delin, BPF_ORD);
	v_zero(B->delout, BPF_ORD);
	v_zero(B->env, ENV_ORD);
	B->env2 = 0;
}

MD void bpvc_init(EncAna *E)
{
	if (!E->bp_started) {
		for (int i = 0; i < NUM_BANDS; i++)
			bpvc_init_band(E, i);
		E->bp_started = 1;
	}
}

#if defined(MELPE_OPCOUNT)
/* census build: the reference's pass structure, op for op */
MN void bpvc_ana(EncAna *E, const int16_t *speech, const int16_t *fpitch, int16_t *bpvc,
		 Word16 *pitch)
{
	PROF_SCOPE(4);
	int16_t sb[BPF_ORD + PITCH_FR];
	Word16 pcorr, t, sc;
	const int16_t *bden = TB(bpf_den), *bnum = TB(bpf_num);
	bpvc_init(E);
	const int NEW = BPF_ORD + PITCH_FR - FRAME;	/* 147 */
	BandState *B = &E->band[0];
	v_copy(&sb[BPF_ORD], B->fsp, PITCH_FR - FRAME);
	v_copy(&sb[NEW], &speech[PITCH_FR - FRAME - PITCHMAX], FRAME);
	iir3_s(&sb[NEW], bden, bnum, B->delin, B->delout, FRAME, 0);
	v_copy(B->fsp, &sb[BPF_ORD + FRAME], PITCH_FR - FRAME);
	f_pitch_scale(&sb[BPF_ORD], &sb[BPF_ORD], PITCH_FR);
	*pitch = frac_pch(&sb[BPF_ORD + PITCHMAX], &bpvc[0], fpitch[0], 5, PITCHMIN, PITCHMAX,
			  PITCHMIN_Q7, PITCHMAX_Q7, 160);
	for (int i = 1; i < 2; i++) {	/* NUM_PITCHES */
		t = frac_pch(&sb[BPF_ORD + PITCHMAX], &pcorr, fpitch[i], 5, PITCHMIN, PITCHMAX,
			     PITCHMIN_Q7, PITCHMAX_Q7, 160);
		if (pcorr > bpvc[0]) {
			*pitch = t;
			bpvc[0] = pcorr;
		}
	}
	for (int i = 1; i < NUM_BANDS; i++) {
		B = &E->band[i];
		v_copy(&sb[BPF_ORD], B->fsp, PITCH_FR - FRAME);
		v_copy(&sb[NEW], &speech[PITCH_FR - FRAME - PITCHMAX], FRAME);
		int fi = i * (BPF_ORD / 2) * 3;
		iir3_s(&sb[NEW], bden + fi, bnum + fi, B->delin, B->delout, FRAME, 0);
		v_copy(B->fsp, &sb[BPF_ORD + FRAME], PITCH_FR - FRAME);
		sc = f_pitch_scale(&sb[BPF_ORD], &sb[BPF_ORD], PITCH_FR);
		frac_pch(&sb[BPF_ORD + PITCHMAX], &bpvc[i], *pitch, 0, PITCHMIN, PITCHMAX,
			 PITCHMIN_Q7, PITCHMAX_Q7, 160);
		/* envelope: the history samples are re-scaled to this frame's scale */
		t = shr(B->env2, sc);
		B->env2 = shr(sb[BPF_ORD + FRAME - 1], (Word16) -sc);
		v_equ_shr(&sb[BPF_ORD - ENV_ORD], B->env, sc, ENV_ORD);
		envelope(&sb[BPF_ORD], t, &sb[BPF_ORD], PITCH_FR);
		v_equ_shr(B->env, &sb[BPF_ORD + FRAME - ENV_ORD], (Word16) -sc, ENV_ORD);
		f_pitch_scale(&sb[BPF_ORD], &sb[BPF_ORD], PITCH_FR);
		frac_pch(&sb[BPF_ORD + PITCHMAX], &pcorr, *pitch, 0, PITCHMIN, PITCHMAX,
			 PITCHMIN_Q7, PITCHMAX_Q7, 160);
		pcorr = sub(pcorr, 1638);
		if (pcorr > bpvc[i])
			bpvc[i] = pcorr;
	}
}

#else

/* One band's pitch window w[0..PITCH_FR) (w = &sb[BPF_ORD]): the band's
 * filtered history bpfsp, then the new frame sp[0..FRAME) through the
 * band's three biquads, the new history written back as it is produced --
 * the reference's copy / iir / copy / f_pitch_scale-energy passes
 * (melp_sub.c:95-110, pit_lib.c:186-203) as one pass over the samples.
 * Returns the window's energy for f_pitch_scale_e. */
MD int64_t bp_window(int16_t *hist, const int16_t *sp, int16_t *w, const int16_t *den,
		     const int16_t *num, int16_t *din, int16_t *dout)
{
	PROF_SCOPE(47);
	const int H = PITCH_FR - FRAME;	/* 141 */
	int64_t e = 0;
#if MELPE_VBATCH_PAIRS
	/* hist and w dword-aligned: both moved two samples per access */
	{
		const u32_alias *hs = reinterpret_cast<const u32_alias *>(hist);
		u32_alias *wd = reinterpret_cast<u32_alias *>(w);
		int k = 0;
		#pragma unroll 1
		for (; k + 8 <= H / 2; k += 8) {
			uint32_t v[8];
			#pragma unroll
			for (int q = 0; q < 8; q++)
				v[q] = hs[k + q];
			#pragma unroll
			for (int q = 0; q < 8; q++) {
				wd[k + q] = v[q];
				e += L_mult(lo16(v[q]), lo16(v[q])) + (int64_t) L_mult(hi16(v[q]), hi16(v[q]));
			}
		}
		for (; k < H / 2; k++) {
			const uint32_t v = hs[k];
			wd[k] = v;
			e += L_mult(lo16(v), lo16(v)) + (int64_t) L_mult(hi16(v), hi16(v));
		}
		const int16_t v = hist[H - 1];
		w[H - 1] = v;
		e += L_mult(v, v);
	}
	/* the new history written back in pairs as it is produced */
	uint32_t pend = 0;
	iir3_s_io(sp, w + H, den, num, din, dout, FRAME, [&](int n, int16_t y) {
		e += L_mult(y, y);
		const int m = n - (FRAME - H);
		if (m >= 0) {
			if (m & 1)
				reinterpret_cast<u32_alias *>(hist)[m >> 1] = pend | ((uint32_t) (uint16_t) y << 16);
			else if (m == H - 1)
				hist[m] = y;
			else
				pend = (uint16_t) y;
		}
	});
	return e;
#else
	int k = 0;
	#pragma unroll 1
	for (; k + 8 <= H; k += 8) {	/* eight loads issued together */
		int16_t v[8];
		#pragma unroll
		for (int q = 0; q < 8; q++)
			v[q] = hist[k + q];
		#pragma unroll
		for (int q = 0; q < 8; q++) {
			w[k + q] = v[q];
			e += L_mult(v[q], v[q]);
		}
	}
	for (; k < H; k++) {
		int16_t v = hist[k];
		w[k] = v;
		e += L_mult(v, v);
	}
	iir3_s_io(sp, w + H, den, num, din, dout, FRAME, [&](int n, int16_t y) {
		e += L_mult(y, y);
		if (n >= FRAME - H)
			hist[n - (FRAME - H)] = y;
	});
	return e;
#endif
}

/* band 0 of bpvc_ana (melp_sub.c:104-135): the lowest band's window, the
 * better of the two pitch candidates' correlations -> bpvc[0], *pitch.
 * `speech` as bpvc_ana's. */
MN void bpvc_band0(EncAna *E, const int16_t *speech, const int16_t *fpitch, int16_t *bpvc0,
		   Word16 *pitch)
{
	alignas(4) int16_t sb[BPF_ORD + PITCH_FR];	/* w = sb + BPF_ORD dword-aligned */
	Word16 pcorr, t;
	BandState *B = &E->band[0];
	const int16_t *sp = &speech[PITCH_FR - FRAME - PITCHMAX];
	int16_t *w = &sb[BPF_ORD];
	int64_t e = bp_window(B->fsp, sp, w, TB(bpf_den), TB(bpf_num), B->delin, B->delout);
	bool ex = true;
	int lsh = 0;
	if (e <= (int64_t) LW_MAX_)	/* the scale read lazily, as in bpvc_band_s */
		lsh = shr(norm_l((Word32) e), 1);
	else
		f_pitch_scale_e(w, w, PITCH_FR, e, &ex);
	*pitch = frac_pch(&sb[BPF_ORD + PITCHMAX], bpvc0, fpitch[0], 5, PITCHMIN, PITCHMAX,
			  PITCHMIN_Q7, PITCHMAX_Q7, 160, ex, lsh);
	for (int i = 1; i < 2; i++) {	/* NUM_PITCHES */
		t = frac_pch(&sb[BPF_ORD + PITCHMAX], &pcorr, fpitch[i], 5, PITCHMIN, PITCHMAX,
			     PITCHMIN_Q7, PITCHMAX_Q7, 160, ex, lsh);
		if (pcorr > *bpvc0) {
			*pitch = t;
			*bpvc0 = pcorr;
		}
	}
}

/* band i = 1..4 of bpvc_ana (melp_sub.c:137-189): the band's window and
 * its envelope, each correlated at band 0's pitch; only band i's memories
 * B and bpvc[i] are touched, so the four bands are independent chains.
 * sp[0..FRAME) are the frame's new samples (`speech` + PITCH_FR - FRAME -
 * PITCHMAX for bpvc_ana's `speech`). */
MN void bpvc_band_s(BandState *B, const int16_t *sp, int i, Word16 pitch, int16_t *bpvci)
{
	alignas(4) int16_t sb[BPF_ORD + PITCH_FR];	/* w = sb + BPF_ORD dword-aligned */
	Word16 pcorr, t, sc;
	int16_t *w = &sb[BPF_ORD];
	const int fi = i * (BPF_ORD / 2) * 3;
	bool ex;
	int64_t e = bp_window(B->fsp, sp, w, TB(bpf_den) + fi, TB(bpf_num) + fi, B->delin, B->delout);
	if (e <= (int64_t) LW_MAX_) {
		/* f_pitch_scale (pit_lib.c:178-203) without its pass over the
		 * window: with the energy e = sum 2x^2 within 32 bits its scale is
		 * a left shift by lsh = norm_l(e) >> 1, and every scaled sample
		 * fits (2 (x 2^lsh)^2 <= e 2^(2 lsh) < 2^31), as does the scaled
		 * window's energy e 4^lsh, so the exact correlators apply.  The
		 * window stays unscaled; frac_pch and envelope shift each sample
		 * as they read it. */
		const int lsh = shr(norm_l((Word32) e), 1);
		sc = (Word16) -lsh;
		frac_pch(&sb[BPF_ORD + PITCHMAX], bpvci, pitch, 0, PITCHMIN, PITCHMAX, PITCHMIN_Q7,
			 PITCHMAX_Q7, 160, true, lsh);
		t = shr(B->env2, sc);
		B->env2 = shr((int16_t) (w[FRAME - 1] * (1 << lsh)), (Word16) -sc);
		v_equ_shr(&sb[BPF_ORD - ENV_ORD], B->env, sc, ENV_ORD);
		e = envelope_e(w, t, w, PITCH_FR, lsh);
		v_equ_shr(B->env, &sb[BPF_ORD + FRAME - ENV_ORD], (Word16) -sc, ENV_ORD);
		if (e <= (int64_t) LW_MAX_) {
			frac_pch(&sb[BPF_ORD + PITCHMAX], &pcorr, pitch, 0, PITCHMIN, PITCHMAX, PITCHMIN_Q7,
				 PITCHMAX_Q7, 160, true, shr(norm_l((Word32) e), 1));
		} else {
			f_pitch_scale_e(w, w, PITCH_FR, e, &ex);
			frac_pch(&sb[BPF_ORD + PITCHMAX], &pcorr, pitch, 0, PITCHMIN, PITCHMAX, PITCHMIN_Q7,
				 PITCHMAX_Q7, 160, ex);
		}
		pcorr = sub(pcorr, 1638);
		if (pcorr > *bpvci)
			*bpvci = pcorr;
		return;
	}
	sc = f_pitch_scale_e(w, w, PITCH_FR, e, &ex);
	frac_pch(&sb[BPF_ORD + PITCHMAX], bpvci, pitch, 0, PITCHMIN, PITCHMAX, PITCHMIN_Q7,
		 PITCHMAX_Q7, 160, ex);
	/* envelope: the history samples are re-scaled to this frame's scale */
	t = shr(B->env2, sc);
	B->env2 = shr(sb[BPF_ORD + FRAME - 1], (Word16) -sc);
	v_equ_shr(&sb[BPF_ORD - ENV_ORD], B->env, sc, ENV_ORD);
	e = envelope_e(w, t, w, PITCH_FR);
	v_equ_shr(B->env, &sb[BPF_ORD + FRAME - ENV_ORD], (Word16) -sc, ENV_ORD);
	f_pitch_scale_e(w, w, PITCH_FR, e, &ex);
	frac_pch(&sb[BPF_ORD + PITCHMAX], &pcorr, pitch, 0, PITCHMIN, PITCHMAX, PITCHMIN_Q7,
		 PITCHMAX_Q7, 160, ex);
	pcorr = sub(pcorr, 1638);
	if (pcorr > *bpvci)
		*bpvci = pcorr;
}

MN void bpvc_band(EncAna *E, const int16_t *speech, int i, Word16 pitch, int16_t *bpvci)
{
	bpvc_band_s(&E->band[i], &speech[PITCH_FR - FRAME - PITCHMAX], i, pitch, bpvci);
}

/* bpvc_ana, melpe/melp_sub.c:77 */
MN void bpvc_ana(EncAna *E, const int16_t *speech, const int16_t *fpitch, int16_t *bpvc,
		 Word16 *pitch)
{
	PROF_SCOPE(4);
	bpvc_init(E);
	bpvc_band0(E, speech, fpitch, &bpvc[0], pitch);
	for (int i = 1; i < NUM_BANDS; i++)
		bpvc_band(E, speech, i, *pitch, &bpvc[i]);
}

#endif

/* ------------------------------------------------------------------ */
/* melpe/pitch.c -- 8-candidate pitch tracker                          */
/* ------------------------------------------------------------------ */

/* ratio :591 / L_ratio :612 */
MD Word16 ratio(Word16 x, Word16 y)
{
	Word16 d = abs_s(sub(x, y));
	Word16 larger = (x > y) ? x : y;
	return divide_s(d, larger);
}

MD Word16 L_ratio(Word16 x, Word32 y)
{
	Word32 lx = L_deposit_l(x);
	Word32 d = L_sub(y, lx);
	if (d < 0)
		d = L_negate(d);
	Word32 larger = (lx > y) ? lx : y;
	return L_divider2(d, larger, 0, 0);
}

/* updateEn :633 */
MN Word16 updateEn(Word16 prev, Word16 ifact, Word16 curr)
{
	Word16 t = sub(shr(curr, 1), shr(prev, 1));
	if (t < negate(1024)) {
		t = shr(log10_fxp(ifact, 15), 1);
		return add(t, prev);
	}
	if (t > 3072) {
		t = shr(log10_fxp(sub(SW_MAX_, ifact), 15), 1);
		return add(t, curr);
	}
	t = shl(t, 2);
	t = pow10_fxp(t, 5);
	t = interp_scalar(t, 32, ifact);
	t = shr(log10_fxp(t, 5), 1);
	return add(prev, t);
}

/* ivfilt's three autocorrelation sums of the updated lp[0 .. PIT_COR_LEN)
 * (lags 0, 1, 2; each term 2 x y, as L40_mac): 219 terms of at most 2^31
 * never reach the 40-bit clamp, so the sums are exact integers and may be
 * formed in any order -- here while lpfilt moves the history down and
 * writes the new samples, instead of in a pass of their own */
struct LpAcor {
	int64_t a0, a1, a2;
	int16_t h1, h2;	/* the last two samples seen */
	int n;
	MM void add(int16_t x)
	{
		a0 += 2 * (int64_t) ((int32_t) x * x);
		if (n >= 1)
			a1 += 2 * (int64_t) ((int32_t) x * h1);
		if (n >= 2)
			a2 += 2 * (int64_t) ((int32_t) x * h2);
		h2 = h1;
		h1 = x;
		n++;
	}
};

/* lpfilt :100 */
MN void lpfilt(const int16_t *in, int16_t *lp, int len, LpAcor *ac = nullptr)
{
	const int16_t *lpar = TB(lpar);
	const Word16 c0 = lpar[0], c1 = lpar[1], c2 = lpar[2], c3 = lpar[3];
#if !defined(MELPE_OPCOUNT)
	if (ac)
		v_batch(&lp[len], lp, PIT_COR_LEN - len, [ac](int, int16_t x) {
			ac->add(x);
			return x;
		});
	else
#endif
	v_copy(lp, &lp[len], PIT_COR_LEN - len);
	/* the four past outputs in registers (the reference reads them back from
	 * lp), the inputs a block ahead; the taps in the reference's order */
	int16_t *y = &lp[PIT_COR_LEN - len];
	Word16 y1 = y[-1], y2 = y[-2], y3 = y[-3], y4 = y[-4];
	v_batch(in, y, len, [&](int, int16_t x) {
		Word32 s = L_shr(L_deposit_h(x), 3);
		s = L_mac(s, y1, c0);
		s = L_mac(s, y2, c1);
		s = L_mac(s, y3, c2);
		s = L_mac(s, y4, c3);
		Word16 o = r_ound(s);
		y4 = y3;
		y3 = y2;
		y2 = y1;
		y1 = o;
#if !defined(MELPE_OPCOUNT)
		if (ac)
			ac->add(o);
#endif
		return o;
	});
}

/* ivfilt :138 -- 2nd-order inverse filter from 40-bit autocorrelations;
 * ac: the sums, formed by lpfilt; *dcsum: remove_dc's sample sum of the
 * updated iv[0 .. PIT_COR_LEN) (an exact int sum), formed while the history
 * moves down and the new samples are written */
MN void ivfilt(int16_t *iv, const int16_t *lp, int len, const LpAcor *ac = nullptr,
	       Word32 *dcsum = nullptr)
{
	int16_t rc[3];
	Word16 pc1, pc2;
	Word32 dsum = 0;
#if !defined(MELPE_OPCOUNT)
	if (ac)
		v_batch(&iv[len], iv, PIT_COR_LEN - len, [&dsum](int, int16_t x) {
			dsum += x;
			return x;
		});
	else
#endif
	v_copy(iv, &iv[len], PIT_COR_LEN - len);
	/* the reference's three autocorrelation sums (lags 0, 1, 2) in one pass
	 * over lp, the samples in pairs (P16); each sum keeps its own chain in
	 * index order and the same terms */
	Word40 a0, a1, a2;
#if !defined(MELPE_OPCOUNT)
	if (ac) {
		a0 = ac->a0;
		a1 = ac->a1;
		a2 = ac->a2;
	} else
#endif
	{
	a0 = L40_mac(0, lp[0], lp[0]);
	a1 = L40_mac(0, lp[1], lp[0]);
	a0 = L40_mac(a0, lp[1], lp[1]);
	a2 = 0;
	{
		int16_t h1 = lp[1], h2 = lp[0];	/* lp[j - 1], lp[j - 2] */
		auto step = [&](int16_t x) {
			a0 = L40_mac(a0, x, x);
			a1 = L40_mac(a1, x, h1);
			a2 = L40_mac(a2, x, h2);
			h2 = h1;
			h1 = x;
		};
		P16 r;
		int np = p16_open(r, lp + 2, PIT_COR_LEN - 2);
		int j = 2;
		for (int k = 0; k < np; k++, j += 2) {
			uint32_t x = p16_next(r);
			step(lo16(x));
			step(hi16(x));
		}
		for (; j < PIT_COR_LEN; j++)
			step(lp[j]);
	}
	}
	Word16 sh = norm32(a0);
	rc[0] = r_ound((Word32) L40_shl(a0, sh));
	rc[1] = r_ound((Word32) L40_shl(a1, sh));
	rc[2] = r_ound((Word32) L40_shl(a2, sh));
	if (rc[0] == 0) {
		pc1 = pc2 = 0;
	} else {
		Word16 rc1 = divide_s(rc[1], rc[0]);
		Word16 t1 = mult(rc1, rc[1]);
		Word16 t2 = sub(rc[0], t1);
		Word16 t3 = sub(rc[2], t1);
		t1 = abs_s(t3);
		if (t1 > t2) {
			pc2 = -4096;
		} else {
			pc2 = divide_s(t1, t2);
			if (t3 < 0)
				pc2 = negate(pc2);
			pc2 = shr(pc2, 3);
		}
		pc1 = mult(rc1, pc2);
	}
	{	/* lp[k - 1], lp[k - 2] ride in registers, lp[k] a block ahead */
		const int k0 = PIT_COR_LEN - len;
		Word16 l1 = lp[k0 - 1], l2 = lp[k0 - 2];
		v_batch(&lp[k0], &iv[k0], len, [&](int, int16_t x) {
			Word32 t = L_shl(L_deposit_l(x), 13);
			t = L_sub(t, L_mult(pc1, l1));
			t = L_sub(t, L_mult(pc2, l2));
			l2 = l1;
			l1 = x;
			const Word16 o = r_ound(L_shl(t, 3));
			dsum += o;
			return o;
		});
	}
	if (dcsum)
		*dcsum = dsum;
}

/* normalised 40-bit correlation step shared by corPeak and frac_cor:
 * combines r0/rk normalisation and returns A/sqrt(r0 rk) in Q15 */
MN Word16 cor_gain(Word32 *Lr0, Word16 *r0s, Word16 rks, Word32 Lrk, Word40 A, bool clip_neg)
{
	Word16 sh = add(*r0s, rks);
	if (sh & 1) {
		*Lr0 = L_shr(*Lr0, 1);
		*r0s = sub(*r0s, 1);
		sh = add(*r0s, rks);
	}
	sh = shr(sh, 1);
	A = L40_shl(A, sh);
	Word16 root = sqrt_Q15(mult(extract_h(*Lr0), extract_h(Lrk)));
	Word16 t = extract_h((Word32) A);
	if (clip_neg && t < 0)
		t = 0;
	return divide_s(t, root);
}

MD void norm40(Word40 *acc, Word16 *sh, Word32 *L)
{
	if (*acc == 0)
		*acc = 1;
	*sh = norm32(*acc);
	*acc = L40_shl(*acc, *sh);
	*L = (Word32) *acc;
}

/* corPeak's peak list, kept in registers while the lags are scanned: up to
 * NODE local maxima ordered by value descending, ties in insertion order.
 * Peaks are inserted in the reference's scan order (lag MAXPITCH down to
 * MINPITCH), so equal values keep the higher lag first, which is the pick
 * melpe/pitch.c:351-359 makes (strict '>' scanning down from MAXPITCH).
 * Zero (non-peak) values never enter: empty slots hold 0. */
MD void peak_insert(int16_t *tv, int16_t *tj, int16_t v, int16_t j)
{
	#pragma unroll
	for (int k = NODE - 1; k >= 0; k--) {
		bool keep = tv[k] >= v;
		bool prev = k > 0 && tv[k > 0 ? k - 1 : 0] >= v;
		int16_t pv = k > 0 ? tv[k - 1] : v, pj = k > 0 ? tj[k - 1] : j;
		tv[k] = keep ? tv[k] : (prev ? v : pv);
		tj[k] = keep ? tj[k] : (prev ? j : pj);
	}
}

/* corPeak's lag block: acc[k] = sum_t pa[t + k / 2] * pq[t + 4 - (k + 1) / 2] */
struct CpLags {
	static constexpr int NA = 4, NB = 5;
	static constexpr int oa(int k) { return k / 2; }
	static constexpr int ob(int k) { return 4 - (k + 1) / 2; }
};

/* corPeak :216; dcsum: remove_dc's sample sum of in[0 .. PIT_COR_LEN),
 * already formed by ivfilt (null: remove_dc forms it) */
MN void corPeak(const int16_t *in, PitTrack *pt, ClassParam *cs, const Word32 *dcsum = nullptr)
{
	PROF_SCOPE(32);
	alignas(4) int16_t pb[PIT_COR_LEN];
	const int PW = PIT_COR_LEN - MAXPITCH;	/* 73 */
	if (dcsum) {
		const Word16 off = remove_dc_off(*dcsum, PIT_COR_LEN);
		v_batch(in, pb, PIT_COR_LEN, [off](int, int16_t x) { return sub(x, off); });
	} else {
		remove_dc(in, pb, PIT_COR_LEN);
	}
	Word40 r0 = 0, rk = 0, A = 0;
	Word16 r0s, rks;
	Word32 Lr0, Lrk;
	{	/* three opening sums, one paired pass */
		auto step = [&](int16_t u, int16_t v) {
			r0 = L40_mac(r0, u, u);
			rk = L40_mac(rk, v, v);
			A = L40_mac(A, u, v);
		};
		P16 ru, rv;
		int np = p16_open(ru, pb, PW), nv = p16_open(rv, pb + MAXPITCH, PW);
		np = np < nv ? np : nv;
		int i = 0;
		#pragma unroll 2
		for (int k = 0; k < np; k++, i += 2) {
			uint32_t x = p16_next(ru), y = p16_next(rv);
			step(lo16(x), lo16(y));
			step(hi16(x), hi16(y));
		}
		for (; i < PW; i++)
			step(pb[i], pb[i + MAXPITCH]);
	}
	norm40(&r0, &r0s, &Lr0);
	norm40(&rk, &rks, &Lrk);
	/* the reference keeps gp[20..147] and picks peaks afterwards
	 * (:298-359); here the gains of the last two lags stay in registers
	 * (g1 = gp[i+1], g2 = gp[i+2]) and each lag's peak value joins the
	 * register peak list as soon as its lower neighbour is known.  The
	 * sentinel -32768 stands for the missing neighbour at both ends
	 * (gains are >= 0), which reproduces the end-point rules. */
	int16_t tv[NODE], tj[NODE];
	for (int k = 0; k < NODE; k++) {
		tv[k] = 0;
		tj[k] = 0;
	}
	int16_t g1 = cor_gain(&Lr0, &r0s, rks, Lrk, A, true), g2 = -32768;
	int lo = 0, hi = MAXPITCH;
	/* The cross terms A of the lag loop are 73-term sums of 2*x*y with
	 * |x*y| <= 2^30, so |A| < 2^37 and the 40-bit clamp of L40_mac never
	 * acts: A is an exact integer sum, order-free.  Lags are taken in
	 * blocks of 8 (lag 146 - n for n = n0..n0+7, n0 even; window start
	 * lo = 1 + n/2) sharing the sample loads of one pass. */
	const int NL = MAXPITCH - MINPITCH;	/* 127 lags 146..20 */
	/* The last block (lags 26..19) takes the 7 remaining lags and one
	 * unused lag 19, whose reads stay inside pb (lo + PW + 19 < 219): one
	 * paired pass instead of seven scalar ones.  The census build keeps the
	 * reference's per-lag tail. */
#if defined(MELPE_OPCOUNT)
	const int NL_BLK = NL & ~7;
#else
	const int NL_BLK = (NL + 7) & ~7;
#endif
	int64_t blk[8];
	/* the r0 / rk updates' samples, loaded eight lags ahead (pb[lo + k],
	 * pb[lo + k + PW]; pb[hi - 1 - k], pb[hi - 1 - k + PW]), each register
	 * queue moving up by one per update */
	int16_t qa[4], qal[4], qb[4], qbl[4];
	{
	PROF_SCOPE(39);
	/* lag n = MAXPITCH - 1 - i; k8 = n & 7, a compile-time constant in the
	 * unrolled block loop below, so the block's sums stay in registers
	 * (indexed by a run-time n & 7 they went through scratch, one store per
	 * block and one load and wait per lag) */
	auto lag = [&](int n, int k8) __attribute__((always_inline)) {
		const int i = MAXPITCH - 1 - n;
		if (k8 == 0) {
			#pragma unroll
			for (int k = 0; k < 4; k++) {
				qa[k] = pb[lo + k];
				qal[k] = pb[lo + k + PW];
				qb[k] = pb[hi - 1 - k];
				qbl[k] = pb[hi - 1 - k + PW];
			}
		}
		if (k8 == 0 && n + 8 <= NL_BLK) {
			const int16_t *pa = &pb[1 + n / 2];
			const int16_t *pq = &pb[143 - n / 2];
#if !defined(MELPE_OPCOUNT)
			/* exact on packed pairs: the a samples split as 256 hi8 + lo8
			 * keep both halves' 73-term sums within 32 bits */
			int32_t hl[16];
			xcorr_pairs<8, CpLags, true>(pa, pq, PW, hl);
			for (int k = 0; k < 8; k++)
				blk[k] = 2 * (256 * (int64_t) hl[k] + hl[8 + k]);
#else
			int64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
			int a0 = pa[0], a1 = pa[1], a2 = pa[2];
			int q0 = pq[0], q1 = pq[1], q2 = pq[2], q3 = pq[3];
			auto step = [&](int a3, int q4) {
				acc[0] += (int64_t) (a0 * q4);
				acc[1] += (int64_t) (a0 * q3);
				acc[2] += (int64_t) (a1 * q3);
				acc[3] += (int64_t) (a1 * q2);
				acc[4] += (int64_t) (a2 * q2);
				acc[5] += (int64_t) (a2 * q1);
				acc[6] += (int64_t) (a3 * q1);
				acc[7] += (int64_t) (a3 * q0);
				a0 = a1;
				a1 = a2;
				a2 = a3;
				q0 = q1;
				q1 = q2;
				q2 = q3;
				q3 = q4;
			};
			/* pa[t + 3], pq[t + 4] two at a time (P16) */
			P16 ra, rq;
			int np = p16_open(ra, pa + 3, PW), nq = p16_open(rq, pq + 4, PW);
			np = np < nq ? np : nq;
			int t = 0;
			#pragma unroll 4
			for (int k = 0; k < np; k++, t += 2) {
				uint32_t x = p16_next(ra), y = p16_next(rq);
				step(lo16(x), lo16(y));
				step(hi16(x), hi16(y));
			}
			for (; t < PW; t++)
				step(pa[t + 3], pq[t + 4]);
			for (int k = 0; k < 8; k++)
				blk[k] = 2 * acc[k];
#endif
		}
		if (i % 2 == 0) {
			r0 = L40_shr((Word40) Lr0, r0s);
			r0 = L40_msu(r0, qa[0], qa[0]);	/* pb[lo], pb[lo + PW] */
			r0 = L40_mac(r0, qal[0], qal[0]);
			norm40(&r0, &r0s, &Lr0);
			lo++;
			#pragma unroll
			for (int k = 0; k < 3; k++) {
				qa[k] = qa[k + 1];
				qal[k] = qal[k + 1];
			}
		} else {
			hi--;
			rk = L40_shr((Word40) Lrk, rks);
			rk = L40_mac(rk, qb[0], qb[0]);	/* pb[hi], pb[hi + PW] */
			rk = L40_msu(rk, qbl[0], qbl[0]);
			norm40(&rk, &rks, &Lrk);
			#pragma unroll
			for (int k = 0; k < 3; k++) {
				qb[k] = qb[k + 1];
				qbl[k] = qbl[k + 1];
			}
		}
		if (n < NL_BLK) {
			A = blk[k8];
			OPC_ADD(OP_L40_mac, PW);	/* census: the reference's per-lag sum */
		} else {
			A = 0;
			for (int j = lo; j < lo + PW; j++)
				A = L40_mac(A, pb[j], pb[j + i]);
		}
		int16_t g = cor_gain(&Lr0, &r0s, rks, Lrk, A, true);
		/* lag i+1 is a peak when above both neighbours */
		peak_insert(tv, tj, (g1 > g2 && g1 > g) ? g1 : (int16_t) 0, (int16_t) (i + 1));
		g2 = g1;
		g1 = g;
	};
#if !defined(MELPE_OPCOUNT)
	for (int n0 = 0; n0 < NL; n0 += 8) {
		#pragma unroll
		for (int k8 = 0; k8 < 8; k8++)
			if (n0 + k8 < NL)
				lag(n0 + k8, k8);
	}
#else
	for (int n = 0; n < NL; n++)
		lag(n, n & 7);
#endif
	peak_insert(tv, tj, (g1 > g2) ? g1 : (int16_t) 0, (int16_t) MINPITCH);
	}
	PROF_SCOPE(40);
	/* The reference's NODE picks (:351-359): pick k is list entry k while
	 * the list has positive entries, then lag MAXPITCH with value 0 (no
	 * entry beats peak[MAXPITCH] once all are zero), and index[MAXPITCH]
	 * ends up pointing at the last such pick.  pit/weight list the picked
	 * lags in ascending order (:361-372), padded with (100, 0). */
	cs->pitch = (tv[0] > 0) ? tj[0] : (int16_t) MAXPITCH;
	cs->corx = tv[0];
	bool full = tv[NODE - 1] > 0, has_max = false;
	for (int k = 0; k < NODE; k++)
		has_max |= tv[k] > 0 && tj[k] == MAXPITCH;
	int16_t ej[NODE], ew[NODE];
	for (int k = 0; k < NODE; k++) {
		if (tv[k] > 0) {
			ej[k] = tj[k];
			ew[k] = (tj[k] == MAXPITCH && !full) ? (int16_t) 0 : tv[k];
		} else if (!has_max && (k == 0 || tv[k > 0 ? k - 1 : 0] > 0)) {
			ej[k] = MAXPITCH;	/* the first zero pick */
			ew[k] = 0;
		} else {
			ej[k] = 1000;	/* unused: sorts last, becomes (100, 0) */
			ew[k] = 0;
		}
	}
	#pragma unroll
	for (int r = 0; r < NODE; r++)	/* odd-even transposition sort on lag */
		#pragma unroll
		for (int k = r & 1; k + 1 < NODE; k += 2) {
			bool sw = ej[k] > ej[k + 1];
			int16_t a = ej[k], b = ej[k + 1], wa = ew[k], wb = ew[k + 1];
			ej[k] = sw ? b : a;
			ej[k + 1] = sw ? a : b;
			ew[k] = sw ? wb : wa;
			ew[k + 1] = sw ? wa : wb;
		}
	for (int k = 0; k < NODE; k++) {
		pt->pit[k] = (ej[k] == 1000) ? (int16_t) 100 : ej[k];
		pt->weight[k] = ew[k];
	}
	for (int i = 0; i < NODE - 1; i++)
		for (int j = i + 1; j < NODE; j++) {
			Word16 t1 = pt->pit[j], t2 = pt->pit[i], t = t2;
			while (t < t1)
				t = add(t, t2);
			t2 = sub(t, shr(t2, 1));
			if (t2 >= t1)
				t = sub(t, pt->pit[i]);
			t = abs_s(sub(pt->pit[j], t));
			t2 = divide_s(t, pt->pit[j]);
			if (t2 < 2621) {
				t1 = mult(pt->weight[i], 6554);
				t2 = sub(pt->weight[j], t1);
				if (t2 < 0)
					t2 = 0;
				pt->weight[j] = t2;
			}
		}
}

/* pitchAuto :63 */
MN void pitchAuto(EncAna *E, const int16_t *in, PitTrack *pt, ClassParam *cs)
{
	PROF_SCOPE(5);
	if (!E->pa.pauto_started) {
		v_zero(E->pa.lpbuf, PIT_COR_LEN);
		v_zero(E->pa.ivbuf, PIT_COR_LEN);
		E->pa.pauto_started = 1;
	}
#if !defined(MELPE_OPCOUNT)
	LpAcor ac = {0, 0, 0, 0, 0, 0};
	Word32 dcsum;
	lpfilt(in, E->pa.lpbuf, PIT_SUBFRAME, &ac);
	ivfilt(E->pa.ivbuf, E->pa.lpbuf, PIT_SUBFRAME, &ac, &dcsum);
	corPeak(E->pa.ivbuf, pt, cs, &dcsum);
#else
	lpfilt(in, E->pa.lpbuf, PIT_SUBFRAME);
	ivfilt(E->pa.ivbuf, E->pa.lpbuf, PIT_SUBFRAME);
	corPeak(E->pa.ivbuf, pt, cs);
#endif
}

/* multiCheck :433 */
MD Word16 multiCheck(Word16 f1, Word16 f2)
{
	if (f1 <= f2) {
		Word16 t = f1;
		f1 = f2;
		f2 = t;
	}
	Word16 m = f2;
	while (m <= f1)
		m = add(m, f2);
	if (sub(m, shr(f2, 1)) > f1)
		m = sub(m, f2);
	return ratio(f1, m);
}

/* trackPitch :471 */
MN Word16 trackPitch(Word16 pitch, const PitTrack *pt)
{
	Word16 idx = -1, co = SW_MIN_;
	for (int i = 0; i < NODE; i++) {
		Word16 t = shl(pt->pit[i], 7);
		if (ratio(t, pitch) < 6554 && pt->weight[i] > co) {
			co = pt->weight[i];
			idx = (Word16) i;
		}
	}
	if (idx < 0) {
		idx = 0;
		Word16 best = abs_s(sub(shl(pt->pit[0], 7), pitch));
		for (int i = 1; i < NODE; i++) {
			Word16 t = abs_s(sub(shl(pt->pit[i], 7), pitch));
			if (t < best) {
				idx = (Word16) i;
				best = t;
			}
		}
	}
	return idx;
}

/* pitLookahead :530 -- dynamic-programming look-ahead over the tracks */
MN Word16 pitLookahead(PitTrack *pt, int num)
{
	for (int i = 0; i < NODE; i++) {
		Word32 s = L_sub(LW_MAX_, L_deposit_h(pt[num].weight[i]));
		pt[num].cost[i] = extract_h(L_mult(extract_h(s), 3200));
	}
	for (int i = num - 1; i >= 0; i--)
		for (int j = 0; j < NODE; j++) {
			Word16 k = trackPitch(shl(pt[i].pit[j], 7), &pt[i + 1]);
			Word32 s = L_sub(LW_MAX_, L_deposit_h(pt[i].weight[j]));
			Word32 c = L_mult(extract_h(s), 3200);
			s = L_sub(L_deposit_h(pt[i].pit[j]), L_deposit_h(pt[i + 1].pit[k]));
			c = L_add(c, L_shl(L_abs(s), 5));
			c = L_add(c, L_deposit_h(pt[i + 1].cost[k]));
			pt[i].cost[j] = extract_h(c);
		}
	Word32 best = L_deposit_h(pt[0].cost[0]);
	int idx = 0;
	for (int i = 1; i < NODE; i++)
		if (L_deposit_h(pt[0].cost[i]) < best) {
			best = L_deposit_h(pt[0].cost[i]);
			idx = i;
		}
	return shl(pt[0].pit[idx], 7);
}

/* ------------------------------------------------------------------ */
/* melpe/classify.c                                                    */
/* ------------------------------------------------------------------ */

/* zeroCrosCount :404 */
#if !defined(MELPE_OPCOUNT)
/* zeroCrosCount given the subframe's sample sum: the signs of sp[i] - off
 * taken as the samples are read (pairs), the dc-free copy never written */
MN Word16 zeroCrosCount_s(const int16_t *sp, Word32 sum)
{
	const Word16 off = remove_dc_off(sum, PIT_SUBFRAME);
	Word16 cnt = 0;
	int ps = sub(sp[0], off) >= 0 ? 1 : -1;
	auto step = [&](int16_t x) {
		int cs = sub(x, off) >= 0 ? 1 : -1;
		cnt += ps + cs == 0;
		ps = cs;
	};
	P16 r;
	int np = p16_open(r, sp + 1, PIT_SUBFRAME - 1);
	int i = 1;
	#pragma unroll 4
	for (int k = 0; k < np; k++, i += 2) {
		uint32_t x = p16_next(r);
		step(lo16(x));
		step(hi16(x));
	}
	for (; i < PIT_SUBFRAME; i++)
		step(sp[i]);
	return divide_s(cnt, PIT_SUBFRAME);
}
#endif

MN Word16 zeroCrosCount(const int16_t *sp)
{
	int16_t d[PIT_SUBFRAME];
	remove_dc(sp, d, PIT_SUBFRAME);
	Word16 cnt = 0;
	int ps = d[0] >= 0 ? 1 : -1;
	for (int i = 1; i < PIT_SUBFRAME; i++) {
		int cs = d[i] >= 0 ? 1 : -1;
		if (ps + cs == 0)
			cnt++;
		ps = cs;
	}
	return divide_s(cnt, PIT_SUBFRAME);
}

/* bandEn :448 */
MN Word16 bandEn(const int16_t *ac, int band)
{
	const int16_t *cf = band == 0 ? TB(enlpf_coef) : TB(enhpf_coef);
	Word32 e = 0;
	for (int i = 1; i < 17; i++)
		e = L_add(e, L_deposit_l(mult(cf[i], ac[i])));
	e = L_shl(e, 1);
	e = L_add(e, L_deposit_l(mult(cf[0], ac[0])));
	if (e < 16384)
		return 0;
	return log10_fxp(extract_l(L_shr(e, 4)), 10);
}

/* The ten cross sums of frac_cor's full +-5 lag scan in one pass.  Lag
 * n = 0..9 is hp-1-n; its window starts at lo_n (the count of even lags in
 * [hp-1-n, hp-1], :540-560), so it reads in[lo_n + t] * in[lo_n + hp-1-n + t]
 * for t < win.  Relative to the first a-start and the last b-start those
 * offsets are compile-time constants once the parity of hp is fixed
 * (ODD: hp odd), both within 0..5, so one pass keeps six a- and six
 * b-samples in registers and loads two samples per t instead of twenty.
 * The sums are 2*x*y over at most 200 terms, |sum| < 2^39: the 40-bit
 * clamp of L40_mac never acts, so int64 sums are the reference's values. */
template <int ODD>
struct FcLags {
	static constexpr int NA = 6, NB = 6;
	static constexpr int lon(int n) { return ODD ? n / 2 + 1 : (n + 1) / 2; }
	static constexpr int oa(int n) { return lon(n) - (ODD ? 1 : 0); }
	static constexpr int ob(int n) { return lon(n) - n + 4; }
};

template <int ODD>
MD void fc_corr10(const int16_t *in, int hp, int win, Word40 *A)
{
	constexpr int lo0 = ODD ? 1 : 0, lo9 = 5;
	const int16_t *pa = &in[lo0], *pb = &in[lo9 + hp - 10];
#if !defined(MELPE_OPCOUNT)
	/* exact on packed pairs, a split as 256 hi8 + lo8 (win <= 200 terms) */
	{
		int32_t hl[20];
		xcorr_pairs<10, FcLags<ODD>, true>(pa, pb, win, hl);
		for (int n = 0; n < 10; n++)
			A[n] = 2 * (256 * (int64_t) hl[n] + hl[10 + n]);
		return;
	}
#endif
	int64_t acc[10];
	int av[6], bv[6];
	for (int k = 0; k < 10; k++)
		acc[k] = 0;
	for (int k = 0; k < 5; k++) {
		av[k] = pa[k];
		bv[k] = pb[k];
	}
	auto step = [&](int a5, int b5) {
		av[5] = a5;
		bv[5] = b5;
		#pragma unroll
		for (int n = 0; n < 10; n++) {
			int lon = ODD ? n / 2 + 1 : (n + 1) / 2;
			int ao = lon - lo0, bo = (lon - n) - (lo9 - 9);
			acc[n] += (int64_t) (av[ao] * bv[bo]);
		}
		#pragma unroll
		for (int k = 0; k < 5; k++) {
			av[k] = av[k + 1];
			bv[k] = bv[k + 1];
		}
	};
	/* pa[t + 5], pb[t + 5] two at a time (P16) */
	P16 ra, rb;
	int np = p16_open(ra, pa + 5, win), nb = p16_open(rb, pb + 5, win);
	np = np < nb ? np : nb;
	int t = 0;
	#pragma unroll 2
	for (int k = 0; k < np; k++, t += 2) {
		uint32_t x = p16_next(ra), y = p16_next(rb);
		step(lo16(x), lo16(y));
		step(hi16(x), hi16(y));
	}
	for (; t < win; t++)
		step(pa[t + 5], pb[t + 5]);
	for (int n = 0; n < 10; n++)
		A[n] = 2 * acc[n];
}

/* The same ten sums without a branch on the parity of hp.  Lanes of a wave
 * carry different pitches, so fc_corr10<0> and fc_corr10<1> would both run,
 * each on part of the wave.  Odd hp's lag n has the window of even hp+1's
 * lag n+1 (lo = n/2 + 1 = (n + 2)/2), so one pass of the even pattern over
 * eleven lags of hpe = hp + (hp & 1) holds both: lag n is sum n + (hp & 1).
 * The b-stream starts at in[hpe - 6], even for every lane, so the pair
 * streams of all lanes also share their alignment. */
struct FcLags11 {
	static constexpr int NA = 6, NB = 6;
	static constexpr int lon(int n) { return (n + 1) / 2; }
	static constexpr int oa(int n) { return lon(n); }
	static constexpr int ob(int n) { return lon(n) - n + 5; }
};

MD void fc_corr_any(const int16_t *in, int hp, int win, Word40 *A)
{
	const int odd = hp & 1;
	int32_t hl[22];
	xcorr_pairs<11, FcLags11, true>(in, &in[hp + odd - 6], win, hl);
	#pragma unroll
	for (int n = 0; n < 10; n++) {
		int32_t h = odd ? hl[n + 1] : hl[n], l = odd ? hl[12 + n] : hl[11 + n];
		A[n] = 2 * (256 * (int64_t) h + l);
	}
}

/* frac_cor :504 -- best normalised correlation within +-5 of pitch */
MN Word16 frac_cor(const int16_t *in, Word16 pitch)
{
	PROF_SCOPE(46);
#if defined(MELPE_DIAG_UNIFORM_PITCH)
	pitch = 80;	/* diagnostics only: every lane at one lag (wrong output) */
#endif
	Word16 lp = sub(pitch, 5), hp = add(pitch, 5);
	if (lp < MINPITCH)
		lp = MINPITCH;
	if (hp > MAXPITCH)
		hp = MAXPITCH;
	Word40 r0 = 0, rk = 0, A = 0;
	Word16 r0s, rks;
	Word32 Lr0, Lrk;
	Word16 win = sub(PIT_COR_LEN, hp);
	/* the reference's three opening sums (:520-530) in one pass: each keeps
	 * its own chain in index order */
	{
		auto step = [&](int16_t u, int16_t v) {
			r0 = L40_mac(r0, u, u);
			rk = L40_mac(rk, v, v);
			A = L40_mac(A, u, v);
		};
		P16 ru, rv;
		int np = p16_open(ru, in, win), nv = p16_open(rv, in + hp, win);
		np = np < nv ? np : nv;
		int i = 0;
		#pragma unroll 2
		for (int k = 0; k < np; k++, i += 2) {
			uint32_t x = p16_next(ru), y = p16_next(rv);
			step(lo16(x), lo16(y));
			step(hi16(x), hi16(y));
		}
		for (; i < win; i++)
			step(in[i], in[i + hp]);
	}
	norm40(&r0, &r0s, &Lr0);
	norm40(&rk, &rks, &Lrk);
	Word16 maxgp = cor_gain(&Lr0, &r0s, rks, Lrk, A, true);
	int lo = 0, hi = hp;
	Word40 blk[10];
#if !defined(MELPE_OPCOUNT)
	/* Lag hp-1-n's window does not depend on how many lags the scan has, so
	 * the ten-lag block holds the sums of a scan clamped at MINPITCH or
	 * MAXPITCH too (its first hp - lp lags; the unused lags read inside
	 * in[0 .. PIT_COR_LEN)).  One pass for every lane, instead of a
	 * per-lag scalar sum wherever a lane's pitch sits near either bound. */
	const bool blocked = true;
	fc_corr_any(in, hp, win, blk);
	/* The r0 / rk updates alternate with the parity of the lag, which
	 * differs between lanes: one update of the selected side per lag,
	 * branch-free (the reference's L40_msu / L40_mac pairs, in order).
	 * Lag i = hp - 1 - n for n < hp - lp <= 10, the loop unrolled so that
	 * blk[n] is a compile-time index (registers, not the private segment) */
	const int nl = hp - lp;
	#pragma unroll
	for (int n = 0; n < 10; n++) {
		if (n >= nl)
			continue;
		const Word16 i = hp - 1 - n;
		const bool ev = (i & 1) == 0;	/* i >= MINPITCH > 0 */
		hi -= !ev;
		const int ia = ev ? lo : hi;
		const int16_t x1 = in[ia], x2 = in[ia + win];
		const Word40 p1 = (Word40) x1 * x1 * 2, p2 = (Word40) x2 * x2 * 2;
		Word40 v = L40_shr((Word40) (ev ? Lr0 : Lrk), ev ? r0s : rks);
		v = clamp40(ev ? v - p1 : v + p1);
		v = clamp40(ev ? v + p2 : v - p2);
		Word16 vs;
		Word32 vL;
		norm40(&v, &vs, &vL);
		Lr0 = ev ? vL : Lr0;
		r0s = ev ? vs : r0s;
		Lrk = ev ? Lrk : vL;
		rks = ev ? rks : vs;
		lo += ev;
		if (blocked) {
			A = blk[n];
		} else {
			A = 0;
			for (int j = lo; j < lo + win; j++)
				A = L40_mac(A, in[j], in[j + i]);
		}
		Word16 g = cor_gain(&Lr0, &r0s, rks, Lrk, A, false);
		if (g > maxgp)
			maxgp = g;
	}
#else
	const bool blocked = (hp - lp) == 10;
	if (blocked) {
		if (hp & 1)
			fc_corr10<1>(in, hp, win, blk);
		else
			fc_corr10<0>(in, hp, win, blk);
	}
	for (Word16 i = sub(hp, 1); i >= lp; i--) {
		if (i % 2 == 0) {
			r0 = L40_shr((Word40) Lr0, r0s);
			r0 = L40_msu(r0, in[lo], in[lo]);
			r0 = L40_mac(r0, in[lo + win], in[lo + win]);
			norm40(&r0, &r0s, &Lr0);
			lo++;
		} else {
			hi--;
			rk = L40_shr((Word40) Lrk, rks);
			rk = L40_mac(rk, in[hi], in[hi]);
			rk = L40_msu(rk, in[hi + win], in[hi + win]);
			norm40(&rk, &rks, &Lrk);
		}
		if (blocked) {
			A = blk[hp - 1 - i];
			OPC_ADD(OP_L40_mac, win);	/* census: the reference's per-lag sum */
		} else {
			A = 0;
			for (int j = lo; j < lo + win; j++)
				A = L40_mac(A, in[j], in[j + i]);
		}
		Word16 g = cor_gain(&Lr0, &r0s, rks, Lrk, A, false);
		if (g > maxgp)
			maxgp = g;
	}
#endif
	return maxgp;
}

/* classify :92 -- silence/unvoiced/voiced/transition decision per 90-sample
 * subframe; cs[-1] is the previous subframe's parameters */
MN void classify(EncAna *E, const int16_t *in, ClassParam *cs, const int16_t *ac)
{
	PROF_SCOPE(6);
	/* so[2..222): the band-passed signal frac_cor reads; so[2..132) is
	 * the previous call's tail (back_sigbuf) except on the first call */
	alignas(4) int16_t so[BPF_ORD / 3 + PIT_COR_LEN];	/* so + 2 dword-aligned */
#if defined(MELPE_OPCOUNT)
	int16_t insp[PIT_SUBFRAME];
#else
	int16_t *insp = nullptr;
#endif
	const bool first = !E->cls.cls_started;
	const int KEEP = PIT_COR_LEN - PIT_SUBFRAME;	/* 130 */
	const int16_t *x;
	int16_t *y;
	int slen;
	if (first) {
		E->voicedEn = 10240;
		E->silenceEn = 6144;
		E->voicedCnt = 0;
		v_zero(E->cls.bpfdel, BPF_ORD + BPF_ORD / 3);
		slen = PIT_COR_LEN;
		x = &in[(PIT_SUBFRAME - PIT_COR_LEN) / 2];
		y = &so[2];
		E->cls.cls_started = 1;
	} else {
		slen = PIT_SUBFRAME;
		x = &in[(PIT_COR_LEN - PIT_SUBFRAME) / 2];
		y = &so[2 + KEEP];
		v_copy(&so[2], E->cls.back_sigbuf, KEEP);
	}
	/* The reference runs the three sections one after the other through
	 * ping-pong buffers (:126-168), section s reading its two past inputs
	 * from bpfdel[2s..2s+1] and past outputs from bpfdel[2s+2..2s+3] (the
	 * next section's past inputs).  Section s at sample j depends only on
	 * section s-1 at samples <= j, so the cascade runs sample by sample
	 * with the four two-sample histories in registers; what is left in
	 * bpfdel afterwards is the same last-two-samples of each stage. */
	{
		PROF_SCOPE(45);
		const int16_t *pn = TB(bpf_num), *pd = TB(bpf_den);
		Biq bq[3];
		for (int k = 0; k < 3; k++) {
			bq[k].n0 = pn[3 * k];
			bq[k].n1 = pn[3 * k + 1];
			bq[k].n2 = pn[3 * k + 2];
			bq[k].d1 = pd[3 * k + 1];
			bq[k].d2 = pd[3 * k + 2];
			bq[k].i0 = E->cls.bpfdel[2 * k + 1];
			bq[k].i1 = E->cls.bpfdel[2 * k];
			bq[k].o0 = E->cls.bpfdel[2 * k + 3];
			bq[k].o1 = E->cls.bpfdel[2 * k + 2];
		}
		/* inputs a block ahead (v_batch); slen is even, as the
		 * reference's pairwise loop assumes */
		v_batch(x, y, slen, [&](int, int16_t v) {
			return biq_step(bq[2], biq_step(bq[1], biq_step(bq[0], v)));
		});
		for (int k = 0; k < 3; k++) {
			E->cls.bpfdel[2 * k] = bq[k].i1;
			E->cls.bpfdel[2 * k + 1] = bq[k].i0;
		}
		E->cls.bpfdel[BPF_ORD] = bq[2].o1;
		E->cls.bpfdel[BPF_ORD + 1] = bq[2].o0;
	}
	v_copy(E->cls.back_sigbuf, &so[2 + PIT_SUBFRAME], KEEP);

	Word16 mx = 0, t1, t2, sh1 = 0;
	Word32 L1, L2 = 0;
#if defined(MELPE_OPCOUNT)
	for (int i = 0; i < PIT_SUBFRAME; i++) {
		t1 = abs_s(in[i]);
		if (mx < t1)
			mx = t1;
		L2 = L_add(L2, t1);
	}
	if (mx == 0) {
		L1 = 0;
	} else if (mx <= 4884) {
		L1 = L_v_magsq(in, PIT_SUBFRAME, 0, 0);
		sh1 = 0;
	} else {
		v_equ_shr(insp, in, 3, PIT_SUBFRAME);
		L1 = L_v_magsq(insp, PIT_SUBFRAME, 0, 0);
		sh1 = 6;
	}
#else
	/* one pass over the subframe (pairs) for the peak, the sum of |x|, both
	 * energy candidates (the L_mac chains of x^2 and of (x >> 3)^2, each in
	 * index order as L_v_magsq over in / insp) and zeroCrosCount's sample
	 * sum; the samples are read once more for the zero crossings */
	(void) insp;
	Word32 q0 = 0, q3 = 0, S = 0;
	{
		auto step = [&](int16_t x) {
			t1 = abs_s(x);
			mx = mx < t1 ? t1 : mx;
			L2 += t1;	/* <= 90 * 32768: L_add never clamps */
			S += x;
			q0 = L_mac(q0, x, x);
			const Word16 u = shr(x, 3);
			q3 = L_mac(q3, u, u);
		};
		P16 r;
		int np = p16_open(r, in, PIT_SUBFRAME);
		int i = 0;
		#pragma unroll 3
		for (int k = 0; k < np; k++, i += 2) {
			uint32_t x = p16_next(r);
			step(lo16(x));
			step(hi16(x));
		}
		for (; i < PIT_SUBFRAME; i++)
			step(in[i]);
	}
	if (mx == 0) {
		L1 = 0;
	} else if (mx <= 4884) {
		L1 = L_shr(q0, 1);
		sh1 = 0;
	} else {
		L1 = L_shr(q3, 1);
		sh1 = 6;
	}
#endif
	while (L1 > SW_MAX_) {
		L1 = L_shr(L1, 2);
		sh1 = add(sh1, 2);
	}
	if (L1 == 0) {
		cs->subEnergy = -20480;
	} else {
		t1 = shr(log10_fxp(extract_l(L1), 0), 1);
		t2 = extract_l(L_shr(L_mult(617, sh1), 1));
		cs->subEnergy = add(t1, t2);
	}
#if defined(MELPE_OPCOUNT)
	cs->zeroCrosRate = zeroCrosCount(in);
#else
	cs->zeroCrosRate = zeroCrosCount_s(in, S);
#endif
	if (L2 == 0) {
		cs->peakiness = 2048;
	} else {
		sh1 = add(sh1, 15);
		if (sh1 & 1) {
			t1 = extract_l(L_shr(L1, 1));
			sh1 = add(sh1, 1);
		} else {
			t1 = extract_l(L1);
		}
		sh1 = shr(sh1, 1);
		t1 = sqrt_Q15(t1);
		sh1 = sub(sh1, 8);
		t2 = extract_l(L_shr(L2, sh1));
		t1 = shr(t1, 7);
		t1 = divide_s(t1, t2);
		cs->peakiness = mult(19429, t1);
	}
	Word16 lhbd = sub(bandEn(ac, 0), bandEn(ac, 1));
	Word16 lbc = frac_cor(&so[2], cs->pitch);
	if (E->silenceEn > sub(E->voicedEn, 3072))
		E->silenceEn = sub(E->voicedEn, 3072);
	Word16 zcd = sub(cs->zeroCrosRate, cs[-1].zeroCrosRate);
	Word16 sed = sub(cs->subEnergy, cs[-1].subEnergy);
	const Word16 vEn = E->voicedEn, sEn = E->silenceEn;
	int16_t cl;
	if (cs->subEnergy < 6144) {
		cl = SILENCE;
	} else if (cs->subEnergy < interp_scalar(vEn, sEn, 21299)) {
		if (cs->zeroCrosRate > 19661 && (cs->corx < 13107 || lbc < 16384))
			cl = UNVOICED;
		else if (lbc > 22938 || (lbc > 13107 && cs->corx > 22938))
			cl = VOICED;
		else if (zcd > 9830 || sed > 4096 || cs->peakiness > 3277)
			cl = TRANSITION;
		else if (cs->zeroCrosRate > 18022 || (lhbd < 2048 && cs->zeroCrosRate > 13107))
			cl = UNVOICED;
		else
			cl = SILENCE;
	} else if (zcd > 6554 || sed > 4096 || cs->peakiness > 3277) {
		cl = (lbc > 22938 || cs->corx > 26214) ? VOICED : TRANSITION;
	} else if (cs->zeroCrosRate < 6554) {
		if (lbc > 16384 || (lbc > 9830 && cs->corx > 19661))
			cl = VOICED;
		else if (cs->subEnergy > interp_scalar(vEn, sEn, 9830))
			cl = (cs->peakiness > 3072) ? TRANSITION : VOICED;
		else
			cl = SILENCE;
	} else if (cs->zeroCrosRate < 16384) {
		if (lbc > 18022 || (lbc > 9830 && cs->corx > 21299))
			cl = VOICED;
		else if (cs->subEnergy < interp_scalar(vEn, sEn, 19661) && lhbd > 4096)
			cl = SILENCE;
		else if (cs->peakiness > 2867)
			cl = TRANSITION;
		else
			cl = UNVOICED;
	} else if (cs->zeroCrosRate < 22938) {
		if ((lbc > 19661 && cs->corx > 9830) || (lbc > 13107 && cs->corx > 22938))
			cl = VOICED;
		else if (cs->peakiness > 3072)
			cl = TRANSITION;
		else
			cl = UNVOICED;
	} else {
		if ((lbc > 21299 && cs->corx > 9830) || (lbc > 14746 && cs->corx > 22938))
			cl = VOICED;
		else if (cs->peakiness > 4096)
			cl = TRANSITION;
		else
			cl = UNVOICED;
	}
	cs->classy = cl;
}

/* ------------------------------------------------------------------ */
/* find_harm, melpe/fs_lib.c:62 -- Fourier magnitudes of the residual */
/* ------------------------------------------------------------------ */
/* find_harm's pitch-independent half: the scaled residual's 512-point real
 * FFT into hb (512 packed complex bins, re | im << 16) */
MN void find_harm_fft(const int16_t *in, uint32_t *hb, int len)
{
#if defined(MELPE_OPCOUNT)
	/* census build: the reference's sequence (fs_lib.c:78-95), the
	 * unpacked rfft with its per-stage block_max guards, same values */
	{
		Word16 m = 0;
		for (int i = 0; i < len; i++) {
			Word16 a = abs_s(in[i]);
			if (a > m)
				m = a;
		}
		Word16 sh = norm_s(m);
		int16_t buf[2 * 512];
		v_zero(buf, 2 * 512);
		for (int i = 0; i < len; i++)
			buf[i] = shl(in[i], sh);
		rfft(buf, 512);
		for (int k = 0; k < 512; k++)
			hb[k] = pk(buf[2 * k], buf[2 * k + 1]);
		return;
	}
#endif
	Word16 mx = 0;
	for (int i = 0; i < len; i++) {
		Word16 t = abs_s(in[i]);
		if (t > mx)
			mx = t;
	}
	Word16 sh = norm_s(mx);
	/* the 512 real input points as 256 complex pairs, zero padded past len;
	 * the scaled input's max |x| is the first guard test's block_max */
	Word16 smx = 0;
	for (int k = 0; k < 256; k++) {
		Word16 a = 2 * k < len ? shl(in[2 * k], sh) : (Word16) 0;
		Word16 b = 2 * k + 1 < len ? shl(in[2 * k + 1], sh) : (Word16) 0;
		hb[k] = pk(a, b);
		smx = pk_amax(hb[k], smx);
	}
	for (int k = 256; k < 512; k++)
		hb[k] = 0;
	rfft_pk(hb, 512, smx);
}

/* find_harm's second half: the peak magnitude around each pitch harmonic,
 * normalised */
MN void find_harm_mag(const uint32_t *hb, int16_t *fsmag, Word16 pitch, Word16 nh)
{
	Word32 Lm[NUM_HARM];
	v_set(fsmag, 8192, nh);
	Word16 fw = shr(divide_s(512, pitch), 2);
	Word16 iw = shr(fw, 6);
	Word16 i2 = shr(iw, 1);
	Word16 t1 = shr(pitch, 9);
	if (nh > t1)
		nh = t1;
	Word16 mfw = fw;
	for (int k = 0; k < nh; k++) {
		Word16 i0 = sub(shr(add(mfw, 32), 6), i2);
		Word32 Lmax = 0;
		for (int j = 0; j < iw; j++) {
			Word16 b = add(i0, (Word16) j);
			Word16 re = pk_re(hb[b]), im = pk_im(hb[b]);
			Word32 t = L_add(L_mult(re, re), L_mult(im, im));
			Lmax = Max_(Lmax, t);
		}
		Lm[k] = Lmax;
		mfw = add(mfw, fw);
	}
	Word40 avg = 1;
	for (int k = 0; k < nh; k++)
		avg = L40_add(avg, Lm[k]);
	t1 = norm32(avg);
	Word32 Lt = (Word32) L40_shl(avg, t1);
	t1 = sub(31, t1);
	Word16 t2 = divide_s(shl(nh, 10), extract_h(Lt));
	Word16 sh = sub(30, t1);
	for (int i = 0; i < nh; i++) {
		t1 = extract_h(L_shl(Lm[i], sh));
		t1 = extract_h(L_shl(L_mult(t1, t2), 2));
		fsmag[i] = sqrt_Q15(t1);
	}
}

MN void find_harm(const int16_t *in, int16_t *fsmag, Word16 pitch, Word16 nh, int len)
{
	PROF_SCOPE(12);
	uint32_t hb[512];
	find_harm_fft(in, hb, len);
	find_harm_mag(hb, fsmag, pitch, nh);
}

}  // namespace mlp

#endif
