/*
 * lsfvq_wave.h -- lsf_vq (melpe/qnt12.c:895-1138) of one channel on one
 * wavefront (k_lsf.hip).
 *
 * lsf_vq's control flow -- the voicing pattern's branch, the stages, the
 * stability fixes -- is per channel, so every lane runs it with the same
 * values.  The two searches are spread over the lanes:
 *   lspVQ (:482)  each stage's visits (c1-major, entry-minor, the
 *                 reference's order) are scored 64 at a time, lane t taking
 *                 visit base + t: WeightedMSE's half-way value p and full
 *                 value f.  The reference's visit enters the M-best list
 *                 iff p < worst and f < worst (:669-700: p >= worst returns
 *                 SW_MAX, which no worst exceeds), with worst the list's
 *                 current last distortion, which only falls.  So a visit
 *                 with max(p, f) >= the worst at the start of its batch is
 *                 rejected by the reference too, and the visits left are
 *                 replayed in order through InsertCand (:735, before equal
 *                 distortions, last slot evicted) with the test re-made --
 *                 the reference's list, for any weights.  Typically a few
 *                 visits of a batch survive the filter.
 *   the interpolation search (:1019-1063)  the 5 x 16 (candidate, pattern)
 *                 pairs, one per lane, each error the reference's chain;
 *                 the winner is the first minimum in the reference's order,
 *                 a wave minimum of (error, pair index).
 * Candidate reconstructions live in LDS (the lanes read them by candidate).
 */
#ifndef MELPE_LSFVQ_WAVE_H
#define MELPE_LSFVQ_WAVE_H

#include "encoder.h"
#include "npp_wave.h"

namespace mlp {
using wv::wsync;

/* lsf_vq's working set, shared by the wave in LDS: every value but the
 * per-visit scores and the candidate-rebuild elements is the same in all
 * lanes, which read it by broadcast; lanes store identical values */
struct LsfShared {
	int16_t lsf[NF][LPC_ORD], qplsp[LPC_ORD], wgt[NF][LPC_ORD], mwgt[2 * LPC_ORD];
	int16_t best0[LPC_ORD], best1[LPC_ORD], res[2 * LPC_ORD];
	int16_t lcand[LSP_INP_CAND][LPC_ORD], lidx[LSP_INP_CAND * LSP_VQ_STAGES];
	int16_t lsf_index[NF][MAX_LSF_STAGE];
	int16_t cand[LSP_VQ_CAND][2 * LPC_ORD];
};

/* lspVQ of one channel across the wave; cand: LDS, LSP_VQ_CAND rows */
template <int DIM>
MD void lspVQ_wv(const int16_t *target, const int16_t *weight, int16_t *qout, const int16_t *cb, int tos,
		 const int16_t *cb_size, int16_t *cb_index, bool flag, LsfShared *W, int lane)
{
	int16_t (*cand)[2 * LPC_ORD] = W->cand;
	/* the candidates' stage indices, row k's stage s in bits 16 s of
	 * ix[k] (index[][]) and nx[k] (nextIndex[][]): wave-uniform registers */
	uint64_t ix[LSP_VQ_CAND], nx[LSP_VQ_CAND];
	auto pick = [](const uint64_t *a, int k) {
		uint64_t v = a[0];
#pragma unroll
		for (int q = 1; q < LSP_VQ_CAND; q++)
			v = k == q ? a[q] : v;
		return v;
	};
	auto fld = [](uint64_t r, int st) { return (int16_t) (r >> (16 * st)); };
	int16_t wr[DIM], tg[DIM];
#pragma unroll
	for (int i = 0; i < DIM; i++) {
		wr[i] = weight[i];
		tg[i] = target[i];
	}
#pragma unroll
	for (int k = 0; k < LSP_VQ_CAND; k++)
		ix[k] = nx[k] = 0;
	for (int t = lane; t < LSP_VQ_CAND * 2 * LPC_ORD; t += WV)
		cand[t / (2 * LPC_ORD)][t % (2 * LPC_ORD)] = 0;
	wsync();
	int ncPrev = 1, cbo = 0;
	for (int s1 = 0; s1 < tos; s1++) {
		/* the M-best list as lspVQ_t's keys: dm * 65536 + tag, tag 0x8000 | r
		 * for row r as it stood, (c1 << 9) | e for a visit of this stage */
		int32_t key[LSP_VQ_CAND];
#pragma unroll
		for (int k = 0; k < LSP_VQ_CAND; k++)
			key[k] = SW_MAX_ * 65536 + (0x8000 | k);
		Word16 maxd = SW_MAX_;
		const int size = cb_size[s1], n = ncPrev * size;
		const int16_t *scb = cb + cbo;
		for (int base = 0; base < n; base += WV) {
			const int t = base + lane;
			Word16 p = SW_MAX_, f = SW_MAX_;
			if (t < n) {
				const int c1 = t / size, e = t - c1 * size;
				const int16_t *x = scb + e * DIM;
				Word32 d = 0;
#pragma unroll
				for (int i = 0; i < DIM / 2; i++) {
					Word16 u = sub(x[i], sub(tg[i], cand[c1][i]));
					d = L_mac(d, wr[i], mult(u, u));
				}
				p = r_ound(d);
#pragma unroll
				for (int i = DIM / 2; i < DIM; i++) {
					Word16 u = sub(x[i], sub(tg[i], cand[c1][i]));
					d = L_mac(d, wr[i], mult(u, u));
				}
				f = r_ound(d);
			}
			uint64_t m = __builtin_amdgcn_ballot_w64(t < n && p < maxd && f < maxd);
			while (m) {
				const int k = __builtin_ctzll(m);
				m &= m - 1;
				const Word16 pk = (Word16) __builtin_amdgcn_readlane((int) p, k);
				const Word16 fk = (Word16) __builtin_amdgcn_readlane((int) f, k);
				if (pk < maxd && fk < maxd) {
					const int tk = base + k, c1 = tk / size, e = tk - c1 * size;
					const int32_t dk = (int32_t) fk * 65536;
					const int32_t nk = dk + ((c1 << 9) | e);
					bool kp[LSP_VQ_CAND];
#pragma unroll
					for (int q = 0; q < LSP_VQ_CAND; q++)
						kp[q] = key[q] < dk;
#pragma unroll
					for (int q = LSP_VQ_CAND - 1; q >= 0; q--)
						key[q] = kp[q] ? key[q]
							       : ((q == 0 || kp[q > 0 ? q - 1 : 0]) ? nk : key[q > 0 ? q - 1 : 0]);
					maxd = (Word16) (key[LSP_VQ_CAND - 1] >> 16);
				}
			}
		}
		{
			/* InsertCand's rows (:735-788) from the keys' tags */
			uint64_t rw[LSP_VQ_CAND];
			const uint64_t lo = (1ull << (16 * s1)) - 1;
#pragma unroll
			for (int k = 0; k < LSP_VQ_CAND; k++) {
				const int t = key[k] & 0xffff;
				rw[k] = (t & 0x8000) ? pick(nx, t & 7)
						     : ((pick(ix, t >> 9) & lo) | ((uint64_t) (t & 511) << (16 * s1)));
			}
#pragma unroll
			for (int k = 0; k < LSP_VQ_CAND; k++)
				nx[k] = rw[k];
		}
		if (!flag && s1 == tos - 1) {
			ncPrev = 1;
		} else {
			Word16 t1 = extract_l(L_shr(L_mult((Word16) ncPrev, (Word16) size), 1));
			Word16 t2 = (s1 == tos - 1) ? LSP_INP_CAND : LSP_VQ_CAND;
			ncPrev = t1 < t2 ? t1 : t2;
		}
#pragma unroll
		for (int c1 = 0; c1 < LSP_VQ_CAND; c1++)
			if (c1 < ncPrev)
				ix[c1] = nx[c1];
		/* the new candidates, one element per lane: the stages' rows added
		 * in stage order (v_add) from zero */
		wsync();
		for (int t = lane; t < ncPrev * DIM; t += WV) {
			const int c1 = t / DIM, i = t - c1 * DIM;
			const int16_t *p2 = cb;
			Word16 v = 0;
			for (int st = 0; st <= s1; st++) {
				Word16 o = extract_l(L_shr(L_mult(fld(pick(ix, c1), st), (Word16) DIM), 1));
				v = add(v, p2[o + i]);
				p2 += extract_l(L_shr(L_mult(cb_size[st], (Word16) DIM), 1));
			}
			cand[c1][i] = v;
		}
		wsync();
		cbo += size * DIM;
	}
	/* one lane per element */
	for (int t = lane; t < ncPrev * tos; t += WV)
		cb_index[t] = fld(pick(ix, t / tos), t % tos);
	for (int t = lane; t < ncPrev * DIM; t += WV)
		qout[t] = cand[t / DIM][t % DIM];
	wsync();
}

/* the interpolation search (qnt12.c:1019-1063) of lsf_vq_u, pair
 * p = k * 16 + i on lane p and p - 64: the winner's candidate, pattern and
 * interpolated vectors */
MD void lsf_interp_wv(const LsfShared *W, int *cand, int16_t *inp, int16_t *best0, int16_t *best1, int lane)
{
	const int16_t *ic = TB(inpCoef);
	int64_t bk = (int64_t) 0x7fffffffffffffffLL;
	for (int pr = lane; pr < LSP_INP_CAND * 16; pr += WV) {
		const int k = pr >> 4, i = pr & 15;
		Word32 err = 0;
		for (int j = 0; j < LPC_ORD; j++) {
			Word16 f = ic[i * 20 + j];
			Word32 acc = L_mult(f, W->qplsp[j]);
			acc = L_mac(acc, sub(16384, f), W->lcand[k][j]);
			acc = L_sub(acc, L_shl(L_deposit_l(W->lsf[0][j]), 15));
			f = ic[i * 20 + j + LPC_ORD];
			Word32 bcc = L_mult(f, W->qplsp[j]);
			bcc = L_mac(bcc, sub(16384, f), W->lcand[k][j]);
			bcc = L_sub(bcc, L_shl(L_deposit_l(W->lsf[1][j]), 15));
			err = L_add(err, lsf_werr(acc, W->wgt[0][j]));
			err = L_add(err, lsf_werr(bcc, W->wgt[1][j]));
			acc = L_shl(L_deposit_l(W->lsf[2][j]), 15);
			acc = L_sub(acc, L_shl(L_deposit_l(W->lcand[k][j]), 15));
			err = L_add(err, lsf_werr(acc, W->wgt[2][j]));
		}
		/* strict '<' in the reference's order: the first minimum */
		const int64_t key = (int64_t) err * 128 + pr;
		bk = key < bk ? key : bk;
	}
#pragma unroll
	for (int o = 32; o >= 1; o >>= 1) {
		const int64_t v = __shfl_xor(bk, o);
		bk = v < bk ? v : bk;
	}
	const int pr = (int) (bk & 127);
	*cand = pr >> 4;
	*inp = (int16_t) (pr & 15);
	if (lane < LPC_ORD) {	/* one lane per element */
		const int j = lane;
		Word16 f = ic[*inp * 20 + j];
		Word32 acc = L_mac(L_mult(f, W->qplsp[j]), sub(16384, f), W->lcand[*cand][j]);
		best0[j] = extract_h(L_shl(acc, 1));
		f = ic[*inp * 20 + j + LPC_ORD];
		acc = L_mac(L_mult(f, W->qplsp[j]), sub(16384, f), W->lcand[*cand][j]);
		best1[j] = extract_h(L_shl(acc, 1));
	}
}

/* lsf_vq_u (quant.h) of one channel on the wave: E the channel's record
 * (global), aux its lsf_aux row, W the wave's LDS */
MD void lsf_vq_wv(EncState *E, const int16_t *aux, LsfShared *W, int lane)
{
	const int16_t melp_cb_size[4] = {256, 64, 32, 32};
	const int16_t res_cb_size[4] = {256, 64, 64, 64};
	const int16_t uv_cb_size[1] = {512};
	const int16_t *cb_uv = TB(lsp_uv_9), *cb_v = TB(lsp_v_256x64x32x32);
	const Word16 uvc = aux[0];
	/* the record's fields into LDS, one element per lane */
	for (int t = lane; t < NF * LPC_ORD; t += WV) {
		W->lsf[t / LPC_ORD][t % LPC_ORD] = E->par[t / LPC_ORD].lsf[t % LPC_ORD];
		W->wgt[t / LPC_ORD][t % LPC_ORD] = aux[LSF_AUX_WGT + t];
	}
	for (int t = lane; t < NF * MAX_LSF_STAGE; t += WV)
		W->lsf_index[t / MAX_LSF_STAGE][t % MAX_LSF_STAGE] =
			E->qpar.lsf_index[t / MAX_LSF_STAGE][t % MAX_LSF_STAGE];
	if (lane < LPC_ORD) {
		Word16 q = E->qplsp[lane];
		if (!E->lsf_started)	/* qnt12.c:911-920 */
			q = divide_s((Word16) (819 * (lane + 1)), shl(LPC_ORD, 10));
		W->qplsp[lane] = q;
	}
	wsync();
#define lsp(i) (W->lsf[i])
	const bool sep = uvc == 7 || uvc == 6 || uvc == 5 || uvc == 3;
	if (sep) {
		for (int i = 0; i < NF - 1; i++) {
			const bool uv = (uvc >> (NF - 1 - i)) & 1;
			lspVQ_wv<LPC_ORD>(lsp(i), W->wgt[i], lsp(i), uv ? cb_uv : cb_v, uv ? 1 : 4,
					  uv ? uv_cb_size : melp_cb_size, W->lsf_index[i], false, W, lane);
		}
	}
	const bool uv2 = uvc & 1;
	const int tos = uv2 ? 1 : 4;
	if (sep)
		lspVQ_wv<LPC_ORD>(lsp(2), W->wgt[2], lsp(2), uv2 ? cb_uv : cb_v, tos,
				  uv2 ? uv_cb_size : melp_cb_size, W->lsf_index[2], false, W, lane);
	else
		lspVQ_wv<LPC_ORD>(lsp(2), W->wgt[2], W->lcand[0], uv2 ? cb_uv : cb_v, tos,
				  uv2 ? uv_cb_size : melp_cb_size, W->lidx, true, W, lane);
	if (!sep) {
		int cnd;
		int16_t inp;
		lsf_interp_wv(W, &cnd, &inp, W->best0, W->best1, lane);
		wsync();
		if (lane < LPC_ORD) {	/* one lane per element */
			const int i = lane;
			lsp(2)[i] = W->lcand[cnd][i];
			W->res[i] = shl(sub(lsp(0)[i], W->best0[i]), 2);
			W->res[i + LPC_ORD] = shl(sub(lsp(1)[i], W->best1[i]), 2);
			W->mwgt[i] = W->wgt[0][i];
			W->mwgt[i + LPC_ORD] = W->wgt[1][i];
			if (i < tos)
				W->lsf_index[0][i] = W->lidx[cnd * tos + i];
			if (i == 0)
				W->lsf_index[1][0] = inp;
		}
		wsync();
		lspVQ_wv<2 * LPC_ORD>(W->res, W->mwgt, W->res, TB(res256x64x64x64), uvc == 1 ? 4 : 2,
				      res_cb_size, W->lsf_index[2], false, W, lane);
		if (lane < LPC_ORD) {
			const int i = lane;
			lsp(0)[i] = add(shr(W->res[i], 2), W->best0[i]);
			lsp(1)[i] = add(shr(W->res[i + LPC_ORD], 2), W->best1[i]);
		}
	}
	wsync();
	/* lspStable / lspSort on registers, then the record written back */
	int16_t l[NF][LPC_ORD];
	for (int f = 0; f < NF; f++)
		for (int i = 0; i < LPC_ORD; i++)
			l[f][i] = lsp(f)[i];
	lspStable(l[0], LPC_ORD);
	lspStable(l[1], LPC_ORD);
	if (!lspStable(l[2], LPC_ORD))
		lspSort(l[2], LPC_ORD);
#undef lsp
	for (int t = lane; t < NF * LPC_ORD; t += WV) {
		int16_t v = 0;
		for (int f = 0; f < NF; f++)
			for (int i = 0; i < LPC_ORD; i++)
				v = (t == f * LPC_ORD + i) ? l[f][i] : v;
		E->par[t / LPC_ORD].lsf[t % LPC_ORD] = v;
	}
	for (int t = lane; t < NF * MAX_LSF_STAGE; t += WV)
		E->qpar.lsf_index[t / MAX_LSF_STAGE][t % MAX_LSF_STAGE] =
			W->lsf_index[t / MAX_LSF_STAGE][t % MAX_LSF_STAGE];
	if (lane < LPC_ORD) {
		int16_t v = 0;
		for (int i = 0; i < LPC_ORD; i++)
			v = lane == i ? l[2][i] : v;
		E->qplsp[lane] = v;
	}
	if (lane == 0)
		E->lsf_started = 1;
}

}	// namespace mlp

#endif
