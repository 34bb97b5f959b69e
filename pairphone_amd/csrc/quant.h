/*
 * quant.h -- 1200 bps quantisers and the 81-bit channel packing, encoder
 * side: restates melpe/qnt12.c (pitch_vq, gain_vq, lsf_vq, quant_bp,
 * quant_jitter, quant_fsmag), melpe/vq_lib.c (vq_lspw, vq_enc, vq_fsw),
 * melpe/melp_chn.c (low_rate_chn_write, parity) and melpe/fec_code.c
 * (low_rate_fec_code).  The sequential candidate-list updates of the
 * reference (wvq1 slot replacement, InsertCand) are kept in order, so ties
 * resolve exactly as there.
 */
#ifndef MELPE_QUANT_H
#define MELPE_QUANT_H

#include "analysis.h"

namespace mlp {

#define PITCH_VQ_CAND 16
#define LSP_VQ_CAND 8
#define LSP_VQ_STAGES 4
#define LSP_INP_CAND 5

/* vq_lspw, melpe/vq_lib.c:70 -- |A(e^jw)|^-0.3 weights */
MN void vq_lspw(int16_t *w, const int16_t *lsp, const int16_t *lpc, int order)
{
	for (int i = 0; i < order; i++)
		w[i] = L_pow_fxp(lpc_aejw(lpc, lsp[i], order), -9830, 19, 11);
	w[8] = mult(w[8], 20971);
	w[9] = mult(w[9], 5242);
}

#ifndef MELPE_SROW
#define MELPE_SROW 7
#endif
#ifndef MELPE_WMSE_POS
#define MELPE_WMSE_POS 1
#endif

/* vq_enc, melpe/vq_lib.c:474 -- full search, first minimum wins */
template <int ORDER>
MN Word32 vq_enc(const int16_t *cb, const int16_t *u_in, int levels, int16_t *uhat,
		 int16_t *index)
{
	const int order = ORDER;
	int16_t u[ORDER];	/* the target in registers for the codebook scan */
#pragma unroll
	for (int j = 0; j < ORDER; j++)
		u[j] = u_in[j];
	int16_t best = 0;
	Word32 dmin = LW_MAX_;
	const int16_t *p = cb;
#if !defined(MELPE_OPCOUNT)
	/* rows of an even order at an even table offset: ORDER / 2 dwords at a
	 * wave-uniform address (scalar loads), the next row's issued before
	 * this one is scored */
	if ((MELPE_SROW & 1) && !(ORDER & 1) && !((cb - g_tab) & 1)) {
		uint32_t rw[ORDER / 2 + 1];
		const u32_alias *r0 = reinterpret_cast<const u32_alias *>(cb);
		#pragma unroll
		for (int q = 0; q < ORDER / 2; q++)
			rw[q] = r0[q];
		for (int i = 0; i < levels; i++) {
			int16_t x[ORDER + 1];
			#pragma unroll
			for (int q = 0; q < ORDER / 2; q++) {
				x[2 * q] = lo16(rw[q]);
				x[2 * q + 1] = hi16(rw[q]);
			}
			const int in = i + 1 < levels ? i + 1 : i;
			const u32_alias *rn = reinterpret_cast<const u32_alias *>(cb + in * ORDER);
			#pragma unroll
			for (int q = 0; q < ORDER / 2; q++)
				rw[q] = rn[q];
			Word32 d = 0;
			#pragma unroll
			for (int j = 0; j < ORDER; j++) {
				Word16 t = sub(u[j], x[j]);
				d = L_mac(d, t, t);
			}
			if (d < dmin) {
				dmin = d;
				best = (int16_t) i;
			}
		}
		p = nullptr;
	} else
#endif
	for (int i = 0; i < levels; i++) {
		Word32 d = 0;
#pragma unroll
		for (int j = 0; j < ORDER; j++) {
			Word16 t = sub(u[j], *p++);
			d = L_mac(d, t, t);
		}
		if (d < dmin) {
			dmin = d;
			best = (int16_t) i;
		}
	}
	*index = best;
	v_copy(uhat, &cb[order * best], order);
	return dmin;
}

/* vq_fsw, melpe/vq_lib.c:512 -- Fourier-magnitude weights (init time) */
MD void vq_fsw(int16_t *wfs, int nh, Word16 pitch)
{
	Word16 w0 = divide_s(16384, pitch);
	for (int i = 0; i < nh; i++) {
		Word16 t = shl(add((Word16) i, 1), 11);
		t = extract_h(L_shl(L_mult(w0, t), 1));
		t = mult(t, t);
		Word32 L = L_add(268435456L, L_mult(22937, t));
		t = L_pow_fxp(L, 22609, 28, 13);
		t = mult(19200, t);
		wfs[i] = divide_s(3744, add(1600, t));
	}
}

/* ------------------------------------------------------------------ */
/* pitch VQ, melpe/qnt12.c:75-353                                      */
/* ------------------------------------------------------------------ */

/* wvq1's distortion of codebook row `row` (:221-260): the weighted terms in
 * j order with the reference's early exit once the sum reaches maxd.  The
 * terms are non-negative and L_add is monotone, so an exited sum is >= maxd,
 * like the full one: the exit never changes whether the entry is kept. */
template <int DIM>
MD Word32 wvq1_err(const int16_t *tgt, const int16_t *wt, const int16_t *row, Word32 maxd)
{
	Word32 err = 0;
	for (int j = 0; j < DIM; j++)
		if (wt[j] > 0) {
			Word16 t = sub(tgt[j], row[j]);
			err = L_add(err, L_shr(L_mult(t, t), 2));
			if (err >= maxd)
				break;
		}
	return err;
}

/* Rows of a 3-wide codebook at an even table offset, read through the
 * two dwords that hold row i (row i starts in the low half for even i) at
 * wave-uniform addresses (scalar loads); take() hands out row i and issues
 * the loads of the next row wanted.  Reads at most one sample past the
 * codebook's last row, inside g_tab. */
struct Row3 {
	const u32_alias *cw;
	uint32_t r0, r1;
	MM void open(const int16_t *cb, int i)
	{
		cw = reinterpret_cast<const u32_alias *>(cb);
		const int d = (3 * i) >> 1;
		r0 = cw[d];
		r1 = cw[d + 1];
	}
	MM void take(int i, int in, int16_t *x)
	{
		const bool odd = i & 1;
		x[0] = odd ? hi16(r0) : lo16(r0);
		x[1] = odd ? lo16(r1) : hi16(r0);
		x[2] = odd ? hi16(r1) : lo16(r1);
		const int d = (3 * in) >> 1;
		r0 = cw[d];
		r1 = cw[d + 1];
	}
};

/* wvq1's distortion of a row held in registers, every weighted term summed:
 * the terms are non-negative and L_add monotone, so the reference's early
 * exit (wvq1_err) never changes whether the entry is kept, and a kept
 * entry's sum is the full one either way */
MD Word32 wvq1_err3(const int16_t *tgt, const int16_t *wt, const int16_t *x)
{
	Word32 err = 0;
	#pragma unroll
	for (int j = 0; j < 3; j++) {
		Word16 t = sub(tgt[j], x[j]);
		Word32 v = L_add(err, L_shr(L_mult(t, t), 2));
		err = wt[j] > 0 ? v : err;
	}
	return err;
}

/* wvq1's update with entry i: it replaces the slot holding the current
 * maximum, then the linear rescan finds the new one (first slot wins).
 * Returns whether the entry was kept. */
MD bool wvq1_push(Word32 err, int i, int16_t *index, Word32 *dist, Word32 &maxd, int &maxi,
		  int cand)
{
	if (!(err < maxd))
		return false;
	index[maxi] = (int16_t) i;
	dist[maxi] = err;
	maxd = 0;
	for (int j = 0; j < cand; j++)
		if (dist[j] > maxd) {
			maxd = dist[j];
			maxi = j;
		}
	return true;
}

/* wvq1 :221 -- keeps `cand` best entries; a new entry replaces the slot
 * holding the current maximum, exactly as the reference's linear rescan */
template <int DIM>
MN void wvq1(const int16_t *tgt_in, const int16_t *wt_in, const int16_t *cb, int cbsize,
	     int16_t *index, Word32 *dist, int cand)
{
	int16_t tgt[DIM], wt[DIM];	/* in registers for the codebook scan */
#pragma unroll
	for (int j = 0; j < DIM; j++) {
		tgt[j] = tgt_in[j];
		wt[j] = wt_in[j];
	}
	for (int j = 0; j < cand; j++)
		dist[j] = LW_MAX_;
	Word32 maxd = LW_MAX_;
	int maxi = 0;
	/* one scan per distinct (codebook, size) among the active lanes, both
	 * wave-uniform inside: rows through the scalar cache (lspVQ_t) */
	const int o_lane = (int) (cb - g_tab);
	for (;;) {
		const int uo = wave_first(o_lane), un = wave_first(cbsize);
		if (o_lane != uo || cbsize != un)
			continue;
		const int16_t *ucb = g_tab + uo;
#if !defined(MELPE_OPCOUNT)
		if ((MELPE_SROW & 2) && DIM == 3 && !(uo & 1)) {
			Row3 rs;
			rs.open(ucb, 0);
			for (int i = 0; i < un; i++) {
				int16_t x[3];
				rs.take(i, i + 1 < un ? i + 1 : i, x);
				wvq1_push(wvq1_err3(tgt, wt, x), i, index, dist, maxd, maxi, cand);
			}
			break;
		}
#endif
		for (int i = 0; i < un; i++)
			wvq1_push(wvq1_err<DIM>(tgt, wt, ucb + i * DIM, maxd), i, index, dist, maxd, maxi,
				  cand);
		break;
	}
}

/* wvq2 :302 */
template <int DIM>
MN int16_t wvq2(const int16_t *tgt_in, const int16_t *wt_in, const int16_t *cb,
		const int16_t *index, const Word32 *dist, int cand)
{
	const int dim = DIM;
	int16_t tgt[DIM], wt[DIM];
#pragma unroll
	for (int j = 0; j < DIM; j++) {
		tgt[j] = tgt_in[j];
		wt[j] = wt_in[j];
	}
	Word32 mn = LW_MAX_;
	int16_t ind = 0;
	for (int i = 0; i < cand; i++) {
		Word32 err = dist[i];
		for (int j = 0; j < dim; j++)
			if (wt[j] > 0) {
				Word16 t = sub(tgt[j], cb[j]);
				err = L_add(err, L_shr(L_mult(t, t), 2));
				if (err >= mn)
					break;
			}
		if (err < mn) {
			mn = err;
			ind = index[i];
		}
		cb += dim;
	}
	return ind;
}

/* pitch_vq :75, in three parts so the multi-wave kernel can spread the
 * codebook search (ana_mw.h): the prelude (targets, weights, the
 * differential targets and their state; the scalar-quantiser and all-unvoiced
 * cases whole), the wvq1 search, and the finish (wvq2 and the outputs) */
struct PvqWork {
	int16_t tgt[NF], deltp[NF], deltw[NF], wt[NF];
	int16_t cnt;	/* voiced frames; the codebook search runs when >= 2 */
};

/* the codebook of the search: all voiced (2048 x 3) or two of three (512) */
MD int pvq_cb(const PvqWork &w, int *size)
{
	*size = w.cnt == NF ? 2048 : 512;
	return w.cnt == NF ? TOFF_pitch_vq_cb_vvv : TOFF_pitch_vq_cb_uvv;
}

MN int pvq_prelude(EncAna *E, MelpParam *par, PvqWork &w)
{
	QuantParam *q = &E->qpar;
	for (int i = 0; i < NF; i++)
		w.tgt[i] = log10_fxp(par[i].pitch, 7);
	int cnt = 0;
	for (int i = 0; i < NF; i++) {
		if (par[i].uv_flag) {
			w.wt[i] = 0;
		} else {
			w.wt[i] = 1;
			cnt++;
		}
	}
	w.cnt = (int16_t) cnt;
	for (int i = 0; i < NF; i++) {
		if (E->pvq_prev_uv_flag || par[i].uv_flag) {
			w.deltp[i] = 0;
			w.deltw[i] = 0;
		} else {
			w.deltp[i] = sub(w.tgt[i], E->pvq_prev_pitch);
			w.deltw[i] = 1;
		}
		E->pvq_prev_pitch = w.tgt[i];
		E->pvq_prev_uv_flag = par[i].uv_flag;
	}
	if (cnt == 0) {
		for (int i = 0; i < NF; i++)
			par[i].pitch = 50;	/* UV_PITCH (Q0, as the reference) */
		E->pvq_prev_qpitch = LOG_UV_PITCH_Q12;
	} else if (cnt == 1) {
		for (int i = 0; i < NF; i++) {
			if (!par[i].uv_flag) {
				quant_u(&w.tgt[i], &q->pitch_index, 5329, 9028, 98, 25088, true, 7);
				par[i].pitch = quant_u_dec(q->pitch_index, 5329, 9028, 25088, 7);
			} else {
				par[i].pitch = LOG_UV_PITCH_Q12;
			}
		}
		E->pvq_prev_qpitch = par[NF - 1].pitch;
		for (int i = 0; i < NF; i++)
			par[i].pitch = pow10_fxp(par[i].pitch, 7);
	}
	return cnt;
}

MN void pvq_finish(EncAna *E, MelpParam *par, const PvqWork &w, const int16_t *il,
		   const Word32 *dl)
{
	int size;
	const int16_t *cb = g_tab + pvq_cb(w, &size);
	int16_t dcb[PITCH_VQ_CAND * NF];
	Word16 k = 0;
	for (int i = 0; i < PITCH_VQ_CAND; i++) {
		Word16 t2 = extract_l(L_shr(L_mult(il[i], NF), 1));
		dcb[k] = sub(cb[t2], E->pvq_prev_qpitch);
		v_copy(&dcb[k + 1], &cb[t2 + 1], NF - 1);
		v_sub(&dcb[k + 1], &cb[t2], NF - 1);
		k = add(k, NF);
	}
	int16_t pi = wvq2<NF>(w.deltp, w.deltw, dcb, il, dl, PITCH_VQ_CAND);
	if (par[NF - 1].uv_flag)
		E->pvq_prev_qpitch = LOG_UV_PITCH_Q12;
	else
		E->pvq_prev_qpitch = cb[pi * NF + NF - 1];
	for (int i = 0; i < NF; i++)
		par[i].pitch = par[i].uv_flag ? (int16_t) UV_PITCH_Q7 : pow10_fxp(cb[pi * NF + i], 7);
	E->qpar.pitch_index = pi;
}

MN void pitch_vq(EncAna *E, MelpParam *par)
{
	PROF_SCOPE(10);
	PvqWork w;
	if (pvq_prelude(E, par, w) < 2)
		return;
	int size;
	const int16_t *cb = g_tab + pvq_cb(w, &size);
	int16_t il[PITCH_VQ_CAND];
	Word32 dl[PITCH_VQ_CAND];
	wvq1<NF>(w.tgt, w.wt, cb, size, il, dl, PITCH_VQ_CAND);
	pvq_finish(E, par, w, il, dl);
}

/* gain_vq :368 -- 1024 x 6 full search with the reference's early skip */
MN void gain_vq(EncAna *E, MelpParam *par)
{
	PROF_SCOPE(11);
	const int16_t *cb = TB(gain_vq_cb);
	int16_t tg[NF * NUM_GAINFR];
	for (int i = 0; i < NF; i++)
		v_copy(&tg[i * NUM_GAINFR], par[i].gain, NUM_GAINFR);
	Word32 minErr = LW_MAX_;
	int16_t idx = 0;
	Word16 b = 0;
#if !defined(MELPE_OPCOUNT)
	/* rows of six at an even offset: three dwords at a wave-uniform address
	 * (scalar loads), the next row's issued before this one is scored.
	 * Every row is scored whole: the terms are non-negative and L_add
	 * monotone, so the reference's skip after the first term (:380) never
	 * changes which row wins. */
	static_assert(NF * NUM_GAINFR == 6 && TOFF_gain_vq_cb % 2 == 0, "gain_vq rows as dwords");
	if (MELPE_SROW & 4) {
		const u32_alias *cw = reinterpret_cast<const u32_alias *>(cb);
		uint32_t r[3] = {cw[0], cw[1], cw[2]};
		for (int i = 0; i < 1024; i++) {
			int16_t x[6];
			#pragma unroll
			for (int q = 0; q < 3; q++) {
				x[2 * q] = lo16(r[q]);
				x[2 * q + 1] = hi16(r[q]);
			}
			const int in = i + 1 < 1024 ? i + 1 : i;
			#pragma unroll
			for (int q = 0; q < 3; q++)
				r[q] = cw[3 * in + q];
			Word32 err = 0;
			#pragma unroll
			for (int j = 0; j < 6; j++) {
				Word16 t = sub(tg[j], x[j]);
				err = L_add(err, L_shr(L_mult(t, t), 3));
			}
			if (err < minErr) {
				minErr = err;
				idx = (int16_t) i;
			}
		}
		b = 0;
	}
	if (!(MELPE_SROW & 4))
#endif
	for (int i = 0; i < 1024; i++) {
		Word16 t = sub(tg[0], cb[b]);
		Word32 err = L_add(0, L_shr(L_mult(t, t), 3));
		if (err < minErr) {
			for (int j = 1; j < NF * NUM_GAINFR; j++) {
				t = sub(tg[j], cb[b + j]);
				err = L_add(err, L_shr(L_mult(t, t), 3));
			}
			if (err < minErr) {
				minErr = err;
				idx = (int16_t) i;
			}
		}
		b = add(b, NF * NUM_GAINFR);
	}
	b = extract_l(L_shr(L_mult(idx, NF * NUM_GAINFR), 1));
	for (int i = 0; i < NF; i++) {
		v_copy(par[i].gain, &cb[b], NUM_GAINFR);
		b = add(b, NUM_GAINFR);
	}
	E->qpar.gain_index[0] = idx;
}

/* quant_bp :447 */
MD void quant_bp(EncAna *E, MelpParam *par)
{
	for (int i = 0; i < NF; i++) {
		par[i].uv_flag = q_bpvc(par[i].bpvc, &E->qpar.bpvc_index[i], NUM_BANDS);
		E->qpar.bpvc_index[i] = TB(bp_index_map)[E->qpar.bpvc_index[i]];
	}
}

/* ------------------------------------------------------------------ */
/* LSF MSVQ, melpe/qnt12.c:482-1138                                    */
/* ------------------------------------------------------------------ */

/* WeightedMSE :669 -- early exit after half the dimensions */
MN Word16 WeightedMSE(int n, const int16_t *w, const int16_t *x, const int16_t *tgt,
		      Word16 max_dmin)
{
	Word32 d = 0;
	Word16 half = shr((Word16) n, 1);
	for (int i = 0; i < half; i++) {
		Word16 t = sub(x[i], tgt[i]);
		d = L_mac(d, w[i], mult(t, t));
	}
	if (r_ound(d) >= max_dmin)
		return SW_MAX_;
	for (int i = half; i < n; i++) {
		Word16 t = sub(x[i], tgt[i]);
		d = L_mac(d, w[i], mult(t, t));
	}
	return r_ound(d);
}

/* InsertCand :735 -- ordered insert into the M-best list */
MN Word16 InsertCand(int c1, int s1, int16_t *dMin, Word16 dist, int16_t entry,
		     int16_t (*nextIndex)[LSP_VQ_STAGES], int16_t (*index)[LSP_VQ_STAGES])
{
	int i = 0;
	while (i < LSP_VQ_CAND && dist > dMin[i])
		i++;
	for (int j = LSP_VQ_CAND - 1; j > i; j--) {
		dMin[j] = dMin[j - 1];
		v_copy(nextIndex[j], nextIndex[j - 1], s1 + 1);
	}
	dMin[i] = dist;
	v_copy(nextIndex[i], index[c1], s1);
	nextIndex[i][s1] = entry;
	return dMin[LSP_VQ_CAND - 1];
}

/* WeightedMSE for a compile-time dimension, target and weights in
 * registers (same arithmetic and early exit as WeightedMSE) */
template <int DIM>
MD Word16 WeightedMSE_t(const int16_t *w, const int16_t *x, const int16_t *tgt, Word16 max_dmin)
{
	OPC_ADD(OP_shr, 1);	/* census: the reference's shr(n, 1) */
	Word32 d = 0;
#pragma unroll
	for (int i = 0; i < DIM / 2; i++) {
		Word16 t = sub(x[i], tgt[i]);
		d = L_mac(d, w[i], mult(t, t));
	}
	if (r_ound(d) >= max_dmin)
		return SW_MAX_;
#pragma unroll
	for (int i = DIM / 2; i < DIM; i++) {
		Word16 t = sub(x[i], tgt[i]);
		d = L_mac(d, w[i], mult(t, t));
	}
	return r_ound(d);
}

/* WeightedMSE_t when every weight is >= 0: each term L_mult(w, m) with
 * m = mult(t, t) >= 0 is 2 w m exactly (no saturation: w, m < 2^15), so the
 * saturating L_mac chain is min(MAX32, 2 S) with S the plain sum of w m,
 * at the half-way point and at the end.  S comes from saturating
 * v_dot2_i32_i16 (min(MAX32, S) for non-negative products) and 2 S
 * saturates exactly when S >= 2^30. */
template <int DIM>
MD Word16 WeightedMSE_pos(const int16_t *w, const int16_t *x, const int16_t *tgt, Word16 max_dmin)
{
	OPC_ADD(OP_shr, 1);
	int16_t m[DIM + 1];
#pragma unroll
	for (int i = 0; i < DIM; i++) {
		const int t = sub(x[i], tgt[i]);
		const int tt = (t * t) >> 15;
		m[i] = (int16_t) (tt > SW_MAX_ ? SW_MAX_ : tt);
	}
	m[DIM] = 0;
	auto pk = [](int16_t lo, int16_t hi) { return (uint32_t) (uint16_t) lo | ((uint32_t) (uint16_t) hi << 16); };
	auto dbl = [](int32_t S) { return S >= (1 << 30) ? (Word32) LW_MAX_ : (Word32) (2 * S); };
	constexpr int H = DIM / 2;
	int32_t S = 0;
#pragma unroll
	for (int i = 0; i < H; i += 2) {
		const bool one = i + 1 >= H;	/* the half's odd last term alone */
		S = sdot2_sat(pk(w[i], one ? (int16_t) 0 : w[i + 1]), pk(m[i], one ? (int16_t) 0 : m[i + 1]), S);
	}
	if (r_ound(dbl(S)) >= max_dmin)
		return SW_MAX_;
#pragma unroll
	for (int i = H; i < DIM; i += 2) {
		const bool one = i + 1 >= DIM;
		S = sdot2_sat(pk(w[i], one ? (int16_t) 0 : w[i + 1]), pk(m[i], one ? (int16_t) 0 : m[i + 1]), S);
	}
	return r_ound(dbl(S));
}

/* lspVQ :482 -- M-best multistage search; qout receives the ncPrev best
 * reconstructions (dim each), cb_index their stage indices (tos each).
 * Specialised per dimension (10: the LSF stages, 20: the interpolation
 * residual) so the target and weights of the codebook scan stay in
 * registers. */
template <int DIM>
MD void lspVQ_t(const int16_t *target, const int16_t *weight, int16_t *qout, const int16_t *cb,
		int tos, const int16_t *cb_size, int16_t *cb_index, bool flag)
{
	PROF_SCOPE(42);
	const int dim = DIM;
	int16_t index[LSP_VQ_CAND][LSP_VQ_STAGES], nextIndex[LSP_VQ_CAND][LSP_VQ_STAGES];
	int16_t cand[LSP_VQ_CAND][2 * LPC_ORD], dMin[LSP_VQ_CAND];
	int16_t wr[DIM];
	bool wpos = true;	/* every weight >= 0: WeightedMSE_pos */
#pragma unroll
	for (int i = 0; i < DIM; i++) {
		wr[i] = weight[i];
		wpos &= wr[i] >= 0;
	}
#if defined(MELPE_OPCOUNT) || !MELPE_WMSE_POS
	wpos = false;
#endif
	for (int i = 0; i < LSP_VQ_CAND; i++) {
		v_zero(cand[i], dim);
		v_zero(index[i], LSP_VQ_STAGES);
		v_zero(nextIndex[i], LSP_VQ_STAGES);
	}
	int ncPrev = 1;
	const int16_t *cbp = cb;
	Word16 off = 0;
	for (int s1 = 0; s1 < tos; s1++) {
		/* The M-best list of this stage lives in registers: distortions
		 * dm[] ascending and, per slot, a tag naming what InsertCand
		 * (:735-788) would have left in nextIndex[slot][0..s1]: (c1, e) for
		 * an entry inserted at this stage (index[c1][0..s1) followed by
		 * e), or -1-r for row r as it stood before the stage, shifted down
		 * by later inserts.  The network below is InsertCand's insert
		 * (before equal distortions, last slot evicted) on registers; the
		 * rows are written out once the stage's scan is done. */
		/* Each slot is one int32 key = dm * 65536 + tag bits: 0x8000 | r
		 * for row r, (c1 << 9) | e for a new entry (c1 < 8, e < 512).
		 * Bits below 2^16 never reorder distortions, so key < d * 65536
		 * exactly when dm < d, and a slot keeps or shifts in one compare
		 * and two selects.  Lanes insert at different entries, so the
		 * wave runs this network for most entries of a scan: its length
		 * is what the scan costs beyond WeightedMSE. */
		int32_t key[LSP_VQ_CAND];
#pragma unroll
		for (int k = 0; k < LSP_VQ_CAND; k++)
			key[k] = SW_MAX_ * 65536 + (0x8000 | k);
		Word16 maxd = SW_MAX_;
		for (int c1 = 0; c1 < ncPrev; c1++) {
			off = 0;
			int16_t ct[DIM];
#pragma unroll
			for (int i = 0; i < DIM; i++)
				ct[i] = sub(target[i], cand[c1][i]);
			/* The codebook rows are the same for every lane that scans
			 * this stage, so the scan runs once per distinct (codebook
			 * offset, size) among the active lanes -- once, unless the
			 * lanes took different branches of lsf_vq -- with both values
			 * wave-uniform: the rows then come through the scalar cache
			 * instead of per-lane vector loads. */
			const int o_lane = (int) (cbp - g_tab), n_lane = cb_size[s1];
			for (;;) {
				const int uo = wave_first(o_lane), un = wave_first(n_lane);
				if (o_lane != uo || n_lane != un)
					continue;
				const int16_t *ucb = g_tab + uo;
#if !defined(MELPE_OPCOUNT)
				/* Rows of an even dimension at an even table offset are
				 * dword-aligned: each row comes as DIM / 2 dwords at a
				 * wave-uniform address (scalar loads), the next row's
				 * issued before this one is scored */
				const bool srow = !(uo & 1);
				uint32_t rw[DIM / 2];
				if (srow) {
					const u32_alias *r0 = reinterpret_cast<const u32_alias *>(ucb);
					#pragma unroll
					for (int q = 0; q < DIM / 2; q++)
						rw[q] = r0[q];
				}
#endif
				for (int e = 0; e < un; e++) {
#if !defined(MELPE_OPCOUNT)
					Word16 d;
					if (srow) {
						int16_t x[DIM];
						#pragma unroll
						for (int q = 0; q < DIM / 2; q++) {
							x[2 * q] = lo16(rw[q]);
							x[2 * q + 1] = hi16(rw[q]);
						}
						const int en = e + 1 < un ? e + 1 : e;
						const u32_alias *rn = reinterpret_cast<const u32_alias *>(ucb + en * DIM);
						#pragma unroll
						for (int q = 0; q < DIM / 2; q++)
							rw[q] = rn[q];
						d = wpos ? WeightedMSE_pos<DIM>(wr, x, ct, maxd)
							 : WeightedMSE_t<DIM>(wr, x, ct, maxd);
					} else {
						d = WeightedMSE_t<DIM>(wr, ucb + e * DIM, ct, maxd);
					}
#else
					Word16 d = WeightedMSE_t<DIM>(wr, ucb + e * DIM, ct, maxd);
#endif
					if (d < maxd) {
						const int32_t dk = (int32_t) d * 65536;
						const int32_t nk = dk + ((c1 << 9) | e);
						bool kp[LSP_VQ_CAND];
#pragma unroll
						for (int k = 0; k < LSP_VQ_CAND; k++)
							kp[k] = key[k] < dk;
#pragma unroll
						for (int k = LSP_VQ_CAND - 1; k >= 0; k--)
							key[k] = kp[k] ? key[k] : ((k == 0 || kp[k > 0 ? k - 1 : 0]) ? nk : key[k > 0 ? k - 1 : 0]);
						maxd = (Word16) (key[LSP_VQ_CAND - 1] >> 16);
					}
					off = add(off, (Word16) dim);
				}
				break;
			}
		}
		{
			int16_t rows[LSP_VQ_CAND][LSP_VQ_STAGES];
			for (int k = 0; k < LSP_VQ_CAND; k++) {
				const int t = key[k] & 0xffff;
				if (!(t & 0x8000)) {
					int c1 = t >> 9;
					for (int i = 0; i < s1; i++)
						rows[k][i] = index[c1][i];
					rows[k][s1] = (int16_t) (t & 511);
				} else {
					for (int i = 0; i <= s1; i++)
						rows[k][i] = nextIndex[t & 0x7fff][i];
				}
			}
			for (int k = 0; k < LSP_VQ_CAND; k++)
				for (int i = 0; i <= s1; i++)
					nextIndex[k][i] = rows[k][i];
			for (int k = 0; k < LSP_VQ_CAND; k++)
				dMin[k] = (int16_t) (key[k] >> 16);
		}
		if (!flag && s1 == tos - 1) {
			ncPrev = 1;
		} else {
			Word16 t1 = extract_l(L_shr(L_mult((Word16) ncPrev, cb_size[s1]), 1));
			Word16 t2 = (s1 == tos - 1) ? LSP_INP_CAND : LSP_VQ_CAND;
			ncPrev = t1 < t2 ? t1 : t2;
		}
		for (int c1 = 0; c1 < ncPrev; c1++) {
			v_zero(cand[c1], dim);
			const int16_t *p2 = cb;
			v_copy(index[c1], nextIndex[c1], s1 + 1);
			for (int i = 0; i <= s1; i++) {
				Word16 o = extract_l(L_shr(L_mult(index[c1][i], (Word16) dim), 1));
				v_add(cand[c1], p2 + o, dim);
				p2 += extract_l(L_shr(L_mult(cb_size[i], (Word16) dim), 1));
			}
		}
		cbp += off;
	}
	for (int i = 0; i < ncPrev; i++) {
		v_copy(&cb_index[i * tos], index[i], tos);
		v_copy(&qout[i * dim], cand[i], dim);
	}
}

MN void lspVQ(const int16_t *target, const int16_t *weight, int16_t *qout, const int16_t *cb,
	      int tos, const int16_t *cb_size, int16_t *cb_index, int dim, bool flag)
{
	if (dim == 2 * LPC_ORD)
		lspVQ_t<2 * LPC_ORD>(target, weight, qout, cb, tos, cb_size, cb_index, flag);
	else
		lspVQ_t<LPC_ORD>(target, weight, qout, cb, tos, cb_size, cb_index, flag);
}

/* lspStable :805 (the reference also prints a warning when unstable) */
MD bool lspStable(int16_t *lsp, int order)
{
	if (lsp[0] < 52)
		lsp[0] = 52;
	for (int i = 0; i < order - 1; i++) {
		Word16 t = add(lsp[i], 205);
		if (lsp[i + 1] < t)
			lsp[i + 1] = t;
	}
	if (lsp[order - 1] > 32702)
		lsp[order - 1] = 32702;
	return !(lsp[order - 1] < lsp[order - 2]);
}

MD void lspSort(int16_t *lsp, int order)	/* :865 */
{
	for (int j = 1; j < order; j++) {
		int16_t t = lsp[j];
		int i = j - 1;
		while (i >= 0 && lsp[i] > t) {
			lsp[i + 1] = lsp[i];
			i--;
		}
		lsp[i + 1] = t;
	}
}

/* interpolation-error term of lsf_vq (qnt12.c:1019-1063): weighted square of
 * a Q15-scaled 32-bit difference through its normalised mantissa */
MD Word32 lsf_werr(Word32 acc, Word16 w)
{
	Word16 t1 = norm_l(acc);
	Word16 t2 = extract_h(L_shl(acc, t1));
	if (t2 == SW_MIN_)
		t2 = -32767;
	t2 = mult(t2, t2);
	Word32 r = L_mult(t2, w);
	t1 = shl(sub(1, t1), 1);
	return L_shl(r, sub(t1, 3));
}

/* the voicing pattern lsf_vq branches on (qnt12.c:934-941): frame 0 in bit 2 */
MD Word16 lsf_uvc(const MelpParam *par)
{
	Word16 uvc = 0;
	for (int i = 0; i < NF; i++)
		uvc = (Word16) ((uvc << 1) | (par[i].uv_flag ? 1 : 0));
	return uvc;
}

/* lsf_vq :895, on the voicing pattern uvc (lsf_uvc of the flags it sees) */
MN void lsf_vq_u(EncAna *E, MelpParam *par, Word16 uvc)
{
	PROF_SCOPE(9);
	QuantParam *q = &E->qpar;
	const int16_t melp_cb_size[4] = {256, 64, 32, 32};
	const int16_t res_cb_size[4] = {256, 64, 64, 64};
	const int16_t uv_cb_size[1] = {512};
	const int16_t *cb_uv = TB(lsp_uv_9), *cb_v = TB(lsp_v_256x64x32x32);
	int16_t lpc[LPC_ORD], wgt[NF][LPC_ORD], mwgt[2 * LPC_ORD];
	int16_t best0[LPC_ORD], best1[LPC_ORD], res[2 * LPC_ORD];
	int16_t lcand[LSP_INP_CAND][LPC_ORD], lidx[LSP_INP_CAND * LSP_VQ_STAGES];
	int16_t il0[LPC_ORD], il1[LPC_ORD];
	/* lsp(i) is par[i].lsf; written as a macro, not an array of pointers:
	 * a pointer loaded back from memory loses its address space and turns
	 * every access through it into a generic (FLAT) access */
#define lsp(i) (par[i].lsf)
	if (!E->lsf_started) {
		Word16 t2 = shl(LPC_ORD, 10), t1 = 819;
		for (int i = 0; i < LPC_ORD; i++) {
			E->qplsp[i] = divide_s(t1, t2);
			t1 = add(t1, 819);
		}
		E->lsf_started = 1;
	}
	{
	PROF_SCOPE(44);
	for (int i = 0; i < NF; i++) {
		lpc_lsp2pred(lsp(i), lpc, LPC_ORD);
		vq_lspw(wgt[i], lsp(i), lpc, LPC_ORD);
	}
	}
	if (uvc & 4)
		v_scale(wgt[0], 6554, LPC_ORD);
	if (uvc & 2)
		v_scale(wgt[1], 6554, LPC_ORD);
	/* One call site per quantisation, its codebook chosen per lane: the
	 * lanes of a wave carry different voicing patterns, and a call site per
	 * (branch, codebook) ran each scan once per site the wave's lanes
	 * used.  lspVQ's scan serialises over the distinct codebooks itself.
	 * Frame 2 is quantised the same way in both of the reference's branches
	 * (melp_cb or the 512-entry uv codebook by its own voicing), only the
	 * candidate list kept differs (flag), so it is one call. */
	const bool sep = uvc == 7 || uvc == 6 || uvc == 5 || uvc == 3;
	if (sep) {
		/* at most one voiced frame: each frame on its own */
		for (int i = 0; i < NF - 1; i++) {
			bool uv = (uvc >> (NF - 1 - i)) & 1;
			lspVQ(lsp(i), wgt[i], lsp(i), uv ? cb_uv : cb_v, uv ? 1 : 4,
			      uv ? uv_cb_size : melp_cb_size, q->lsf_index[i], LPC_ORD, false);
		}
	}
	const bool uv2 = uvc & 1;
	const int tos = uv2 ? 1 : 4;
	lspVQ(lsp(2), wgt[2], sep ? lsp(2) : lcand[0], uv2 ? cb_uv : cb_v, tos,
	      uv2 ? uv_cb_size : melp_cb_size, sep ? q->lsf_index[2] : lidx, LPC_ORD, !sep);
	if (!sep) {
		Word32 minErr = LW_MAX_;
		int cand = 0;
		int16_t inp = 0;
		const int16_t *ic = TB(inpCoef);
		{
		PROF_SCOPE(43);
#if !defined(MELPE_OPCOUNT)
		/* Every error term lsf_werr() is >= 0 when the weights are (they
		 * are: |A(e^jw)|^-0.3 scaled by 6554 at most), so each candidate's
		 * saturating L_add chain is min(LW_MAX, exact sum), whatever the
		 * term order.  That lets the search run j outer, the 16
		 * interpolation patterns inner: each j's six operands are loaded
		 * once per candidate instead of once per pattern, the frame-2 term
		 * (pattern-free) is added once, and the interpolated vectors are
		 * rebuilt only for the winner.  Candidates and patterns are still
		 * compared in the reference's order with strict '<'. */
		bool wpos = true;
		for (int f = 0; f < NF; f++)
			for (int j = 0; j < LPC_ORD; j++)
				wpos &= wgt[f][j] >= 0;
		EXACT_STAT(wpos ? 5 : 4);
		if (wpos) {
			for (int k = 0; k < LSP_INP_CAND; k++) {
				Word32 e3 = 0;
				for (int j = 0; j < LPC_ORD; j++) {
					Word32 acc = L_shl(L_deposit_l(lsp(2)[j]), 15);
					acc = L_sub(acc, L_shl(L_deposit_l(lcand[k][j]), 15));
					e3 = L_add(e3, lsf_werr(acc, wgt[2][j]));
				}
				/* four patterns at a time: their chains in registers; j
				 * in pairs, the coefficients of both as one dword per
				 * pattern and half at a wave-uniform address (scalar
				 * loads: inpCoef sits at an even offset, rows of 20) */
				static_assert(TOFF_inpCoef % 2 == 0 && LPC_ORD % 2 == 0, "inpCoef dwords");
				const u32_alias *ic32 = reinterpret_cast<const u32_alias *>(ic);
				#pragma unroll 1
				for (int i0 = 0; i0 < 16; i0 += 4) {
					Word32 errs[4] = {e3, e3, e3, e3};
					#pragma unroll 1
					for (int j0 = 0; j0 < LPC_ORD; j0 += 2) {
						uint32_t fa[4], fb[4];
						#pragma unroll
						for (int q = 0; q < 4; q++) {
							fa[q] = ic32[((i0 + q) * 20 + j0) >> 1];
							fb[q] = ic32[((i0 + q) * 20 + j0 + LPC_ORD) >> 1];
						}
						#pragma unroll
						for (int h = 0; h < 2; h++) {
							const int j = j0 + h;
							const Word16 qp = E->qplsp[j], lc = lcand[k][j];
							const Word32 l0 = L_shl(L_deposit_l(lsp(0)[j]), 15);
							const Word32 l1 = L_shl(L_deposit_l(lsp(1)[j]), 15);
							const Word16 w0 = wgt[0][j], w1 = wgt[1][j];
							#pragma unroll
							for (int q = 0; q < 4; q++) {
								Word16 f = h ? hi16(fa[q]) : lo16(fa[q]);
								Word32 acc = L_mac(L_mult(f, qp), sub(16384, f), lc);
								acc = L_sub(acc, l0);
								f = h ? hi16(fb[q]) : lo16(fb[q]);
								Word32 bcc = L_mac(L_mult(f, qp), sub(16384, f), lc);
								bcc = L_sub(bcc, l1);
								errs[q] = L_add(errs[q], lsf_werr(acc, w0));
								errs[q] = L_add(errs[q], lsf_werr(bcc, w1));
							}
						}
					}
					#pragma unroll
					for (int q = 0; q < 4; q++)
						if (errs[q] < minErr) {
							minErr = errs[q];
							cand = k;
							inp = (int16_t) (i0 + q);
						}
				}
			}
			for (int j = 0; j < LPC_ORD; j++) {
				Word16 f = ic[inp * 20 + j];
				Word32 acc = L_mac(L_mult(f, E->qplsp[j]), sub(16384, f), lcand[cand][j]);
				best0[j] = extract_h(L_shl(acc, 1));
				f = ic[inp * 20 + j + LPC_ORD];
				acc = L_mac(L_mult(f, E->qplsp[j]), sub(16384, f), lcand[cand][j]);
				best1[j] = extract_h(L_shl(acc, 1));
			}
		} else
#endif
		for (int k = 0; k < LSP_INP_CAND; k++)
			for (int i = 0; i < 16; i++) {
				Word32 err = 0;
				for (int j = 0; j < LPC_ORD; j++) {
					Word16 f = ic[i * 20 + j];
					Word32 acc = L_mult(f, E->qplsp[j]);
					acc = L_mac(acc, sub(16384, f), lcand[k][j]);
					il0[j] = extract_h(L_shl(acc, 1));
					acc = L_sub(acc, L_shl(L_deposit_l(lsp(0)[j]), 15));
					f = ic[i * 20 + j + LPC_ORD];
					Word32 bcc = L_mult(f, E->qplsp[j]);
					bcc = L_mac(bcc, sub(16384, f), lcand[k][j]);
					il1[j] = extract_h(L_shl(bcc, 1));
					bcc = L_sub(bcc, L_shl(L_deposit_l(lsp(1)[j]), 15));
					err = L_add(err, lsf_werr(acc, wgt[0][j]));
					err = L_add(err, lsf_werr(bcc, wgt[1][j]));
					acc = L_shl(L_deposit_l(lsp(2)[j]), 15);
					acc = L_sub(acc, L_shl(L_deposit_l(lcand[k][j]), 15));
					err = L_add(err, lsf_werr(acc, wgt[2][j]));
				}
				if (err < minErr) {
					minErr = err;
					cand = k;
					inp = (int16_t) i;
					v_copy(best0, il0, LPC_ORD);
					v_copy(best1, il1, LPC_ORD);
				}
			}
		}
		v_copy(lsp(2), lcand[cand], LPC_ORD);
		v_copy(q->lsf_index[0], &lidx[cand * tos], tos);
		q->lsf_index[1][0] = inp;
		for (int i = 0; i < LPC_ORD; i++) {
			res[i] = shl(sub(lsp(0)[i], best0[i]), 2);
			res[i + LPC_ORD] = shl(sub(lsp(1)[i], best1[i]), 2);
		}
		v_copy(mwgt, wgt[0], LPC_ORD);
		v_copy(mwgt + LPC_ORD, wgt[1], LPC_ORD);
		lspVQ(res, mwgt, res, TB(res256x64x64x64), uvc == 1 ? 4 : 2, res_cb_size,
		      q->lsf_index[2], 2 * LPC_ORD, false);
		for (int i = 0; i < LPC_ORD; i++) {
			lsp(0)[i] = add(shr(res[i], 2), best0[i]);
			lsp(1)[i] = add(shr(res[i + LPC_ORD], 2), best1[i]);
		}
	}
	lspStable(lsp(0), LPC_ORD);
	lspStable(lsp(1), LPC_ORD);
	if (!lspStable(lsp(2), LPC_ORD))
		lspSort(lsp(2), LPC_ORD);
	v_copy(E->qplsp, lsp(2), LPC_ORD);
#undef lsp
}

MN void lsf_vq(EncAna *E, MelpParam *par)
{
	lsf_vq_u(E, par, lsf_uvc(par));
}

/* quant_jitter :1198 */
MN void quant_jitter(EncAna *E, MelpParam *par)
{
	Word16 uvc = 0;
	int16_t jit[NF];
	for (int i = 0; i < NF; i++) {
		uvc = shl(uvc, 1);
		uvc |= par[i].uv_flag;
		jit[i] = par[i].jitter;
	}
	bool flag = false;
	switch (uvc) {
	case 6:
		flag = jit[2] == MAX_JITTER_Q15;
		break;
	case 5:
	case 4:
	case 1:
		flag = jit[1] == MAX_JITTER_Q15;
		break;
	case 3:
		flag = jit[0] == MAX_JITTER_Q15;
		break;
	case 0: {
		int c = 0;
		for (int i = 0; i < NF; i++)
			if (jit[i] == MAX_JITTER_Q15)
				c++;
		flag = c >= 2;
		break;
	}
	default:
		break;
	}
	for (int i = 0; i < NF; i++)
		jit[i] = par[i].uv_flag ? (int16_t) MAX_JITTER_Q15 : (int16_t) 0;
	if (flag && uvc == 0)
		jit[0] = jit[1] = jit[2] = MAX_JITTER_Q15;
	for (int i = 0; i < NF; i++)
		par[i].jitter = jit[i];
	E->qpar.jit_index[0] = flag;
}

/* quant_fsmag :1277 */
MN void quant_fsmag(EncAna *E, MelpParam *par)
{
	PROF_SCOPE(13);
	int16_t qmag[NUM_HARM];
	int cnt = 0, last = -1;
	for (int i = 0; i < NF; i++) {
		if (par[i].uv_flag) {
			v_set(par[i].fs_mag, 8192, NUM_HARM);
		} else {
			window_Q(par[i].fs_mag, g_der.w_fs, par[i].fs_mag, NUM_HARM, 14);
			last = i;
			cnt++;
		}
	}
	if (cnt > 0)
		vq_enc<NUM_HARM>(TB(fsvq_cb), par[last].fs_mag, 256, qmag, &E->qpar.fs_index);
	if (cnt > 1) {
		if (E->fsm_prev_uv || par[0].uv_flag) {
			for (int i = 0; i <= last; i++)
				if (!par[i].uv_flag)
					v_copy(par[i].fs_mag, qmag, NUM_HARM);
		} else if (par[1].uv_flag) {
			v_copy(par[0].fs_mag, E->fsm_prev_fsmag, NUM_HARM);
			v_copy(par[last].fs_mag, qmag, NUM_HARM);
		} else if (par[2].uv_flag) {
			v_copy(par[1].fs_mag, qmag, NUM_HARM);
			for (int i = 0; i < NUM_HARM; i++)
				par[0].fs_mag[i] = add(shr(qmag[i], 1), shr(E->fsm_prev_fsmag[i], 1));
		} else {
			v_copy(par[2].fs_mag, qmag, NUM_HARM);
			for (int i = 0; i < NUM_HARM; i++) {
				Word16 p = E->fsm_prev_fsmag[i], v = qmag[i];
				par[0].fs_mag[i] = add(mult(p, 21845), mult(v, 10923));
				par[1].fs_mag[i] = add(mult(p, 10923), mult(v, 21845));
			}
		}
	} else if (cnt == 1) {
		v_copy(par[last].fs_mag, qmag, NUM_HARM);
	}
	E->fsm_prev_uv = par[NF - 1].uv_flag;
	if (E->fsm_prev_uv)
		v_set(E->fsm_prev_fsmag, 8192, NUM_HARM);
	else
		v_copy(E->fsm_prev_fsmag, par[NF - 1].fs_mag, NUM_HARM);
}

/* ------------------------------------------------------------------ */
/* FEC + channel write, melpe/fec_code.c, melpe/melp_chn.c             */
/* ------------------------------------------------------------------ */

MD Word16 binprod(const int16_t *x, const int16_t *y, int n)	/* fec_code.c binprod_int */
{
	Word16 v = 0;
	for (int i = 0; i < n; i++)
		v ^= x[i] & y[i];
	return v;
}

/* vgetbits: dest[n-1..0] <- bits bit_pos..bit_pos-n+1 of source */
MD void vgetbits(int16_t *dest, Word16 src, Word16 bit_pos, Word16 n)
{
	if (n >= 0 && bit_pos >= sub(n, 1)) {
		src = shr(src, (Word16) (bit_pos - n + 1));
		for (int i = sub(n, 1); i >= 0; i--) {
			dest[i] = (int16_t) (src & 1);
			src = shr(src, 1);
		}
	}
}

/* vsetbits: bits bit_pos.. of *dest <- source[0..n-1] */
MD void vsetbits(int16_t *dest, Word16 bit_pos, Word16 n, const int16_t *src)
{
	if (n >= 0 && bit_pos >= n - 1)
		for (int i = 0, j = bit_pos; i < n; i++, j--) {
			*dest &= ~(1 << j);
			*dest |= src[i] << j;
		}
}

MD void sbc_enc(int16_t *x, int n, int k, const int16_t *pmat)
{
	for (int i = k; i < n; i++, pmat += k)
		x[i] = binprod(x, pmat, k);
}

MD void crc4_enc(int16_t *bit, int nbits)
{
	int16_t d[4] = {0, 0, 0, 0};
	int ll = nbits + 4;
	for (int i = 1; i <= nbits; i++) {
		int16_t x = (int16_t) (d[3] ^ bit[ll - i]);
		d[3] = d[2];
		d[2] = d[1];
		d[1] = (int16_t) (x ^ d[0]);
		d[0] = x;
	}
	v_copy(bit, d, 4);
}

/* low_rate_fec_code :955 -- protects all-unvoiced superframes */
MN void low_rate_fec_code(QuantParam *q)
{
	if (!(q->uv_flag[0] && q->uv_flag[1] && q->uv_flag[2]))
		return;
	int16_t c84[8], c74[7], c13[13];
	const int16_t *p84 = TB(pmat84), *p74 = TB(pmat74);
	vgetbits(c84, q->gain_index[0], 9, 4);
	sbc_enc(c84, 8, 4, p84);
	vsetbits(&q->fs_index, 7, 4, &c84[4]);
	vgetbits(c84, q->gain_index[0], 5, 4);
	sbc_enc(c84, 8, 4, p84);
	vsetbits(&q->fs_index, 3, 4, &c84[4]);
	vgetbits(c74, q->gain_index[0], 1, 2);
	c74[2] = c74[3] = 0;
	sbc_enc(c74, 7, 4, p74);
	vsetbits(&q->bpvc_index[0], 1, 2, &c74[4]);
	vsetbits(&q->jit_index[0], 0, 1, &c74[6]);
	for (int f = 0; f < NF; f++) {
		vgetbits(&c13[4], q->lsf_index[f][0], 8, 9);
		crc4_enc(c13, 9);
		vsetbits(&q->lsf_index[f][1], 3, 4, &c13[0]);
	}
}

MD Word16 parity(Word16 x, int len)	/* melp_chn.c:1367 */
{
	Word16 p = 0;
	for (int i = 0; i < len; i++) {
		p ^= x & 1;
		x >>= 1;
	}
	return p;
}

/* low_rate_chn_write :262 -- 81-bit superframe into chbuf (11 bytes) */
MN void low_rate_chn_write(EncAna *E)
{
	PROF_SCOPE(14);
	QuantParam *q = &E->qpar;
	unsigned char bb[81];
	BitCursor bc = {bb, 0};
	low_rate_fec_code(q);
	E->sync_bit = sub(1, E->sync_bit);
	pack_code(E->sync_bit, &bc, 1, 1);
	int cnt = 0;
	for (int i = 0; i < NF; i++)
		if (!q->uv_flag[i])
			cnt++;
	Word16 uv_index = 0, bp1 = 0, bp2 = 0, lsp_prot = 0;
	if (cnt <= 1) {
		if (!q->uv_flag[0])
			bp2 = 3;
		else if (!q->uv_flag[1])
			bp2 = 2;
		else if (!q->uv_flag[2])
			bp2 = 1;
		if (bp2 == 0)
			q->pitch_index = 0;	/* UV_PIND */
		else
			q->pitch_index = TB(low_rate_pitch_enc)[bp2 * 99 + q->pitch_index];
	} else if (cnt == 2) {
		if (q->uv_flag[0]) {
			uv_index = 4;
			bp1 = 3;
		} else if (q->uv_flag[1]) {
			uv_index = 2;
			bp1 = 2;
		} else if (q->uv_flag[2]) {
			uv_index = 1;
			bp1 = 1;
			lsp_prot = 7;
		}
	} else {
		uv_index = (int16_t) (q->pitch_index / 512);
		q->pitch_index = sub(q->pitch_index, (int16_t) (uv_index * 512));
		uv_index = TB(vvv_index_map)[uv_index];
	}
	pack_code(uv_index, &bc, 3, 1);
	pack_code(parity(uv_index, 3), &bc, 1, 1);
	pack_code(q->pitch_index, &bc, 9, 1);
	const int16_t u1 = q->uv_flag[0], u2 = q->uv_flag[1], cu = q->uv_flag[2];
	int16_t (*L)[MAX_LSF_STAGE] = q->lsf_index;
	if (u1 == 1 && u2 == 1 && cu == 1) {
		pack_code(L[0][0], &bc, 9, 1);
		pack_code(L[1][0], &bc, 9, 1);
		pack_code(L[2][0], &bc, 9, 1);
		pack_code(L[0][1], &bc, 4, 1);
		pack_code(L[1][1], &bc, 4, 1);
		pack_code(L[2][1], &bc, 4, 1);
		pack_code(lsp_prot, &bc, 3, 1);
	} else if (u1 == 1 && u2 == 1 && cu != 1) {
		pack_code(L[0][0], &bc, 9, 1);
		pack_code(L[1][0], &bc, 9, 1);
		pack_code(L[2][0], &bc, 8, 1);
		pack_code(L[2][1], &bc, 6, 1);
		pack_code(L[2][2], &bc, 5, 1);
		pack_code(L[2][3], &bc, 5, 1);
	} else if (u1 == 1 && u2 != 1 && cu == 1) {
		pack_code(L[0][0], &bc, 9, 1);
		pack_code(L[1][0], &bc, 8, 1);
		pack_code(L[1][1], &bc, 6, 1);
		pack_code(L[1][2], &bc, 5, 1);
		pack_code(L[1][3], &bc, 5, 1);
		pack_code(L[2][0], &bc, 9, 1);
	} else if (u1 != 1 && u2 == 1 && cu == 1) {
		pack_code(L[0][0], &bc, 8, 1);
		pack_code(L[0][1], &bc, 6, 1);
		pack_code(L[0][2], &bc, 5, 1);
		pack_code(L[0][3], &bc, 5, 1);
		pack_code(L[1][0], &bc, 9, 1);
		pack_code(L[2][0], &bc, 9, 1);
	} else {
		const bool vvu = (u1 != 1 && u2 != 1 && cu == 1);
		if (vvu) {
			pack_code(L[0][0], &bc, 9, 1);
		} else {
			pack_code(L[0][0], &bc, 8, 1);
			pack_code(L[0][1], &bc, 6, 1);
			pack_code(L[0][2], &bc, 5, 1);
			pack_code(L[0][3], &bc, 5, 1);
		}
		pack_code(L[1][0], &bc, 4, 1);
		if (vvu) {
			pack_code(L[2][0], &bc, 8, 1);
			pack_code(L[2][1], &bc, 6, 1);
			pack_code(L[2][2], &bc, 6, 1);
			pack_code(L[2][3], &bc, 6, 1);
			pack_code(lsp_prot, &bc, 3, 1);
		} else {
			pack_code(L[2][0], &bc, 8, 1);
			pack_code(L[2][1], &bc, 6, 1);
		}
	}
	pack_code(q->gain_index[0], &bc, 10, 1);
	for (int i = 0; i < NF; i++)
		if (!q->uv_flag[i])
			pack_code(q->bpvc_index[i], &bc, 2, 1);
	if (cnt == 2) {
		pack_code(bp1, &bc, 2, 1);
	} else if (cnt == 1) {
		pack_code(bp2, &bc, 2, 1);
		pack_code(bp1, &bc, 2, 1);
	} else if (cnt == 0) {
		pack_code(q->bpvc_index[0], &bc, 2, 1);
		pack_code(bp2, &bc, 2, 1);
		pack_code(bp1, &bc, 2, 1);
	}
	pack_code(q->fs_index, &bc, 8, 1);
	pack_code(q->jit_index[0], &bc, 1, 1);
	/* chbuf: LSB first, chwordsize = 8 (melpe.c:79); the reference's
	 * "|= 0x8000" on a byte (melp_chn.c:439) is a no-op */
	BitCursor cc = {E->chbuf, 0};
	for (int i = 0; i < 81; i++)
		pack_code(bb[i], &cc, 1, 8);
}

}  // namespace mlp

#endif
