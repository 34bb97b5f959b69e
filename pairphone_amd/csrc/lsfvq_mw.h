/*
 * lsfvq_mw.h -- lsf_vq (melpe/qnt12.c:895-1138) of one channel spread over
 * the waves of the multi-wave analysis kernel (ana_mw.h).
 *
 * lsf_vq is a short chain of searches: per frame, or for frame 2 and then
 * the interpolation residual, an M-best multistage search lspVQ (qnt12.c:
 * 482) whose stages each score ncPrev x size codebook entries with
 * WeightedMSE (:669) and keep the eight best through InsertCand (:735),
 * plus, between the two lspVQs, the 5 x 16 interpolation-pattern search
 * (:1019-1063).  The scoring is the cost and is independent per entry; the
 * M-best update is cheap but order-dependent (ties).  So
 * each step is two phases:
 *   compute  every wave scores its contiguous slice of the visit sequence
 *            (c1-major, entry-minor): the rounded distortion after half the
 *            dimensions (WeightedMSE's early-exit test) and after all of
 *            them.  It runs the reference's M-best update on its slice
 *            alone and stores, in order, only the visits that update kept,
 *            with their (c1, entry) tag, in a per-channel row in HBM;
 *   scan     the leader (virtual wave 0) replays the reference's loop over
 *            the stored visits of slices 0..3 in order -- SW_MAX when the
 *            half-way value reaches the current worst, then InsertCand's
 *            insert.
 * Why skipping the other visits is exact: the M-best list holds the eight
 * smallest distortions d seen so far (an insert drops the largest, an equal
 * one is rejected), and with non-negative weights the half-way value is at
 * most the full one f, so a visit enters iff f < worst.  The slice's list has
 * seen a subset of the visits the reference's has at that point, so its
 * worst is >= the reference's: a visit the slice rejected, the reference
 * rejects.  A channel with a negative weight stores every visit (the scan is
 * then the sequential search itself, for any weights).
 * The interpolation search is split by (candidate, pattern) pairs in the
 * reference's order, each wave keeping its first minimum, the leader the
 * first minimum over the waves.
 *
 * The jobs of a channel depend on its voicing pattern (:956-1125): at most
 * one voiced frame -> an lspVQ per frame (1 stage for an unvoiced frame, 4
 * for a voiced one); otherwise lspVQ of frame 2 keeping 5 candidates, the
 * interpolation search, and lspVQ of the 20-dim residual (2 or 4 stages).
 * Every path fits LQ_SLOTS (compute, scan) pairs; a channel that finishes
 * early idles.  The channels of one wave may be on different steps.
 */
#ifndef MELPE_LSFVQ_MW_H
#define MELPE_LSFVQ_MW_H

#include "encoder.h"

namespace mlp {

/* steps of the longest path: frame 2 (4 stages) + interpolation + residual
 * (2 stages), or frame 2 unvoiced (1) + interpolation + residual (4); the
 * separate frames take at most 4 + 1 + 1 */
#define LQ_SLOTS 7
#define LQ_VISITS 512	/* the most entries one stage scores */
#define LQ_ROW 1024	/* dwords per channel of the score buffer (visits, pitch-VQ survivors) */
#define LQ_NV 4	/* slices per step (the schedule's virtual waves) */
#define LQ_BATCH 16	/* stored pairs read per batch by the leader's scan */
#ifndef MELPE_LQ_GATHER
#define MELPE_LQ_GATHER 1
#endif
#define LQ_SCAP (LQ_VISITS / LQ_NV)	/* stored visits per slice: every visit of the slice fits */
static_assert(LQ_NV * 2 * LQ_SCAP <= LQ_ROW, "lsf slices exceed the score row");

#define LQ_PAIRS (LSP_INP_CAND * 16)	/* interpolation (candidate, pattern) pairs */

/* the lsf block's exchange words (offsets from its base in the block) */
enum {
	XL_JOB = 0,	/* 0 idle, 1 an lspVQ stage, 2 the interpolation search */
	XL_DIM, XL_STAGE, XL_NC, XL_CB0LO, XL_CB0HI,	/* stage 0's codebook offset in g_tab */
	XL_SIZES,	/* [4] stage sizes */
	XL_ROWS = XL_SIZES + LSP_VQ_STAGES,	/* [8][4] index rows of the candidates */
	XL_TGT = XL_ROWS + LSP_VQ_CAND * LSP_VQ_STAGES,	/* [20] */
	XL_WGT = XL_TGT + 2 * LPC_ORD,	/* [20] */
	XL_NS = XL_WGT + 2 * LPC_ORD,	/* [LQ_NV] visits each slice stored */
	XL_PART = XL_NS + LQ_NV,	/* [LQ_NV][3] interpolation: err lo, hi, pair */
	XL_IP_LCAND = XL_PART + 3 * LQ_NV,	/* [5][10] frame 2's candidates */
	XL_IP_QPLSP = XL_IP_LCAND + LSP_INP_CAND * LPC_ORD,	/* [10] */
	XL_IP_LSP = XL_IP_QPLSP + LPC_ORD,	/* [3][10] the frames' LSFs */
	XL_IP_WGT = XL_IP_LSP + NF * LPC_ORD,	/* [3][10] their weights */
	XL_WORDS = XL_IP_WGT + NF * LPC_ORD
};

/* the leader's private state across the block's phases */
struct LsfLead {
	int16_t wgt[NF][LPC_ORD];
	int16_t uvc, sep, job, stage, tos, dim, flag, ncPrev, done, step;
	int16_t tgt[2 * LPC_ORD], wr[2 * LPC_ORD];
	int32_t cb0;
	int16_t sizes[LSP_VQ_STAGES];
	int16_t index[LSP_VQ_CAND][LSP_VQ_STAGES], nextIndex[LSP_VQ_CAND][LSP_VQ_STAGES];
	int16_t cand[LSP_VQ_CAND][2 * LPC_ORD];
	int16_t lcand[LSP_INP_CAND][LPC_ORD], lidx[LSP_INP_CAND * LSP_VQ_STAGES];
	int16_t best0[LPC_ORD], best1[LPC_ORD], tos2;
	int16_t ns[LQ_NV];	/* the step's stored visits per slice */
};

/* the stored pair of one visit: rounded half-way and full distortion */
MD uint32_t lq_pack(int16_t h, int16_t f)
{
	return (uint32_t) (uint16_t) h | ((uint32_t) (uint16_t) f << 16);
}

/* WeightedMSE (qnt12.c:669) without the exit: both values it may return on */
template <int DIM>
MD uint32_t lq_wmse(const int16_t *w, const int16_t *x, const int16_t *tgt)
{
	Word32 d = 0;
#pragma unroll
	for (int i = 0; i < DIM / 2; i++) {
		Word16 t = sub(x[i], tgt[i]);
		d = L_mac(d, w[i], mult(t, t));
	}
	Word16 h = r_ound(d);
#pragma unroll
	for (int i = DIM / 2; i < DIM; i++) {
		Word16 t = sub(x[i], tgt[i]);
		d = L_mac(d, w[i], mult(t, t));
	}
	return lq_pack(h, r_ound(d));
}

/* lq_wmse when every weight is >= 0 (WeightedMSE_pos's sums, quant.h) */
template <int DIM>
MD uint32_t lq_wmse_pos(const int16_t *w, const int16_t *x, const int16_t *tgt)
{
	int16_t m[DIM];
#pragma unroll
	for (int i = 0; i < DIM; i++) {
		const int t = sub(x[i], tgt[i]);
		const int tt = (t * t) >> 15;
		m[i] = (int16_t) (tt > SW_MAX_ ? SW_MAX_ : tt);
	}
	auto pk = [](int16_t lo, int16_t hi) { return (uint32_t) (uint16_t) lo | ((uint32_t) (uint16_t) hi << 16); };
	auto dbl = [](int32_t S) { return S >= (1 << 30) ? (Word32) LW_MAX_ : (Word32) (2 * S); };
	constexpr int H = DIM / 2;
	int32_t S = 0;
#pragma unroll
	for (int i = 0; i < H; i += 2) {
		const bool one = i + 1 >= H;
		S = sdot2_sat(pk(w[i], one ? (int16_t) 0 : w[i + 1]), pk(m[i], one ? (int16_t) 0 : m[i + 1]), S);
	}
	const Word16 h = r_ound(dbl(S));
#pragma unroll
	for (int i = H; i < DIM; i += 2) {
		const bool one = i + 1 >= DIM;
		S = sdot2_sat(pk(w[i], one ? (int16_t) 0 : w[i + 1]), pk(m[i], one ? (int16_t) 0 : m[i + 1]), S);
	}
	return lq_pack(h, r_ound(dbl(S)));
}

/* ---------------------------------------------------------------- */
/* leader                                                           */
/* ---------------------------------------------------------------- */

MD void lq_vq_start(LsfLead &L, const int16_t *tgt, const int16_t *wgt, int dim, int cb0,
		    const int16_t *sizes, int tos, bool flag)
{
	L.dim = (int16_t) dim;
	L.cb0 = cb0;
	L.tos = (int16_t) tos;
	L.flag = flag;
	L.stage = 0;
	L.ncPrev = 1;
	for (int i = 0; i < dim; i++) {
		L.tgt[i] = tgt[i];
		L.wr[i] = wgt[i];
	}
	for (int s = 0; s < LSP_VQ_STAGES; s++)
		L.sizes[s] = s < tos ? sizes[s] : (int16_t) 0;
	for (int k = 0; k < LSP_VQ_CAND; k++) {
		v_zero(L.cand[k], 2 * LPC_ORD);
		v_zero(L.index[k], LSP_VQ_STAGES);
		v_zero(L.nextIndex[k], LSP_VQ_STAGES);
	}
}

/* the codebooks of lsf_vq (qnt12.c:898-906) */
#define LQ_CB_UV (TOFF_lsp_uv_9)
#define LQ_CB_V (TOFF_lsp_v_256x64x32x32)
#define LQ_CB_RES (TOFF_res256x64x64x64)

MD void lq_frame_vq(LsfLead &L, MelpParam *par, int i, bool flag)
{
	const int16_t melp_sz[4] = {256, 64, 32, 32}, uv_sz[1] = {512};
	const bool uv = (L.uvc >> (NF - 1 - i)) & 1;
	lq_vq_start(L, par[i].lsf, L.wgt[i], LPC_ORD, uv ? LQ_CB_UV : LQ_CB_V, uv ? uv_sz : melp_sz,
		    uv ? 1 : 4, flag);
}

/* the job after `job` (sep: frames 0, 1, 2; else frame 2, interpolation,
 * residual), or done */
MD void lq_next_job(LsfLead &L, MelpParam *par, int job)
{
	L.job = (int16_t) job;
	if (job >= 3) {
		L.done = 1;
		return;
	}
	if (L.sep)
		lq_frame_vq(L, par, job, false);
	else if (job == 0)
		lq_frame_vq(L, par, NF - 1, true);
	/* job 1 (interpolation) has no lspVQ state; job 2 is started by the
	 * interpolation's reduction (it needs the residual) */
}

/* lsf_vq's prelude (qnt12.c:908-955): weights, voicing pattern, first job */
MD void lq_prelude(LsfLead &L, EncAna *E, MelpParam *par)
{
	int16_t lpc[LPC_ORD];
	if (!E->lsf_started) {
		Word16 t2 = shl(LPC_ORD, 10), t1 = 819;
		for (int i = 0; i < LPC_ORD; i++) {
			E->qplsp[i] = divide_s(t1, t2);
			t1 = add(t1, 819);
		}
		E->lsf_started = 1;
	}
	for (int i = 0; i < NF; i++) {
		lpc_lsp2pred(par[i].lsf, lpc, LPC_ORD);
		vq_lspw(L.wgt[i], par[i].lsf, lpc, LPC_ORD);
	}
	Word16 uvc = 0;
	for (int i = 0; i < NF; i++) {
		uvc = shl(uvc, 1);
		if (par[i].uv_flag) {
			uvc |= 1;
			if (i < 2)
				v_scale(L.wgt[i], 6554, LPC_ORD);
		}
	}
	L.uvc = uvc;
	L.sep = uvc == 7 || uvc == 6 || uvc == 5 || uvc == 3;
	L.done = 0;
	L.step = 0;
	lq_next_job(L, par, 0);
}

/* publish the next compute step */
template <class X>
MD void lq_publish(const LsfLead &L, const EncAna *E, const MelpParam *par, X &xc, int b)
{
	if (L.done) {
		xc.put(b + XL_JOB, 0);
		return;
	}
	if (!L.sep && L.job == 1) {
		xc.put(b + XL_JOB, 2);
		for (int k = 0; k < LSP_INP_CAND; k++)
			for (int j = 0; j < LPC_ORD; j++)
				xc.put(b + XL_IP_LCAND + k * LPC_ORD + j, L.lcand[k][j]);
		for (int j = 0; j < LPC_ORD; j++)
			xc.put(b + XL_IP_QPLSP + j, E->qplsp[j]);
		for (int f = 0; f < NF; f++)
			for (int j = 0; j < LPC_ORD; j++) {
				xc.put(b + XL_IP_LSP + f * LPC_ORD + j, par[f].lsf[j]);
				xc.put(b + XL_IP_WGT + f * LPC_ORD + j, L.wgt[f][j]);
			}
		return;
	}
	xc.put(b + XL_JOB, 1);
	xc.put(b + XL_DIM, L.dim);
	xc.put(b + XL_STAGE, L.stage);
	xc.put(b + XL_NC, L.ncPrev);
	xc.put(b + XL_CB0LO, (int16_t) (L.cb0 & 0xffff));
	xc.put(b + XL_CB0HI, (int16_t) (L.cb0 >> 16));
	for (int s = 0; s < LSP_VQ_STAGES; s++)
		xc.put(b + XL_SIZES + s, L.sizes[s]);
	for (int k = 0; k < LSP_VQ_CAND; k++)
		for (int s = 0; s < LSP_VQ_STAGES; s++)
			xc.put(b + XL_ROWS + k * LSP_VQ_STAGES + s, L.index[k][s]);
	if (L.stage == 0)
		for (int i = 0; i < L.dim; i++) {
			xc.put(b + XL_TGT + i, L.tgt[i]);
			xc.put(b + XL_WGT + i, L.wr[i]);
		}
}

/* the scan of one lspVQ stage over the stored pairs (lspVQ_t's stage body,
 * quant.h, with the scores read instead of computed) */
template <class D>
MD void lq_vq_scan(LsfLead &L, const D &db)
{
	const int s1 = L.stage, size = L.sizes[s1], n = L.ncPrev * size;
	int32_t key[LSP_VQ_CAND];
#pragma unroll
	for (int k = 0; k < LSP_VQ_CAND; k++)
		key[k] = SW_MAX_ * 65536 + (0x8000 | k);
	Word16 maxd = SW_MAX_;
	/* each slice's stored visits in order, read LQ_BATCH at a time (every
	 * load of a batch issued before the first is used) */
	(void) n;
	for (int v = 0; v < LQ_NV; v++) {
		const int ns = L.ns[v];
		for (int k0 = 0; k0 < ns; k0 += LQ_BATCH) {
			uint32_t tb[LQ_BATCH], pb[LQ_BATCH];
#pragma unroll
			for (int b = 0; b < LQ_BATCH; b++) {
				const bool in = k0 + b < ns;
				tb[b] = in ? db.get(v * 2 * LQ_SCAP + 2 * (k0 + b)) : 0u;
				pb[b] = in ? db.get(v * 2 * LQ_SCAP + 2 * (k0 + b) + 1) : 0u;
			}
#pragma unroll
			for (int b = 0; b < LQ_BATCH; b++) {
				if (k0 + b >= ns)
					break;
				const int16_t h = (int16_t) (pb[b] & 0xffff), f = (int16_t) (pb[b] >> 16);
				const Word16 d = (h >= maxd) ? (Word16) SW_MAX_ : f;
				if (d < maxd) {
					const int32_t dk = (int32_t) d * 65536;
					const int32_t nk = dk + (int32_t) tb[b];	/* (c1 << 9) | entry */
					bool kp[LSP_VQ_CAND];
#pragma unroll
					for (int k = 0; k < LSP_VQ_CAND; k++)
						kp[k] = key[k] < dk;
#pragma unroll
					for (int k = LSP_VQ_CAND - 1; k >= 0; k--)
						key[k] = kp[k] ? key[k] : ((k == 0 || kp[k > 0 ? k - 1 : 0]) ? nk : key[k > 0 ? k - 1 : 0]);
					maxd = (Word16) (key[LSP_VQ_CAND - 1] >> 16);
				}
			}
		}
	}
	int16_t rows[LSP_VQ_CAND][LSP_VQ_STAGES];
	for (int k = 0; k < LSP_VQ_CAND; k++) {
		const int t = key[k] & 0xffff;
		if (!(t & 0x8000)) {
			int c = t >> 9;
			for (int i = 0; i < s1; i++)
				rows[k][i] = L.index[c][i];
			rows[k][s1] = (int16_t) (t & 511);
		} else {
			for (int i = 0; i <= s1; i++)
				rows[k][i] = L.nextIndex[t & 0x7fff][i];
		}
	}
	for (int k = 0; k < LSP_VQ_CAND; k++)
		for (int i = 0; i <= s1; i++)
			L.nextIndex[k][i] = rows[k][i];
	if (!L.flag && s1 == L.tos - 1) {
		L.ncPrev = 1;
	} else {
		Word16 t1 = extract_l(L_shr(L_mult(L.ncPrev, L.sizes[s1]), 1));
		Word16 t2 = (s1 == L.tos - 1) ? LSP_INP_CAND : LSP_VQ_CAND;
		L.ncPrev = t1 < t2 ? t1 : t2;
	}
	const int dim = L.dim;
	for (int c = 0; c < L.ncPrev; c++) {
		v_zero(L.cand[c], dim);
		const int16_t *p2 = g_tab + L.cb0;
		v_copy(L.index[c], L.nextIndex[c], s1 + 1);
		for (int i = 0; i <= s1; i++) {
			Word16 o = extract_l(L_shr(L_mult(L.index[c][i], (Word16) dim), 1));
			v_add(L.cand[c], p2 + o, dim);
			p2 += extract_l(L_shr(L_mult(L.sizes[i], (Word16) dim), 1));
		}
	}
	L.stage++;
}

/* lsf_vq's end (qnt12.c:1127-1137) */
MD void lq_epilogue(EncAna *E, MelpParam *par)
{
	lspStable(par[0].lsf, LPC_ORD);
	lspStable(par[1].lsf, LPC_ORD);
	if (!lspStable(par[2].lsf, LPC_ORD))
		lspSort(par[2].lsf, LPC_ORD);
	v_copy(E->qplsp, par[2].lsf, LPC_ORD);
}

/* the leader's scan phase: finish the step computed last phase, start and
 * publish the next */
template <class X, class D>
MD void lq_scan(LsfLead &L, EncAna *E, MelpParam *par, X &xc, int b, const D &db)
{
	if (L.done)
		return;
	QuantParam *q = &E->qpar;
	if (!L.sep && L.job == 1) {
		/* the interpolation search's reduction: the first minimum */
		Word32 minErr = LW_MAX_;
		int best = 0;
		for (int v = 0; v < LQ_NV; v++) {
			Word32 err = (Word32) ((uint32_t) (uint16_t) xc.get(b + XL_PART + 3 * v) |
					       ((uint32_t) (uint16_t) xc.get(b + XL_PART + 3 * v + 1) << 16));
			if (err < minErr) {
				minErr = err;
				best = xc.get(b + XL_PART + 3 * v + 2);
			}
		}
		const int cand = best >> 4, inp = best & 15;
		const int16_t *ic = TB(inpCoef);
		for (int j = 0; j < LPC_ORD; j++) {
			Word16 f = ic[inp * 20 + j];
			Word32 acc = L_mac(L_mult(f, E->qplsp[j]), sub(16384, f), L.lcand[cand][j]);
			L.best0[j] = extract_h(L_shl(acc, 1));
			f = ic[inp * 20 + j + LPC_ORD];
			acc = L_mac(L_mult(f, E->qplsp[j]), sub(16384, f), L.lcand[cand][j]);
			L.best1[j] = extract_h(L_shl(acc, 1));
		}
		int16_t res[2 * LPC_ORD], mwgt[2 * LPC_ORD];
		for (int i = 0; i < LPC_ORD; i++) {
			res[i] = shl(sub(par[0].lsf[i], L.best0[i]), 2);
			res[i + LPC_ORD] = shl(sub(par[1].lsf[i], L.best1[i]), 2);
		}
		v_copy(par[2].lsf, L.lcand[cand], LPC_ORD);
		v_copy(q->lsf_index[0], &L.lidx[cand * L.tos2], L.tos2);
		q->lsf_index[1][0] = (int16_t) inp;
		v_copy(mwgt, L.wgt[0], LPC_ORD);
		v_copy(mwgt + LPC_ORD, L.wgt[1], LPC_ORD);
		const int16_t res_sz[4] = {256, 64, 64, 64};
		L.job = 2;
		lq_vq_start(L, res, mwgt, 2 * LPC_ORD, LQ_CB_RES, res_sz, L.uvc == 1 ? 4 : 2, false);
	} else {
		for (int v = 0; v < LQ_NV; v++)
			L.ns[v] = xc.get(b + XL_NS + v);
		lq_vq_scan(L, db);
		if (L.stage == L.tos) {
			/* the lspVQ's outputs (lspVQ_t's last lines) */
			if (L.sep) {
				const int i = L.job;
				v_copy(q->lsf_index[i], L.index[0], L.tos);
				v_copy(par[i].lsf, L.cand[0], LPC_ORD);
				lq_next_job(L, par, L.job + 1);
			} else if (L.job == 0) {
				for (int c = 0; c < L.ncPrev; c++) {
					v_copy(&L.lidx[c * L.tos], L.index[c], L.tos);
					v_copy(L.lcand[c], L.cand[c], LPC_ORD);
				}
				L.tos2 = L.tos;
				lq_next_job(L, par, 1);
			} else {
				v_copy(q->lsf_index[2], L.index[0], L.tos);
				for (int i = 0; i < LPC_ORD; i++) {
					par[0].lsf[i] = add(shr(L.cand[0][i], 2), L.best0[i]);
					par[1].lsf[i] = add(shr(L.cand[0][i + LPC_ORD], 2), L.best1[i]);
				}
				L.done = 1;
			}
			if (L.done)
				lq_epilogue(E, par);
		}
	}
	lq_publish(L, E, par, xc, b);
}

/* ---------------------------------------------------------------- */
/* every wave: its slice of the published step                      */
/* ---------------------------------------------------------------- */

template <int DIM, class X, class D>
MD void lq_vq_slice(X &xc, int b, D &db, int v, int cbs, int size, int nc, int s)
{
	int16_t wr[DIM], tgt[DIM], ct[DIM];
#pragma unroll
	for (int i = 0; i < DIM; i++) {
		wr[i] = xc.get(b + XL_WGT + i);
		tgt[i] = xc.get(b + XL_TGT + i);
	}
	const int cb0 = (int) (uint16_t) xc.get(b + XL_CB0LO) | ((int) xc.get(b + XL_CB0HI) << 16);
	const int n = nc * size, lo = v * n / LQ_NV, hi = (v + 1) * n / LQ_NV;
	bool all = false;	/* a negative weight: store every visit */
#pragma unroll
	for (int i = 0; i < DIM; i++)
		all |= wr[i] < 0;
	/* the slice's own M-best distortions, ascending (only their multiset
	 * decides what the slice keeps) */
	int16_t lk[LSP_VQ_CAND];
#pragma unroll
	for (int k = 0; k < LSP_VQ_CAND; k++)
		lk[k] = SW_MAX_;
	int ns = 0;
	int c1 = -1;
#if !defined(MELPE_OPCOUNT)
	/* the rows as dwords at wave-uniform addresses (scalar loads; the lsf
	 * codebooks' stages start at even offsets), the next visit's row issued
	 * before this one is scored */
	const bool srow = !(cbs & 1);
	uint32_t rw[DIM / 2];
	if (srow && lo < hi) {
		const u32_alias *r0 = reinterpret_cast<const u32_alias *>(g_tab + cbs + (lo % size) * DIM);
	#pragma unroll
		for (int i = 0; i < DIM / 2; i++)
			rw[i] = r0[i];
	}
#endif
	for (int u = lo; u < hi; u++) {
		const int c = u / size, e = u - c * size;
		if (c != c1) {
			c1 = c;
			/* candidate c's reconstruction so far (lspVQ_t's cand) */
			int16_t cand[DIM];
#pragma unroll
			for (int i = 0; i < DIM; i++)
				cand[i] = 0;
			const int16_t *p2 = g_tab + cb0;
			for (int i = 0; i < s; i++) {
				const int16_t r = xc.get(b + XL_ROWS + c * LSP_VQ_STAGES + i);
				Word16 o = extract_l(L_shr(L_mult(r, (Word16) DIM), 1));
				v_add(cand, p2 + o, DIM);
				p2 += extract_l(L_shr(L_mult(xc.get(b + XL_SIZES + i), (Word16) DIM), 1));
			}
#pragma unroll
			for (int i = 0; i < DIM; i++)
				ct[i] = sub(tgt[i], cand[i]);
		}
#if !defined(MELPE_OPCOUNT)
		uint32_t pr;
		if (srow) {
			int16_t x[DIM];
	#pragma unroll
			for (int i = 0; i < DIM / 2; i++) {
				x[2 * i] = lo16(rw[i]);
				x[2 * i + 1] = hi16(rw[i]);
			}
			const int en = (u + 1 < hi) ? (e + 1 < size ? e + 1 : 0) : e;
			const u32_alias *rn = reinterpret_cast<const u32_alias *>(g_tab + cbs + en * DIM);
	#pragma unroll
			for (int i = 0; i < DIM / 2; i++)
				rw[i] = rn[i];
			pr = lq_wmse<DIM>(wr, x, ct);
		} else {
			pr = lq_wmse<DIM>(wr, g_tab + cbs + e * DIM, ct);
		}
#else
		const uint32_t pr = lq_wmse<DIM>(wr, g_tab + cbs + e * DIM, ct);
#endif
		const int16_t h = (int16_t) (pr & 0xffff), f = (int16_t) (pr >> 16);
		const Word16 lmax = lk[LSP_VQ_CAND - 1];
		const Word16 d = (h >= lmax) ? (Word16) SW_MAX_ : f;
		const bool keep = d < lmax;
		if (keep) {	/* sorted insert, the largest drops out */
#pragma unroll
			for (int k = LSP_VQ_CAND - 1; k >= 0; k--) {
				const int16_t prev = k > 0 ? lk[k - 1] : (int16_t) -32768;
				lk[k] = (prev > d) ? prev : ((lk[k] > d) ? d : lk[k]);
			}
		}
		if (keep || all) {
			db.put(v * 2 * LQ_SCAP + 2 * ns, (uint32_t) ((c << 9) | e));
			db.put(v * 2 * LQ_SCAP + 2 * ns + 1, pr);
			ns++;
		}
	}
	xc.put(b + XL_NS + v, (int16_t) ns);
}

#if MELPE_LQ_GATHER
/* lq_vq_slice with the stage, size, candidates and codebook per lane: the
 * codebook rows are gathered through the vector memory path (dword loads,
 * the lsf codebooks' rows are 4-byte aligned) instead of one scalar-cache
 * pass per distinct stage among the wave's channels (32,768 channels:
 * 9.83 vs 9.95 ms per k_enc_ana_mw launch, profiles/r03_m_*) */
template <int DIM, class X, class D>
MD void lq_vq_slice_g(X &xc, int b, D &db, int v, int cbs, int size, int nc, int s)
{
	int16_t wr[DIM], tgt[DIM], ct[DIM];
#pragma unroll
	for (int i = 0; i < DIM; i++) {
		wr[i] = xc.get(b + XL_WGT + i);
		tgt[i] = xc.get(b + XL_TGT + i);
	}
	const int cb0 = (int) (uint16_t) xc.get(b + XL_CB0LO) | ((int) xc.get(b + XL_CB0HI) << 16);
	const int n = nc * size, lo = v * n / LQ_NV, hi = (v + 1) * n / LQ_NV;
	bool all = false;
#pragma unroll
	for (int i = 0; i < DIM; i++)
		all |= wr[i] < 0;
	int16_t lk[LSP_VQ_CAND];
#pragma unroll
	for (int k = 0; k < LSP_VQ_CAND; k++)
		lk[k] = SW_MAX_;
	int ns = 0;
	int c = lo / size, e = lo - c * size;
	bool fresh = true;
	for (int u = lo; u < hi; u++) {
		if (fresh) {
			fresh = false;
			int16_t cand[DIM];
#pragma unroll
			for (int i = 0; i < DIM; i++)
				cand[i] = 0;
			const int16_t *p2 = g_tab + cb0;
			for (int i = 0; i < s; i++) {
				const int16_t r = xc.get(b + XL_ROWS + c * LSP_VQ_STAGES + i);
				Word16 o = extract_l(L_shr(L_mult(r, (Word16) DIM), 1));
				v_add(cand, p2 + o, DIM);
				p2 += extract_l(L_shr(L_mult(xc.get(b + XL_SIZES + i), (Word16) DIM), 1));
			}
#pragma unroll
			for (int i = 0; i < DIM; i++)
				ct[i] = sub(tgt[i], cand[i]);
		}
		int16_t x[DIM];
		const u32_alias *row = (const u32_alias *) (g_tab + cbs + e * DIM);
#pragma unroll
		for (int i = 0; i < DIM / 2; i++) {
			const uint32_t w2 = row[i];
			x[2 * i] = (int16_t) (w2 & 0xffff);
			x[2 * i + 1] = (int16_t) (w2 >> 16);
		}
#if !defined(MELPE_OPCOUNT) && MELPE_WMSE_POS
		const uint32_t pr = all ? lq_wmse<DIM>(wr, x, ct) : lq_wmse_pos<DIM>(wr, x, ct);
#else
		const uint32_t pr = lq_wmse<DIM>(wr, x, ct);
#endif
		const int16_t h = (int16_t) (pr & 0xffff), f = (int16_t) (pr >> 16);
		const Word16 lmax = lk[LSP_VQ_CAND - 1];
		const Word16 d = (h >= lmax) ? (Word16) SW_MAX_ : f;
		const bool keep = d < lmax;
		if (keep) {
#pragma unroll
			for (int k = LSP_VQ_CAND - 1; k >= 0; k--) {
				const int16_t prev = k > 0 ? lk[k - 1] : (int16_t) -32768;
				lk[k] = (prev > d) ? prev : ((lk[k] > d) ? d : lk[k]);
			}
		}
		if (keep || all) {
			db.put(v * 2 * LQ_SCAP + 2 * ns, (uint32_t) ((c << 9) | e));
			db.put(v * 2 * LQ_SCAP + 2 * ns + 1, pr);
			ns++;
		}
		if (++e == size) {
			e = 0;
			c++;
			fresh = true;
		}
	}
	xc.put(b + XL_NS + v, (int16_t) ns);
}
#endif

/* the interpolation search over pairs [20v, 20v + 20) (qnt12.c:1019-1063,
 * the general chain: any weights) */
template <class X>
MD void lq_interp_slice(X &xc, int b, int v)
{
	const int16_t *ic = TB(inpCoef);
	Word32 minErr = LW_MAX_;
	int best = -1;
	const int lo = v * LQ_PAIRS / LQ_NV, hi = (v + 1) * LQ_PAIRS / LQ_NV;
	for (int c = lo; c < hi; c++) {
		const int k = c >> 4, i = c & 15;
		Word32 err = 0;
		/* the pattern's 20 coefficients as ten dwords at a wave-uniform
		 * address (scalar loads; inpCoef at an even offset) */
		const u32_alias *ic32 = reinterpret_cast<const u32_alias *>(ic + i * 20);
		uint32_t fw[10];
	#pragma unroll
		for (int q = 0; q < 10; q++)
			fw[q] = ic32[q];
	#pragma unroll
		for (int j = 0; j < LPC_ORD; j++) {
			const Word16 qp = xc.get(b + XL_IP_QPLSP + j);
			const Word16 lc = xc.get(b + XL_IP_LCAND + k * LPC_ORD + j);
			Word16 f = (j & 1) ? hi16(fw[j >> 1]) : lo16(fw[j >> 1]);
			Word32 acc = L_mult(f, qp);
			acc = L_mac(acc, sub(16384, f), lc);
			acc = L_sub(acc, L_shl(L_deposit_l(xc.get(b + XL_IP_LSP + j)), 15));
			f = ((j + LPC_ORD) & 1) ? hi16(fw[(j + LPC_ORD) >> 1]) : lo16(fw[(j + LPC_ORD) >> 1]);
			Word32 bcc = L_mult(f, qp);
			bcc = L_mac(bcc, sub(16384, f), lc);
			bcc = L_sub(bcc, L_shl(L_deposit_l(xc.get(b + XL_IP_LSP + LPC_ORD + j)), 15));
			err = L_add(err, lsf_werr(acc, xc.get(b + XL_IP_WGT + j)));
			err = L_add(err, lsf_werr(bcc, xc.get(b + XL_IP_WGT + LPC_ORD + j)));
			acc = L_shl(L_deposit_l(xc.get(b + XL_IP_LSP + 2 * LPC_ORD + j)), 15);
			acc = L_sub(acc, L_shl(L_deposit_l(lc), 15));
			err = L_add(err, lsf_werr(acc, xc.get(b + XL_IP_WGT + 2 * LPC_ORD + j)));
		}
		if (err < minErr) {
			minErr = err;
			best = c;
		}
	}
	xc.put(b + XL_PART + 3 * v, (int16_t) (minErr & 0xffff));
	xc.put(b + XL_PART + 3 * v + 1, (int16_t) ((uint32_t) minErr >> 16));
	xc.put(b + XL_PART + 3 * v + 2, (int16_t) (best < 0 ? 0 : best));
}

/* virtual wave v's compute phase */
template <class X, class D>
MD void lq_compute(X &xc, int b, D &db, int v)
{
	const int job = xc.get(b + XL_JOB);
	if (job == 2) {
		lq_interp_slice(xc, b, v);
		return;
	}
	if (job != 1)
		return;
	const int dim = xc.get(b + XL_DIM), s = xc.get(b + XL_STAGE), nc = xc.get(b + XL_NC);
	const int cb0 = (int) (uint16_t) xc.get(b + XL_CB0LO) | ((int) xc.get(b + XL_CB0HI) << 16);
	int cbs = cb0;
	for (int i = 0; i < s; i++)
		cbs += xc.get(b + XL_SIZES + i) * dim;
	const int size = xc.get(b + XL_SIZES + s);
#if MELPE_LQ_GATHER
	for (;;) {	/* one pass per dimension */
		const int udim = wave_first(dim);
		if (dim != udim)
			continue;
		if (udim == 2 * LPC_ORD)
			lq_vq_slice_g<2 * LPC_ORD>(xc, b, db, v, cbs, size, nc, s);
		else
			lq_vq_slice_g<LPC_ORD>(xc, b, db, v, cbs, size, nc, s);
		break;
	}
	return;
#endif
	/* one pass per distinct (codebook stage, size, dim, candidates) among
	 * the wave's channels, with those values wave-uniform inside: the
	 * codebook rows come through the scalar cache (as lspVQ_t's scan) */
	for (;;) {
		const int ucb = wave_first(cbs), usz = wave_first(size), udim = wave_first(dim),
			  unc = wave_first(nc), us = wave_first(s);
		if (cbs != ucb || size != usz || dim != udim || nc != unc || s != us)
			continue;
		if (udim == 2 * LPC_ORD)
			lq_vq_slice<2 * LPC_ORD>(xc, b, db, v, ucb, usz, unc, us);
		else
			lq_vq_slice<LPC_ORD>(xc, b, db, v, ucb, usz, unc, us);
		break;
	}
}

}  // namespace mlp

#endif
