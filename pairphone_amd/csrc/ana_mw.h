/*
 * ana_mw.h -- analysis() (melpe/melp_ana.c:119-267) of one channel split
 * over the waves of a workgroup: the lanes-per-channel mode of the analysis
 * kernel (k_enc_ana_mw).
 *
 * A superframe's analysis is three frames of melp_ana followed by sc_ana,
 * the quantisers and the channel packing.  Inside melp_ana several chains
 * touch disjoint state (state.h groups) and meet only at a few scalars:
 *   v0  lowpass + find_pitch -> band 0 of bpvc_ana -> residual / peakiness
 *       -> pitch_ana -> gains -> pitch average            (the driver chain)
 *   v1  LPC -> LSFs (lpc_pred2lsp is the costly part); bands 1, 2
 *   v2  pitchAuto of both subframes (corPeak over 127 lags); band 3
 *   v3  classify of both subframes; band 4
 * Bands 1..4 of a frame need band 0's pitch of that frame and classify
 * needs pitchAuto's peak pitch / correlation of its subframe, so they run
 * one phase behind: phase i (i < NF) is frame i's driver chain, LPC and
 * pitchAuto beside frame i-1's bands and classify.  Values cross waves
 * through the per-channel exchange block (LDS on the GPU), in a phase after
 * the one that produced them.  The tail (melp_ana.c:162-265) splits the
 * same way where the reference's order allows it:
 *   phase NF    v0 lsf_vq's prelude (it reads only the LSFs and voicing)
 *               and its first step alone, v1..v3 frame NF-1's bands and
 *               classify, v2 gain_vq + the jitter quantiser
 *   NF+1 ..     lsf_vq's other searches, each step scored by all four
 *               waves and replayed in order by v0 (lsfvq_mw.h)
 *   MW_PH_SC    v0 sc_ana and pitch_vq's prelude, after gathering
 *               classify's and pitchAuto's tracks (through the HBM record)
 *               and the band voicings and gains (exchange block); v1..v3
 *               the residual spectrum of frame v-1 (find_harm's FFT needs
 *               only the quantised LSFs)
 *   +1          pitch_vq's codebook search, a quarter per wave (pv_slice)
 *   +2          v0 the search's replay, pitch_vq's finish, quant_bp,
 *               quant_jitter
 *   +3          find_harm's harmonic magnitudes of frame i on v(i+1)
 *   +4          v0 quant_fsmag, the channel write.
 * Phase 0 also runs the global-pitch chain of all three frames on v3 (it
 * depends on nothing else), so v0 takes frames 1 and 2's from the block.
 *
 * Every chain keeps the reference's operation order on its own data, so the
 * result is bit-identical to the serial analysis() whatever the number of
 * physical waves NW: virtual wave v runs on physical wave v % NW, and the
 * virtual waves that share a physical wave share its copy of the state
 * (their write sets are disjoint).  NW = 1 is a serial order itself.
 */
#ifndef MELPE_ANA_MW_H
#define MELPE_ANA_MW_H

#include "lsfvq_mw.h"

namespace mlp {

#define MW_NV 4	/* virtual waves of the schedule */
/* frames, the lsf block's prelude, its (compute, scan) pairs, sc_ana &c.,
 * find_harm, packing */
#define MW_PH_LQ (NF + 1)	/* first compute phase of the lsf block */
/* lsf_vq's first step runs on v0 in phase NF, the rest in the block */
#define MW_LQ_PAIRS (LQ_SLOTS - 1)
#define MW_PH_SC (MW_PH_LQ + 2 * MW_LQ_PAIRS)
#define MW_PHASES (MW_PH_SC + 5)
#define PV_CAP 128	/* kept entries a wave stores per pitch-VQ slice (lqbuf row) */
static_assert(MW_NV * 2 * PV_CAP <= LQ_ROW, "pitch-VQ survivors exceed the score row");

/* the per-channel exchange block, in int16 words */
enum {
	XS_SUBPITCH = 0,	/* [NF] band 0's pitch of frame i (v0 -> v1..v3) */
	XS_BPVC = XS_SUBPITCH + NF,	/* [NF][NUM_BANDS] bands 1..4 (-> v0) */
	XS_LSF = XS_BPVC + NF * NUM_BANDS,	/* [NF][LPC_ORD] (v1 -> v0) */
	XS_CSPC = XS_LSF + NF * LPC_ORD,	/* [2 NF][2] pitchAuto's pitch, corx (v2 -> v3) */
	XS_UV = XS_CSPC + 2 * NF * 2,	/* [NF] voicing of frame i (v0 -> v1's lsf_vq) */
	XS_LIDX = XS_UV + NF,	/* [NF][MAX_LSF_STAGE] lsf_vq's indices (v1 -> v0) */
	XS_QPLSP = XS_LIDX + NF * MAX_LSF_STAGE,	/* [LPC_ORD] + started flag (v1 -> v0) */
	XS_FHP = XS_QPLSP + LPC_ORD + 1,	/* [NF] quantised pitch (v0 -> find_harm's waves) */
	XS_FHUV = XS_FHP + NF,	/* [NF] voicing after quant_bp (ditto) */
	XS_FSMAG = XS_FHUV + NF,	/* [NF][NUM_HARM] find_harm's magnitudes (-> v0) */
	XS_GAIN = XS_FSMAG + NF * NUM_HARM,	/* [NF][NUM_GAINFR] gains (v0 -> v2 -> v0) */
	XS_JIT = XS_GAIN + NF * NUM_GAINFR,	/* [NF] jitter (v0 -> v2 -> v0) */
	XS_GJIDX = XS_JIT + NF,	/* gain_index[0], jit_index[NF] (v2 -> v0) */
	XS_GP = XS_GJIDX + 1 + NF,	/* [NF] global pitch fpitch[1] of frame i (v3 -> v0) */
	XS_LPF = XS_GP + NF,	/* [2 LPF_ORD] its lowpass memories after frame NF-1 (v3 -> v0) */
	XS_LQ = XS_LPF + 2 * LPF_ORD,	/* the lsf block's words (lsfvq_mw.h XL_*) */
	XS_WORDS = XS_LQ + XL_WORDS,
	/* the pitch-VQ search's words, over the lsf block's (done by then) */
	XP_JOB = XS_LQ,	/* 1: the codebook search runs */
	XP_CNT,	/* voiced frames (the codebook) */
	XP_TGT,	/* [NF] */
	XP_WT = XP_TGT + NF,	/* [NF] */
	XP_NS = XP_WT + NF,	/* [MW_NV] entries each slice kept (-1: more than PV_CAP) */
	XP_END = XP_NS + MW_NV
};
static_assert(XP_END <= XS_WORDS, "pitch-VQ words overflow the lsf block");

/* what v0 keeps from a frame's first phase for its second and the tail */
struct AnaMwTmp {
	int16_t peak[NF];
	LsfLead lq;	/* lsf_vq's leader state (virtual wave 0) */
	PvqWork pv;	/* pitch_vq's prelude, for its finish two phases on */
	uint32_t hb[512];	/* v1..v3: the frame's residual spectrum (find_harm_fft) */
};

/*
 * pitch_vq's codebook search (wvq1, qnt12.c:221) split over the waves: wave
 * v scans the v-th quarter of the codebook with its own candidate list, kept
 * by the reference's rule, and stores the entries that list kept, in order.
 * The reference's list holds the `cand` smallest distortions seen so far
 * (a kept entry replaces the maximum; an equal one is rejected), so at any
 * entry its maximum is <= the slice list's, which has seen a subset: an entry
 * the slice rejected, the reference rejects too.  The leader then replays
 * the stored entries of slices 0..3 in codebook order through the
 * reference's update, which is the reference's scan with rejections skipped.
 */
template <class X, class D>
MD void pv_slice(X &xc, D &db, int v)
{
	if (!xc.get(XP_JOB))
		return;
	PvqWork w;
	w.cnt = xc.get(XP_CNT);
	for (int j = 0; j < NF; j++) {
		w.tgt[j] = xc.get(XP_TGT + j);
		w.wt[j] = xc.get(XP_WT + j);
	}
	int size;
	const int off = pvq_cb(w, &size);
	for (;;) {	/* one pass per distinct codebook among the lanes */
		const int uo = wave_first(off), un = wave_first(size);
		if (off != uo || size != un)
			continue;
		const int16_t *ucb = g_tab + uo;
		int16_t il[PITCH_VQ_CAND];
		Word32 dl[PITCH_VQ_CAND];
		for (int j = 0; j < PITCH_VQ_CAND; j++)
			dl[j] = LW_MAX_;
		Word32 maxd = LW_MAX_;
		int maxi = 0, n = 0;
		const int lo = v * un / MW_NV, hi = (v + 1) * un / MW_NV;
#if !defined(MELPE_OPCOUNT)
		static_assert(NF == 3 && TOFF_pitch_vq_cb_vvv % 2 == 0 && TOFF_pitch_vq_cb_uvv % 2 == 0,
			      "pitch codebooks as Row3 streams");
		Row3 rs;
		if (lo < hi)
			rs.open(ucb, lo);
#endif
		for (int i = lo; i < hi; i++) {
#if !defined(MELPE_OPCOUNT)
			int16_t x[3];
			rs.take(i, i + 1 < hi ? i + 1 : i, x);
			const Word32 err = wvq1_err3(w.tgt, w.wt, x);
#else
			const Word32 err = wvq1_err<NF>(w.tgt, w.wt, ucb + i * NF, maxd);
#endif
			if (wvq1_push(err, i, il, dl, maxd, maxi, PITCH_VQ_CAND)) {
				if (n < PV_CAP) {
					db.put(v * 2 * PV_CAP + 2 * n, (uint32_t) i);
					db.put(v * 2 * PV_CAP + 2 * n + 1, (uint32_t) err);
				}
				n++;
			}
		}
		xc.put(XP_NS + v, (int16_t) (n > PV_CAP ? -1 : n));
		break;
	}
}

/* the leader's replay of the slices' kept entries: wvq1's il / dl */
template <class X, class D>
MD void pv_replay(const PvqWork &w, X &xc, const D &db, int16_t *il, Word32 *dl)
{
	int size;
	const int16_t *cb = g_tab + pvq_cb(w, &size);
	for (int j = 0; j < PITCH_VQ_CAND; j++)
		dl[j] = LW_MAX_;
	Word32 maxd = LW_MAX_;
	int maxi = 0;
	for (int v = 0; v < MW_NV; v++) {
		const int n = xc.get(XP_NS + v);
		if (n < 0) {	/* more kept entries than stored: rescan the slice */
			for (int i = v * size / MW_NV; i < (v + 1) * size / MW_NV; i++)
				wvq1_push(wvq1_err<NF>(w.tgt, w.wt, cb + i * NF, maxd), i, il, dl, maxd,
					  maxi, PITCH_VQ_CAND);
			continue;
		}
		for (int k0 = 0; k0 < n; k0 += 8) {	/* eight entries' loads at once */
			uint32_t ib[8], eb[8];
#pragma unroll
			for (int b = 0; b < 8; b++) {
				const bool in = k0 + b < n;
				ib[b] = in ? db.get(v * 2 * PV_CAP + 2 * (k0 + b)) : 0u;
				eb[b] = in ? db.get(v * 2 * PV_CAP + 2 * (k0 + b) + 1) : 0u;
			}
#pragma unroll
			for (int b = 0; b < 8; b++)
				if (k0 + b < n)
					wvq1_push((Word32) eb[b], (int) ib[b], il, dl, maxd, maxi,
						  PITCH_VQ_CAND);
		}
	}
}

/* the part of each physical wave's private copy that differs from the HBM
 * record before any phase: dc removal of the three frames (melp_ana.c:
 * 140-145; each wave filters its own copy, only wave 0 keeps the result),
 * reading the superframe's PCM (4-byte aligned) where the caller holds it:
 * the three frames are one run of the same biquads */
MD void ana_mw_begin(EncAna *E, const int16_t *sp_in)
{
	static_assert(BLOCK % 36 == 0, "dc removal batches");
	iir3_d_batched(sp_in, &E->hpspeech[IN_BEG], TB(dc_den), TB(dc_num), E->dcdelin,
		       E->dcdelout_hi, E->dcdelout_lo, BLOCK);
}

/* band k (1..4) of frame i on a non-driver wave */
template <class X>
MD void ana_mw_band(EncAna *E, X &xc, int i, int k)
{
	if (!E->bp_started && i == 0)	/* bpvc_ana's first call, on this band's copy */
		bpvc_init_band(E, k);
	const int16_t *speech = &E->hpspeech[i * FRAME];
	int16_t *b = &E->par[i].bpvc[k];
	bpvc_band(E, &speech[FRAME_END], k, xc.get(XS_SUBPITCH + i), b);
	xc.put(XS_BPVC + i * NUM_BANDS + k, *b);
}

/* classify of frame i's two subframes, with pitchAuto's results of those
 * subframes taken from the exchange block; the frame's autocorrelation is
 * recomputed here (lpc_acor, a few hundred ops) instead of exchanged */
template <class X>
MD void ana_mw_classify(EncAna *E, X &xc, int i)
{
	const int16_t *speech = &E->hpspeech[i * FRAME];
	int16_t ac[17];
	lpc_acor(&speech[FRAME_END - LPC_FRAME / 2], TB(win_cof), ac, 4, 16, LPC_FRAME);
	for (int s = 0; s < PIT_SUBNUM; s++) {
		ClassParam *cs = &E->classStat[CUR_TRACK + i * PIT_SUBNUM + s + 1];
		cs->pitch = xc.get(XS_CSPC + 2 * (i * PIT_SUBNUM + s));
		cs->corx = xc.get(XS_CSPC + 2 * (i * PIT_SUBNUM + s) + 1);
		ana_track_cl(E, speech, i, s, ac);
	}
}

/* virtual wave v's work in phase p; rec is the channel's HBM record, which
 * carries classify's and pitchAuto's tracks to v0 before phase NF+1 */
template <class X, class D>
MD void ana_mw_phase(EncAna *E, EncAna *rec, X &xc, D &db, AnaMwTmp &tmp, int v, int p)
{
	if (p < NF) {
		const int i = p;
		const int16_t *speech = &E->hpspeech[i * FRAME];
		MelpParam *par = &E->par[i];
		if (v == 0) {
			int16_t ac[17], lpc[LPC_ORD + 1];
			Word16 sp;
			ana_first(E);
			/* the global pitch of frames 1.. comes from v3, which ran the
			 * lowpass chain ahead in phase 0 */
			if (i == 0)
				ana_global_pitch(E, speech);
			else
				E->fpitch[1] = xc.get(XS_GP + i);
			bpvc_init(E);
			bpvc_band0(E, &speech[FRAME_END], E->fpitch, &par->bpvc[0], &sp);
			par->jitter = (par->bpvc[0] < VJIT_Q14) ? (int16_t) MAX_JITTER_Q15 : (int16_t) 0;
			ana_lpc<false>(E, speech, ac, lpc, nullptr);
			Word16 t = ana_resid(E, speech, lpc);
			ana_peaky(par->bpvc, t, 0, 0);
			tmp.peak[i] = t;
			xc.put(XS_SUBPITCH + i, sp);
			ana_pitch_gain<false>(E, speech, par, sp);
			xc.put(XS_UV + i, par->uv_flag);
			for (int k = 0; k < NUM_GAINFR; k++)
				xc.put(XS_GAIN + i * NUM_GAINFR + k, par->gain[k]);
			xc.put(XS_JIT + i, par->jitter);
		} else if (v == 1) {
			int16_t ac[17], lpc[LPC_ORD + 1];
			ana_lpc<false>(E, speech, ac, lpc, par->lsf);
			for (int k = 0; k < LPC_ORD; k++)
				xc.put(XS_LSF + i * LPC_ORD + k, par->lsf[k]);
			if (i > 0) {
				ana_mw_band(E, xc, i - 1, 1);
				ana_mw_band(E, xc, i - 1, 2);
			}
		} else if (v == 2) {
			for (int s = 0; s < PIT_SUBNUM; s++) {
				ana_track_pa(E, speech, i, s);
				const ClassParam *cs = &E->classStat[CUR_TRACK + i * PIT_SUBNUM + s + 1];
				xc.put(XS_CSPC + 2 * (i * PIT_SUBNUM + s), cs->pitch);
				xc.put(XS_CSPC + 2 * (i * PIT_SUBNUM + s) + 1, cs->corx);
			}
			if (i > 0)
				ana_mw_band(E, xc, i - 1, 3);
		} else if (i > 0) {
			ana_mw_classify(E, xc, i - 1);
			ana_mw_band(E, xc, i - 1, 4);
		} else {
			/* the global pitch chain (lowpass memories + find_pitch) of
			 * every frame: it reads only the speech and its own memories
			 * (melp_ana.c:324-354), so it runs here, ahead of v0, which
			 * repeats frame 0's itself.  It starts from the record's
			 * memories in local copies: v0 may share this state copy
			 * (NW < 4) and has already advanced them by frame 0. */
			int16_t din[LPF_ORD], dout[LPF_ORD], sb[SIG_LENGTH];
			for (int k = 0; k < LPF_ORD; k++) {
				din[k] = rec->ana_started ? rec->lpfsp_delin[k] : (int16_t) 0;
				dout[k] = rec->ana_started ? rec->lpfsp_delout[k] : (int16_t) 0;
			}
			for (int k = 0; k < NF; k++)
				xc.put(XS_GP + k, global_pitch(&E->hpspeech[k * FRAME], sb, din, dout));
			for (int k = 0; k < LPF_ORD; k++) {
				xc.put(XS_LPF + k, din[k]);
				xc.put(XS_LPF + LPF_ORD + k, dout[k]);
			}
		}
	} else if (p == NF) {
		MelpParam *par = E->par;
		if (v == 0) {
			for (int i = 0; i < NF; i++)
				for (int k = 0; k < LPC_ORD; k++)
					par[i].lsf[k] = xc.get(XS_LSF + i * LPC_ORD + k);
			lq_prelude(tmp.lq, E, par);
			lq_publish(tmp.lq, E, par, xc, XS_LQ);
			/* the first lspVQ stage (one candidate: 256 or 512 visits),
			 * all four slices here -- v0 is otherwise idle in this phase */
			for (int sl = 0; sl < LQ_NV; sl++)
				lq_compute(xc, XS_LQ, db, sl);
			lq_scan(tmp.lq, E, par, xc, XS_LQ, db);
		} else if (v == 1) {
			ana_mw_band(E, xc, NF - 1, 1);
			ana_mw_band(E, xc, NF - 1, 2);
		} else if (v == 2) {
			ana_mw_band(E, xc, NF - 1, 3);
			lane_copy16(rec->pitTrack, E->pitTrack, sizeof(E->pitTrack));
			/* gain_vq and the jitter quantiser read only the gains and
			 * jitters (melp_ana.c:168-170) */
			for (int i = 0; i < NF; i++) {
				for (int k = 0; k < NUM_GAINFR; k++)
					par[i].gain[k] = xc.get(XS_GAIN + i * NUM_GAINFR + k);
				par[i].jitter = xc.get(XS_JIT + i);
			}
			gain_vq(E, par);
			for (int i = 0; i < NF; i++)
				quant_u(&par[i].jitter, &E->qpar.jit_index[i], 0, MAX_JITTER_Q15, 2,
					SW_MAX_, true, 7);
			for (int i = 0; i < NF; i++) {
				for (int k = 0; k < NUM_GAINFR; k++)
					xc.put(XS_GAIN + i * NUM_GAINFR + k, par[i].gain[k]);
				xc.put(XS_JIT + i, par[i].jitter);
				xc.put(XS_GJIDX + 1 + i, E->qpar.jit_index[i]);
			}
			xc.put(XS_GJIDX, E->qpar.gain_index[0]);
		} else {
			ana_mw_classify(E, xc, NF - 1);
			ana_mw_band(E, xc, NF - 1, 4);
			lane_copy16(rec->classStat, E->classStat, sizeof(E->classStat));
			rec->voicedEn = E->voicedEn;
			rec->silenceEn = E->silenceEn;
			rec->voicedCnt = E->voicedCnt;
		}
	} else if (p < MW_PH_SC) {
		/* the lsf block: (compute on every wave, scan on the leader) */
		if (((p - MW_PH_LQ) & 1) == 0) {
			lq_compute(xc, XS_LQ, db, v);
		} else if (v == 0) {
			lq_scan(tmp.lq, E, E->par, xc, XS_LQ, db);
			if (p == MW_PH_SC - 1)	/* done: the quantised LSFs, for find_harm */
				for (int i = 0; i < NF; i++)
					for (int k = 0; k < LPC_ORD; k++)
						xc.put(XS_LSF + i * LPC_ORD + k, E->par[i].lsf[k]);
		}
	} else if (p == MW_PH_SC) {
		if (v >= 1 && v <= NF) {
			/* find_harm's FFT of frame v-1 needs only the quantised LSFs:
			 * it runs here, beside sc_ana, and its magnitudes, which need
			 * the quantised pitch, three phases on */
			const int i = v - 1;
			MelpParam *par = &E->par[i];
			for (int k = 0; k < LPC_ORD; k++)
				par->lsf[k] = xc.get(XS_LSF + i * LPC_ORD + k);
			ana_fsmag_fft(E, par, i, tmp.hb);
			return;
		}
		if (v != 0)
			return;
		MelpParam *par = E->par;
		lane_copy16(E->pitTrack, rec->pitTrack, sizeof(E->pitTrack));
		lane_copy16(E->classStat, rec->classStat, sizeof(E->classStat));
		E->voicedEn = rec->voicedEn;
		E->silenceEn = rec->silenceEn;
		E->voicedCnt = rec->voicedCnt;
		for (int i = 0; i < NF; i++) {
			for (int k = 1; k < NUM_BANDS; k++)
				par[i].bpvc[k] = xc.get(XS_BPVC + i * NUM_BANDS + k);
			ana_peaky(par[i].bpvc, tmp.peak[i], 1, 2);
			for (int k = 0; k < NUM_GAINFR; k++)
				par[i].gain[k] = xc.get(XS_GAIN + i * NUM_GAINFR + k);
			par[i].jitter = xc.get(XS_JIT + i);
			E->qpar.jit_index[i] = xc.get(XS_GJIDX + 1 + i);
		}
		E->qpar.gain_index[0] = xc.get(XS_GJIDX);
		/* analysis_tail's order without lsf_vq / gain_vq / quant_u (done);
		 * pitch_vq's codebook search runs on every wave next phase */
		sc_ana(E, par);
		const int cnt = pvq_prelude(E, par, tmp.pv);
		xc.put(XP_JOB, cnt >= 2);
		if (cnt >= 2) {
			xc.put(XP_CNT, (int16_t) cnt);
			for (int j = 0; j < NF; j++) {
				xc.put(XP_TGT + j, tmp.pv.tgt[j]);
				xc.put(XP_WT + j, tmp.pv.wt[j]);
			}
		}
	} else if (p == MW_PH_SC + 1) {
		pv_slice(xc, db, v);
	} else if (p == MW_PH_SC + 2) {
		if (v != 0)
			return;
		MelpParam *par = E->par;
		if (tmp.pv.cnt >= 2) {
			int16_t il[PITCH_VQ_CAND];
			Word32 dl[PITCH_VQ_CAND];
			pv_replay(tmp.pv, xc, db, il, dl);
			pvq_finish(E, par, tmp.pv, il, dl);
		}
		quant_bp(E, par);
		quant_jitter(E, par);
		for (int i = 0; i < NF; i++) {
			xc.put(XS_FHP + i, par[i].pitch);
			xc.put(XS_FHUV + i, par[i].uv_flag);
		}
	} else if (p == MW_PH_SC + 3) {
		if (v == 0 || v > NF)
			return;
		/* ana_fsmag_frame's second half (melp_ana.c:224-236) on the
		 * spectrum of phase MW_PH_SC */
		const int i = v - 1;
		MelpParam *par = &E->par[i];
		par->pitch = xc.get(XS_FHP + i);
		par->uv_flag = xc.get(XS_FHUV + i);
		v_set(par->fs_mag, 8192, NUM_HARM);
		if (!par->uv_flag)
			find_harm_mag(tmp.hb, par->fs_mag, par->pitch, NUM_HARM);
		for (int k = 0; k < NUM_HARM; k++)
			xc.put(XS_FSMAG + i * NUM_HARM + k, par->fs_mag[k]);
	} else if (v == 0) {
		for (int i = 0; i < NF; i++)
			for (int k = 0; k < NUM_HARM; k++)
				E->par[i].fs_mag[k] = xc.get(XS_FSMAG + i * NUM_HARM + k);
		for (int k = 0; k < LPF_ORD; k++) {
			E->lpfsp_delin[k] = xc.get(XS_LPF + k);
			E->lpfsp_delout[k] = xc.get(XS_LPF + LPF_ORD + k);
		}
		ana_pack(E);
	}
}

/* Physical wave w's private copy of the record, before any phase: wave 0
 * takes the driver group and band 0 whole; every other virtual wave on any
 * wave only what its chains read -- the speech history and dc memories (it
 * runs dc_rmv itself), the parameters, the tracks and trackers (pitchAuto /
 * classify fill them, sc_ana's shift is wave 0's), lsf_vq's memory -- plus
 * its own group.  Nothing else of the copy is read before it is written;
 * the host build (emu_encode_ana_mw) fills the rest of each copy with a
 * pattern to check exactly that. */
MD void ana_mw_copy_in(EncAna *E, const EncAna *rec, int w, int nw)
{
	auto cp32 = [&](size_t off, size_t len) {
		lane_copy32((char *) E + off, (const char *) rec + off, len);
	};
	auto cp16 = [&](size_t off, size_t len) {
		lane_copy16((char *) E + off, (const char *) rec + off, len);
	};
	const size_t bs = sizeof(BandState), band0 = offsetof(EncAna, band);
	if (w == 0) {
		cp32(ENC_DRV_BEG, ENC_ANA_LIVE - ENC_DRV_BEG);
		cp32(band0, bs);
	} else {
		cp32(offsetof(EncAna, hpspeech), sizeof(int16_t) * IN_BEG);
		/* dc memories, parameters, energies, the tracks and trackers */
		cp32(ENC_DRV_BEG, offsetof(EncAna, ana_started) - ENC_DRV_BEG);
		cp16(offsetof(EncAna, bp_started), sizeof(int16_t));
		cp16(offsetof(EncAna, lsf_started), sizeof(int16_t) * (1 + LPC_ORD));
	}
	for (int v = w; v < MW_NV; v += nw) {
		if (v == 1)
			cp32(band0 + bs, 2 * bs);
		else if (v == 2) {
			cp32(offsetof(EncAna, pa), sizeof(PautoState));
			cp32(band0 + 3 * bs, bs);
		} else if (v == 3) {
			cp32(offsetof(EncAna, cls), sizeof(ClsState));
			cp32(band0 + 4 * bs, bs);
		}
	}
}

/* the byte ranges of the record virtual wave v owns (and writes back): the
 * driver group up to the carried speech history (the rest of the record is
 * working storage, state.h) */
MD int ana_mw_owned(int v, size_t *off, size_t *len)
{
	const size_t cls = offsetof(EncAna, cls), pa = offsetof(EncAna, pa);
	const size_t bs = sizeof(BandState);
	auto band = [&](int k) { return offsetof(EncAna, band) + k * bs; };
	switch (v) {
	case 0:
		off[0] = ENC_DRV_BEG;
		len[0] = ENC_ANA_LIVE - ENC_DRV_BEG;
		off[1] = band(0);
		len[1] = bs;
		return 2;
	case 1:
		off[0] = band(1);
		len[0] = 2 * bs;
		return 1;
	case 2:
		off[0] = pa;
		len[0] = sizeof(PautoState);
		off[1] = band(3);
		len[1] = bs;
		return 2;
	default:
		off[0] = cls;
		len[0] = sizeof(ClsState);
		off[1] = band(4);
		len[1] = bs;
		return 2;
	}
}

}  // namespace mlp

#endif
