/*
 * encoder.h -- one superframe of MELPe-1200 analysis + quantisation for one
 * channel: melpe_a (melpe/melpe.c:91-99) = 3 x npp + analysis().
 *
 * analysis()  restates melpe/melp_ana.c:119-267
 * melp_ana()  restates melpe/melp_ana.c:280-469
 * sc_ana()    restates melpe/melp_ana.c:522-953
 */
#ifndef MELPE_ENCODER_H
#define MELPE_ENCODER_H

#include "quant.h"

namespace mlp {

/* melp_ana :280 -- analysis of one 180-sample frame; `speech` points at
 * hpspeech[i*FRAME] (the window spans speech[0 .. FRAME_END+PITCHMAX]).
 * R24: the reference's rate == RATE2400 branches (melp_ana.c:370-391, 411,
 * 441, 460): LPC autocorrelation to order 10, LSFs of the unexpanded LPC
 * (kept as top_lpc), no pitch tracking / classification, the 2400 gain
 * window, and no voicing decision here (q_bpvc makes it) */
/* Timing knockouts (diagnostics only, never in a product build): compiled
 * with -DMELPE_KO_<stage>, the stage is skipped, so an A/B of kernel times
 * prices it in the product code itself, free of profiler perturbation.
 * The output of such a build is wrong by construction. */

/* melp_ana's parts.  Each touches only its own chain's state (state.h
 * groups), so melp_ana below runs them in the reference's order while the
 * multi-wave analysis kernel (ana_mw.h) runs the independent chains on
 * different waves of one workgroup. */

/* the first call's initialisation (melp_ana.c:300-306) */
MD void ana_first(EncAna *E)
{
	if (!E->ana_started) {
		v_zero(E->lpfsp_delin, LPF_ORD);
		v_zero(E->lpfsp_delout, LPF_ORD);
		E->pitch_avg = DEFAULT_PITCH_Q7;
		v_set(E->fpitch, DEFAULT_PITCH_Q7, 2);
		E->ana_started = 1;
	}
}

/* lowpass for the global pitch, whose filter memory advances by FRAME only,
 * then the integer pitch search (melp_ana.c:324-354) -> fpitch[1] (Q7);
 * sigbuf is this frame's scratch */
MN Word16 global_pitch(const int16_t *speech, int16_t *sb, int16_t *delin, int16_t *delout)
{
	Word16 dontcare;
#if !defined(MELPE_OPCOUNT)
	/* the copy, the lowpass (memories kept after FRAME samples) and
	 * f_pitch_scale's energy in one pass, as bpvc_ana's windows; with the
	 * energy within 32 bits the scale is read lazily (frac_pch) */
	{
		int64_t e = 0;
		auto acc = [&](int, int16_t y) { e += L_mult(y, y); };
		iir3_s_io(&speech[PITCH_BEG], &sb[LPF_ORD], TB(lpf_den), TB(lpf_num), delin, delout, FRAME, acc);
		int16_t tin[6], tout[6];
		v_copy(tin, delin, 6);
		v_copy(tout, delout, 6);
		iir3_s_io(&speech[PITCH_BEG + FRAME], &sb[LPF_ORD + FRAME], TB(lpf_den), TB(lpf_num), tin, tout,
			  PITCH_FR - FRAME, acc);
		bool ex = true;
		int lsh = 0;
		if (e <= (int64_t) LW_MAX_)
			lsh = shr(norm_l((Word32) e), 1);
		else
			f_pitch_scale_e(&sb[LPF_ORD], &sb[LPF_ORD], PITCH_FR, e, &ex);
		Word16 p = find_pitch(&sb[LPF_ORD + PITCH_FR / 2], &dontcare, 2 * PITCHMIN, PITCHMAX,
				      PITCHMAX, ex, lsh);
		return shl(p, 7);
	}
#endif
	v_copy(&sb[LPF_ORD], &speech[PITCH_BEG], PITCH_FR);
	iir3_s(&sb[LPF_ORD], TB(lpf_den), TB(lpf_num), delin, delout, PITCH_FR, FRAME);
	bool ex;
	f_pitch_scale(&sb[LPF_ORD], &sb[LPF_ORD], PITCH_FR, &ex);
	Word16 p = find_pitch(&sb[LPF_ORD + PITCH_FR / 2], &dontcare, 2 * PITCHMIN, PITCHMAX,
			      PITCHMAX, ex);
	return shl(p, 7);
}

MN void ana_global_pitch(EncAna *E, const int16_t *speech)
{
#if !defined(MELPE_KO_GPITCH)
	E->fpitch[1] = global_pitch(speech, E->sigbuf, E->lpfsp_delin, E->lpfsp_delout);
#endif
}

/* LPC analysis (melp_ana.c:366-393): ac[17] (the autocorrelation classify
 * also reads), lpc[0..LPC_ORD] and, when lsf is given, the LSFs */
template <bool R24>
MN void ana_lpc(EncAna *E, const int16_t *speech, int16_t *ac, int16_t *lpc, int16_t *lsf)
{
	lpc_acor(&speech[FRAME_END - LPC_FRAME / 2], TB(win_cof), ac, 4, R24 ? LPC_ORD : 16,
		 LPC_FRAME);
	lpc[0] = 4096;
	lpc_schr(ac, &lpc[1], LPC_ORD);
	if (R24) {
		lpc_pred2lsp(&lpc[1], lsf, LPC_ORD);
		v_copy(E->top_lpc, &lpc[1], LPC_ORD);
	} else {
		lpc_bwex(&lpc[1], &lpc[1], 32571, LPC_ORD);
		if (lsf) {
			lpc_pred2lsp(&lpc[1], lsf, LPC_ORD);
			lpc_clmp(lsf, 409, LPC_ORD);
		}
	}
}

/* the prediction residual into sigbuf and its peakiness (melp_ana.c:395-399) */
MN Word16 ana_resid(EncAna *E, const int16_t *speech, const int16_t *lpc)
{
	int16_t *sb = E->sigbuf;
	zerflt(&speech[PITCH_BEG], lpc, &sb[LPF_ORD], LPC_ORD, PITCH_FR);
	return peakiness(&sb[LPF_ORD + PITCHMAX / 2], PITCHMAX);
}

/* extreme peakiness forces the lower bands voiced (melp_ana.c:401-410) */
MD void ana_peaky(int16_t *bpvc, Word16 t, int lo, int hi)
{
	if (t > 5488 && lo == 0)
		bpvc[0] = 16384;
	if (t > 6553)
		for (int k = lo > 1 ? lo : 1; k <= hi && k <= 2; k++)
			bpvc[k] = 16384;
}

/* pitchAuto + classify of one 90-sample subframe of frame subnum
 * (melp_ana.c:411-426): sub 0 / 1 */
MN void ana_track_pa(EncAna *E, const int16_t *speech, int subnum, int sub)
{
	int ct = CUR_TRACK + subnum * PIT_SUBNUM;
#if !defined(MELPE_KO_PAUTO)
	pitchAuto(E, &speech[FRAME_END + sub * PIT_SUBFRAME + PIT_COR_LEN / 2],
		  &E->pitTrack[ct + sub + 1], &E->classStat[ct + sub + 1]);
#endif
}

MN void ana_track_cl(EncAna *E, const int16_t *speech, int subnum, int sub, const int16_t *ac)
{
	int ct = CUR_TRACK + subnum * PIT_SUBNUM;
#if !defined(MELPE_KO_CLASSIFY)
	classify(E, &speech[FRAME_END + sub * PIT_SUBFRAME + PIT_SUBFRAME / 2],
		 &E->classStat[ct + sub + 1], ac);
#endif
}

/* final pitch, gains, pitch average and voicing (melp_ana.c:428-468) */
template <bool R24>
MN void ana_pitch_gain(EncAna *E, const int16_t *speech, MelpParam *par, Word16 sub_pitch)
{
	int16_t *sb = E->sigbuf;
	Word16 pcorr, t;
#if !defined(MELPE_KO_PITCHANA)
	par->pitch = pitch_ana(E, &speech[FRAME_END], &sb[LPF_ORD + PITCHMAX], sub_pitch,
			       E->pitch_avg, &pcorr);
#else
	par->pitch = sub_pitch;
	pcorr = 0;
#endif
	for (int i = 0; i < NUM_GAINFR; i++) {
		/* one call site, its window arguments by voicing (a wave with both
		 * kinds of frames would run two) */
		const bool v = par->bpvc[0] > BPTHRESH_Q14;
		par->gain[i] = gain_ana(&speech[FRAME_BEG + (i + 1) * 90],
					v ? sub_pitch : (Word16) (R24 ? 15257 : 15258), v ? 120 : 0, 320);
	}
	t = (par->gain[NUM_GAINFR - 1] > 7680) ? pcorr : (Word16) 0;
	E->pitch_avg = p_avg_update(E, par->pitch, t, VMIN_Q14);
	if (!R24)
		par->uv_flag = (par->bpvc[0] > BPTHRESH_Q14) ? 0 : 1;
	E->fpitch[0] = E->fpitch[1];
}

template <bool R24>
MN void melp_ana(EncAna *E, const int16_t *speech, MelpParam *par, int subnum)
{
	PROF_SCOPE(1);
	int16_t ac[17], lpc[LPC_ORD + 1];
	Word16 sub_pitch;
	ana_first(E);
	ana_global_pitch(E, speech);
#if defined(MELPE_KO_BPVC)
	sub_pitch = E->fpitch[0];
	v_set(par->bpvc, 0, NUM_BANDS);
#else
	bpvc_ana(E, &speech[FRAME_END], E->fpitch, par->bpvc, &sub_pitch);
#endif
	par->jitter = (par->bpvc[0] < VJIT_Q14) ? (int16_t) MAX_JITTER_Q15 : (int16_t) 0;
	ana_lpc<R24>(E, speech, ac, lpc, par->lsf);
	const Word16 peak = ana_resid(E, speech, lpc);
	ana_peaky(par->bpvc, peak, 0, 2);
	if (!R24) {
		for (int i = 0; i < PIT_SUBNUM; i++) {
			ana_track_pa(E, speech, subnum, i);
			ana_track_cl(E, speech, subnum, i, ac);
		}
	}
	ana_pitch_gain<R24>(E, speech, par, sub_pitch);
}

/* subenergyRelation1/2 :955/:980 (plain int arithmetic, as the reference) */
MD bool subEnRel1(const ClassParam *cs, int c)
{
	int pg = cs[c - 2].subEnergy, lg = cs[c - 1].subEnergy, og = cs[c].subEnergy;
	int ng = cs[c + 1].subEnergy, fg = cs[c + 2].subEnergy;
	return ((lg - pg < 1024) && (og - lg < 1024) && (ng - og < 1024) &&
		((pg - lg > 2458) || (lg - og > 2458) || (og - ng > 2458))) ||
	       ((og - lg < 614) && (ng - og < 614) &&
		(((lg - pg < 614) && ((pg - og > 1638) || (lg - ng > 1638))) ||
		 ((fg - ng < 614) && ((lg - ng > 1638) || (og - fg > 1638)))));
}

MD bool subEnRel2(const ClassParam *cs, int c)
{
	int pg = cs[c - 2].subEnergy, lg = cs[c - 1].subEnergy, og = cs[c].subEnergy;
	int ng = cs[c + 1].subEnergy, fg = cs[c + 2].subEnergy;
	return ((lg - og < 614) && (og - ng < 614) &&
		(((pg - lg < 614) && ((og - pg > 1638) || (ng - lg > 1638))) ||
		 ((ng - fg < 614) && ((ng - lg > 1638) || (fg - og > 1638))))) ||
	       ((pg - lg < 1024) && (lg - og < 1024) && (og - ng < 1024) &&
		((lg - pg > 2458) || (og - lg > 2458) || (ng - og > 2458)));
}

/* the pitch-track correction shared by frames 0 and 1 of sc_ana when the
 * tracks disagree (melp_ana.c:590-640 and 700-760) */
MN void sc_track_fix(PitTrack *pt, int16_t *pitch, Word16 prev_pitch)
{
	Word16 i1 = trackPitch(prev_pitch, pt);
	Word16 cand = shl(pt->pit[i1], 7);
	Word16 i2 = trackPitch(*pitch, pt);
	Word16 w12 = sub(pt->weight[i1], pt->weight[i2]);
	if (multiCheck(*pitch, cand) < 2621) {
		if ((*pitch > cand && w12 > -6554) || w12 > 6554)
			*pitch = cand;
	} else if (w12 > -3277) {
		*pitch = cand;
	}
}

/* sc_ana :522 -- superframe pitch smoothing and bpvc smoothing */
MN void sc_ana(EncAna *E, MelpParam *par)
{
	PROF_SCOPE(8);
	ClassParam *cs = E->classStat;
	PitTrack *pt = E->pitTrack;
	int16_t bpc[NUM_BANDS], sbp[NF + 1], uv[NF + 1];
	Word16 cand, np, t1, t2, i1, i2, idx;
	for (int i = 0; i < NF; i++) {
		int c = i * PIT_SUBNUM + CUR_TRACK;
		if (cs[c].classy == SILENCE && cs[c - 1].classy == SILENCE)
			E->silenceEn = updateEn(E->silenceEn, 29491, cs[c].subEnergy);
	}
	uv[0] = E->sc_prev_uv;
	uv[1] = par[0].uv_flag;
	uv[2] = par[1].uv_flag;
	uv[3] = par[2].uv_flag;
	Word16 prev_pitch = E->sc_prev_pitch;

	/* ---- frame 0 ---- */
	int c = CUR_TRACK;
	E->voicedCnt = uv[1] ? 0 : E->voicedCnt + 1;
	if (!uv[1] && !uv[2] && !uv[3] && !subEnRel1(cs, c)) {
		if (E->voicedCnt < 2 || subEnRel2(cs, c)) {
			cand = pitLookahead(&pt[c], 3);
			if (ratio(par[0].pitch, cand) > 4915) {
				if (ratio(cand, par[1].pitch) < 4915)
					par[0].pitch = cand;
				else if (ratio(par[1].pitch, par[2].pitch) < 4915 &&
					 ratio(par[0].pitch, par[1].pitch) > 4915)
					par[0].pitch = par[1].pitch;
				else if (ratio(par[0].pitch, par[1].pitch) > 4915)
					par[0].pitch = cand;
			}
		} else if (!uv[0]) {
			i1 = shr(sub(par[0].pitch, prev_pitch), 7);
			i2 = shr(sub(par[1].pitch, par[0].pitch), 7);
			if (abs_s(i1) > 5 && abs_s(i2) > 5 && i1 * i2 < 0) {
				cand = pitLookahead(&pt[c], 3);
				if (ratio(prev_pitch, cand) < 4915 || ratio(cand, par[1].pitch) < 6554)
					par[0].pitch = cand;
				else
					par[0].pitch = add(shr(prev_pitch, 1), shr(par[1].pitch, 1));
			} else if (ratio(par[0].pitch, prev_pitch) > 4915 &&
				   (ratio(par[1].pitch, prev_pitch) < 4915 ||
				    ratio(par[2].pitch, prev_pitch) < 4915)) {
				sc_track_fix(&pt[c], &par[0].pitch, prev_pitch);
			} else if (L_ratio(par[0].pitch, (Word32) (prev_pitch * 2)) < 2621 ||
				   L_ratio(par[0].pitch, (Word32) (prev_pitch * 3)) < 2621) {
				cand = pitLookahead(&pt[c], 4);
				if (ratio(cand, prev_pitch) < 3277)
					par[0].pitch = cand;
			}
		}
	}
	prev_pitch = shl(shr(par[0].pitch, 7), 7);

	/* ---- frame 1 ---- */
	c = CUR_TRACK + 2;
	E->voicedCnt = uv[2] ? 0 : E->voicedCnt + 1;
	if (!uv[2] && !subEnRel1(cs, c)) {
		if (E->voicedCnt < 2 || subEnRel2(cs, c)) {
			cand = pitLookahead(&pt[c], 3);
			if (ratio(par[1].pitch, cand) > 4915) {
				if (ratio(cand, par[2].pitch) < 4915) {
					par[1].pitch = cand;
				} else {
					np = pitLookahead(&pt[c + 1], 3);
					if (ratio(np, par[2].pitch) < 4915) {
						if (ratio(cand, np) < 4915)
							par[1].pitch = cand;
						else if (ratio(par[1].pitch, np) > 4915)
							par[1].pitch = np;
					} else if (ratio(cand, np) < 4915) {
						par[1].pitch = cand;
					}
				}
			}
		} else if (!uv[1]) {
			i1 = shr(sub(par[1].pitch, prev_pitch), 7);
			i2 = shr(sub(par[2].pitch, par[1].pitch), 7);
			cand = pitLookahead(&pt[c], 3);
			if (abs_s(i1) > 5 && abs_s(i2) > 5 && i1 * i2 < 0) {
				if (ratio(prev_pitch, cand) < 4915 || ratio(cand, par[2].pitch) < 6554)
					par[1].pitch = cand;
				else
					par[1].pitch = add(shr(prev_pitch, 1), shr(par[2].pitch, 1));
			} else if (ratio(par[1].pitch, prev_pitch) > 4915 &&
				   (ratio(par[2].pitch, prev_pitch) < 4915 ||
				    ratio(cand, prev_pitch) < 4915)) {
				if (ratio(cand, prev_pitch) < 4915)
					par[1].pitch = cand;
				else
					sc_track_fix(&pt[c], &par[1].pitch, prev_pitch);
			} else if (L_ratio(par[1].pitch, (Word32) (prev_pitch * 2)) < 2621 ||
				   L_ratio(par[1].pitch, (Word32) (prev_pitch * 3)) < 2621) {
				cand = pitLookahead(&pt[c], 4);
				if (ratio(cand, prev_pitch) < 3277)
					par[1].pitch = cand;
			}
		}
	}
	prev_pitch = shl(shr(par[1].pitch, 7), 7);

	/* ---- frame 2 ---- */
	c = CUR_TRACK + 4;
	E->voicedCnt = uv[3] ? 0 : E->voicedCnt + 1;
	if (!uv[3] && cs[c + 1].classy == VOICED && cs[c + 2].classy == VOICED &&
	    !subEnRel1(cs, c)) {
		if (E->voicedCnt < 2 || subEnRel2(cs, c)) {
			cand = pitLookahead(&pt[c], 2);
			if (ratio(par[2].pitch, cand) > 4915) {
				np = pitLookahead(&pt[c + 1], 1);
				if (ratio(np, cand) < 4915)
					par[2].pitch = cand;
				else if (ratio(par[2].pitch, np) >= 4915)
					par[2].pitch = np;
			}
		} else if (!uv[2]) {
			cand = pitLookahead(&pt[c], 2);
			i1 = shr(sub(par[2].pitch, prev_pitch), 7);
			i2 = shr(sub(cand, par[2].pitch), 7);
			if (abs_s(i1) > 5 && abs_s(i2) > 5 && i1 * i2 < 0) {
				if (ratio(prev_pitch, cand) < 4915) {
					par[2].pitch = cand;
				} else {
					i1 = trackPitch(cand, &pt[c]);
					i2 = trackPitch(par[2].pitch, &pt[c]);
					Word16 w12 = sub(pt[c].weight[i1], pt[c].weight[i2]);
					if (multiCheck(par[2].pitch, cand) < 2621) {
						if ((par[2].pitch > cand && w12 > -6554) || w12 > 6554)
							par[2].pitch = cand;
					} else {
						i1 = trackPitch(prev_pitch, &pt[c]);
						cand = shl(pt[c].pit[i1], 7);
						w12 = sub(pt[c].weight[i1], pt[c].weight[i2]);
						if (multiCheck(par[2].pitch, cand) < 2621) {
							if ((par[2].pitch > cand && w12 > -6554) || w12 > 6554)
								par[2].pitch = cand;
						} else {
							par[2].pitch = add(shr(prev_pitch, 1), shr(cand, 1));
						}
					}
				}
			}
		}
	}

	/* ---- bandpass voicing smoothing (melp_ana.c:855-925) ---- */
	sbp[0] = E->sc_prev_sbp3;
	for (int i = 0; i < NF; i++) {
		v_copy(bpc, par[i].bpvc, NUM_BANDS);
		if (q_bpvc(bpc, &idx, NUM_BANDS))
			sbp[i + 1] = -1;
		else
			sbp[i + 1] = TB(inv_bp_index_map)[TB(bp_index_map)[idx]];
	}
	const int vEn = E->voicedEn;
	for (int i = 1; i < NF; i++) {
		c = CUR_TRACK + (i - 1) * 2;
		if (sbp[i - 1] > 12 && sbp[i + 1] > 12) {
			if (cs[c].subEnergy > vEn - 1024 ||
			    (par[i - 1].bpvc[2] > 8192 && par[i - 1].bpvc[3] > 8192)) {
				if (sbp[i] < 12)
					sbp[i] = 12;
			} else if (sbp[i] < 8) {
				sbp[i] = 8;
			}
		} else if (sbp[i - 1] > 8 && sbp[i + 1] > 8) {
			if (cs[c].subEnergy > vEn - 2048 ||
			    (par[i - 1].bpvc[2] > 6554 && par[i - 1].bpvc[3] > 6554)) {
				if (sbp[i] < 8)
					sbp[i] = 8;
			}
		} else if (sbp[i - 1] < 8 && sbp[i + 1] < 8) {
			if (cs[c].subEnergy < vEn - 1024 && par[i - 1].bpvc[3] < 11469) {
				if (sbp[i] > 12)
					sbp[i] = 12;
			}
		}
	}
	c = CUR_TRACK + 4;
	if (cs[c].subEnergy > vEn - 614 && sbp[2] > 12 && par[1].bpvc[2] > 8192 &&
	    par[1].bpvc[3] > 8192) {
		if (sbp[3] < 12)
			sbp[3] = 12;
	} else if (cs[c].subEnergy > vEn - 1024 && sbp[2] > 8 && par[1].bpvc[2] > 7273 &&
		   par[1].bpvc[3] > 7273) {
		if (sbp[3] < 8)
			sbp[3] = 8;
	}
	for (int i = 0; i < NF; i++) {
		t1 = par[i].bpvc[0];
		q_bpvc_dec(par[i].bpvc, sbp[i + 1], 0, NUM_BANDS);
		par[i].bpvc[0] = t1;
	}
	E->sc_prev_sbp3 = sbp[3];
	for (int i = 0; i < NF; i++) {
		c = i * PIT_SUBNUM + CUR_TRACK;
		if (E->voicedCnt > 2)
			E->voicedEn = updateEn(E->voicedEn, 29491, cs[c].subEnergy);
		if (E->voicedEn < cs[c].subEnergy)
			E->voicedEn = cs[c].subEnergy;
	}
	for (int i = 0; i < TRACK_NUM - NF * PIT_SUBNUM; i++) {
		cs[i] = cs[i + NF * PIT_SUBNUM];
		pt[i] = pt[i + NF * PIT_SUBNUM];
	}
	E->sc_prev_uv = par[NF - 1].uv_flag;
	E->sc_prev_pitch = shl(shr(par[NF - 1].pitch, 7), 7);
	(void) t2;
}

/* a progress checkpoint of the lane analysis kernel (progprio.h); a no-op
 * everywhere else */
#ifndef ANA_CKPT
#define ANA_CKPT(j) ((void) 0)
#endif

/* analysis :119 -- 540 NPP-processed samples -> quantised params + chbuf */
/* analysis() in the two parts the GPU runs as separate kernels:
 * analysis_frame: dc removal and melp_ana of frame i (melp_ana.c:140-160);
 * analysis_tail: sc_ana, the quantisers and channel packing (:162-265) */
MD void analysis_frame(EncAna *E, const int16_t *sp_in, int i)
{
	dc_rmv(&sp_in[i * FRAME], &E->hpspeech[IN_BEG + i * FRAME], E->dcdelin,
	       E->dcdelout_hi, E->dcdelout_lo, FRAME);
	melp_ana<false>(E, &E->hpspeech[i * FRAME], &E->par[i], i);
}

/* the Fourier magnitudes of frame i (melp_ana.c:224-236): the LPC residual
 * of the quantised LSFs, windowed, through find_harm; 8192s when unvoiced */
MN void ana_fsmag_frame(EncAna *E, MelpParam *par, int i)
{
	int16_t lpc[LPC_ORD + 1];
	lpc[0] = 4096;
	v_set(par->fs_mag, 8192, NUM_HARM);
	if (!par->uv_flag) {
		lpc_lsp2pred(par->lsf, &lpc[1], LPC_ORD);
		zerflt(&E->hpspeech[i * FRAME + FRAME_END - LPC_FRAME / 2], lpc, E->sigbuf, LPC_ORD,
		       LPC_FRAME);
		window(E->sigbuf, TB(win_cof), E->sigbuf, LPC_FRAME);
#if !defined(MELPE_KO_HARM)
		find_harm(E->sigbuf, par->fs_mag, par->pitch, NUM_HARM, LPC_FRAME);
#endif
	}
}

/* ana_fsmag_frame's pitch-independent half, run before the frame's pitch is
 * quantised (ana_mw.h): the residual of the quantised LSFs, windowed, and
 * its FFT (melp_ana.c:224-233) */
MN void ana_fsmag_fft(EncAna *E, MelpParam *par, int i, uint32_t *hb)
{
	int16_t lpc[LPC_ORD + 1];
	lpc[0] = 4096;
	lpc_lsp2pred(par->lsf, &lpc[1], LPC_ORD);
	zerflt(&E->hpspeech[i * FRAME + FRAME_END - LPC_FRAME / 2], lpc, E->sigbuf, LPC_ORD,
	       LPC_FRAME);
	window(E->sigbuf, TB(win_cof), E->sigbuf, LPC_FRAME);
	find_harm_fft(E->sigbuf, hb, LPC_FRAME);
}

/* quant_fsmag, the channel write and the history shift (melp_ana.c:238-265) */
MN void ana_pack(EncAna *E)
{
	MelpParam *par = E->par;
	quant_fsmag(E, par);
	for (int i = 0; i < NF; i++)
		E->qpar.uv_flag[i] = par[i].uv_flag;
	low_rate_chn_write(E);
	v_copy(E->hpspeech, &E->hpspeech[NF * FRAME], IN_BEG);
}

MN void analysis_tail(EncAna *E)
{
	MelpParam *par = E->par;
	sc_ana(E, par);
#if !defined(MELPE_KO_LSFVQ)
	lsf_vq(E, par);
#endif
	pitch_vq(E, par);
	gain_vq(E, par);
	for (int i = 0; i < NF; i++)
		quant_u(&par[i].jitter, &E->qpar.jit_index[i], 0, MAX_JITTER_Q15, 2, SW_MAX_,
			true, 7);
	quant_bp(E, par);
	quant_jitter(E, par);
	for (int i = 0; i < NF; i++)
		ana_fsmag_frame(E, &par[i], i);
	ana_pack(E);
}

/* analysis() in the split form of the lane-per-channel kernels (k_ana.hip
 * k_enc_ana, k_harm.hip): analysis_a runs everything before the Fourier
 * magnitudes, writes each voiced frame's windowed residual of the quantised
 * LSFs to res[i * LPC_FRAME ..] (melp_ana.c:224-233, the input of
 * find_harm; an unvoiced frame's row is not written) and does the history
 * shift; the magnitudes go into par[i].fs_mag (k_enc_harm), then
 * analysis_b packs the superframe.  The shift reads only hpspeech, which
 * nothing after it reads, so moving it ahead of the packing changes no
 * value. */
MN void analysis_a2(EncAna *E, int16_t *res)
{
	MelpParam *par = E->par;
	sc_ana(E, par);
#if !defined(MELPE_KO_LSFVQ)
	lsf_vq(E, par);
#endif
	ANA_CKPT(4);
	pitch_vq(E, par);
	gain_vq(E, par);
	for (int i = 0; i < NF; i++)
		quant_u(&par[i].jitter, &E->qpar.jit_index[i], 0, MAX_JITTER_Q15, 2, SW_MAX_,
			true, 7);
	quant_bp(E, par);
	quant_jitter(E, par);
	for (int i = 0; i < NF; i++) {
		if (par[i].uv_flag)
			continue;
		int16_t lpc[LPC_ORD + 1];
		lpc[0] = 4096;
		lpc_lsp2pred(par[i].lsf, &lpc[1], LPC_ORD);
		zerflt(&E->hpspeech[i * FRAME + FRAME_END - LPC_FRAME / 2], lpc, E->sigbuf, LPC_ORD,
		       LPC_FRAME);
		window(E->sigbuf, TB(win_cof), E->sigbuf, LPC_FRAME);
		v_copy(&res[i * LPC_FRAME], E->sigbuf, LPC_FRAME);
	}
	v_copy(E->hpspeech, &E->hpspeech[NF * FRAME], IN_BEG);
}

MN void analysis_a(EncAna *E, const int16_t *sp_in, int16_t *res)
{
#if defined(MELPE_KO_ANALYSIS)
	return;
#endif
	for (int i = 0; i < NF; i++) {
		analysis_frame(E, sp_in, i);
		ANA_CKPT(i + 1);
	}
	analysis_a2(E, res);
}

/* the history shift at the end of analysis (melp_ana.c:262) */
MD void ana_shift(EncAna *E)
{
	v_copy(E->hpspeech, &E->hpspeech[NF * FRAME], IN_BEG);
}

MN void analysis_b(EncAna *E)
{
	MelpParam *par = E->par;
	quant_fsmag(E, par);
	for (int i = 0; i < NF; i++)
		E->qpar.uv_flag[i] = par[i].uv_flag;
	low_rate_chn_write(E);
}

MN void analysis(EncAna *E, const int16_t *sp_in)
{
	PROF_SCOPE(15);
#if defined(MELPE_KO_ANALYSIS)
	return;
#endif
	for (int i = 0; i < NF; i++)
		analysis_frame(E, sp_in, i);
	analysis_tail(E);
}

/* debug aid: analysis() stopped after `upto` of its stages (1 = dc_rmv +
 * melp_ana, 2 = + sc_ana, 3 = + lsf_vq, 4 = + pitch/gain/jitter/bp,
 * 5 = + Fourier magnitudes, 6 = + channel write) */
MN void analysis_upto(EncAna *E, const int16_t *sp_in, int upto)
{
	MelpParam *par = E->par;
	int16_t lpc[LPC_ORD + 1];
	for (int i = 0; i < NF; i++) {
		dc_rmv(&sp_in[i * FRAME], &E->hpspeech[IN_BEG + i * FRAME], E->dcdelin,
		       E->dcdelout_hi, E->dcdelout_lo, FRAME);
		melp_ana<false>(E, &E->hpspeech[i * FRAME], &par[i], i);
	}
	if (upto < 2)
		return;
	sc_ana(E, par);
	if (upto < 3)
		return;
	lpc[0] = 4096;
	lsf_vq(E, par);
	if (upto < 4)
		return;
	pitch_vq(E, par);
	gain_vq(E, par);
	for (int i = 0; i < NF; i++)
		quant_u(&par[i].jitter, &E->qpar.jit_index[i], 0, MAX_JITTER_Q15, 2, SW_MAX_,
			true, 7);
	quant_bp(E, par);
	quant_jitter(E, par);
	if (upto < 5)
		return;
	for (int i = 0; i < NF; i++) {
		v_set(par[i].fs_mag, 8192, NUM_HARM);
		if (!par[i].uv_flag) {
			lpc_lsp2pred(par[i].lsf, &lpc[1], LPC_ORD);
			zerflt(&E->hpspeech[i * FRAME + FRAME_END - LPC_FRAME / 2], lpc, E->sigbuf,
			       LPC_ORD, LPC_FRAME);
			window(E->sigbuf, TB(win_cof), E->sigbuf, LPC_FRAME);
			find_harm(E->sigbuf, par[i].fs_mag, par[i].pitch, NUM_HARM, LPC_FRAME);
		}
	}
	quant_fsmag(E, par);
	if (upto < 6)
		return;
	for (int i = 0; i < NF; i++)
		E->qpar.uv_flag[i] = par[i].uv_flag;
	low_rate_chn_write(E);
	v_copy(E->hpspeech, &E->hpspeech[NF * FRAME], IN_BEG);
}

/* melpe_a :91 -- sp (540) is denoised in place, then analysed; the 11-byte
 * frame is left in E->chbuf */
MN void encode_superframe(EncState *S, NppScratch *w, int16_t *sp)
{
	PROF_SCOPE(16);
	npp_frame(&S->npp, w, sp, sp);
	npp_frame(&S->npp, w, sp + FRAME, sp + FRAME);
	npp_frame(&S->npp, w, sp + 2 * FRAME, sp + 2 * FRAME);
	analysis(&S->a, sp);
}

}  // namespace mlp

#endif
