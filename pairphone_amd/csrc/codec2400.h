/*
 * codec2400.h -- the 2400 bps MELP mode of the reference codec, one frame
 * (180 samples <-> 54 bits in 7 bytes) per call, per channel.
 *
 * The reference compiles this path but never reaches it: melpe_i pins rate
 * = RATE1200 (melpe/melpe.c:76) and the 2400 entry points it declares,
 * melpe_i2 / melpe_al (melpe/melpe.c:57-58), have no bodies.  Restated from
 * the rate == RATE2400 branches of
 *   analysis()        melpe/melp_ana.c:119-267 (one frame, MSVQ LSFs, log
 *                     pitch, q_gain, jitter flag, q_bpvc, fsvq)
 *   melp_ana()        melpe/melp_ana.c:370-391, 411, 441, 460 (encoder.h,
 *                     template argument R24)
 *   vq_ms4            melpe/vq_lib.c:118-404 (M-best multistage tree search)
 *   vq_msd2           melpe/vq_lib.c:413-451
 *   q_gain/_dec       melpe/melp_sub.c:636-762
 *   fec_code/_decode  melpe/fec_code.c:908-948, 993-1060
 *   melp_chn_write    melpe/melp_chn.c:109-148
 *   melp_chn_read     melpe/melp_chn.c:150-247
 *   synthesis()       melpe/melp_syn.c:110-147 (one frame) and melp_syn's
 *                     rate test (:213, decoder.h template argument R24)
 * Parity: oracle/ref_tool enc24gen / dec24gen run the reference's own
 * functions at RATE2400 (tests/test_r2400.py).
 */
#ifndef MELPE_CODEC2400_H
#define MELPE_CODEC2400_H

#include "encoder.h"
#include "decoder.h"

namespace mlp {

#define R24_BYTES 7
#define R24_BITS 54
#define OLD_IN_BEG 231		/* PITCH_BEG + PITCH_FR - FRAME */
#define MSVQ_M 8
#define MSVQ_MAXCNT 256
#define PIT_QLO_Q12 5329
#define PIT_QUP_Q12 9028
#define PIT_QLEV_M1 98
#define PIT_QLEV_M1_Q8 25088
#define GN_QLO_Q8 2560
#define GN_QUP_Q8 19712
#define GN_QLEV_M1 31
#define GN_QLEV_M1_Q10 31744
#define GAIN_INT_DB_Q8 1280
#define THREE_Q8 768
#define SIX_Q8 1536
#define SIX_Q12 24576
#define UV_PIND 0
#define INVAL_PIND 1
#define BEP_UNCORR (-2)

MD int msvq_levels(int s) { return s == 0 ? 128 : 64; }	/* global.c:35 */
MD int msvq_bits(int s) { return s == 0 ? 7 : 6; }	/* global.c:34 */

/* vq_ms4 :118 for the 2400 LSF MSVQ: M = 8 best paths through 4 stages of
 * 128, 64, 64, 64 ten-dimensional entries, at most MSVQ_MAXCNT list
 * replacements over the whole search.  lsf is the target on entry and the
 * reconstruction on exit; w (the vq_lspw weights) is rescaled in place. */
MN void vq_ms4_lsf(const int16_t *cb, int16_t *lsf, const int16_t *mean, int16_t *w,
		   int16_t *idx_out)
{
	int j = 0;
	for (int i = 0; i < LPC_ORD; i++) {
		if (w[i] > 16384) {		/* MAXWT4 */
			j = 3;
			break;
		} else if (w[i] > 8192) {	/* MAXWT2 */
			j = 2;
		} else if (w[i] > 4096) {	/* MAXWT */
			if (j == 0)
				j = 1;
		}
	}
	for (int i = 0; i < LPC_ORD; i++)
		w[i] = shr(w[i], (Word16) j);
	/* parent (p) and current (n) node buffers, swapped per stage */
	int16_t ind[2][MSVQ_M * MSVQ_STAGES], parent[2][MSVQ_M];
	int16_t err[2][MSVQ_M * LPC_ORD], dist[2][MSVQ_M];
	int16_t tpe[MSVQ_M * LPC_ORD], uhw[LPC_ORD], ut[LPC_ORD];
	for (int i = 0; i < MSVQ_M * MSVQ_STAGES; i++)
		ind[0][i] = ind[1][i] = 0;
	for (int c = 0; c < MSVQ_M; c++)
		parent[0][c] = parent[1][c] = 0;
	for (int i = 0; i < LPC_ORD; i++)
		ut[i] = sub(lsf[i], mean[i]);
	for (int i = 0; i < LPC_ORD; i++)
		ut[i] = shl(ut[i], 2);	/* Q17 */
	Word32 L = 0;
	for (int i = 0; i < LPC_ORD; i++)
		L = L_mac(L, mult(ut[i], w[i]), ut[i]);
	Word16 t0 = extract_h(L);
	int nb = 1;	/* the initial nodes are the "current" buffer */
	for (int c = 0; c < MSVQ_M; c++) {
		for (int i = 0; i < LPC_ORD; i++)
			err[nb][c * LPC_ORD + i] = ut[i];
		dist[nb][c] = t0;
	}
	const int16_t *cbp = cb;
	int m = 1, inner = 0;
	for (int s = 0; s < MSVQ_STAGES; s++) {
		const int16_t *cbs = cbp;
		nb ^= 1;
		const int pb = nb ^ 1;
		int pmax = 0;
		for (int i = 0; i < m * LPC_ORD; i++)
			tpe[i] = shr(err[pb][i], 2);
		for (int c = 0; c < MSVQ_M; c++)
			dist[nb][c] = SW_MAX_;
		const int lev = msvq_levels(s);
		for (int e = 0; e < lev; e++) {
			Word32 Lt = 0;
			for (int i = 0; i < LPC_ORD; i++, cbp++) {
				Word32 L1 = L_mult(*cbp, w[i]);
				uhw[i] = negate(extract_h(L_shl(L1, 3)));
				Lt = L_mac(Lt, *cbp, extract_h(L1));
			}
			Word16 usq = extract_h(Lt);
			for (int c = 0; c < m; c++) {
				Word32 Ld = L_deposit_h(add(dist[pb][c], usq));
				for (int i = 0; i < LPC_ORD; i++)
					Ld = L_mac(Ld, tpe[c * LPC_ORD + i], uhw[i]);
				Word16 d = extract_h(Ld);
				if (d <= dist[nb][pmax]) {
					dist[nb][pmax] = d;
					ind[nb][pmax * MSVQ_STAGES + s] = (int16_t) e;
					parent[nb][pmax] = (int16_t) c;
					if (inner < MSVQ_MAXCNT) {
						inner++;
						if (inner < MSVQ_MAXCNT) {
							pmax = 0;	/* the new worst of the best */
							for (int i = 1; i < MSVQ_M; i++)
								if (dist[nb][i] > dist[nb][pmax])
									pmax = i;
						} else {
							/* the counter is spent: from here on only the
							 * best candidate is kept (:300-313) */
							for (int i = 1; i < MSVQ_M; i++)
								if (dist[nb][i] < dist[nb][pmax])
									pmax = i;
						}
					}
				}
			}
		}
		for (int c = 0; c < MSVQ_M; c++) {
			const int pc = parent[nb][c];
			const int16_t *row = &cbs[ind[nb][c * MSVQ_STAGES + s] * LPC_ORD];
			for (int i = 0; i < LPC_ORD; i++)
				err[nb][c * LPC_ORD + i] = sub(err[pb][pc * LPC_ORD + i], row[i]);
			for (int k = 0; k < s; k++)
				ind[nb][c * MSVQ_STAGES + k] = ind[pb][pc * MSVQ_STAGES + k];
		}
		m *= lev;
		if (m > MSVQ_M)
			m = MSVQ_M;
	}
	int best = 0;
	for (int i = 1; i < MSVQ_M; i++)
		if (dist[nb][i] < dist[nb][best])
			best = i;
	for (int s = 0; s < MSVQ_STAGES; s++)
		idx_out[s] = ind[nb][best * MSVQ_STAGES + s];
	for (int i = 0; i < LPC_ORD; i++)
		lsf[i] = mean[i];
	const int16_t *cbs = cb;
	for (int s = 0; s < MSVQ_STAGES; s++) {
		const int16_t *row = &cbs[ind[nb][best * MSVQ_STAGES + s] * LPC_ORD];
		for (int i = 0; i < LPC_ORD; i++)
			lsf[i] = add(lsf[i], shr(row[i], 2));
		cbs += msvq_levels(s) * LPC_ORD;
	}
}

/* vq_msd2 :413 -- multistage VQ reconstruction (mean may be null) */
MD void vq_msd2(const int16_t *cb, int16_t *u_hat, const int16_t *mean, const int16_t *idx,
		int stages, bool msvq, int p, Word16 diff_q)
{
	Word32 L[LPC_ORD];
	for (int i = 0; i < p; i++)
		L[i] = L_shl(L_deposit_l(mean ? mean[i] : (int16_t) 0), diff_q);
	const int16_t *cbs = cb;
	for (int s = 0; s < stages; s++) {
		const int16_t *row = &cbs[idx[s] * p];
		for (int j = 0; j < p; j++)
			L[j] = L_add(L[j], L_deposit_l(row[j]));
		cbs += (msvq ? msvq_levels(s) : 256) * p;
	}
	for (int i = 0; i < p; i++)
		u_hat[i] = extract_l(L_shr(L[i], diff_q));
}

/* q_gain :636 -- uniform log quantiser of the second gain, the first
 * interpolated (index 0) or coded with 7 levels between its neighbours */
MN void q_gain(int16_t *prev_gain, int16_t *gain, int16_t *gidx)
{
	quant_u(&gain[1], &gidx[1], GN_QLO_Q8, GN_QUP_Q8, GN_QLEV_M1, GN_QLEV_M1_Q10, false, 5);
	if (gain[0] < GN_QLO_Q8)
		gain[0] = GN_QLO_Q8;
	if (gain[0] > GN_QUP_Q8)
		gain[0] = GN_QUP_Q8;
	Word16 t = add(shr(gain[1], 1), shr(*prev_gain, 1));
	if (abs_s(sub(gain[1], *prev_gain)) < GAIN_INT_DB_Q8 && abs_s(sub(gain[0], t)) < THREE_Q8) {
		gain[0] = t;
		gidx[0] = 0;
	} else {
		Word16 lo, hi;
		if (*prev_gain < gain[1]) {
			lo = *prev_gain;
			hi = gain[1];
		} else {
			lo = gain[1];
			hi = *prev_gain;
		}
		lo = sub(lo, SIX_Q8);
		hi = add(hi, SIX_Q8);
		if (lo < GN_QLO_Q8)
			lo = GN_QLO_Q8;
		if (hi > GN_QUP_Q8)
			hi = GN_QUP_Q8;
		quant_u(&gain[0], &gidx[0], lo, hi, 6, SIX_Q12, false, 3);
		gidx[0] = add(gidx[0], 1);	/* skip the all-zero code */
	}
	*prev_gain = gain[1];
}

/* q_gain_dec :697 */
MN void q_gain_dec(int16_t *prev_gain, int16_t *prev_err, int16_t *gain, const int16_t *gidx)
{
	gain[1] = quant_u_dec(gidx[1], GN_QLO_Q8, GN_QUP_Q8, GN_QLEV_M1_Q10, 5);
	if (gidx[0] == 0) {
		if (abs_s(sub(gain[1], *prev_gain)) > GAIN_INT_DB_Q8) {
			if (!*prev_err)		/* bit error: no gain excursion */
				gain[1] = *prev_gain;
			*prev_err = 1;
		} else {
			*prev_err = 0;
		}
		gain[0] = add(shr(gain[1], 1), shr(*prev_gain, 1));
	} else {
		*prev_err = 0;
		Word16 lo, hi;
		if (*prev_gain < gain[1]) {
			lo = *prev_gain;
			hi = gain[1];
		} else {
			lo = gain[1];
			hi = *prev_gain;
		}
		lo = sub(lo, SIX_Q8);
		hi = add(hi, SIX_Q8);
		if (lo < GN_QLO_Q8)
			lo = GN_QLO_Q8;
		if (hi > GN_QUP_Q8)
			hi = GN_QUP_Q8;
		gain[0] = quant_u_dec(sub(gidx[0], 1), lo, hi, SIX_Q12, 3);
	}
	*prev_gain = gain[1];
}

/* fec_code :908 -- unvoiced frames carry Hamming parity in spare bits */
MD void fec_code24(QuantParam *q)
{
	const int16_t *p84 = TB(pmat84), *p74 = TB(pmat74);
	int16_t c84[8], c74[7];
	q->pitch_index = (int16_t) (q->pitch_index + 1);	/* room for the UV code */
	if (q->uv_flag[0]) {
		q->pitch_index = UV_PIND;
		vgetbits(c84, q->msvq_index[0], 6, 4);
		sbc_enc(c84, 8, 4, p84);
		vsetbits(&q->bpvc_index[0], 3, 4, &c84[4]);
		vgetbits(c74, q->msvq_index[0], 2, 3);
		c74[3] = 0;
		sbc_enc(c74, 7, 4, p74);
		vsetbits(&q->fsvq_index, 7, 3, &c74[4]);
		vgetbits(c74, q->gain_index[1], 4, 4);
		sbc_enc(c74, 7, 4, p74);
		vsetbits(&q->fsvq_index, 4, 3, &c74[4]);
		vgetbits(c74, q->gain_index[1], 0, 1);
		vgetbits(&c74[1], q->gain_index[0], 2, 3);
		sbc_enc(c74, 7, 4, p74);
		vsetbits(&q->fsvq_index, 1, 2, &c74[4]);
		vsetbits(&q->jit_index[0], 0, 1, &c74[6]);
	}
	q->pitch_index = TB(pitch_enc)[q->pitch_index];
}

/* fec_decode :993 */
MD Word16 fec_decode24(QuantParam *q, Word16 erase)
{
	const int16_t *p84 = TB(pmat84), *p74 = TB(pmat74);
	int16_t c84[8], c74[7];
	q->pitch_index = TB(pitch_dec)[q->pitch_index];
	q->uv_flag[0] = q->pitch_index == UV_PIND;
	if (!q->uv_flag[0]) {
		erase |= (Word16) (q->pitch_index == INVAL_PIND);
		if (!erase)
			q->pitch_index = (int16_t) (q->pitch_index - 2);
	}
	if (q->uv_flag[0] && !erase) {
		vgetbits(c84, q->msvq_index[0], 6, 4);
		vgetbits(&c84[4], q->bpvc_index[0], 3, 4);
		Word16 bep = sbc_dec(c84, 8, 4, p84, TB(syntab84));
		erase |= (Word16) (bep == BEP_UNCORR);
		vsetbits(&q->msvq_index[0], 6, 4, c84);
		q->bpvc_index[0] = 0;
		if (!erase) {
			vgetbits(c74, q->msvq_index[0], 2, 3);
			c74[3] = 0;
			vgetbits(&c74[4], q->fsvq_index, 7, 3);
			sbc_dec(c74, 7, 4, p74, TB(syntab74));
			vsetbits(&q->msvq_index[0], 2, 3, c74);
			vgetbits(c74, q->gain_index[1], 4, 4);
			vgetbits(&c74[4], q->fsvq_index, 4, 3);
			sbc_dec(c74, 7, 4, p74, TB(syntab74));
			vsetbits(&q->gain_index[1], 4, 4, c74);
			vgetbits(c74, q->gain_index[1], 0, 1);
			vgetbits(&c74[1], q->gain_index[0], 2, 3);
			vgetbits(&c74[4], q->fsvq_index, 1, 2);
			vgetbits(&c74[6], q->jit_index[0], 0, 1);
			sbc_dec(c74, 7, 4, p74, TB(syntab74));
			vsetbits(&q->gain_index[1], 0, 1, c74);
			vsetbits(&q->gain_index[0], 2, 3, &c74[1]);
			q->jit_index[0] = 1;
		}
	}
	return erase;
}

/* melp_chn_write :109 -- 54 bits: fields into a bit buffer, then out in
 * bit_order (melp_chn.c:77) into chbuf[0..6] */
MN void melp_chn_write24(EncAna *E)
{
	QuantParam *q = &E->qpar;
	fec_code24(q);
	unsigned char bb[R24_BITS];
	BitCursor bc = {bb, 0};
	pack_code(q->gain_index[1], &bc, 5, 1);
	E->sync_bit = sub(1, E->sync_bit);
	pack_code(E->sync_bit, &bc, 1, 1);
	pack_code(q->gain_index[0], &bc, 3, 1);
	pack_code(q->pitch_index, &bc, 7, 1);
	pack_code(q->jit_index[0], &bc, 1, 1);
	pack_code(q->bpvc_index[0], &bc, NUM_BANDS - 1, 1);
	for (int s = 0; s < MSVQ_STAGES; s++)
		pack_code(q->msvq_index[s], &bc, (int16_t) msvq_bits(s), 1);
	pack_code(q->fsvq_index, &bc, 8, 1);
	const int16_t *order = TB(bit_order);
	BitCursor oc = {E->chbuf, 0};
	for (int i = 0; i < R24_BITS; i++)
		pack_code(bb[order[i]], &oc, 1, 8);
}

/* melp_chn_read :150 -- returns the erase flag */
MN Word16 melp_chn_read24(DecState *D, MelpParam *par, const MelpParam *prev)
{
	QuantParam *q = &D->qpar;
	unsigned char bb[R24_BITS];
	const int16_t *order = TB(bit_order);
	BitCursor ic = {D->chbuf, 0};
	Word16 erase = 0, v;
	for (int i = 0; i < R24_BITS; i++) {
		/* ERASE_MASK & an unsigned char is always 0 */
		erase |= unpack_code(&ic, &v, 1, 8, 0x4000);
		bb[order[i]] = (unsigned char) v;
	}
	BitCursor bc = {bb, 0};
	unpack_code(&bc, &q->gain_index[1], 5, 1, 0);
	unpack_code(&bc, &v, 1, 1, 0);		/* sync bit */
	unpack_code(&bc, &q->gain_index[0], 3, 1, 0);
	unpack_code(&bc, &q->pitch_index, 7, 1, 0);
	unpack_code(&bc, &q->jit_index[0], 1, 1, 0);
	unpack_code(&bc, &q->bpvc_index[0], NUM_BANDS - 1, 1, 0);
	for (int s = 0; s < MSVQ_STAGES; s++)
		unpack_code(&bc, &q->msvq_index[s], (int16_t) msvq_bits(s), 1, 0);
	unpack_code(&bc, &q->fsvq_index, 8, 1, 0);
	q->uv_flag[0] = 0;
	erase = fec_decode24(q, erase);
	if (erase) {		/* frame repeat, both gains = the last one */
		*par = *prev;
		par->gain[0] = par->gain[NUM_GAINFR - 1];
	} else {
		vq_msd2(TB(msvq_cb), par->lsf, TB(msvq_cb_mean), q->msvq_index, MSVQ_STAGES, true,
			LPC_ORD, 2);
		if (q->uv_flag[0])
			v_set(par->fs_mag, 8192, NUM_HARM);
		else
			vq_msd2(TB(fsvq_cb), par->fs_mag, nullptr, &q->fsvq_index, 1, false, NUM_HARM,
				0);
		q_gain_dec(&D->qgd_prev_gain, &D->qgd_prev_err, par->gain, q->gain_index);
		par->uv_flag = q->uv_flag[0];
		if (q->uv_flag[0])
			par->pitch = UV_PITCH_Q7;
		else
			par->pitch = pow10_fxp(quant_u_dec(q->pitch_index, PIT_QLO_Q12, PIT_QUP_Q12,
							   PIT_QLEV_M1_Q8, 7), 7);
		par->jitter = q->jit_index[0] == 0 ? (int16_t) 0 : (int16_t) MAX_JITTER_Q15;
		q_bpvc_dec(par->bpvc, q->bpvc_index[0], q->uv_flag[0], NUM_BANDS);
	}
	return erase;
}

/* analysis() at RATE2400: one NPP-processed 180-sample frame -> chbuf[0..6] */
MN void analysis24(EncAna *E, const int16_t *sp_in)
{
	MelpParam *par = &E->par[0];
	QuantParam *q = &E->qpar;
	int16_t lpc[LPC_ORD + 1], w[LPC_ORD];
	dc_rmv(sp_in, &E->hpspeech[OLD_IN_BEG], E->dcdelin, E->dcdelout_hi, E->dcdelout_lo, FRAME);
	melp_ana<true>(E, &E->hpspeech[0], par, 0);
	lpc[0] = 4096;
	v_copy(&lpc[1], E->top_lpc, LPC_ORD);
	vq_lspw(w, par->lsf, &lpc[1], LPC_ORD);
	vq_ms4_lsf(TB(msvq_cb), par->lsf, TB(msvq_cb_mean), w, q->msvq_index);
	lpc_clmp(par->lsf, 409, LPC_ORD);
	par->pitch = log10_fxp(par->pitch, 7);
	quant_u(&par->pitch, &q->pitch_index, PIT_QLO_Q12, PIT_QUP_Q12, PIT_QLEV_M1, PIT_QLEV_M1_Q8,
		true, 7);
	par->pitch = pow10_fxp(par->pitch, 7);
	q_gain(&E->qg_prev_gain, par->gain, q->gain_index);
	if (par->jitter < shr(MAX_JITTER_Q15, 1)) {
		par->jitter = 0;
		q->jit_index[0] = 0;
	} else {
		par->jitter = MAX_JITTER_Q15;
		q->jit_index[0] = 1;
	}
	par->uv_flag = q_bpvc(par->bpvc, &q->bpvc_index[0], NUM_BANDS);
	v_set(par->fs_mag, 8192, NUM_HARM);
	if (!par->uv_flag) {
		lpc_lsp2pred(par->lsf, &lpc[1], LPC_ORD);
		zerflt(&E->hpspeech[FRAME_END - LPC_FRAME / 2], lpc, E->sigbuf, LPC_ORD, LPC_FRAME);
		window(E->sigbuf, TB(win_cof), E->sigbuf, LPC_FRAME);
		find_harm(E->sigbuf, par->fs_mag, par->pitch, NUM_HARM, LPC_FRAME);
	}
	window_Q(par->fs_mag, g_der.w_fs, par->fs_mag, NUM_HARM, 14);
	vq_enc<NUM_HARM>(TB(fsvq_cb), par->fs_mag, 256, par->fs_mag, &q->fsvq_index);
	q->uv_flag[0] = par->uv_flag;
	melp_chn_write24(E);
	v_copy(E->hpspeech, &E->hpspeech[FRAME], IN_BEG);
}

/* synthesis() at RATE2400: chbuf[0..6] -> 180 samples */
MN void decode_frame24(DecState *D, int16_t *out)
{
	if (D->syn_begin > 0)
		v_copy(out, D->sigsave, D->syn_begin);
	D->erase = melp_chn_read24(D, &D->par[0], &D->prev_par);
	D->par[0].uv_flag = D->qpar.uv_flag[0];
	melp_syn<true>(D, &D->par[0], out);
}

}  // namespace mlp

#endif
