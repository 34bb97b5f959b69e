/*
 * decoder.h -- one superframe of MELPe-1200 decoding for one channel:
 * melpe_s (melpe/melpe.c:102-107) = unpack + dequantise + synthesis.
 *
 * Restates melpe/melp_syn.c (synthesis, melp_syn), melpe/harm.c
 * (harm_syn_pitch, realIDFT, set_fc), melpe/postfilt.c, melpe/melp_chn.c
 * (low_rate_chn_read), melpe/fec_code.c (low_rate_fec_decode) and the
 * decoder helpers of melpe/melp_sub.c (noise_est, noise_sup, lin_int_bnd,
 * scale_adj) and melpe/qnt12.c (deqnt_msvq), with every static in DecState.
 */
#ifndef MELPE_DECODER_H
#define MELPE_DECODER_H

#include "quant.h"

namespace mlp {

/* ------------------------------------------------------------------ */
/* melpe/melp_sub.c decoder helpers                                   */
/* ------------------------------------------------------------------ */

/* lin_int_bnd :424 */
MD Word16 lin_int_bnd(Word16 x, Word16 xmin, Word16 xmax, Word16 ymin, Word16 ymax)
{
	if (x <= xmin)
		return ymin;
	if (x >= xmax)
		return ymax;
	Word16 t = mult(sub(x, xmin), sub(ymax, ymin));
	return add(ymin, divide_s(t, sub(xmax, xmin)));
}

/* noise_est :465 */
MD void noise_est(Word16 gain, int16_t *ng, Word16 up, Word16 down, Word16 mn, Word16 mx)
{
	Word32 Lng = L_deposit_h(*ng);
	Word16 t1 = r_ound(L_add(Lng, L_shl(L_deposit_l(up), 5)));
	Word16 t2 = r_ound(L_add(Lng, L_shl(L_deposit_l(down), 7)));
	if (gain > t1)
		*ng = t1;
	else if (gain < t2)
		*ng = t2;
	else
		*ng = gain;
	if (*ng < mn)
		*ng = mn;
	if (*ng > mx)
		*ng = mx;
}

/* noise_sup :513 */
MN void noise_sup(int16_t *gain, Word16 ng, Word16 max_noise, Word16 max_att, Word16 nfact)
{
	Word16 sup;
	if (ng > max_noise)
		ng = max_noise;
	Word16 lev = sub(*gain, add(ng, nfact));
	if (lev > 0) {
		Word16 t = extract_h(L_shl(L_mult(-3276, lev), 4));
		t = pow10_fxp(t, 14);
		t = sub(16384, t);
		sup = mult(-20480, log10_fxp(t, 14));
		if (sup > max_att)
			sup = max_att;
	} else {
		sup = max_att;
	}
	*gain = sub(*gain, sup);
}

/* scale_adj :768 -- match the period's energy to the target gain with a
 * SCALEOVER-sample cross-fade from the previous scale */
/* scale_adj; msq0 >= 0: the first energy (L_v_magsq of sp >> 4), already
 * summed by the caller (syn_chain); out: where the scaled samples go (sp
 * itself, or the caller's next buffer, which saves a copy pass) */
MN void scale_adj(DecState *D, int16_t *sp, Word16 gain, int len, Word16 over, Word16 inv_over,
		  Word32 msq0 = -1, int16_t *out = nullptr)
{
	PROF_SCOPE(21);
	Word16 sh = 4, t;
	if (!out)
		out = sp;
#if defined(MELPE_OPCOUNT)
	/* census build: the reference's passes */
	int16_t tb[PITCHMAX + 8];
	v_equ_shr(tb, sp, sh, len);
	Word32 msq = L_v_magsq(tb, len, 0, 1);
	(void) msq0;
#else
	/* L_v_magsq(tb, len, 0, 1) of tb = sp >> 4: its final shift is 0 */
	Word32 msq = msq0 >= 0 ? msq0 : magsq_shr(sp, len, sh);
#endif
	if (msq) {
		t = sub(norm_l(msq), 1);
		sh = sub(sh, shr(t, 1));
	} else {
		sh = 0;
	}
#if defined(MELPE_OPCOUNT)
	v_equ_shr(tb, sp, sh, len);
	msq = L_v_magsq(tb, len, 0, 0);
#else
	/* L_v_magsq(tb, len, 0, 0) of tb = sp >> sh: its final shift is -1 */
	msq = L_shl(magsq_shr(sp, len, sh), -1);
#endif
	sh = shl(sh, 1);
	t = shl(256, sh);
	sh = log10_fxp(t, 8);
	msq = L_add(msq, 1);
	Word16 lmsq = L_log10_fxp(msq, 0);
	msq = L_add(L_shl(L_deposit_l(lmsq), 1), L_deposit_l(sh));
	Word16 llen = log10_fxp(shl((Word16) len, 7), 7);
	Word32 L = L_shl(L_deposit_l(gain), 1);
	L = L_sub(L, msq);
	L = L_add(L, L_deposit_l(llen));
	L = L_shr(L, 1);
	Word16 scale = pow10_fxp(extract_l(L), 13);
	for (int i = 1; i < over; i++) {
		t = shl(sub(over, (Word16) i), 11);
		t = extract_h(L_shl(L_mult(t, inv_over), 1));
		Word32 i1 = L_mult(D->prev_scale, t);
		t = shl((Word16) i, 11);
		t = extract_h(L_shl(L_mult(t, inv_over), 1));
		Word32 i2 = L_mult(scale, t);
		Word32 s = extract_h(L_add(i1, i2));
		out[i - 1] = extract_h(L_shl(L_mult(sp[i - 1], (Word16) s), 2));
	}
#if defined(MELPE_OPCOUNT)
	v_scale_shl(&sp[over - 1], scale, (int16_t) (len - over + 1), 2);
#else
	v_batch(&sp[over - 1], &out[over - 1], len - over + 1, [scale](int, int16_t x) {
		return (int16_t) extract_h(L_shl(L_mult(x, scale), 2));	/* v_scale_shl :462 */
	});
#endif
	D->prev_scale = scale;
}

/* deqnt_msvq, melpe/qnt12.c:1158 */
MD void deqnt_msvq(int16_t *qout, const int16_t *cb, int tos, const int16_t *cb_size,
		   const int16_t *index, int dim)
{
	v_zero(qout, dim);
	const int16_t *p = cb;
	for (int i = 0; i < tos; i++) {
		v_add(qout, p + extract_l(L_shr(L_mult(index[i], (Word16) dim), 1)), dim);
		p += extract_l(L_shr(L_mult(cb_size[i], (Word16) dim), 1));
	}
}

/* ------------------------------------------------------------------ */
/* FEC decode, melpe/fec_code.c                                        */
/* ------------------------------------------------------------------ */

MD Word16 sbc_syn(const int16_t *x, int n, int k, const int16_t *pmat)
{
	Word16 r = 0;
	for (int i = k, j = n - k - 1; i < n; i++, j--, pmat += k)
		r = add(r, (Word16) ((x[i] ^ binprod(x, pmat, k)) << j));
	return r;
}

MD Word16 sbc_dec(int16_t *x, int n, int k, const int16_t *pmat, const int16_t *syntab)
{
	Word16 bep = syntab[sbc_syn(x, n, k, pmat)];
	if (bep > -1)
		x[bep] ^= 1;
	return bep;
}

MD Word16 crc4_dec(const int16_t *bit, int nbits)
{
	int16_t d[4];
	for (int i = 1; i <= 4; i++)
		d[4 - i] = bit[nbits - i];
	for (int i = 5; i <= nbits; i++) {
		int16_t x = d[3];
		d[3] = d[2];
		d[2] = d[1];
		d[1] = (int16_t) (x ^ d[0]);
		d[0] = (int16_t) (x ^ bit[nbits - i]);
	}
	return (Word16) (d[0] | d[1] | d[2] | d[3]);
}

/* low_rate_fec_decode :1062 */
MD Word16 low_rate_fec_decode(QuantParam *q, Word16 erase, int16_t *lsp_check)
{
	if (!(q->uv_flag[0] && q->uv_flag[1] && q->uv_flag[2]))
		return erase;
	int16_t c84[8], c74[7], c13[13];
	const int16_t *p84 = TB(pmat84), *p74 = TB(pmat74);
	vgetbits(c84, q->gain_index[0], 9, 4);
	vgetbits(&c84[4], q->fs_index, 7, 4);
	Word16 b = sbc_dec(c84, 8, 4, p84, TB(syntab84));
	erase |= b == -2;
	vsetbits(q->gain_index, 9, 4, c84);
	vgetbits(c84, q->gain_index[0], 5, 4);
	vgetbits(&c84[4], q->fs_index, 3, 4);
	b = sbc_dec(c84, 8, 4, p84, TB(syntab84));
	erase |= b == -2;
	vsetbits(q->gain_index, 5, 4, c84);
	if (!erase) {
		vgetbits(c74, q->gain_index[0], 1, 2);
		c74[2] = c74[3] = 0;
		vgetbits(&c74[4], q->bpvc_index[0], 1, 2);
		vgetbits(&c74[6], q->jit_index[0], 0, 1);
		sbc_dec(c74, 7, 4, p74, TB(syntab74));
		vsetbits(q->gain_index, 1, 2, c74);
		for (int f = 0; f < NF; f++) {
			vgetbits(&c13[4], q->lsf_index[f][0], 8, 9);
			vgetbits(&c13[0], q->lsf_index[f][1], 3, 4);
			lsp_check[f] = crc4_dec(c13, 13);
		}
	}
	return erase;
}

/* ------------------------------------------------------------------ */
/* low_rate_chn_read, melpe/melp_chn.c:456-1362                         */
/* ------------------------------------------------------------------ */

MD void set_uv3(QuantParam *q, MelpParam *par, int16_t a, int16_t b, int16_t c)
{
	q->uv_flag[0] = par[0].uv_flag = a;
	q->uv_flag[1] = par[1].uv_flag = b;
	q->uv_flag[2] = par[2].uv_flag = c;
}

/* the pitch-index interpretation shared by three branches of the UV
 * pattern decoding (melp_chn.c:549-600 etc.): low_rate_pitch_dec, then the
 * popcount of the raw index picks the single-voiced pattern; `prot` is the
 * protection field that must agree, `uuu_prot` the one for all-unvoiced */
MD void rd_pitch_pattern(QuantParam *q, MelpParam *par, Word16 uuu_prot, Word16 prot_bp2,
			 Word16 *erase_uuu, int16_t *fl_lsp, int16_t *fl_pitch)
{
	int j = q->pitch_index;
	q->pitch_index = TB(low_rate_pitch_dec)[q->pitch_index];
	if (q->pitch_index == 0) {	/* UV_PIND */
		set_uv3(q, par, 1, 1, 1);
		if (uuu_prot != 0) {
			*erase_uuu |= 1;
			*fl_lsp = 0;
			*fl_pitch = 0;
		}
	} else if (q->pitch_index == 1) {	/* INVAL_PIND */
		*erase_uuu |= 1;
		*fl_lsp = 0;
		*fl_pitch = 0;
	} else {
		q->pitch_index -= 2;
		int k = 0;
		for (int i = 0; i < 9; i++) {
			if ((j & 1) == 1)
				k++;
			j >>= 1;
		}
		int want = -1;
		if (k == 6 || k == 7) {
			set_uv3(q, par, 1, 1, 0);
			want = 1;
		} else if (k == 4) {
			set_uv3(q, par, 1, 0, 1);
			want = 2;
		} else if (k == 5) {
			set_uv3(q, par, 0, 1, 1);
			want = 3;
		}
		if (want >= 0 && prot_bp2 != want) {
			*erase_uuu |= 1;
			*fl_lsp = 0;
			*fl_pitch = 0;
		}
	}
}

MN Word16 low_rate_chn_read(DecState *D)
{
	PROF_SCOPE(17);
	QuantParam *q = &D->qpar;
	MelpParam *par = D->par;
	const MelpParam *prev = &D->prev_par;
	const int16_t v_cb_size[4] = {256, 64, 32, 32};
	const int16_t res_cb_size[4] = {256, 64, 64, 64};
	const int16_t uv_cb_size[1] = {512};
	unsigned char bb[81];
	int16_t lsp_check[NF] = {0, 0, 0};
	int16_t il1[LPC_ORD], il2[LPC_ORD], res[2 * LPC_ORD], wfs[NUM_HARM];
	Word16 erase = 0, erase_uuu = 0, erase_vvv = 0, flag_parity = 0;
	int16_t fl_lsp = 1, fl_pitch = 1;
	Word16 idx, dontcare, uv_index, uv_parity, prot_bp1, prot_bp2, prot_lsp;
	if (!D->rd_started) {
		Word16 t2 = shl(LPC_ORD, 10), t1 = 819;
		for (int i = 0; i < LPC_ORD; i++) {
			D->rd_qplsp[i] = divide_s(t1, t2);
			t1 = add(t1, 819);
		}
		v_set(D->rd_prev_gain, 2560, 2 * NF * NUM_GAINFR);
		v_set(D->rd_prev_fsmag, 8192, NUM_HARM);
		D->rd_started = 1;
	}
	/* chbuf -> one bit per byte (ERASE_MASK & byte is always 0) */
	BitCursor cc = {D->chbuf, 0};
	for (int i = 0; i < 81; i++) {
		erase |= unpack_code(&cc, &idx, 1, 8, 0x4000);
		bb[i] = (unsigned char) idx;
	}
	BitCursor bc = {bb, 0};
	unpack_code(&bc, &dontcare, 1, 1, 0);
	unpack_code(&bc, &uv_index, 3, 1, 0);
	unpack_code(&bc, &uv_parity, 1, 1, 0);
	unpack_code(&bc, &q->pitch_index, 9, 1, 0);
	BitCursor b1 = {bc.p + 39, 0};
	unpack_code(&b1, &prot_lsp, 3, 1, 0);
	unpack_code(&b1, &dontcare, 10, 1, 0);
	unpack_code(&b1, &dontcare, 2, 1, 0);
	unpack_code(&b1, &prot_bp2, 2, 1, 0);
	unpack_code(&b1, &prot_bp1, 2, 1, 0);
	if (uv_parity != parity(uv_index, 3))
		flag_parity |= 1;

	if (uv_index == 0) {
		if (!flag_parity || prot_bp1 == 0) {
			rd_pitch_pattern(q, par, prot_bp2, prot_bp2, &erase_uuu, &fl_lsp, &fl_pitch);
		} else {
			if (prot_bp2 == 1 && prot_lsp == 7)
				set_uv3(q, par, 0, 0, 1);
			else if (prot_bp2 == 2)
				set_uv3(q, par, 0, 1, 0);
			else if (prot_bp2 == 3)
				set_uv3(q, par, 1, 0, 0);
			else {
				erase_vvv |= 1;
				fl_lsp = 0;
				fl_pitch = 2;
			}
		}
	} else if (uv_index == 1 || uv_index == 2 || uv_index == 4) {
		if (!flag_parity) {
			if (uv_index == 1)
				set_uv3(q, par, 0, 0, 1);
			else if (uv_index == 2)
				set_uv3(q, par, 0, 1, 0);
			else
				set_uv3(q, par, 1, 0, 0);
		} else if (prot_bp1 == 0) {
			rd_pitch_pattern(q, par, prot_lsp, prot_bp2, &erase_uuu, &fl_lsp, &fl_pitch);
		} else if (prot_bp1 == 1 && prot_lsp == 7) {
			set_uv3(q, par, 0, 0, 1);
		} else {
			erase_vvv |= 1;
		}
	} else if (uv_index == 3 || uv_index == 5) {
		if (!flag_parity) {
			set_uv3(q, par, 0, 0, 0);
			if (uv_index == 5)
				q->pitch_index = (int16_t) (q->pitch_index + 512);
		} else if (prot_bp1 == 1 && prot_lsp == 7) {
			set_uv3(q, par, 0, 0, 1);
		} else {
			erase_vvv |= 1;
			if (uv_index == 5)
				q->pitch_index = (int16_t) (q->pitch_index + 512);
		}
	} else if (uv_index == 6) {
		if (!flag_parity) {
			set_uv3(q, par, 0, 0, 0);
			q->pitch_index = (int16_t) (q->pitch_index + 1024);
		} else {
			if (prot_bp1 == 2)
				set_uv3(q, par, 0, 1, 0);
			/* the reference's second test is not an else-if (melp_chn.c:808) */
			if (prot_bp1 == 3) {
				set_uv3(q, par, 1, 0, 0);
			} else {
				erase_vvv |= 1;
				q->pitch_index = (int16_t) (q->pitch_index + 1024);
			}
		}
	} else if (uv_index == 7) {
		if (!flag_parity)
			set_uv3(q, par, 0, 0, 0);
		else
			erase_vvv |= 1;
		q->pitch_index = (int16_t) (q->pitch_index + 1536);
	}
	if (erase_uuu)
		set_uv3(q, par, 1, 1, 1);
	if (erase_vvv)
		set_uv3(q, par, 0, 0, 0);

	int last = -1, cnt = 0;
	for (int i = 0; i < NF; i++)
		if (!q->uv_flag[i]) {
			cnt++;
			last = i;
		}
	const int16_t u1 = q->uv_flag[0], u2 = q->uv_flag[1], cu = q->uv_flag[2];
	int16_t (*L)[MAX_LSF_STAGE] = q->lsf_index;
	if (u1 == 1 && u2 == 1 && cu == 1) {
		unpack_code(&bc, &L[0][0], 9, 1, 0);
		unpack_code(&bc, &L[1][0], 9, 1, 0);
		unpack_code(&bc, &L[2][0], 9, 1, 0);
		unpack_code(&bc, &L[0][1], 4, 1, 0);
		unpack_code(&bc, &L[1][1], 4, 1, 0);
		unpack_code(&bc, &L[2][1], 4, 1, 0);
		unpack_code(&bc, &dontcare, 3, 1, 0);
	} else if (u1 == 1 && u2 == 1 && cu != 1) {
		unpack_code(&bc, &L[0][0], 9, 1, 0);
		unpack_code(&bc, &L[1][0], 9, 1, 0);
		unpack_code(&bc, &L[2][0], 8, 1, 0);
		unpack_code(&bc, &L[2][1], 6, 1, 0);
		unpack_code(&bc, &L[2][2], 5, 1, 0);
		unpack_code(&bc, &L[2][3], 5, 1, 0);
	} else if (u1 == 1 && u2 != 1 && cu == 1) {
		unpack_code(&bc, &L[0][0], 9, 1, 0);
		unpack_code(&bc, &L[1][0], 8, 1, 0);
		unpack_code(&bc, &L[1][1], 6, 1, 0);
		unpack_code(&bc, &L[1][2], 5, 1, 0);
		unpack_code(&bc, &L[1][3], 5, 1, 0);
		unpack_code(&bc, &L[2][0], 9, 1, 0);
	} else if (u1 != 1 && u2 == 1 && cu == 1) {
		unpack_code(&bc, &L[0][0], 8, 1, 0);
		unpack_code(&bc, &L[0][1], 6, 1, 0);
		unpack_code(&bc, &L[0][2], 5, 1, 0);
		unpack_code(&bc, &L[0][3], 5, 1, 0);
		unpack_code(&bc, &L[1][0], 9, 1, 0);
		unpack_code(&bc, &L[2][0], 9, 1, 0);
	} else {
		const bool vvu = (u1 != 1 && u2 != 1 && cu == 1);
		if (vvu) {
			unpack_code(&bc, &L[0][0], 9, 1, 0);
		} else {
			unpack_code(&bc, &L[0][0], 8, 1, 0);
			unpack_code(&bc, &L[0][1], 6, 1, 0);
			unpack_code(&bc, &L[0][2], 5, 1, 0);
			unpack_code(&bc, &L[0][3], 5, 1, 0);
		}
		unpack_code(&bc, &L[1][0], 4, 1, 0);
		if (vvu) {
			unpack_code(&bc, &L[2][0], 8, 1, 0);
			unpack_code(&bc, &L[2][1], 6, 1, 0);
			unpack_code(&bc, &L[2][2], 6, 1, 0);
			unpack_code(&bc, &L[2][3], 6, 1, 0);
			unpack_code(&bc, &dontcare, 3, 1, 0);
		} else {
			unpack_code(&bc, &L[2][0], 8, 1, 0);
			unpack_code(&bc, &L[2][1], 6, 1, 0);
		}
	}
	unpack_code(&bc, &q->gain_index[0], 10, 1, 0);
	for (int i = 0; i < NF; i++)
		if (!q->uv_flag[i])
			unpack_code(&bc, &q->bpvc_index[i], 2, 1, 0);
	if (cnt == 2) {
		unpack_code(&bc, &prot_bp1, 2, 1, 0);
	} else if (cnt == 1) {
		unpack_code(&bc, &prot_bp2, 2, 1, 0);
		unpack_code(&bc, &prot_bp1, 2, 1, 0);
	} else if (cnt == 0) {
		for (int i = 0; i < NF; i++)
			unpack_code(&bc, &q->bpvc_index[i], 2, 1, 0);
	}
	unpack_code(&bc, &q->fs_index, 8, 1, 0);
	unpack_code(&bc, &q->jit_index[0], 1, 1, 0);
	erase = low_rate_fec_decode(q, erase, lsp_check);

	/* pitch */
	if (fl_pitch == 1) {
		if (cnt == 0) {
			for (int i = 0; i < NF; i++)
				par[i].pitch = LOG_UV_PITCH_Q12;
		} else if (cnt == 1) {
			for (int i = 0; i < NF; i++) {
				if (!par[i].uv_flag)
					par[i].pitch = quant_u_dec(q->pitch_index, 5329, 9028, 25088, 7);
				else
					par[i].pitch = LOG_UV_PITCH_Q12;
				par[i].pitch = pow10_fxp(par[i].pitch, 7);
			}
		} else {
			const int16_t *cb = cnt == NF ? TB(pitch_vq_cb_vvv) : TB(pitch_vq_cb_uvv);
			int k = q->pitch_index;
			for (int i = 0; i < NF; i++)
				par[i].pitch = par[i].uv_flag == 1 ? (int16_t) UV_PITCH_Q7
								   : pow10_fxp(cb[k * NF + i], 7);
		}
	} else if (fl_pitch == 2) {
		const int16_t *cb = TB(pitch_vq_cb_uvv);
		int k = q->pitch_index;
		for (int i = 0; i < NF; i++)
			par[i].pitch = pow10_fxp(cb[k * NF + i], 7);
	}

	/* LSF */
	const int16_t *cb_uv = TB(lsp_uv_9), *cb_v = TB(lsp_v_256x64x32x32);
	if (fl_lsp) {
		if (u1 == 1 && u2 == 1 && cu == 1) {
			for (int f = 0; f < NF; f++)
				deqnt_msvq(par[f].lsf, cb_uv, 1, uv_cb_size, L[f], LPC_ORD);
		} else if (u1 == 1 && u2 == 1 && cu != 1) {
			deqnt_msvq(par[0].lsf, cb_uv, 1, uv_cb_size, L[0], LPC_ORD);
			deqnt_msvq(par[1].lsf, cb_uv, 1, uv_cb_size, L[1], LPC_ORD);
			deqnt_msvq(par[2].lsf, cb_v, 4, v_cb_size, L[2], LPC_ORD);
		} else if (u1 == 1 && u2 != 1 && cu == 1) {
			deqnt_msvq(par[0].lsf, cb_uv, 1, uv_cb_size, L[0], LPC_ORD);
			deqnt_msvq(par[1].lsf, cb_v, 4, v_cb_size, L[1], LPC_ORD);
			deqnt_msvq(par[2].lsf, cb_uv, 1, uv_cb_size, L[2], LPC_ORD);
		} else if (u1 != 1 && u2 == 1 && cu == 1) {
			deqnt_msvq(par[0].lsf, cb_v, 4, v_cb_size, L[0], LPC_ORD);
			deqnt_msvq(par[1].lsf, cb_uv, 1, uv_cb_size, L[1], LPC_ORD);
			deqnt_msvq(par[2].lsf, cb_uv, 1, uv_cb_size, L[2], LPC_ORD);
		} else {
			const bool vvu = (u1 != 1 && u2 != 1 && cu == 1);
			if (vvu)
				deqnt_msvq(par[2].lsf, cb_uv, 1, uv_cb_size, L[0], LPC_ORD);
			else
				deqnt_msvq(par[2].lsf, cb_v, 4, v_cb_size, L[0], LPC_ORD);
			const int16_t *ic = TB(inpCoef) + L[1][0] * 20;
			for (int j = 0; j < LPC_ORD; j++) {
				Word16 f = ic[j];
				Word32 acc = L_mult(f, D->rd_qplsp[j]);
				acc = L_mac(acc, sub(16384, f), par[2].lsf[j]);
				il1[j] = extract_h(L_shl(acc, 1));
				f = ic[j + LPC_ORD];
				acc = L_mult(f, D->rd_qplsp[j]);
				acc = L_mac(acc, sub(16384, f), par[2].lsf[j]);
				il2[j] = extract_h(L_shl(acc, 1));
			}
			deqnt_msvq(res, TB(res256x64x64x64), vvu ? 4 : 2, res_cb_size, L[2], 20);
			for (int i = 0; i < LPC_ORD; i++) {
				par[0].lsf[i] = add(shr(res[i], 2), il1[i]);
				par[1].lsf[i] = add(shr(res[i + LPC_ORD], 2), il2[i]);
			}
		}
		if (u1 == 1 && u2 == 1 && cu == 1) {
			const int c0 = lsp_check[0], c1 = lsp_check[1], c2 = lsp_check[2];
			for (int i = 0; i < LPC_ORD; i++) {
				if (c0 == 1 && c1 == 1 && c2 == 1) {
					par[0].lsf[i] = par[1].lsf[i] = par[2].lsf[i] = prev->lsf[i];
				} else if (c0 == 1 && c1 == 1 && c2 == 0) {
					par[0].lsf[i] = add(mult(prev->lsf[i], 21845), mult(par[2].lsf[i], 10923));
					par[1].lsf[i] = add(mult(prev->lsf[i], 10923), mult(par[2].lsf[i], 21845));
				} else if (c0 == 1 && c1 == 0 && c2 == 1) {
					par[0].lsf[i] = add(shr(prev->lsf[i], 1), shr(par[1].lsf[i], 1));
					par[2].lsf[i] = par[1].lsf[i];
				} else if (c0 == 0 && c1 == 1 && c2 == 1) {
					par[1].lsf[i] = par[0].lsf[i];
					par[2].lsf[i] = par[0].lsf[i];
				} else if (c0 == 1 && c1 == 0 && c2 == 0) {
					par[0].lsf[i] = add(shr(prev->lsf[i], 1), shr(par[1].lsf[i], 1));
				} else if (c0 == 0 && c1 == 1 && c2 == 0) {
					par[1].lsf[i] = add(shr(par[0].lsf[i], 1), shr(par[2].lsf[i], 1));
				} else if (c0 == 0 && c1 == 0 && c2 == 1) {
					par[2].lsf[i] = par[1].lsf[i];
				}
			}
		}
		for (int f = 0; f < NF; f++)
			if (!lspStable(par[f].lsf, LPC_ORD))
				lspSort(par[f].lsf, LPC_ORD);
		v_copy(D->rd_qplsp, par[NF - 1].lsf, LPC_ORD);
	} else {
		for (int i = 0; i < NF; i++)
			v_copy(par[i].lsf, prev->lsf, LPC_ORD);
		v_copy(D->rd_qplsp, par[NF - 1].lsf, LPC_ORD);
	}

	/* gain, bandpass voicing, Fourier magnitudes, jitter */
	const int16_t *gcb = TB(gain_vq_cb) + q->gain_index[0] * NUM_GAINFR * NF;
	for (int i = 0; i < NF; i++)
		for (int j = 0; j < NUM_GAINFR; j++)
			par[i].gain[j] = gcb[i * NUM_GAINFR + j];
	for (int i = 0; i < NF; i++)
		q_bpvc_dec(par[i].bpvc, TB(inv_bp_index_map)[q->bpvc_index[i]], q->uv_flag[i],
			   NUM_BANDS);
	if (cnt != 0) {
		v_copy(par[last].fs_mag, TB(fsvq_cb) + NUM_HARM * q->fs_index, NUM_HARM);
		v_copy(wfs, par[last].fs_mag, NUM_HARM);
	}
	if (cnt > 1) {
		if (D->rd_prev_uv) {
			for (int i = 0; i < last; i++)
				if (!par[i].uv_flag)
					v_copy(par[i].fs_mag, par[last].fs_mag, NUM_HARM);
		} else if (par[0].uv_flag) {
			v_copy(par[1].fs_mag, par[last].fs_mag, NUM_HARM);
		} else if (par[1].uv_flag) {
			v_copy(par[0].fs_mag, D->rd_prev_fsmag, NUM_HARM);
		} else if (par[2].uv_flag) {
			for (int i = 0; i < NUM_HARM; i++)
				par[0].fs_mag[i] = add(shr(wfs[i], 1), shr(D->rd_prev_fsmag[i], 1));
		} else {
			for (int i = 0; i < NUM_HARM; i++) {
				Word16 p = D->rd_prev_fsmag[i], v = wfs[i];
				par[0].fs_mag[i] = add(mult(p, 21845), mult(v, 10923));
				par[1].fs_mag[i] = add(mult(p, 10923), mult(v, 21845));
			}
		}
	}
	D->rd_prev_uv = par[NF - 1].uv_flag;
	if (par[NF - 1].uv_flag) {
		v_set(D->rd_prev_fsmag, 8192, NUM_HARM);
		window_Q(D->rd_prev_fsmag, g_der.w_fs, D->rd_prev_fsmag, NUM_HARM, 14);
	} else {
		v_copy(D->rd_prev_fsmag, par[NF - 1].fs_mag, NUM_HARM);
	}
	for (int i = 0; i < NF; i++)
		par[i].jitter = par[i].uv_flag == 1 ? (int16_t) MAX_JITTER_Q15 : (int16_t) 0;
	if (cnt != 0 || !(u1 == 0 && u2 == 1 && cu == 0)) {
		if (q->jit_index[0] == 1) {
			if (u1 && u2 && cu)
				;
			else if (u1 && u2 && !cu)
				par[2].jitter = MAX_JITTER_Q15;
			else if (u1 && !u2 && cu)
				par[1].jitter = MAX_JITTER_Q15;
			else if (!u1 && u2 && cu)
				par[0].jitter = MAX_JITTER_Q15;
			else if (u1 && !u2 && !cu)
				par[1].jitter = MAX_JITTER_Q15;
			else if (!u1 && u2 && !cu)
				;
			else if (!u1 && !u2 && cu)
				par[1].jitter = MAX_JITTER_Q15;
			else
				par[0].jitter = par[1].jitter = par[2].jitter = MAX_JITTER_Q15;
		}
	}

	/* smoothing on parity errors / gain jumps (melp_chn.c:1268-1325) */
	const Word16 SM = 16383, SM1 = sub(32767, 16383);
	if (flag_parity) {
		Word16 p = prev->pitch;
		for (int i = 0; i < NF; i++) {
			if (par[i].uv_flag)
				par[i].pitch = UV_PITCH_Q7;
			else
				par[i].pitch = add(mult(SM, p), mult(SM1, par[i].pitch));
			p = par[i].pitch;
		}
		p = prev->gain[1];
		for (int i = 0; i < NF; i++)
			for (int j = 0; j < NUM_GAINFR; j++) {
				par[i].gain[j] = add(mult(SM, p), mult(SM1, par[i].gain[j]));
				p = par[i].gain[j];
			}
		for (int j = 0; j < LPC_ORD; j++) {
			p = prev->lsf[j];
			for (int i = 0; i < NF; i++) {
				par[i].lsf[j] = add(mult(SM, p), mult(SM1, par[i].lsf[j]));
				p = par[i].lsf[j];
			}
		}
	} else {
		Word32 s1 = 0, s2 = 0;
		for (int i = 0; i < 2 * NF * NUM_GAINFR; i++)
			s1 = L_add(s1, L_deposit_l(D->rd_prev_gain[i]));
		s1 = L_shr(s1, 1);
		for (int i = 0; i < NF; i++)
			for (int j = 0; j < NUM_GAINFR; j++)
				s2 = L_add(s2, L_deposit_l(par[i].gain[j]));
		if (s2 > L_add(s1, 92160L) || s2 < L_sub(s1, 92160L)) {
			s1 = L_mpy_ls(L_shr(s1, 1), 10923);
			Word16 t = extract_l(s1);
			for (int i = 0; i < NF; i++)
				for (int j = 0; j < NUM_GAINFR; j++) {
					par[i].gain[j] = add(mult(SM, t), mult(SM1, par[i].gain[j]));
					t = par[i].gain[j];
				}
		}
	}
	for (int i = 0; i < NF * NUM_GAINFR; i++)
		D->rd_prev_gain[i] = D->rd_prev_gain[i + NF * NUM_GAINFR];
	for (int i = 0; i < NF; i++)
		for (int j = 0; j < NUM_GAINFR; j++)
			D->rd_prev_gain[NF * NUM_GAINFR + i * NUM_GAINFR + j] = par[i].gain[j];

	if (erase) {
		for (int i = 0; i < NF; i++) {
			par[i].pitch = UV_PITCH_Q7;
			v_copy(par[i].lsf, prev->lsf, LPC_ORD);
			par[i].gain[0] = par[i].gain[1] = prev->gain[1];
			v_zero(par[i].bpvc, NUM_BANDS);
			v_set(par[i].fs_mag, 8192, NUM_HARM);
			par[i].jitter = MAX_JITTER_Q15;
		}
		v_copy(D->rd_qplsp, par[NF - 1].lsf, LPC_ORD);
		D->rd_prev_uv = 1;
		v_set(D->rd_prev_fsmag, 8192, NUM_HARM);
	} else if (erase_uuu) {
		for (int i = 0; i < NF; i++) {
			par[i].pitch = UV_PITCH_Q7;
			v_zero(par[i].bpvc, NUM_BANDS);
			v_set(par[i].fs_mag, 8192, NUM_HARM);
			par[i].jitter = MAX_JITTER_Q15;
		}
		D->rd_prev_uv = 1;
		v_set(D->rd_prev_fsmag, 8192, NUM_HARM);
	} else if (erase_vvv) {
		for (int i = 0; i < NF; i++) {
			v_zero(&par[i].bpvc[1], NUM_BANDS - 1);
			v_set(par[i].fs_mag, 8192, NUM_HARM);
		}
		D->rd_prev_uv = 0;
		v_set(D->rd_prev_fsmag, 8192, NUM_HARM);
	}
	return erase;
}

/* ------------------------------------------------------------------ */
/* harmonic excitation, melpe/harm.c                                   */
/* ------------------------------------------------------------------ */

#ifndef IDFT_BLK
#define IDFT_BLK 12
#endif
static_assert(IDFT_BLK < PITCHMIN, "realIDFT's fast path reduces i + q mod len with one subtraction");

/* realIDFT's cosine table entry i for period len (melpe/harm.c:70-80) */
MD Word16 idft_cos_entry_w(Word16 w, int i)
{
	Word32 L = L_mult(w, (Word16) i);
	if (L > 524288L)
		L = L_sub(1048576L, L);
	else if (L == 524288L)
		L = L_sub(L, 1);
	return cos_fxp(extract_l(L_shr(L, 4)));
}

MD Word16 idft_cos_entry(Word16 len, int i)
{
	return idft_cos_entry_w(divide_s(16, len), i);	/* w = TWO_Q3 / len */
}

MD void derive_idft_cos(DerivedTables *d)
{
	for (int len = 1; len <= PITCHMAX; len++)
		for (int i = 0; i < len; i++)
			d->idft_cos[len][i] = idft_cos_entry((Word16) len, i);
}

/* Where realIDFT reads its cosine rows.  Lane-mode synthesis gathers one
 * entry per lane per harmonic, each lane from the row of its own period
 * length: through the vector memory path that is up to 64 cache lines per
 * instruction (the texture addresser's rate, not HBM, bounds it).  k_dec.hip
 * (MELPE_IDFT_LDS) stages the table packed in the block's LDS instead -- row
 * len at (len - 1) * len / 2, 12,880 entries, 25.8 KB shared by the block's
 * four waves -- where a gather costs bank cycles.  Elsewhere: g_der.  (Rows
 * stored twice over, so that an index in [0, 2 len) needs no reduction,
 * measured 14.2 vs 13.9 ms at 262,144 channels: the 51.5 KB table halves
 * the blocks a CU holds.) */
#define IDFT_LDS_WORDS (PITCHMAX * (PITCHMAX + 1) / 2)
#if defined(MELPE_IDFT_LDS)
extern __shared__ int16_t s_idft_cos[];
#define IDFT_ROW(len) (s_idft_cos + (((len) - 1) * (len)) / 2)
#else
#define IDFT_ROW(len) (g_der.idft_cos[len])
#endif
/* entry k in [0, 2 len) of a row */
#define IDFT_AT(c, k, len) ((c)[(k) >= (len) ? (k) - (len) : (k)])

/* (a + b) mod n for a, b in [0, n): the conditional subtraction as an
 * unsigned min (a + b - n wraps above a + b when a + b < n) */
MD int mod_add(int a, int b, int n)
{
	const unsigned s = (unsigned) (a + b), r = s - (unsigned) n;
	return (int) (s < r ? s : r);
}

/* phase mod len in [0, len); decoded phases lie in [0, len] */
MD int16_t idft_phase_mod(int p, int len)
{
	if ((unsigned) p >= (unsigned) len) {
		p -= len;
		if ((unsigned) p >= (unsigned) len) {
			p %= len;
			if (p < 0)
				p += len;
		}
	}
	return (int16_t) p;
}

/* realIDFT :63 -- direct real inverse DFT of one pitch period.  The
 * reference steps the cosine index k by adding phase[j], wrapping into
 * [0, len), then subtracting phase[j] and adding i, so before harmonic j
 * it is (j*i + phase[j]) mod len; that index is carried incrementally here
 * (one conditional subtraction per step, phase[j] reduced mod len once).  The
 * cosines come from the per-len table built at init. */
MN void realIDFT(int16_t *mag, const int16_t *phase, int16_t *sig, Word16 len)
{
	PROF_SCOPE(49);
	Word16 len2 = add(shr(len, 1), 1);
	Word16 w = divide_s(16, len);	/* TWO_Q3 */
#if defined(MELPE_OPCOUNT)
	/* census build: the reference's own sequence of basic ops (c[] built
	 * per call, index stepped with add/sub wraps), same values */
	int16_t cbuf[PITCHMAX];
	for (int i = 0; i < len; i++)
		cbuf[i] = idft_cos_entry_w(w, i);
	const int16_t *c = cbuf;
#else
	const int16_t *c = IDFT_ROW(len);
	int16_t phm[PITCHMAX / 2 + 1];
#endif
	w = shr(w, 1);
	Word16 w2 = shr(w, 1);
	Word16 t = sub(len2, 1);
	int i;
#if defined(MELPE_OPCOUNT)
	mag[0] = mult(mag[0], w2);
	for (i = 1; i < t; i++)
		mag[i] = mult(mag[i], w);
	if (shl((Word16) i, 1) == len)
		mag[i] = mult(mag[i], w2);
	else
		mag[i] = mult(mag[i], w);
#else
	/* one pass over the harmonics: the magnitude scaling (w2 on the first
	 * and, for an even len, the last), the fast path's bound A = sum |mag|,
	 * phase[j] mod len, and the fast path's packed (2 mag, phase) word; the
	 * next harmonic's inputs are loaded before this one's stores */
	int A = 0;
	int pk[PITCHMAX / 2 + 2];	/* (2 mag[j]) * 256 + (phase[j] mod len): len <= PITCHMAX < 256 */
	{
		const bool even = shl(t, 1) == len;
		int16_t mn = mag[0], pn = 0;
		for (int j = 0; j < len2; j++) {
			const int16_t mj = mn, pj = pn;
			if (j + 1 < len2) {
				mn = mag[j + 1];
				pn = phase[j + 1];
			}
			const Word16 m = mult(mj, (j == 0 || (j == t && even)) ? w2 : w);
			mag[j] = m;
			A += m < 0 ? -m : m;
			if (j) {
				const int16_t p = idft_phase_mod(pj, len);
				phm[j] = p;
				pk[j] = 2 * (int) m * 256 + p;
			}
		}
		pk[len2] = 0;
	}
#endif
#if !defined(MELPE_OPCOUNT)
	/* No-clamp fast path.  Every partial sum of an output's chain is
	 * mag[0] * 2^16 plus terms 2 mag[j] c[k] with |c| <= 2^15, so with
	 * A = sum |mag[j]| (j = 0 .. len2-1) it stays within A * 2^16, and the
	 * rounding adds 2^15: A <= 32766 proves neither L_mac nor r_ound can
	 * clamp, the chain is an exact integer sum in any order, and each term
	 * is one 24-bit multiply-add (|2 mag| < 2^17).  Decoded magnitudes are
	 * scaled by 2/len, so this is the common case; a wave with any lane
	 * outside it runs the saturating chain below for all of them.
	 *
	 * Loop order: harmonic j outer, the block's IDFT_BLK outputs inner.
	 * Output t reads entry (j t + phase[j]) mod len, so along the block
	 * the index steps by j (< len: one conditional subtraction, done as an
	 * unsigned min), and the block's first index follows from
	 * base = (j i) mod len, stepped by i per harmonic.  The block's table
	 * gathers are issued together before its multiply-adds, and harmonic
	 * j + 1's (2 mag, phase) word is loaded while j's are in flight. */
	{
		if (wave_all(A <= 32766)) {
			const int m0 = (int) mag[0] * 65536 + 32768;
			for (i = 0; i < len; i += IDFT_BLK) {
				int Lq[IDFT_BLK];
#pragma unroll
				for (int q = 0; q < IDFT_BLK; q++)
					Lq[q] = m0;
				int base = 0;	/* (j * i) mod len */
				int nxt = pk[1];
				for (int j = 1; j < len2; j++) {
					const int cur = nxt;
					nxt = pk[j + 1];
					const int m2 = cur >> 8;
					base = mod_add(base, i, len);
					int k = mod_add(base, cur & 255, len);
					int cv[IDFT_BLK];
#pragma unroll
					for (int q = 0; q < IDFT_BLK; q++) {
						cv[q] = c[k];
						k = mod_add(k, j, len);
					}
#pragma unroll
					for (int q = 0; q < IDFT_BLK; q++)
						Lq[q] += m2 * cv[q];
				}
#pragma unroll
				for (int q = 0; q < IDFT_BLK; q++)
					if (i + q < len)
						sig[i + q] = (int16_t) (Lq[q] >> 16);
			}
			return;
		}
	}
#endif
	for (i = 0; i < len; i++) {
		Word32 L = L_deposit_h(mag[0]);
#if defined(MELPE_OPCOUNT)
		Word16 k = (Word16) i;
		for (int j = 1; j < len2; j++) {
			k = add(k, phase[j]);
			while (k < 0)
				k = add(k, len);
			while (k >= len)
				k = sub(k, len);
			L = L_mac(L, mag[j], c[k]);
			k = sub(k, phase[j]);
			k = add(k, (Word16) i);
		}
#else
		if (i + IDFT_BLK <= len) {
			/* IDFT_BLK output samples at once: independent L_mac
			 * chains (each in the reference's j order) sharing the
			 * mag[] / phm[] loads, table gathers issued together */
			Word32 Lq[IDFT_BLK];
			int bq[IDFT_BLK];	/* (j * (i + q)) mod len */
#pragma unroll
			for (int q = 0; q < IDFT_BLK; q++) {
				Lq[q] = L;
				bq[q] = 0;
			}
			for (int j = 1; j < len2; j++) {
				Word16 m = mag[j];
				int p = phm[j];
				int16_t cv[IDFT_BLK];
#pragma unroll
				for (int q = 0; q < IDFT_BLK; q++) {
					bq[q] += i + q;
					if (bq[q] >= len)
						bq[q] -= len;
					int k = bq[q] + p;
					if (k >= len)
						k -= len;
					cv[q] = c[k];
				}
#pragma unroll
				for (int q = 0; q < IDFT_BLK; q++)
					Lq[q] = L_mac(Lq[q], m, cv[q]);
			}
#pragma unroll
			for (int q = 0; q < IDFT_BLK; q++)
				sig[i + q] = r_ound(Lq[q]);
			i += IDFT_BLK - 1;
			continue;
		}
		int base = 0;	/* (j * i) mod len */
		for (int j = 1; j < len2; j++) {
			base += i;
			if (base >= len)
				base -= len;
			int k = base + phm[j];
			if (k >= len)
				k -= len;
			L = L_mac(L, mag[j], c[k]);
		}
#endif
		sig[i] = r_ound(L);
	}
}

/* set_fc :145 -- mixed-excitation cutoff from the voicing pattern */
MD Word16 set_fc(int16_t *bpvc)
{
	/* syn_bp_map of the reference (harm.c:150-153), in Hz */
	const int16_t map[16] = {500, 500, 500, 500, 500, 500, 500, 4000,
				 1000, 1000, 1000, 4000, 2000, 3000, 3000, 4000};
	if (bpvc[0] < 8192)
		return 0;
	int k = 0;
	bpvc[0] = 16384;
	for (int i = 1; i < NUM_BANDS; i++) {
		k <<= 1;
		if (bpvc[i] > 8192) {
			bpvc[i] = 16384;
			k |= 1;
		} else {
			bpvc[i] = 0;
		}
	}
	return (Word16) (map[k] << 3);
}

/* harm_syn_pitch :192 */
MN void harm_syn_pitch(DecState *D, const int16_t *amp, int16_t *sig, Word16 fc, Word16 len)
{
	PROF_SCOPE(19);
	int16_t rnd[129], mag[129], phase[129];
	Word16 fc1, fc2, factor;
#if defined(MELPE_OPCOUNT)
	v_zero(phase, 129);
#endif
	/* (no zeroing of phase[] outside the census build: the loops below
	 * write phase[0 .. max(mc, len/2)], every entry realIDFT reads) */
	{
		uint32_t seed = D->seed;
		for (int i = 0; i < len / 2 + 1; i++)
			rnd[i] = mult(len, rand_minstdgen(&seed));
		D->seed = seed;
	}
	if (fc <= 4000) {
		fc1 = mult(13926, fc);
		fc2 = mult(17203, fc);
		factor = SW_MAX_;
	} else if (fc <= 8000) {
		fc1 = mult(15565, fc);
		fc2 = mult(17203, fc);
		factor = 29491;
	} else if (fc <= 16000) {
		fc1 = mult(16056, fc);
		fc2 = mult(16712, fc);
		factor = 26214;
	} else if (fc <= 24000) {
		fc1 = mult(15565, fc);
		fc2 = mult(17203, fc);
		factor = 24576;
	} else {
		fc1 = mult(15073, fc);
		fc2 = shift_r(fc, -1);
		factor = 22938;
	}
	Word16 t1 = divide_s(fc1, shl(8000, 2));
	Word16 t2 = divide_s(fc2, shl(8000, 2));
	Word16 vc = mult(t1, len);
	Word16 mc = mult(t2, len);
	Word16 tot = (Word16) ((len / 2) + 1);
	v_copy(mag, amp, add(vc, 1));
	t1 = 0;
	t2 = shr(extract_l(L_mult(1, len)), 1);
	while (t2 >= 2 * len)
		t2 = sub(t2, (Word16) (2 * len));
	for (int i = 0; i < mc + 1; i++) {
		phase[i] = shr(t1, 1);
		t1 = add(t1, t2);
		if (t1 >= 2 * len)
			t1 = sub(t1, (Word16) (2 * len));
	}
	int idx = 0;
	for (Word16 i = add(vc, 1); i < add(mc, 1); i++, idx++) {
		Word16 fn = divide_s(sub(i, vc), sub(mc, vc));
		t1 = add(mult(factor, fn), sub(SW_MAX_, fn));
		mag[i] = mult(amp[i], t1);
		t2 = sub(phase[i], mult(fn, rnd[idx]));
		if (t2 < 0)
			t2 = add(t2, len);
		phase[i] = t2;
	}
	for (Word16 i = add(mc, 1); i < tot; i++, idx++) {
		mag[i] = mult(amp[i], factor);
		t2 = negate(rnd[idx]);
		if (t2 < 0)
			t2 = add(t2, len);
		phase[i] = t2;
	}
	realIDFT(mag, phase, sig, len);
}

/* ------------------------------------------------------------------ */
/* postfilter, melpe/postfilt.c                                        */
/* ------------------------------------------------------------------ */

/* block energy in (mantissa, shift) form (postfilt.c:95-110 / 220-235) */
MD Word16 pf_energy(const int16_t *sp, Word16 *sh_out)
{
	PROF_SCOPE(52);
	Word16 mx = 0;
	Word32 sum = 0;
	Word16 ts;
#if defined(MELPE_OPCOUNT)
	for (int i = 0; i < FRAME; i++) {
		Word16 t = abs_s(sp[i]);
		if (mx < t)
			mx = t;
	}
	ts = norm_s(mx);
	for (int i = 0; i < FRAME; i++) {
		Word16 t = shl(sp[i], ts);
		sum = L_add(sum, L_shr(L_mult(t, t), 8));
	}
#else
	/* Both passes on packed pairs, branch-free.  ts = norm_s(max |x|), so
	 * shl(x, ts) never saturates and is x << ts; each term is at most
	 * (2^31 - 1) >> 8, and FRAME of them stay below 2^31, so L_add never
	 * clamps and the sum may be formed in any order. */
	static_assert(FRAME % 2 == 0, "pairs");
	{
		P16 r;
		const int np = p16_open(r, sp, FRAME);
		int i = 0;
#pragma unroll 8
		for (int k = 0; k < np; k++, i += 2) {
			const uint32_t x = p16_next(r);
			const Word16 a = abs_s(lo16(x)), b = abs_s(hi16(x));
			mx = a > mx ? a : mx;
			mx = b > mx ? b : mx;
		}
		for (; i < FRAME; i++) {
			const Word16 a = abs_s(sp[i]);
			mx = a > mx ? a : mx;
		}
	}
	ts = norm_s(mx);
	{
		P16 r;
		const int np = p16_open(r, sp, FRAME);
		int i = 0;
		int32_t acc = 0;
#pragma unroll 8
		for (int k = 0; k < np; k++, i += 2) {
			const uint32_t x = p16_next(r);
			const Word16 a = (Word16) (lo16(x) * (1 << ts)), b = (Word16) (hi16(x) * (1 << ts));
			acc += (int32_t) ((uint32_t) L_mult(a, a) >> 8);
			acc += (int32_t) ((uint32_t) L_mult(b, b) >> 8);
		}
		for (; i < FRAME; i++) {
			const Word16 a = (Word16) (sp[i] * (1 << ts));
			acc += (int32_t) ((uint32_t) L_mult(a, a) >> 8);
		}
		sum = acc;
	}
#endif
	Word16 sh = sub(8, shl(ts, 1));
	ts = norm_l(sum);
	*sh_out = sub(sh, ts);
	return extract_h(L_shl(sum, ts));
}

/* The postfilter's pole-zero taps L_add(L, L_mult(m, a)) / L_sub(L,
 * L_mult(m, a)).  With no coefficient at MIN16 (mult() never returns it, so
 * only an imported record could hold one; checked per call over the wave)
 * L_mult(m, a) is m * 2a exactly and is never MIN32, so each tap is one
 * 24-bit multiply and one clamped add or subtract.  pz_run instantiates the
 * filter loop for both forms and runs the one the check allows. */
template <bool DBL>
struct PzTaps {
	int32_t f2[LPC_ORD], i2[LPC_ORD];
	const int16_t *f, *i;
	MM PzTaps(const int16_t *af, const int16_t *ai) : f(af), i(ai)
	{
#pragma unroll
		for (int k = 0; k < LPC_ORD; k++) {
			f2[k] = 2 * (int32_t) af[k];
			i2[k] = 2 * (int32_t) ai[k];
		}
	}
	MM Word32 fir(Word32 L, Word16 m, int k) const
	{
		return DBL ? sat_add32(L, (int32_t) m * f2[k]) : L_add(L, L_mult(m, f[k]));
	}
	MM Word32 iir(Word32 L, Word16 m, int k) const
	{
		return DBL ? sat_sub32(L, (int32_t) m * i2[k]) : L_sub(L, L_mult(m, i[k]));
	}
};

template <class F>
MD void pz_run(const int16_t *af, const int16_t *ai, F loop)
{
	bool ok = true;
#pragma unroll
	for (int k = 0; k < LPC_ORD; k++)
		ok &= af[k] != SW_MIN_ && ai[k] != SW_MIN_;
#if defined(MELPE_OPCOUNT)
	ok = false;
#endif
	if (wave_all(ok))
		loop(PzTaps<true>(af, ai));
	else
		loop(PzTaps<false>(af, ai));
}

/* postfilt :60 */
MN void postfilt(DecState *D, int16_t *sp, const int16_t *prev_lsf, const int16_t *cur_lsf)
{
	PROF_SCOPE(20);
	const int16_t syn_inp[4] = {4096, 12288, 20480, 28672};
	int16_t synLPC[LPC_ORD], inplsf[LPC_ORD], synhp[45], m1o[LPC_ORD], m2o[LPC_ORD];
	int16_t nokori[20];
	Word16 sp_sh, op_sh, t, t1, t2;
	Word32 L;
	Word16 spE = pf_energy(sp, &sp_sh);
	for (int i = 0; i < 4; i++) {
		for (int j = 0; j < LPC_ORD; j++)
			inplsf[j] = add(mult(prev_lsf[j], sub(SW_MAX_, syn_inp[i])),
					mult(cur_lsf[j], syn_inp[i]));
		lpc_lsp2pred(inplsf, synLPC, LPC_ORD);
		t = mult(4915, synLPC[1]);
		if (t > 2048)
			t = 2048;
		if (t < 0)
			t = 0;
		Word16 emph = shl(t, 3);
		{
			Word16 hpm = D->pf_hpm;
			v_batch(&sp[i * 45], synhp, 45, [&](int, int16_t x) {
				const Word16 u = mult(emph, hpm);
				hpm = x;
				return (int16_t) sub(x, u);
			});
			D->pf_hpm = hpm;
		}
		if (i == 0) {
			/* run the previous frame's filter over the first 20 samples for
			 * the cross-fade tail */
			Word16 af[LPC_ORD], ai[LPC_ORD];
#pragma unroll
			for (int k = 0; k < LPC_ORD; k++) {
				m1o[k] = D->pf_mem1[k];
				m2o[k] = D->pf_mem2[k];
				af[k] = D->pf_aFIR[k];
				ai[k] = D->pf_aIIR[k];
			}
			pz_run(af, ai, [&](const auto &pc) {
			Word16 xn = synhp[0];	/* the next sample, loaded one ahead */
			for (int j = 0; j < 20; j++) {
				const Word16 x = xn;
				xn = synhp[j + 1 < 45 ? j + 1 : 44];
				L = 0;
#pragma unroll
				for (int k = 0; k < LPC_ORD; k++)
					L = pc.fir(L, m1o[k], k);
#pragma unroll
				for (int k = LPC_ORD - 1; k > 0; k--)
					m1o[k] = m1o[k - 1];
				m1o[0] = x;
				L = L_add(L, L_shl(L_deposit_l(x), 13));
#pragma unroll
				for (int k = 0; k < LPC_ORD; k++)
					L = pc.iir(L, m2o[k], k);
#pragma unroll
				for (int k = LPC_ORD - 1; k > 0; k--)
					m2o[k] = m2o[k - 1];
				t1 = extract_l(L_shr(L, 13));
				m2o[0] = t1;
				Word16 wt = sub(SW_MAX_, (Word16) (j * 1638));	/* window[j] */
				t1 = mult(wt, t1);
				nokori[j] = extract_l(L_shr(L_mult(D->pf_gain, t1), 15));
			}
			});
		}
		t1 = 18678;	/* ALPH */
		t2 = 24576;	/* BETA */
		for (int j = 0; j < LPC_ORD; j++) {
			D->pf_aFIR[j] = mult(synLPC[j], t1);
			D->pf_aIIR[j] = mult(synLPC[j], t2);
			t1 = mult(18678, t1);
			t2 = mult(24576, t2);
		}
		{	/* pole-zero filter; memories and coefficients held in
			 * registers for the subframe (shifts become renames) */
			Word16 m1[LPC_ORD], m2[LPC_ORD], af[LPC_ORD], ai[LPC_ORD];
#pragma unroll
			for (int k = 0; k < LPC_ORD; k++) {
				m1[k] = D->pf_mem1[k];
				m2[k] = D->pf_mem2[k];
				af[k] = D->pf_aFIR[k];
				ai[k] = D->pf_aIIR[k];
			}
			pz_run(af, ai, [&](const auto &pc) {
			Word16 xn = synhp[0];	/* the next sample, loaded one ahead */
			for (int j = 0; j < 45; j++) {
				const Word16 x = xn;
				xn = synhp[j + 1 < 45 ? j + 1 : 44];
				L = 0;
#pragma unroll
				for (int k = 0; k < LPC_ORD; k++)
					L = pc.fir(L, m1[k], k);
#pragma unroll
				for (int k = LPC_ORD - 1; k > 0; k--)
					m1[k] = m1[k - 1];
				m1[0] = x;
				L = L_add(L, L_shl(L_deposit_l(x), 13));
#pragma unroll
				for (int k = 0; k < LPC_ORD; k++)
					L = pc.iir(L, m2[k], k);
#pragma unroll
				for (int k = LPC_ORD - 1; k > 0; k--)
					m2[k] = m2[k - 1];
				L = L_shr(L, 13);
				m2[0] = extract_l(L);
				sp[i * 45 + j] = extract_l(L);
			}
			});
#pragma unroll
			for (int k = 0; k < LPC_ORD; k++) {
				D->pf_mem1[k] = m1[k];
				D->pf_mem2[k] = m2[k];
			}
		}
	}
	Word16 opE = pf_energy(sp, &op_sh);
	if (op_sh >= -22) {
		spE = shr(spE, 1);
		sp_sh = add(sp_sh, 1);
		Word16 ts = sub(sp_sh, op_sh);
		if (ts & 1) {
			spE = shr(spE, 1);
			ts = add(ts, 1);
		}
		t = divide_s(spE, opE);
		ts = shr(ts, 1);
		t = sqrt_Q15(t);
		ts = sub(ts, 1);
		D->pf_gain = shl(t, ts);
	} else {
		D->pf_gain = 0;
	}
	/* the gain, the first 20 samples' cross-fade with the previous
	 * filter's tail and v_scale(sp, 29088) in one pass, each sample's ops in
	 * the reference's order */
	{
		const Word16 g = D->pf_gain;
		v_batch(sp, sp, FRAME, [&](int i, int16_t x) {
			Word16 y = extract_l(L_shr(L_mult(g, x), 15));
			if (i < 20)
				y = add(mult(y, (Word16) (i * 1638)), nokori[i]);
			return (int16_t) mult(y, 29088);
		});
	}
	iir2_d(sp, TB(lpf3500_den), TB(lpf3500_num), D->lpf_din, D->lpf_dhi, D->lpf_dlo,
	       TB(hpf60_den), TB(hpf60_num), D->hpf_din, D->hpf_dhi, D->hpf_dlo, FRAME);
}

/* ------------------------------------------------------------------ */
/* melp_syn :160 -- pitch-synchronous synthesis of one frame          */
/* ------------------------------------------------------------------ */
/* R24: the reference's rate == RATE2400 frame (melp_syn.c:213: the
 * unvoiced-frame parameter override is 1200 bps only) */
/* One pitch period's synthesis filters (melp_syn.c:395-428) in one pass
 * over its samples, in place on s[0 .. len): v_scale(pulse_gain), lpc_syn
 * (ase_den, memory ase_del), zerflt(ase_num; its history the same ase_del),
 * zerflt_Q(tilt, memory tilt_del), lpc_syn(lpc, memory lpc_del).  Filter k
 * at sample i needs only filter k-1's samples <= i and its own past, so
 * interleaving them sample by sample equals the reference's five in-place
 * passes; each sample's L_mac / L_msu chain is the reference's, in its tap
 * order.  The delay lines ride in registers (no history copies through
 * scratch), the inputs come a block ahead.  Returns the first energy of
 * scale_adj (L_v_magsq of the outputs >> 4), summed as they leave.
 * DBL: no coefficient is MIN16, so L_mac / L_msu are a 24-bit multiply by
 * the doubled coefficient and one clamped add (2c fits; 2xc cannot clamp). */
template <bool DBL>
MD Word32 syn_chain_t(DecState *D, int16_t *s, int len, Word16 pulse_gain, const int16_t *aden,
		      const int16_t *anum, const int16_t *tilt, const int16_t *lpc)
{
	int32_t cd[LPC_ORD], cn[LPC_ORD + 1], cl[LPC_ORD], ct0, ct1;
	int16_t w[LPC_ORD], v[LPC_ORD];	/* y2[i-1-k] (lpc_syn 1 / zerflt), y5[i-1-k] */
#pragma unroll
	for (int k = 0; k < LPC_ORD; k++) {
		cd[k] = DBL ? 2 * (int32_t) aden[k] : aden[k];
		cl[k] = DBL ? 2 * (int32_t) lpc[k] : lpc[k];
		w[k] = D->ase_del[LPC_ORD - 1 - k];
		v[k] = D->lpc_del[LPC_ORD - 1 - k];
	}
#pragma unroll
	for (int k = 0; k <= LPC_ORD; k++)
		cn[k] = DBL ? 2 * (int32_t) anum[k] : anum[k];
	ct0 = DBL ? 2 * (int32_t) tilt[0] : tilt[0];
	ct1 = DBL ? 2 * (int32_t) tilt[1] : tilt[1];
	int16_t y3p = D->tilt_del[0];
	Word32 e = 0;
	auto msu = [&](Word32 acc, int16_t x, int32_t c) {
		return DBL ? sat_sub32(acc, (int32_t) x * c) : L_msu(acc, x, (Word16) c);
	};
	auto mac = [&](Word32 acc, int16_t x, int32_t c) {
		return DBL ? sat_add32(acc, (int32_t) x * c) : L_mac(acc, x, (Word16) c);
	};
	v_batch(s, s, len, [&](int, int16_t x0) {
		const int16_t x1 = mult(x0, pulse_gain);
		/* lpc_syn(aden): y2 */
		Word32 acc = L_shr(L_deposit_h(x1), 3);
#pragma unroll
		for (int i = LPC_ORD; i > 0; i--)
			acc = msu(acc, w[i - 1], cd[i - 1]);
		const int16_t y2 = r_ound(L_shl(acc, 3));
		/* zerflt(anum, Q12): y3 over y2[i .. i-10] */
		acc = mac(0, y2, cn[0]);
#pragma unroll
		for (int j = 1; j <= LPC_ORD; j++)
			acc = mac(acc, w[j - 1], cn[j]);
		const int16_t y3 = r_ound(L_shl(acc, 3));
#pragma unroll
		for (int k = LPC_ORD - 1; k > 0; k--)
			w[k] = w[k - 1];
		w[0] = y2;
		/* zerflt_Q(tilt, order 1, Q15): y4 */
		acc = mac(mac(0, y3, ct0), y3p, ct1);
		const int16_t y4 = r_ound(acc);
		y3p = y3;
		/* lpc_syn(lpc): y5 */
		acc = L_shr(L_deposit_h(y4), 3);
#pragma unroll
		for (int i = LPC_ORD; i > 0; i--)
			acc = msu(acc, v[i - 1], cl[i - 1]);
		const int16_t y5 = r_ound(L_shl(acc, 3));
#pragma unroll
		for (int k = LPC_ORD - 1; k > 0; k--)
			v[k] = v[k - 1];
		v[0] = y5;
		const Word16 t = shr(y5, 4);	/* scale_adj's first energy */
		e = L_mac(e, t, t);
		return y5;
	});
#pragma unroll
	for (int k = 0; k < LPC_ORD; k++) {
		D->ase_del[k] = w[LPC_ORD - 1 - k];
		D->lpc_del[k] = v[LPC_ORD - 1 - k];
	}
	D->tilt_del[0] = y3p;
	return e;
}

MD Word32 syn_chain(DecState *D, int16_t *s, int len, Word16 pulse_gain, const int16_t *aden,
		    const int16_t *anum, const int16_t *tilt, const int16_t *lpc)
{
	bool dbl = tilt[0] != SW_MIN_ && tilt[1] != SW_MIN_;
	for (int k = 0; k < LPC_ORD; k++)
		dbl &= aden[k] != SW_MIN_ && lpc[k] != SW_MIN_;
	for (int k = 0; k <= LPC_ORD; k++)
		dbl &= anum[k] != SW_MIN_;
	if (wave_all(dbl))
		return syn_chain_t<true>(D, s, len, pulse_gain, aden, anum, tilt, lpc);
	return syn_chain_t<false>(D, s, len, pulse_gain, aden, anum, tilt, lpc);
}

/* melp_syn's per-frame values (melp_syn.c:160-295): the first-call setup,
 * the noise estimate, the frame's LPC gain and tilt and the mixing filters'
 * voicing split.  Shared by the serial form and the two-wave decoder's
 * excitation side. */
struct SynFrame {
	Word16 lpc_gain, cur_tilt;
	int16_t cur_p[MIX_ORD + 1], cur_n[MIX_ORD + 1];
};

template <bool R24>
MD void syn_frame_begin(DecState *D, MelpParam *par, SynFrame &F)
{
	int16_t refc[LPC_ORD], lpc[LPC_ORD + 1];
	MelpParam *prev = &D->prev_par;
	Word16 t1, t2;
	if (!D->syn_started) {
		D->noise_gain = par->gain[NUM_GAINFR - 1];
		D->prev_tilt = 0;
		v_zero(D->prev_pcof, MIX_ORD + 1);
		v_zero(D->prev_ncof, MIX_ORD + 1);
		D->prev_ncof[MIX_ORD / 2] = SW_MAX_;
		v_zero(D->disp_del, DISP_ORD);
		v_zero(D->ase_del, LPC_ORD);
		v_zero(D->tilt_del, 1);
		D->syn_started = 1;
	} else if (!D->erase) {
		for (int i = 0; i < NUM_GAINFR; i++) {
			noise_est(par->gain[i], &D->noise_gain, 17691, -17749, 2560, 20480);
			noise_sup(&par->gain[i], D->noise_gain, 5120, 1536, 768);
		}
	}
	if (par->uv_flag && !R24) {
		v_set(par->fs_mag, 8192, NUM_HARM);
		par->pitch = UV_PITCH_Q7;
		par->jitter = 8192;	/* X025_Q15 */
	}
	if (!par->uv_flag && !D->erase)
		window_Q(par->fs_mag, g_der.w_fs_inv, par->fs_mag, NUM_HARM, 14);
	lpc_clmp(par->lsf, 409, LPC_ORD);
	lpc_lsp2pred(par->lsf, &lpc[1], LPC_ORD);
	Word16 lpc_gain = lpc_pred2refl(&lpc[1], refc, LPC_ORD);
	F.lpc_gain = sqrt_fxp(lpc_gain, 15);
	F.cur_tilt = (refc[0] < 0) ? shr(refc[0], 1) : (Word16) 0;
	t1 = shr(prev->pitch, 1);
	t2 = add(1536, prev->gain[NUM_GAINFR - 1]);
	if (par->pitch < t1 && par->gain[0] > t2)
		prev->pitch = par->pitch;
	v_zero(F.cur_p, MIX_ORD + 1);
	v_zero(F.cur_n, MIX_ORD + 1);
	const int16_t *bpc = TB(bp_cof);
	for (int i = 0; i < NUM_BANDS; i++) {
		if (par->bpvc[i] > 8192)
			v_add(F.cur_p, bpc + i * (MIX_ORD + 1), MIX_ORD + 1);
		else
			v_add(F.cur_n, bpc + i * (MIX_ORD + 1), MIX_ORD + 1);
	}
}

/* one pitch period's parameters (melp_syn.c:300-394): length, gains, the
 * synthesis filters' coefficients and the harmonic amplitudes */
struct SynPer {
	Word16 len, gain, fc, pulse_gain;
	int16_t lpc[LPC_ORD + 1], ase_num[LPC_ORD + 1], ase_den[LPC_ORD], tilt_cof[2];
	int16_t fs_real[PITCHMAX];
};

MD void syn_period(DecState *D, MelpParam *par, const SynFrame &F, Word16 sb0, SynPer &P)
{
	PROF_SCOPE(50);
	MelpParam *prev = &D->prev_par;
	int16_t lsf[LPC_ORD], pul[MIX_ORD + 1], noi[MIX_ORD + 1];
	Word16 t1, t2;
	Word16 ifact = divide_s(sb0, FRAME);
	Word16 gcnt, ifg, intfact;
	if (sb0 >= 90) {
		gcnt = 2;
		ifg = divide_s(sub(sb0, 90), 90);
	} else {
		gcnt = 1;
		ifg = divide_s(sb0, 90);
	}
	Word32 La = L_mult(par->gain[gcnt - 1], ifg);
	Word32 Lb = L_mult(gcnt > 1 ? par->gain[gcnt - 2] : prev->gain[NUM_GAINFR - 1],
			   sub(SW_MAX_, ifg));
	Word16 gain = extract_h(L_add(La, Lb));
	t1 = sub(par->gain[NUM_GAINFR - 1], prev->gain[NUM_GAINFR - 1]);
	if (abs_s(t1) > 1536) {
		t2 = sub(gain, prev->gain[NUM_GAINFR - 1]);
		if ((t2 > 0 && t1 < 0) || (t2 < 0 && t1 > 0)) {
			intfact = 0;
		} else {
			t1 = abs_s(t1);
			t2 = abs_s(t2);
			intfact = (t2 >= t1) ? (Word16) SW_MAX_ : divide_s(t2, t1);
		}
	} else {
		intfact = ifact;
	}
	interp_array(prev->lsf, par->lsf, lsf, intfact, LPC_ORD);
	lpc_lsp2pred(lsf, &P.lpc[1], LPC_ORD);
	Word16 sig_prob = lin_int_bnd(gain, add(D->noise_gain, 3072), add(D->noise_gain, 7680),
				      0, SW_MAX_);
	P.ase_num[0] = 4096;
	lpc_bwex(&P.lpc[1], &P.ase_num[1], mult(sig_prob, 16384), LPC_ORD);
	lpc_bwex(&P.lpc[1], P.ase_den, mult(sig_prob, 26214), LPC_ORD);
	Word16 if1 = sub(SW_MAX_, intfact);
	t1 = add(mult(F.cur_tilt, intfact), mult(D->prev_tilt, if1));
	P.tilt_cof[0] = SW_MAX_;
	P.tilt_cof[1] = mult(sig_prob, t1);
	t1 = add(mult(F.lpc_gain, intfact), mult(D->prev_lpc_gain, if1));
	Word16 syn_gain = mult(32000, t1);
	Word16 pitch = add(mult(par->pitch, intfact), mult(prev->pitch, if1));
	P.pulse_gain = extract_h(L_shl(L_mult(syn_gain, sqrt_fxp(pitch, 7)), 4));
	t1 = sqrt_fxp(ifact, 15);
	interp_array(D->prev_pcof, F.cur_p, pul, t1, MIX_ORD + 1);
	interp_array(D->prev_ncof, F.cur_n, noi, t1, MIX_ORD + 1);
	Word16 fc_prev = set_fc(prev->bpvc);
	Word16 fc_cur = set_fc(par->bpvc);
	t2 = sub(SW_MAX_, t1);
	P.fc = add(mult(t1, fc_cur), mult(t2, fc_prev));
	Word16 jitter = add(mult(par->jitter, ifact), mult(prev->jitter, sub(SW_MAX_, ifact)));
	P.gain = mult(26214, gain);	/* X005_Q19 */
	int16_t r;
	rand_num(&r, SW_MAX_, 1, &D->seed);
	t1 = shr(mult(jitter, r), 1);
	t1 = mult(pitch, sub(16384, t1));
	Word16 len = shift_r(t1, -6);
	if (len < PITCHMIN)
		len = PITCHMIN;
	if (len > PITCHMAX)
		len = PITCHMAX;
	P.len = len;
	v_set(P.fs_real, 8192, len);
	P.fs_real[0] = 0;
	interp_array(prev->fs_mag, par->fs_mag, &P.fs_real[1], intfact, NUM_HARM);
}

/* the dispersion FIR over the frame's run of periods, the frame's output
 * and the next frame's start (melp_syn.c:436-447): pre[0 .. DISP_ORD) is
 * the dispersion history, pre[DISP_ORD ..] the run from sb_start to
 * D->syn_begin */
MD void syn_disperse(DecState *D, int16_t *pre, Word16 sb_start, int16_t *out)
{
	/* The dispersion FIR (melp_syn.c:436-440) runs per period on the period
	 * with the previous period's last DISP_ORD pre-dispersion samples as its
	 * history (disp_del, also when a period is shorter than that): the same
	 * FIR over the frame's periods end to end.  It runs here once over the
	 * whole run, every lane of the wave together, instead of once per
	 * period count the wave's channels take; each output sample's L_mac
	 * chain is the reference's.  The run's part past FRAME is the next
	 * frame's start (sigsave). */
	PROF_SCOPE(51);
	const int total = D->syn_begin - sb_start;
	v_copy(D->disp_del, &pre[total], DISP_ORD);
	static_assert(DISP_ORD == 64, "zerflt_Q's unrolled dispersion path (dsp.h)");
	zerflt_Q(&pre[DISP_ORD], TB(disp_cof), &pre[DISP_ORD], DISP_ORD, total, 15);
	v_copy(&out[sb_start], &pre[DISP_ORD], FRAME - sb_start);
	v_copy(D->sigsave, &pre[DISP_ORD + FRAME - sb_start], total - (FRAME - sb_start));
}

/* the frame's parameters become the previous frame's (melp_syn.c:455-468) */
MD void syn_frame_end(DecState *D, const MelpParam *par, const SynFrame &F)
{
	v_copy(D->prev_pcof, F.cur_p, MIX_ORD + 1);
	v_copy(D->prev_ncof, F.cur_n, MIX_ORD + 1);
	D->prev_par = *par;
	D->prev_tilt = F.cur_tilt;
	D->prev_lpc_gain = F.lpc_gain;
	D->syn_begin = sub(D->syn_begin, FRAME);
}

template <bool R24>
MN void melp_syn(DecState *D, MelpParam *par, int16_t *out)
{
	PROF_SCOPE(18);
	const int BEGIN = DISP_ORD;	/* max(MIX_ORD, DISP_ORD) */
	int16_t sb[BEGIN + PITCHMAX];
	SynFrame F;
	syn_frame_begin<R24>(D, par, F);
	/* pre[0 .. DISP_ORD): the dispersion history; then the frame's periods
	 * from syn_begin on, before dispersion (at most FRAME + PITCHMAX) */
	int16_t pre[DISP_ORD + FRAME + PITCHMAX];
	const Word16 sb_start = D->syn_begin;
	v_copy(pre, D->disp_del, DISP_ORD);
	while (D->syn_begin < FRAME) {
		const Word16 sb0 = D->syn_begin;
		SynPer P;
		syn_period(D, par, F, sb0, P);
		const Word16 len = P.len;
		harm_syn_pitch(D, P.fs_real, &sb[BEGIN], P.fc, len);
#if !defined(MELPE_OPCOUNT)
		{
			/* the filter chain in one pass, then scale_adj writing the
			 * period straight into the frame's run */
			Word32 e0 = syn_chain(D, &sb[BEGIN], len, P.pulse_gain, P.ase_den, P.ase_num, P.tilt_cof,
					      &P.lpc[1]);
			scale_adj(D, &sb[BEGIN], P.gain, len, 10, 26214, e0, &pre[DISP_ORD + sb0 - sb_start]);
			D->syn_begin = add(sb0, len);
			continue;
		}
#endif
		v_scale(&sb[BEGIN], P.pulse_gain, len);
		v_copy(&sb[BEGIN - LPC_ORD], D->ase_del, LPC_ORD);
		lpc_syn(&sb[BEGIN], &sb[BEGIN], P.ase_den, LPC_ORD, len);
		v_copy(D->ase_del, &sb[BEGIN + len - LPC_ORD], LPC_ORD);
		zerflt(&sb[BEGIN], P.ase_num, &sb[BEGIN], LPC_ORD, len);
		v_copy(&sb[BEGIN - 1], D->tilt_del, 1);
		v_copy(D->tilt_del, &sb[len + BEGIN - 1], 1);
		zerflt_Q(&sb[BEGIN], P.tilt_cof, &sb[BEGIN], 1, len, 15);
		v_copy(&sb[BEGIN - LPC_ORD], D->lpc_del, LPC_ORD);
		lpc_syn(&sb[BEGIN], &sb[BEGIN], &P.lpc[1], LPC_ORD, len);
		v_copy(D->lpc_del, &sb[len + BEGIN - LPC_ORD], LPC_ORD);
		scale_adj(D, &sb[BEGIN], P.gain, len, 10, 26214);
		/* the period's pre-dispersion samples join the frame's run */
		v_copy(&pre[DISP_ORD + sb0 - sb_start], &sb[BEGIN], len);
		D->syn_begin = add(sb0, len);
	}
	syn_disperse(D, pre, sb_start, out);
	/* the reference postfilters the frame inside the loop, in its last
	 * period (melp_syn.c:448); nothing after it in the loop reads out[] or
	 * the postfilter state, so the call follows the loop -- where every
	 * lane of the wave makes it together */
	postfilt(D, out, D->prev_par.lsf, par->lsf);
	syn_frame_end(D, par, F);
}

#if !defined(MELPE_OPCOUNT)
/* ------------------------------------------------------------------ */
/* the two-wave decoder (k_dec2.hip): melp_syn split into the excitation */
/* side (wave A) and the filter side (wave B) of the same 64 channels     */
/* ------------------------------------------------------------------ */

/* Per frame, A hands B (through a per-channel buffer of HB_WORDS dwords,
 * int16 pairs low half first): the period count and the run's length, the
 * two LSF vectors the postfilter interpolates, each period's length, gains
 * and filter coefficients, and the run of excitation samples.  A period is
 * at least PITCHMIN long and the frame's loop starts below FRAME, so a frame
 * has at most HB_MAXPER periods and a run of at most FRAME + PITCHMAX - 1
 * samples. */
#define HB_MAXPER ((FRAME + PITCHMIN - 1) / PITCHMIN)
enum {
	HB_NP = 0,	/* periods | run length << 16 */
	HB_LSF = 1,	/* prev_par.lsf, then par->lsf (clamped): 2 x LPC_ORD / 2 */
	HB_PER = HB_LSF + LPC_ORD,	/* HB_PW per period */
	HB_PW = 2 + 3 * LPC_ORD / 2,	/* len | pulse_gain, gain | tilt, ase_den, ase_num[1..], lpc[1..] */
	HB_EXC = HB_PER + HB_MAXPER * HB_PW,
	HB_WORDS = HB_EXC + (FRAME + PITCHMAX) / 2,
};
static_assert(LPC_ORD % 2 == 0, "coefficient vectors packed in pairs");

MD uint32_t hb_pack(int16_t lo, int16_t hi)
{
	return (uint32_t) (uint16_t) lo | ((uint32_t) (uint16_t) hi << 16);
}

template <class Hb>
MD void hb_put_vec(Hb &hb, int k, const int16_t *v, int n)
{
	for (int i = 0; i < n; i += 2)
		hb.put(k + i / 2, hb_pack(v[i], v[i + 1]));
}

template <class Hb>
MD void hb_get_vec(const Hb &hb, int k, int16_t *v, int n)
{
	for (int i = 0; i < n; i += 2) {
		const uint32_t x = hb.get(k + i / 2);
		v[i] = lo16(x);
		v[i + 1] = hi16(x);
	}
}

/* wave A's melp_syn: every period's parameters and excitation
 * (harm_syn_pitch), handed over instead of filtered; the state it moves on
 * is DecState's excitation side */
template <class Hb>
MN void melp_syn_a(DecState *D, MelpParam *par, Hb hb)
{
	PROF_SCOPE(18);
	SynFrame F;
	syn_frame_begin<false>(D, par, F);
	alignas(4) int16_t run[FRAME + PITCHMAX + 1];
	const Word16 sb_start = D->syn_begin;
	int np = 0;
	while (D->syn_begin < FRAME) {
		const Word16 sb0 = D->syn_begin;
		SynPer P;
		syn_period(D, par, F, sb0, P);
		harm_syn_pitch(D, P.fs_real, &run[sb0 - sb_start], P.fc, P.len);
		const int k = HB_PER + np * HB_PW;
		hb.put(k, hb_pack(P.len, P.pulse_gain));
		hb.put(k + 1, hb_pack(P.gain, P.tilt_cof[1]));
		hb_put_vec(hb, k + 2, P.ase_den, LPC_ORD);
		hb_put_vec(hb, k + 2 + LPC_ORD / 2, &P.ase_num[1], LPC_ORD);
		hb_put_vec(hb, k + 2 + LPC_ORD, &P.lpc[1], LPC_ORD);
		np++;
		D->syn_begin = add(sb0, P.len);
	}
	const int total = D->syn_begin - sb_start;
	run[total] = 0;
	hb.put(HB_NP, (uint32_t) np | ((uint32_t) total << 16));
	hb_put_vec(hb, HB_LSF, D->prev_par.lsf, LPC_ORD);
	hb_put_vec(hb, HB_LSF + LPC_ORD / 2, par->lsf, LPC_ORD);
	for (int i = 0; i < total; i += 2)
		hb.put(HB_EXC + i / 2, hb_pack(run[i], run[i + 1]));
	syn_frame_end(D, par, F);
}

/* wave B's melp_syn on A's hand-over: the synthesis filters and scale_adj
 * per period, the dispersion, the postfilter; the state it moves on is
 * DecState's filter side (its syn_begin and syn_started are a private
 * replica of A's, advanced the same way) */
template <class Hb>
MN void melp_syn_b(DecState *D, const Hb hb, int16_t *out)
{
	PROF_SCOPE(18);
	if (!D->syn_started) {	/* the filter side of the first call's setup */
		v_zero(D->disp_del, DISP_ORD);
		v_zero(D->ase_del, LPC_ORD);
		v_zero(D->tilt_del, 1);
		D->syn_started = 1;
	}
	const uint32_t h = hb.get(HB_NP);
	const int np = (int) (h & 0xffff), total = (int) (h >> 16);
	int16_t prev_lsf[LPC_ORD], cur_lsf[LPC_ORD];
	hb_get_vec(hb, HB_LSF, prev_lsf, LPC_ORD);
	hb_get_vec(hb, HB_LSF + LPC_ORD / 2, cur_lsf, LPC_ORD);
	alignas(4) int16_t run[FRAME + PITCHMAX + 1];
	/* (reading the run in blocks of 8 dwords, loads issued together, measured
	 * slower: 3.13 vs 3.02 ms at 32,768 channels, profiles/r06c_*) */
	for (int i = 0; i < total; i += 2) {
		const uint32_t x = hb.get(HB_EXC + i / 2);
		run[i] = lo16(x);
		run[i + 1] = hi16(x);
	}
	int16_t pre[DISP_ORD + FRAME + PITCHMAX];
	const Word16 sb_start = D->syn_begin;
	v_copy(pre, D->disp_del, DISP_ORD);
	int r = 0;
	for (int p = 0; p < np; p++) {
		const int k = HB_PER + p * HB_PW;
		const uint32_t w0 = hb.get(k), w1 = hb.get(k + 1);
		const Word16 len = lo16(w0), pulse_gain = hi16(w0), gain = lo16(w1);
		int16_t ase_den[LPC_ORD], ase_num[LPC_ORD + 1], lpc[LPC_ORD], tilt[2];
		tilt[0] = SW_MAX_;
		tilt[1] = hi16(w1);
		ase_num[0] = 4096;
		hb_get_vec(hb, k + 2, ase_den, LPC_ORD);
		hb_get_vec(hb, k + 2 + LPC_ORD / 2, &ase_num[1], LPC_ORD);
		hb_get_vec(hb, k + 2 + LPC_ORD, lpc, LPC_ORD);
		Word32 e0 = syn_chain(D, &run[r], len, pulse_gain, ase_den, ase_num, tilt, lpc);
		scale_adj(D, &run[r], gain, len, 10, 26214, e0, &pre[DISP_ORD + r]);
		r += len;
	}
	D->syn_begin = add(sb_start, (Word16) total);
	syn_disperse(D, pre, sb_start, out);
	postfilt(D, out, prev_lsf, cur_lsf);
	D->syn_begin = sub(D->syn_begin, FRAME);
}

/* The two-wave decoder's phase program for one superframe: phase p (0 ..
 * NF) has wave A (role 0) read the channel (p = 0) and synthesise frame p's
 * excitation into buffer p & 1, while wave B (role 1) filters frame p - 1
 * from buffer (p - 1) & 1 into out (B also lays down the previous
 * superframe's carried samples at p = 0).  Phases are separated by a
 * barrier; the buffers are the only data the two waves share. */
template <class Hb>
MD void dec2_phase(DecState *D, int16_t *out, Hb hb0, Hb hb1, int role, int p)
{
	if (role == 0) {
		if (p == 0)
			D->erase = low_rate_chn_read(D);
		if (p < NF)
			melp_syn_a(D, &D->par[p], (p & 1) ? hb1 : hb0);
	} else if (p == 0) {
		/* syn_begin < PITCHMAX <= BLOCK always, so the reference's
		 * "impossible" syn_begin > frameSize branch (melp_syn.c:120-125)
		 * is not restated */
		if (D->syn_begin > 0)
			v_copy(out, D->sigsave, D->syn_begin);
	} else {
		const int i = p - 1;
		melp_syn_b(D, (i & 1) ? hb1 : hb0, &out[i * FRAME]);
		if (D->syn_begin > 0 && i < NF - 1)
			v_copy(&out[(i + 1) * FRAME], D->sigsave, D->syn_begin);
	}
}
#define DEC2_PHASES (NF + 1)
#endif

/* synthesis :110 -- melpe_s: D->chbuf (11 bytes) -> 540 samples */
/* a progress checkpoint of the lane decoder (progprio.h); a no-op elsewhere */
#ifndef DEC_CKPT
#define DEC_CKPT(j) ((void) 0)
#endif

MN void decode_superframe(DecState *D, int16_t *out)
{
	PROF_SCOPE(22);
	/* syn_begin < PITCHMAX <= BLOCK always, so the reference's "impossible"
	 * syn_begin > frameSize branch (melp_syn.c:120-125) is not restated */
	if (D->syn_begin > 0)
		v_copy(out, D->sigsave, D->syn_begin);
	D->erase = low_rate_chn_read(D);
	for (int i = 0; i < NF; i++) {
		melp_syn<false>(D, &D->par[i], &out[i * FRAME]);
		if (D->syn_begin > 0 && i < NF - 1)
			v_copy(&out[(i + 1) * FRAME], D->sigsave, D->syn_begin);
		DEC_CKPT(i + 1);
	}
}

}  // namespace mlp

#endif
