/*
 * npp.h -- noise pre-processor (minimum-statistics noise estimate +
 * log-MMSE spectral gain, 256-point window, 180-sample hop), restating
 * melpe/npp.c with every static of that file moved into NppState.
 *
 * Entry point: npp_frame() == npp() (melpe/npp.c:170).  State persists per
 * channel; npp_reset() gives the fresh-process state.
 */
#ifndef MELPE_NPP_H
#define MELPE_NPP_H

#include <stddef.h>

#include "dsp.h"

namespace mlp {

#define NPP_WIN 256
#define NPP_HOP 180
#define NPP_OVL 76
#define NPP_NB 129
#define NPP_NMINWIN 8
#define NPP_LMINWIN 9
#define GM_MIN 3932
#define ENH_QK_MAX 32735
#define ENH_QK_MIN 33
#define NOISE_BIAS 23170

struct NppState {
	int16_t started;	/* npp() first_time done (npp.c:174) */
	int16_t qk_started;	/* compute_qk first_time done (npp.c:293) */
	int16_t pf_started;	/* process_frame first_time done (npp.c:1215) */
	int16_t enh_i;
	int16_t SN_LT, SN_LT_shift, n_pwr, n_pwr_shift;
	int16_t var_rel_av, alphacorr;
	int16_t minspec_counter, circb_index;
	int16_t Ksi_min_var, YY_LT, YY_LT_shift, SN_LT0, SN_LT0_shift;
	int16_t lambdaD[NPP_NB], lambdaD_shift[NPP_NB];
	int16_t sm_shift[NPP_NB], noise_shift[NPP_NB];
	int16_t av_shift[NPP_NB], av2_shift[NPP_NB];
	int16_t act_min[NPP_NB], act_min_shift[NPP_NB];
	int16_t ksi[NPP_NB], ksi_shift[NPP_NB];
	int16_t smoothedspect[NPP_NB], var_sp_av[NPP_NB], var_sp_2[NPP_NB];
	int16_t noisespect[NPP_NB];
	int16_t qla[NPP_NB];
	int16_t agal[NPP_NB], agal_shift[NPP_NB];
	int16_t qk[NPP_NB], Gain[NPP_NB];
	int16_t speech_in[NPP_WIN];
	int16_t overlap[NPP_OVL];
	/* ---- min-statistics memory: touched only by min_search and
	 * minstat_init, once per frame.  Kept last so the wave kernel can hold
	 * the part above in LDS (NPP_HOT_BYTES) and leave this part in the HBM
	 * record; every access goes through the `m` view of those functions. */
	int16_t act_min_sub[NPP_NB], act_min_sub_shift[NPP_NB];
	int16_t localflag[NPP_NB];
	int16_t circb_min[NPP_NB], circb_min_shift[NPP_NB];
	int16_t circb[NPP_NMINWIN][NPP_NB], circb_shift[NPP_NMINWIN][NPP_NB];
	int16_t pad_;	/* size multiple of 4: kernels copy state by dwords */
};
#define NPP_HOT_BYTES offsetof(NppState, act_min_sub)
static_assert(NPP_HOT_BYTES % 4 == 0, "NppState hot part copied by dwords");
static_assert(sizeof(NppState) % 4 == 0, "NppState copied by dwords");

/* per-frame scratch that the reference keeps in file statics but rewrites
 * before every read (YY, vk, noisespect2, var_rel, alpha_var, ybuf; its
 * temp_yy is a local of the functions using it) */
struct NppScratch {
	int16_t YY[NPP_NB], YY_shift[NPP_NB];
	int16_t vk[NPP_NB], vk_shift[NPP_NB];
	int16_t noisespect2[NPP_NB], noise2_shift[NPP_NB];
	int16_t var_rel[NPP_NB], alpha_var[NPP_NB];
	int16_t ybuf[2 * NPP_WIN + 2];
};

/* The wave form's scratch (npp_wave.h): vk, noisespect2 and alpha_var are
 * written and read back for the same bin within one pass over the bins, so
 * there they are the lane's registers (the per-bin functions take them as
 * parameters); only what crosses bins or passes stays in LDS. */
struct NppScratchW {
	int16_t YY[NPP_NB], YY_shift[NPP_NB];
	int16_t var_rel[NPP_NB];
	/* the first (NPP_WIN + 2) dwords double as wv_enh_init's temp_yy
	 * (npp_wave.h NppWave), which runs while ybuf is live: ybuf after it */
	int16_t pad_[2 * (NPP_WIN + 2) - 3 * NPP_NB];
	int16_t ybuf[2 * NPP_WIN + 2];
};
static_assert(offsetof(NppScratchW, ybuf) == 4 * (NPP_WIN + 2), "ybuf clear of wv_enh_init's temp_yy");

MD void npp_reset(NppState *s)
{
	int16_t *p = (int16_t *) s;
	for (unsigned i = 0; i < sizeof(NppState) / 2; i++)
		p[i] = 0;
	s->Ksi_min_var = GM_MIN;	/* npp.c:1219 */
}

/* comp_data_shift :866 -- compares num1*2^shift1 with num2*2^shift2 */
MD Word16 cmp_shift(Word16 n1, Word16 s1, Word16 n2, Word16 s2)
{
	if (n1 > 0 && n2 < 0)
		return 1;
	if (n1 < 0 && n2 > 0)
		return -1;
	Word16 d = sub(s1, s2);
	if (d > 0)
		n2 = shr(n2, d);
	else
		n1 = shl(n1, d);
	return sub(n1, n2);
}

/* normalised (mantissa, exponent) of a positive 32-bit value */
MD Word16 npp_norm_hi(Word32 v, Word16 *sh)
{
	*sh = norm_l(v);
	return extract_h(L_shl(v, *sh));
}

/* term i of the sum of a block-floating-point spectrum (npp.c:524-535 and
 * 1316-1328); the end bins count half.  Every term is non-negative and at
 * most 2^23 (mantissa < 2^15, shift <= 8 since maxs >= vs[i]), so the
 * reference's saturating L_add chain over 129 terms never saturates and any
 * summation order gives the same value. */
MD Word32 npp_spec_term(const int16_t *v, const int16_t *vs, Word16 maxs, int i)
{
	Word16 half = (i == 0 || i == NPP_NB - 1) ? 7 : 8;
	return L_shl(L_deposit_l(v[i]), sub(half, sub(maxs, vs[i])));
}

MD Word32 npp_spec_sum(const int16_t *v, const int16_t *vs, Word16 maxs)
{
	Word32 s = npp_spec_term(v, vs, maxs, 0);
	s = L_add(s, npp_spec_term(v, vs, maxs, NPP_NB - 1));
	for (int i = 1; i < NPP_NB - 1; i++)
		s = L_add(s, npp_spec_term(v, vs, maxs, i));
	return s;
}

/* gain_mod :211 -- speech-presence-uncertainty modification of the gain */
MD void npp_gain_mod_bin(const NppState *s, Word16 vk, Word16 vk_shift, const int16_t *qk,
			 int16_t *GainD, int i)
{
	{
		Word16 t = sub(SW_MAX_, qk[i]);
		if (t == 0)
			t = 1;
		Word16 sh = norm_s(t);
		t = shl(t, sh);
		Word16 tsh = negate(sh);
		Word32 L = L_mult(t, t);
		sh = norm_l(L);
		Word16 t2 = extract_h(L_shl(L, sh));
		Word16 t2sh = sub(shl(tsh, 1), sh);
		L = L_mult(vk, -23637);
		sh = add(vk_shift, 1);
		L = L_shr(L, sub(15, sh));
		sh = sub(s->ksi_shift[i], tsh);
		Word16 t3, t4;
		if (sh > 0) {
			t4 = add(s->ksi_shift[i], 1);
			t3 = add(shr(t, add(sh, 1)), shr(s->ksi[i], 1));
		} else {
			t4 = add(tsh, 1);
			t3 = add(shr(t, 1), shl(s->ksi[i], sub(sh, 1)));
		}
		Word32 Lt = L_mult(t3, qk[i]);
		L = L_add(L, L_deposit_h(t4));
		sh = extract_h(L);
		t4 = (Word16) (extract_l(L_shr(L, 1)) & 0x7fff);
		Word16 t1 = shr(mult(t4, 9864), 3);
		t1 = pow10_fxp(t1, 14);
		Lt = L_mpy_ls(Lt, t1);
		t3 = norm_l(Lt);
		t1 = extract_h(L_shl(Lt, t3));
		sh = add(sh, sub(1, t3));
		t1 = shr(t1, 1);
		t2 = shr(t2, 1);
		t = sub(sh, t2sh);
		if (t > 0) {
			t3 = add(t1, shr(t2, t));
			t4 = shr(t2, t);
		} else {
			t3 = add(shl(t1, t), t2);
			t4 = t2;
		}
		t = divide_s(t4, t3);
		if (t < GM_MIN)
			t = GM_MIN;
		GainD[i] = mult(GainD[i], t);
	}
}

MN void npp_gain_mod(const NppState *s, const NppScratch *w, const int16_t *qk,
		     int16_t *GainD, int m)
{
	for (int i = 0; i < m; i++)
		npp_gain_mod_bin(s, w->vk[i], w->vk_shift[i], qk, GainD, i);
}

/* compute_qk :289 -- a-priori speech absence probability */
MD void npp_compute_qk_bin(NppState *s, int16_t *qk, const int16_t *gk, const int16_t *gks,
			   Word16 thr, bool first, int i)
{
	if (first)
		s->qla[i] = 16384;
	s->qla[i] = mult(s->qla[i], 30597);
	if (cmp_shift(gk[i], gks[i], thr, 0) < 0)
		s->qla[i] = add(s->qla[i], 2171);
	qk[i] = s->qla[i];
}

MN void npp_compute_qk(NppState *s, int16_t *qk, const int16_t *gk, const int16_t *gks,
		       Word16 thr)
{
	bool first = !s->qk_started;
	for (int i = 0; i < NPP_NB; i++)
		npp_compute_qk_bin(s, qk, gk, gks, thr, first, i);
	s->qk_started = 1;
}

/* gain_log_mmse :319 */
MD void npp_gain_log_mmse_bin(NppState *s, int16_t &vk, int16_t &vk_shift, const int16_t *qk,
			      int16_t *Gain, const int16_t *gk, const int16_t *gks, int i)
{
	{
		Word16 t1 = sub(SW_MAX_, qk[i]);
		Word16 sh = norm_s(t1);
		t1 = shl(t1, sh);
		Word16 t2 = sub(s->ksi_shift[i], (Word16) -sh);
		if (t2 > 0) {
			t1 = shr(t1, add(t2, 1));
			t1 = add(t1, shr(s->ksi[i], 1));
			t2 = shr(s->ksi[i], 1);
		} else {
			t1 = add(shr(t1, 1), shl(s->ksi[i], sub(t2, 1)));
			t2 = shl(s->ksi[i], sub(t2, 1));
		}
		Word16 kv = divide_s(t2, t1);
		Word32 L = L_mult(kv, gk[i]);
		sh = norm_l(L);
		vk = extract_h(L_shl(L, sh));
		vk_shift = sub(gks[i], sh);
		if (cmp_shift(vk, vk_shift, 32767, -52) < 0) {
			vk = 32767;
			vk_shift = -52;
		}
		if (cmp_shift(vk, vk_shift, 26214, -3) < 0) {
			t1 = log10_fxp(vk, 15);
			L = L_shl(L_deposit_l(t1), 14);
			L = L_add(L, L_shl(L_mult(vk_shift, 9864), 10));
			L = L_mpy_ls(L, -18923);
			L = L_sub(L, 10066330L);
		} else if (cmp_shift(vk, vk_shift, 25600, 8) > 0) {
			L = 1;
			vk = 25600;
			vk_shift = 8;
		} else if (cmp_shift(vk, vk_shift, 32767, 0) > 0) {
			L = L_mult(vk, -17039);
			L = L_sub(L, L_shr(L_deposit_h(8520), vk_shift));
			L = L_shr(L, sub(14, vk_shift));
			L = L_mpy_ls(L, 27213);
			sh = extract_h(L_shl(L, 1));
			t1 = (Word16) (extract_l(L) & 0x7fff);
			t1 = shr(mult(t1, 9864), 3);
			t1 = pow10_fxp(t1, 14);
			L = L_shl(L_deposit_l(t1), 10);
			L = L_shl(L, sh);
		} else {
			t1 = vk;
			if (vk_shift != 0)
				t1 = shl(t1, vk_shift);
			t1 = log10_fxp(t1, 15);
			L = L_shl(L_deposit_l(t1), 13);
			L = L_mpy_ls(L, -25297);
			L = L_add(L, 2785018L);
		}
		L = L_mpy_ls(L, 23637);
		sh = shr(extract_h(L), 8);
		if (cmp_shift(kv, sh, 32767, 0) > 0) {
			Gain[i] = 32767;
			return;
		}
		t1 = extract_l(L_shr(L, 9));
		t1 = (Word16) (t1 & 0x7fff);
		t1 = shr(mult(t1, 9864), 3);
		t1 = pow10_fxp(t1, 14);
		L = L_shl(L_deposit_h(kv), sh);
		L = L_mpy_ls(L, t1);
		if (L_sub(L, 1073676288L) > 0)
			Gain[i] = 32767;
		else
			Gain[i] = extract_h(L_shl(L, 1));
	}
}

MN void npp_gain_log_mmse(NppState *s, NppScratch *w, const int16_t *qk, int16_t *Gain,
			  const int16_t *gk, const int16_t *gks, int m)
{
	for (int i = 0; i < m; i++)
		npp_gain_log_mmse_bin(s, w->vk[i], w->vk_shift[i], qk, Gain, gk, gks, i);
}

/* ksi_min_adapt :428 */
MN Word16 npp_ksi_min_adapt(bool nflag, Word16 kmin, Word16 snlt, Word16 snlt_sh)
{
	if (nflag)
		return kmin;
	Word32 L;
	Word16 sh;
	if (snlt_sh > 0) {
		L = L_add(L_deposit_l(snlt), L_shr(16384, snlt_sh));
		sh = snlt_sh;
	} else {
		L = L_add(L_shl(L_deposit_l(snlt), snlt_sh), 16384);
		sh = 0;
	}
	if (L > SW_MAX_) {
		L = L_shr(L, 1);
		sh = add(sh, 1);
	}
	Word16 t = log10_fxp(extract_l(L), 15);
	L = L_shr(L_mult(t, 8844), 9);
	L = L_add(L, L_mult(sh, 21299));
	L = L_sub(L, 472742L);
	sh = extract_h(L);
	t = (Word16) (extract_l(L_shr(L, 1)) & 0x7fff);
	t = shr(mult(t, 9864), 3);
	t = pow10_fxp(t, 14);
	L = L_shl(L_mult(kmin, t), 1);
	t = extract_h(L);
	if (cmp_shift(t, sh, 8192, 0) > 0)
		return 8192;
	return shl(t, sh);
}

/* smoothing_win :486 -- taper the initial noise spectrum estimate */
MD void npp_smoothing_win(int16_t *x)
{
	const int16_t *wf = TB(wtr_front);
	for (int i = 1; i < 32; i++)
		x[i] = mult(x[i], wf[i]);
	for (int i = NPP_WIN - 32 + 1; i < NPP_WIN; i++)
		x[i] = mult(x[i], wf[NPP_WIN - i]);
	v_zero(&x[32], NPP_WIN - 64 + 1);
}

/* smoothed_periodogram :511 -- optimal recursive smoothing of |Y|^2.
 * Scalar part: the smoothing-parameter correction (alphacorr) from the
 * spectrum sum, and the lower bound amin; returns anum. */
MD Word16 npp_sm_period_scalars(NppState *s, Word16 maxs, Word32 L, Word16 YY_av, Word16 yy_shift,
				Word16 *amin_out)
{
	if (L == 0)
		L = 1;
	Word16 t = sub(norm_l(L), 1);
	Word16 sav = extract_h(L_shl(L, t));
	Word16 savs = sub(add(maxs, 1), t);
	Word16 acn = divide_s(sav, YY_av);
	Word16 sh = sub(savs, yy_shift);
	if (sh <= 0) {
		if (sh > -15)
			acn = sub(shl(acn, sh), SW_MAX_);
		else
			acn = negate(SW_MAX_);
		sh = 0;
	} else if (sh < 15) {
		acn = sub(acn, shr(SW_MAX_, sh));
	}
	acn = mult(acn, acn);
	acn = shr(acn, 1);
	sh = shl(sh, 1);
	if (sh < 15)
		acn = add(acn, shr(16384, sh));
	if (acn == 0) {
		acn = SW_MAX_;
	} else if (sh < 15) {
		acn = divide_s(shr(16384, sh), acn);
	} else {
		acn = 0;
	}
	if (acn < 22938)
		acn = 22938;
	s->alphacorr = extract_h(L_add(L_mult(22938, s->alphacorr), L_mult(9830, acn)));

	if (cmp_shift(s->SN_LT, s->SN_LT_shift, 16384, 15) > 0)
		L = 536870912L;
	else if (cmp_shift(s->SN_LT, s->SN_LT_shift, 32, 15) < 0)
		L = 1048576L;
	else
		L = L_shl(L_deposit_l(s->SN_LT), s->SN_LT_shift);
	t = L_log10_fxp(L, 15);
	t = shl(t, 1);
	t = mult(t, -10240);
	Word16 amin = pow10_fxp(t, 15);
	if (amin > 9830)
		amin = 9830;
	else if (amin < 1638)
		amin = 1638;
	*amin_out = amin;
	return mult(30802, s->alphacorr);
}

/* per-bin part of smoothed_periodogram */
template <class SC>
MD void npp_sm_period_bin(NppState *s, SC *w, Word16 anum, Word16 amin, int i, int16_t &ns2, int16_t &ns2_shift,
			  int16_t &alpha_var)
{
	Word16 ns = s->noisespect[i];
	Word32 Lt, L;
	Word16 sh = sub(s->sm_shift[i], s->noise_shift[i]);
	if (sh > 0) {
		Lt = L_sub(L_deposit_h(s->smoothedspect[i]),
			   L_shr(L_deposit_h(s->noisespect[i]), sh));
		sh = s->sm_shift[i];
	} else {
		Lt = L_sub(L_shr(L_deposit_h(s->smoothedspect[i]), abs_s(sh)),
			   L_deposit_h(ns));
		sh = s->noise_shift[i];
	}
	Word16 t1 = norm_l(Lt);
	Word16 t = extract_h(L_shl(Lt, t1));
	sh = sub(sh, t1);
	L = L_mult(ns, ns);
	Word16 nsh = norm_l(L);
	ns = extract_h(L_shl(L, nsh));
	Word16 nssh = sub(shl(s->noise_shift[i], 1), nsh);
	ns2 = ns;
	ns2_shift = nssh;
	if (t == SW_MIN_)
		L = 0x7fffffff;
	else
		L = L_mult(t, t);
	nsh = norm_l(L);
	t = extract_h(L_shl(L, nsh));
	Word16 tsh = (t == 0) ? (Word16) -20 : sub(shl(sh, 1), nsh);
	t1 = sub(tsh, nssh);
	if (t1 > 0) {
		t = shr(t, 1);
		ns = shr(ns, add(t1, 1));
	} else {
		ns = shr(ns, 1);
		t = shl(t, sub(t1, 1));
	}
	Word16 ta = divide_s(ns, add(t, ns));
	ta = mult(ta, anum);
	if (ta < amin)
		ta = amin;
	t = sub(SW_MAX_, ta);
	alpha_var = ta;
	Word16 ds = sub(w->YY_shift[i], s->sm_shift[i]);
	if (ds > 0) {
		L = L_shr(L_mult(ta, s->smoothedspect[i]), ds);
		L = L_add(L, L_mult(t, w->YY[i]));
		s->sm_shift[i] = w->YY_shift[i];
	} else {
		L = L_mult(ta, s->smoothedspect[i]);
		L = L_add(L, L_shl(L_mult(t, w->YY[i]), ds));
	}
	if (L < 1)
		L = 1;
	sh = norm_l(L);
	s->smoothedspect[i] = extract_h(L_shl(L, sh));
	s->sm_shift[i] = sub(s->sm_shift[i], sh);
}

MN void npp_smoothed_periodogram(NppState *s, NppScratch *w, Word16 YY_av, Word16 yy_shift)
{
	Word16 maxs = SW_MIN_;
	for (int i = 0; i < NPP_NB; i++)
		if (s->sm_shift[i] > maxs)
			maxs = s->sm_shift[i];
	Word32 L = npp_spec_sum(s->smoothedspect, s->sm_shift, maxs);
	Word16 amin;
	Word16 anum = npp_sm_period_scalars(s, maxs, L, YY_av, yy_shift, &amin);
	for (int i = 0; i < NPP_NB; i++)
		npp_sm_period_bin(s, w, anum, amin, i, w->noisespect2[i], w->noise2_shift[i], w->alpha_var[i]);
}

/* bias_compensation :695, first per-bin pass: the variance estimates and
 * the relative variance var_rel[i] (0..16384) */
template <class SC>
MD void npp_bias1_bin(NppState *s, SC *w, int i, Word16 alpha_var, Word16 ns2, Word16 ns2_shift)
{
	Word16 beta = mult(alpha_var, alpha_var);
	if (beta > 26214)
		beta = 26214;
	Word32 L = L_mult(sub(SW_MAX_, beta), s->smoothedspect[i]);
	Word16 ds = sub(s->sm_shift[i], s->av_shift[i]);
	Word32 m1;
	if (ds > 0) {
		m1 = L_add(L_shr(L_mult(beta, s->var_sp_av[i]), ds), L);
		s->av_shift[i] = s->sm_shift[i];
	} else {
		m1 = L_add(L_mult(beta, s->var_sp_av[i]), L_shl(L, ds));
	}
	if (m1 < 1)
		m1 = 1;
	Word16 s1 = norm_l(m1);
	s->var_sp_av[i] = extract_h(L_shl(m1, s1));
	s->av_shift[i] = sub(s->av_shift[i], s1);
	Word16 ds2 = sub(shl(s->sm_shift[i], 1), s->av2_shift[i]);
	Word32 m2;
	if (ds2 > 0) {
		m2 = L_add(L_shr(L_mult(beta, s->var_sp_2[i]), ds2),
			   L_mpy_ls(L, s->smoothedspect[i]));
		s->av2_shift[i] = shl(s->sm_shift[i], 1);
	} else {
		m2 = L_add(L_mult(beta, s->var_sp_2[i]),
			   L_shl(L_mpy_ls(L, s->smoothedspect[i]), ds2));
	}
	if (m2 < 1)
		m2 = 1;
	s1 = norm_l(m2);
	s->var_sp_2[i] = extract_h(L_shl(m2, s1));
	s->av2_shift[i] = sub(s->av2_shift[i], s1);
	L = L_mult(s->var_sp_av[i], s->var_sp_av[i]);
	Word16 s3 = sub(s->av2_shift[i], shl(s->av_shift[i], 1));
	Word16 s4;
	if (s3 > 0) {
		L = L_sub(L_deposit_h(s->var_sp_2[i]), L_shr(L, s3));
		s4 = s->av2_shift[i];
	} else {
		L = L_sub(L_shl(L_deposit_h(s->var_sp_2[i]), s3), L);
		s4 = shl(s->av_shift[i], 1);
	}
	s1 = sub(norm_l(L), 1);
	Word16 t1 = extract_h(L_shl(L, s1));
	Word16 t = sub(sub(s4, s1), ns2_shift);
	w->var_rel[i] = divide_s(t1, ns2);
	if (cmp_shift(w->var_rel[i], t, 16384, 0) > 0)
		w->var_rel[i] = 16384;
	else
		w->var_rel[i] = shl(w->var_rel[i], t);
	if (w->var_rel[i] < 0)
		w->var_rel[i] = 0;
}

/* the scalar middle of bias_compensation: vsum = sum of var_rel over the
 * bins (each 0..16384, so the reference's L_add chain never saturates and
 * any order gives the same sum); returns vsq, sets f1/f2 */
template <class SC>
MD Word16 npp_bias_scalars(NppState *s, const SC *w, Word32 vsum, Word16 *f1, Word16 *f2)
{
	vsum = L_shl(vsum, 1);
	vsum = L_sub(vsum, L_deposit_l(w->var_rel[0]));
	vsum = L_sub(vsum, L_deposit_l(w->var_rel[NPP_NB - 1]));
	s->var_rel_av = extract_l(L_shr(vsum, 8));
	if (s->var_rel_av < 0)
		s->var_rel_av = 0;
	Word16 vsq = mult(12288, sqrt_Q15(s->var_rel_av));
	vsq = add(8192, vsq);
	*f1 = extract_h(L_shl(L_mult(vsq, 16521), 1));
	*f2 = extract_h(L_shl(L_mult(vsq, 18643), 1));
	return vsq;
}

/* second per-bin pass: the bias-compensated spectra for the minimum search */
template <class SC>
MD void npp_bias2_bin(const NppState *s, const SC *w, int16_t &bsp, int16_t &bsh,
		      int16_t &bsub, int16_t &bsubsh, Word16 vsq, Word16 f1, Word16 f2, int i)
{
	Word32 L3 = L_mult(vsq, s->smoothedspect[i]);
	Word16 vr = w->var_rel[i];
	Word32 L4 = L_mult(vr, s->smoothedspect[i]);
	Word16 t = add(19543, shr(vr, 1));
	t = add(11656, shr(mult(vr, t), 1));
	Word32 L = L_mpy_ls(L_mpy_ls(L4, f1), t);
	L = L_add(L_shr(L3, 6), L_shr(L, 1));
	if (L < 1)
		L = 1;
	Word16 s1 = norm_l(L);
	bsp = extract_h(L_shl(L, s1));
	bsh = add(s->sm_shift[i], sub(8, s1));
	t = add(13968, shr(vr, 2));
	t = add(11909, shr(mult(vr, t), 1));
	L = L_mpy_ls(L_mpy_ls(L4, f2), t);
	L = L_add(L_shr(L3, 4), L_shr(L, 1));
	if (L < 1)
		L = 1;
	s1 = norm_l(L);
	bsub = extract_h(L_shl(L, s1));
	bsubsh = add(s->sm_shift[i], sub(6, s1));
}

MN void npp_bias_compensation(NppState *s, NppScratch *w, int16_t *bsp, int16_t *bsh,
			      int16_t *bsub, int16_t *bsubsh)
{
	Word32 vsum = 0;
	for (int i = 0; i < NPP_NB; i++) {
		npp_bias1_bin(s, w, i, w->alpha_var[i], w->noisespect2[i], w->noise2_shift[i]);
		vsum = L_add(vsum, L_deposit_l(w->var_rel[i]));
	}
	Word16 f1, f2;
	Word16 vsq = npp_bias_scalars(s, w, vsum, &f1, &f2);
	for (int i = 0; i < NPP_NB; i++)
		npp_bias2_bin(s, w, bsp[i], bsh[i], bsub[i], bsubsh[i], vsq, f1, f2, i);
}

/* noise_slope :843 */
MD Word16 npp_noise_slope(const NppState *s)
{
	if (s->var_rel_av > 5898)
		return 2703;
	if (s->var_rel_av < 983 || s->enh_i < 50)
		return 18022;
	if (s->var_rel_av < 1638)
		return 9011;
	if (s->var_rel_av < 1966)
		return 4506;
	return 2703;
}

/* min_search :889 -- minimum tracking over 8 windows of 9 frames.  Every
 * loop of the reference touches bin i only, so the per-bin part runs each
 * bin through the whole branch; the counters advance afterwards. */
MD void npp_min_search_bin(NppState *s, NppState *m, int16_t bsp, int16_t bsh, int16_t bsub,
			   int16_t bsubsh, Word16 slope, int i)
{
	if (s->minspec_counter == 0) {
		if (cmp_shift(bsp, bsh, s->act_min[i], s->act_min_shift[i]) < 0) {
			s->act_min[i] = bsp;
			s->act_min_shift[i] = bsh;
			m->act_min_sub[i] = bsub;
			m->act_min_sub_shift[i] = bsubsh;
			m->localflag[i] = 0;
		}
		m->circb[s->circb_index][i] = s->act_min[i];
		m->circb_shift[s->circb_index][i] = s->act_min_shift[i];
		Word16 t1 = m->circb[0][i], t2 = m->circb_shift[0][i];
		for (int k = 1; k < NPP_NMINWIN; k++)
			if (cmp_shift(m->circb[k][i], m->circb_shift[k][i], t1, t2) < 0) {
				t1 = m->circb[k][i];
				t2 = m->circb_shift[k][i];
			}
		m->circb_min[i] = t1;
		m->circb_min_shift[i] = t2;
		Word16 t = mult(slope, m->circb_min[i]);
		Word16 ts = add(m->circb_min_shift[i], 4);
		if (m->localflag[i] &&
		    cmp_shift(m->act_min_sub[i], m->act_min_sub_shift[i],
			      m->circb_min[i], m->circb_min_shift[i]) > 0 &&
		    cmp_shift(m->act_min_sub[i], m->act_min_sub_shift[i], t, ts) < 0) {
			m->circb_min[i] = m->act_min_sub[i];
			m->circb_min_shift[i] = m->act_min_sub_shift[i];
			for (int k = 0; k < NPP_NMINWIN; k++) {
				m->circb[k][i] = m->circb_min[i];
				m->circb_shift[k][i] = m->circb_min_shift[i];
			}
		}
		m->localflag[i] = 0;
	} else if (s->minspec_counter == 1) {
		s->act_min[i] = bsp;
		s->act_min_shift[i] = bsh;
		m->act_min_sub[i] = bsub;
		m->act_min_sub_shift[i] = bsubsh;
	} else {
		if (cmp_shift(bsp, bsh, s->act_min[i], s->act_min_shift[i]) < 0) {
			s->act_min[i] = bsp;
			s->act_min_shift[i] = bsh;
			m->act_min_sub[i] = bsub;
			m->act_min_sub_shift[i] = bsubsh;
			m->localflag[i] = 1;
		}
		if (cmp_shift(m->act_min_sub[i], m->act_min_sub_shift[i],
			      m->circb_min[i], m->circb_min_shift[i]) < 0) {
			m->circb_min[i] = m->act_min_sub[i];
			m->circb_min_shift[i] = m->act_min_sub_shift[i];
		}
		s->noisespect[i] = m->circb_min[i];
		s->noise_shift[i] = m->circb_min_shift[i];
		Word32 L = L_mult(NOISE_BIAS, s->noisespect[i]);
		if (L < 0x40000000L) {
			L = L_shl(L, 1);
			s->lambdaD_shift[i] = s->noise_shift[i];
		} else {
			s->lambdaD_shift[i] = add(s->noise_shift[i], 1);
		}
		s->lambdaD[i] = extract_h(L);
	}
}

MD void npp_min_search_post(NppState *s)
{
	if (s->minspec_counter == 0) {
		s->circb_index = add(s->circb_index, 1);
		if (s->circb_index == NPP_NMINWIN)
			s->circb_index = 0;
	}
	s->minspec_counter = add(s->minspec_counter, 1);
	if (s->minspec_counter == NPP_LMINWIN)
		s->minspec_counter = 0;
}

MN void npp_min_search(NppState *s, const int16_t *bsp, const int16_t *bsh,
		       const int16_t *bsub, const int16_t *bsubsh)
{
	Word16 slope = npp_noise_slope(s);
	for (int i = 0; i < NPP_NB; i++)
		npp_min_search_bin(s, s, bsp[i], bsh[i], bsub[i], bsubsh[i], slope, i);
	npp_min_search_post(s);
}

/* minstat_init :1164 */
MN void npp_minstat_init(NppState *s)
{
	v_copy(s->smoothedspect, s->lambdaD, NPP_NB);
	v_scale(s->smoothedspect, NOISE_BIAS, NPP_NB);
	for (int k = 0; k < NPP_NMINWIN; k++) {
		v_copy(s->circb[k], s->smoothedspect, NPP_NB);
		v_copy(s->circb_shift[k], s->lambdaD_shift, NPP_NB);
	}
	v_copy(s->sm_shift, s->lambdaD_shift, NPP_NB);
	v_copy(s->act_min, s->smoothedspect, NPP_NB);
	v_copy(s->act_min_shift, s->lambdaD_shift, NPP_NB);
	v_copy(s->act_min_sub, s->smoothedspect, NPP_NB);
	v_copy(s->act_min_sub_shift, s->lambdaD_shift, NPP_NB);
	v_copy(s->noisespect, s->smoothedspect, NPP_NB);
	v_copy(s->noise_shift, s->lambdaD_shift, NPP_NB);
	for (int i = 0; i < NPP_NB; i++) {
		s->var_sp_av[i] = mult(s->smoothedspect[i], 20066);
		s->av_shift[i] = add(s->lambdaD_shift[i], 1);
		Word32 L = L_mult(s->smoothedspect[i], s->smoothedspect[i]);
		Word16 sh = norm_l(L);
		s->var_sp_2[i] = extract_h(L_shl(L, sh));
		s->av2_shift[i] = sub(shl(s->lambdaD_shift[i], 1), sub(sh, 1));
	}
	s->alphacorr = 29491;
}

/* enh_init :1023 -- initial noise estimate from the first 256 samples */
MN void npp_enh_init(NppState *s, NppScratch *w, int16_t *noise)
{
	int16_t *yb = w->ybuf;
	int32_t ty[NPP_WIN + 2];
	window(noise, TB(sqrt_tukey_256_180), noise, NPP_WIN);
	Word16 mx = 1;
	for (int i = 0; i < NPP_WIN; i++) {
		Word16 t = abs_s(noise[i]);
		if (t > mx)
			mx = t;
	}
	Word16 sh = norm_s(mx);
	Word16 ash = sub(15, sh);
	v_zero(yb, 2 * NPP_WIN + 2);
	for (int i = 0; i < NPP_WIN; i++)
		yb[2 * i] = shl(noise[i], sh);
	Word16 g = fft_npp(yb, 1);
	ty[0] = L_shr(L_mult(yb[0], yb[0]), 1);
	ty[1] = 0;
	ty[NPP_WIN] = L_shr(L_mult(yb[NPP_WIN], yb[NPP_WIN]), 1);
	ty[NPP_WIN + 1] = 0;
	for (int i = 2; i < NPP_WIN - 1; i += 2) {
		ty[i + 1] = 0;
		ty[i] = L_shr(L_add(L_mult(yb[i], yb[i]), L_mult(yb[i + 1], yb[i + 1])), 1);
	}
	Word32 L = ty[0];
	for (int i = 1; i < NPP_WIN + 1; i++)
		if (L < ty[i])
			L = ty[i];
	sh = norm_l(L);
	for (int i = 0; i < NPP_WIN + 1; i++)
		yb[i] = extract_h(L_shl(ty[i], sh));
	sh = sub(shl(add(ash, g), 1), add(sh, 7));
	for (int i = 0; i < NPP_WIN / 2 - 1; i++) {
		yb[NPP_WIN + 2 * i + 2] = yb[NPP_WIN - 2 * i - 2];
		yb[NPP_WIN + 2 * i + 3] = negate(yb[NPP_WIN - 2 * i - 1]);
	}
	g = fft_npp(yb, -1);
	sh = add(sh, g);
	sh = sub(sh, 8);
	for (int i = 0; i < NPP_WIN; i++)
		noise[i] = yb[2 * i];
	mx = 0;
	for (int i = 0; i < NPP_WIN; i++) {
		Word16 t = abs_s(noise[i]);
		if (t > mx)
			mx = t;
	}
	Word16 t = norm_s(mx);
	sh = sub(sh, t);
	for (int i = 0; i < NPP_WIN; i++)
		noise[i] = shl(noise[i], t);
	npp_smoothing_win(noise);
	v_zero(yb, 2 * NPP_WIN + 2);
	for (int i = 0; i < NPP_WIN; i++)
		yb[2 * i] = noise[i];
	g = fft_npp(yb, 1);
	for (int i = 0; i <= NPP_WIN * 2; i += 2)
		if (yb[i] < 0)
			yb[i] = 0;
	Word16 nsh = add(sh, g);
	L = L_add(L_shl(L_mult(181, yb[0]), 7), 2);
	sh = norm_l(L);
	s->lambdaD[0] = extract_h(L_shl(L, sh));
	s->lambdaD_shift[0] = add(nsh, sub(1, sh));
	L = L_shr(L, 8);
	Word32 Ld = L_add(L_shl(L_mult(181, yb[NPP_WIN]), 7), 2);
	sh = norm_l(Ld);
	s->lambdaD[NPP_WIN / 2] = extract_h(L_shl(Ld, sh));
	s->lambdaD_shift[NPP_WIN / 2] = add(nsh, sub(1, sh));
	L = L_add(L, L_shr(Ld, 8));
	for (int i = 1; i < NPP_WIN / 2; i++) {
		Ld = L_add(L_shl(L_mult(181, yb[2 * i]), 7), 2);
		sh = norm_l(Ld);
		s->lambdaD[i] = extract_h(L_shl(Ld, sh));
		s->lambdaD_shift[i] = add(nsh, sub(1, sh));
		L = L_add(L, L_shr(Ld, 7));
	}
	sh = norm_l(L);
	s->n_pwr = extract_h(L_shl(L, sh));
	s->n_pwr_shift = sub(add(nsh, 1), sh);
	s->SN_LT = divide_s(14648, s->n_pwr);
	s->SN_LT_shift = sub(22, s->n_pwr_shift);
	npp_minstat_init(s);
}

/* a-priori SNR (decision-directed) of bin i, npp.c:1420-1465 */
MD void npp_ksi_bin(NppState *s, const int16_t *gk, const int16_t *gks, int i)
{
	Word32 L = L_mpy_ls(L_mult(s->agal[i], s->agal[i]), 30474);
	if (L < 1)
		L = 1;
	Word16 sh = norm_l(L);
	Word16 t1 = extract_h(L_shl(L, sh));
	Word16 t2 = sub(shl(s->agal_shift[i], 1), add(sh, 8));
	Word16 t3 = s->lambdaD[i];
	Word16 t4 = s->lambdaD_shift[i];
	if (sub(t3, t1) < 0) {
		t1 = shr(t1, 1);
		t2 = (Word16) (t2 + 1);
	}
	s->ksi[i] = divide_s(t1, t3);
	s->ksi_shift[i] = sub(t2, t4);
	if (cmp_shift(gk[i], gks[i], NOISE_BIAS, 0) > 0) {
		L = L_shr(L_deposit_h(NOISE_BIAS), gks[i]);
		L = L_sub(L_deposit_h(gk[i]), L);
		sh = norm_l(L);
		t1 = extract_h(L_shl(L, sh));
		t1 = mult(t1, 18350);
		t2 = sub(gks[i], add(sh, 3));
		sh = sub(s->ksi_shift[i], t2);
		if (sh > 0) {
			s->ksi[i] = add(shr(s->ksi[i], 1), shr(t1, (Word16) (sh + 1)));
			s->ksi_shift[i] = add(s->ksi_shift[i], 1);
		} else {
			s->ksi[i] = add(shl(s->ksi[i], (Word16) (sh - 1)), shr(t1, 1));
			s->ksi_shift[i] = add(t2, 1);
		}
	}
}

/* process_frame :1212 -- one 256-sample analysis/synthesis frame */
MN void npp_process_frame(NppState *s, NppScratch *w, const int16_t *in, int16_t *out)
{
	int16_t *yb = w->ybuf;
	int32_t ty[NPP_WIN + 2];
	int16_t Ymag[NPP_NB], Ymag_shift[NPP_NB], GainD[NPP_NB];
	int16_t gk[NPP_NB], gks[NPP_NB];
	int16_t bsp[NPP_NB], bsub[NPP_NB], bsh[NPP_NB], bsubsh[NPP_NB];
	int16_t analy[NPP_WIN];
	Word16 sh, t, t1, t2, t3, t4;
	Word32 L;

	if (!s->pf_started) {
		v_zero(s->agal, NPP_NB);
		v_zero(s->agal_shift, NPP_NB);
		v_set(s->ksi, GM_MIN, NPP_NB);
		v_zero(s->ksi_shift, NPP_NB);
		v_set(s->qk, ENH_QK_MAX, NPP_NB);
		v_set(s->Gain, GM_MIN, NPP_NB);
		s->YY_LT = 0;
		s->YY_LT_shift = 0;
		s->SN_LT0 = s->SN_LT;
		s->SN_LT0_shift = s->SN_LT_shift;
		s->pf_started = 1;
	}
	/* GainD is a local of the reference: only its first call fills it
	 * (npp.c:1246); the enh_i == 1 branch below does not overwrite it */
	v_set(GainD, GM_MIN, NPP_NB);
	if (s->enh_i < 50)
		s->enh_i++;
	window(in, TB(sqrt_tukey_256_180), analy, NPP_WIN);
	Word16 mx = 1;
	for (int i = 0; i < NPP_WIN; i++) {
		t1 = abs_s(analy[i]);
		if (t1 > mx)
			mx = t1;
	}
	sh = norm_s(mx);
	Word16 ash = sub(15, sh);
	for (int i = 0; i < NPP_WIN; i++)
		analy[i] = shl(analy[i], sh);
	v_zero(yb, 2 * NPP_WIN + 2);
	for (int i = 0; i < 2 * NPP_WIN; i += 2)
		yb[i] = analy[i / 2];
	Word16 g = fft_npp(yb, 1);
	Word16 Ysh = add(ash, g);
	Word16 YYavs = shl(Ysh, 1);
	ty[0] = L_mult(yb[0], yb[0]);
	ty[NPP_NB - 1] = L_mult(yb[NPP_WIN], yb[NPP_WIN]);
	for (int i = 1; i < NPP_NB - 1; i++)
		ty[i] = L_add(L_mult(yb[2 * i], yb[2 * i]), L_mult(yb[2 * i + 1], yb[2 * i + 1]));
	Word16 maxs = SW_MIN_;
	for (int i = 0; i < NPP_NB; i++) {
		if (ty[i] < 1)
			ty[i] = 1;
		sh = norm_l(ty[i]);
		w->YY[i] = extract_h(L_shl(ty[i], sh));
		w->YY_shift[i] = sub(YYavs, sh);
		if (maxs < w->YY_shift[i])
			maxs = w->YY_shift[i];
	}
	for (int i = 0; i < NPP_NB; i++) {
		t = w->YY[i];
		Word16 ts = w->YY_shift[i];
		if (ts & 1) {
			t = shr(t, 1);
			ts = add(ts, 1);
		}
		Ymag[i] = sqrt_Q15(t);
		Ymag_shift[i] = shr(ts, 1);
		w->YY_shift[i] = sub(w->YY_shift[i], 8);
	}
	/* maxs is taken before the -8 (npp.c:1300-1330) */
	L = L_shl(L_deposit_l(w->YY[0]), sub(7, sub(maxs, w->YY_shift[0])));
	L = L_add(L, L_shl(L_deposit_l(w->YY[NPP_NB - 1]),
			   sub(7, sub(maxs, w->YY_shift[NPP_NB - 1]))));
	for (int i = 1; i < NPP_NB - 1; i++)
		L = L_add(L, L_shl(L_deposit_l(w->YY[i]), sub(8, sub(maxs, w->YY_shift[i]))));
	if (L == 0)
		L = 1;
	t1 = norm_l(L);
	Word16 YY_av = extract_h(L_shl(L, t1));
	Word16 YY_av_shift = sub(add(maxs, 1), t1);

	npp_smoothed_periodogram(s, w, YY_av, YY_av_shift);
	npp_bias_compensation(s, w, bsp, bsh, bsub, bsubsh);
	npp_min_search(s, bsp, bsh, bsub, bsubsh);

	for (int i = 0; i < NPP_NB; i++) {
		gk[i] = divide_s(shr(w->YY[i], 1), s->lambdaD[i]);
		gks[i] = sub(add(w->YY_shift[i], 1), s->lambdaD_shift[i]);
	}
	L = L_shl(L_deposit_l(gk[0]), 7);
	sh = sub(gks[0], 1);
	for (int i = 1; i < NPP_NB - 1; i++) {
		t1 = sub(sh, gks[i]);
		if (t1 > 0) {
			L = L_add(L, L_shr(L_deposit_l(gk[i]), sub(t1, 7)));
		} else {
			L = L_add(L_shl(L, t1), L_shl(L_deposit_l(gk[i]), 7));
			sh = gks[i];
		}
	}
	t1 = sub(sh, sub(gks[NPP_NB - 1], 1));
	if (t1 > 0) {
		L = L_add(L, L_shr(L_deposit_l(gk[NPP_NB - 1]), sub(t1, 7)));
	} else {
		L = L_add(L_shl(L, t1), L_shl(L_deposit_l(gk[NPP_NB - 1]), 7));
		sh = sub(gks[NPP_NB - 1], 1);
	}
	if (L == 0)
		L = 1;
	t1 = norm_l(L);
	Word16 gav = extract_h(L_shl(L, t1));
	Word16 gavs = add(sub(sh, t1), 2);
	Word16 gmax = gk[0], gmaxs = gks[0];
	for (int i = 1; i < NPP_NB; i++)
		if (cmp_shift(gmax, gmaxs, gk[i], gks[i]) < 0) {
			gmax = gk[i];
			gmaxs = gks[i];
		}
	bool nflag = false;
	if (cmp_shift(gmax, gmaxs, 18102, 6) < 0 && cmp_shift(gav, gavs, 23170, 1) < 0) {
		nflag = true;
		t1 = mult(s->n_pwr, 23170);
		t2 = add(s->n_pwr_shift, 2);
		if (cmp_shift(YY_av, YY_av_shift, t1, t2) > 0)
			nflag = false;
	}

	if (s->enh_i == 1) {
		for (int i = 0; i < NPP_NB; i++) {
			ty[i] = L_mult(Ymag[i], GM_MIN);
			sh = norm_l(ty[i]);
			s->agal[i] = extract_h(L_shl(ty[i], sh));
			s->agal_shift[i] = sub(Ymag_shift[i], sh);
		}
	} else {
		for (int i = 0; i < NPP_NB; i++)
			npp_ksi_bin(s, gk, gks, i);
		t1 = mult(29491, s->Ksi_min_var);
		t2 = mult(3277, npp_ksi_min_adapt(nflag, GM_MIN, s->SN_LT, s->SN_LT_shift));
		s->Ksi_min_var = add(t1, t2);
		sh = norm_s(s->Ksi_min_var);
		t1 = shl(s->Ksi_min_var, sh);
		for (int i = 0; i < NPP_NB; i++)
			if (cmp_shift(s->ksi[i], s->ksi_shift[i], t1, negate(sh)) < 0) {
				s->ksi[i] = t1;
				s->ksi_shift[i] = negate(sh);
			}
		v_set(s->qk, ENH_QK_MAX, NPP_NB);
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
				if (sh > 0) {
					s->YY_LT = add(t1, shr(t3, sh));
					s->YY_LT_shift = t2;
				} else {
					s->YY_LT = add(shl(t1, sh), t3);
					s->YY_LT_shift = t4;
				}
				s->YY_LT_shift = add(s->YY_LT_shift, 1);
				if (sub(s->YY_LT, s->n_pwr) > 0) {
					s->YY_LT = shr(s->YY_LT, 1);
					s->YY_LT_shift = add(s->YY_LT_shift, 1);
				}
				s->SN_LT = divide_s(s->YY_LT, s->n_pwr);
				s->SN_LT_shift = sub(s->YY_LT_shift, s->n_pwr_shift);
				if (cmp_shift(s->SN_LT, s->SN_LT_shift, SW_MAX_, 0) < 0) {
					s->SN_LT = s->SN_LT0;
					s->SN_LT_shift = s->SN_LT0_shift;
				} else {
					L = L_sub(L_deposit_h(s->SN_LT),
						  L_shr(L_deposit_h(SW_MAX_), s->SN_LT_shift));
					sh = norm_l(L);
					s->SN_LT = extract_h(L_shl(L, sh));
					s->SN_LT_shift = sub(s->SN_LT_shift, sh);
				}
				s->SN_LT0 = s->SN_LT;
				s->SN_LT0_shift = s->SN_LT_shift;
			}
			npp_compute_qk(s, s->qk, gk, gks, 19273);
			for (int i = 0; i < NPP_NB; i++) {
				if (s->qk[i] > ENH_QK_MAX)
					s->qk[i] = ENH_QK_MAX;
				else if (s->qk[i] < ENH_QK_MIN)
					s->qk[i] = ENH_QK_MIN;
			}
		}
		npp_gain_log_mmse(s, w, s->qk, s->Gain, gk, gks, NPP_NB);
		v_copy(GainD, s->Gain, NPP_NB);
		npp_gain_mod(s, w, s->qk, GainD, NPP_NB);
		for (int i = 0; i < NPP_NB; i++) {
			L = L_mult(GainD[i], Ymag[i]);
			sh = norm_l(L);
			s->agal[i] = extract_h(L_shl(L, sh));
			s->agal_shift[i] = sub(Ymag_shift[i], sh);
		}
	}
	for (int i = 0; i < NPP_WIN + 2; i++)
		ty[i] = L_mult(yb[i], GainD[i / 2]);
	Word32 Lmax = 0;
	for (int i = 0; i < NPP_WIN + 2; i++)
		if (Lmax < L_abs(ty[i]))
			Lmax = L_abs(ty[i]);
	sh = norm_l(Lmax);
	for (int i = 0; i < NPP_WIN + 2; i++)
		yb[i] = extract_h(L_shl(ty[i], sh));
	sh = sub(Ysh, sh);
	for (int i = 0; i < NPP_WIN / 2 - 1; i++) {
		yb[NPP_WIN + 2 * i + 2] = yb[NPP_WIN - 2 * i - 2];
		yb[NPP_WIN + 2 * i + 3] = negate(yb[NPP_WIN - 2 * i - 1]);
	}
	g = fft_npp(yb, -1);
	sh = add(sh, g);
	sh = sub(sh, 8);
	const int16_t *win = TB(sqrt_tukey_256_180);
	for (int i = 0; i < NPP_WIN; i++)
		out[i] = mult(shl(yb[2 * i], sub(sh, 15)), win[i]);
	/* noise power for the next frame (npp.c:1621-1635) */
	maxs = SW_MIN_;
	for (int i = 0; i < NPP_NB; i++)
		if (maxs < s->lambdaD_shift[i])
			maxs = s->lambdaD_shift[i];
	L = npp_spec_sum(s->lambdaD, s->lambdaD_shift, maxs);
	if (L == 0)
		L = 1;
	sh = norm_l(L);
	s->n_pwr = extract_h(L_shl(L, sh));
	s->n_pwr_shift = add(sub(maxs, sh), 1);
}

/* npp :170 -- 180 new samples in, 180 enhanced samples out (in place ok).
 * On the first call the initial noise estimate reads 256 samples from sp_in
 * when the codec runs at 1200 bps (npp.c:176-189), else 180 after 76 zeros. */
MN void npp_frame(NppState *s, NppScratch *w, const int16_t *sp_in, int16_t *sp_out,
		  bool rate1200 = true)
{
	PROF_SCOPE(0);
	int16_t outbuf[NPP_WIN];
	if (!s->started) {
		int16_t noise[NPP_WIN];
		if (rate1200) {
			v_copy(noise, sp_in, NPP_WIN);
		} else {	/* rate global still 0: melpe_n before melpe_i */
			v_zero(noise, NPP_OVL);
			v_copy(&noise[NPP_OVL], sp_in, NPP_HOP);
		}
		npp_enh_init(s, w, noise);
		v_zero(s->speech_in, NPP_WIN);
		s->started = 1;
	}
	v_copy(s->speech_in, &s->speech_in[NPP_HOP], NPP_OVL);
	v_copy(&s->speech_in[NPP_OVL], sp_in, NPP_HOP);
	npp_process_frame(s, w, s->speech_in, outbuf);
	v_add(outbuf, s->overlap, NPP_OVL);
	v_copy(s->overlap, &outbuf[NPP_HOP], NPP_OVL);
	v_copy(sp_out, outbuf, NPP_HOP);
}

}  // namespace mlp

#endif
