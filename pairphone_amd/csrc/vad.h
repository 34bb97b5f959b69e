/*
 * vad.h -- PairPhone's voice activity detector: the
 * AMR VAD option 2 of vad/vad2.c, run on six 80-sample windows per MELPe
 * superframe (tx.c:234-239, melpe_enc.c:48-53) to decide whether a
 * superframe is encoded (melpe_a) or sent as silence.
 *
 * One lane per channel, as the codec: VadState is the reference's vadState2
 * (vad/vad2.h:76-103) field for field, one record per channel in HBM, and
 * every function below restates its reference counterpart in the same
 * operation order with the AMR basic ops (vad/basicop2.c), whose saturation
 * rules differ from MELPe's mathhalf in places (shl/shr of negative counts,
 * L_shl by looping, shr_r/L_shr_r rounding), so they are restated here and
 * not shared with ops.h.  Word16 = int16_t, Word32 = int32_t
 * (vad/typedefs.h:88-123 on this ABI).
 *
 * Shared by the GPU kernel (engine.hip) and the host-emulation build.
 */
#ifndef MELPE_VAD_H
#define MELPE_VAD_H

#include <stdint.h>

#if defined(__HIPCC__)
#define VA_FN __host__ __device__ static inline
#else
#define VA_FN static inline
#endif

#define VA_FRM_LEN 80
#define VA_DELAY 24
#define VA_FFT_LEN 128
#define VA_NUM_CHAN 16

/* vad/vad2.h:76-103; zeroed by vad2_reset (vad/vad2.c:876-899) */
struct VadState {
	int16_t pre_emp_mem, update_cnt, hyster_cnt, last_update_cnt;
	int16_t ch_enrg_long_db[VA_NUM_CHAN];
	int32_t Lframe_cnt;
	int32_t Lch_enrg[VA_NUM_CHAN];
	int32_t Lch_noise[VA_NUM_CHAN];
	int16_t last_normb_shift, tsnr, hangover, burstcount, fupdate_flag, negSNRvar,
		negSNRbias, shift_state;
	int32_t L_R0, L_Rmax;
	int32_t LTP_flag;	/* never set on the MELPe path (LTP_flag_update is AMR-only) */
};

/* basic-op census (host count build only, tools/opcount.py): every AMR
 * basic op entered from VAD code, nested op calls not counted (SURVEY.md
 * §8(d) rule) */
#if defined(MELPE_OPCOUNT) && !defined(__HIP__)
extern "C" uint64_t melpe_vad_ops;
extern "C" int melpe_vad_depth;
struct VaOpScope {
	VaOpScope()
	{
		if (!melpe_vad_depth++)
			melpe_vad_ops++;
	}
	~VaOpScope() { melpe_vad_depth--; }
};
#define VA_OP() VaOpScope va_op_scope_
#else
#define VA_OP()
#endif

/* ---- AMR basic ops (vad/basicop2.c) ---------------------------------- */
#define VA_MAX32 ((int32_t) 0x7fffffff)
#define VA_MIN32 ((int32_t) 0x80000000)

VA_FN int16_t va_sat(int32_t x)
{
	return x > 32767 ? 32767 : (x < -32768 ? (int16_t) -32768 : (int16_t) x);
}
VA_FN int32_t va_sat32(int64_t x)
{
	return x > VA_MAX32 ? VA_MAX32 : (x < VA_MIN32 ? VA_MIN32 : (int32_t) x);
}
VA_FN int16_t va_add(int16_t a, int16_t b) { VA_OP(); return va_sat((int32_t) a + b); }	/* :134 */
VA_FN int16_t va_sub(int16_t a, int16_t b) { VA_OP(); return va_sat((int32_t) a - b); }	/* :181 */
VA_FN int16_t va_abs_s(int16_t a)	/* :222 */
{
	VA_OP();
	return a == (int16_t) -32768 ? (int16_t) 32767 : (int16_t) (a < 0 ? -a : a);
}
VA_FN int16_t va_shr_pos(int16_t v, int n)	/* shr, n >= 0 (:354) */
{
	return n >= 15 ? (int16_t) (v < 0 ? -1 : 0) : (int16_t) (v >> n);
}
VA_FN int16_t va_shl_pos(int16_t v, int n)	/* shl, n >= 0 (:282) */
{
	if (n > 15)
		return v == 0 ? (int16_t) 0 : (int16_t) (v > 0 ? 32767 : -32768);
	int32_t r = (int32_t) v * ((int32_t) 1 << n);
	if (r != (int32_t) (int16_t) r)
		return (int16_t) (v > 0 ? 32767 : -32768);
	return (int16_t) r;
}
VA_FN int16_t va_shl(int16_t v, int16_t n)
{
	VA_OP();
	if (n < 0)
		return va_shr_pos(v, n < -16 ? 16 : -n);
	return va_shl_pos(v, n);
}
VA_FN int16_t va_shr(int16_t v, int16_t n)
{
	VA_OP();
	if (n < 0)
		return va_shl_pos(v, n < -16 ? 16 : -n);
	return va_shr_pos(v, n);
}
VA_FN int16_t va_mult(int16_t a, int16_t b)	/* :427 */
{
	VA_OP();
	return va_sat(((int32_t) a * b) >> 15);
}
VA_FN int16_t va_mult_r(int16_t a, int16_t b)	/* :1285 */
{
	VA_OP();
	return va_sat(((int32_t) a * b + 0x4000) >> 15);
}
VA_FN int32_t va_L_mult(int16_t a, int16_t b)	/* :481 */
{
	VA_OP();
	int32_t p = (int32_t) a * b;
	return p == 0x40000000 ? VA_MAX32 : p * 2;
}
VA_FN int32_t va_L_add(int32_t a, int32_t b) { VA_OP(); return va_sat32((int64_t) a + b); }	/* :927 */
VA_FN int32_t va_L_sub(int32_t a, int32_t b) { VA_OP(); return va_sat32((int64_t) a - b); }	/* :979 */
VA_FN int32_t va_L_mac(int32_t c, int16_t a, int16_t b) { VA_OP(); return va_L_add(c, va_L_mult(a, b)); }
VA_FN int32_t va_L_msu(int32_t c, int16_t a, int16_t b) { VA_OP(); return va_L_sub(c, va_L_mult(a, b)); }
VA_FN int32_t va_L_negate(int32_t x) { VA_OP(); return x == VA_MIN32 ? VA_MAX32 : -x; }	/* :1240 */
VA_FN int32_t va_L_shr_pos(int32_t x, int n)	/* L_shr, n >= 0 (:1416) */
{
	return n >= 31 ? (x < 0 ? -1 : 0) : (x >> n);
}
/* L_shl, n > 0 (:1340): the reference doubles n times and saturates as soon
 * as the value leaves the 32-bit range, i.e. a saturating shift */
VA_FN int32_t va_L_shl_pos(int32_t x, int n)
{
	if (x == 0)
		return 0;
	if (n >= 32)
		return x > 0 ? VA_MAX32 : VA_MIN32;
	return va_sat32((int64_t) x * ((int64_t) 1 << n));
}
VA_FN int32_t va_L_shl(int32_t x, int16_t n)
{
	VA_OP();
	if (n <= 0)
		return va_L_shr_pos(x, n < -32 ? 32 : -n);
	return va_L_shl_pos(x, n);
}
VA_FN int32_t va_L_shr(int32_t x, int16_t n)
{
	VA_OP();
	if (n < 0)
		return va_L_shl_pos(x, n < -32 ? 32 : -n);
	return va_L_shr_pos(x, n);
}
VA_FN int16_t va_shr_r(int16_t v, int16_t n)	/* :1495 */
{
	VA_OP();
	if (n > 15)
		return 0;
	int16_t r = va_shr(v, n);
	if (n > 0 && (v & ((int16_t) 1 << (n - 1))))
		r++;
	return r;
}
VA_FN int32_t va_L_shr_r(int32_t x, int16_t n)	/* :1764 */
{
	VA_OP();
	if (n > 31)
		return 0;
	int32_t r = va_L_shr(x, n);
	if (n > 0 && (x & ((int32_t) 1 << (n - 1))))
		r++;
	return r;
}
VA_FN int16_t va_extract_h(int32_t x) { VA_OP(); return (int16_t) (x >> 16); }
VA_FN int16_t va_extract_l(int32_t x) { VA_OP(); return (int16_t) x; }
VA_FN int32_t va_L_deposit_h(int16_t v) { VA_OP(); return (int32_t) ((uint32_t) (int32_t) v << 16); }
VA_FN int16_t va_round(int32_t x) { VA_OP(); return va_extract_h(va_L_add(x, 0x8000)); }	/* bround :652 */
VA_FN int16_t va_norm_s(int16_t v)	/* :1938 */
{
	VA_OP();
	if (v == 0)
		return 0;
	if (v == -1)
		return 15;
	int32_t u = v < 0 ? ~v : v;
	return (int16_t) (__builtin_clz((uint32_t) u) - 17);
}
VA_FN int16_t va_norm_l(int32_t x)	/* :2105 */
{
	VA_OP();
	if (x == 0)
		return 0;
	if (x == -1)
		return 31;
	uint32_t u = (uint32_t) (x < 0 ? ~x : x);
	return (int16_t) (__builtin_clz(u) - 1);
}
/* div_s (:2008); callers guarantee 0 < num <= den */
VA_FN int16_t va_div_s(int16_t num, int16_t den)
{
	VA_OP();
	if (num == 0)
		return 0;
	if (num == den)
		return 32767;
	int32_t n = num, d = den;
	int16_t out = 0;
	for (int it = 0; it < 15; it++) {
		out = (int16_t) (out << 1);
		n <<= 1;
		if (n >= d) {
			n = va_L_sub(n, d);
			out = va_add(out, 1);
		}
	}
	return out;
}

/* ---- oper_32b.c, log2.c, pow2.c --------------------------------------- */
VA_FN void va_L_Extract(int32_t L, int16_t *hi, int16_t *lo)	/* oper_32b.c L_Extract */
{
	*hi = va_extract_h(L);
	*lo = va_extract_l(va_L_msu(va_L_shr(L, 1), *hi, 16384));
}
VA_FN int32_t va_Mpy_32_16(int16_t hi, int16_t lo, int16_t n)	/* oper_32b.c Mpy_32_16 */
{
	return va_L_mac(va_L_mult(hi, n), va_mult(lo, n), 1);
}
/* log2.c Log2 + Log2_norm, table vad/log2.tab */
VA_FN void va_Log2(int32_t L_x, int16_t *exponent, int16_t *fraction)
{
	static const int16_t tab[33] = {
		0, 1455, 2866, 4236, 5568, 6863, 8124, 9352, 10549, 11716,
		12855, 13967, 15054, 16117, 17156, 18172, 19167, 20142, 21097, 22033,
		22951, 23852, 24735, 25603, 26455, 27291, 28113, 28922, 29716, 30497,
		31266, 32023, 32767};
	int16_t exp = va_norm_l(L_x);
	L_x = va_L_shl(L_x, exp);
	if (L_x <= 0) {
		*exponent = 0;
		*fraction = 0;
		return;
	}
	*exponent = va_sub(30, exp);
	L_x = va_L_shr(L_x, 9);
	int16_t i = va_extract_h(L_x);
	L_x = va_L_shr(L_x, 1);
	int16_t a = (int16_t) (va_extract_l(L_x) & 0x7fff);
	i = va_sub(i, 32);
	int32_t L_y = va_L_deposit_h(tab[i]);
	int16_t tmp = va_sub(tab[i], tab[i + 1]);
	L_y = va_L_msu(L_y, tmp, a);
	*fraction = va_extract_h(L_y);
}
/* pow2.c Pow2, table vad/pow2.tab */
VA_FN int32_t va_Pow2(int16_t exponent, int16_t fraction)
{
	static const int16_t tab[33] = {
		16384, 16743, 17109, 17484, 17867, 18258, 18658, 19066, 19484, 19911,
		20347, 20792, 21247, 21713, 22188, 22674, 23170, 23678, 24196, 24726,
		25268, 25821, 26386, 26964, 27554, 28158, 28774, 29405, 30048, 30706,
		31379, 32066, 32767};
	int32_t L_x = va_L_mult(fraction, 32);
	int16_t i = va_extract_h(L_x);
	L_x = va_L_shr(L_x, 1);
	int16_t a = (int16_t) (va_extract_l(L_x) & 0x7fff);
	L_x = va_L_deposit_h(tab[i]);
	int16_t tmp = va_sub(tab[i], tab[i + 1]);
	L_x = va_L_msu(L_x, tmp, a);
	return va_L_shr_r(L_x, va_sub(30, exponent));
}

/* ---- vad2.c ----------------------------------------------------------- */
VA_FN int16_t va_fn10Log10(int32_t L_Input, int16_t fbits)	/* vad2.c:104 */
{
	int16_t integer, fraction;
	va_Log2(L_Input, &integer, &fraction);
	integer = va_sub(integer, fbits);
	int32_t Ltmp = va_Mpy_32_16(integer, fraction, 24660);
	Ltmp = va_L_shr_r(Ltmp, 5 + 1);
	return va_extract_l(Ltmp);
}

VA_FN int16_t va_block_norm(const int16_t *in, int16_t *out, int16_t length, int16_t headroom)
{	/* vad2.c:165 */
	int16_t max = va_abs_s(in[0]);
	for (int i = 1; i < length; i++) {
		int16_t ad = va_abs_s(in[i]);
		if (va_sub(ad, max) > 0)
			max = ad;
	}
	int16_t scnt;
	if (max != 0) {
		scnt = va_sub(va_norm_s(max), headroom);
		for (int i = 0; i < length; i++)
			out[i] = va_shl(in[i], scnt);
	} else {
		scnt = va_sub(16, headroom);
		for (int i = 0; i < length; i++)
			out[i] = 0;
	}
	return scnt;
}

/* r_fft.c: 64-point complex FFT of the packed 128-sample real frame
 * (c_fft, bit reversal then 6 radix-2 stages with per-stage >>1), then the
 * real-FFT split (r_fft) */
VA_FN void va_r_fft(int16_t *x)
{
	static const int16_t phs[128] = {
		32767, 0, 32729, -1608, 32610, -3212, 32413, -4808,
		32138, -6393, 31786, -7962, 31357, -9512, 30853, -11039,
		30274, -12540, 29622, -14010, 28899, -15447, 28106, -16846,
		27246, -18205, 26320, -19520, 25330, -20788, 24279, -22006,
		23170, -23170, 22006, -24279, 20788, -25330, 19520, -26320,
		18205, -27246, 16846, -28106, 15447, -28899, 14010, -29622,
		12540, -30274, 11039, -30853, 9512, -31357, 7962, -31786,
		6393, -32138, 4808, -32413, 3212, -32610, 1608, -32729,
		0, -32768, -1608, -32729, -3212, -32610, -4808, -32413,
		-6393, -32138, -7962, -31786, -9512, -31357, -11039, -30853,
		-12540, -30274, -14010, -29622, -15447, -28899, -16846, -28106,
		-18205, -27246, -19520, -26320, -20788, -25330, -22006, -24279,
		-23170, -23170, -24279, -22006, -25330, -20788, -26320, -19520,
		-27246, -18205, -28106, -16846, -28899, -15447, -29622, -14010,
		-30274, -12540, -30853, -11039, -31357, -9512, -31786, -7962,
		-32138, -6393, -32413, -4808, -32610, -3212, -32729, -1608};
	const int SIZE = 128;
	/* c_fft: bit reversal over complex pairs */
	for (int i = 0, j = 0; i < SIZE - 2; i += 2) {
		if (j > i) {
			int16_t t = x[i];
			x[i] = x[j];
			x[j] = t;
			t = x[i + 1];
			x[i + 1] = x[j + 1];
			x[j + 1] = t;
		}
		int k = SIZE / 2;
		while (j >= k) {
			j -= k;
			k >>= 1;
		}
		j += k;
	}
	for (int st = 0; st < 6; st++) {
		int jj = 2 << st, kk = jj << 1, ii2 = (SIZE / 2 >> st) << 1;
		int ji = 0;
		for (int j = 0; j < jj; j += 2) {
			for (int k = j; k < SIZE; k += kk) {
				int kj = k + jj;
				int32_t fr = va_L_mult(x[kj], phs[ji]);
				fr = va_L_msu(fr, x[kj + 1], phs[ji + 1]);
				int32_t fi = va_L_mult(x[kj + 1], phs[ji]);
				fi = va_L_mac(fi, x[kj], phs[ji + 1]);
				int16_t t1 = va_round(fr), t2 = va_round(fi);
				x[kj] = va_shr(va_sub(x[k], t1), 1);
				x[kj + 1] = va_shr(va_sub(x[k + 1], t2), 1);
				x[k] = va_shr(va_add(x[k], t1), 1);
				x[k + 1] = va_shr(va_add(x[k + 1], t2), 1);
			}
			ji += ii2;
		}
	}
	/* r_fft: DC / foldover, then the remaining positive frequencies */
	int16_t r1 = x[0], r2 = x[1];
	x[0] = va_add(r1, r2);
	x[1] = va_sub(r1, r2);
	for (int i = 2, j = SIZE - 2; i <= SIZE / 2; i += 2, j = SIZE - i) {
		int16_t f1r = va_add(x[i], x[j]);
		int16_t f1i = va_sub(x[i + 1], x[j + 1]);
		int16_t f2r = va_add(x[i + 1], x[j + 1]);
		int16_t f2i = va_sub(x[j], x[i]);
		int32_t L1r = va_L_deposit_h(f1r), L1i = va_L_deposit_h(f1i), L;
		L = va_L_mac(L1r, f2r, phs[i]);
		L = va_L_msu(L, f2i, phs[i + 1]);
		x[i] = va_round(va_L_shr(L, 1));
		L = va_L_mac(L1i, f2i, phs[i]);
		L = va_L_mac(L, f2r, phs[i + 1]);
		x[i + 1] = va_round(va_L_shr(L, 1));
		L = va_L_mac(L1r, f2r, phs[j]);
		L = va_L_mac(L, f2i, phs[j + 1]);
		x[j] = va_round(va_L_shr(L, 1));
		L = va_L_negate(L1i);
		L = va_L_msu(L, f2i, phs[j]);
		L = va_L_mac(L, f2r, phs[j + 1]);
		x[j + 1] = va_round(va_L_shr(L, 1));
	}
}

/* vad2() (vad/vad2.c:203-820): one 80-sample frame, returns VAD(m) */
VA_FN int16_t va_vad2(const int16_t *farray, VadState *st)
{
	static const int8_t ch_tbl[VA_NUM_CHAN][2] = {
		{2, 3}, {4, 5}, {6, 7}, {8, 9}, {10, 11}, {12, 13}, {14, 16}, {17, 19},
		{20, 22}, {23, 26}, {27, 30}, {31, 35}, {36, 41}, {42, 48}, {49, 55}, {56, 63}};
	static const int16_t ch_tbl_sh[VA_NUM_CHAN] = {
		16384, 16384, 16384, 16384, 16384, 16384, 10923, 10923,
		10923, 8192, 8192, 6554, 5461, 4681, 4681, 4096};
	static const int8_t vm_tbl[90] = {
		2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2,
		3, 3, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 7, 7, 7,
		8, 8, 9, 9, 10, 10, 11, 12, 12, 13, 13, 14, 15,
		15, 16, 17, 17, 18, 19, 20, 20, 21, 22, 23, 24,
		24, 25, 26, 27, 28, 28, 29, 30, 31, 32, 33, 34,
		35, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45,
		46, 47, 48, 49, 50, 50, 50, 50, 50, 50, 50, 50,
		50, 50};
	static const int8_t hangover_table[20] = {
		30, 30, 30, 30, 30, 30, 28, 26, 24, 22, 20, 18, 16, 14, 12, 10, 8, 8, 8, 8};
	static const int8_t burstcount_table[20] = {
		8, 8, 8, 8, 8, 8, 8, 8, 7, 6, 5, 4, 4, 4, 4, 4, 4, 4, 4, 4};
	static const int16_t vm_threshold_table[20] = {
		34, 34, 34, 34, 34, 34, 34, 34, 34, 34, 34, 40, 51, 71, 100, 139, 191, 257, 337, 432};
	/* per shift_state: noise floor, min channel energy, initial noise,
	 * fractional bits, state-change shift, energy norm shift (vad2.c:305-313) */
	const int16_t noise_floor_chan[2] = {512, 16}, min_chan_enrg[2] = {32, 1},
		      ine_noise[2] = {8192, 256}, fbits[2] = {9, 4},
		      state_change_shift_r[2] = {4 - 9, 9 - 4}, enrg_norm_shift[2] = {9 - 1 + 2, 4 - 1 + 2};
	const int16_t PRE_EMP_FAC = -26214, CEE_SM_FAC = 18022, ONE_MINUS_CEE_SM_FAC = 14746,
		      CNE_SM_FAC = 3277, ONE_MINUS_CNE_SM_FAC = 29491, HIGH_ALPHA = 29491,
		      LOW_ALPHA = 22938, ALPHA_RANGE = 29491 - 22938, DEV_THLD = 7168;

	int16_t input_buffer[VA_FRM_LEN], data_buffer[VA_FFT_LEN];
	int16_t ch_snr[VA_NUM_CHAN], ch_enrg_db[VA_NUM_CHAN];
	int16_t alpha, one_m_alpha, tmp, hi1, lo1, xt, ivad;
	int32_t Ltmp, Ltmp1, Ltmp2;

	st->Lframe_cnt = va_L_add(st->Lframe_cnt, 1);
	int16_t normb_shift = va_block_norm(farray, input_buffer, VA_FRM_LEN, 2);

	for (int i = 0; i < VA_DELAY; i++)
		data_buffer[i] = 0;
	st->pre_emp_mem = va_shr_r(st->pre_emp_mem, va_sub(st->last_normb_shift, normb_shift));
	st->last_normb_shift = normb_shift;
	data_buffer[VA_DELAY] = va_add(input_buffer[0], va_mult(PRE_EMP_FAC, st->pre_emp_mem));
	for (int i = VA_DELAY + 1, j = 1; i < VA_DELAY + VA_FRM_LEN; i++, j++)
		data_buffer[i] = va_add(input_buffer[j], va_mult(PRE_EMP_FAC, input_buffer[j - 1]));
	st->pre_emp_mem = input_buffer[VA_FRM_LEN - 1];
	for (int i = VA_DELAY + VA_FRM_LEN; i < VA_FFT_LEN; i++)
		data_buffer[i] = 0;

	va_r_fft(data_buffer);

	int state_change = 0;
	if (st->shift_state == 0) {
		if (va_sub(normb_shift, -2 + 2) <= 0) {
			state_change = 1;
			st->shift_state = 1;
		}
	} else {
		if (va_sub(normb_shift, -2 + 5) >= 0) {
			state_change = 1;
			st->shift_state = 0;
		}
	}
	const int ss = st->shift_state;
	if (state_change)
		for (int i = 0; i < VA_NUM_CHAN; i++)
			st->Lch_enrg[i] = va_L_shr(st->Lch_enrg[i], state_change_shift_r[ss]);

	if (va_L_sub(st->Lframe_cnt, 1) == 0) {
		alpha = 32767;
		one_m_alpha = 0;
	} else {
		alpha = CEE_SM_FAC;
		one_m_alpha = ONE_MINUS_CEE_SM_FAC;
	}
	for (int i = 0; i < VA_NUM_CHAN; i++) {
		int32_t Lenrg = 0;
		for (int j = ch_tbl[i][0]; j <= ch_tbl[i][1]; j++) {
			Lenrg = va_L_mac(Lenrg, data_buffer[2 * j], data_buffer[2 * j]);
			Lenrg = va_L_mac(Lenrg, data_buffer[2 * j + 1], data_buffer[2 * j + 1]);
		}
		Lenrg = va_L_shr_r(Lenrg, va_sub(va_shl(normb_shift, 1), enrg_norm_shift[ss]));
		tmp = va_mult(alpha, ch_tbl_sh[i]);
		va_L_Extract(Lenrg, &hi1, &lo1);
		Ltmp = va_Mpy_32_16(hi1, lo1, tmp);
		va_L_Extract(st->Lch_enrg[i], &hi1, &lo1);
		st->Lch_enrg[i] = va_L_add(Ltmp, va_Mpy_32_16(hi1, lo1, one_m_alpha));
		if (va_L_sub(st->Lch_enrg[i], min_chan_enrg[ss]) < 0)
			st->Lch_enrg[i] = min_chan_enrg[ss];
	}

	int32_t Ltce = 0;
	for (int i = 0; i < VA_NUM_CHAN; i++)
		Ltce = va_L_add(Ltce, st->Lch_enrg[i]);

	int32_t Lpeak = 0;
	for (int i = 2; i < VA_NUM_CHAN; i++)
		if (va_L_sub(st->Lch_enrg[i], Lpeak) > 0)
			Lpeak = st->Lch_enrg[i];
	va_L_Extract(Ltce, &hi1, &lo1);
	Ltmp = va_Mpy_32_16(hi1, lo1, 20480);
	int p2a_flag = va_L_sub(Lpeak, Ltmp) > 0;

	if (va_L_sub(st->Lframe_cnt, 4) <= 0) {
		if (p2a_flag) {
			for (int i = 0; i < VA_NUM_CHAN; i++)
				st->Lch_noise[i] = 8192;
		} else {
			for (int i = 0; i < VA_NUM_CHAN; i++) {
				if (va_L_sub(st->Lch_enrg[i], ine_noise[ss]) < 0)
					st->Lch_noise[i] = 8192;
				else if (ss == 1)
					st->Lch_noise[i] = va_L_shr(st->Lch_enrg[i], state_change_shift_r[0]);
				else
					st->Lch_noise[i] = st->Lch_enrg[i];
			}
		}
	}

	int16_t vm_sum = 0;
	for (int i = 0; i < VA_NUM_CHAN; i++) {
		ch_enrg_db[i] = va_fn10Log10(st->Lch_enrg[i], fbits[ss]);
		int16_t ch_noise_db = va_fn10Log10(st->Lch_noise[i], 9);
		ch_snr[i] = va_sub(ch_enrg_db[i], ch_noise_db);
		int16_t ch_snrq = va_shr_r(va_mult(21845, ch_snr[i]), 6);
		int j = va_sub(ch_snrq, 89) < 0 ? (ch_snrq > 0 ? ch_snrq : 0) : 89;
		vm_sum = va_add(vm_sum, vm_tbl[j]);
	}

	if (va_L_sub(st->Lframe_cnt, 4) <= 0 || st->fupdate_flag == 1) {
		int16_t tce_db = 14320;
		st->negSNRvar = 0;
		st->negSNRbias = 0;
		int32_t Ltne = 0;
		for (int i = 0; i < VA_NUM_CHAN; i++)
			Ltne = va_L_add(Ltne, st->Lch_noise[i]);
		int16_t tne_db = va_fn10Log10(Ltne, 9);
		xt = va_sub(tce_db, tne_db);
		st->tsnr = xt;
	} else {
		Ltmp1 = 0;
		for (int i = 0; i < VA_NUM_CHAN; i++) {
			Ltmp2 = va_L_shr(va_L_mult(ch_snr[i], 10885), 8);
			va_L_Extract(Ltmp2, &hi1, &lo1);
			hi1 = va_add(hi1, 3);
			Ltmp1 = va_L_add(Ltmp1, va_Pow2(hi1, lo1));
		}
		xt = va_fn10Log10(Ltmp1, 4 + 3);
		if (va_sub(xt, st->tsnr) > 0)
			st->tsnr = va_round(va_L_add(va_L_mult(29491, st->tsnr), va_L_mult(3277, xt)));
		else if (va_sub(xt, va_mult(20480, st->tsnr)) > 0)
			st->tsnr = va_round(va_L_add(va_L_mult(32702, st->tsnr), va_L_mult(66, xt)));
	}

	int16_t tsnrq = va_shr(va_mult(st->tsnr, 10923), 8);
	if (va_sub(tsnrq, 19) > 0)
		tsnrq = 19;
	else if (tsnrq < 0)
		tsnrq = 0;

	if (xt < 0) {
		tmp = va_round(va_L_shl(va_L_mult(xt, xt), 7));
		st->negSNRvar = va_round(va_L_add(va_L_mult(32440, st->negSNRvar), va_L_mult(328, tmp)));
		if (va_sub(st->negSNRvar, 1024) > 0)
			st->negSNRvar = 1024;
		tmp = va_mult_r(va_shl(va_sub(st->negSNRvar, 166), 4), 24576);
		st->negSNRbias = tmp < 0 ? (int16_t) 0 : va_shr(tmp, 8);
	}

	tmp = va_add(vm_threshold_table[tsnrq], st->negSNRbias);
	if (va_sub(vm_sum, tmp) > 0) {
		ivad = 1;
		st->burstcount = va_add(st->burstcount, 1);
		if (va_sub(st->burstcount, burstcount_table[tsnrq]) > 0)
			st->hangover = hangover_table[tsnrq];
	} else {
		st->burstcount = 0;
		st->hangover = va_sub(st->hangover, 1);
		if (st->hangover <= 0) {
			ivad = 0;
			st->hangover = 0;
		} else {
			ivad = 1;
		}
	}

	int16_t ch_enrg_dev = 0;
	if (va_L_sub(st->Lframe_cnt, 1) == 0) {
		for (int i = 0; i < VA_NUM_CHAN; i++)
			st->ch_enrg_long_db[i] = ch_enrg_db[i];
	} else {
		for (int i = 0; i < VA_NUM_CHAN; i++)
			ch_enrg_dev = va_add(ch_enrg_dev,
					     va_abs_s(va_sub(st->ch_enrg_long_db[i], ch_enrg_db[i])));
	}

	tmp = va_sub(st->tsnr, xt);
	if (tmp <= 0 || st->tsnr <= 0) {
		alpha = HIGH_ALPHA;
		one_m_alpha = (int16_t) (32768 - HIGH_ALPHA);
	} else if (va_sub(tmp, st->tsnr) > 0) {
		alpha = LOW_ALPHA;
		one_m_alpha = (int16_t) (32768 - LOW_ALPHA);
	} else {
		tmp = va_div_s(tmp, st->tsnr);
		alpha = va_sub(HIGH_ALPHA, va_mult(ALPHA_RANGE, tmp));
		one_m_alpha = va_sub(32767, alpha);
	}
	for (int i = 0; i < VA_NUM_CHAN; i++) {
		Ltmp1 = va_L_mult(one_m_alpha, ch_enrg_db[i]);
		Ltmp2 = va_L_mult(alpha, st->ch_enrg_long_db[i]);
		st->ch_enrg_long_db[i] = va_round(va_L_add(Ltmp1, Ltmp2));
	}

	int update_flag = 0;
	st->fupdate_flag = 0;
	if (va_sub(vm_sum, 35) <= 0) {
		if (st->burstcount == 0) {
			update_flag = 1;
			st->update_cnt = 0;
		}
	} else if (va_L_sub(Ltce, noise_floor_chan[ss]) > 0) {
		if (va_sub(ch_enrg_dev, DEV_THLD) < 0 && !p2a_flag && st->LTP_flag == 0) {
			st->update_cnt = va_add(st->update_cnt, 1);
			if (va_sub(st->update_cnt, 50) >= 0) {
				update_flag = 1;
				st->fupdate_flag = 1;
			}
		}
	}
	if (va_sub(st->update_cnt, st->last_update_cnt) == 0)
		st->hyster_cnt = va_add(st->hyster_cnt, 1);
	else
		st->hyster_cnt = 0;
	st->last_update_cnt = st->update_cnt;
	if (va_sub(st->hyster_cnt, 6) > 0)
		st->update_cnt = 0;

	if (update_flag) {
		tmp = ss == 1 ? state_change_shift_r[0] : (int16_t) 0;
		for (int i = 0; i < VA_NUM_CHAN; i++) {
			va_L_Extract(va_L_shr(st->Lch_enrg[i], tmp), &hi1, &lo1);
			Ltmp = va_Mpy_32_16(hi1, lo1, CNE_SM_FAC);
			va_L_Extract(st->Lch_noise[i], &hi1, &lo1);
			st->Lch_noise[i] = va_L_add(Ltmp, va_Mpy_32_16(hi1, lo1, ONE_MINUS_CNE_SM_FAC));
			if (va_L_sub(st->Lch_noise[i], 32) < 0)
				st->Lch_noise[i] = 32;
		}
	}
	return ivad;
}

/* the six vad2 windows of one 540-sample superframe (tx.c:234-239,
 * melpe_enc.c:48-53): offsets 10, 100, ..., 460; returns the sum of the six
 * decisions (0 = the superframe is silence) */
VA_FN int va_superframe(const int16_t *sp, VadState *st)
{
	int n = 0;
	for (int k = 0; k < 6; k++)
		n += va_vad2(sp + 10 + 90 * k, st);
	return n;
}

#endif
