/*
 * k_harm.hip -- the Fourier magnitudes of melpe_a (melpe/melp_ana.c:224-236,
 * find_harm at melpe/fs_lib.c:62) with one WAVEFRONT per channel, and the
 * lane-per-channel tail after them (quant_fsmag, the channel write).
 *
 * In the lane-per-channel analysis each lane ran find_harm's 512-point real
 * FFT alone, 2 KB of private state per channel: 12% of k_enc_ana at
 * 262,144 channels.  Here k_enc_ana stops after writing each voiced frame's
 * windowed residual (analysis_a), k_enc_harm runs the FFT across the 64
 * lanes of a wave in LDS -- the NPP's wave FFT (npp_wave.h wv_cfft256: the
 * same fft_lib.c cfft, same per-stage guard scaling) plus rfft's split and
 * twiddle passes with one step per lane -- and the harmonic peak search, and
 * k_enc_tail packs the superframe (analysis_b).  Every value is the
 * reference's: the passes are the reference's steps, which touch disjoint
 * bins, in its arithmetic.
 */
#include "kern.h"
#include "npp_wave.h"

MELPE_TU(harm)

using namespace mlp::wv;

/* find_harm_fft + find_harm_mag (analysis.h) of one frame, the windowed
 * residual's samples lane + 64 t in v[t] (0 past LPC_FRAME), the result
 * into fsmag[0..10) */
MD void wv_find_harm(const int16_t v[4], int16_t *fsmag, Word16 pitch, uint32_t *x, const WvConst *kc,
		     int lane)
{
	int16_t *d0 = (int16_t *) x;	/* 256 complex points, re / im interleaved */
	/* the input's max |x|, its scale, the packed points zero padded */
	int mx = 0;
#pragma unroll
	for (int t = 0; t < 4; t++)
		mx = max(mx, (int) abs_s(v[t]));
	const Word16 sh = norm_s((Word16) wmax(mx));
#pragma unroll
	for (int t = 0; t < 8; t++) {
		const int i = lane + WV * t;	/* real point i = short i of d0 */
		d0[i] = (t < 4) ? shl(v[t], sh) : (int16_t) 0;
	}
	wsync();
	wv_cfft256(d0, kc, lane);
	/* rfft's guard for the split: max |x| of the FFT's output */
	mx = 0;
#pragma unroll
	for (int t = 0; t < 8; t++)
		mx = max(mx, (int) abs_s(d0[lane + WV * t]));
	const Word16 s = wmax(mx) > 16383 ? 1 : 0;
	/* split steps k = 1..127 (rfft_pk split_step): step k touches x[k],
	 * x[256 - k], x[512 - k], x[256 + k], disjoint across k */
	const int n2 = 256, n = 512;
	for (int k = lane + 1; k < n2 / 2; k += WV) {
		uint32_t A = pk_shr(x[k], s), B = pk_shr(x[n2 - k], s);
		Word16 ar = pk_re(A), ai = pk_im(A), br = pk_re(B), bi = pk_im(B);
		Word16 r1 = add_shr(ar, br);
		Word32 a = L_shl(L_sub(ai, bi), 16);
		Word16 r2 = add_shr(ai, bi);
		Word32 b = L_shl(L_sub(ar, br), 16);
		x[k] = pk(r1, r2);
		x[n2 - k] = pk(r1, r2);
		Word16 bh = extract_h(L_shr(b, 1)), ah = extract_h(L_shr(a, 1));
		b = L_negate(b);
		a = L_negate(a);
		x[n - k] = pk(ah, bh);
		x[n2 + k] = pk(extract_h(L_shr(a, 1)), extract_h(L_shr(b, 1)));
	}
	if (lane == 0) {	/* x[0], x[128], x[256], x[384]: no split step's */
		x[n2 + n2 / 2] = 0;
		x[n2 / 2] = pk_shr(x[n2 / 2], s);
		uint32_t z = pk_shr(x[0], s);
		x[0] = pk(add(pk_re(z), pk_im(z)), 0);
		x[n2] = pk(sub(pk_re(z), pk_im(z)), 0);
	}
	wsync();
	/* twiddle steps k = 1..255 (rfft_pk twid_step): x[k], x[512 - k] */
	const int16_t *wrt = g_der.wr, *wit = g_der.wi;
	for (int k = lane + 1; k < n2; k += WV) {
		uint32_t A = x[k], B = x[n - k];
		Word16 wr = wrt[k], wi = wit[k];
		Word16 a1 = pk_re(A), a2 = pk_im(A), b1 = pk_re(B), b2 = pk_im(B);
		Word32 t = L_deposit_h(a1);
		t = L_add(t, L_mult(a2, wr));
		t = L_add(t, 0x8000);
		t = L_shl(L_shr(t, 16), 16);
		t = L_sub(t, L_mult(b2, wi));
		t = L_add(t, 0x8000);
		Word32 u = L_deposit_h(b1);
		u = L_sub(u, L_mult(a2, wi));
		u = L_add(u, 0x8000);
		u = L_shl(L_shr(u, 16), 16);
		u = L_sub(u, L_mult(b2, wr));
		u = L_add(u, 0x8000);
		x[k] = pk(extract_h(t), extract_h(u));
		x[n - k] = pk(extract_h(t), extract_h(L_negate(u)));
	}
	wsync();
	/* find_harm_mag: harmonic k's peak power on lane k */
	Word16 fw = shr(divide_s(512, pitch), 2);
	Word16 iw = shr(fw, 6);
	Word16 i2 = shr(iw, 1);
	Word16 nh = NUM_HARM, t1 = shr(pitch, 9);
	if (nh > t1)
		nh = t1;
	Word32 Lmax = 0;
	if (lane < nh) {
		Word16 mfw = fw;
		for (int k = 0; k < lane; k++)
			mfw = add(mfw, fw);
		Word16 i0 = sub(shr(add(mfw, 32), 6), i2);
		for (int j = 0; j < iw; j++) {
			Word16 b = add(i0, (Word16) j);
			Word16 re = pk_re(x[b]), im = pk_im(x[b]);
			Word32 t = L_add(L_mult(re, re), L_mult(im, im));
			Lmax = Max_(Lmax, t);
		}
	}
	/* avg = 1 + the Lm: at most ten terms below 2^31, so the reference's
	 * 40-bit chain cannot clamp and its order is free */
	Word40 avg = 1;
	for (int k = 0; k < nh; k++)
		avg += (Word40) __shfl(Lmax, k);
	t1 = norm32(avg);
	Word32 Lt = (Word32) L40_shl(avg, t1);
	t1 = sub(31, t1);
	Word16 t2 = divide_s(shl(nh, 10), extract_h(Lt));
	Word16 sh2 = sub(30, t1);
	if (lane < NUM_HARM) {
		Word16 f = 8192;
		if (lane < nh) {
			Word16 q = extract_h(L_shl(Lmax, sh2));
			q = extract_h(L_shl(L_mult(q, t2), 2));
			f = sqrt_Q15(q);
		}
		fsmag[lane] = f;
	}
	wsync();
}

/* the windowed residuals k_enc_ana (mode 1) left in res */
/* one wave per live channel: slot g runs channel perm[g] (the engine's
 * lane order) or channel g under the mask; the three frames in order */
__global__ __launch_bounds__(WAVE) void k_enc_harm(EncState *enc, const int16_t *res,
						   const uint8_t *active, int n, const int *perm,
						   const int *nlive, AnaGate gate)
{
	int c = blockIdx.x;
	if (perm) {
		const int L = *nlive;
		if (!gate.open(L) || c >= L)
			return;
		c = perm[c];
	} else if (c >= n || (active && !active[c])) {
		return;
	}
	const int lane = threadIdx.x;
	__shared__ uint32_t x[512];
	WvConst kc;
	wv_const_init(&kc, lane);
	for (int i = 0; i < NF; i++) {
		MelpParam *par = &enc[c].a.par[i];
		const Word16 uv = par->uv_flag, pitch = par->pitch;
		if (uv) {	/* ana_fsmag_frame: 8192s, no FFT */
			if (lane < NUM_HARM)
				par->fs_mag[lane] = 8192;
			continue;
		}
		int16_t v[4];
		const int16_t *w = res + ((size_t) c * NF + i) * LPC_FRAME;
#pragma unroll
		for (int t = 0; t < 4; t++) {
			const int k = lane + WV * t;
			v[t] = k < LPC_FRAME ? w[k] : (int16_t) 0;
		}
		wv_find_harm(v, par->fs_mag, pitch, x, &kc, lane);
	}
}

extern "C" int kl_enc_harm(EncState *enc, const int16_t *res, const uint8_t *active, int n,
			   const int *perm, const int *nlive, AnaGate gate, hipStream_t s)
{
	k_enc_harm<<<n, WAVE, 0, s>>>(enc, res, active, n, perm, nlive, gate);
	return (int) hipGetLastError();
}

/* the superframe's packing after the magnitudes (analysis_b), lane per
 * channel, on the part of the record it reads and writes */
struct TailLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	EncAna S;
};

__global__ __launch_bounds__(WAVE, 4) void k_enc_tail(EncState *enc, uint8_t *bits, const uint8_t *active,
						   int n, const int *perm, const int *nlive, AnaGate gate)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (perm) {
		const int L = *nlive;
		if (!gate.open(L) || c >= L)
			return;
		c = perm[c];
	} else if (c >= n || (active && !active[c])) {
		return;
	}
	TailLane L;
	PIN_FRAME(L);
	/* par + qpar, and fsm_prev_uv .. chbuf, widened to dwords (the extra
	 * int16 at either end goes back unchanged) */
	constexpr size_t o = offsetof(EncAna, par), e = offsetof(EncAna, voicedEn);
	constexpr size_t o2 = offsetof(EncAna, fsm_prev_uv) & ~(size_t) 3;
	constexpr size_t e2 = (offsetof(EncAna, top_lpc) + 3) & ~(size_t) 3;
	static_assert(o % 4 == 0 && e % 4 == 0, "the tail's record ranges are dword copies");
	EncAna *R = &enc[c].a;
	lane_copy((char *) &L.S + o, (const char *) R + o, e - o);
	lane_copy((char *) &L.S + o2, (const char *) R + o2, e2 - o2);
	analysis_b(&L.S);
	lane_copy((char *) R + o, (const char *) &L.S + o, e - o);
	lane_copy((char *) R + o2, (const char *) &L.S + o2, e2 - o2);
	for (int k = 0; k < 11; k++)
		bits[(size_t) c * 11 + k] = L.S.chbuf[k];
}

extern "C" int kl_enc_tail(EncState *enc, uint8_t *bits, const uint8_t *active, int n,
			   const int *perm, const int *nlive, AnaGate gate, hipStream_t s)
{
	k_enc_tail<<<grid_for(n), WAVE, 0, s>>>(enc, bits, active, n, perm, nlive, gate);
	return (int) hipGetLastError();
}

extern "C" size_t kl_harm_private(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *) k_enc_tail) == hipSuccess ? a.localSizeBytes : 0;
}

/* private-segment bytes per lane of k_enc_harm (one wave per channel) */
extern "C" size_t kl_harm_wave_private(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *) k_enc_harm) == hipSuccess ? a.localSizeBytes : 0;
}

extern "C" int kl_harm_warm(int n, hipStream_t s)
{
	k_enc_harm<<<n, WAVE, 0, s>>>(nullptr, nullptr, nullptr, 0, nullptr, nullptr, AnaGate{});
	k_enc_tail<<<grid_for(n), WAVE, 0, s>>>(nullptr, nullptr, nullptr, 0, nullptr, nullptr, AnaGate{});
	return (int) hipGetLastError();
}
