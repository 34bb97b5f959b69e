/*
 * k_npp.hip -- the noise pre-processor kernels: melpe_n on F frames per
 * channel (melpe/melpe.c:63-67) and the NPP half of melpe_a (three npp()
 * calls on the superframe, melpe/melpe.c:94-96), one lane per channel, in
 * place on the caller's PCM.
 */
#include "kern.h"

MELPE_TU(npp)

struct NppLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	NppScratch w;
	NppState S;
	int16_t x[BLOCK + NPP_OVL];
};

/* melpe_n on `frames` frames per channel; channel c's samples at
 * sp[c*stride ...], the first call of a channel reads 256 samples */
__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_npp(EncState *enc, int16_t *sp, int frames, int stride,
					      const uint8_t *active, int n, int rate1200)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || (active && !active[c]))
		return;
	NppLane L;
	PIN_FRAME(L);
	lane_copy(&L.S, &enc[c].npp, sizeof(NppState));
	int16_t *x = sp + (size_t) c * stride;
	for (int f = 0; f < frames; f++) {
		/* frame f plus the look-ahead the first call reads */
		int m = stride - f * NPP_HOP;
		m = m < NPP_WIN ? m : NPP_WIN;
		for (int i = 0; i < NPP_WIN; i++)
			L.x[i] = i < m ? x[f * NPP_HOP + i] : (int16_t) 0;
		npp_frame(&L.S, &L.w, L.x, L.x, rate1200 != 0);
		for (int i = 0; i < NPP_HOP; i++)
			x[f * NPP_HOP + i] = L.x[i];
	}
	lane_copy(&enc[c].npp, &L.S, sizeof(NppState));
}

/* the NPP part of melpe_a: frames 0..2 of every active channel's 540-sample
 * superframe, in place */
__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_enc_npp(EncState *enc, int16_t *sp, const uint8_t *active,
						  int n)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || (active && !active[c]))
		return;
	NppLane L;
	PIN_FRAME(L);
	lane_copy(&L.S, &enc[c].npp, sizeof(NppState));
	int16_t *x = sp + (size_t) c * BLOCK;
	lane_copy(L.x, x, sizeof(int16_t) * BLOCK);
	npp_frame(&L.S, &L.w, L.x, L.x);
	npp_frame(&L.S, &L.w, L.x + FRAME, L.x + FRAME);
	npp_frame(&L.S, &L.w, L.x + 2 * FRAME, L.x + 2 * FRAME);
	lane_copy(x, L.x, sizeof(int16_t) * BLOCK);
	lane_copy(&enc[c].npp, &L.S, sizeof(NppState));
}

extern "C" int kl_npp(EncState *enc, int16_t *sp, int frames, int stride, const uint8_t *active,
		      int n, int rate1200, hipStream_t s)
{
	k_npp<<<grid_for(n), WAVE, 0, s>>>(enc, sp, frames, stride, active, n, rate1200);
	return (int) hipGetLastError();
}

extern "C" int kl_enc_npp(EncState *enc, int16_t *sp, const uint8_t *active, int n, hipStream_t s)
{
	k_enc_npp<<<grid_for(n), WAVE, 0, s>>>(enc, sp, active, n);
	return (int) hipGetLastError();
}
