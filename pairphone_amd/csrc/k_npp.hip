/*
 * k_npp.hip -- the noise pre-processor kernels: melpe_n on F frames per
 * channel (melpe/melpe.c:63-67) and the NPP half of melpe_a (three npp()
 * calls on the superframe, melpe/melpe.c:94-96), in place on the caller's
 * PCM.  One wavefront (one 64-thread workgroup) per channel, the channel's
 * NPP state and frame scratch in LDS (npp_wave.h).
 */
/* Channels (one wave each) per workgroup, and the fixed-point math tables'
 * LDS copy (dsp.h MELPE_MATH_LDS): with one channel per workgroup each
 * wave has its own copy (8,690 B of channel image + 1,052 B of tables: 16
 * waves per CU).  Measured: 8 channels per workgroup sharing one copy lost
 * 0.4 ms against one (whole-workgroup dispatch), and without the tables
 * the per-bin log / pow lookups cost 0.5 ms more (profiles/r06_*_npp*). */
#ifndef MELPE_NPP_WG_WAVES
#define MELPE_NPP_WG_WAVES 1
#endif
#ifndef MELPE_NPP_MATH_LDS
#define MELPE_NPP_MATH_LDS 1
#endif
#if MELPE_NPP_MATH_LDS
#define MELPE_MATH_LDS
#endif
#include "kern.h"
#include "npp_wave.h"

MELPE_TU(npp)

#define NPP_WG (WAVE * MELPE_NPP_WG_WAVES)
#if MELPE_NPP_MATH_LDS
static_assert((160 * 1024 / (MELPE_NPP_WG_WAVES * sizeof(mlp::wv::NppWave) + MTAB_WORDS * sizeof(int16_t))) *
			      MELPE_NPP_WG_WAVES >= 16,
	      "16 NPP waves per CU (the register budget's four per SIMD)");
#define NPP_LDS_DYN (MTAB_WORDS * sizeof(int16_t))
/* every wave of the workgroup helps fill the table, before any returns */
#define NPP_TABLES_IN()                                                        \
	do {                                                                   \
		for (int i_ = threadIdx.x; i_ < MTAB_WORDS; i_ += blockDim.x) \
			s_mtab[i_] = g_tab[mtab_src(i_)];                     \
		__syncthreads();                                               \
	} while (0)
#else
#define NPP_LDS_DYN 0
#define NPP_TABLES_IN() (void) 0
#endif

/* waves per SIMD the NPP kernels are compiled for: the LDS image
 * (NppWave, 9,980 B) lets 16 waves share a CU, and 4 per SIMD caps the
 * registers at 128 */
#ifndef NPP_WAVES_PER_EU
#define NPP_WAVES_PER_EU 4
#endif
#define NPP_WPE __attribute__((amdgpu_waves_per_eu(NPP_WAVES_PER_EU)))

using namespace mlp::wv;

/* melpe_n on `frames` frames per channel; channel c's samples at
 * sp[c*stride ...]; the first call of a channel reads 256 samples (or what
 * the row holds, zero-extended) */
__global__ __launch_bounds__(NPP_WG) NPP_WPE void k_npp(EncState *enc, int16_t *sp, int frames, int stride,
					      const uint8_t *active, int n, int rate1200)
{
	__shared__ NppWave Ws[MELPE_NPP_WG_WAVES];
	NPP_TABLES_IN();
	/* the wave's channel, wave-uniform (readfirstlane: the compiler does
	 * not know threadIdx.x / 64 is), so its record and sample addresses
	 * stay scalar */
	const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = threadIdx.x % WAVE;
	const int c = blockIdx.x * MELPE_NPP_WG_WAVES + w;
	if (c >= n || (active && !active[c]))
		return;
	NppWave &W = Ws[w];
	WvConst kc;
	wv_const_init(&kc, lane);
	wv_state_in(&W, &enc[c].npp, lane);
	int16_t *x = sp + (size_t) c * stride;
	for (int f = 0; f < frames; f++)
		wv_npp_frame(&W, &enc[c].npp, x + f * NPP_HOP, stride - f * NPP_HOP, rate1200 != 0, &kc, lane);
	wv_state_out(&enc[c].npp, &W, lane);
}

/* the NPP part of melpe_a: frames 0..2 of every active channel's 540-sample
 * superframe, in place */
__global__ __launch_bounds__(NPP_WG) NPP_WPE void k_enc_npp(EncState *enc, int16_t *sp, const uint8_t *active,
						  int n)
{
	__shared__ NppWave Ws[MELPE_NPP_WG_WAVES];
	NPP_TABLES_IN();
	/* the wave's channel, wave-uniform (readfirstlane: the compiler does
	 * not know threadIdx.x / 64 is), so its record and sample addresses
	 * stay scalar */
	const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = threadIdx.x % WAVE;
	const int c = blockIdx.x * MELPE_NPP_WG_WAVES + w;
	if (c >= n || (active && !active[c]))
		return;
	NppWave &W = Ws[w];
	WvConst kc;
	wv_const_init(&kc, lane);
	wv_state_in(&W, &enc[c].npp, lane);
	int16_t *x = sp + (size_t) c * BLOCK;
	for (int f = 0; f < NF; f++)
		wv_npp_frame(&W, &enc[c].npp, x + f * FRAME, BLOCK - f * FRAME, true, &kc, lane);
	wv_state_out(&enc[c].npp, &W, lane);
}

static unsigned npp_grid(int n)
{
	return (unsigned) ((n + MELPE_NPP_WG_WAVES - 1) / MELPE_NPP_WG_WAVES);
}

extern "C" int kl_npp(EncState *enc, int16_t *sp, int frames, int stride, const uint8_t *active,
		      int n, int rate1200, hipStream_t s)
{
	k_npp<<<npp_grid(n), NPP_WG, NPP_LDS_DYN, s>>>(enc, sp, frames, stride, active, n, rate1200);
	return (int) hipGetLastError();
}

extern "C" int kl_enc_npp(EncState *enc, int16_t *sp, const uint8_t *active, int n, hipStream_t s)
{
	k_enc_npp<<<npp_grid(n), NPP_WG, NPP_LDS_DYN, s>>>(enc, sp, active, n);
	return (int) hipGetLastError();
}

/* private-segment bytes per lane of the wave-per-channel NPP kernels
 * (engine.hip engine_reserve) */
extern "C" size_t kl_npp_private(void)
{
	hipFuncAttributes a, b;
	size_t x = hipFuncGetAttributes(&a, (const void *) k_enc_npp) == hipSuccess ? a.localSizeBytes : 0;
	size_t y = hipFuncGetAttributes(&b, (const void *) k_npp) == hipSuccess ? b.localSizeBytes : 0;
	return x > y ? x : y;
}

extern "C" int kl_npp_warm(int n, hipStream_t s)
{
	k_enc_npp<<<npp_grid(n), NPP_WG, NPP_LDS_DYN, s>>>(nullptr, nullptr, nullptr, 0);
	return (int) hipGetLastError();
}
