/*
 * k_ana.hip -- the analysis half of melpe_a (melpe/melpe.c:97-98:
 * analysis() + the 11-byte frame): dc removal, melp_ana per frame, sc_ana,
 * the quantisers and channel packing, one lane per channel, reading the
 * NPP output k_enc_npp left in the caller's PCM.
 */
#include <stdlib.h>
#define MELPE_PROG_PRIO	/* progprio.h: ANA_CKPT */
#include "kern.h"

MELPE_TU(ana)

/* the lane's frame: the analysis state only (not the NPP state), whose
 * live prefix moves in and out (state.h ENC_ANA_LIVE), and the PCM block */
struct AnaLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	EncAna S;
	int16_t x[BLOCK];
};

/* MODE 0: the whole analysis and the bits here (MELPE_HARM=0).
 * MODE 1: the split form (encoder.h analysis_a): the windowed residuals to
 *         res (NF x LPC_FRAME per channel), the Fourier magnitudes and the
 *         packing in k_harm.hip. */
#if defined(MELPE_WAVE_TIMES)
/* diagnostics (tools/wave_times.py): each wave's start and end on the
 * chip-wide 100 MHz counter, to see how the launch's waves finish */
__device__ unsigned long long g_wave_t[2 * 16384];
/* the wave's placement: HW_ID (wave, SIMD, CU, SH, SE) and XCC_ID */
__device__ unsigned g_wave_hw[2 * 16384];
extern "C" int kl_wave_times(unsigned long long *out, int n)
{
	return (int) hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_t), sizeof(unsigned long long) * n);
}
extern "C" int kl_wave_hw(unsigned *out, int n)
{
	return (int) hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_hw), sizeof(unsigned) * n);
}
#define WT_START() const unsigned long long wt0_ = __builtin_amdgcn_s_memrealtime()
#define WT_END()                                                                         \
	do {                                                                             \
		if (threadIdx.x == 0 && blockIdx.x < 16384) {                            \
			g_wave_t[2 * blockIdx.x] = wt0_;                                 \
			g_wave_t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime(); \
			g_wave_hw[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  \
			g_wave_hw[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20); \
		}                                                                        \
	} while (0)
#else
#define WT_START() (void) 0
#define WT_END() (void) 0
#endif

template <int MODE>
__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_enc_ana(EncState *enc, const int16_t *sp, uint8_t *bits,
						  const uint8_t *active, int n, const int *perm,
						  const int *nlive, int16_t *res, AnaGate gate, int prio)
{
	/* lane g runs channel perm[g] when the engine ordered the live channels
	 * by pitch class (engine.hip, MELPE_BIN), else channel g under the mask;
	 * the whole launch stands down unless the live count is the gate's
	 * (engine.hip ana_launch enqueues this and the four-wave kernel) */
	WT_START();
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (perm) {
		const int L = *nlive;
		if (!gate.open(L))
			return;
		gate.mark(c == 0 && L > 0, 1);	/* no live channel: the tag stays 0 */
		if (c >= L)
			return;
		/* progprio.h: the counter is the sort's control word nlive[2] */
		PP_BEGIN(prio ? (unsigned *) (nlive + 2) : nullptr, (L + WAVE - 1) / WAVE);
		c = perm[c];
	} else {
		PP_BEGIN(nullptr, 1);
		gate.mark(c == 0, 1);
		if (c >= n || (active && !active[c]))
			return;
	}
	AnaLane L;
	PIN_FRAME(L);
	constexpr size_t nb = ENC_ANA_LIVE;
	static_assert(offsetof(AnaLane, S) % 16 == 0, "the record copy is in 16-byte pieces");
	lane_copy_x4(&L.S, &enc[c].a, nb);
	lane_copy(L.x, sp + (size_t) c * BLOCK, sizeof(int16_t) * BLOCK);
	if (MODE == 0)
		analysis(&L.S, L.x);
	else
		analysis_a(&L.S, L.x, res + (size_t) c * NF * LPC_FRAME);
	lane_copy_x4(&enc[c].a, &L.S, nb);
	if (MODE == 0)
		for (int k = 0; k < 11; k++)
			bits[(size_t) c * 11 + k] = L.S.chbuf[k];
	WT_END();
}

/* debug aid: analysis cut after `upto` stages (0 = nothing) */
__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_enc_ana_dbg(EncState *enc, const int16_t *sp, int n, int upto)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	PP_BEGIN(nullptr, 1);
	if (c >= n || upto <= 0)
		return;
	AnaLane L;
	PIN_FRAME(L);
	lane_copy(&L.S, &enc[c].a, ENC_ANA_LIVE);
	lane_copy(L.x, sp + (size_t) c * BLOCK, sizeof(int16_t) * BLOCK);
	analysis_upto(&L.S, L.x, upto);
	lane_copy(&enc[c].a, &L.S, ENC_ANA_LIVE);
}

/* MELPE_ANA_LDS (diagnostic): reserve that many bytes of LDS per wave to cap
 * the resident waves per CU (occupancy experiments) */
static unsigned ana_lds_bytes(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("MELPE_ANA_LDS");
		v = e ? atoi(e) : 0;
	}
	return (unsigned) v;
}

/* MELPE_ANA_PRIO=0: no progress-driven priority (progprio.h), for A/Bs */
static int ana_prio_mode(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("MELPE_ANA_PRIO");
		v = e ? (atoi(e) != 0) : 1;
	}
	return v;
}

extern "C" int kl_enc_ana(EncState *enc, const int16_t *sp, uint8_t *bits, const uint8_t *active,
			  int n, const int *perm, const int *nlive, int16_t *res, AnaGate gate, hipStream_t s)
{
	const int pm = ana_prio_mode();
	if (res)
		k_enc_ana<1><<<grid_for(n), WAVE, ana_lds_bytes(), s>>>(enc, sp, bits, active, n, perm, nlive, res,
									 gate, pm);
	else
		k_enc_ana<0><<<grid_for(n), WAVE, ana_lds_bytes(), s>>>(enc, sp, bits, active, n, perm, nlive, res,
									 gate, pm);
	return (int) hipGetLastError();
}

extern "C" int kl_enc_ana_dbg(EncState *enc, const int16_t *sp, int n, int upto, hipStream_t s)
{
	k_enc_ana_dbg<<<grid_for(n), WAVE, 0, s>>>(enc, sp, n, upto);
	return (int) hipGetLastError();
}

/* the grid of a launch over n channels with no live channel (every lane
 * exits at once): the runtime still reserves the private-segment scratch
 * such a launch needs (engine.hip engine_reserve) */
/* private-segment bytes per lane of the kernel (engine.hip engine_reserve) */
extern "C" size_t kl_ana_private(void)
{
	hipFuncAttributes a, b;	/* both forms: MELPE_HARM=0 runs k_enc_ana<0> */
	size_t x = hipFuncGetAttributes(&a, (const void *) k_enc_ana<1>) == hipSuccess ? a.localSizeBytes : 0;
	size_t y = hipFuncGetAttributes(&b, (const void *) k_enc_ana<0>) == hipSuccess ? b.localSizeBytes : 0;
	return x > y ? x : y;
}

extern "C" int kl_ana_warm(int n, hipStream_t s)
{
	k_enc_ana<1><<<grid_for(n), WAVE, 0, s>>>(nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
						 AnaGate{}, 0);
	return (int) hipGetLastError();
}
