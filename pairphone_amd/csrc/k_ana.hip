/*
 * k_ana.hip -- the analysis half of melpe_a (melpe/melpe.c:97-98:
 * analysis() + the 11-byte frame): dc removal, melp_ana per frame, sc_ana,
 * the quantisers and channel packing, one lane per channel, reading the
 * NPP output k_enc_npp left in the caller's PCM.
 */
#include <stdlib.h>
#include <hip/hip_runtime.h>

/* progress-driven issue priority (MELPE_ANA_PRIO 6, experiment): every wave
 * counts its checkpoints (encoder.h ANA_CKPT: after each frame and after
 * lsf_vq) on one counter, and a wave behind the average takes a higher
 * priority, one ahead a lower */
struct AnaProg {
	unsigned cnt;
	int mode;
};
__device__ AnaProg g_ana_prog;
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void ana_ckpt(int j)
{
	if (g_ana_prog.mode != 6)
		return;
	unsigned before = 0;
	if (__builtin_amdgcn_readfirstlane(threadIdx.x) == threadIdx.x)
		before = atomicAdd(&g_ana_prog.cnt, 1u);
	before = __builtin_amdgcn_readfirstlane(before);
	const int avg4 = (int) ((4ull * before) / gridDim.x);	/* checkpoints passed per wave, x4 */
	const int d = 4 * (j - 1) - avg4;			/* > 0: ahead of the average */
	if (d < -2)
		__builtin_amdgcn_s_setprio(3);
	else if (d < 0)
		__builtin_amdgcn_s_setprio(2);
	else if (d < 2)
		__builtin_amdgcn_s_setprio(1);
	else
		__builtin_amdgcn_s_setprio(0);
}
#define ANA_CKPT(j) ana_ckpt(j)
#endif
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

/* The wave's issue priority from its place in the lane order.  The order
 * runs from the lightest classes to the heaviest (voiced, long pitch), and
 * with every wave resident from the first cycle the launch lasts as long as
 * its heaviest waves: measured per wave at 262,144 channels
 * (profiles/r06_m_wave_place.txt), the first 1/32 of the order takes 19.4 ms,
 * the last 24.6 ms, and each SIMD holds four waves from across the order.
 * Mode 1: quartile q of the order runs at priority q; mode 2: the lower half
 * at 1, the upper at 3 (priority 0 is then left to the next superframe's NPP
 * waves in the pipelined step). */
__device__ __forceinline__ void ana_wave_prio(int mode, int w, int nw)
{
	if (mode <= 0)
		return;
	const int q = (4 * w) / nw;	/* 0..3, wave-uniform */
	if (mode == 3) {
		if (q >= 2)
			__builtin_amdgcn_s_setprio(1);
	} else if (mode == 4) {
		if (q == 3)
			__builtin_amdgcn_s_setprio(1);
	} else if (mode == 5) {
		if (q == 1 || q == 2)
			__builtin_amdgcn_s_setprio(1);
		else if (q == 3)
			__builtin_amdgcn_s_setprio(2);
	} else if (mode == 6) {
		__builtin_amdgcn_s_setprio(1);
	} else if (mode == 1) {
		if (q == 1)
			__builtin_amdgcn_s_setprio(1);
		else if (q == 2)
			__builtin_amdgcn_s_setprio(2);
		else if (q >= 3)
			__builtin_amdgcn_s_setprio(3);
	} else {
		if (q >= 2)
			__builtin_amdgcn_s_setprio(3);
		else
			__builtin_amdgcn_s_setprio(1);
	}
}

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
		ana_wave_prio(prio, blockIdx.x, (L + WAVE - 1) / WAVE);
		c = perm[c];
	} else {
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

/* MELPE_ANA_PRIO: the waves' issue priority by lane order (ana_wave_prio) */
static int ana_prio_mode(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("MELPE_ANA_PRIO");
		v = e ? atoi(e) : 0;
	}
	return v;
}

extern "C" int kl_enc_ana(EncState *enc, const int16_t *sp, uint8_t *bits, const uint8_t *active,
			  int n, const int *perm, const int *nlive, int16_t *res, AnaGate gate, hipStream_t s)
{
	const int pm = ana_prio_mode();
	if (pm == 6) {	/* the progress counter restarts with each launch */
		static const AnaProg z = {0u, 6};
		hipError_t er = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ana_prog), &z, sizeof(z), 0,
						       hipMemcpyHostToDevice, s);
		if (er != hipSuccess)
			return (int) er;
	}
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
