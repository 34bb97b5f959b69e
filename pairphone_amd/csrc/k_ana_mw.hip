/*
 * k_ana_mw.hip -- the lanes-per-channel analysis kernel (ana_mw.h), in its
 * own translation unit so it compiles beside k_ana.hip.
 */
#include "kern.h"
#include "ana_mw.h"

MELPE_TU(anamw)

/*
 * Lanes-per-channel analysis (ana_mw.h): a workgroup of NW waves runs the
 * same 64 channels, lane t of every wave on channel t, each wave on its own
 * private copy of the record.  The superframe's independent chains (band 0
 * + pitch/gain, LPC + bands 1-2, pitchAuto + band 3, classify + band 4)
 * run on different waves; the few scalars one chain hands another cross
 * through the per-channel exchange block in LDS, ordered by the barrier
 * between phases.  Used when the channels alone would leave SIMDs idle
 * (engine.hip ana_waves): at 32,768 channels lane-per-channel is 512 waves
 * for 1,024 SIMDs.
 */
/* phase timers of the profiling build (tools/mw_prof.py): wave-cycles of
 * virtual wave v in phase p at slot 64 + 5p + v, the phase's wall time seen
 * by wave 0 (barrier included) at 64 + 5p + 4; copy-in / write-back / dc
 * removal after */
#define MW_SLOT(p, v) (64 + 5 * (p) + (v))
#if defined(MELPE_PROF)
#define MW_T0(t) unsigned long long t = __builtin_amdgcn_s_memtime()
#define MW_T1(t, slot)                                                          \
	do {                                                                    \
		unsigned long long _d = __builtin_amdgcn_s_memtime() - (t);     \
		if (__builtin_amdgcn_readfirstlane(threadIdx.x) == threadIdx.x) \
			atomicAdd(&g_prof[slot], _d);                           \
	} while (0)
#else
#define MW_T0(t) (void) 0
#define MW_T1(t, slot) (void) 0
#endif
static_assert(MW_SLOT(MW_PHASES, 2) < 256, "MW timer slots");

struct LdsXch {
	int16_t *w;
	int t;
	__device__ int16_t get(int k) const { return w[k * WAVE + t]; }
	__device__ void put(int k, int16_t v) { w[k * WAVE + t] = v; }
};

/* lsf_vq's score rows (lsfvq_mw.h): visit u of lane `slot` at
 * p[u * stride + slot], coalesced across the wave */
struct GlbDb {
	uint32_t *p;
	size_t stride;
	__device__ uint32_t get(int u) const { return p[(size_t) u * stride]; }
	__device__ void put(int u, uint32_t x) const { p[(size_t) u * stride] = x; }
};

struct AnaMwLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	EncAna S;
	AnaMwTmp tmp;
};

/* resident waves per SIMD the MW kernel is compiled for (caps its VGPRs at
 * 512 / n).  The request must be one the workgroup's LDS allows, or the
 * compiler drops it and allocates for one wave per SIMD (309 VGPRs): the
 * exchange block is 44.7 KB, so three workgroups per CU at most. */
#ifndef MELPE_MW_WAVES
#define MELPE_MW_WAVES 2
#endif
static_assert(MELPE_MW_WAVES * (XS_WORDS * WAVE * 2) <= 160 * 1024, "MW occupancy request exceeds the LDS");

template <int NW>
__global__ __launch_bounds__(WAVE * NW, MELPE_MW_WAVES) void k_enc_ana_mw(EncState *enc, const int16_t *sp,
									    uint8_t *bits, const uint8_t *active,
									    int n, const int *perm, const int *nlive,
									    uint32_t *lqbuf, AnaGate gate)
{
	__shared__ int16_t xs[XS_WORDS * WAVE];
	const int w = threadIdx.x / WAVE, t = threadIdx.x % WAVE;
	/* groups of 64 slots, grid-stride: the engine launches at most 512
	 * workgroups (all resident, two per CU), which take every live slot
	 * however many there are (engine.hip ana_launch picks this kernel from
	 * a live count that may be a superframe old) */
	const int count = perm ? *nlive : n;
	/* the engine enqueues this and the lane kernels, each gated on the
	 * live count: uniform per launch, so every wave leaves before a barrier */
	if (perm && !gate.open(count))
		return;
	gate.mark(blockIdx.x == 0 && threadIdx.x == 0 && count > 0, NW);	/* 0 live: tag stays 0 */
	for (int grp = blockIdx.x; grp * WAVE < count; grp += gridDim.x) {
	int c = grp * WAVE + t;
	bool live;
	if (perm) {
		live = c < *nlive;
		c = live ? perm[c] : 0;
	} else {
		live = c < n && (!active || active[c]);
	}
	AnaMwLane L;
	PIN_FRAME(L);
	LdsXch xc{xs, t};
	GlbDb db{lqbuf + blockIdx.x * WAVE + t, (size_t) gridDim.x * WAVE};
	EncAna *rec = &enc[c].a;
	MW_T0(tb);
	if (live)
		ana_mw_copy_in(&L.S, rec, w, NW);
	MW_T1(tb, MW_SLOT(MW_PHASES, 0));
	MW_T0(td);
	if (live)
		ana_mw_begin(&L.S, sp + (size_t) c * BLOCK);
	MW_T1(td, MW_SLOT(MW_PHASES, 2));
	for (int p = 0; p < MW_PHASES; p++) {
		MW_T0(tp);
		if (live)
			for (int v = w; v < MW_NV; v += NW) {
				MW_T0(tv);
				ana_mw_phase(&L.S, rec, xc, db, L.tmp, v, p);
				MW_T1(tv, MW_SLOT(p, v));
			}
		/* phase NF hands classify's / pitchAuto's tracks to wave 0
		 * through the record: device-scope fences around the barrier
		 * (the lsf block's score rows pass within the workgroup, which
		 * __syncthreads orders) */
		if (p == NF)
			__threadfence();
		__syncthreads();
		if (p == NF)
			__threadfence();
		if (w == 0)
			MW_T1(tp, MW_SLOT(p, 4));
	}
	if (live) {
		MW_T0(te);
		for (int v = w; v < MW_NV; v += NW) {
			size_t off[2], len[2];
			int m = ana_mw_owned(v, off, len);
			for (int k = 0; k < m; k++)
				lane_copy((char *) rec + off[k], (const char *) &L.S + off[k], len[k]);
		}
		if (w == 0)
			for (int k = 0; k < 11; k++)
				bits[(size_t) c * 11 + k] = L.S.chbuf[k];
		MW_T1(te, MW_SLOT(MW_PHASES, 1));
	}
	__syncthreads();	/* the next group reuses the exchange block */
	}
}

/* workgroups of a launch over n slots: every group resident (two per CU,
 * MW_MAX_GROUPS in all), larger counts grid-stride */
#define MW_MAX_GROUPS 512
static unsigned mw_grid(int n)
{
	unsigned g = grid_for(n);
	return g < MW_MAX_GROUPS ? (g ? g : 1) : MW_MAX_GROUPS;
}

/* lqbuf: LQ_ROW x (mw_grid(n) * WAVE) dwords (kl_enc_ana_mw_lq_words) */
extern "C" size_t kl_enc_ana_mw_lq_words(int n)
{
	return (size_t) LQ_ROW * mw_grid(n) * WAVE;
}

extern "C" int kl_enc_ana_mw(EncState *enc, const int16_t *sp, uint8_t *bits, const uint8_t *active,
			     int n, const int *perm, const int *nlive, int nw, uint32_t *lqbuf,
			     AnaGate gate, hipStream_t s)
{
	/* 4 waves per 64 channels (2 measured no better at any channel count
	 * and cost a third more compile time; ana_mw.h supports any count) */
	if (nw == 4)
		k_enc_ana_mw<4><<<mw_grid(n), WAVE * 4, 0, s>>>(enc, sp, bits, active, n, perm, nlive, lqbuf,
								gate);
	else
		return (int) hipErrorInvalidValue;
	return (int) hipGetLastError();
}

extern "C" size_t kl_ana_mw_private(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *) k_enc_ana_mw<4>) == hipSuccess ? a.localSizeBytes : 0;
}

extern "C" int kl_ana_mw_warm(int n, hipStream_t s)
{
	k_enc_ana_mw<4><<<mw_grid(n), WAVE * 4, 0, s>>>(nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr,
							nullptr, AnaGate{});
	return (int) hipGetLastError();
}
