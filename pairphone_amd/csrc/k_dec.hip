/*
 * k_dec.hip -- melpe_s (melpe/melpe.c:102-107): channel read, synthesis and
 * postfilter of one superframe per active channel, one lane per channel.
 */
#define MELPE_IDFT_LDS	/* realIDFT's table from LDS (decoder.h) */
#define MELPE_PROG_PRIO	/* progprio.h: DEC_CKPT in k_decode */
#include <stdlib.h>
#include "kern.h"

MELPE_TU(dec)

/* up to four waves per block share one LDS copy of the realIDFT table;
 * kl_decode picks the widest block that still gives every CU four blocks */
#define DEC_BLOCK 256

struct DecLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	DecState S;
	int16_t out[BLOCK];
};

__global__ __launch_bounds__(DEC_BLOCK, MELPE_DEC_WAVES) void k_decode(DecState *dec, int16_t *sp,
						      const uint8_t *bits, const uint8_t *active, int n,
						      const int *perm, const int *nlive, int prio)
{
	for (int len = 1; len <= PITCHMAX; len++)
		for (int i = threadIdx.x; i < len; i += blockDim.x)
			s_idft_cos[((len - 1) * len) / 2 + i] = g_der.idft_cos[len][i];
	/* progprio.h: the counter is the sort's control word nlive[2] */
	if (perm)
		PP_BEGIN(prio ? (unsigned *) (nlive + 2) : nullptr, (*nlive + WAVE - 1) / WAVE);
	else
		PP_BEGIN(nullptr, 1);
	__syncthreads();
	/* lane g decodes channel perm[g] when the engine ordered the live
	 * channels by pitch class (engine.hip, MELPE_BIN) */
	int c = blockIdx.x * blockDim.x + threadIdx.x;
	if (perm) {
		if (c >= *nlive)
			return;
		c = perm[c];
	} else if (c >= n || (active && !active[c])) {
		return;
	}
	DecLane L;
	PIN_FRAME(L);
	static_assert(sizeof(DecState) % 16 == 0 && offsetof(DecLane, S) % 16 == 0, "16-byte record copy");
	lane_copy_x4(&L.S, &dec[c], sizeof(DecState));
	for (int k = 0; k < 11; k++)
		L.S.chbuf[k] = bits[(size_t) c * 11 + k];
	decode_superframe(&L.S, L.out);
	lane_copy_x4(&dec[c], &L.S, sizeof(DecState));
	lane_copy(sp + (size_t) c * BLOCK, L.out, sizeof(int16_t) * BLOCK);
}

/* MELPE_DEC_PRIO=0: no progress-driven priority (progprio.h), for A/Bs */
static int dec_prio_mode(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("MELPE_DEC_PRIO");
		v = e ? (atoi(e) != 0) : 1;
	}
	return v;
}

extern "C" int kl_decode(DecState *dec, int16_t *sp, const uint8_t *bits, const uint8_t *active,
			 int n, const int *perm, const int *nlive, hipStream_t s)
{
	int b = DEC_BLOCK;
	while (b > WAVE && (n + b - 1) / b < 1024)
		b /= 2;
	k_decode<<<(n + b - 1) / b, b, IDFT_LDS_WORDS * sizeof(int16_t), s>>>(dec, sp, bits, active, n, perm, nlive,
									     dec_prio_mode());
	return (int) hipGetLastError();
}

/*
 * The two-wave decoder (decoder.h melp_syn_a / melp_syn_b): for channel
 * counts that leave SIMDs idle in lane mode (32,768 channels are 512 waves
 * for 1,024 SIMDs), each group of 64 channels gets two waves, lane t of both
 * on channel t, each wave on its own private copy of the record.  Wave A
 * reads the channel and synthesises each frame's excitation (the parameter
 * interpolation, harm_syn_pitch / realIDFT); wave B runs the synthesis
 * filters, scale_adj, the dispersion FIR and the postfilter one frame
 * behind, on what A handed over through a coalesced HBM buffer (word k of
 * lane t at k * 64 + t, two frame buffers per group).  A workgroup holds
 * DEC2_GROUPS groups sharing one LDS copy of the realIDFT table (only A
 * reads it).  Each wave writes back its own side of the record (state.h
 * DEC_B_BEG); B writes the PCM.
 */
#ifndef DEC2_GROUPS
#define DEC2_GROUPS 2
#endif
#define DEC2_BLOCK (2 * WAVE * DEC2_GROUPS)

struct HbG {
	uint32_t *p;
	__device__ uint32_t get(int k) const { return p[(size_t) k * WAVE]; }
	__device__ void put(int k, uint32_t v) const { p[(size_t) k * WAVE] = v; }
};

struct Dec2Lane {
	uint8_t guard[FLAT_GUARD_BYTES];
	DecState S;
	int16_t out[BLOCK];
};

__global__ __launch_bounds__(DEC2_BLOCK, MELPE_DEC_WAVES) void k_decode2(DecState *dec, int16_t *sp,
							const uint8_t *bits, const uint8_t *active, int n,
							const int *perm, const int *nlive, uint32_t *hbuf)
{
	for (int len = 1; len <= PITCHMAX; len++)
		for (int i = threadIdx.x; i < len; i += blockDim.x)
			s_idft_cos[((len - 1) * len) / 2 + i] = g_der.idft_cos[len][i];
	PP_BEGIN(nullptr, 1);	/* no checkpoint is on its path; kept off all the same */
	__syncthreads();
	const int w = threadIdx.x / WAVE, t = threadIdx.x % WAVE;
	const int grp = blockIdx.x * DEC2_GROUPS + (w >> 1), role = w & 1;
	int c = grp * WAVE + t;
	bool live;
	if (perm) {
		live = c < *nlive;
		c = live ? perm[c] : 0;
	} else {
		live = c < n && (!active || active[c]);
	}
	Dec2Lane L;
	PIN_FRAME(L);
	if (live) {
		lane_copy_x4(&L.S, &dec[c], sizeof(DecState));
		if (role == 0)
			for (int k = 0; k < 11; k++)
				L.S.chbuf[k] = bits[(size_t) c * 11 + k];
	}
	const HbG hb0{hbuf + (size_t) (2 * grp) * HB_WORDS * WAVE + t};
	const HbG hb1{hbuf + (size_t) (2 * grp + 1) * HB_WORDS * WAVE + t};
	for (int p = 0; p < DEC2_PHASES; p++) {
		if (live)
			dec2_phase(&L.S, L.out, hb0, hb1, role, p);
		__syncthreads();
	}
	if (live) {
		if (role == 0) {
			lane_copy_x4(&dec[c], &L.S, DEC_B_BEG);
		} else {
			lane_copy_x4((char *) &dec[c] + DEC_B_BEG, (const char *) &L.S + DEC_B_BEG,
				     sizeof(DecState) - DEC_B_BEG);
			lane_copy(sp + (size_t) c * BLOCK, L.out, sizeof(int16_t) * BLOCK);
		}
	}
}

static unsigned dec2_grid(int n)
{
	const int per = WAVE * DEC2_GROUPS;
	return (unsigned) ((n + per - 1) / per);
}

/* hand-over buffer of a launch over n channels, in dwords */
extern "C" size_t kl_decode2_hb_words(int n)
{
	return (size_t) dec2_grid(n) * DEC2_GROUPS * 2 * HB_WORDS * WAVE;
}

extern "C" int kl_decode2(DecState *dec, int16_t *sp, const uint8_t *bits, const uint8_t *active, int n,
			  const int *perm, const int *nlive, uint32_t *hbuf, hipStream_t s)
{
	if (n <= 0)
		return 0;
	k_decode2<<<dec2_grid(n), DEC2_BLOCK, IDFT_LDS_WORDS * sizeof(int16_t), s>>>(dec, sp, bits, active, n,
										     perm, nlive, hbuf);
	return (int) hipGetLastError();
}

extern "C" size_t kl_dec2_private(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *) k_decode2) == hipSuccess ? a.localSizeBytes : 0;
}

extern "C" int kl_dec2_warm(int n, hipStream_t s)
{
	k_decode2<<<dec2_grid(n), DEC2_BLOCK, IDFT_LDS_WORDS * sizeof(int16_t), s>>>(
		nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr);
	return (int) hipGetLastError();
}

extern "C" size_t kl_dec_private(void)
{
	hipFuncAttributes a;
	return hipFuncGetAttributes(&a, (const void *) k_decode) == hipSuccess ? a.localSizeBytes : 0;
}

extern "C" int kl_dec_warm(int n, hipStream_t s)
{
	int b = DEC_BLOCK;
	while (b > WAVE && (n + b - 1) / b < 1024)
		b /= 2;
	k_decode<<<(n + b - 1) / b, b, IDFT_LDS_WORDS * sizeof(int16_t), s>>>(nullptr, nullptr, nullptr, nullptr,
									     0, nullptr, nullptr, 0);
	return (int) hipGetLastError();
}
