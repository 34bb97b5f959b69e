/*
 * k_dec.hip -- melpe_s (melpe/melpe.c:102-107): channel read, synthesis and
 * postfilter of one superframe per active channel, one lane per channel.
 */
#define MELPE_IDFT_LDS	/* realIDFT's table from LDS (decoder.h) */
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
						      const int *perm, const int *nlive)
{
	for (int len = 1; len <= PITCHMAX; len++)
		for (int i = threadIdx.x; i < len; i += blockDim.x)
			s_idft_cos[((len - 1) * len) / 2 + i] = g_der.idft_cos[len][i];
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

extern "C" int kl_decode(DecState *dec, int16_t *sp, const uint8_t *bits, const uint8_t *active,
			 int n, const int *perm, const int *nlive, hipStream_t s)
{
	int b = DEC_BLOCK;
	while (b > WAVE && (n + b - 1) / b < 1024)
		b /= 2;
	k_decode<<<(n + b - 1) / b, b, IDFT_LDS_WORDS * sizeof(int16_t), s>>>(dec, sp, bits, active, n, perm, nlive);
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
									     0, nullptr, nullptr);
	return (int) hipGetLastError();
}
