/*
 * k_dec.hip -- melpe_s (melpe/melpe.c:102-107): channel read, synthesis and
 * postfilter of one superframe per active channel, one lane per channel.
 */
#include "kern.h"

MELPE_TU(dec)

struct DecLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	DecState S;
	int16_t out[BLOCK];
};

__global__ __launch_bounds__(WAVE, MELPE_DEC_WAVES) void k_decode(DecState *dec, int16_t *sp, const uint8_t *bits,
						 const uint8_t *active, int n)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || (active && !active[c]))
		return;
	DecLane L;
	PIN_FRAME(L);
	lane_copy(&L.S, &dec[c], sizeof(DecState));
	for (int k = 0; k < 11; k++)
		L.S.chbuf[k] = bits[(size_t) c * 11 + k];
	decode_superframe(&L.S, L.out);
	lane_copy(&dec[c], &L.S, sizeof(DecState));
	lane_copy(sp + (size_t) c * BLOCK, L.out, sizeof(int16_t) * BLOCK);
}

extern "C" int kl_decode(DecState *dec, int16_t *sp, const uint8_t *bits, const uint8_t *active,
			 int n, hipStream_t s)
{
	k_decode<<<grid_for(n), WAVE, 0, s>>>(dec, sp, bits, active, n);
	return (int) hipGetLastError();
}
