/*
 * k_r24.hip -- the 2400 bps MELP mode (codec2400.h): analysis + packing of
 * one NPP-processed 180-sample frame per channel (the NPP frame runs in
 * k_npp at RATE2400), and channel read + synthesis of one 7-byte frame per
 * channel.  One lane per channel, state copied to the lane's private
 * segment as in k_ana.hip / k_dec.hip.
 */
#include "kern.h"
#include "codec2400.h"

MELPE_TU(r24)

struct Ana24Lane {
	uint8_t guard[FLAT_GUARD_BYTES];
	EncAna S;
	int16_t x[FRAME];
};

__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_enc24(EncState *enc, const int16_t *sp,
								  uint8_t *bits, const uint8_t *active,
								  int n)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || (active && !active[c]))
		return;
	Ana24Lane L;
	PIN_FRAME(L);
	lane_copy(&L.S, &enc[c].a, sizeof(EncAna));
	lane_copy(L.x, sp + (size_t) c * FRAME, sizeof(int16_t) * FRAME);
	analysis24(&L.S, L.x);
	lane_copy(&enc[c].a, &L.S, sizeof(EncAna));
	for (int k = 0; k < R24_BYTES; k++)
		bits[(size_t) c * R24_BYTES + k] = L.S.chbuf[k];
}

struct Dec24Lane {
	uint8_t guard[FLAT_GUARD_BYTES];
	DecState S;
	int16_t out[FRAME];
};

__global__ __launch_bounds__(WAVE, MELPE_DEC_WAVES) void k_dec24(DecState *dec, int16_t *sp,
								  const uint8_t *bits, const uint8_t *active,
								  int n)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || (active && !active[c]))
		return;
	Dec24Lane L;
	PIN_FRAME(L);
	lane_copy(&L.S, &dec[c], sizeof(DecState));
	for (int k = 0; k < R24_BYTES; k++)
		L.S.chbuf[k] = bits[(size_t) c * R24_BYTES + k];
	decode_frame24(&L.S, L.out);
	lane_copy(&dec[c], &L.S, sizeof(DecState));
	lane_copy(sp + (size_t) c * FRAME, L.out, sizeof(int16_t) * FRAME);
}

extern "C" int kl_enc24(EncState *enc, const int16_t *sp, uint8_t *bits, const uint8_t *active,
			int n, hipStream_t s)
{
	k_enc24<<<grid_for(n), WAVE, 0, s>>>(enc, sp, bits, active, n);
	return (int) hipGetLastError();
}

extern "C" int kl_dec24(DecState *dec, int16_t *sp, const uint8_t *bits, const uint8_t *active,
			int n, hipStream_t s)
{
	k_dec24<<<grid_for(n), WAVE, 0, s>>>(dec, sp, bits, active, n);
	return (int) hipGetLastError();
}
