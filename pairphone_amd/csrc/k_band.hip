/*
 * k_band.hip -- bands 1..4 of bpvc_ana (melpe/melp_sub.c:137-189) for the
 * superframe's three frames, one lane per (channel, band).
 *
 * In the lane-per-channel analysis the five voicing bands of each frame ran
 * one after the other inside k_enc_ana: a third of its time (a build with
 * bpvc_ana knocked out, profiles/r03_q_ko_*).  Band 0 decides the frame's
 * pitch and stays in melp_ana; bands 1..4 are four independent chains (each
 * touches only its own filter / envelope memories and bpvc[j]) whose result
 * nothing in melp_ana reads (encoder.h melp_ana, analysis_a1).  So k_enc_ana
 * runs the frames with band 0 (mode 2), this kernel runs the four chains,
 * four lanes per channel with a few hundred bytes of state each, and
 * k_enc_ana runs the superframe (mode 3).  Every value is the reference's:
 * the chains run the reference's steps in its order and arithmetic.
 */
#include "kern.h"

MELPE_TU(band)

struct BandLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	BandState B;
};

/* lane 4 s + (j - 1) runs band j of slot s: channel perm[s] (the engine's
 * lane order, which keeps a channel's four bands in one wave) or channel s
 * under the mask */
__global__ __launch_bounds__(WAVE, 4) void k_enc_band(EncState *enc, const int16_t *bw,
						      const uint8_t *active, int n, const int *perm,
						      const int *nlive)
{
	const int g = blockIdx.x * WAVE + threadIdx.x;
	int c = g >> 2;
	const int j = 1 + (g & 3);
	if (perm) {
		if (c >= *nlive)
			return;
		c = perm[c];
	} else if (c >= n || (active && !active[c])) {
		return;
	}
	BandLane L;
	PIN_FRAME(L);
	static_assert(offsetof(EncState, band) % 4 == 0 && sizeof(BandState) % 4 == 0,
		      "the band memories are dword copies");
	lane_copy(&L.B, &enc[c].band[j], sizeof(BandState));
	int16_t w[2 * NF];
	for (int k = 0; k < 2 * NF; k++)
		w[k] = bw[(size_t) c * 2 * NF + k];
	ana_band_frames(&L.B, enc[c].hpspeech, j, w, enc[c].par);
	lane_copy(&enc[c].band[j], &L.B, sizeof(BandState));
}

extern "C" int kl_enc_band(EncState *enc, const int16_t *bw, const uint8_t *active, int n,
			   const int *perm, const int *nlive, hipStream_t s)
{
	k_enc_band<<<grid_for(4 * n), WAVE, 0, s>>>(enc, bw, active, n, perm, nlive);
	return (int) hipGetLastError();
}
