/*
 * k_ana.hip -- the analysis half of melpe_a (melpe/melpe.c:97-98:
 * analysis() + the 11-byte frame): dc removal, melp_ana per frame, sc_ana,
 * the quantisers and channel packing, one lane per channel, reading the
 * NPP output k_enc_npp left in the caller's PCM.
 */
#include <stdlib.h>
#include "kern.h"

MELPE_TU(ana)

struct AnaLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	EncState S;	/* only the part after the NPP state is live */
	int16_t x[BLOCK];
};

/* MODE 0: the whole analysis and the bits here (MELPE_HARM=0).
 * MODE 1: the split form (encoder.h analysis_a): the windowed residuals to
 *         res (NF x LPC_FRAME per channel), the Fourier magnitudes and the
 *         packing in k_harm.hip.
 * MODE 2: analysis_a1, the frames with band 0 of bpvc_ana only, bw (2 x NF
 *         per channel) for k_band.hip, which runs bands 1..4;
 * MODE 3: analysis_a2, the superframe up to the residuals (as MODE 1's
 *         second half).  It neither reads nor writes the band memories.
 * MODE 4: analysis_c, everything before lsf_vq's turn but lsf_vq, the
 *         voicing pattern it sees and its weights into bw (LSF_AUX words
 *         per channel, encoder.h lsf_aux; k_lsf.hip, then k_enc_harm
 *         forms the residuals and k_enc_tail shifts the history). */
template <int MODE>
__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_enc_ana(EncState *enc, const int16_t *sp, uint8_t *bits,
						  const uint8_t *active, int n, const int *perm,
						  const int *nlive, int16_t *res, int16_t *bw)
{
	/* lane g runs channel perm[g] when the engine ordered the live channels
	 * by pitch class (engine.hip, MELPE_BIN), else channel g under the mask */
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (perm) {
		if (c >= *nlive)
			return;
		c = perm[c];
	} else if (c >= n || (active && !active[c])) {
		return;
	}
	AnaLane L;
	PIN_FRAME(L);
	constexpr size_t nb = MODE == 3 ? offsetof(EncState, band) - ENC_ANA_OFF : ENC_ANA_BYTES;
	static_assert(nb % 4 == 0, "the record copy is in dwords");
	lane_copy((char *) &L.S + ENC_ANA_OFF, (const char *) &enc[c] + ENC_ANA_OFF, nb);
	if (MODE != 3)
		lane_copy(L.x, sp + (size_t) c * BLOCK, sizeof(int16_t) * BLOCK);
	if (MODE == 0)
		analysis(&L.S, L.x);
	else if (MODE == 1)
		analysis_a(&L.S, L.x, res + (size_t) c * NF * LPC_FRAME);
	else if (MODE == 2) {
		int16_t w[2 * NF];
		analysis_a1(&L.S, L.x, w);
		for (int k = 0; k < 2 * NF; k++)
			bw[(size_t) c * 2 * NF + k] = w[k];
	} else if (MODE == 3) {
		analysis_a2(&L.S, res + (size_t) c * NF * LPC_FRAME);
	} else {
		Word16 u;
		analysis_c(&L.S, L.x, &u);
		int16_t aux[LSF_AUX];
		lsf_aux(L.S.par, u, aux);
		for (int k = 0; k < LSF_AUX; k++)
			bw[(size_t) c * LSF_AUX + k] = aux[k];
	}
	lane_copy((char *) &enc[c] + ENC_ANA_OFF, (const char *) &L.S + ENC_ANA_OFF, nb);
	if (MODE == 0)
		for (int k = 0; k < 11; k++)
			bits[(size_t) c * 11 + k] = L.S.chbuf[k];
}

/* debug aid: analysis cut after `upto` stages (0 = nothing) */
__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_enc_ana_dbg(EncState *enc, const int16_t *sp, int n, int upto)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || upto <= 0)
		return;
	AnaLane L;
	PIN_FRAME(L);
	lane_copy((char *) &L.S + ENC_ANA_OFF, (const char *) &enc[c] + ENC_ANA_OFF, ENC_ANA_BYTES);
	lane_copy(L.x, sp + (size_t) c * BLOCK, sizeof(int16_t) * BLOCK);
	analysis_upto(&L.S, L.x, upto);
	lane_copy((char *) &enc[c] + ENC_ANA_OFF, (const char *) &L.S + ENC_ANA_OFF, ENC_ANA_BYTES);
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

extern "C" int kl_enc_ana(EncState *enc, const int16_t *sp, uint8_t *bits, const uint8_t *active,
			  int n, const int *perm, const int *nlive, int16_t *res, hipStream_t s)
{
	if (res)
		k_enc_ana<1><<<grid_for(n), WAVE, ana_lds_bytes(), s>>>(enc, sp, bits, active, n, perm, nlive, res,
									  nullptr);
	else
		k_enc_ana<0><<<grid_for(n), WAVE, ana_lds_bytes(), s>>>(enc, sp, bits, active, n, perm, nlive, res,
									  nullptr);
	return (int) hipGetLastError();
}

/* part 1: analysis_a1 (bw out), part 2: analysis_a2 (res out), part 3:
 * analysis_c (the voicing pattern per channel into bw) */
extern "C" int kl_enc_ana_part(EncState *enc, const int16_t *sp, int16_t *bw, int16_t *res,
			       const uint8_t *active, int n, const int *perm, const int *nlive, int part,
			       hipStream_t s)
{
	if (part == 3)
		k_enc_ana<4><<<grid_for(n), WAVE, ana_lds_bytes(), s>>>(enc, sp, nullptr, active, n, perm, nlive,
									  nullptr, bw);
	else if (part == 1)
		k_enc_ana<2><<<grid_for(n), WAVE, ana_lds_bytes(), s>>>(enc, sp, nullptr, active, n, perm, nlive,
									  nullptr, bw);
	else
		k_enc_ana<3><<<grid_for(n), WAVE, ana_lds_bytes(), s>>>(enc, nullptr, nullptr, active, n, perm,
									  nlive, res, nullptr);
	return (int) hipGetLastError();
}

extern "C" int kl_enc_ana_dbg(EncState *enc, const int16_t *sp, int n, int upto, hipStream_t s)
{
	k_enc_ana_dbg<<<grid_for(n), WAVE, 0, s>>>(enc, sp, n, upto);
	return (int) hipGetLastError();
}
