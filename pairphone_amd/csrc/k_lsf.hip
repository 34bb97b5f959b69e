/*
 * k_lsf.hip -- lsf_vq (melpe/qnt12.c:895-1138) with one WAVEFRONT per
 * channel (lsfvq_wave.h).
 *
 * In the lane-per-channel analysis each lane ran its channel's M-best
 * searches alone: about 5 ms of k_enc_ana at 262,144 channels (a build with
 * lsf_vq knocked out, profiles/r03_ko_*).  k_enc_ana (mode 4) now stops
 * before lsf_vq and leaves the voicing pattern lsf_vq sees; this kernel
 * quantises the LSFs with the searches spread over the wave, and
 * k_enc_harm forms the residuals from them.
 */
#include "kern.h"
#include "lsfvq_wave.h"

MELPE_TU(lsf)

/* one wave per live channel: slot g runs channel perm[g] (the engine's lane
 * order) or channel g under the mask; aux: k_enc_ana mode 4's hand-over */
__global__ __launch_bounds__(WAVE) void k_enc_lsf(EncState *enc, const int16_t *aux, const uint8_t *active,
						  int n, const int *perm, const int *nlive)
{
	int c = blockIdx.x;
	if (perm) {
		if (c >= *nlive)
			return;
		c = perm[c];
	} else if (c >= n || (active && !active[c])) {
		return;
	}
	__shared__ LsfShared W;
	lsf_vq_wv(&enc[c], aux + (size_t) c * LSF_AUX, &W, threadIdx.x);
}

extern "C" int kl_enc_lsf(EncState *enc, const int16_t *aux, const uint8_t *active, int n,
			  const int *perm, const int *nlive, hipStream_t s)
{
	k_enc_lsf<<<n, WAVE, 0, s>>>(enc, aux, active, n, perm, nlive);
	return (int) hipGetLastError();
}
