/*
 * codec.h -- everything a per-channel MELPe-1200 lane runs, plus the one-time
 * derivation of g_der (the tables the reference builds on first use).
 */
#ifndef MELPE_CODEC_H
#define MELPE_CODEC_H

#include "encoder.h"
#include "decoder.h"
#include "derived.h"

namespace mlp {

/* melp_ana_init's w_fs / w_fs_inv (melpe/melp_ana.c:482-487) */
MD void derive_fs_weights(DerivedTables *d)
{
	vq_fsw(d->w_fs, NUM_HARM, 30720);
	for (int i = 0; i < NUM_HARM; i++)
		d->w_fs_inv[i] = divide_s(8192, d->w_fs[i]);
}

MD void derive_all(DerivedTables *d)
{
	derive_fft_twiddles(d);
	derive_lsp_cos(d);
	derive_fs_weights(d);
	derive_idft_cos(d);
}

/* g_lspgrid from the derived cosine grid (host side: the device copy is in
 * constant memory) */
static inline void derive_lspgrid(const int16_t *lsp_cos, int16_t *grid)
{
	for (int b = 0; b < LSPGRID_BLOCKS; b++)
		for (int u = 0; u < 8; u++)
			for (int k = 1; k <= 5; k++)
				grid[40 * b + 5 * u + k - 1] = lsp_cos[(k * (8 * b + u)) & 511];
}

}  // namespace mlp

#endif
