/*
 * tables.h -- constant tables of the codec as seen by the device code.
 *
 * g_tab holds the standard's codebooks and filter tables, extracted from the
 * reference objects by oracle/dump_tables.py into
 * pairphone_amd/data/melpe_tables.bin and uploaded once per device
 * (hipMemcpyToSymbol).  g_der holds the tables the reference computes on first
 * use (FFT twiddles melpe/fft_lib.c:285, the LSP cosine grid
 * melpe/lpc_lib.c:640-657, the Fourier-magnitude weights melpe/vq_lib.c:512,
 * the postfilter cross-fade window melpe/postfilt.c:73); an init kernel fills
 * it with init_derived() (dsp.h).
 */
#ifndef MELPE_TABLES_H
#define MELPE_TABLES_H

#include "ops.h"
#include "tables_gen.h"

alignas(16) MDEV_TAB int16_t g_tab[MELPE_TABLE_WORDS];	/* codebooks at even offsets: dword rows */
#define TB(name) ((const int16_t *) (g_tab + TOFF_##name))

struct DerivedTables {
	int16_t wr[257];	/* cos twiddles, + one dead slot read by cfft/rfft */
	int16_t wi[257];	/* sin twiddles */
	int16_t lsp_cos[512];	/* cos grid for lsp_to_freq */
	int16_t w_fs[10];	/* Fourier-magnitude VQ weights, Q14 */
	int16_t w_fs_inv[10];
	int16_t pf_window[20];	/* postfilter gain cross-fade window */
	int16_t pad[2];
	/* realIDFT's cosine table for period len (melpe/harm.c:70-80): it
	 * depends on len only, so it is built once for every len 1..160 */
	int16_t idft_cos[161][160];
};

MDEV_CONST DerivedTables g_der;

/* lsp_to_freq's grid values in the order its scan reads them:
 * g_lspgrid[40 b + 5 u + k - 1] = lsp_cos[(k (8 b + u)) mod 512], grid point
 * i = 8 b + u, term k = 1..5 (order 10).  Data-independent and read at
 * wave-uniform addresses, so it lives in constant memory and comes through
 * scalar loads (a block's 40 values in five dwordx4-sized pieces) instead of
 * one vector load per value; filled from g_der.lsp_cos after the derivation
 * (derive_lspgrid), on the host. */
#define LSPGRID_BLOCKS 33	/* 8 b + u covers the 257 points 0..256 */
alignas(16) MDEV_TAB int16_t g_lspgrid[LSPGRID_BLOCKS * 40];

#endif
