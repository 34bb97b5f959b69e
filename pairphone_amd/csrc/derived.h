/*
 * derived.h -- fills g_der, the tables the reference computes lazily on
 * first use.  Runs once per device (one lane of an init kernel) and once on
 * the host emulation build.
 */
#ifndef MELPE_DERIVED_H
#define MELPE_DERIVED_H

#include "dsp.h"

namespace mlp {

MD void derive_fft_twiddles(DerivedTables *d)	/* fs_init, melpe/fft_lib.c:285 */
{
	Word16 step = shl(2, norm_s(256));
	Word16 th = 0;
	for (int i = 0; i < 256; i++) {
		d->wr[i] = cos_fxp(th);
		d->wi[i] = sin_fxp(th);
		th = add(th, step);
	}
	d->wr[256] = 0;	/* dead read past the end in cfft/rfft */
	d->wi[256] = 0;
}

MD void derive_lsp_cos(DerivedTables *d)	/* melpe/lpc_lib.c:640-652 */
{
	Word16 th = 0;
	for (int i = 0; i <= 128; i++) {
		d->lsp_cos[i] = cos_fxp(th);
		d->lsp_cos[i + 256] = negate(d->lsp_cos[i]);
		th = add(th, 128);
	}
	for (int i = 0, a = 128, b = 128; i < 128; i++, a++, b--) {
		d->lsp_cos[a] = negate(d->lsp_cos[b]);
		d->lsp_cos[a + 256] = d->lsp_cos[b];
	}
}

}  // namespace mlp

#endif
