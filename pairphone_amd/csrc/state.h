/*
 * state.h -- explicit per-channel state of the engine.
 *
 * The reference keeps one codec instance per process in globals
 * (melpe/global.c:20-53) and ~90 function statics.
 * Here every one of them is a field of EncState / DecState, one instance per
 * channel in HBM; *_reset() gives the state of a fresh process.
 */
#ifndef MELPE_STATE_H
#define MELPE_STATE_H

#include "npp.h"

namespace mlp {

struct EncState {
	NppState npp;
};

struct DecState {
	int16_t dummy;
};

MD void enc_reset(EncState *e)
{
	npp_reset(&e->npp);
}

MD void dec_reset(DecState *d)
{
	d->dummy = 0;
}

}  // namespace mlp

#endif
