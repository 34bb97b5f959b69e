/*
 * synth.h -- deterministic, integer-only speech-like test-signal generator.
 *
 * Used by (1) the benchmark (as a HIP kernel, one lane per channel, so
 * hundreds of thousands of channels of input are made directly in HBM),
 * (2) the tests and (3) the oracle harness (oracle/ref_tool.c) that feeds the
 * same samples to the reference codec.  Pure 32-bit integer arithmetic, so
 * every compiler and target produces the same samples for the same seed.
 *
 * The signal follows the distribution described in SURVEY.md section 8(d):
 * segments of 0.2-0.6 s that are voiced (p=0.55: pulse train with f0 in
 * 90-240 Hz plus vibrato, through three formant resonators, peak ~3k-12k),
 * unvoiced (p=0.25: resonator-coloured noise, peak ~0.5k-3k) or near-silence
 * (p=0.20: |x| < 40).  Channel c of run seed s uses seed synth_mix(s, c).
 *
 * C99 / C++ / HIP compatible: define SYN_FN before inclusion to add
 * __device__ qualifiers.
 */
#ifndef MELPE_SYNTH_H
#define MELPE_SYNTH_H

#include <stdint.h>

#ifndef SYN_FN
#define SYN_FN static inline
#endif

typedef struct {
	uint32_t rng;		/* xorshift32 state, never 0 */
	int32_t seg_left;	/* samples left in the current segment */
	int32_t seg_type;	/* 0 voiced, 1 unvoiced, 2 silence */
	int32_t amp;		/* output gain, Q8 */
	int32_t base_period;	/* pitch period, Q8 samples */
	int32_t phase;		/* position inside the period, Q8 */
	int32_t vib_pos, vib_step;	/* vibrato triangle position (Q16) and step */
	int32_t fset;		/* formant set index */
	int32_t y1[3], y2[3];	/* resonator memories */
} synth_state;

/* Resonator coefficient pairs (a1, a2) in Q14 for five vowel-like formant
 * sets (F1,F2,F3 with bandwidths 90/110/170 Hz at fs = 8 kHz), and one
 * high-frequency resonator for unvoiced segments. */
#define SYN_NSETS 5

SYN_FN uint32_t synth_mix(uint32_t seed, uint32_t ch)
{
	uint32_t h = seed * 0x9E3779B1u ^ (ch + 0x7F4A7C15u) * 0x85EBCA77u;
	h ^= h >> 15;
	h *= 0x2C1B3C6Du;
	h ^= h >> 12;
	h *= 0x297A2D39u;
	h ^= h >> 15;
	return h ? h : 0x1234567u;
}

SYN_FN uint32_t synth_next(synth_state *s)
{
	uint32_t x = s->rng;
	x ^= x << 13;
	x ^= x >> 17;
	x ^= x << 5;
	s->rng = x;
	return x;
}

SYN_FN void synth_init(synth_state *s, uint32_t seed)
{
	int k;
	s->rng = seed ? seed : 0x1234567u;
	s->seg_left = 0;
	s->seg_type = 2;
	s->amp = 0;
	s->base_period = 64 << 8;
	s->phase = 0;
	s->vib_pos = 0;
	s->vib_step = 0;
	s->fset = 0;
	for (k = 0; k < 3; k++) {
		s->y1[k] = 0;
		s->y2[k] = 0;
	}
}

SYN_FN void synth_new_segment(synth_state *s)
{
	uint32_t r = synth_next(s) % 100u;
	s->seg_left = 1600 + (int32_t) (synth_next(s) % 3201u);
	if (r < 55u) {
		int32_t f0 = 90 + (int32_t) (synth_next(s) % 151u);
		s->seg_type = 0;
		s->base_period = (8000 << 8) / f0;
		s->fset = (int32_t) (synth_next(s) % SYN_NSETS);
		/* target peak 3k..12k, divided by the measured peak gain of
		 * the formant set (Q8) */
		{
			const int32_t inv_gain[SYN_NSETS] = { 427, 1160, 135, 256, 222 };
			int32_t peak = 3000 + (int32_t) (synth_next(s) % 9001u);
			s->amp = (peak * inv_gain[s->fset]) >> 8;
		}
		s->vib_step = 3 + (int32_t) (synth_next(s) % 6u);
	} else if (r < 80u) {
		s->seg_type = 1;
		s->amp = 24 + (int32_t) (synth_next(s) % 121u);
	} else {
		s->seg_type = 2;
		s->amp = 0;
	}
}

/* Produces n samples into out[].  State carries across calls, so a stream
 * generated in pieces equals the stream generated at once. */
SYN_FN void synth_block(synth_state *s, int16_t *out, int n)
{
	/* formant (a1) for each of the 5 sets x 3 resonators, and shared a2 */
	const int32_t a1t[15] = {
		26572, 20568, -10383, 30922, -7086, -21844, 28929, 3933,
		-11284, 28513, 24797, -9701, 30756, 24337, -5744
	};
	const int32_t a2t[3] = { -15266, -15028, -14336 };
	int i, k;
	for (i = 0; i < n; i++) {
		int32_t x, y;
		if (s->seg_left <= 0)
			synth_new_segment(s);
		s->seg_left--;
		if (s->seg_type == 0) {
			int32_t tri, period;
			/* triangle vibrato of +-3% with a period of ~0.25-0.7 s */
			s->vib_pos = (s->vib_pos + s->vib_step) & 0xFFFF;
			tri = s->vib_pos < 0x8000 ? s->vib_pos - 0x4000 : 0xC000 - s->vib_pos;
			period = s->base_period + (int32_t) (((int64_t) s->base_period * tri) >> 19);
			s->phase += 256;
			x = (int32_t) (synth_next(s) & 255u) - 128;	/* aspiration */
			if (s->phase >= period) {
				s->phase -= period;
				x += 12000;
			}
			for (k = 0; k < 3; k++) {
				int64_t acc = (int64_t) x * 4096 + (int64_t) a1t[s->fset * 3 + k] * s->y1[k] +
				    (int64_t) a2t[k] * s->y2[k];
				y = (int32_t) (acc >> 14);
				if (y > 1000000) y = 1000000;
				if (y < -1000000) y = -1000000;
				s->y2[k] = s->y1[k];
				s->y1[k] = y;
				x = y;
			}
			y = (int32_t) (((int64_t) x * s->amp) >> 10);
		} else if (s->seg_type == 1) {
			x = (int32_t) (synth_next(s) & 4095u) - 2048;
			{
				int32_t acc = x * 4096 - 8806 * s->y1[0] - 8080 * s->y2[0];
				y = acc >> 14;
				s->y2[0] = s->y1[0];
				s->y1[0] = y;
			}
			y = (y * s->amp) >> 6;
		} else {
			y = (int32_t) (synth_next(s) % 61u) - 30;
			s->y1[0] = s->y1[1] = s->y1[2] = 0;
			s->y2[0] = s->y2[1] = s->y2[2] = 0;
		}
		if (y > 32767) y = 32767;
		if (y < -32768) y = -32768;
		out[i] = (int16_t) y;
	}
}

#endif
