/*
 * modem.h -- PairPhone's pseudo-voice BPSK modem, the TX step after the
 * voice-frame crypt (tx.c:271 Modulate) and the RX step before it
 * (rx.c:294-297 Demodulate), restated per channel with explicit state.
 *
 *   modem_tx_bits   the 90 transmitted bits of one packet: 81 payload bits
 *                   in 9 symbols of 9 + a parity bit (even, odd for the
 *                   last symbol), interleaved bit-major (modem/modem.c:147-162)
 *   modem_sample    one 48 kHz output sample: 36 samples per bit of a
 *                   1333 Hz carrier, the bit's waveform picked by the ISI
 *                   (bit changed) and anti-VAD muting (every other packet)
 *                   flags, first half-period halved (:163-166)
 *   modem_demod     one Demodulate call (:186-637): carrier phase search by
 *                   square-wave correlation over 24 periods, 6 bits by
 *                   correlation against 4 adaptive equaliser tables, block
 *                   synchronisation from the parity pattern (90 lag
 *                   metrics), per-symbol parity FEC flipping the weakest bit
 *
 * The reference computes the demodulator in float with double-precision
 * constants (ffg *= 0.95 is a double multiply rounded to float, ...); the
 * restatement performs the same operations in the same order and precision,
 * with contraction into FMAs disabled, so it is bit-exact with the
 * reference's x86-64 (SSE) build.  State = the reference's file statics
 * (modem.c:48-73) per channel.
 */
#ifndef MELPE_MODEM_H
#define MELPE_MODEM_H

#include <stdint.h>
#include <math.h>

#ifndef MODEM_FN
#define MODEM_FN static inline
#endif

/* dword view of int16 sample rows (aliases them) */
typedef uint32_t modem_u32a __attribute__((__may_alias__));

#define MODEM_BITS 90
#define MODEM_PKT_SAMPLES 3240	/* 90 bits x 36 samples at 48 kHz */
#define MODEM_BLOCK_SAMPLES 216	/* one Demodulate call: 6 bits */
#define MODEM_LOOKAHEAD 1080	/* rx.c:246: samples that must be buffered per call */

struct ModemState {
	/* Modulate (modem.c:67-68) */
	int32_t lastb, vadtr;
	/* Demodulate (modem.c:48-65) */
	uint32_t r[9], rr, dr;
	int32_t lag, cnt, u, cq;
	float fr[MODEM_BITS], fd[MODEM_BITS];
	float mlag, qq, f180, falign;
	float ffg[4][36];
	int8_t oldq, blk, lock, align;
};

/* the waveform table, modem.c:76-122: {normal, shaped, muted, shaped and
 * muted} x {bit 0, bit 1}; the shaped+muted rows are the shaped ones / 2 in
 * C integer division */
MODEM_FN int modem_wave(int idx, int ii)
{
	/* half-periods: the second half of each row is the negated first, except
	 * the two -8000 / -4000 entries of the normal and muted rows (index 33 of
	 * bit 0, 15 of bit 1), which the table spells with one unit more */
	static const int16_t normal[18] = {0, 2778, 5472, 7999, 10284, 12256, 13856, 15035, 15756,
					    16000, 15756, 15035, 13856, 12256, 10284, 7999, 5472, 2778};
	static const int16_t shaped[18] = {0, 244, 965, 2144, 3744, 5716, 8001, 10528, 13222,
					    16000, 13222, 10528, 8001, 5716, 3744, 2144, 965, 244};
	static const int16_t muted[18] = {0, 1389, 2736, 3999, 5142, 6128, 6928, 7517, 7878,
					   8000, 7878, 7517, 6928, 6128, 5142, 3999, 2736, 1389};
	int bit = idx & 1, kind = idx >> 1;	/* 0 normal, 1 shaped, 2 muted, 3 both */
	int h = ii < 18 ? ii : ii - 18;
	int v;
	if (kind == 1 || kind == 3)
		v = shaped[h];
	else if (kind == 0)
		v = normal[h];
	else
		v = muted[h];
	int neg = (ii >= 18) ^ bit;	/* bit 0 starts positive */
	if (neg)
		v = -v;
	/* the asymmetric spellings of the table: index 15 of the negative half
	 * of bit 1 / index 33 of bit 0 read -8000 (normal) and -4000 (muted)
	 * where the mirror gives -7999 / -3999 */
	if (h == 15 && neg && (kind == 0 || kind == 2))
		v -= 1;
	if (kind == 3)
		v /= 2;		/* C division: toward zero */
	return v;
}

/* transmitted bit t (0..89) of packet `data` (modem.c:147-162) */
MODEM_FN int modem_tx_bit(const uint8_t *data, int t)
{
	int i = t / 9, j = t - 9 * (t / 9);	/* bit i of symbol j */
	if (i < 9) {
		int k = j * 9 + i;
		return (data[k >> 3] >> (k & 7)) & 1;
	}
	int p = (j == 8);	/* parity: odd for the last symbol only */
	for (int m = 0; m < 9; m++) {
		int k = j * 9 + m;
		p ^= (data[k >> 3] >> (k & 7)) & 1;
	}
	return p;
}

/* output sample s (0..3239) given the packet's bit t, the previous bit and
 * the packet's muting flag (modem.c:163-166) */
MODEM_FN int16_t modem_sample(int b, int prev, int vadtr, int ii)
{
	int idx = b + ((b ^ prev) ? 2 : 0) + (vadtr ? 4 : 0);
	int v = modem_wave(idx, ii);
	if (ii < 18)
		v /= 2;
	return (int16_t) v;
}

MODEM_FN void modem_reset(ModemState *s)
{
	uint8_t *p = (uint8_t *) s;
	for (unsigned i = 0; i < sizeof(ModemState); i++)
		p[i] = 0;
	s->align = 1;		/* modem.c:64-65 */
	s->falign = 50.0f;
}

/* float op helpers in the reference's precision: x *= <double constant> is
 * a double multiply rounded to float, f += fabs(x) a double add */
MODEM_FN float fmul_d(float x, double c) { return (float) ((double) x * c); }
/* a float division, correctly rounded on both targets (a double quotient
 * rounded to float is the correctly rounded float quotient) */
MODEM_FN float fdiv(float a, float b) { return (float) ((double) a / (double) b); }

/* one Demodulate call (modem.c:186-637): `frame` = the caller's sample
 * pointer (at least MODEM_LOOKAHEAD samples valid), data[12] in/out;
 * returns the samples consumed */
MODEM_FN int modem_demod(ModemState *S, const int16_t *frame, uint8_t *data)
{
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
	const int16_t *sp = frame + 9;
	int q = 0;
	/* carrier phase: |x[k] - x[k+18]| summed over 24 periods per offset.
	 * Integer sums, so the order is free: period by period, the period's
	 * 54 samples read as 27 sample pairs (dword loads from the even sample
	 * at or below sp, realigned by one sample when sp is odd), the 36
	 * offsets' sums kept in registers. */
	{
		int e[36];
		for (int j = 0; j < 36; j++)
			e[j] = 0;
		const int odd = (int) (((uintptr_t) sp >> 1) & 1);
		/* the even sample at or below sp: 4-byte aligned (int16 rows) */
		const modem_u32a *bw = (const modem_u32a *) (sp - odd);
		for (int i = 0; i < 24; i++) {
			uint32_t dw[28], v[27];
			for (int t = 0; t < 28; t++) {
				/* the 28th dword (odd starts only) is within the
				 * window: sp[881] is the last sample read below */
				dw[t] = (t < 27 || odd) ? bw[18 * i + t] : 0u;
			}
			for (int t = 0; t < 27; t++)
				v[t] = odd ? (dw[t] >> 16) | (dw[t + 1] << 16) : dw[t];
			for (int j = 0; j < 36; j++) {
				const uint32_t a = v[j >> 1], c = v[(j + 18) >> 1];
				const int x0 = (int16_t) ((j & 1) ? a >> 16 : a);
				const int x1 = (int16_t) ((j & 1) ? c >> 16 : c);
				const int d = x0 - x1;
				e[j] += d < 0 ? -d : d;
			}
		}
		int best = 0;
		for (int j = 0; j < 36; j++)
			if (e[j] > best) {
				best = e[j];
				q = j;
			}
	}
	S->f180 = fmul_d(S->f180, 0.9);
	if (q > 17) {
		q -= 18;
		S->f180 -= 1.0f;
	} else {
		S->f180 += 1.0f;
	}
	if (fabsf(S->f180) < 1.0f) {
		if (S->lock)
			for (int i = 0; i < MODEM_BITS; i++)
				S->fr[i] = 0.0f;
		S->lock = 0;
	} else if (fabsf(S->f180) > 9.0f) {
		S->lock = 1;
	}
	q -= 9;
	if (S->f180 < 0.0f)
		sp += 18;
	sp += q;
	S->qq = fmul_d(S->qq, 0.999);
	S->mlag = fmul_d(S->mlag, 0.99);
	if (S->oldq == q) {
		S->qq += 1.0f;
	} else {
		S->oldq = (int8_t) q;
		S->mlag += (float) q;
	}
	S->cq += q;	/* kk / the jitter filter are dead in the reference (:297) */

	data[11] &= 0x7F;
	int lastbit = 0, pp = 0;
	for (int k = 0; k < 6; k++) {
		const int16_t *x = sp + k * 36;
		int u = 504 * S->u;
		for (int i = 0; i < 36; i++)
			u += x[i];
		u = u / 540;
		S->u = u;
		float spn[36];
		for (int i = 0; i < 36; i++)
			spn[i] = (float) (x[i] - u);
		float g0 = 0.0f, g1 = 0.0f;
		for (int i = 0; i < 36; i++)
			g0 += spn[i] * S->ffg[0][i];
		for (int i = 0; i < 36; i++)
			g0 -= spn[i] * S->ffg[1][i];
		for (int i = 0; i < 36; i++)
			g1 += spn[i] * S->ffg[2][i];
		for (int i = 0; i < 36; i++)
			g1 -= spn[i] * S->ffg[3][i];
		if (fabsf(g1) > fabsf(g0))
			g0 = g1;
		int b = g0 >= 0.0f ? 0 : 1;
		int t = b + ((lastbit ^ b) << 1);	/* table of this bit */
		float f = 0.0f;
		for (int i = 0; i < 36; i++) {
			float w = fmul_d(S->ffg[t][i], 0.95);
			w += (float) (x[i] - u);
			S->ffg[t][i] = w;
			f = (float) ((double) f + fabs((double) w));
		}
		f = fdiv(f, 48.0f);
		if (f == 0.0f)
			f = 1.0f;
		g0 = fdiv(g0, f);
		lastbit = b;
		S->dr = (S->dr << 1) | (uint32_t) b;

		/* block synchronisation from the parity pattern */
		int j = S->cnt * 6 + k;
		int sym = j % 9;
		S->r[sym] = (S->r[sym] << 1) | (uint32_t) b;
		uint32_t p = 0x3FFu & S->r[sym];
		p ^= p >> 1;
		p ^= p >> 2;
		p ^= p >> 4;
		p ^= p >> 8;
		S->rr = (S->rr << 1) | (p & 1u);
		S->fr[j] = fmul_d(S->fr[j], S->lock ? 0.999 : 0.99);
		if (S->rr & 1u) {
			uint32_t z = S->rr;
			for (int m = 0; m < 8; m++) {
				z >>= 1;
				if (!(z & 1u))
					S->fr[j] += 1.0f;
			}
		}
		int pos = (j - S->lag) - 1;
		if (pos < 0)
			pos += 90;
		/* soft bit: correlation over the bit's energy (newalgos, :453-458) */
		int64_t ge = 0;
		for (int i = 0; i < 36; i++)
			ge = (int64_t) ((float) ge + spn[i] * spn[i]);
		ge = (int64_t) sqrt((double) ge);
		if (ge < 1)
			ge = 1;
		S->fd[pos] = fdiv(g0, (float) ge);

		if (j == S->lag) {	/* last bit of the block: output it */
			for (int i = 0; i < 12; i++)
				data[i] = 0;
			int kk = 0, bb = 0;
			for (int ii = 0; ii < 9; ii++) {
				float fm = 100000.0f;
				int par = (ii == 8);
				for (int jj = 0; jj < 10; jj++) {
					float v = S->fd[jj * 9 + ii];
					int hb = v > 0.0f;
					if (fabsf(v) <= fm) {
						fm = fabsf(v);
						pp = kk;
					}
					if (jj < 9) {
						if (hb)
							data[kk >> 3] ^= (uint8_t) (1u << (kk & 7));
						par ^= hb;
						kk++;
					} else if (hb != par) {
						bb++;
						if (pp != kk)
							data[pp >> 3] ^= (uint8_t) (1u << (pp & 7));
					}
				}
			}
			data[11] = (uint8_t) bb;
			S->falign = fmul_d(S->falign, 0.9);
			S->falign += (float) bb;
			if (S->falign > 40.0f && S->align) {
				S->align = 0;
				for (int i = 0; i < MODEM_BITS; i++)
					S->fr[i] = 0.0f;
				for (int i = 0; i < 36; i++) {
					S->ffg[0][i] = (float) modem_wave(0, i);
					S->ffg[1][i] = (float) modem_wave(1, i);
					S->ffg[2][i] = S->ffg[0][i];
					S->ffg[3][i] = S->ffg[1][i];
				}
			} else if (S->falign < 30.0f && !S->align) {
				S->align = 1;
			}
			if (!S->blk) {
				data[11] |= 0x80;
				S->blk = 1;
			}
		}
	}
	S->cnt++;
	if (S->cnt >= 15) {
		S->cnt = 0;
		float fm = 0.0f;
		for (int i = 0; i < MODEM_BITS; i++)
			if (fm < S->fr[i]) {
				fm = S->fr[i];
				S->lag = i;
			}
		if (!S->blk)
			data[11] |= 0x8F;
		else
			S->blk = 0;
	}
	data[10] = (uint8_t) (data[10] + (S->lag << 1));
	if (S->align)
		data[11] |= 0x40;
	if (S->lock)
		data[11] |= 0x20;
	if (S->qq > 50.0f)
		data[11] |= 0x10;
	return MODEM_BLOCK_SAMPLES + q;
}

#endif
