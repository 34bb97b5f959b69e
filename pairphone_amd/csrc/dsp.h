/*
 * dsp.h -- DSP / vector / math / LPC / FFT library of the MELPe engine.
 *
 * Restates, with the same fixed-point arithmetic, melpe/dsp_sub.c,
 * melpe/mat_lib.c, melpe/math_lib.c, melpe/lpc_lib.c and melpe/fft_lib.c.
 * Every routine runs on one lane (one channel) of a wavefront; the caller
 * supplies all state explicitly (there are no statics: the reference's lazily
 * computed tables live in g_der, see tables.h).  Heap scratch of the
 * reference (v_get, melpe/mat_lib.c:578) becomes fixed-size locals.
 */
#ifndef MELPE_DSP_H
#define MELPE_DSP_H

#include "ops.h"
#include "tables.h"

namespace mlp {

/*
 * Paired int16 streams.  The lane's private segment is swizzled per dword
 * (kern.h), so a 16-bit scratch load costs one VMEM instruction and one
 * 256-byte row of the wave, exactly like a 32-bit load.  P16 reads an int16
 * stream p[0], p[1], ... two samples per dword load, which halves the VMEM
 * instructions (and the rows fetched) of a pass.  A stream that starts at an
 * odd sample -- a per-lane property, since offsets such as the pitch lag
 * differ between channels -- is re-aligned with one byte permute.  The
 * values and their order are unchanged, so every L_mac chain below is the
 * reference's.
 */
MD uint32_t perm_b32(uint32_t hi, uint32_t lo, uint32_t sel)
{
#if defined(__HIP_DEVICE_COMPILE__)
	return __builtin_amdgcn_perm(hi, lo, sel);
#else
	uint64_t v = ((uint64_t) hi << 32) | lo;
	uint32_t r = 0;
	for (int k = 0; k < 4; k++)
		r |= (uint32_t) ((v >> (8 * ((sel >> (8 * k)) & 7))) & 0xff) << (8 * k);
	return r;
#endif
}

struct P16 {
	const u32_alias *w;
	uint32_t prev, sel;
};

/* Opens the stream p[0..n) and returns how many pairs p16_next may deliver:
 * n / 2 for an even start, (n - 1) / 2 for an odd one (whose last dword
 * would straddle the end).  No byte outside p[0..n) is read, so no access
 * leaves the array the stream lies in; the caller takes the remaining one
 * to three samples one by one. */
MD int p16_open(P16 &r, const int16_t *p, int n)
{
	int odd = (int) ((reinterpret_cast<uintptr_t>(p) >> 1) & 1);
	r.w = reinterpret_cast<const u32_alias *>(p + odd);
	r.prev = (odd && n > 0) ? (uint32_t) (uint16_t) p[0] << 16 : 0u;
	r.sel = odd ? 0x05040302u : 0x07060504u;
	int np = (n - odd) >> 1;
	return np > 0 ? np : 0;
}

/* the next two samples: p[2k] in the low half, p[2k + 1] in the high half */
MD uint32_t p16_next(P16 &r)
{
	uint32_t cur = *r.w++;
	uint32_t v = perm_b32(cur, r.prev, r.sel);
	r.prev = cur;
	return v;
}

MD int16_t lo16(uint32_t v) { return (int16_t) (v & 0xffffu); }
MD int16_t hi16(uint32_t v) { return (int16_t) (v >> 16); }

/*
 * Exact correlation sums on packed pairs.  Where a caller has proved that a
 * saturating L_mac chain cannot clamp (every partial sum of |2ab|, in any
 * order, stays within 32 bits), the chain equals the plain integer sum, which
 * may then be formed in any order: two products per v_dot2_i32_i16 instead
 * of a mul and two clamped adds per product.
 */
MD int32_t sdot2(uint32_t a, uint32_t b, int32_t c)	/* c + a.lo*b.lo + a.hi*b.hi */
{
#if defined(__HIP_DEVICE_COMPILE__)
	typedef short v2s __attribute__((ext_vector_type(2)));
	return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, a), __builtin_bit_cast(v2s, b), c,
				      false);
#else
	return (int32_t) ((uint32_t) c + (uint32_t) ((int32_t) lo16(a) * lo16(b)) +
			  (uint32_t) ((int32_t) hi16(a) * hi16(b)));
#endif
}

/* c + a.lo*b.lo + a.hi*b.hi, saturated to 32 bits (the clamp bit) */
MD int32_t sdot2_sat(uint32_t a, uint32_t b, int32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
	typedef short v2s __attribute__((ext_vector_type(2)));
	return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, a), __builtin_bit_cast(v2s, b), c,
				      true);
#else
	int64_t v = (int64_t) c + (int64_t) lo16(a) * lo16(b) + (int64_t) hi16(a) * hi16(b);
	return v > LW_MAX_ ? LW_MAX_ : (v < LW_MIN_ ? LW_MIN_ : (int32_t) v);
#endif
}

/* the pair one sample later: (lo's high half, hi's low half) */
/* both int16 halves of v shifted left by s (0 <= s < 16), each in its own
 * half (v_pk_lshlrev_b16); callers guarantee no half overflows */
MD uint32_t pk_shl16(uint32_t v, int s)
{
#if defined(__HIP_DEVICE_COMPILE__)
	typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
	u16x2 x = __builtin_bit_cast(u16x2, v);
	u16x2 y = x << (u16x2) {(uint16_t) s, (uint16_t) s};
	return __builtin_bit_cast(uint32_t, y);
#else
	return ((uint32_t) (uint16_t) ((v & 0xffffu) << s)) | ((uint32_t) (uint16_t) ((v >> 16) << s) << 16);
#endif
}

MD uint32_t pair_mid(uint32_t hi, uint32_t lo)
{
#if defined(__HIP_DEVICE_COMPILE__)
	return __builtin_amdgcn_alignbit(hi, lo, 16);
#else
	return (lo >> 16) | (hi << 16);
#endif
}

/* x = 256 * hi8(x) + lo8(x) per half: hi8 signed (arithmetic >> 8), lo8 in
 * [0, 255] -- products with an int16 then fit 23 bits, so up to 256 of them
 * sum exactly in 32 */
MD uint32_t pk_hi8(uint32_t x)
{
#if defined(__HIP_DEVICE_COMPILE__)
	typedef short v2s __attribute__((ext_vector_type(2)));
	return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2s, x) >> (v2s) {8, 8});
#else
	return (uint32_t) (uint16_t) (lo16(x) >> 8) | ((uint32_t) (uint16_t) (hi16(x) >> 8) << 16);
#endif
}
MD uint32_t pk_lo8(uint32_t x) { return x & 0x00ff00ffu; }

/*
 * Pair streams for the exact correlators.  PairStream p[0..n) yields the
 * pairs (p[2m], p[2m+1]), m < ceil(n/2), p[n] taken as 0 when n is odd.
 * Raw dword d of the stream is the d-th aligned dword from p (p + 1 for an
 * odd start); those wholly inside p[0..n) are "full", the one holding the
 * last sample alone is the "partial" one, read as a 16-bit load.  Pair m is
 * raw dword m (even start) or the perm of raw m and m - 1 (odd start, raw
 * -1 being p[0] << 16).  Nothing outside p[0..n) is read.
 */
struct PairStream {
	const u32_alias *w;
	uint32_t sel, prev0, partial;
	int nfull;
};
MD void ps_open(PairStream &s, const int16_t *p, int n)
{
	int odd = (int) ((reinterpret_cast<uintptr_t>(p) >> 1) & 1);
	s.w = reinterpret_cast<const u32_alias *>(p + odd);
	s.sel = odd ? 0x05040302u : 0x07060504u;
	s.prev0 = odd ? (uint32_t) (uint16_t) p[0] << 16 : 0u;
	s.nfull = odd ? (n - 1) >> 1 : n >> 1;
	s.partial = (odd ^ (n & 1)) ? (uint32_t) (uint16_t) p[n - 1] : 0u;
}
/* raw dword d >= 0, any d: full ones loaded (index clamped, so the load is
 * always inside), the partial one and anything past it selected */
MD uint32_t ps_raw(const PairStream &s, int d)
{
	int c = d < s.nfull ? d : s.nfull - 1;
	uint32_t v = s.w[c > 0 ? c : 0];
	v = d < s.nfull ? v : (d == s.nfull ? s.partial : 0u);
	return d < 0 ? s.prev0 : v;
}
/* four consecutive pairs m0 .. m0 + 3 (m0 >= 1), loads issued together */
MD void ps_pairs4(const PairStream &s, int m0, uint32_t *out)
{
	uint32_t r[5];
	#pragma unroll
	for (int i = 0; i < 5; i++)
		r[i] = ps_raw(s, m0 - 1 + i);
	#pragma unroll
	for (int i = 0; i < 4; i++)
		out[i] = perm_b32(r[i + 1], r[i], s.sel);
}
/* pairs 0 .. N-1 (N small), loads issued together */
template <int N>
MD void ps_head(const PairStream &s, uint32_t *out)
{
	uint32_t r[N > 0 ? N : 1];
	#pragma unroll
	for (int i = 0; i < N; i++)
		r[i] = ps_raw(s, i);
	#pragma unroll
	for (int i = 0; i < N; i++)
		out[i] = perm_b32(r[i], i ? r[i - 1] : s.prev0, s.sel);
}
/* full four-dword groups available from pair m0 on */
MD int ps_full_groups(const PairStream &s, int m0)
{
	int g = (s.nfull - m0) >> 2;
	return g > 0 ? g : 0;
}

/* Chunks of four full raw dwords (pairs m0 + 4c .. m0 + 4c + 3), PD chunks
 * in flight: next4() returns chunk c and issues the load of chunk c + PD
 * (past the last chunk the last one is re-read, never a dword outside). */
template <int PD>
struct P16C {
	const u32_alias *w;
	uint32_t prev, sel;
	uint32_t buf[PD][4];
	int next, last;
};
template <int PD>
MD void p16c_load(P16C<PD> &s, uint32_t *d)
{
	int c = s.next < s.last ? s.next : s.last;
	const u32_alias *q = s.w + 4 * c;
	d[0] = q[0];
	d[1] = q[1];
	d[2] = q[2];
	d[3] = q[3];
	s.next++;
}
template <int PD>
MD void p16c_open(P16C<PD> &s, const PairStream &ps, int m0, int nchunks)
{
	s.w = ps.w + m0;
	s.prev = m0 > 0 ? ps.w[m0 - 1] : ps.prev0;
	s.sel = ps.sel;
	s.next = 0;
	s.last = nchunks - 1;
	if (nchunks > 0)
		#pragma unroll
		for (int d = 0; d < PD; d++)
			p16c_load(s, s.buf[d]);
}
template <int PD>
MD void p16c_next4(P16C<PD> &s, uint32_t *out)
{
	uint32_t raw[4];
	#pragma unroll
	for (int i = 0; i < 4; i++)
		raw[i] = s.buf[0][i];
	#pragma unroll
	for (int d = 0; d + 1 < PD; d++)
		#pragma unroll
		for (int i = 0; i < 4; i++)
			s.buf[d][i] = s.buf[d + 1][i];
	p16c_load(s, s.buf[PD - 1]);
	#pragma unroll
	for (int i = 0; i < 4; i++)
		out[i] = perm_b32(raw[i], i ? raw[i - 1] : s.prev, s.sel);
	s.prev = raw[3];
}

#ifndef MELPE_XC_PD
#define MELPE_XC_PD 2
#endif

/*
 * K lag sums of one block, exactly: out[k] = sum_{j<len} pa[j + S::oa(k)] *
 * pb[j + S::ob(k)], 0 <= oa < S::NA, 0 <= ob < S::NB.  Reads pa[0 .. len +
 * NA - 1) and pb[0 .. len + NB - 1) only.  The sums must fit 32 bits (the
 * caller's bound); with SPLIT the a samples are split as 256 * hi8 + lo8 and
 * the two 32-bit halves returned separately (hi in out[k], lo in out[K + k]),
 * for sums that only fit 40 bits.
 *
 * Steps t take j = 2t, 2t + 1 from windows of pairs: a pair at an even
 * offset o is window entry o / 2, one at an odd offset the pair_mid of two
 * neighbours.  Steps go four at a time, each group refilling the windows
 * with four pairs per stream: full chunks prefetched ahead (P16C), the last
 * groups through clamped loads with the steps past the end masked off.  Only
 * an odd len leaves one j, summed sample by sample.
 */
template <int K, class S, bool SPLIT>
MD void xcorr_pairs(const int16_t *pa, const int16_t *pb, int len, int32_t *out)
{
	constexpr int NA = S::NA, NB = S::NB;
	constexpr int MA = NA / 2 + 1, MB = NB / 2 + 1;	/* pairs a step reads */
	constexpr int NH = SPLIT ? 2 : 1;
	constexpr int PD = MELPE_XC_PD;
	int32_t acc[NH * K];
	#pragma unroll
	for (int k = 0; k < NH * K; k++)
		acc[k] = 0;
	const int T = len >> 1;
	int jt = 0;	/* first j of the sample-by-sample tail */
	if (T >= 4) {
		PairStream sa, sb;
		ps_open(sa, pa, len + NA - 1);
		ps_open(sb, pb, len + NB - 1);
		/* windows of steps 4g .. 4g + 3: pairs (and mids) */
		uint32_t wa[NH][MA + 3], ma[NH][MA + 3], wb[MB + 3], mb[MB + 3];
		auto put_a = [&](int m, uint32_t x) {
			wa[0][m] = SPLIT ? pk_hi8(x) : x;
			if (SPLIT)
				wa[NH - 1][m] = pk_lo8(x);
		};
		{
			uint32_t ha[MA], hb[MB];
			ps_head<MA - 1>(sa, ha);
			ps_head<MB - 1>(sb, hb);
			#pragma unroll
			for (int m = 0; m < MA - 1; m++)
				put_a(m, ha[m]);
			#pragma unroll
			for (int m = 0; m < MB - 1; m++)
				wb[m] = hb[m];
		}
		#pragma unroll
		for (int m = 0; m + 1 < MA - 1; m++)
			#pragma unroll
			for (int h = 0; h < NH; h++)
				ma[h][m] = pair_mid(wa[h][m + 1], wa[h][m]);
		#pragma unroll
		for (int m = 0; m + 1 < MB - 1; m++)
			mb[m] = pair_mid(wb[m + 1], wb[m]);
		/* one group: the four new pairs xa/xb, steps st < nst */
		auto group = [&](const uint32_t *xa, const uint32_t *xb, int nst) {
			#pragma unroll
			for (int i = 0; i < 4; i++) {
				put_a(MA - 1 + i, xa[i]);
				wb[MB - 1 + i] = xb[i];
			}
			#pragma unroll
			for (int m = MA - 2; m < MA + 2; m++)
				#pragma unroll
				for (int h = 0; h < NH; h++)
					if (m >= 0)
						ma[h][m] = pair_mid(wa[h][m + 1], wa[h][m]);
			#pragma unroll
			for (int m = MB - 2; m < MB + 2; m++)
				if (m >= 0)
					mb[m] = pair_mid(wb[m + 1], wb[m]);
			#pragma unroll
			for (int st = 0; st < 4; st++)
				#pragma unroll
				for (int k = 0; k < K; k++) {
					const int oa = S::oa(k), ob = S::ob(k);
					const int ia = st + (oa >> 1), ib = st + (ob >> 1);
					uint32_t y = (ob & 1) ? mb[ib] : wb[ib];
					#pragma unroll
					for (int h = 0; h < NH; h++) {
						uint32_t x = (oa & 1) ? ma[h][ia] : wa[h][ia];
						int32_t v = sdot2(x, y, acc[h * K + k]);
						acc[h * K + k] = st < nst ? v : acc[h * K + k];
					}
				}
			#pragma unroll
			for (int m = 0; m < MA - 1; m++)
				#pragma unroll
				for (int h = 0; h < NH; h++) {
					wa[h][m] = wa[h][m + 4];
					if (m < MA - 2)
						ma[h][m] = ma[h][m + 4];
				}
			#pragma unroll
			for (int m = 0; m < MB - 1; m++) {
				wb[m] = wb[m + 4];
				if (m < MB - 2)
					mb[m] = mb[m + 4];
			}
		};
		int G = T >> 2, ga = ps_full_groups(sa, MA - 1), gb = ps_full_groups(sb, MB - 1);
		G = G < ga ? G : ga;
		G = G < gb ? G : gb;
		if (G > 0) {
			P16C<PD> ca, cb;
			p16c_open(ca, sa, MA - 1, G);
			p16c_open(cb, sb, MB - 1, G);
			#pragma unroll 1
			for (int g = 0; g < G; g++) {
				uint32_t xa[4], xb[4];
				p16c_next4(ca, xa);
				p16c_next4(cb, xb);
				group(xa, xb, 4);
			}
		}
		#pragma unroll 1
		for (int t = 4 * G; t < T; t += 4) {
			uint32_t xa[4], xb[4];
			ps_pairs4(sa, MA - 1 + t, xa);
			ps_pairs4(sb, MB - 1 + t, xb);
			group(xa, xb, T - t);
		}
		jt = 2 * T;
	}
	/* an odd len's last j (or a short len's every j), sample by sample */
	for (int j = jt; j < len; j++) {
		#pragma unroll
		for (int k = 0; k < K; k++) {
			int x = pa[j + S::oa(k)], y = pb[j + S::ob(k)];
			if (SPLIT) {
				acc[k] += (x >> 8) * y;
				acc[K + k] += (x & 0xff) * y;
			} else {
				acc[k] += x * y;
			}
		}
	}
	#pragma unroll
	for (int k = 0; k < NH * K; k++)
		out[k] = acc[k];
}

/* find_pitch's lag blocks (fp_corrK below): lag n0 + k reads
 * pa[j + (k + 1) / 2] * pb[j + (k + 1) / 2 - k + BMAX], BMAX = (K - 1) - K / 2 */
template <int K>
struct FpLags {
	static constexpr int BMAX = (K - 1) - K / 2;
	static constexpr int NA = K / 2 + 1, NB = BMAX + 1;
	static constexpr int oa(int k) { return (k + 1) / 2; }
	static constexpr int ob(int k) { return (k + 1) / 2 - k + BMAX; }
};

/* sum of squares, exactly (caller's bound) */
MD int32_t magsq_pairs(const int16_t *p, int n)
{
	int32_t acc0 = 0, acc1 = 0;
	P16 r;
	int np = p16_open(r, p, n);
	int i = 0;
	#pragma unroll 4
	for (int k = 0; k < np; k++, i += 2) {
		uint32_t x = p16_next(r);
		if (k & 1)
			acc1 = sdot2(x, x, acc1);
		else
			acc0 = sdot2(x, x, acc0);
	}
	for (; i < n; i++)
		acc0 += (int32_t) p[i] * p[i];
	return acc0 + acc1;
}

/* L_mac chain of shr(a[i], sh) squared, i = 0 .. n-1, read straight from
 * a[] in pairs: L_v_magsq (mat_lib.c:358) of the shifted copy the reference
 * builds with v_equ_shr, without writing it; equal to L_v_magsq(tb, n, 0,
 * 1) (final shift 0), and to L_v_magsq(tb, n, 0, 0) once shifted right by 1
 * (decoder scale_adj, analysis gain_ana) */
MD Word32 magsq_shr(const int16_t *a, int n, Word16 sh)
{
	Word32 acc = 0;
	P16 ra;
	int np = p16_open(ra, a, n);
	int i = 0;
#pragma unroll 8
	for (int k = 0; k < np; k++, i += 2) {
		uint32_t x = p16_next(ra);
		const Word16 t0 = shr(lo16(x), sh), t1 = shr(hi16(x), sh);
		acc = L_mac(acc, t0, t0);
		acc = L_mac(acc, t1, t1);
	}
	for (; i < n; i++) {
		const Word16 t = shr(a[i], sh);
		acc = L_mac(acc, t, t);
	}
	return acc;
}

/* ------------------------------------------------------------------ */
/* vectors: melpe/mat_lib.c                                           */
/* ------------------------------------------------------------------ */

/* d[i] = f(s[i]), i ascending: samples read in pairs (P16), written as
 * dwords after a one-sample head when d starts at an odd sample.  A
 * destination overlapping the source from above (d in (s, s + n)) gets the
 * plain loop: there the forward order is what the reference's smearing
 * copy produces. */
template <class F>
MD void v_map(int16_t *d, const int16_t *s, int n, F f)
{
	if (d > s && d < s + n) {
		for (int i = 0; i < n; i++)
			d[i] = f(s[i]);
		return;
	}
	int i = 0;
	if (n > 0 && ((reinterpret_cast<uintptr_t>(d) >> 1) & 1)) {
		d[0] = f(s[0]);
		i = 1;
	}
	P16 r;
	int np = p16_open(r, s + i, n - i);
	u32_alias *dw = reinterpret_cast<u32_alias *>(d + i);
	auto put = [&](uint32_t x) {
		uint32_t y0 = (uint16_t) f(lo16(x));	/* f may carry state: */
		uint32_t y1 = (uint16_t) f(hi16(x));	/* sample order matters */
		*dw++ = y0 | (y1 << 16);
	};
	/* four pairs loaded before any is stored: the stores may alias the
	 * source (in place, or d below s), so the compiler could not hoist the
	 * next loads over them; reading ahead is safe for both cases */
	int k = 0;
	for (; k + 4 <= np; k += 4, i += 8) {
		uint32_t x0 = p16_next(r), x1 = p16_next(r), x2 = p16_next(r), x3 = p16_next(r);
		put(x0);
		put(x1);
		put(x2);
		put(x3);
	}
	for (; k < np; k++, i += 2)
		put(p16_next(r));
	for (; i < n; i++)
		d[i] = f(s[i]);
}

#ifndef MELPE_VMAP_COPY
#define MELPE_VMAP_COPY 0
#endif
#ifndef MELPE_VMAP_IIR
#define MELPE_VMAP_IIR 0
#endif

/* out[i] = f(i, in[i]) for i = 0 .. n-1, in order, the inputs loaded a block
 * ahead of the outputs stored.  A plain loop over scratch arrays waits for
 * every load: the compiler cannot move a load above the previous store when
 * the two arrays may overlap, so each element costs a full memory round
 * trip.  Here the loads of in[i + B .. i + 2B) are issued before out[i .. i
 * + B) is stored, one wait per block.  Valid when out and in are disjoint,
 * the same array, or out lies below in (a shift down: every in[j] is read
 * before out[j] can overwrite it); a copy upward into an overlapping range
 * runs element by element, as the reference's forward loop. */
#ifndef MELPE_VBATCH_PAIRS
#define MELPE_VBATCH_PAIRS 1
#endif
template <int B = 8, class F>
MD void v_batch(const int16_t *in, int16_t *out, int n, F f)
{
	int i = 0;
#if MELPE_VBATCH_PAIRS
	/* Paired form: the private segment is interleaved per dword across the
	 * wave, so a 2-byte access costs the vector memory pipeline as much as a
	 * 4-byte one.  Inputs come two per dword (P16, any alignment), B / 2
	 * dwords a block ahead; outputs go out as dwords after a one-sample head
	 * when out starts at an odd sample.  Same order of f calls, same
	 * overlap rules (reads run ahead of writes by at least a block). */
	if (n >= 2 * B + 1 && !(out > in && out < in + n)) {
		constexpr int Q = B / 2;
		if ((reinterpret_cast<uintptr_t>(out) >> 1) & 1) {
			out[0] = f(0, in[0]);
			i = 1;
		}
		P16 r;
		const int np = p16_open(r, in + i, n - i);
		u32_alias *dw = reinterpret_cast<u32_alias *>(out + i);
		if (np >= 2 * Q) {
			uint32_t v[Q];
			#pragma unroll
			for (int q = 0; q < Q; q++)
				v[q] = p16_next(r);
			int k = 0;
			#pragma unroll 1
			for (; k + 2 * Q <= np; k += Q) {
				uint32_t nv[Q];
				#pragma unroll
				for (int q = 0; q < Q; q++)
					nv[q] = p16_next(r);
				#pragma unroll
				for (int q = 0; q < Q; q++) {
					const uint32_t y0 = (uint16_t) f(i + 2 * q, lo16(v[q]));
					const uint32_t y1 = (uint16_t) f(i + 2 * q + 1, hi16(v[q]));
					dw[k + q] = y0 | (y1 << 16);
				}
				i += 2 * Q;
				#pragma unroll
				for (int q = 0; q < Q; q++)
					v[q] = nv[q];
			}
			#pragma unroll
			for (int q = 0; q < Q; q++) {
				const uint32_t y0 = (uint16_t) f(i + 2 * q, lo16(v[q]));
				const uint32_t y1 = (uint16_t) f(i + 2 * q + 1, hi16(v[q]));
				dw[k + q] = y0 | (y1 << 16);
			}
			i += 2 * Q;
			k += Q;
			for (; k < np; k++, i += 2) {
				const uint32_t x = p16_next(r);
				const uint32_t y0 = (uint16_t) f(i, lo16(x));
				const uint32_t y1 = (uint16_t) f(i + 1, hi16(x));
				dw[k] = y0 | (y1 << 16);
			}
		} else {
			for (int k = 0; k < np; k++, i += 2) {
				const uint32_t x = p16_next(r);
				const uint32_t y0 = (uint16_t) f(i, lo16(x));
				const uint32_t y1 = (uint16_t) f(i + 1, hi16(x));
				dw[k] = y0 | (y1 << 16);
			}
		}
	}
#else
	if (n >= 2 * B && !(out > in && out < in + n)) {
		int16_t v[B];
		#pragma unroll
		for (int q = 0; q < B; q++)
			v[q] = in[q];
		#pragma unroll 1
		for (; i + 2 * B <= n; i += B) {
			int16_t nv[B];
			#pragma unroll
			for (int q = 0; q < B; q++)
				nv[q] = in[i + B + q];
			#pragma unroll
			for (int q = 0; q < B; q++)
				out[i + q] = f(i + q, v[q]);
			#pragma unroll
			for (int q = 0; q < B; q++)
				v[q] = nv[q];
		}
		#pragma unroll
		for (int q = 0; q < B; q++)
			out[i + q] = f(i + q, v[q]);
		i += B;
	}
#endif
	for (; i < n; i++)
		out[i] = f(i, in[i]);
}

MD void v_copy(int16_t *d, const int16_t *s, int n)	/* v_equ :136 */
{
#if MELPE_VMAP_COPY
	v_map(d, s, n, [](int16_t x) { return x; });
#else
	v_batch(s, d, n, [](int, int16_t x) { return x; });
#endif
}

MD void v_copy32(int32_t *d, const int32_t *s, int n)	/* L_v_equ :237 */
{
	for (int i = 0; i < n; i++)
		d[i] = s[i];
}

MD void v_zero(int16_t *d, int n)	/* v_zap :567 */
{
	for (int i = 0; i < n; i++)
		d[i] = 0;
}

MD void v_set(int16_t *d, int16_t val, int n)	/* fill dsp_sub.c:87 */
{
	for (int i = 0; i < n; i++)
		d[i] = val;
}

MD void v_add(int16_t *a, const int16_t *b, int n)	/* :87 */
{
	for (int i = 0; i < n; i++)
		a[i] = add(a[i], b[i]);
}

MD void v_sub(int16_t *a, const int16_t *b, int n)	/* :520 */
{
	for (int i = 0; i < n; i++)
		a[i] = sub(a[i], b[i]);
}

MD void v_equ_shr(int16_t *d, const int16_t *s, int16_t sc, int n)	/* :186 */
{
#if MELPE_VMAP_COPY
	v_map(d, s, n, [sc](int16_t x) { return (int16_t) shr(x, sc); });
#else
	v_batch(s, d, n, [sc](int, int16_t x) { return (int16_t) shr(x, sc); });
#endif
}

MD void v_scale(int16_t *a, int16_t sc, int n)	/* :409 */
{
#if MELPE_VMAP_COPY
	v_map(a, a, n, [sc](int16_t x) { return (int16_t) mult(x, sc); });
#else
	v_batch(a, a, n, [sc](int, int16_t x) { return (int16_t) mult(x, sc); });
#endif
}

MD void v_scale_shl(int16_t *a, int16_t sc, int n, int16_t sh)	/* :462 */
{
	for (int i = 0; i < n; i++)
		a[i] = extract_h(L_shl(L_mult(a[i], sc), sh));
}

/* L_v_inner :293 -- sum of products, then shift to the output Q.  The
 * samples come in pairs (P16) and the unrolled body issues a batch of loads
 * before the saturating (order dependent, so strictly sequential)
 * accumulation consumes them. */
MN Word32 L_v_inner(const int16_t *__restrict__ a, const int16_t *__restrict__ b, int n,
		    int16_t qa, int16_t qb, int16_t qout)
{
	Word32 acc = 0;
	P16 ra, rb;
	int np = p16_open(ra, a, n), nb = p16_open(rb, b, n);
	np = np < nb ? np : nb;
	int i = 0;
#pragma unroll 8
	for (int k = 0; k < np; k++, i += 2) {
		uint32_t x = p16_next(ra), y = p16_next(rb);
		acc = L_mac(acc, lo16(x), lo16(y));
		acc = L_mac(acc, hi16(x), hi16(y));
	}
	for (; i < n; i++)
		acc = L_mac(acc, a[i], b[i]);
	return L_shl(acc, sub(qout, add(add(qa, qb), 1)));
}

/* L_v_magsq :352 */
MN Word32 L_v_magsq(const int16_t *__restrict__ a, int n, int16_t qa, int16_t qout)
{
	Word32 acc = 0;
	P16 ra;
	int np = p16_open(ra, a, n);
	int i = 0;
#pragma unroll 8
	for (int k = 0; k < np; k++, i += 2) {
		uint32_t x = p16_next(ra);
		acc = L_mac(acc, lo16(x), lo16(x));
		acc = L_mac(acc, hi16(x), hi16(x));
	}
	for (; i < n; i++)
		acc = L_mac(acc, a[i], a[i]);
	return L_shl(acc, sub(sub(qout, shl(qa, 1)), 1));
}

/* ------------------------------------------------------------------ */
/* math: melpe/math_lib.c                                             */
/* ------------------------------------------------------------------ */

/* L_divider2 :105 -- signed 32/32 -> Q15 division through divide_s */
MN Word16 L_divider2(Word32 num, Word32 den, int16_t nsh, int16_t dsh)
{
	bool neg = (num < 0) != (den < 0);
	int16_t k = 0;
	Word32 d = L_abs(L_shl(den, dsh));
	Word32 nn = L_abs(L_shr(num, nsh));
	while (d > (Word32) SW_MAX_) {
		d = L_shr(d, 1);
		k = add(k, 1);
	}
	nn = L_shr(nn, k);
	Word16 q = divide_s(extract_l(nn), extract_l(d));
	return neg ? negate(q) : q;
}

/* The fixed-point math tables (log10_fxp, L_log10_fxp, pow10_fxp) from an
 * LDS copy (MELPE_MATH_LDS, the NPP kernels: their per-bin log / pow
 * lookups gather at per-lane indices, from constant memory a global-memory
 * round trip each), else from the table blob */
#define MOFF_pow10_q_table 0
#define MOFF_pow10_tens_table (MOFF_pow10_q_table + TLEN_pow10_q_table)
#define MOFF_log_table (MOFF_pow10_tens_table + TLEN_pow10_tens_table)
#define MOFF_pow10_table (MOFF_log_table + TLEN_log_table)
#define MTAB_WORDS (MOFF_pow10_table + TLEN_pow10_table)	/* 526 */
#if defined(MELPE_MATH_LDS) && defined(__HIP__)
extern __shared__ int16_t s_mtab[];
#define TBM(name) ((const int16_t *) (s_mtab + MOFF_##name))
#else
#define TBM(name) TB(name)
#endif
/* word i of the packed copy: the four tables end to end */
MD int mtab_src(int i)
{
	return i < MOFF_pow10_tens_table ? TOFF_pow10_q_table + i
	       : i < MOFF_log_table	 ? TOFF_pow10_tens_table + (i - MOFF_pow10_tens_table)
	       : i < MOFF_pow10_table	 ? TOFF_log_table + (i - MOFF_log_table)
					 : TOFF_pow10_table + (i - MOFF_pow10_table);
}

/* log10_fxp :169 */
MN Word16 log10_fxp(Word16 x, Word16 Q)
{
	const int16_t *lt = TBM(log_table);
	Word16 sh = sub(7, Q);
	if (!x)
		return (Word16) -SW_MAX_;
	Word16 i2 = shr(x, 7);
	while (!i2 && x) {
		x = shl(x, 1);
		sh = sub(sh, 1);
		i2 = shr(x, 7);
	}
	Word16 i1 = sub(i2, 1);
	Word16 frac = shl((Word16) (x & 127), 8);
	Word16 ic = mult(sub(lt[i2], lt[i1]), frac);
	Word32 acc = L_shr(L_mult(lt[1], sh), 2);
	Word16 t = add(shr(lt[i1], 1), extract_l(acc));
	return add(t, shr(ic, 1));
}

/* L_log10_fxp :242 */
MN Word16 L_log10_fxp(Word32 x, Word16 Q)
{
	const int16_t *lt = TBM(log_table);
	Word16 sh = sub(23, Q);
	if (!x)
		return (Word16) -SW_MAX_;
	Word16 i2 = extract_l(L_shr(x, 23));
	while (!i2 && x) {
		x = L_shl(x, 1);
		sh = sub(sh, 1);
		i2 = extract_l(L_shr(x, 23));
	}
	Word16 i1 = sub(i2, 1);
	Word32 frac = L_shl(x & (Word32) 0x7fffff, 8);
	Word16 ic = extract_h(L_mpy_ls(frac, sub(lt[i2], lt[i1])));
	Word32 acc = L_shr(L_mult(lt[1], sh), 3);
	Word16 t = add(shr(lt[i1], 2), extract_l(acc));
	return add(t, shr(ic, 2));
}

/* pow10_fxp :308 */
MN Word16 pow10_fxp(Word16 x, Word16 Q)
{
	const int16_t *tab = TBM(pow10_table);
	const int16_t *tens = TBM(pow10_tens_table);
	const int16_t *qt = TBM(pow10_q_table);
	Word16 tm = shr(x, 12);
	if (tm < -4)
		return 0;
	if (tm > 4)
		return SW_MAX_;
	Word16 i1 = shr((Word16) (x & 0x0ff0), 4);
	Word16 i2 = add(i1, 1);
	Word16 frac = shl((Word16) (x & 0x000f), 11);
	Word16 ic = mult(sub(tab[i2], tab[i1]), frac);
	Word16 m = add(tab[i1], ic);
	Word16 ti = add(tm, 4);
	Word32 y = L_mult(tens[ti], m);
	if (tm >= 0) {
		y = L_shr(y, sub(12, Q));
		Word16 r = extract_l(y);
		if (extract_h(y))
			r = SW_MAX_;
		return r;
	}
	return extract_l(L_shr(y, sub(add(qt[ti], 12), Q)));
}

MD Word16 sqrt_fxp(Word16 x, Word16 Q)	/* :432 */
{
	if (!x)
		return 0;
	return pow10_fxp(shr(log10_fxp(x, Q), 1), Q);
}

MD Word16 L_sqrt_fxp(Word32 x, Word16 Q)	/* :471 (no halving: as the reference) */
{
	if (!x)
		return 0;
	return pow10_fxp(L_log10_fxp(x, Q), Q);
}

MD Word16 L_pow_fxp(Word32 x, Word16 pw, Word16 qin, Word16 qout)	/* :517 */
{
	if (!x)
		return 0;
	Word16 t = L_log10_fxp(x, qin);
	t = mult(pw, shl(t, 1));
	return pow10_fxp(t, qout);
}

/* sin_fxp :556 / cos_fxp :643 -- quarter-wave table interpolation */
MD Word16 sin_fxp(Word16 x)
{
	const int16_t *tab = TB(sin_table);
	bool neg = x < 0;
	Word16 tx = neg ? negate(x) : x;
	if (tx > 16384)
		tx = sub(SW_MAX_, tx);
	Word16 i1 = shr(tx, 7);
	if (i1 == 128)
		return neg ? negate(tab[i1]) : tab[i1];
	Word16 m = shl(sub(tx, shl(i1, 7)), 8);
	Word16 y = add(tab[i1], mult(m, sub(tab[i1 + 1], tab[i1])));
	return neg ? negate(y) : y;
}

MD Word16 cos_fxp(Word16 x)
{
	const int16_t *tab = TB(cos_table);
	bool neg = false;
	Word16 tx = x < 0 ? negate(x) : x;
	if (tx > 16384) {
		tx = sub(SW_MAX_, tx);
		neg = true;
	}
	Word16 i1 = shr(tx, 7);
	if (i1 == 128)
		return 0;
	Word16 m = shl(sub(tx, shl(i1, 7)), 8);
	Word16 y = add(tab[i1], mult(m, sub(tab[i1 + 1], tab[i1])));
	return neg ? negate(y) : y;
}

/* sqrt_Q15 :733 -- Taylor series square root of a Q15 value */
MN Word16 sqrt_Q15(Word16 x)
{
	if (x == 0)
		return 0;
	Word32 A = L_deposit_h(x);
	Word16 sh = norm_l(A);
	A = L_shl(A, sh);
	bool odd = (sh & 1) != 0;
	sh = negate(shl(sh, -1));
	A = L_shl(A, -1);
	A = L_sub(A, L_deposit_h(0x4000));
	Word16 x2 = extract_h(A);
	A = L_add(A, L_deposit_h(0x4000));
	A = L_add(A, L_deposit_h(0x4000));
	Word32 t = L_mult(x2, x2);
	t = -t;
	A = L_add(A, L_shl(t, -1));
	t = L_mult((Word16) L_shl(t, -16), (Word16) L_shl(t, -16));
	Word16 x24 = extract_h(t);
	A = L_sub(A, L_mult(x24, 0x5000));
	A = L_add(A, L_mult(0x7000, mult(x24, x2)));
	Word32 cube = L_mult(mult(x2, x2), x2);
	A = L_add(A, L_shl(cube, -1));
	A = L_add(A, L_shl(0x80, 8));
	if (odd) {
		A = L_mult((Word16) L_shl(A, -16), 0x5A82);
		A = L_add(A, L_shl(0x80, 8));
	}
	A = L_shl(A, sh);
	return extract_h(A);
}

MD Word16 add_shr(Word16 a, Word16 b)	/* :781 */
{
	return (Word16) L_shr(L_add(L_deposit_l(a), L_deposit_l(b)), 1);
}

/* ------------------------------------------------------------------ */
/* filters and helpers: melpe/dsp_sub.c                               */
/* ------------------------------------------------------------------ */

/* envelope :62 -- rectify + 2nd-order smoother; out[-1], out[-2] are history */
MN void envelope(const int16_t *in, int16_t prev_in, int16_t *out, int n)
{
	/* the two past outputs ride in registers (out may be in: in[i] is
	 * always read before out[i] is written, as in the reference); the
	 * inputs come a block ahead (v_batch) */
	Word16 pa = abs_s(prev_in), y1 = out[-1], y2 = out[-2];
	v_batch(in, out, n, [&](int, int16_t x) {
		Word16 ca = abs_s(x);
		Word32 acc = L_shr(L_deposit_h(sub(ca, pa)), 5);
		acc = L_mac(acc, 31565, y1);
		acc = L_mac(acc, -15415, y2);
		Word16 y = r_ound(L_shl(acc, 1));
		y2 = y1;
		y1 = y;
		pa = ca;
		return y;
	});
}

/* envelope, returning the exact energy (sum of L_mult(y, y)) of what it
 * wrote, for f_pitch_scale_e (bpvc_ana); lsh > 0: the input is in[i]
 * scaled up by 2^lsh, the caller having proved no sample overflows
 * (bpvc_band_s) */
MD int64_t envelope_e(const int16_t *in, int16_t prev_in, int16_t *out, int n, int lsh = 0)
{
	PROF_SCOPE(48);
	Word16 pa = abs_s(prev_in), y1 = out[-1], y2 = out[-2];
	int64_t e = 0;
	const int m = 1 << lsh;
	v_batch(in, out, n, [&](int, int16_t x) {
		Word16 ca = abs_s((int16_t) (x * m));
		Word32 acc = L_shr(L_deposit_h(sub(ca, pa)), 5);
		acc = L_mac(acc, 31565, y1);
		acc = L_mac(acc, -15415, y2);
		Word16 y = r_ound(L_shl(acc, 1));
		e += L_mult(y, y);
		y2 = y1;
		y1 = y;
		pa = ca;
		return y;
	});
	return e;
}

/* interp_array :113 */
MD void interp_array(const int16_t *prev, const int16_t *curr, int16_t *out,
		     int16_t f, int n)
{
	if (f == 0) {
		v_copy(out, prev, n);
	} else if (f == SW_MAX_) {
		v_copy(out, curr, n);
	} else {
		Word16 f2 = sub(SW_MAX_, f);
		for (int i = 0; i < n; i++)
			out[i] = add(mult(f, curr[i]), mult(f2, prev[i]));
	}
}

MD Word16 interp_scalar(Word16 prev, Word16 curr, Word16 f)	/* :697 */
{
	Word16 o;
	interp_array(&prev, &curr, &o, f, 1);
	return o;
}

MD Word16 median3(const int16_t *in)	/* :136 */
{
	Word16 lo = Min_(in[0], in[1]), hi = Max_(in[0], in[1]), t = in[2];
	if (t < lo)
		return lo;
	if (t > hi)
		return hi;
	return t;
}

/* Bit packer state: pack_code :160 / unpack_code :485 write/read LSB first,
 * wsize bits per byte. */
struct BitCursor {
	unsigned char *p;
	int16_t bit;
};

MD void pack_code(Word16 code, BitCursor *c, int16_t nbits, int16_t wsize)
{
	for (int i = 0; i < nbits; i++) {
		Word16 b = (Word16) (code & 1);
		if (c->bit == 0)
			*c->p = (unsigned char) b;
		else
			*c->p |= (unsigned char) shl(b, c->bit);
		c->bit = add(c->bit, 1);
		if (c->bit >= wsize) {
			c->bit = 0;
			c->p++;
		}
		code = shr(code, 1);
	}
}

MD int16_t unpack_code(BitCursor *c, Word16 *code, int16_t nbits, int16_t wsize,
		       uint16_t erase_mask)
{
	Word16 v = 0;
	int16_t ret = (int16_t) (*c->p & erase_mask);
	for (int i = 0; i < nbits; i++) {
		Word16 bit = c->bit;
		v |= shl(shr((Word16) ((Word16) *c->p & shl(1, bit)), bit), (Word16) i);
		c->bit = add(c->bit, 1);
		if (c->bit >= wsize) {
			c->bit = 0;
			c->p++;
		}
	}
	*code = v;
	if (c->bit != 0)
		ret |= *c->p & erase_mask;
	return ret;
}

/* peakiness :200 -- L2/L1 ratio of a residual, Q11 */
MN Word16 peakiness(const int16_t *in, int n)
{
	int16_t tb[512];
	Word16 sc = 4;
	v_equ_shr(tb, in, sc, n);
	Word32 e = L_v_magsq(tb, n, 0, 1);
	if (e) {
		sc = sub(sc, shr(norm_l(e), 1));
		if (sc < 0)
			sc = 0;
	} else {
		sc = 0;
	}
	Word32 sabs = 0;
	for (int i = 0; i < n; i++)
		sabs = L_add(sabs, L_deposit_l(abs_s(in[i])));
	if (sc)
		v_equ_shr(tb, in, sc, n);
	if (sabs <= 0)
		return 0;
	e = sc ? L_v_magsq(tb, n, 0, 0) : L_v_magsq(in, n, 0, 0);
	e = L_deposit_l(L_sqrt_fxp(e, 0));
	Word16 pf = L_divider2(e, sabs, 0, 0);
	if (pf > 20723)
		return SW_MAX_;
	Word16 s1 = add(sc, 5);
	Word16 rn = sqrt_fxp(shl((Word16) n, 7), 7);
	return extract_h(L_shl(L_mult(pf, rn), s1));
}

/* quant_u :259 -- uniform scalar quantiser, returns the index */
MN void quant_u(int16_t *val, int16_t *idx, Word16 qmin, Word16 qmax,
		Word16 nlev, Word16 nlev_q, bool dbl, Word16 scale)
{
	Word16 step = divide_s(sub(qmax, qmin), nlev_q);
	int16_t i;
	if (dbl) {
		Word32 Lstep = L_deposit_l(step);
		Word32 Lhalf = L_shr(Lstep, 1);
		Word32 Lb = L_add(L_shl(L_deposit_l(qmin), scale), Lhalf);
		Word32 Lin = L_shl(L_deposit_l(*val), scale);
		for (i = 0; i < nlev; i++) {
			if (Lin < Lb)
				break;
			Lb = L_add(Lb, Lstep);
		}
		*val = extract_l(L_shr(L_sub(Lb, Lhalf), scale));
	} else {
		step = shr(step, scale);
		Word16 half = shr(step, 1);
		Word16 b = add(qmin, half);
		for (i = 0; i < nlev; i++) {
			if (*val < b)
				break;
			b = add(b, step);
		}
		*val = sub(b, half);
	}
	*idx = i;
}

/* quant_u_dec :318 */
MD Word16 quant_u_dec(Word16 idx, Word16 qmin, Word16 qmax, Word16 nlev_q, Word16 scale)
{
	Word16 step = divide_s(sub(qmax, qmin), nlev_q);
	Word32 t = L_shr(L_mult(step, idx), 1);
	t = L_add(L_shl(L_deposit_l(qmin), scale), t);
	return extract_l(L_shr(t, scale));
}

/* rand_minstdgen :367 -- Park-Miller minimal standard generator computed
 * with 16x16 products; *seed is the per-channel `next` (initially 1). */
MD Word16 rand_minstdgen(uint32_t *seed)
{
	uint32_t nx = *seed;
	uint16_t x0 = (uint16_t) extract_l((Word32) nx);
	uint16_t x1 = (uint16_t) extract_h((Word32) nx);
	uint32_t p, q, t1, t2, t3;
	t1 = (uint32_t) 16807u * x1;
	p = (uint32_t) L_shr((Word32) t1, 15);
	t1 = (uint32_t) L_shl((Word32) (t1 & 0x00007fff), 16);
	t2 = (uint32_t) 16807u * x0;
	t3 = (uint32_t) L_sub(LW_MAX_, (Word32) t1);
	if (t2 > t3) {
		t1 = (uint32_t) L_sub((Word32) t1, (Word32) 0x7fffffff);
		t1 = (uint32_t) L_sub((Word32) t1, 1);
		q = (uint32_t) L_add((Word32) t1, (Word32) t2);
		p = (uint32_t) L_add((Word32) p, 1);
	} else {
		q = (uint32_t) L_add((Word32) t1, (Word32) t2);
	}
	t3 = (uint32_t) L_sub(LW_MAX_, (Word32) p);
	if (q > t3) {
		t1 = (uint32_t) L_sub((Word32) p, (Word32) 0x7fffffff);
		t1 = (uint32_t) L_add((Word32) t1, (Word32) q);
	} else {
		t1 = (uint32_t) L_add((Word32) p, (Word32) q);
	}
	*seed = t1;
	return (Word16) (uint16_t) extract_h((Word32) t1);
}

MD void rand_num(int16_t *out, Word16 amp, int n, uint32_t *seed)	/* :343 */
{
	for (int i = 0; i < n; i++) {
		Word16 t = sub(rand_minstdgen(seed), 16384);
		out[i] = mult(amp, shl(t, 1));
	}
}

MD void window(const int16_t *in, const int16_t *w, int16_t *out, int n)	/* :532 */
{
	for (int i = 0; i < n; i++)
		out[i] = mult(w[i], in[i]);
}

MD void window_Q(const int16_t *in, const int16_t *w, int16_t *out, int n, Word16 qin)	/* :549 */
{
	Word16 sh = sub(15, qin);
	for (int i = 0; i < n; i++)
		out[i] = extract_h(L_shl(L_mult(w[i], in[i]), sh));
}

/* zerflt :569 / zerflt_Q :591 -- FIR over in[-order..n-1], run backwards so
 * that in == out is allowed.  Coefficients live in registers and four
 * outputs share one sliding window of inputs (each output's sum is still
 * accumulated in the reference's tap order). */
template <int ORDER>
MD void zerflt_q_fixed(const int16_t *in, const int16_t *c, int16_t *out, int n, Word16 sc)
{
	Word16 cf[ORDER + 1];
#pragma unroll
	for (int j = 0; j <= ORDER; j++)
		cf[j] = c[j];
	int i = n - 1;
	for (; i >= 3; i -= 4) {
		Word16 x[ORDER + 4];	/* x[k] = in[i - k] */
#pragma unroll
		for (int k = 0; k < ORDER + 4; k++)
			x[k] = in[i - k];
		Word32 a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
		for (int j = 0; j <= ORDER; j++) {
			a0 = L_mac(a0, x[j], cf[j]);
			a1 = L_mac(a1, x[j + 1], cf[j]);
			a2 = L_mac(a2, x[j + 2], cf[j]);
			a3 = L_mac(a3, x[j + 3], cf[j]);
		}
		out[i] = r_ound(L_shl(a0, sc));
		out[i - 1] = r_ound(L_shl(a1, sc));
		out[i - 2] = r_ound(L_shl(a2, sc));
		out[i - 3] = r_ound(L_shl(a3, sc));
	}
	for (; i >= 0; i--) {
		Word32 acc = 0;
#pragma unroll
		for (int j = 0; j <= ORDER; j++)
			acc = L_mac(acc, in[i - j], cf[j]);
		out[i] = r_ound(L_shl(acc, sc));
	}
}

/* long FIR (the decoder's 65-tap dispersion filter): eight outputs share a
 * sliding window of eight inputs, one new load per tap; each output keeps
 * the reference's tap-order L_mac chain */
MD void zerflt_q_long(const int16_t *in, const int16_t *c, int16_t *out, int order, int n,
		      Word16 sc)
{
	int i = n - 1;
	for (; i >= 7; i -= 8) {
		Word16 w0 = in[i], w1 = in[i - 1], w2 = in[i - 2], w3 = in[i - 3];
		Word16 w4 = in[i - 4], w5 = in[i - 5], w6 = in[i - 6], w7 = in[i - 7];
		Word32 a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
		for (int j = 0; j <= order; j++) {
			Word16 cj = c[j];
			a0 = L_mac(a0, w0, cj);
			a1 = L_mac(a1, w1, cj);
			a2 = L_mac(a2, w2, cj);
			a3 = L_mac(a3, w3, cj);
			a4 = L_mac(a4, w4, cj);
			a5 = L_mac(a5, w5, cj);
			a6 = L_mac(a6, w6, cj);
			a7 = L_mac(a7, w7, cj);
			w0 = w1;
			w1 = w2;
			w2 = w3;
			w3 = w4;
			w4 = w5;
			w5 = w6;
			w6 = w7;
			if (j < order)	/* no read below in[-order] */
				w7 = in[i - 8 - j];
		}
		out[i] = r_ound(L_shl(a0, sc));
		out[i - 1] = r_ound(L_shl(a1, sc));
		out[i - 2] = r_ound(L_shl(a2, sc));
		out[i - 3] = r_ound(L_shl(a3, sc));
		out[i - 4] = r_ound(L_shl(a4, sc));
		out[i - 5] = r_ound(L_shl(a5, sc));
		out[i - 6] = r_ound(L_shl(a6, sc));
		out[i - 7] = r_ound(L_shl(a7, sc));
	}
	for (; i >= 0; i--) {
		Word32 acc = 0;
		for (int j = 0; j <= order; j++)
			acc = L_mac(acc, in[i - j], c[j]);
		out[i] = r_ound(L_shl(acc, sc));
	}
}

/* the decoder's dispersion FIR (ORDER = DISP_ORD): eight outputs per block,
 * the block's ORDER + 8 inputs loaded together up front (one memory wait per
 * block instead of one per tap).  With no coefficient at MIN16 -- checked
 * on entry -- L_mult(x, c) is x * 2c exactly, so each tap of an output's
 * chain is one 24-bit multiply and one saturating add, in the reference's
 * tap order. */
template <int ORDER>
MD bool zerflt_q_blk8(const int16_t *in, const int16_t *c, int16_t *out, int n, Word16 sc)
{
	bool ok = true;
	for (int j = 0; j <= ORDER; j++)
		ok &= c[j] != SW_MIN_;
	if (!ok)
		return false;
	int i = n - 1;
#pragma unroll 1
	for (; i >= 7; i -= 8) {
		int16_t w[ORDER + 8];	/* w[k] = in[i - k] */
#pragma unroll
		for (int k = 0; k < ORDER + 8; k++)
			w[k] = in[i - k];
		Word32 a[8];
#pragma unroll
		for (int q = 0; q < 8; q++)
			a[q] = 0;
#pragma unroll
		for (int j = 0; j <= ORDER; j++) {
			const int32_t c2 = 2 * (int32_t) c[j];
#pragma unroll
			for (int q = 0; q < 8; q++)
				a[q] = sat_add32(a[q], (int32_t) w[j + q] * c2);
		}
#pragma unroll
		for (int q = 0; q < 8; q++)
			out[i - q] = r_ound(L_shl(a[q], sc));
	}
	for (; i >= 0; i--) {
		Word32 acc = 0;
		for (int j = 0; j <= ORDER; j++)
			acc = L_mac(acc, in[i - j], c[j]);
		out[i] = r_ound(L_shl(acc, sc));
	}
	return true;
}

MN void zerflt_Q(const int16_t *in, const int16_t *c, int16_t *out, int order,
		 int n, Word16 qc)
{
	PROF_SCOPE(28);
	Word16 sc = sub(15, qc);
	if (order >= 16) {
#if !defined(MELPE_OPCOUNT)
		if (order == 64 && zerflt_q_blk8<64>(in, c, out, n, sc))	/* DISP_ORD */
			return;
#endif
		zerflt_q_long(in, c, out, order, n, sc);
		return;
	}
	if (order == 10) {
		zerflt_q_fixed<10>(in, c, out, n, sc);
		return;
	}
	if (order == 1) {
		zerflt_q_fixed<1>(in, c, out, n, sc);
		return;
	}
	for (int i = n - 1; i >= 0; i--) {
		Word32 acc = 0;
		for (int j = 0; j <= order; j++)
			acc = L_mac(acc, in[i - j], c[j]);
		out[i] = r_ound(L_shl(acc, sc));
	}
}

MD void zerflt(const int16_t *in, const int16_t *c, int16_t *out, int order, int n)
{
	zerflt_Q(in, c, out, order, n, 12);
}

/* iir_2nd_d :615 -- biquad with a double-precision (hi/lo) output memory;
 * coefficients and memories held in registers across the block */
MN void iir_2nd_d(const int16_t *in, const int16_t *den, const int16_t *num,
		  int16_t *out, int16_t *din, int16_t *dhi, int16_t *dlo, int n)
{
	PROF_SCOPE(26);
	const Word16 d1 = den[1], d2 = den[2], n0 = num[0], n1 = num[1], n2 = num[2];
	Word16 i0 = din[0], i1 = din[1], h0 = dhi[0], h1 = dhi[1], l0 = dlo[0], l1 = dlo[1];
	for (int i = 0; i < n; i++) {
		Word16 x = shr(in[i], 1);
		Word32 acc = L_mult(l0, d1);
		acc = L_mac(acc, l1, d2);
		acc = L_shr(acc, 14);
		acc = L_mac(acc, h0, d1);
		acc = L_mac(acc, h1, d2);
		acc = L_mac(acc, x, n0);
		acc = L_mac(acc, i0, n1);
		acc = L_mac(acc, i1, n2);
		acc = L_shl(acc, 2);
		i1 = i0;
		i0 = x;
		h1 = h0;
		l1 = l0;
		h0 = extract_h(acc);
		l0 = (Word16) (shr(extract_l(acc), 2) & 0x3FFF);
		out[i] = r_ound(L_shl(acc, 1));
	}
	din[0] = i0;
	din[1] = i1;
	dhi[0] = h0;
	dhi[1] = h1;
	dlo[0] = l0;
	dlo[1] = l1;
}

/* iir_2nd_s :660 -- biquad, single precision memories */
MN void iir_2nd_s(const int16_t *in, const int16_t *den, const int16_t *num,
		  int16_t *out, int16_t *din, int16_t *dout, int n)
{
	PROF_SCOPE(27);
	const Word16 d1 = den[1], d2 = den[2], n0 = num[0], n1 = num[1], n2 = num[2];
	Word16 i0 = din[0], i1 = din[1], o0 = dout[0], o1 = dout[1];
	for (int i = 0; i < n; i++) {
		Word16 x = in[i];
		Word32 acc = L_mult(x, n0);
		acc = L_mac(acc, i0, n1);
		acc = L_mac(acc, i1, n2);
		acc = L_mac(acc, o0, d1);
		acc = L_mac(acc, o1, d2);
		acc = L_shl(acc, 2);
		i1 = i0;
		i0 = x;
		Word16 y = r_ound(acc);
		out[i] = y;
		o1 = o0;
		o0 = y;
	}
	din[0] = i0;
	din[1] = i1;
	dout[0] = o0;
	dout[1] = o1;
}

/* One biquad step of iir_2nd_s (single-precision memories), the section
 * state in registers. */
struct Biq {
	Word16 n0, n1, n2, d1, d2, i0, i1, o0, o1;
};

MD Word16 biq_step(Biq &b, Word16 x)
{
	Word32 acc = L_mult(x, b.n0);
	acc = L_mac(acc, b.i0, b.n1);
	acc = L_mac(acc, b.i1, b.n2);
	acc = L_mac(acc, b.o0, b.d1);
	acc = L_mac(acc, b.o1, b.d2);
	acc = L_shl(acc, 2);
	b.i1 = b.i0;
	b.i0 = x;
	Word16 y = r_ound(acc);
	b.o1 = b.o0;
	b.o0 = y;
	return y;
}

/* Three cascaded iir_2nd_s sections (section s: den + 3s, num + 3s, memories
 * din/dout[2s..2s+1]) run in place on x[0..n), sample by sample.  Section s
 * at sample i depends only on section s-1 at samples <= i and on its own
 * past, so this equals the reference's three sequential in-place calls.
 * Samples move in blocks of 4 (loads issued together, one wait per block;
 * MELPE_VMAP_IIR: in pairs through v_map, measured slower).
 * snap > 0 (a multiple of 4): the memories left behind are those after
 * sample snap-1 -- the reference's filter-then-save-then-restore around a
 * two-part call (melp_ana.c:324-346, pit_lib.c:604-622). */
MD void iir3_s(int16_t *x, const int16_t *den, const int16_t *num, int16_t *din, int16_t *dout,
	       int n, int snap)
{
	Biq b[3];
	for (int s = 0; s < 3; s++) {
		b[s].n0 = num[3 * s];
		b[s].n1 = num[3 * s + 1];
		b[s].n2 = num[3 * s + 2];
		b[s].d1 = den[3 * s + 1];
		b[s].d2 = den[3 * s + 2];
		b[s].i0 = din[2 * s];
		b[s].i1 = din[2 * s + 1];
		b[s].o0 = dout[2 * s];
		b[s].o1 = dout[2 * s + 1];
	}
	Biq keep[3];
#if MELPE_VMAP_IIR
	auto filt = [&](int16_t v) -> int16_t { return biq_step(b[2], biq_step(b[1], biq_step(b[0], v))); };
	if (snap > 0) {
		v_map(x, x, snap, filt);
		for (int s = 0; s < 3; s++)
			keep[s] = b[s];
		v_map(x + snap, x + snap, n - snap, filt);
	} else {
		v_map(x, x, n, filt);
	}
#else
	/* inputs a block ahead (v_batch); the memories after sample snap - 1
	 * are taken as sample snap is about to be filtered */
	v_batch(x, x, n, [&](int i, int16_t v) {
		if (i == snap)
			for (int s = 0; s < 3; s++)
				keep[s] = b[s];
		return biq_step(b[2], biq_step(b[1], biq_step(b[0], v)));
	});
#endif
	for (int s = 0; s < 3; s++) {
		const Biq &o = snap > 0 ? keep[s] : b[s];
		din[2 * s] = o.i0;
		din[2 * s + 1] = o.i1;
		dout[2 * s] = o.o0;
		dout[2 * s + 1] = o.o1;
	}
}

/* iir3_s from in[] to out[] (no snapshot), handing each output to
 * f(i, y) as it is produced (bpvc_ana's fused window pass) */
template <class F>
MD void iir3_s_io(const int16_t *in, int16_t *out, const int16_t *den, const int16_t *num,
		  int16_t *din, int16_t *dout, int n, F f)
{
	Biq b[3];
	for (int s = 0; s < 3; s++) {
		b[s].n0 = num[3 * s];
		b[s].n1 = num[3 * s + 1];
		b[s].n2 = num[3 * s + 2];
		b[s].d1 = den[3 * s + 1];
		b[s].d2 = den[3 * s + 2];
		b[s].i0 = din[2 * s];
		b[s].i1 = din[2 * s + 1];
		b[s].o0 = dout[2 * s];
		b[s].o1 = dout[2 * s + 1];
	}
	/* in place or disjoint: inputs a block ahead of the outputs (v_batch) */
	v_batch(in, out, n, [&](int i, int16_t v) {
		int16_t y = biq_step(b[2], biq_step(b[1], biq_step(b[0], v)));
		f(i, y);
		return y;
	});
	for (int s = 0; s < 3; s++) {
		din[2 * s] = b[s].i0;
		din[2 * s + 1] = b[s].i1;
		dout[2 * s] = b[s].o0;
		dout[2 * s + 1] = b[s].o1;
	}
}

/* One step of iir_2nd_d (double-precision output memory hi/lo) */
struct Biqd {
	Word16 n0, n1, n2, d1, d2, i0, i1, h0, h1, l0, l1;
};

MD Word16 biqd_step(Biqd &b, Word16 in)
{
	Word16 x = shr(in, 1);
	Word32 acc = L_mult(b.l0, b.d1);
	acc = L_mac(acc, b.l1, b.d2);
	acc = L_shr(acc, 14);
	acc = L_mac(acc, b.h0, b.d1);
	acc = L_mac(acc, b.h1, b.d2);
	acc = L_mac(acc, x, b.n0);
	acc = L_mac(acc, b.i0, b.n1);
	acc = L_mac(acc, b.i1, b.n2);
	acc = L_shl(acc, 2);
	b.i1 = b.i0;
	b.i0 = x;
	b.h1 = b.h0;
	b.l1 = b.l0;
	b.h0 = extract_h(acc);
	b.l0 = (Word16) (shr(extract_l(acc), 2) & 0x3FFF);
	return r_ound(L_shl(acc, 1));
}

/* dc_rmv's three cascaded iir_2nd_d sections (melp_sub.c:211-245), in -> out,
 * sample by sample (equal to the reference's three in-place passes),
 * samples in blocks of 4 */
MD void iir3_d(const int16_t *in, int16_t *out, const int16_t *den, const int16_t *num,
	       int16_t *din, int16_t *dhi, int16_t *dlo, int n)
{
	Biqd b[3];
	for (int s = 0; s < 3; s++) {
		b[s].n0 = num[3 * s];
		b[s].n1 = num[3 * s + 1];
		b[s].n2 = num[3 * s + 2];
		b[s].d1 = den[3 * s + 1];
		b[s].d2 = den[3 * s + 2];
		b[s].i0 = din[2 * s];
		b[s].i1 = din[2 * s + 1];
		b[s].h0 = dhi[2 * s];
		b[s].h1 = dhi[2 * s + 1];
		b[s].l0 = dlo[2 * s];
		b[s].l1 = dlo[2 * s + 1];
	}
#if MELPE_VMAP_IIR
	v_map(out, in, n, [&](int16_t v) -> int16_t {
		return biqd_step(b[2], biqd_step(b[1], biqd_step(b[0], v)));
	});
#else
	v_batch(in, out, n, [&](int, int16_t v) {
		return biqd_step(b[2], biqd_step(b[1], biqd_step(b[0], v)));
	});
#endif
	for (int s = 0; s < 3; s++) {
		din[2 * s] = b[s].i0;
		din[2 * s + 1] = b[s].i1;
		dhi[2 * s] = b[s].h0;
		dhi[2 * s + 1] = b[s].h1;
		dlo[2 * s] = b[s].l0;
		dlo[2 * s + 1] = b[s].l1;
	}
}

/* iir3_d from a 4-byte aligned input of n samples (n a multiple of 36), read
 * 18 dwords at a time with every load of a batch issued before the filter
 * uses the first: the input is the caller's PCM in global memory, one
 * channel per lane, where each load waits a full memory latency */
MD void iir3_d_batched(const int16_t *in, int16_t *out, const int16_t *den, const int16_t *num,
		       int16_t *din, int16_t *dhi, int16_t *dlo, int n)
{
	Biqd b[3];
	for (int s = 0; s < 3; s++) {
		b[s].n0 = num[3 * s];
		b[s].n1 = num[3 * s + 1];
		b[s].n2 = num[3 * s + 2];
		b[s].d1 = den[3 * s + 1];
		b[s].d2 = den[3 * s + 2];
		b[s].i0 = din[2 * s];
		b[s].i1 = din[2 * s + 1];
		b[s].h0 = dhi[2 * s];
		b[s].h1 = dhi[2 * s + 1];
		b[s].l0 = dlo[2 * s];
		b[s].l1 = dlo[2 * s + 1];
	}
	const u32_alias *p = (const u32_alias *) in;
	for (int i = 0; i < n; i += 36) {
		uint32_t v[18];
#pragma unroll
		for (int k = 0; k < 18; k++)
			v[k] = p[i / 2 + k];
#pragma unroll
		for (int k = 0; k < 18; k++) {
			out[i + 2 * k] = biqd_step(b[2], biqd_step(b[1], biqd_step(b[0], (int16_t) (v[k] & 0xffff))));
			out[i + 2 * k + 1] = biqd_step(b[2], biqd_step(b[1], biqd_step(b[0], (int16_t) (v[k] >> 16))));
		}
	}
	for (int s = 0; s < 3; s++) {
		din[2 * s] = b[s].i0;
		din[2 * s + 1] = b[s].i1;
		dhi[2 * s] = b[s].h0;
		dhi[2 * s + 1] = b[s].h1;
		dlo[2 * s] = b[s].l0;
		dlo[2 * s + 1] = b[s].l1;
	}
}

MD void biqd_load(Biqd &b, const int16_t *den, const int16_t *num, const int16_t *din,
		  const int16_t *dhi, const int16_t *dlo)
{
	b.n0 = num[0];
	b.n1 = num[1];
	b.n2 = num[2];
	b.d1 = den[1];
	b.d2 = den[2];
	b.i0 = din[0];
	b.i1 = din[1];
	b.h0 = dhi[0];
	b.h1 = dhi[1];
	b.l0 = dlo[0];
	b.l1 = dlo[1];
}

MD void biqd_store(const Biqd &b, int16_t *din, int16_t *dhi, int16_t *dlo)
{
	din[0] = b.i0;
	din[1] = b.i1;
	dhi[0] = b.h0;
	dhi[1] = b.h1;
	dlo[0] = b.l0;
	dlo[1] = b.l1;
}

/* two different iir_2nd_d filters in cascade, in place, sample by sample
 * (postfilter's lpf3500 then hpf60: equal to the two sequential passes) */
MD void iir2_d(int16_t *x, const int16_t *den1, const int16_t *num1, int16_t *din1,
	       int16_t *dhi1, int16_t *dlo1, const int16_t *den2, const int16_t *num2,
	       int16_t *din2, int16_t *dhi2, int16_t *dlo2, int n)
{
	Biqd a, b;
	biqd_load(a, den1, num1, din1, dhi1, dlo1);
	biqd_load(b, den2, num2, din2, dhi2, dlo2);
#if MELPE_VMAP_IIR
	v_map(x, x, n, [&](int16_t v) -> int16_t { return biqd_step(b, biqd_step(a, v)); });
#else
	v_batch(x, x, n, [&](int, int16_t v) { return biqd_step(b, biqd_step(a, v)); });
#endif
	biqd_store(a, din1, dhi1, dlo1);
	biqd_store(b, din2, dhi2, dlo2);
}

/* ------------------------------------------------------------------ */
/* LPC: melpe/lpc_lib.c                                               */
/* ------------------------------------------------------------------ */

#define LPC_ACOR_MAX 16

/* The lag sums of lpc_acor in one pass over the samples: sample i adds
 * w[i] * w[i - j] to lag j (j = 1..ORD), the last ORD samples held in
 * registers.  Each lag's saturating chain still runs in ascending i, as the
 * reference's per-lag loop (lpc_lib.c:146-152); the missing terms of the
 * first ORD samples are L_mac(acc, x, 0), which leaves acc unchanged. */
template <int ORD>
MD void acor_lags(const int16_t *w, int n, Word32 *lags)
{
	Word32 acc[ORD];
	int16_t h[ORD];	/* h[k] = w[i - 1 - k] */
	#pragma unroll
	for (int k = 0; k < ORD; k++) {
		acc[k] = 0;
		h[k] = 0;
	}
	auto step = [&](int16_t x) {
		#pragma unroll
		for (int k = 0; k < ORD; k++)
			acc[k] = L_mac(acc[k], x, h[k]);
		#pragma unroll
		for (int k = ORD - 1; k > 0; k--)
			h[k] = h[k - 1];
		h[0] = x;
	};
	P16 r;
	int np = p16_open(r, w, n);
	int i = 0;
	#pragma unroll 2
	for (int k = 0; k < np; k++, i += 2) {
		uint32_t x = p16_next(r);
		step(lo16(x));
		step(hi16(x));
	}
	for (; i < n; i++)
		step(w[i]);
	#pragma unroll
	for (int k = 0; k < ORD; k++)
		lags[k + 1] = acc[k];
}

/* lpc_acor :93 -- windowed, normalised autocorrelation with lag window */
MN void lpc_acor(const int16_t *in, const int16_t *win, int16_t *r,
		 Word16 hf_corr, int order, int n)
{
	PROF_SCOPE(24);
	const int16_t *lagw = TB(lagw_cof);
	int16_t w[200];
	Word16 nv, sf;
	for (int i = 0; i < n; i++)
		w[i] = mult(win[i], shr(in[i], 4));
	Word32 e = L_v_magsq(w, n, 0, 1);
	if (e) {
		nv = sub(4, shr(norm_l(e), 1));
		if (nv < 0)
			nv = 0;
	} else {
		nv = 0;
	}
	for (int i = 0; i < n; i++)
		w[i] = shr(mult(win[i], in[i]), nv);
	e = L_v_magsq(w, n, 0, 1);
	if (e > 0) {
		nv = sub(norm_l(e), 1);
		e = L_shl(e, nv);
		e = L_add(e, L_mpy_ls(e, hf_corr));
		Word16 t = norm_s(extract_h(e));
		e = L_shl(e, t);
		nv = add(nv, t);
		r[0] = r_ound(e);
		sf = divide_s(16382, r[0]);
		e = L_shl(L_mpy_ls(e, sf), 1);
		r[0] = r_ound(e);
	} else {
		nv = 0;
		r[0] = SW_MAX_;
		sf = 0;
	}
	Word32 lags[LPC_ACOR_MAX + 1];
#if defined(MELPE_OPCOUNT)
	/* census build: the reference's per-lag loops */
	for (int j = 1; j <= order; j++) {
		Word32 acc = 0;
		for (int i = j; i < n; i++)
			acc = L_mac(acc, w[i], w[i - j]);
		lags[j] = acc;
	}
#else
	if (order == 16)
		acor_lags<16>(w, n, lags);
	else
		acor_lags<10>(w, n, lags);
#endif
	for (int j = 1; j <= order; j++) {
		Word32 acc = lags[j];
		acc = L_shl(acc, nv);
		acc = L_shl(L_mpy_ls(acc, sf), 1);
		acc = L_mpy_ls(acc, lagw[j - 1]);
		r[j] = r_ound(acc);
	}
}

/* lpc_aejw :198 -- |A(e^jw)|^2 */
MN Word32 lpc_aejw(const int16_t *lpc, Word16 omega, int order)
{
	if (order == 0)
		return 524288L;
	Word16 cs = cos_fxp(omega);
	Word16 sn = negate(sin_fxp(omega));
	Word16 a = lpc[order - 1];
	Word16 re = shr(mult(cs, a), 3);
	Word16 im = shr(mult(sn, a), 3);
	for (int i = order - 2; i >= 0; i--) {
		re = add(re, shr(lpc[i], 3));
		Word16 t = im;
		im = add(mult(cs, t), mult(sn, re));
		re = sub(mult(cs, re), mult(sn, t));
	}
	re = add(re, 512);
	Word32 m = L_add(L_mult(re, re), L_mult(im, im));
	return m < 54 ? 54 : m;
}

MD void lpc_bwex(const int16_t *lpc, int16_t *aw, Word16 gamma, int order)	/* :271 */
{
	Word16 g = gamma;
	for (int i = 0; i < order; i++) {
		aw[i] = mult(lpc[i], g);
		g = mult(g, gamma);
	}
}

/* lpc_clmp :312 -- sort, then enforce a minimum LSF separation */
MN void lpc_clmp(int16_t *lsp, Word16 delta, int order)
{
	bool unsorted = true;
	for (int j = 0; unsorted && j < 10; j++) {
		unsorted = false;
		for (int i = 0; i < order - 1; i++)
			if (lsp[i] > lsp[i + 1]) {
				Word16 t = lsp[i + 1];
				lsp[i + 1] = lsp[i];
				lsp[i] = t;
				unsorted = true;
			}
	}
	if (unsorted)
		return;
	for (int j = 0; j < 10; j++) {
		for (int i = 0; i < order - 1; i++) {
			Word16 d = sub(lsp[i + 1], lsp[i]);
			if (d >= delta)
				continue;
			Word16 s1, s2;
			s1 = s2 = shr(sub(delta, d), 1);
			if (i == 0 && lsp[i] < delta) {
				s1 = shr(lsp[i], 1);
			} else if (i > 0) {
				Word16 t = sub(lsp[i], lsp[i - 1]);
				if (t < delta)
					s1 = 0;
				else if (t < shl(delta, 1))
					s1 = shr(sub(t, delta), 1);
			}
			if (i == order - 2 && lsp[i + 1] > sub(SW_MAX_, delta)) {
				s2 = shr(sub(SW_MAX_, lsp[i + 1]), 1);
			} else if (i < order - 2) {
				Word16 t = sub(lsp[i + 2], lsp[i + 1]);
				if (t < delta)
					s2 = 0;
				else if (t < shl(delta, 1))
					s2 = shr(sub(t, delta), 1);
			}
			lsp[i] = sub(lsp[i], s1);
			lsp[i + 1] = add(lsp[i + 1], s2);
		}
	}
}

/* lpc_refl2pred :531 */
MD void lpc_refl2pred(const int16_t *refc, int16_t *lpc, int order)
{
	int16_t a1[16];
	for (int i = 0; i < order; i++) {
		lpc[i] = shift_r(refc[i], -3);
		v_copy(a1, lpc, i);
		for (int j = 0; j < i; j++)
			lpc[j] = add(a1[j], mult(refc[i], a1[i - j - 1]));
	}
}

/* lpc_schr :444 -- Schur recursion, returns the prediction error */
MN Word16 lpc_schr(const int16_t *r, int16_t *lpc, int order)
{
	Word32 y1[16], y2[17];
	int16_t refc[16];
	refc[0] = divide_s(abs_s(r[1]), abs_s(r[0]));
	if ((r[1] ^ r[0]) >= 0)
		refc[0] = negate(refc[0]);
	y2[0] = L_deposit_h(r[1]);
	y2[1] = L_add(L_deposit_h(r[0]), L_mult(refc[0], r[1]));
	for (int i = 1; i < order; i++) {
		y1[0] = L_deposit_h(r[i + 1]);
		Word32 acc = L_deposit_h(r[i + 1]);
		for (int j = 0; j < i; j++) {
			y1[j + 1] = L_add(y2[j], L_mpy_ls(acc, refc[j]));
			acc = L_add(acc, L_mpy_ls(y2[j], refc[j]));
		}
		if (acc > y2[i]) {
			v_zero(&refc[i], order - i);
			break;
		}
		Word16 sh = norm_l(y2[i]);
		Word16 t1 = abs_s(extract_h(L_shl(acc, sh)));
		Word16 t2 = abs_s(extract_h(L_shl(y2[i], sh)));
		refc[i] = divide_s(t1, t2);
		if ((acc ^ y2[i]) >= 0)
			refc[i] = negate(refc[i]);
		y2[i + 1] = L_add(y2[i], L_mpy_ls(acc, refc[i]));
		v_copy32(y2, y1, i + 1);
	}
	lpc_refl2pred(refc, lpc, order);
	Word16 alpha = r[0];
	for (int i = 0; i < order; i++)
		alpha = mult(alpha, sub(SW_MAX_, mult(refc[i], refc[i])));
	return alpha;
}

/* lsp_to_freq :626 -- root search of P/Q on a 257-point cosine grid */
MN void lsp_to_freq(const int16_t *lsp, int16_t *freq, int order)
{
	const int16_t *lc = g_der.lsp_cos;
	/* default_w = divide_s(ONE_Q11, order << 10), :654-655 */
	Word16 dw = divide_s(2048, shl((Word16) order, 10));
	Word16 dw0 = shr(dw, 1);
	bool prev_less = true;
	Word32 mag[3];
	Word16 smag[3];
	mag[0] = mag[1] = 0x7fffffff;
	smag[0] = smag[1] = 0x7fff;
	mag[2] = 0;
	smag[2] = 0;
	Word16 p2 = shr((Word16) order, 1);
	Word16 count = 0;
	/* a root's interpolation operands, divided after the scan: lanes find
	 * their roots at different grid points, so dividing at each would run
	 * the divider for the wave at nearly every point.  Only a scan with
	 * exactly p2 roots keeps them (else the defaults below overwrite
	 * freq[0 .. p2)), so later roots need no slot. */
	Word32 rn[6], rd[6];
	int16_t ri[6];
	/* The reference steps the grid index by pc = add(pc, i), wrapping at
	 * 512 (:668-672): term k of point i reads lsp_cos[k*i mod 512], never
	 * saturating (k*i <= 1280).  Those indices are wave-uniform and
	 * independent of the data, so the polynomial values of 8 grid points
	 * are formed first (their 40 table loads issued together), then the
	 * sign-change scan walks them in order. */
#if !defined(MELPE_OPCOUNT)
	/* order 10: the block's 40 grid values from g_lspgrid, twenty dwords
	 * at a wave-uniform address (scalar loads), and the five coefficients
	 * held in registers */
	const bool grid = p2 == 5;
	int16_t cf[6];
	#pragma unroll
	for (int j = 0; j < 6; j++)
		cf[j] = j <= p2 ? lsp[j] : (int16_t) 0;
#endif
	for (int i0 = 0; i0 <= 256; i0 += 8) {
		Word32 accs[8];
#if !defined(MELPE_OPCOUNT)
		if (grid) {
			const u32_alias *gw = reinterpret_cast<const u32_alias *>(g_lspgrid) + 5 * (i0 >> 1);
			uint32_t w[20];
			#pragma unroll
			for (int q = 0; q < 20; q++)
				w[q] = gw[q];
			#pragma unroll
			for (int u = 0; u < 8; u++) {
				Word32 acc = L_mult(cf[5], 8192);
				#pragma unroll
				for (int k = 1; k <= 5; k++) {
					const int n = 5 * u + k - 1;
					const Word16 c = (n & 1) ? hi16(w[n >> 1]) : lo16(w[n >> 1]);
					acc = L_add(acc, L_shr(L_mult(cf[5 - k], c), 1));
				}
				accs[u] = acc;
			}
		} else
#endif
		#pragma unroll
		for (int u = 0; u < 8; u++) {
			int i = i0 + u;
			Word32 acc = L_mult(lsp[p2], 8192);
			for (int j = p2 - 1; j >= 0; j--)
				acc = L_add(acc, L_shr(L_mult(lsp[j], lc[((p2 - j) * i) & 511]), 1));
			accs[u] = acc;
		}
		int nu = (256 - i0 + 1) < 8 ? (256 - i0 + 1) : 8;
		for (int u = 0; u < nu; u++) {
			int i = i0 + u;
			OPC_ADD(OP_add, p2);	/* census: the reference's index steps */
			Word32 acc = accs[u];
			smag[2] = extract_h(acc);
			mag[2] = L_abs(acc);
			if (mag[2] < mag[1]) {
				prev_less = true;
			} else {
				if (prev_less && (smag[0] ^ smag[2]) < 0) {
					if (count < 6) {
						rn[count] = L_shr(L_sub(mag[0], mag[2]), 1);
						rd[count] = L_add(L_sub(mag[0], L_shl(mag[1], 1)), mag[2]);
						ri[count] = (int16_t) i;
					}
					count = add(count, 1);
				}
				prev_less = false;
			}
			mag[0] = mag[1];
			mag[1] = mag[2];
			smag[0] = smag[1];
			smag[1] = smag[2];
		}
	}
	if (count != p2) {
		freq[0] = dw0;
		for (int i = 1; i < p2; i++)
			freq[i] = add(freq[i - 1], dw);
	} else {
		for (int k = 0; k < p2; k++) {
			Word16 t = shr(L_divider2(rn[k], rd[k], 0, 0), 9);
			t = add(shl(sub(ri[k], 1), 6), t);
			freq[k] = divide_s(t, shl(512, 5));
		}
	}
}

/* lpc_pred2lsp :566 */
MN void lpc_pred2lsp(const int16_t *lpc, int16_t *lsf, int order)
{
	PROF_SCOPE(25);
	Word32 Lp[6], Lq[6];
	int16_t pc[6], qc[6], pf[6], qf[6];
	Word16 p2 = shr((Word16) order, 1);
	Lp[0] = Lq[0] = 67108864L;
	for (int i = 1; i <= p2; i++) {
		Word32 ai = L_shr(L_deposit_h(lpc[i - 1]), 2);
		Word32 api = L_shr(L_deposit_h(lpc[order - i]), 2);
		Lp[i] = L_add(L_sub(ai, api), Lp[i - 1]);
		Lq[i] = L_sub(L_add(ai, api), Lq[i - 1]);
	}
	for (int i = 0; i <= p2; i++) {
		pc[i] = r_ound(Lp[i]);
		qc[i] = r_ound(Lq[i]);
	}
	lsp_to_freq(pc, pf, order);
	lsp_to_freq(qc, qf, order);
	for (int i = 0; i < p2; i++) {
		lsf[2 * i] = qf[i];
		lsf[2 * i + 1] = pf[i];
	}
}

/* lpc_pred2refl :751 -- returns the residual energy, *refc = first refl. */
MN Word16 lpc_pred2refl(const int16_t *lpc, int16_t *refc, int order)
{
	int16_t b[16], b1[16];
	Word16 energy = SW_MAX_;
	v_copy(b, lpc, order);
	for (int i = order - 1; i >= 0; i--) {
		if (b[i] >= 4096)
			b[i] = 4095;
		if (b[i] <= -4096)
			b[i] = -4095;
		Word32 acc = L_shl(L_sub(33554431L, L_mult(b[i], b[i])), 6);
		energy = mult(energy, extract_h(acc));
		Word16 sh = norm_l(acc);
		Word16 e = extract_h(L_shl(acc, sh));
		v_copy(b1, b, i);
		for (int j = 0; j < i; j++) {
			acc = L_mult(b[i], b1[i - j - 1]);
			acc = L_sub(L_shl(L_deposit_l(b1[j]), 13), acc);
			Word16 sgn = extract_h(acc);
			acc = L_abs(acc);
			Word16 s1 = norm_l(acc);
			Word16 t = extract_h(L_shl(acc, s1));
			if (t > e) {
				t = shr(t, 1);
				s1 = sub(s1, 1);
			}
			b[j] = divide_s(t, e);
			s1 = sub(sub(s1, 3), sh);
			b[j] = shr(b[j], s1);
			if (sgn < 0)
				b[j] = negate(b[j]);
		}
	}
	*refc = shl(b[0], 3);
	return energy;
}

/* lpc_lsp2pred :827 -- LSF (Q15) to predictor (Q12); clamps lsf in place */
MN void lpc_lsp2pred(int16_t *lsf, int16_t *lpc, int order)
{
	Word32 f0[6], f1[6];
	lpc_clmp(lsf, 0, order);
	Word16 p2 = shr((Word16) order, 1);
	f0[0] = f1[0] = 33554431L;
	f0[1] = L_shr(L_deposit_h(negate(cos_fxp(lsf[0]))), 5);
	f1[1] = L_shr(L_deposit_h(negate(cos_fxp(lsf[1]))), 5);
	int k = 2;
	for (int i = 2; i <= p2; i++) {
		Word16 c0 = negate(cos_fxp(lsf[k++]));
		Word16 c1 = negate(cos_fxp(lsf[k++]));
		f0[i] = f0[i - 2];
		f1[i] = f1[i - 2];
		for (int j = i; j >= 2; j--) {
			f0[j] = L_add(f0[j], L_add(L_shl(L_mpy_ls(f0[j - 1], c0), 1), f0[j - 2]));
			f1[j] = L_add(f1[j], L_add(L_shl(L_mpy_ls(f1[j - 1], c1), 1), f1[j - 2]));
		}
		f0[1] = L_add(f0[1], L_shl(L_mpy_ls(f0[0], c0), 1));
		f1[1] = L_add(f1[1], L_shl(L_mpy_ls(f1[0], c1), 1));
	}
	for (int i = p2 - 1; i >= 0; i--) {
		f0[i + 1] = L_add(f0[i + 1], f0[i]);
		f1[i + 1] = L_sub(f1[i + 1], f1[i]);
		lpc[i] = extract_h(L_shl(L_add(f0[i + 1], f1[i + 1]), 2));
		lpc[order - 1 - i] = extract_h(L_shl(L_sub(f0[i + 1], f1[i + 1]), 2));
	}
}

/* lpc_lsp2pred for order 10 on registers: lsf[] is lpc_clmp(lsf, 0, 10)'s
 * result on entry -- with delta 0 the clamp is its bubble sort alone (the
 * separation pass finds no gap below 0), done here as nine branch-free
 * passes -- and the recursion is lpc_lsp2pred's, unrolled */
MD void lsf_sort10(int16_t *l)
{
#pragma unroll
	for (int p = 0; p < 9; p++)
#pragma unroll
		for (int i = 0; i < 9; i++) {
			const int16_t a = l[i], b = l[i + 1];
			l[i] = a > b ? b : a;
			l[i + 1] = a > b ? a : b;
		}
}

MD void lsp2pred10(const int16_t *lsf, int16_t *lpc)
{
	Word32 f0[6], f1[6];
	f0[0] = f1[0] = 33554431L;
	f0[1] = L_shr(L_deposit_h(negate(cos_fxp(lsf[0]))), 5);
	f1[1] = L_shr(L_deposit_h(negate(cos_fxp(lsf[1]))), 5);
#pragma unroll
	for (int i = 2; i <= 5; i++) {
		const Word16 c0 = negate(cos_fxp(lsf[2 * i - 2]));
		const Word16 c1 = negate(cos_fxp(lsf[2 * i - 1]));
		f0[i] = f0[i - 2];
		f1[i] = f1[i - 2];
#pragma unroll
		for (int j = i; j >= 2; j--) {
			f0[j] = L_add(f0[j], L_add(L_shl(L_mpy_ls(f0[j - 1], c0), 1), f0[j - 2]));
			f1[j] = L_add(f1[j], L_add(L_shl(L_mpy_ls(f1[j - 1], c1), 1), f1[j - 2]));
		}
		f0[1] = L_add(f0[1], L_shl(L_mpy_ls(f0[0], c0), 1));
		f1[1] = L_add(f1[1], L_shl(L_mpy_ls(f1[0], c1), 1));
	}
#pragma unroll
	for (int i = 4; i >= 0; i--) {
		f0[i + 1] = L_add(f0[i + 1], f0[i]);
		f1[i + 1] = L_sub(f1[i + 1], f1[i]);
		lpc[i] = extract_h(L_shl(L_add(f0[i + 1], f1[i + 1]), 2));
		lpc[9 - i] = extract_h(L_shl(L_sub(f0[i + 1], f1[i + 1]), 2));
	}
}

/* lpc_syn :922 -- all-pole synthesis, y[-order..-1] is the memory; the
 * order-10 case keeps coefficients and the output history in registers */
MD void lpc_syn(const int16_t *x, int16_t *y, const int16_t *a, int order, int n)
{
	PROF_SCOPE(29);
	if (order == 10) {
		Word16 c[10], h[10];	/* h[k] = y[j - 1 - k] */
		bool dbl = true;
#pragma unroll
		for (int k = 0; k < 10; k++) {
			c[k] = a[k];
			h[k] = y[-1 - k];
			dbl &= c[k] != SW_MIN_;
		}
		int j = 0;
#if !defined(MELPE_OPCOUNT)
		/* With no coefficient at MIN16, L_msu(acc, h, c) is the saturating
		 * acc - h * 2c; the inputs are loaded a block of eight ahead of
		 * the outputs stored (x == y, or y below x: each x[j] is read
		 * before y[j] can overwrite it) */
		if (n >= 16 && wave_all(dbl) && !(y > x && y < x + n)) {
			int32_t c2[10];
#pragma unroll
			for (int k = 0; k < 10; k++)
				c2[k] = 2 * (int32_t) c[k];
			auto step = [&](int16_t xv) {
				Word32 acc = L_shr(L_deposit_h(xv), 3);
#pragma unroll
				for (int i = 10; i > 0; i--)
					acc = sat_sub32(acc, (int32_t) h[i - 1] * c2[i - 1]);
				Word16 v = r_ound(L_shl(acc, 3));
#pragma unroll
				for (int k = 9; k > 0; k--)
					h[k] = h[k - 1];
				h[0] = v;
				return v;
			};
			int16_t v[8];
#pragma unroll
			for (int q = 0; q < 8; q++)
				v[q] = x[q];
#pragma unroll 1
			for (; j + 16 <= n; j += 8) {
				int16_t nv[8];
#pragma unroll
				for (int q = 0; q < 8; q++)
					nv[q] = x[j + 8 + q];
#pragma unroll
				for (int q = 0; q < 8; q++)
					y[j + q] = step(v[q]);
#pragma unroll
				for (int q = 0; q < 8; q++)
					v[q] = nv[q];
			}
#pragma unroll
			for (int q = 0; q < 8; q++)
				y[j + q] = step(v[q]);
			j += 8;
		}
#endif
		for (; j < n; j++) {
			Word32 acc = L_shr(L_deposit_h(x[j]), 3);
#pragma unroll
			for (int i = 10; i > 0; i--)
				acc = L_msu(acc, h[i - 1], c[i - 1]);
			Word16 v = r_ound(L_shl(acc, 3));
			y[j] = v;
#pragma unroll
			for (int k = 9; k > 0; k--)
				h[k] = h[k - 1];
			h[0] = v;
		}
		return;
	}
	for (int j = 0; j < n; j++) {
		Word32 acc = L_shr(L_deposit_h(x[j]), 3);
		for (int i = order; i > 0; i--)
			acc = L_msu(acc, y[j - i], a[i - 1]);
		y[j] = r_ound(L_shl(acc, 3));
	}
}

/* ------------------------------------------------------------------ */
/* FFT: melpe/fft_lib.c                                               */
/* ------------------------------------------------------------------ */

/* max |x| over d[0..n-1] through the saturating ops, as the reference */
MD Word16 block_max(const int16_t *d, int n)
{
	Word16 m = 0;
	for (int i = 0; i < n; i++) {
		Word16 a = abs_s(d[i]);
		if (sub(m, a) < 0)
			m = a;
	}
	return m;
}

/* cfft :115 -- in-place radix-2 DIT complex FFT of nn points (2*nn shorts)
 * with per-stage block floating point; returns the number of halvings. */
MN Word16 cfft(int16_t *d0, Word16 nn)
{
	PROF_SCOPE(30);
	const int16_t *wrt = g_der.wr, *wit = g_der.wi;
	int16_t *d = d0 - 1;	/* 1-based view, as the reference */
	Word16 g = 0;
	Word16 n = shl(nn, 1);
	Word16 j = 1;
	for (Word16 i = 1; i < n; i += 2) {
		if (j > i) {
			int16_t t = d[j];
			d[j] = d[i];
			d[i] = t;
			t = d[j + 1];
			d[j + 1] = d[i + 1];
			d[i + 1] = t;
		}
		Word16 m = nn;
		while (m >= 2 && j > m) {
			j = sub(j, m);
			m = shr(m, 1);
		}
		j = add(j, m);
	}
	if (block_max(d0, n) > 16383) {
		g += 1;
		for (int i = 0; i < n; i++)
			d0[i] = shr(d0[i], 1);
	}
	for (int i = 0; i < n; i += 4) {
		Word16 pr = d0[i], qr = d0[i + 2], pi = d0[i + 1], qi = d0[i + 3];
		d0[i] = add(pr, qr);
		d0[i + 2] = sub(pr, qr);
		d0[i + 1] = add(pi, qi);
		d0[i + 3] = sub(pi, qi);
	}
	if (block_max(d0, n) > 16383) {
		g += 1;
		for (int i = 0; i < n; i++)
			d0[i] = shr(d0[i], 1);
	}
	for (int i = 0; i < n; i += 8) {
		Word16 pr = d0[i], qr = d0[i + 4], pi = d0[i + 1], qi = d0[i + 5];
		d0[i] = add(pr, qr);
		d0[i + 4] = sub(pr, qr);
		d0[i + 1] = add(pi, qi);
		d0[i + 5] = sub(pi, qi);
		pr = d0[i + 2];
		qr = d0[i + 6];
		pi = d0[i + 3];
		qi = d0[i + 7];
		d0[i + 2] = add(pr, qi);
		d0[i + 6] = sub(pr, qi);
		d0[i + 3] = sub(pi, qr);
		d0[i + 7] = add(pi, qr);
	}
	Word16 mmax = 8;
	Word16 istep_idx = shr(nn, 1);
	while (n > mmax) {
		Word16 mx = block_max(d0, n);
		if (mx > 16383) {
			g += 2;
			for (int i = 0; i < n; i++)
				d0[i] = shr(d0[i], 2);
		} else if (mx > 8191) {
			g += 1;
			for (int i = 0; i < n; i++)
				d0[i] = shr(d0[i], 1);
		}
		Word16 istep = shl(mmax, 1);
		Word16 idx = 0;
		istep_idx = shr(istep_idx, 1);
		Word16 wr = SW_MAX_, wi = 0;
		for (Word16 m = 1; m < mmax; m += 2) {
			for (Word16 i = m; i <= n; i = add(i, istep)) {
				Word16 jj = add(i, mmax);
				Word32 tr = L_add(L_mult(wr, d[jj]), L_mult(wi, d[jj + 1]));
				tr = L_add(tr, L_shl(0x80, 8));
				tr = L_shl(L_shr(tr, 16), 16);
				Word16 pr = d[i], qr = d[jj];
				d[i] = extract_h(L_add(L_deposit_h(pr), tr));
				d[jj] = extract_h(L_sub(L_deposit_h(pr), tr));
				Word32 ti = L_sub(L_mult(wi, qr), L_mult(wr, d[jj + 1]));
				ti = L_add(ti, L_shl(0x80, 8));
				ti = L_shl(L_shr(ti, 16), 16);
				Word16 pi = d[i + 1];
				d[i + 1] = extract_h(L_sub(L_deposit_h(pi), ti));
				d[jj + 1] = extract_h(L_add(L_deposit_h(pi), ti));
			}
			idx = add(idx, istep_idx);
			wr = wrt[idx];
			wi = wit[idx];
		}
		mmax = istep;
	}
	return g;
}

/* fft_npp :270 -- 256-point complex FFT, dir < 0 gives the inverse order */
MD Word16 fft_npp(int16_t *d, Word16 dir)
{
	Word16 g = cfft(d, 256);
	if (dir < 0) {
		for (int n = 1; n < 128; n++) {
			int16_t t = d[2 * n];
			d[2 * n] = d[2 * (256 - n)];
			d[2 * (256 - n)] = t;
			t = d[2 * n + 1];
			d[2 * n + 1] = d[2 * (256 - n) + 1];
			d[2 * (256 - n) + 1] = t;
		}
	}
	return g;
}

/* rfft :33 -- real FFT of n points through an n/2-point complex FFT;
 * d must hold 2n shorts */
MN void rfft(int16_t *d, Word16 n)
{
	PROF_SCOPE(31);
	const int16_t *wrt = g_der.wr, *wit = g_der.wi;
	Word16 n2 = shr(n, 1);
	cfft(d, n2);
	if (block_max(d, n) > 16383)
		for (int i = 0; i < n; i++)
			d[i] = shr(d[i], 1);
	for (int i = 2; i < n2; i += 2) {
		Word16 r1 = add_shr(d[i], d[n - i]);
		Word32 a = L_shl(L_sub(d[i + 1], d[n - i + 1]), 16);
		Word16 r2 = add_shr(d[i + 1], d[n - i + 1]);
		Word32 b = L_shl(L_sub(d[i], d[n - i]), 16);
		d[i] = r1;
		d[n - i] = r1;
		d[2 * n - i + 1] = extract_h(L_shr(b, 1));
		b = L_negate(b);
		d[n + i + 1] = extract_h(L_shr(b, 1));
		d[i + 1] = r2;
		d[n - i + 1] = r2;
		d[2 * n - i] = extract_h(L_shr(a, 1));
		a = L_negate(a);
		d[n + i] = extract_h(L_shr(a, 1));
	}
	d[n + n2] = 0;
	d[n + n2 + 1] = 0;
	Word16 r1 = add(d[0], d[1]);
	Word16 i1 = sub(d[0], d[1]);
	d[0] = r1;
	d[1] = 0;
	d[n] = i1;
	d[n + 1] = 0;
	int idx = 1;
	Word16 wr = wrt[idx], wi = wit[idx];
	for (int i = 2; i < n; i += 2) {
		Word16 a1 = d[i], b1 = d[2 * n - i], a2 = d[i + 1], b2 = d[2 * n - i + 1];
		Word32 t = L_deposit_h(a1);
		t = L_add(t, L_mult(a2, wr));
		t = L_add(t, L_shl(0x0080, 8));
		t = L_shl(L_shr(t, 16), 16);
		t = L_sub(t, L_mult(b2, wi));
		t = L_add(t, L_shl(0x0080, 8));
		d[i] = extract_h(t);
		d[2 * n - i] = extract_h(t);
		Word32 u = L_deposit_h(b1);
		u = L_sub(u, L_mult(a2, wi));
		u = L_add(u, L_shl(0x0080, 8));
		u = L_shl(L_shr(u, 16), 16);
		u = L_sub(u, L_mult(b2, wr));
		u = L_add(u, L_shl(0x0080, 8));
		d[i + 1] = extract_h(u);
		d[2 * n - i + 1] = extract_h(L_negate(u));
		idx += 1;
		wr = wrt[idx];
		wi = wit[idx];
	}
}

/* ------------------------------------------------------------------ */
/* Packed FFT for the lane-per-channel analysis (find_harm): complex    */
/* sample k is one dword (re | im << 16), so every butterfly moves two  */
/* dwords instead of four shorts, and the block-floating-point guard of */
/* each stage (block_max, then a shift of every sample) is fused into   */
/* the passes: the max is tracked while the previous stage writes, the  */
/* shift is applied as the next stage reads.  Same values, same order   */
/* of saturating operations per output as cfft / rfft above.            */
/* ------------------------------------------------------------------ */
MD Word16 pk_re(uint32_t w) { return (Word16) (int16_t) (w & 0xffffu); }
MD Word16 pk_im(uint32_t w) { return (Word16) (int16_t) (w >> 16); }
MD uint32_t pk(Word16 re, Word16 im) { return (uint32_t) (uint16_t) re | ((uint32_t) (uint16_t) im << 16); }
MD Word16 pk_amax(uint32_t w, Word16 m)
{
	Word16 a = abs_s(pk_re(w)), b = abs_s(pk_im(w));
	m = a > m ? a : m;
	return b > m ? b : m;
}
MD uint32_t pk_shr(uint32_t w, Word16 s) { return s ? pk(shr(pk_re(w), s), shr(pk_im(w), s)) : w; }

/* cfft :115 on nn complex samples x[0..nn); `mx` = max |x| of the input
 * (as block_max over its 2nn shorts); returns the halvings, and the max |x|
 * of the output in *omx (for the caller's next guard test) */
MN Word16 cfft_pk(uint32_t *x, int nn, Word16 mx, Word16 *omx)
{
	PROF_SCOPE(30);
	const int16_t *wrt = g_der.wr, *wit = g_der.wi;
	Word16 g = 0;
	/* bit reversal: the reference's j recurrence on 1-based short indices
	 * swaps sample i with r = bitrev(i) whenever r > i.  The swaps are
	 * disjoint, so they go eight samples at a time, every load of a batch
	 * issued before its stores. */
	{
		const int lg = 31 - __builtin_clz(nn);
		auto rev = [lg](int i) {
#if defined(__HIP_DEVICE_COMPILE__)
			return (int) (__builtin_bitreverse32((uint32_t) i) >> (32 - lg));
#else
			int r = 0;
			for (int b = 0; b < lg; b++)
				r |= ((i >> b) & 1) << (lg - 1 - b);
			return r;
#endif
		};
		#pragma unroll 1
		for (int i0 = 0; i0 < nn; i0 += 8) {
			uint32_t xi[8], xr[8];
			int r[8];
			#pragma unroll
			for (int k = 0; k < 8; k++) {
				r[k] = rev(i0 + k);
				xi[k] = x[i0 + k];
				xr[k] = x[r[k]];
			}
			#pragma unroll
			for (int k = 0; k < 8; k++)
				if (r[k] > i0 + k) {
					x[i0 + k] = xr[k];
					x[r[k]] = xi[k];
				}
		}
	}
	Word16 s = 0;
	if (mx > 16383) {
		g += 1;
		s = 1;
	}
	/* stage 1: pairs */
	mx = 0;
	for (int k = 0; k < nn; k += 2) {
		uint32_t p = pk_shr(x[k], s), q = pk_shr(x[k + 1], s);
		Word16 pr = pk_re(p), pi = pk_im(p), qr = pk_re(q), qi = pk_im(q);
		uint32_t a = pk(add(pr, qr), add(pi, qi)), b = pk(sub(pr, qr), sub(pi, qi));
		x[k] = a;
		x[k + 1] = b;
		mx = pk_amax(b, pk_amax(a, mx));
	}
	s = 0;
	if (mx > 16383) {
		g += 1;
		s = 1;
	}
	/* stage 2: quads, the second pair with the -j twiddle */
	mx = 0;
	for (int k = 0; k < nn; k += 4) {
		uint32_t p0 = pk_shr(x[k], s), p1 = pk_shr(x[k + 1], s);
		uint32_t q0 = pk_shr(x[k + 2], s), q1 = pk_shr(x[k + 3], s);
		Word16 pr = pk_re(p0), pi = pk_im(p0), qr = pk_re(q0), qi = pk_im(q0);
		uint32_t a0 = pk(add(pr, qr), add(pi, qi)), b0 = pk(sub(pr, qr), sub(pi, qi));
		pr = pk_re(p1);
		pi = pk_im(p1);
		qr = pk_re(q1);
		qi = pk_im(q1);
		uint32_t a1 = pk(add(pr, qi), sub(pi, qr)), b1 = pk(sub(pr, qi), add(pi, qr));
		x[k] = a0;
		x[k + 2] = b0;
		x[k + 1] = a1;
		x[k + 3] = b1;
		mx = pk_amax(b1, pk_amax(a1, pk_amax(b0, pk_amax(a0, mx))));
	}
	/* radix-2 stages; half = the reference's mmax / 2 in complex samples.
	 * A stage's butterflies are independent (and the guard max is order
	 * free), so they go four at a time -- twiddles m0 .. m0 + 3 of one group,
	 * two contiguous quads of samples -- with the next quad pair loaded before
	 * this one is stored.  Twiddle m is the reference's running table index
	 * m * istep, m = 0 taking (SW_MAX, 0). */
	int istep_idx = nn >> 1;
	for (int half = 4; half < nn; half <<= 1) {
		s = 0;
		if (mx > 16383) {
			g += 2;
			s = 2;
		} else if (mx > 8191) {
			g += 1;
			s = 1;
		}
		istep_idx >>= 1;
		Word16 nmx = 0;
		const int nb = nn >> 3;	/* quads of butterflies */
		auto base = [half](int b) { int q = 4 * b; return (q / half) * 2 * half + q % half; };
		uint32_t P[4], Q[4];
		{
			const int c0 = base(0);
			#pragma unroll
			for (int k = 0; k < 4; k++) {
				P[k] = x[c0 + k];
				Q[k] = x[c0 + half + k];
			}
		}
		#pragma unroll 1
		for (int b = 0; b < nb; b++) {
			const int ci = base(b), cn = base(b + 1 < nb ? b + 1 : b);
			uint32_t NP[4], NQ[4];
			#pragma unroll
			for (int k = 0; k < 4; k++) {
				NP[k] = x[cn + k];
				NQ[k] = x[cn + half + k];
			}
			const int m0 = ci & (half - 1);
			#pragma unroll
			for (int k = 0; k < 4; k++) {
				const int m = m0 + k;
				Word16 wr = m ? wrt[m * istep_idx] : (Word16) SW_MAX_;
				Word16 wi = m ? wit[m * istep_idx] : (Word16) 0;
				uint32_t Pk = pk_shr(P[k], s), Qk = pk_shr(Q[k], s);
				Word16 pr = pk_re(Pk), pi = pk_im(Pk), qr = pk_re(Qk), qi = pk_im(Qk);
				Word32 tr = L_add(L_mult(wr, qr), L_mult(wi, qi));
				tr = L_add(tr, 0x8000);
				tr = L_shl(L_shr(tr, 16), 16);
				Word32 ti = L_sub(L_mult(wi, qr), L_mult(wr, qi));
				ti = L_add(ti, 0x8000);
				ti = L_shl(L_shr(ti, 16), 16);
				uint32_t a = pk(extract_h(L_add(L_deposit_h(pr), tr)),
						extract_h(L_sub(L_deposit_h(pi), ti)));
				uint32_t bb = pk(extract_h(L_sub(L_deposit_h(pr), tr)),
						 extract_h(L_add(L_deposit_h(pi), ti)));
				x[ci + k] = a;
				x[ci + half + k] = bb;
				nmx = pk_amax(bb, pk_amax(a, nmx));
			}
			#pragma unroll
			for (int k = 0; k < 4; k++) {
				P[k] = NP[k];
				Q[k] = NQ[k];
			}
		}
		mx = nmx;
	}
	*omx = mx;
	return g;
}

/* rfft :33 on n real points held as n/2 packed complex samples in
 * x[0..n/2), output n packed complex bins in x[0..n); `mx` = max |x| of
 * the input */
MN void rfft_pk(uint32_t *x, int n, Word16 mx)
{
	PROF_SCOPE(31);
	const int16_t *wrt = g_der.wr, *wit = g_der.wi;
	const int n2 = n >> 1;		/* complex points of the inner FFT */
	cfft_pk(x, n2, mx, &mx);
	Word16 s = mx > 16383 ? 1 : 0;
	/* the k-th step reads x[k], x[n2 - k] and writes x[k], x[n2 - k],
	 * x[n - k], x[n2 + k]: disjoint across k (k < n2 / 2), so four steps
	 * share one batch of loads */
	auto split_step = [&](int k, uint32_t A, uint32_t B) {
		A = pk_shr(A, s);
		B = pk_shr(B, s);
		Word16 ar = pk_re(A), ai = pk_im(A), br = pk_re(B), bi = pk_im(B);
		Word16 r1 = add_shr(ar, br);
		Word32 a = L_shl(L_sub(ai, bi), 16);
		Word16 r2 = add_shr(ai, bi);
		Word32 b = L_shl(L_sub(ar, br), 16);
		x[k] = pk(r1, r2);
		x[n2 - k] = pk(r1, r2);
		Word16 bh = extract_h(L_shr(b, 1)), ah = extract_h(L_shr(a, 1));
		b = L_negate(b);
		a = L_negate(a);
		x[n - k] = pk(ah, bh);
		x[n2 + k] = pk(extract_h(L_shr(a, 1)), extract_h(L_shr(b, 1)));
	};
	int k1 = 1;
	#pragma unroll 1
	for (; k1 + 4 <= n2 / 2; k1 += 4) {
		uint32_t A[4], B[4];
		#pragma unroll
		for (int q = 0; q < 4; q++) {
			A[q] = x[k1 + q];
			B[q] = x[n2 - k1 - q];
		}
		#pragma unroll
		for (int q = 0; q < 4; q++)
			split_step(k1 + q, A[q], B[q]);
	}
	for (; k1 < n2 / 2; k1++)
		split_step(k1, x[k1], x[n2 - k1]);
	x[n2 + n2 / 2] = 0;
	x[n2 / 2] = pk_shr(x[n2 / 2], s);
	uint32_t z = pk_shr(x[0], s);
	x[0] = pk(add(pk_re(z), pk_im(z)), 0);
	x[n2] = pk(sub(pk_re(z), pk_im(z)), 0);
	/* step k reads and writes x[k], x[n - k] with twiddle k (the
	 * reference's running index): disjoint across k < n2, four per batch */
	auto twid_step = [&](int k, uint32_t A, uint32_t B) {
		Word16 wr = wrt[k], wi = wit[k];
		Word16 a1 = pk_re(A), a2 = pk_im(A), b1 = pk_re(B), b2 = pk_im(B);
		Word32 t = L_deposit_h(a1);
		t = L_add(t, L_mult(a2, wr));
		t = L_add(t, 0x8000);
		t = L_shl(L_shr(t, 16), 16);
		t = L_sub(t, L_mult(b2, wi));
		t = L_add(t, 0x8000);
		Word32 u = L_deposit_h(b1);
		u = L_sub(u, L_mult(a2, wi));
		u = L_add(u, 0x8000);
		u = L_shl(L_shr(u, 16), 16);
		u = L_sub(u, L_mult(b2, wr));
		u = L_add(u, 0x8000);
		x[k] = pk(extract_h(t), extract_h(u));
		x[n - k] = pk(extract_h(t), extract_h(L_negate(u)));
	};
	int k2 = 1;
	#pragma unroll 1
	for (; k2 + 4 <= n2; k2 += 4) {
		uint32_t A[4], B[4];
		#pragma unroll
		for (int q = 0; q < 4; q++) {
			A[q] = x[k2 + q];
			B[q] = x[n - k2 - q];
		}
		#pragma unroll
		for (int q = 0; q < 4; q++)
			twid_step(k2 + q, A[q], B[q]);
	}
	for (; k2 < n2; k2++)
		twid_step(k2, x[k2], x[n - k2]);
}

}  // namespace mlp

#endif
