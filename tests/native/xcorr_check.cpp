/*
 * xcorr_check.cpp -- the exact packed-pair correlators of dsp.h/analysis.h
 * (xcorr_pairs, fp_sums9, magsq_pairs, shr_energy_inplace; host build of
 * the device code)
 * against plain integer sums, over every length 1..260, both start
 * parities and random int16 data.  Each stream lives in its own heap block
 * ending exactly at its last sample, so an AddressSanitizer build flags any
 * read past a stream (tests/test_xcorr.py).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "codec.h"

using namespace mlp;

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static int16_t rnd16(int amp)
{
	rng ^= rng << 13;
	rng ^= rng >> 7;
	rng ^= rng << 17;
	return (int16_t) ((int) (rng % (2u * amp + 1)) - amp);
}

/* n samples at an odd or even int16 offset, the block ending at p + n */
struct Buf {
	int16_t *base, *p;
	Buf(int n, int odd, int amp)
	{
		base = (int16_t *) malloc(sizeof(int16_t) * (n + odd) + 1);
		p = base + odd;
		for (int i = 0; i < n; i++)
			p[i] = rnd16(amp);
	}
	~Buf() { free(base); }
};

static int bad = 0;

template <int K, class S, bool SPLIT>
static void check(int len, int oa_odd, int ob_odd, int amp)
{
	Buf a(len + S::NA - 1, oa_odd, amp), b(len + S::NB - 1, ob_odd, amp);
	int32_t out[2 * K];
	xcorr_pairs<K, S, SPLIT>(a.p, b.p, len, out);
	for (int k = 0; k < K; k++) {
		int64_t ref = 0;
		for (int j = 0; j < len; j++)
			ref += (int64_t) a.p[j + S::oa(k)] * b.p[j + S::ob(k)];
		int64_t got = SPLIT ? 256 * (int64_t) out[k] + out[K + k] : out[k];
		if (got != ref && bad++ < 10)
			printf("K=%d split=%d len=%d odd=%d/%d lag %d: %lld != %lld\n", K, SPLIT, len,
			       oa_odd, ob_odd, k, (long long) got, (long long) ref);
	}
}

static void check9(int len, int oa_odd, int ob_odd)
{
	Buf a(len, oa_odd, 2000), b(len + 2, ob_odd, 2000);
	int32_t q[9];
	fp_sums9(a.p, b.p, len, q);
	int64_t r[9] = {0};
	for (int j = 0; j < len; j++) {
		int64_t x = a.p[j], y0 = b.p[j], y1 = b.p[j + 1], y2 = b.p[j + 2];
		int64_t t[9] = {x * x, y0 * y0, x * y0, x * y1, x * y2, y1 * y2, y1 * y1, y2 * y2, y0 * y1};
		for (int k = 0; k < 9; k++)
			r[k] += t[k];
	}
	for (int k = 0; k < 9; k++)
		if (q[k] != r[k] && bad++ < 10)
			printf("sums9 len=%d odd=%d/%d sum %d: %d != %lld\n", len, oa_odd, ob_odd, k, q[k],
			       (long long) r[k]);
	Buf m(len, oa_odd, 2000);
	int64_t e = 0;
	for (int j = 0; j < len; j++)
		e += (int64_t) m.p[j] * m.p[j];
	if (magsq_pairs(m.p, len) != e && bad++ < 10)
		printf("magsq len=%d odd=%d\n", len, oa_odd);
}

static void check_shr(int n, int odd, int sc)
{
	Buf a(n, odd, 32768);
	std::vector<int16_t> ref(a.p, a.p + n);
	int64_t e = 0;
	for (int i = 0; i < n; i++) {
		ref[i] = shr(ref[i], (Word16) sc);
		e += (int64_t) ref[i] * ref[i];
	}
	int32_t got = shr_energy_inplace(a.p, n, (Word16) sc);
	int64_t want = e > LW_MAX_ ? LW_MAX_ : e;
	if ((got != want || memcmp(ref.data(), a.p, 2 * n)) && bad++ < 10)
		printf("shr_energy n=%d odd=%d sc=%d: %d != %lld\n", n, odd, sc, got, (long long) want);
}

int main()
{
	for (int n = 0; n <= 330; n++)
		for (int odd = 0; odd < 2; odd++)
			for (int sc = -6; sc <= 6; sc += 3)
				check_shr(n, odd, sc);
	for (int len = 1; len <= 260; len++)
		for (int oa = 0; oa < 2; oa++)
			for (int ob = 0; ob < 2; ob++) {
				/* 32-bit sums: |x| <= 2000 keeps 260 * 2000^2 * 2 < 2^31 */
				check<8, FpLags<8>, false>(len, oa, ob, 2000);
				check<12, FpLags<12>, false>(len, oa, ob, 2000);
				/* split: full int16 range, up to 256 terms */
				if (len <= 250) {
					check<8, CpLags, true>(len, oa, ob, 32768);
					check<10, FcLags<0>, true>(len, oa, ob, 32768);
					check<10, FcLags<1>, true>(len, oa, ob, 32768);
				}
				check9(len, oa, ob);
			}
	printf("%s %d mismatches\n", bad ? "FAIL" : "OK", bad);
	return bad != 0;
}
