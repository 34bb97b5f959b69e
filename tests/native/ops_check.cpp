// Basic-op parity: our ops.h (host build) vs the reference's compiled
// operators exported by oracle/_ref/libref_ops.so.  Exhaustive over the
// 16-bit x shift / 16-bit x 16-bit (sampled) domains, randomised elsewhere.
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include "ops.h"

extern "C" {
int16_t ref_add(int16_t, int16_t); int16_t ref_sub(int16_t, int16_t);
int32_t ref_L_add(int32_t, int32_t); int32_t ref_L_sub(int32_t, int32_t);
int16_t ref_mult(int16_t, int16_t); int32_t ref_L_mult(int16_t, int16_t);
int16_t ref_shr(int16_t, int16_t); int16_t ref_shl(int16_t, int16_t);
int32_t ref_L_shr(int32_t, int16_t); int32_t ref_L_shl(int32_t, int16_t);
int16_t ref_shift_r(int16_t, int16_t); int32_t ref_L_shift_r(int32_t, int16_t);
int16_t ref_abs_s(int16_t); int32_t ref_L_abs(int32_t);
int32_t ref_L_mac(int32_t, int16_t, int16_t); int32_t ref_L_msu(int32_t, int16_t, int16_t);
int16_t ref_msu_r(int32_t, int16_t, int16_t);
int16_t ref_negate(int16_t); int32_t ref_L_negate(int32_t);
int16_t ref_extract_h(int32_t); int16_t ref_extract_l(int32_t); int16_t ref_r_ound(int32_t);
int16_t ref_norm_l(int32_t); int16_t ref_norm_s(int16_t); int16_t ref_divide_s(int16_t, int16_t);
int64_t ref_L40_add(int64_t, int32_t); int64_t ref_L40_sub(int64_t, int32_t);
int64_t ref_L40_mac(int64_t, int16_t, int16_t); int64_t ref_L40_msu(int64_t, int16_t, int16_t);
int64_t ref_L40_shl(int64_t, int16_t); int64_t ref_L40_shr(int64_t, int16_t);
int64_t ref_L40_negate(int64_t); int16_t ref_norm32(int64_t); int32_t ref_L_sat32(int64_t);
int32_t ref_L_mpy_ls(int32_t, int16_t);
}

static uint64_t rs = 88172645463325252ull;
static uint32_t rnd() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (uint32_t) rs; }
static int32_t rnd32() {
	static const int32_t edge[] = {0, 1, -1, 2, -2, 0x7fffffff, (int32_t) 0x80000000, 0x7ffffffe,
		(int32_t) 0x80000001, 0x40000000, (int32_t) 0xc0000000, 0x3fffffff, (int32_t) 0xbfffffff,
		0x8000, 0x7fff, -0x8000, 0xffff, 0x10000};
	uint32_t k = rnd() % 8;
	if (k == 0) return edge[rnd() % (sizeof(edge) / sizeof(edge[0]))];
	if (k == 1) return (int32_t) (rnd() >> (rnd() % 32)) * ((rnd() & 1) ? 1 : -1);
	return (int32_t) rnd();
}
static int16_t rnd16() { return (int16_t) (rnd32() >> (rnd() % 2 ? 16 : 0)); }
static int64_t rnd40() { int64_t v = ((int64_t) (int32_t) rnd() << 8) ^ (rnd() & 0xff); return v >> (rnd() % 40); }

static long fails = 0;
#define CHK(name, a, b) do { if ((a) != (b)) { if (fails++ < 20) fprintf(stderr, "%s mismatch\n", name); } } while (0)

int main(int argc, char **argv)
{
	long nrand = argc > 1 ? atol(argv[1]) : 2000000;
	// exhaustive 16-bit x shift
	for (int a = -32768; a < 32768; a++)
		for (int n = -40; n <= 40; n++) {
			CHK("shl", shl(a, n), ref_shl(a, n));
			CHK("shr", shr(a, n), ref_shr(a, n));
			CHK("shift_r", shift_r(a, n), ref_shift_r(a, n));
		}
	for (int a = -32768; a < 32768; a++) {
		CHK("abs_s", abs_s(a), ref_abs_s(a));
		CHK("negate", negate(a), ref_negate(a));
		CHK("norm_s", norm_s(a), ref_norm_s(a));
		for (int b = -32768; b < 32768; b += 7) {
			CHK("add", add(a, b), ref_add(a, b));
			CHK("sub", sub(a, b), ref_sub(a, b));
			CHK("mult", mult(a, b), ref_mult(a, b));
			CHK("L_mult", L_mult(a, b), ref_L_mult(a, b));
			CHK("divide_s", divide_s(a, b), ref_divide_s(a, b));
		}
		CHK("mult-edge", mult(a, -32768), ref_mult(a, -32768));
		CHK("div-edge", divide_s(a, 32767), ref_divide_s(a, 32767));
	}
	// 40-bit edges: +-2^k, +-2^k +- 1 for every k, every shift in [-45, 45]
	for (int k = 0; k <= 39; k++)
		for (int d = -1; d <= 1; d++)
			for (int sg = -1; sg <= 1; sg += 2) {
				int64_t z = sg * (((int64_t) 1 << k) + d);
				if (z > ((int64_t) 1 << 39) || z < -((int64_t) 1 << 39))
					continue;	/* outside the 40-bit format: the reference exits */
				CHK("norm32-edge", norm32(z), ref_norm32(z));
				for (int n = -45; n <= 45; n++) {
					CHK("L40_shl-edge", L40_shl(z, n), ref_L40_shl(z, n));
					CHK("L40_shr-edge", L40_shr(z, n), ref_L40_shr(z, n));
				}
			}
	for (long i = 0; i < nrand; i++) {
		int32_t x = rnd32(), y = rnd32();
		int16_t a = rnd16(), b = rnd16(), n = (int16_t) ((int) (rnd() % 81) - 40);
		int64_t z = rnd40();
		CHK("L_add", L_add(x, y), ref_L_add(x, y));
		CHK("L_sub", L_sub(x, y), ref_L_sub(x, y));
		CHK("L_shl", L_shl(x, n), ref_L_shl(x, n));
		CHK("L_shr", L_shr(x, n), ref_L_shr(x, n));
		CHK("L_shift_r", L_shift_r(x, n), ref_L_shift_r(x, n));
		CHK("L_abs", L_abs(x), ref_L_abs(x));
		CHK("L_negate", L_negate(x), ref_L_negate(x));
		CHK("L_mac", L_mac(x, a, b), ref_L_mac(x, a, b));
		CHK("L_msu", L_msu(x, a, b), ref_L_msu(x, a, b));
		CHK("msu_r", msu_r(x, a, b), ref_msu_r(x, a, b));
		CHK("extract_h", extract_h(x), ref_extract_h(x));
		CHK("extract_l", extract_l(x), ref_extract_l(x));
		CHK("r_ound", r_ound(x), ref_r_ound(x));
		CHK("norm_l", norm_l(x), ref_norm_l(x));
		CHK("L_mpy_ls", L_mpy_ls(x, a), ref_L_mpy_ls(x, a));
		CHK("L40_add", L40_add(z, x), ref_L40_add(z, x));
		CHK("L40_sub", L40_sub(z, x), ref_L40_sub(z, x));
		CHK("L40_mac", L40_mac(z, a, b), ref_L40_mac(z, a, b));
		CHK("L40_msu", L40_msu(z, a, b), ref_L40_msu(z, a, b));
		int16_t n40 = (int16_t) ((int) (rnd() % 31) - 15);
		CHK("L40_shl", L40_shl(z, n40), ref_L40_shl(z, n40));
		CHK("L40_shr", L40_shr(z, n40), ref_L40_shr(z, n40));
		CHK("L40_negate", L40_negate(z), ref_L40_negate(z));
		CHK("norm32", norm32(z), ref_norm32(z));
		CHK("L_sat32", L_sat32(z), ref_L_sat32(z));
	}
	printf("%s %ld mismatches\n", fails ? "FAIL" : "OK", fails);
	return fails ? 1 : 0;
}
