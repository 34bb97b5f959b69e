/*
 * ref_ops.c -- non-inline exports of the REFERENCE basic ops
 * (melpe/mathhalf_i.h:120-2170, melpe/mathdp31.c:71) for the basic-op parity
 * tests (TEST INFRASTRUCTURE ONLY).  Compiled against the reference headers
 * where they lie; loaded by tests/test_basicops.py through ctypes.
 */
#include <stdint.h>
#include "sc1200.h"
#include "mathhalf.h"
#include "mathdp31.h"

#define W1(n, r, t1) r ref_##n(t1 a) { return melpe_##n(a); }
#define W2(n, r, t1, t2) r ref_##n(t1 a, t2 b) { return melpe_##n(a, b); }
#define W3(n, r, t1, t2, t3) r ref_##n(t1 a, t2 b, t3 c) { return melpe_##n(a, b, c); }

W2(add, int16_t, int16_t, int16_t)
W2(sub, int16_t, int16_t, int16_t)
W2(L_add, int32_t, int32_t, int32_t)
W2(L_sub, int32_t, int32_t, int32_t)
W2(mult, int16_t, int16_t, int16_t)
W2(L_mult, int32_t, int16_t, int16_t)
W2(shr, int16_t, int16_t, int16_t)
W2(shl, int16_t, int16_t, int16_t)
W2(L_shr, int32_t, int32_t, int16_t)
W2(L_shl, int32_t, int32_t, int16_t)
W2(shift_r, int16_t, int16_t, int16_t)
W2(L_shift_r, int32_t, int32_t, int16_t)
W1(abs_s, int16_t, int16_t)
W1(L_abs, int32_t, int32_t)
W3(L_mac, int32_t, int32_t, int16_t, int16_t)
W3(L_msu, int32_t, int32_t, int16_t, int16_t)
W3(msu_r, int16_t, int32_t, int16_t, int16_t)
W1(negate, int16_t, int16_t)
W1(L_negate, int32_t, int32_t)
W1(extract_h, int16_t, int32_t)
W1(extract_l, int16_t, int32_t)
W1(r_ound, int16_t, int32_t)
W1(norm_l, int16_t, int32_t)
W1(norm_s, int16_t, int16_t)
W2(divide_s, int16_t, int16_t, int16_t)
W2(L40_add, int64_t, int64_t, int32_t)
W2(L40_sub, int64_t, int64_t, int32_t)
W3(L40_mac, int64_t, int64_t, int16_t, int16_t)
W3(L40_msu, int64_t, int64_t, int16_t, int16_t)
W2(L40_shl, int64_t, int64_t, int16_t)
W2(L40_shr, int64_t, int64_t, int16_t)
W1(L40_negate, int64_t, int64_t)
W1(norm32, int16_t, int64_t)
W1(L_sat32, int32_t, int64_t)

int32_t ref_L_mpy_ls(int32_t a, int16_t b) { return L_mpy_ls(a, b); }

/* the same operators selected by id, over arrays, for the device basic-op
 * test (tests/test_device_ops.py): ids and argument conventions of
 * pairphone_amd/csrc/ops_eval.h */
#define Word16 int16_t
#define Word32 int32_t
#define Word40 int64_t
#define add(x, y) melpe_add(x, y)
#define sub(x, y) melpe_sub(x, y)
#define L_add(x, y) melpe_L_add(x, y)
#define L_sub(x, y) melpe_L_sub(x, y)
#define L_mult(x, y) melpe_L_mult(x, y)
#define extract_h(x) melpe_extract_h(x)
#define extract_l(x) melpe_extract_l(x)
#define mult(x, y) melpe_mult(x, y)
#define L_mac(x, y, z) melpe_L_mac(x, y, z)
#define L_msu(x, y, z) melpe_L_msu(x, y, z)
#define r_ound(x) melpe_r_ound(x)
#define msu_r(x, y, z) melpe_msu_r(x, y, z)
#define negate(x) melpe_negate(x)
#define L_negate(x) melpe_L_negate(x)
#define abs_s(x) melpe_abs_s(x)
#define L_abs(x) melpe_L_abs(x)
#define shl(x, y) melpe_shl(x, y)
#define shr(x, y) melpe_shr(x, y)
#define L_shr(x, y) melpe_L_shr(x, y)
#define L_shl(x, y) melpe_L_shl(x, y)
#define shift_r(x, y) melpe_shift_r(x, y)
#define L_shift_r(x, y) melpe_L_shift_r(x, y)
#define norm_l(x) melpe_norm_l(x)
#define norm_s(x) melpe_norm_s(x)
#define divide_s(x, y) melpe_divide_s(x, y)
#define L40_add(x, y) melpe_L40_add(x, y)
#define L40_sub(x, y) melpe_L40_sub(x, y)
#define L40_mac(x, y, z) melpe_L40_mac(x, y, z)
#define L40_msu(x, y, z) melpe_L40_msu(x, y, z)
#define L40_shl(x, y) melpe_L40_shl(x, y)
#define L40_shr(x, y) melpe_L40_shr(x, y)
#define L40_negate(x) melpe_L40_negate(x)
#define norm32(x) melpe_norm32(x)
#define L_sat32(x) melpe_L_sat32(x)
#include "../pairphone_amd/csrc/ops_eval.h"

int ref_ops_eval(int op, const int64_t *A, const int32_t *B, const int32_t *C, int64_t *out,
		 long n)
{
	long i;
	if (op < 0 || op >= MELPE_OPS_EVAL_COUNT)
		return -1;
	for (i = 0; i < n; i++) {
		int64_t a = A[i];
		int32_t b = B ? B[i] : 0, c = C ? C[i] : 0;
		int64_t r = 0;
		switch (op) {
#define OPS_CASE(id, name, call) case id: r = (int64_t) (call); break;
		MELPE_OPS_EVAL_LIST(OPS_CASE)
#undef OPS_CASE
		}
		out[i] = r;
	}
	return 0;
}
