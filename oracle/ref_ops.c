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
