/*
 * ops_eval.h -- one basic operator of ops.h selected by id, for the device
 * basic-op parity test (engine.hip k_ops_eval, melpe_ops_eval_dev) and its
 * checker (oracle/ref_ops.c ref_ops_eval, which evaluates the reference's
 * own operators, melpe/mathhalf_i.h:120-2170 and melpe/mathdp31.c:71, with
 * the same ids and argument conventions).
 *
 * Arguments are passed widened: a (int64: 16-, 32- or 40-bit first operand),
 * b and c (int32: second and third operand, 16-bit where the op takes
 * Word16); the result is returned widened to int64.
 */
#ifndef MELPE_OPS_EVAL_H
#define MELPE_OPS_EVAL_H

/* X(id, name, call) -- the call uses a, b, c narrowed to the op's types */
#define MELPE_OPS_EVAL_LIST(X)                                             \
	X(0, add, add((Word16) a, (Word16) b))                              \
	X(1, sub, sub((Word16) a, (Word16) b))                              \
	X(2, L_add, L_add((Word32) a, (Word32) b))                          \
	X(3, L_sub, L_sub((Word32) a, (Word32) b))                          \
	X(4, L_mult, L_mult((Word16) a, (Word16) b))                        \
	X(5, extract_h, extract_h((Word32) a))                              \
	X(6, extract_l, extract_l((Word32) a))                              \
	X(7, mult, mult((Word16) a, (Word16) b))                            \
	X(8, L_mac, L_mac((Word32) a, (Word16) b, (Word16) c))              \
	X(9, L_msu, L_msu((Word32) a, (Word16) b, (Word16) c))              \
	X(10, r_ound, r_ound((Word32) a))                                   \
	X(11, msu_r, msu_r((Word32) a, (Word16) b, (Word16) c))             \
	X(12, negate, negate((Word16) a))                                   \
	X(13, L_negate, L_negate((Word32) a))                               \
	X(14, abs_s, abs_s((Word16) a))                                     \
	X(15, L_abs, L_abs((Word32) a))                                     \
	X(16, shl, shl((Word16) a, (Word16) b))                             \
	X(17, shr, shr((Word16) a, (Word16) b))                             \
	X(18, L_shr, L_shr((Word32) a, (Word16) b))                         \
	X(19, L_shl, L_shl((Word32) a, (Word16) b))                         \
	X(20, shift_r, shift_r((Word16) a, (Word16) b))                     \
	X(21, L_shift_r, L_shift_r((Word32) a, (Word16) b))                 \
	X(22, norm_l, norm_l((Word32) a))                                   \
	X(23, norm_s, norm_s((Word16) a))                                   \
	X(24, divide_s, divide_s((Word16) a, (Word16) b))                   \
	X(25, L40_add, L40_add((Word40) a, (Word32) b))                     \
	X(26, L40_sub, L40_sub((Word40) a, (Word32) b))                     \
	X(27, L40_mac, L40_mac((Word40) a, (Word16) b, (Word16) c))         \
	X(28, L40_msu, L40_msu((Word40) a, (Word16) b, (Word16) c))         \
	X(29, L40_shl, L40_shl((Word40) a, (Word16) b))                     \
	X(30, L40_shr, L40_shr((Word40) a, (Word16) b))                     \
	X(31, L40_negate, L40_negate((Word40) a))                           \
	X(32, norm32, norm32((Word40) a))                                   \
	X(33, L_sat32, L_sat32((Word40) a))                                 \
	X(34, L_mpy_ls, L_mpy_ls((Word32) a, (Word16) b))

#define MELPE_OPS_EVAL_COUNT 35

#endif
