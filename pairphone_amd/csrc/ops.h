/*
 * ops.h -- saturating fixed-point basic operators, bit-exact with the
 * reference's ETSI/TI-style library (melpe/mathhalf_i.h, melpe/mathdp31.c).
 *
 * Compiled for gfx950 (device code of the HIP kernels) and, for CPU-side
 * testing only, for the host.  The definitions are closed forms that were
 * checked against the reference's compiled operators (tests/test_basicops.py,
 * exhaustive over the 16-bit domains, randomised over 32/40-bit ones):
 *
 *   add/sub/L_add            = clamp of the exact sum   (mathhalf_i.h:120,586,692)
 *   L_sub                    = clamp, except L_sub(0, MIN32) = MIN32 (:719-730)
 *   L_mult(a,b)              = sat(2ab)                 (:1387)
 *   shl/shr/L_shl/L_shr      = saturating shift, right shifts capped (:781-1047)
 *   norm_l(x)                = clz(x ^ x>>31) - 1       (:1256)
 *   L40_*                    = int64 with a +-2^39 clamp (:1763-2168)
 *
 * On gfx950 the 32-bit saturating adds lower to v_add_i32 ... clamp.
 */
#ifndef MELPE_OPS_H
#define MELPE_OPS_H

#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define MD __device__ __attribute__((always_inline)) inline
#define MM __device__ __attribute__((always_inline)) inline	/* member functions */
#define MF __device__
/* big routines stay out of line: bounded compile time and register use */
#if defined(MELPE_INLINE_ALL)
#define MN __device__ __attribute__((always_inline)) inline
#else
#define MN __device__ __noinline__
#endif
/* per translation unit: every kernel TU is its own code object and uploads
 * its own copy (kern.h MELPE_TU) */
#define MDEV_CONST static __device__
/* read-only after the one-time upload: constant address space, so uniform
 * reads become scalar loads */
#define MDEV_TAB static __constant__
#else
#define MD static inline
#define MM inline
#define MF static
#define MN static
#define MDEV_CONST static
#define MDEV_TAB static
#endif

/* Basic-op census for the roofline figure (host count build only, see
 * tools/opcount.py): OPC(k) counts op k when it is entered from codec code,
 * not from inside another op -- the SURVEY.md 8(d) rule. */
#if defined(MELPE_OPCOUNT) && !defined(__HIP__)
extern "C" uint64_t melpe_opcount[64];
extern "C" int melpe_opdepth;
extern "C" uint64_t melpe_stagecount[64];
extern "C" int melpe_opstage;
struct OpScope {
	explicit OpScope(int k)
	{
		if (!melpe_opdepth++) {
			melpe_opcount[k]++;
			melpe_stagecount[melpe_opstage]++;
		}
	}
	~OpScope() { melpe_opdepth--; }
};
/* exclusive attribution of ops to the innermost PROF_SCOPE stage */
struct StageScope {
	int prev;
	explicit StageScope(int k) : prev(melpe_opstage) { melpe_opstage = k + 1; }
	~StageScope() { melpe_opstage = prev; }
};
#define OPC(k) OpScope op_scope_(k)
/* n more (or, n < 0, fewer) top-level ops of kind k: keeps the census equal
 * to the reference's op sequence where a code path computes the same values
 * with fewer or different operations (blocked correlations, fused sums) */
#define OPC_ADD(k, n) do { if (!melpe_opdepth) { melpe_opcount[k] += (uint64_t) (int64_t) (n); melpe_stagecount[melpe_opstage] += (uint64_t) (int64_t) (n); } } while (0)
#else
#define OPC(k)
#define OPC_ADD(k, n) do { } while (0)
#endif
enum { OP_add = 0, OP_sub = 1, OP_L_sub = 3, OP_L_mult = 4, OP_extract_l = 6, OP_L_mac = 10, OP_shl = 18, OP_shr = 19,
       OP_L_shr = 20, OP_L_shl = 21, OP_divide_s = 26, OP_L40_mac = 29 };
#define PROF_CAT2(a, b) a##b
#define PROF_CAT(a, b) PROF_CAT2(a, b)
/* Stage timer (profiling build only, -DMELPE_PROF): PROF_SCOPE(k) adds the
 * wave's s_memtime ticks spent in the enclosing function to g_prof[k]
 * (inclusive of callees; first active lane records).  tools/stage_prof.py.
 * Slots 0..63 are the named stages (prof_names.txt), 64.. the multi-wave
 * analysis kernel's phases (ana_mw.h MW_PROF). */
#if defined(MELPE_PROF) && defined(__HIP__)
/* one counter block per kernel translation unit (each TU is its own code
 * object; melpe_prof_read sums them) */
#define MELPE_PROF_SLOTS 256
static __device__ unsigned long long g_prof[MELPE_PROF_SLOTS];
#endif
#if defined(MELPE_PROF) && defined(__HIP_DEVICE_COMPILE__)
struct ProfScope {
	int k;
	unsigned long long t0;
	__device__ explicit ProfScope(int kk) : k(kk), t0(__builtin_amdgcn_s_memtime()) {}
	__device__ ~ProfScope()
	{
		unsigned long long dt = __builtin_amdgcn_s_memtime() - t0;
#if defined(MELPE_PROF_QUART)
		/* per quarter of the grid (the lane order: light -> heavy classes) */
		const int q = k < 64 ? (int) ((4 * blockIdx.x) / gridDim.x) : 0;
		if (__builtin_amdgcn_readfirstlane(threadIdx.x) == threadIdx.x)
			atomicAdd(&g_prof[k + 64 * q], dt);
#else
		if (__builtin_amdgcn_readfirstlane(threadIdx.x) == threadIdx.x)
			atomicAdd(&g_prof[k], dt);
#endif
	}
};
#define PROF_SCOPE(k) ProfScope PROF_CAT(prof_scope_, __LINE__)(k)
#elif defined(MELPE_OPCOUNT) && !defined(__HIP__)
#define PROF_SCOPE(k) StageScope PROF_CAT(stage_scope_, __LINE__)(k)
#else
#define PROF_SCOPE(k)
#endif
#define MELPE_OP_NAMES "add sub L_add L_sub L_mult extract_h extract_l L_deposit_h L_deposit_l mult L_mac L_msu r_ound msu_r negate L_negate abs_s L_abs shl shr L_shr L_shl shift_r L_shift_r norm_l norm_s divide_s L40_add L40_sub L40_mac L40_msu L40_shl L40_shr L40_negate norm32 L_sat32 L_mpy_ls"

/* a dword that may alias any type: record copies (kern.h lane_copy, the
 * NPP state image) move int16/int32/uint8 fields as dwords */
typedef uint32_t __attribute__((__may_alias__)) u32_alias;

typedef int16_t __attribute__((__may_alias__)) i16_alias;

/* int16 copy of a record field (no alignment beyond 2 assumed) */
MD void lane_copy16(void *dst, const void *src, size_t bytes)
{
	i16_alias *d = (i16_alias *) dst;
	const i16_alias *s = (const i16_alias *) src;
	const int n = (int) (bytes / 2);
	int i = 0;
	for (; i + 32 <= n; i += 32) {	/* 32 loads in flight, as lane_copy32 */
		int16_t v[32];
#pragma unroll
		for (int k = 0; k < 32; k++)
			v[k] = s[i + k];
#pragma unroll
		for (int k = 0; k < 32; k++)
			d[i + k] = v[k];
	}
	for (; i < n; i++)
		d[i] = s[i];
}

/* dword copy (offsets and sizes multiples of 4), 32 loads in flight: the
 * record reads are one channel per lane, each its own cache line, so the
 * copy is latency-bound */
MD void lane_copy32(void *dst, const void *src, size_t bytes)
{
	u32_alias *d = (u32_alias *) dst;
	const u32_alias *s = (const u32_alias *) src;
	const int n = (int) (bytes / 4);
	int i = 0;
	for (; i + 32 <= n; i += 32) {
		uint32_t v[32];
#pragma unroll
		for (int k = 0; k < 32; k++)
			v[k] = s[i + k];
#pragma unroll
		for (int k = 0; k < 32; k++)
			d[i + k] = v[k];
	}
	for (; i < n; i++)
		d[i] = s[i];
}


/* the value of the first active lane (device), for waterfall loops over the
 * distinct values a lane-varying operand takes; the host build runs one
 * channel, whose value it is */
MD int wave_first(int v)
{
#if defined(__HIP_DEVICE_COMPILE__)
	return __builtin_amdgcn_readfirstlane(v);
#else
	return v;
#endif
}

/* whether p holds in every active lane (device); the host build's one
 * channel */
MD bool wave_all(bool p)
{
#if defined(__HIP_DEVICE_COMPILE__)
	return __builtin_amdgcn_ballot_w64(!p) == 0;
#else
	return p;
#endif
}

typedef int16_t Word16;
typedef int32_t Word32;
typedef int64_t Word40;

#define SW_MAX_ 32767
#define SW_MIN_ (-32768)
#define LW_MAX_ ((int32_t) 0x7fffffff)
#define LW_MIN_ ((int32_t) 0x80000000)
#define MAX40_ ((int64_t) 1 << 39)
#define MIN40_ (-((int64_t) 1 << 39))

MD Word16 sat16(Word32 x)
{
	return (Word16) (x > SW_MAX_ ? SW_MAX_ : (x < SW_MIN_ ? SW_MIN_ : x));
}

MD Word32 sat_add32(Word32 a, Word32 b)
{
#if defined(__clang__)
	return __builtin_elementwise_add_sat(a, b);
#else
	int64_t s = (int64_t) a + b;
	return (Word32) (s > LW_MAX_ ? LW_MAX_ : (s < LW_MIN_ ? LW_MIN_ : s));
#endif
}

MD Word32 sat_sub32(Word32 a, Word32 b)
{
#if defined(__clang__)
	return __builtin_elementwise_sub_sat(a, b);
#else
	int64_t s = (int64_t) a - b;
	return (Word32) (s > LW_MAX_ ? LW_MAX_ : (s < LW_MIN_ ? LW_MIN_ : s));
#endif
}

MD Word16 add(Word16 a, Word16 b) { OPC(0); return sat16((Word32) a + b); }
MD Word16 sub(Word16 a, Word16 b) { OPC(1); return sat16((Word32) a - b); }
MD Word32 L_add(Word32 a, Word32 b) { OPC(2); return sat_add32(a, b); }

MD Word32 L_sub(Word32 a, Word32 b)
{
	OPC(3);
	/* reference quirk: with a == 0 no overflow check is made and
	 * 0 - MIN32 wraps to MIN32 (mathhalf_i.h:724-729) */
	if (a == 0 && b == LW_MIN_)
		return LW_MIN_;
	return sat_sub32(a, b);
}

MD Word32 L_mult(Word16 a, Word16 b)
{
	OPC(4);
	Word32 p = (Word32) a * (Word32) b;
	return sat_add32(p, p);
}

MD Word16 extract_h(Word32 x) { OPC(5); return (Word16) (x >> 16); }
MD Word16 extract_l(Word32 x) { OPC(6); return (Word16) x; }
MD Word32 L_deposit_h(Word16 a) { OPC(7); return (Word32) ((uint32_t) (int32_t) a << 16); }
MD Word32 L_deposit_l(Word16 a) { OPC(8); return (Word32) a; }

MD Word16 mult(Word16 a, Word16 b) { OPC(9); return extract_h(L_mult(a, b)); }
MD Word32 L_mac(Word32 acc, Word16 a, Word16 b) { OPC(10); return sat_add32(acc, L_mult(a, b)); }
/* L_mult never returns MIN32, so L_sub's quirk cannot trigger here */
MD Word32 L_msu(Word32 acc, Word16 a, Word16 b) { OPC(11); return sat_sub32(acc, L_mult(a, b)); }
MD Word16 r_ound(Word32 x) { OPC(12); return extract_h(sat_add32(x, 0x8000)); }
MD Word16 msu_r(Word32 acc, Word16 a, Word16 b) { OPC(13); return r_ound(L_msu(acc, a, b)); }

MD Word16 negate(Word16 a) { OPC(14); return a == SW_MIN_ ? (Word16) SW_MAX_ : (Word16) -a; }
MD Word32 L_negate(Word32 a) { OPC(15); return a == LW_MIN_ ? LW_MAX_ : -a; }
MD Word16 abs_s(Word16 a) { OPC(16); return a == SW_MIN_ ? (Word16) SW_MAX_ : (Word16) (a < 0 ? -a : a); }
MD Word32 L_abs(Word32 a) { OPC(17); return a == LW_MIN_ ? LW_MAX_ : (a < 0 ? -a : a); }

/* shl/shr: mathhalf_i.h:781-935, branch-free.  For any 16-bit a and n:
 * a right shift by min(-n, 15) when n < 0 (15 and beyond give the sign),
 * else a * 2^min(n, 16) clamped to 16 bits (a nonzero a shifted by 15 or
 * more saturates to its sign, as the reference's n >= 15 case, except -1 << 15
 * = MIN16, which the reference returns too).  shr(a, n) = shl(a, -n) over
 * the whole range, n <= -15 included.  Without branches the compiler keeps
 * the loads of an element loop in flight across elements. */
MD Word16 shl_core(Word16 a, int n)
{
	const int sn = n < 0 ? (-n < 15 ? -n : 15) : 0;
	const int sp = n > 0 ? (n < 16 ? n : 16) : 0;
	int v = ((int) a * (1 << sp)) >> sn;
	v = v > SW_MAX_ ? SW_MAX_ : (v < SW_MIN_ ? SW_MIN_ : v);
	return (Word16) v;
}

MD Word16 shl(Word16 a, Word16 n)
{
	OPC(18);
	return shl_core(a, n);
}

MD Word16 shr(Word16 a, Word16 n)
{
	OPC(19);
	return shl_core(a, -(int) n);
}

/* L_shl/L_shr: mathhalf_i.h:942-1047 */
/* branch-free, as shl: a right shift by min(-n, 31) for n < 0, else
 * a * 2^min(n, 32) in 64 bits clamped to 32; L_shr(a, n) = L_shl(a, -n)
 * over the whole range */
MD Word32 L_shl_core(Word32 a, int n)
{
	const int sn = n < 0 ? (-n < 31 ? -n : 31) : 0;
	const int sp = n > 0 ? (n < 32 ? n : 32) : 0;
	int64_t v = ((int64_t) a * ((int64_t) 1 << sp)) >> sn;
	v = v > LW_MAX_ ? LW_MAX_ : (v < LW_MIN_ ? LW_MIN_ : v);
	return (Word32) v;
}

MD Word32 L_shl(Word32 a, Word16 n)
{
	OPC(21);
	return L_shl_core(a, n);
}

MD Word32 L_shr(Word32 a, Word16 n)
{
	OPC(20);
	return L_shl_core(a, -(int) n);
}

/* shift_r / L_shift_r: mathhalf_i.h:1108-1230 */
MD Word16 shift_r(Word16 a, Word16 n)
{
	OPC(22);
	if (n >= 0)
		return shl(a, n);
	if (n < -15)
		return 0;
	return add(shl(a, n), (Word16) (shl(a, (Word16) (n + 1)) & 1));
}

MD Word32 L_shift_r(Word32 a, Word16 n)
{
	OPC(23);
	if (n < -31)
		return 0;
	if (n < 0)
		return L_add(L_shl(a, n), L_shl(a, (Word16) (n + 1)) & 1);
	return L_shl(a, n);
}

MD Word16 norm_l(Word32 x)
{
	OPC(24);
	uint32_t u;
	if (x == 0)
		return 0;
	u = (uint32_t) (x ^ (x >> 31));
	if (u == 0)
		return 31;
#if defined(__HIP__)
	return (Word16) (__clz((int) u) - 1);
#else
	return (Word16) (__builtin_clz(u) - 1);
#endif
}

MD Word16 norm_s(Word16 a) { OPC(25); return norm_l(L_deposit_h(a)); }

/* divide_s: floor(num * 2^15 / den) for 0 <= num < den.  On the device the
 * quotient comes from one float reciprocal and one integer correction
 * instead of a 32-bit integer division: N = num << 15 < 2^30 converts with
 * relative error <= 2^-24 and v_rcp_f32 is within 1 ulp, so the float
 * estimate q' of N / den satisfies |q' - N / den| < 2^-7 (N / den < 2^15);
 * truncated, it is floor(N / den) or one below or above it, and the
 * remainder N - q den (exact: q den < 2^31) picks the right one. */
MD Word16 divide_s(Word16 num, Word16 den)
{
	OPC(26);
	if (num < 0 || den < 0 || num > den)
		return 0;
	if (num == den)
		return SW_MAX_;
#if defined(__HIP_DEVICE_COMPILE__)
	const int32_t N = (int32_t) num << 15, d = den;
	int32_t q = (int32_t) ((float) N * __builtin_amdgcn_rcpf((float) d));
	const int32_t r = N - q * d;
	q += (r >= d) ? 1 : 0;
	q -= (r < 0) ? 1 : 0;
	return (Word16) q;
#else
	return (Word16) ((0x8000 * (Word32) num) / (Word32) den);
#endif
}

/* ---- 40-bit accumulator (mathhalf_i.h:1763-2168) ---- */
MD Word40 clamp40(Word40 v) { return v > MAX40_ ? MAX40_ : (v < MIN40_ ? MIN40_ : v); }
MD Word40 L40_add(Word40 acc, Word32 x) { OPC(27); return clamp40(acc + (Word40) x); }
MD Word40 L40_sub(Word40 acc, Word32 x) { OPC(28); return clamp40(acc - (Word40) x); }
MD Word40 L40_mac(Word40 acc, Word16 a, Word16 b) { OPC(29); return clamp40(acc + (Word40) a * (Word40) b * 2); }
MD Word40 L40_msu(Word40 acc, Word16 a, Word16 b) { OPC(30); return clamp40(acc - (Word40) a * (Word40) b * 2); }
MD Word40 L40_shr(Word40 acc, Word16 n);
/* the reference doubles with a clamp test per step (mathhalf_i.h); as the
 * magnitude only grows, that equals one clamp of acc * 2^n */
MD Word40 L40_shl(Word40 acc, Word16 n)
{
	OPC(31);
	if (n < 0)
		return L40_shr(acc, (Word16) -n);
	if (n == 0 || acc == 0)
		return acc;
	if (n >= 40)
		return acc > 0 ? MAX40_ : MIN40_;
	if (acc > (MAX40_ >> n))
		return MAX40_;
	if (acc < (MIN40_ >> n))
		return MIN40_;
	return acc * ((Word40) 1 << n);
}
MD Word40 L40_shr(Word40 acc, Word16 n)
{
	OPC(32);
	if (n < 0)
		return L40_shl(acc, (Word16) -n);
	return acc >> (n > 62 ? 62 : n);	/* floor(acc/2) repeated */
}
MD Word40 L40_negate(Word40 acc)
{
	OPC(33);
	acc = -acc;
	return acc > MAX40_ ? MAX40_ : acc;
}
/* norm32 (mathhalf_i.h:2108): the shift that brings acc into [2^30, 2^31)
 * (positive) or [-2^31, -2^30) (negative) by the reference's halving /
 * doubling loops, in closed form: 30 - floor(log2 acc) for acc > 0,
 * 31 - ceil(log2 -acc) for acc < 0 */
MD Word16 norm32(Word40 acc)
{
	OPC(34);
	if (acc > 0) {
#if defined(__HIP__)
		return (Word16) (30 - (63 - __clzll(acc)));
#else
		return (Word16) (30 - (63 - __builtin_clzll((unsigned long long) acc)));
#endif
	}
	if (acc < 0) {
		uint64_t m = (uint64_t) (-acc);
		if (m == 1)
			return 31;
#if defined(__HIP__)
		int cl = 64 - __clzll((long long) (m - 1));	/* ceil(log2 m) */
#else
		int cl = 64 - __builtin_clzll(m - 1);
#endif
		return (Word16) (31 - cl);
	}
	return 0;
}
MD Word32 L_sat32(Word40 acc)
{
	OPC(35);
	return (Word32) (acc > LW_MAX_ ? LW_MAX_ : (acc < LW_MIN_ ? LW_MIN_ : acc));
}

/* mathdp31.c:71-83 */
MD Word32 L_mpy_ls(Word32 L_var2, Word16 var1)
{
	OPC(36);
	Word16 lo = (Word16) (shr(extract_l(L_var2), 1) & 0x7fff);
	Word32 out = L_shr(L_mult(var1, lo), 15);
	return L_mac(out, var1, extract_h(L_var2));
}

#define Max_(a, b) (((a) > (b)) ? (a) : (b))
#define Min_(a, b) (((a) > (b)) ? (b) : (a))

#endif
