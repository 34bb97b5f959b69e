/*
 * kern.h -- shared by the kernel translation units (k_npp.hip, k_ana.hip,
 * k_dec.hip, engine.hip).
 *
 * Each TU is compiled separately (in parallel) into its own code object, so
 * each has its own copy of the constant tables (g_tab, g_der: tables.h) and
 * exports an upload function, MELPE_TU(name) -> melpe_tu_<name>_upload(),
 * that engine.hip calls once per device.  Kernels are launched through
 * extern "C" wrappers defined next to them (a kernel can only be launched
 * from its own TU without relocatable device code).
 *
 * Execution model: one lane per channel.  A kernel copies the
 * part of the channel's state it uses from its HBM record into the lane's
 * private segment, runs, and copies it back.  The private segment is
 * swizzled per dword across the wave (lane l's dword d at (d*64+l)*4), so
 * the codec's same-index accesses of the 64 channels of a wave coalesce,
 * while the HBM record stays a plain per-channel struct.
 */
#ifndef MELPE_KERN_H
#define MELPE_KERN_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "progprio.h"	/* before the codec: its checkpoint hooks */
#include "codec.h"

using namespace mlp;

#define WAVE 64
/* minimum resident waves per SIMD the encoder / decoder kernels are compiled
 * for (caps VGPRs at 512 / n) */
#ifndef MELPE_ENC_WAVES
#define MELPE_ENC_WAVES 4
#endif
#ifndef MELPE_DEC_WAVES
#define MELPE_DEC_WAVES 4
#endif

/*
 * Private-segment guard.  On gfx950 a FLAT load/store is aperture-checked on
 * its base register BEFORE the unsigned immediate offset is added.  Code that
 * only sees a generic pointer (any out-of-line callee) may fold p[i - k]
 * into (p - k)[i] + offset:k, so a private object lying within 4 KiB of the
 * bottom of the lane's private segment faults with MEMORY_APERTURE_VIOLATION
 * (tools/exp/flat_private.hip, mode 2, reproduces it).  Every kernel that
 * calls into the codec therefore owns exactly one private object whose first
 * member is this guard; callee frames sit above the kernel frame, so no
 * private object the codec touches starts below FLAT_GUARD_BYTES.
 * Since round 4 the build itself fails on any FLAT instruction in a codec
 * kernel (build.py check_no_flat: the codec TUs inline their whole call
 * tree, so every private access is a scratch_ instruction), which removes
 * the hazard the guard covered.  The guard was 4,608 bytes (31% of the lane
 * analysis' frame); the A/B at 262,144 channels measured it time-neutral
 * (profiles/r06_c_flat_guard_ab_262k.txt) and it only inflated every
 * queue's scratch reservation, so it is 16 bytes now (the frame layouts
 * keep their 16-byte alignment).
 */
#ifndef FLAT_GUARD_BYTES
#define FLAT_GUARD_BYTES 16
#endif

/* keep the guard alive: the compiler may not drop or shrink the object */
#define PIN_FRAME(obj) __asm__ volatile("" : : "v"(&(obj)) : "memory")

/* per-lane copy between a channel's HBM record and the lane's private
 * segment, 4 bytes at a time (sizes and offsets are multiples of 4).  The
 * dwords are may_alias: the records are read and written field by field as
 * int16/int32/uint8, and a plain uint32_t copy would let type-based alias
 * analysis treat the last field stores before the copy-out as dead (it did,
 * in k_dec24: the tail of melp_syn never reached HBM); u32_alias is in
 * ops.h. */
__device__ __forceinline__ void lane_copy(void *dst, const void *src, size_t bytes)
{
	u32_alias *d = (u32_alias *) dst;
	const u32_alias *s = (const u32_alias *) src;
#pragma unroll 8
	for (size_t i = 0; i < bytes / 4; i++)
		d[i] = s[i];
}

/* lane_copy for 16-byte aligned ranges (sizes multiples of 16): one
 * dwordx4 load / store per 16 bytes, eight in flight, so each lane pulls a
 * whole 128-byte line of its record per batch instead of re-touching it
 * over four dword batches while the wave's other 63 records stream past */
typedef uint32_t v4u32 __attribute__((ext_vector_type(4), __may_alias__));
__device__ __forceinline__ void lane_copy_x4(void *dst, const void *src, size_t bytes)
{
	v4u32 *d = (v4u32 *) dst;
	const v4u32 *s = (const v4u32 *) src;
#pragma unroll 8
	for (size_t i = 0; i < bytes / 16; i++)
		d[i] = s[i];
}

#define MELPE_CHK(expr) do { hipError_t _e = (expr); if (_e != hipSuccess) return (int) _e; } while (0)

/* per-TU table upload (+ derivation of g_der) and stage-timer readout */
#define MELPE_TU(name)                                                          \
	__global__ void k_derive_##name()                                       \
	{                                                                       \
		if (threadIdx.x == 0 && blockIdx.x == 0)                        \
			derive_all(&g_der);                                     \
	}                                                                       \
	extern "C" int melpe_tu_##name##_upload(const void *blob, size_t bytes) \
	{                                                                       \
		if (bytes != sizeof(int16_t) * MELPE_TABLE_WORDS)               \
			return -1;                                              \
		MELPE_CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_tab), blob, bytes));   \
		k_derive_##name<<<1, WAVE>>>();                                 \
		MELPE_CHK(hipGetLastError());                                   \
		MELPE_CHK(hipDeviceSynchronize());                              \
		int16_t lc_[512], grid_[LSPGRID_BLOCKS * 40];                   \
		MELPE_CHK(hipMemcpyFromSymbol(lc_, HIP_SYMBOL(g_der), sizeof(lc_), \
					      offsetof(DerivedTables, lsp_cos))); \
		derive_lspgrid(lc_, grid_);                                     \
		MELPE_CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_lspgrid), grid_, sizeof(grid_))); \
		return 0;                                                       \
	}                                                                       \
	MELPE_TU_PROF(name)

#if defined(MELPE_PROF)
#define MELPE_TU_PROF(name)                                                     \
	extern "C" int melpe_tu_##name##_prof(uint64_t *acc)                    \
	{                                                                       \
		unsigned long long h[MELPE_PROF_SLOTS];                         \
		MELPE_CHK(hipDeviceSynchronize());                              \
		MELPE_CHK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_prof), sizeof(h))); \
		for (int i = 0; i < MELPE_PROF_SLOTS; i++)                      \
			acc[i] += h[i];                                         \
		memset(h, 0, sizeof(h));                                        \
		MELPE_CHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), h, sizeof(h))); \
		return 0;                                                       \
	}
#else
#define MELPE_TU_PROF(name)                                                     \
	extern "C" int melpe_tu_##name##_prof(uint64_t *acc)                    \
	{                                                                       \
		(void) acc;                                                     \
		return -1;                                                      \
	}
#endif

/* The device-side choice of analysis mapping (engine.hip ana_launch): a
 * launch works only when the live count L its lane-order sort counted lies
 * in (lo, hi], and the launch that works writes its mapping (waves per 64
 * channels: 1 lane, 4 four-wave) into *tag.  The default is always open and
 * writes nothing. */
struct AnaGate {
	int lo = -1, hi = 0x7fffffff;
	int *tag = nullptr;
	__device__ bool open(int L) const { return L > lo && L <= hi; }
	__device__ void mark(bool leader, int waves) const
	{
		if (tag && leader)
			*tag = waves;
	}
};

static inline unsigned grid_for(int n)
{
	return (unsigned) ((n + WAVE - 1) / WAVE);
}


#endif
