/*
 * progprio.h -- progress-driven issue priority of the lane-per-channel codec
 * kernels (k_enc_ana, k_decode), compiled in where a TU defines
 * MELPE_PROG_PRIO before including kern.h.
 *
 * Such a launch holds every one of its waves resident from its first cycle
 * (four per SIMD at 262,144 channels), so it lasts as long as its slowest
 * wave, and the SIMD's arbiter, which favours the oldest wave at equal
 * priority, decides much of who is slowest.  Measured per wave on the lane
 * analysis (profiles/r06_m_wave_place.txt, r06_q_stage_quarters.txt): the
 * first quarter of the lane order -- dispatched first, so the oldest wave on
 * each SIMD -- took 19.4 ms and the last 24.6 ms; even data-independent
 * stages (lpc_acor) ran 37% slower in the last quarter, and inverting the
 * priority by quarter inverted the times.  So each wave counts the
 * checkpoints it passes (ANA_CKPT in encoder.h: after each frame and after
 * lsf_vq; DEC_CKPT in decoder.h: after each frame) on one counter per launch
 * and sets its priority from how far it is behind the average.  The waves
 * then end together (profiles/r06_r_prio_wave_times.txt).  The four-wave
 * analysis (k_enc_ana_mw) measured neutral with a checkpoint every fourth
 * phase (7.47-7.51 vs 7.48-7.57 ms at 32,768 channels,
 * profiles/r06_t_mw_prio_ab.txt): its workgroup barriers already pace its
 * waves, so it has none.  The counter is
 * word 2 NBIN + 2 of the lane-order sort's control block (engine.hip
 * BinBuf, zeroed by k_bin_scan before each launch), so it needs the lane
 * order; MELPE_ANA_PRIO=0 / MELPE_DEC_PRIO=0 turn it off for A/Bs.
 * Priority changes only the order in which waves issue, never a value.
 */
#ifndef MELPE_PROGPRIO_H
#define MELPE_PROGPRIO_H

#if defined(MELPE_PROG_PRIO) && defined(__HIP_DEVICE_COMPILE__)
static __shared__ unsigned *s_pp_cnt;	/* the launch's counter; null: off */
static __shared__ int s_pp_nw;		/* its live waves */

/* at the start of a kernel, by every lane of every wave of the workgroup
 * (the same values) */
__device__ __forceinline__ void pp_begin(unsigned *cnt, int nw)
{
	s_pp_cnt = cnt;
	s_pp_nw = nw > 0 ? nw : 1;
	if (cnt)
		__builtin_amdgcn_s_setprio(1);
}

/* checkpoint j (1, 2, ...) of the wave */
__device__ __forceinline__ void pp_ckpt(int j)
{
	unsigned *cnt = s_pp_cnt;
	if (!cnt)
		return;
	/* a global-address-space atomic (the pointer came through LDS, which
	 * would otherwise leave a generic FLAT access: build.py check_no_flat) */
	typedef __attribute__((address_space(1))) unsigned gu32;
	unsigned before = 0;
	if (__builtin_amdgcn_readfirstlane(threadIdx.x) == threadIdx.x)
		before = __hip_atomic_fetch_add((gu32 *) cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	before = __builtin_amdgcn_readfirstlane(before);
	/* checkpoints passed before this one, per wave on average and by this
	 * wave, times 4: d > 0 ahead of the average, d < 0 behind */
	const int d = 4 * (j - 1) - (int) ((4ull * before) / (unsigned) s_pp_nw);
	if (d < -2)
		__builtin_amdgcn_s_setprio(3);
	else if (d < 0)
		__builtin_amdgcn_s_setprio(2);
	else if (d < 2)
		__builtin_amdgcn_s_setprio(1);
	else
		__builtin_amdgcn_s_setprio(0);
}
#define PP_BEGIN(cnt, nw) pp_begin((cnt), (nw))
#define ANA_CKPT(j) pp_ckpt(j)
#define DEC_CKPT(j) pp_ckpt(j)
#else
#define PP_BEGIN(cnt, nw) ((void) 0)
#endif

#endif
