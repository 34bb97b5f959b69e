/*
 * engine.hip -- the MI355X MELPe-1200 engine: HIP kernels + the C ABI
 * (include/melpe.h drop-in, include/melpe_batch.h batched).
 *
 * Execution model: one lane per channel.  A channel-superframe is strictly
 * sequential (every stage carries state into the next and the reference's
 * saturating arithmetic is order dependent), so the parallelism is across
 * channels: a wave processes 64 channels in lock-step, a launch processes
 * every active channel of the engine.  Per-channel state lives in HBM
 * (EncState / DecState), the codebooks in g_tab (uploaded once per device).
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <string>
#include <mutex>

#include "codec.h"
#define SYN_FN __host__ __device__ static inline
#include "synth.h"
#include "../../include/melpe.h"
#include "../../include/melpe_batch.h"

using namespace mlp;

/* ------------------------------------------------------------------ */
/* embedded constant tables (oracle/dump_tables.py output)            */
/* ------------------------------------------------------------------ */
#if !defined(__HIP_DEVICE_COMPILE__)
__asm__(".section .rodata\n"
	".balign 16\n"
	".global melpe_tables_blob\n"
	"melpe_tables_blob:\n"
	".incbin \"" MELPE_TABLES_BIN "\"\n"
	".global melpe_tables_blob_end\n"
	"melpe_tables_blob_end:\n"
	".previous\n");
#endif
extern "C" const unsigned char melpe_tables_blob[];
extern "C" const unsigned char melpe_tables_blob_end[];

#define WAVE 64
/* minimum resident waves per SIMD the encoder / decoder kernels are compiled
 * for (caps VGPRs at 512 / n) */
#ifndef MELPE_ENC_WAVES
#define MELPE_ENC_WAVES 2
#endif
#ifndef MELPE_DEC_WAVES
#define MELPE_DEC_WAVES 4
#endif

#if defined(MELPE_PROF)
__device__ unsigned long long g_prof[64];
#endif

/* ------------------------------------------------------------------ */
/* kernels                                                            */
/* ------------------------------------------------------------------ */

__global__ void k_init_tables()
{
	if (threadIdx.x == 0 && blockIdx.x == 0) {
		derive_all(&g_der);
	}
}

__global__ __launch_bounds__(WAVE) void k_reset(EncState *enc, DecState *dec,
						 const uint8_t *mask, int n, int which)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || (mask && !mask[c]))
		return;
	if (which & 1)
		enc_reset(&enc[c]);
	if (which & 2)
		dec_reset(&dec[c]);
}

/*
 * Private-segment guard.  On gfx950 a FLAT load/store is aperture-checked on
 * its base register BEFORE the unsigned immediate offset is added.  Code that
 * only sees a generic pointer (every __noinline__ callee) may fold p[i - k]
 * into (p - k)[i] + offset:k, so a private object lying within 4 KiB of the
 * bottom of the lane's private segment faults with MEMORY_APERTURE_VIOLATION
 * (tools/exp/flat_private.hip, mode 2, reproduces it).  Every kernel that
 * calls into the codec therefore owns exactly one private object whose first
 * member is this guard; callee frames sit above the kernel frame, so no
 * private object the codec touches starts below FLAT_GUARD_BYTES.
 */
#define FLAT_GUARD_BYTES 4608

struct NppLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	NppScratch w;
};

struct DecLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	int16_t out[BLOCK];
};

struct EncLanePriv {
	uint8_t guard[FLAT_GUARD_BYTES];
	NppScratch w;
	EncState S;
	int16_t x[BLOCK];
};

/* per-lane copy between a channel's HBM record and the lane's private
 * segment, 4 bytes at a time (sizes are multiples of 4) */
__device__ __forceinline__ void lane_copy(void *dst, const void *src, size_t bytes)
{
	uint32_t *d = (uint32_t *) dst;
	const uint32_t *s = (const uint32_t *) src;
	for (size_t i = 0; i < bytes / 4; i++)
		d[i] = s[i];
}

/* keep the guard alive: the compiler may not drop or shrink the object */
#define PIN_FRAME(obj) __asm__ volatile("" : : "v"(&(obj)) : "memory")

/* melpe_n on `frames` frames per channel (melpe/melpe.c:63-67) */
__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_npp(EncState *enc, int16_t *sp, int frames,
					       int stride, const uint8_t *active, int n,
					       int rate1200)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || (active && !active[c]))
		return;
	NppLane L;
	PIN_FRAME(L);
	int16_t *x = sp + (size_t) c * stride;
	for (int f = 0; f < frames; f++)
		npp_frame(&enc[c].npp, &L.w, x + f * NPP_HOP, x + f * NPP_HOP, rate1200 != 0);
}

/* melpe_a on every active channel (melpe/melpe.c:91-99): one lane per
 * channel, sp (C x 540) in place, bits (C x 11) out */
__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_encode(EncState *enc, int16_t *sp, uint8_t *bits,
						  const uint8_t *active, int n)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || (active && !active[c]))
		return;
#if defined(MELPE_PRIVATE_STATE)
	EncLanePriv L;
	PIN_FRAME(L);
	lane_copy(&L.S, &enc[c], sizeof(EncState));
	int16_t *x = sp + (size_t) c * BLOCK;
	lane_copy(L.x, x, sizeof(L.x));
	encode_superframe(&L.S, &L.w, L.x);
	lane_copy(&enc[c], &L.S, sizeof(EncState));
	lane_copy(x, L.x, sizeof(L.x));
	for (int k = 0; k < 11; k++)
		bits[(size_t) c * 11 + k] = L.S.chbuf[k];
#else
	NppLane L;
	PIN_FRAME(L);
	EncState *E = &enc[c];
	encode_superframe(E, &L.w, sp + (size_t) c * BLOCK);
	for (int k = 0; k < 11; k++)
		bits[(size_t) c * 11 + k] = E->chbuf[k];
#endif
}

/* debug aid: encode with the pipeline cut after `upto` stages (0 = NPP only) */
__global__ __launch_bounds__(WAVE, MELPE_ENC_WAVES) void k_encode_dbg(EncState *enc, int16_t *sp, int n, int upto)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n)
		return;
	NppLane L;
	PIN_FRAME(L);
	EncState *E = &enc[c];
	int16_t *x = sp + (size_t) c * BLOCK;
	npp_frame(&E->npp, &L.w, x, x);
	npp_frame(&E->npp, &L.w, x + FRAME, x + FRAME);
	npp_frame(&E->npp, &L.w, x + 2 * FRAME, x + 2 * FRAME);
	if (upto > 0)
		analysis_upto(E, x, upto);
}

/* melpe_s on every active channel (melpe/melpe.c:102-107): bits (C x 11) in,
 * sp (C x 540) out */
__global__ __launch_bounds__(WAVE, MELPE_DEC_WAVES) void k_decode(DecState *dec, int16_t *sp,
						  const uint8_t *bits, const uint8_t *active, int n)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n || (active && !active[c]))
		return;
	DecLane L;
	PIN_FRAME(L);
	DecState *D = &dec[c];
	for (int k = 0; k < 11; k++)
		D->chbuf[k] = bits[(size_t) c * 11 + k];
	decode_superframe(D, L.out);
	int16_t *o = sp + (size_t) c * BLOCK;
	for (int i = 0; i < BLOCK; i++)
		o[i] = L.out[i];
}

/* melpe_i on channel 0 of the single-stream engine: melp_ana_init +
 * melp_syn_init (melpe/melpe.c:72-88) */
__global__ void k_melpe_i(EncState *enc, DecState *dec)
{
	if (threadIdx.x == 0) {
		enc_melpe_i(enc);
		dec_melpe_i(dec);
	}
}

/* The reference's analysis and synthesis share melp_par, quant_par and chbuf
 * (melpe/global.c:27-39).  For the single-stream drop-in the engine keeps
 * them in EncState and hands them to the decoder around each melpe_s, so an
 * interleaved melpe_a / melpe_s sequence sees exactly the reference's
 * process-global state.  dir 0: encoder -> decoder, 1: decoder -> encoder. */
__global__ void k_share_params(EncState *enc, DecState *dec, int dir)
{
	if (threadIdx.x != 0)
		return;
	if (dir == 0) {
		for (int i = 0; i < NF; i++)
			dec->par[i] = enc->par[i];
		dec->qpar = enc->qpar;
	} else {
		for (int i = 0; i < NF; i++)
			enc->par[i] = dec->par[i];
		enc->qpar = dec->qpar;
		for (int k = 0; k < 11; k++)
			enc->chbuf[k] = dec->chbuf[k];
	}
}

__global__ __launch_bounds__(WAVE) void k_synth_seed(synth_state *s, uint32_t seed,
						      uint32_t ch0, int n)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c < n)
		synth_init(&s[c], synth_mix(seed, ch0 + (uint32_t) c));
}

__global__ __launch_bounds__(WAVE) void k_synth(synth_state *s, int16_t *out, int samples, int n)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= n)
		return;
	synth_state st = s[c];
	synth_block(&st, out + (size_t) c * samples, samples);
	s[c] = st;
}

/* ------------------------------------------------------------------ */
/* host side                                                          */
/* ------------------------------------------------------------------ */

static thread_local std::string g_err;

static int fail(const char *what, hipError_t e)
{
	g_err = std::string(what) + ": " + hipGetErrorString(e);
	return -1;
}

static int fail_msg(const std::string &m)
{
	g_err = m;
	return -2;
}

#define HIPCHK(expr) do { hipError_t _e = (expr); if (_e != hipSuccess) return fail(#expr, _e); } while (0)

struct melpe_engine {
	int device = 0;
	int channels = 0;
	hipStream_t stream = nullptr;
	hipEvent_t ev0 = nullptr, ev1 = nullptr;
	EncState *d_enc = nullptr;
	DecState *d_dec = nullptr;
	synth_state *d_syn = nullptr;
	int16_t *d_pcm = nullptr;	/* staging for *_host calls */
	unsigned char *d_bits = nullptr;
	uint8_t *d_mask = nullptr;
	float last_ms = 0.f;
};

static std::mutex g_dev_mu;
static bool g_dev_ready[64];

static int ensure_device_tables(int dev)
{
	std::lock_guard<std::mutex> lk(g_dev_mu);
	if (dev < 0 || dev >= 64)
		return fail_msg("bad device index");
	if (g_dev_ready[dev])
		return 0;
	size_t bytes = (size_t) (melpe_tables_blob_end - melpe_tables_blob);
	if (bytes != sizeof(int16_t) * MELPE_TABLE_WORDS)
		return fail_msg("embedded table blob has the wrong size");
	HIPCHK(hipSetDevice(dev));
	HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_tab), melpe_tables_blob, bytes));
	k_init_tables<<<1, WAVE>>>();
	HIPCHK(hipGetLastError());
	HIPCHK(hipDeviceSynchronize());
	g_dev_ready[dev] = true;
	return 0;
}

static inline unsigned grid_for(int n)
{
	return (unsigned) ((n + WAVE - 1) / WAVE);
}

static void ev_begin(melpe_engine *e, hipStream_t s)
{
	hipEventRecord(e->ev0, s);
}

static void ev_end(melpe_engine *e, hipStream_t s, bool sync)
{
	hipEventRecord(e->ev1, s);
	if (sync) {
		hipEventSynchronize(e->ev1);
		hipEventElapsedTime(&e->last_ms, e->ev0, e->ev1);
	} else {
		e->last_ms = -1.f;	/* resolved lazily in melpe_last_kernel_ms */
	}
}

extern "C" {

const char *melpe_last_error(void)
{
	return g_err.c_str();
}

int melpe_engine_create(melpe_engine **out, int device, int channels)
{
	if (!out || channels <= 0)
		return fail_msg("melpe_engine_create: bad arguments");
	int ndev = 0;
	HIPCHK(hipGetDeviceCount(&ndev));
	if (device < 0 || device >= ndev)
		return fail_msg("melpe_engine_create: no such HIP device");
	int rc = ensure_device_tables(device);
	if (rc)
		return rc;
	melpe_engine *e = new melpe_engine();
	e->device = device;
	e->channels = channels;
	HIPCHK(hipSetDevice(device));
	HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
	HIPCHK(hipEventCreate(&e->ev0));
	HIPCHK(hipEventCreate(&e->ev1));
	HIPCHK(hipMalloc(&e->d_enc, sizeof(EncState) * (size_t) channels));
	HIPCHK(hipMalloc(&e->d_dec, sizeof(DecState) * (size_t) channels));
	HIPCHK(hipMalloc(&e->d_syn, sizeof(synth_state) * (size_t) channels));
	HIPCHK(hipMalloc(&e->d_pcm, sizeof(int16_t) * MELPE_SF_SAMPLES * (size_t) channels));
	HIPCHK(hipMalloc(&e->d_bits, (size_t) MELPE_SF_BYTES * channels));
	HIPCHK(hipMalloc(&e->d_mask, (size_t) channels));
	*out = e;
	return melpe_engine_reset(e, nullptr, 3);
}

int melpe_engine_destroy(melpe_engine *e)
{
	if (!e)
		return 0;
	hipSetDevice(e->device);
	if (e->stream)
		hipStreamSynchronize(e->stream);
	hipFree(e->d_enc);
	hipFree(e->d_dec);
	hipFree(e->d_syn);
	hipFree(e->d_pcm);
	hipFree(e->d_bits);
	hipFree(e->d_mask);
	if (e->ev0)
		hipEventDestroy(e->ev0);
	if (e->ev1)
		hipEventDestroy(e->ev1);
	if (e->stream)
		hipStreamDestroy(e->stream);
	delete e;
	return 0;
}

int melpe_engine_channels(const melpe_engine *e)
{
	return e ? e->channels : 0;
}

static const uint8_t *stage_mask(melpe_engine *e, const uint8_t *mask_host, int *rc)
{
	*rc = 0;
	if (!mask_host)
		return nullptr;
	hipError_t er = hipMemcpyAsync(e->d_mask, mask_host, (size_t) e->channels,
				       hipMemcpyHostToDevice, e->stream);
	if (er != hipSuccess)
		*rc = fail("hipMemcpyAsync(mask)", er);
	return e->d_mask;
}

int melpe_engine_reset(melpe_engine *e, const uint8_t *mask_host, int which)
{
	if (!e)
		return fail_msg("null engine");
	HIPCHK(hipSetDevice(e->device));
	int rc;
	const uint8_t *m = stage_mask(e, mask_host, &rc);
	if (rc)
		return rc;
	k_reset<<<grid_for(e->channels), WAVE, 0, e->stream>>>(e->d_enc, e->d_dec, m,
								  e->channels, which);
	HIPCHK(hipGetLastError());
	HIPCHK(hipStreamSynchronize(e->stream));
	return 0;
}

static int npp_launch(melpe_engine *e, int16_t *d_sp, int frames, int stride,
		      const uint8_t *d_act, hipStream_t s, bool sync, int rate1200)
{
	if (frames <= 0 || stride < frames * MELPE_FRAME_SAMPLES)
		return fail_msg("melpe_npp: bad frames/stride");
	HIPCHK(hipSetDevice(e->device));
	ev_begin(e, s);
	k_npp<<<grid_for(e->channels), WAVE, 0, s>>>(e->d_enc, d_sp, frames, stride, d_act,
						       e->channels, rate1200);
	HIPCHK(hipGetLastError());
	ev_end(e, s, sync);
	return 0;
}

int melpe_npp_dev(melpe_engine *e, void *d_sp, int frames, int stride, const void *d_active,
		  void *hip_stream)
{
	if (!e || !d_sp)
		return fail_msg("melpe_npp_dev: null argument");
	return npp_launch(e, (int16_t *) d_sp, frames, stride, (const uint8_t *) d_active,
			  (hipStream_t) hip_stream, false, 1);
}

int melpe_npp_host(melpe_engine *e, int16_t *sp, int frames, int stride, const uint8_t *active)
{
	if (!e || !sp)
		return fail_msg("melpe_npp_host: null argument");
	HIPCHK(hipSetDevice(e->device));
	size_t bytes = sizeof(int16_t) * (size_t) stride * e->channels;
	int16_t *d = nullptr;
	HIPCHK(hipMalloc(&d, bytes));
	int rc;
	const uint8_t *m = stage_mask(e, active, &rc);
	if (!rc) {
		hipMemcpyAsync(d, sp, bytes, hipMemcpyHostToDevice, e->stream);
		rc = npp_launch(e, d, frames, stride, m, e->stream, true, 1);
		if (!rc) {
			hipError_t er = hipMemcpyAsync(sp, d, bytes, hipMemcpyDeviceToHost, e->stream);
			if (er == hipSuccess)
				er = hipStreamSynchronize(e->stream);
			if (er != hipSuccess)
				rc = fail("npp copy back", er);
		}
	}
	hipFree(d);
	return rc;
}

static int encode_launch(melpe_engine *e, unsigned char *d_bits, int16_t *d_sp,
			 const uint8_t *d_act, hipStream_t s, bool sync)
{
	HIPCHK(hipSetDevice(e->device));
	ev_begin(e, s);
	k_encode<<<grid_for(e->channels), WAVE, 0, s>>>(e->d_enc, d_sp, d_bits, d_act,
							  e->channels);
	HIPCHK(hipGetLastError());
	ev_end(e, s, sync);
	return 0;
}

int melpe_encode_dev(melpe_engine *e, void *d_bits, void *d_sp, const void *d_active,
		     void *hip_stream)
{
	if (!e || !d_bits || !d_sp)
		return fail_msg("melpe_encode_dev: null argument");
	return encode_launch(e, (unsigned char *) d_bits, (int16_t *) d_sp,
			     (const uint8_t *) d_active, (hipStream_t) hip_stream, false);
}

int melpe_encode_host(melpe_engine *e, unsigned char *bits, int16_t *sp, const uint8_t *active)
{
	if (!e || !bits || !sp)
		return fail_msg("melpe_encode_host: null argument");
	HIPCHK(hipSetDevice(e->device));
	size_t pb = sizeof(int16_t) * BLOCK * (size_t) e->channels;
	size_t bb = (size_t) 11 * e->channels;
	int rc;
	const uint8_t *m = stage_mask(e, active, &rc);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(e->d_pcm, sp, pb, hipMemcpyHostToDevice, e->stream));
	if (active)	/* inactive channels keep the caller's bits */
		HIPCHK(hipMemcpyAsync(e->d_bits, bits, bb, hipMemcpyHostToDevice, e->stream));
	rc = encode_launch(e, e->d_bits, e->d_pcm, m, e->stream, true);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(sp, e->d_pcm, pb, hipMemcpyDeviceToHost, e->stream));
	HIPCHK(hipMemcpyAsync(bits, e->d_bits, bb, hipMemcpyDeviceToHost, e->stream));
	HIPCHK(hipStreamSynchronize(e->stream));
	return 0;
}

static int decode_launch(melpe_engine *e, int16_t *d_sp, const unsigned char *d_bits,
			 const uint8_t *d_act, hipStream_t s, bool sync)
{
	HIPCHK(hipSetDevice(e->device));
	ev_begin(e, s);
	k_decode<<<grid_for(e->channels), WAVE, 0, s>>>(e->d_dec, d_sp, d_bits, d_act,
							  e->channels);
	HIPCHK(hipGetLastError());
	ev_end(e, s, sync);
	return 0;
}

int melpe_decode_dev(melpe_engine *e, void *d_sp, const void *d_bits, const void *d_active,
		     void *hip_stream)
{
	if (!e || !d_sp || !d_bits)
		return fail_msg("melpe_decode_dev: null argument");
	return decode_launch(e, (int16_t *) d_sp, (const unsigned char *) d_bits,
			     (const uint8_t *) d_active, (hipStream_t) hip_stream, false);
}

int melpe_decode_host(melpe_engine *e, int16_t *sp, const unsigned char *bits,
		      const uint8_t *active)
{
	if (!e || !bits || !sp)
		return fail_msg("melpe_decode_host: null argument");
	HIPCHK(hipSetDevice(e->device));
	size_t pb = sizeof(int16_t) * BLOCK * (size_t) e->channels;
	size_t bb = (size_t) 11 * e->channels;
	int rc;
	const uint8_t *m = stage_mask(e, active, &rc);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(e->d_bits, bits, bb, hipMemcpyHostToDevice, e->stream));
	if (active)	/* inactive channels keep the caller's samples */
		HIPCHK(hipMemcpyAsync(e->d_pcm, sp, pb, hipMemcpyHostToDevice, e->stream));
	rc = decode_launch(e, e->d_pcm, e->d_bits, m, e->stream, true);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(sp, e->d_pcm, pb, hipMemcpyDeviceToHost, e->stream));
	HIPCHK(hipStreamSynchronize(e->stream));
	return 0;
}

int melpe_synth_seed(melpe_engine *e, uint32_t run_seed, uint32_t first_channel)
{
	if (!e)
		return fail_msg("null engine");
	HIPCHK(hipSetDevice(e->device));
	k_synth_seed<<<grid_for(e->channels), WAVE, 0, e->stream>>>(e->d_syn, run_seed,
								      first_channel, e->channels);
	HIPCHK(hipGetLastError());
	HIPCHK(hipStreamSynchronize(e->stream));
	return 0;
}

int melpe_synth_dev(melpe_engine *e, void *d_sp, int samples, void *hip_stream)
{
	if (!e || !d_sp || samples <= 0)
		return fail_msg("melpe_synth_dev: bad arguments");
	HIPCHK(hipSetDevice(e->device));
	k_synth<<<grid_for(e->channels), WAVE, 0, (hipStream_t) hip_stream>>>(
		e->d_syn, (int16_t *) d_sp, samples, e->channels);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_synth_host(uint32_t run_seed, uint32_t channel, int16_t *out, int samples)
{
	synth_state st;
	synth_init(&st, synth_mix(run_seed, channel));
	synth_block(&st, out, samples);
	return 0;
}

int melpe_debug_encode_stage(melpe_engine *e, void *d_sp, int upto)
{
	HIPCHK(hipSetDevice(e->device));
	k_encode_dbg<<<grid_for(e->channels), WAVE, 0, e->stream>>>(e->d_enc, (int16_t *) d_sp,
								      e->channels, upto);
	HIPCHK(hipGetLastError());
	HIPCHK(hipStreamSynchronize(e->stream));
	return 0;
}

int melpe_prof_read(uint64_t *out, int n)
{
#if defined(MELPE_PROF)
	unsigned long long h[64];
	HIPCHK(hipDeviceSynchronize());
	HIPCHK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_prof), sizeof(h)));
	for (int i = 0; i < n && i < 64; i++)
		out[i] = h[i];
	memset(h, 0, sizeof(h));
	HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), h, sizeof(h)));
	return 64;
#else
	(void) out;
	(void) n;
	return fail_msg("not a profiling build (-DMELPE_PROF)");
#endif
}

double melpe_last_kernel_ms(const melpe_engine *ce)
{
	melpe_engine *e = (melpe_engine *) ce;
	if (!e)
		return 0.0;
	if (e->last_ms < 0.f) {
		if (hipEventSynchronize(e->ev1) != hipSuccess ||
		    hipEventElapsedTime(&e->last_ms, e->ev0, e->ev1) != hipSuccess)
			e->last_ms = 0.f;
	}
	return e->last_ms;
}

/* ------------------------------------------------------------------ */
/* single-stream drop-in (include/melpe.h)                            */
/* ------------------------------------------------------------------ */

static melpe_engine *g_single = nullptr;
static bool g_single_rate1200 = false;	/* melpe_i sets rate = RATE1200 */

static melpe_engine *single_engine(void)
{
	if (!g_single) {
		if (melpe_engine_create(&g_single, 0, 1)) {
			fprintf(stderr, "libmelpe_amd: no usable GPU: %s\n", g_err.c_str());
			abort();
		}
	}
	return g_single;
}

void melpe_n(short *sp)
{
	melpe_engine *e = single_engine();
	int16_t buf[256];
	/* the first call reads 256 samples (melpe/npp.c:178-179) */
	memcpy(buf, sp, sizeof(int16_t) * 180);
	memcpy(buf + 180, sp + 180, sizeof(int16_t) * 76);
	int16_t *d = e->d_pcm;
	if (hipMemcpy(d, buf, sizeof(buf), hipMemcpyHostToDevice) != hipSuccess ||
	    npp_launch(e, d, 1, 256, nullptr, e->stream, true, g_single_rate1200 ? 1 : 0) ||
	    hipMemcpy(sp, d, sizeof(int16_t) * 180, hipMemcpyDeviceToHost) != hipSuccess) {
		fprintf(stderr, "libmelpe_amd: melpe_n failed: %s\n", g_err.c_str());
		abort();
	}
}

int melpe_single_reset(void)
{
	melpe_engine *e = single_engine();
	g_single_rate1200 = false;
	return melpe_engine_reset(e, nullptr, 3);
}

void melpe_i(void)
{
	melpe_engine *e = single_engine();
	k_melpe_i<<<1, WAVE, 0, e->stream>>>(e->d_enc, e->d_dec);
	if (hipGetLastError() != hipSuccess || hipStreamSynchronize(e->stream) != hipSuccess) {
		fprintf(stderr, "libmelpe_amd: melpe_i failed\n");
		abort();
	}
	g_single_rate1200 = true;
}

void melpe_a(unsigned char *buf, short *sp)
{
	melpe_engine *e = single_engine();
	if (melpe_encode_host(e, buf, sp, nullptr)) {
		fprintf(stderr, "libmelpe_amd: melpe_a failed: %s\n", g_err.c_str());
		abort();
	}
}

void melpe_s(short *sp, unsigned char *buf)
{
	melpe_engine *e = single_engine();
	k_share_params<<<1, WAVE, 0, e->stream>>>(e->d_enc, e->d_dec, 0);
	int rc = hipGetLastError() != hipSuccess;
	if (!rc)
		rc = melpe_decode_host(e, sp, buf, nullptr);
	if (!rc) {
		k_share_params<<<1, WAVE, 0, e->stream>>>(e->d_enc, e->d_dec, 1);
		rc = hipGetLastError() != hipSuccess || hipStreamSynchronize(e->stream) != hipSuccess;
	}
	if (rc) {
		fprintf(stderr, "libmelpe_amd: melpe_s failed: %s\n", g_err.c_str());
		abort();
	}
}

}  // extern "C"
