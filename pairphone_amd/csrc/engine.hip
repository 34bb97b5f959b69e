/*
 * engine.hip -- host side of the MI355X MELPe-1200 engine: the C ABI
 * (include/melpe.h drop-in, include/melpe_batch.h batched), device table
 * upload, and the small kernels (reset, init, parameter sharing, the
 * synthetic test-signal generator).
 *
 * The codec kernels live in their own translation units, compiled in
 * parallel (pairphone_amd/build.py) and linked into libmelpe_amd.so:
 *   k_npp.hip  melpe_n, and the NPP half of melpe_a (melpe/melpe.c:94-96)
 *   k_ana.hip  the analysis half of melpe_a (melpe/melpe.c:97-98)
 *   k_dec.hip  melpe_s (melpe/melpe.c:102-107)
 * Execution model: one lane per channel (kern.h).  Per-channel
 * state lives in HBM (EncState / DecState), the codebooks in each TU's
 * constant tables (uploaded once per device).
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <string>
#include <mutex>
#include <vector>

#include "kern.h"
#define SYN_FN __host__ __device__ static inline
#include "synth.h"
#include "voice_crypt.h"
#include "vad.h"
#include "ops_eval.h"
#include "helpers_eval.h"
#define MODEM_FN __host__ __device__ static inline
#include "modem.h"
#include "../../include/melpe.h"
#include "../../include/melpe_batch.h"

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

MELPE_TU(eng)

/* kernels of the other translation units (k_npp.hip, k_ana.hip, k_dec.hip) */
extern "C" {
int melpe_tu_npp_upload(const void *blob, size_t bytes);
int melpe_tu_ana_upload(const void *blob, size_t bytes);
int melpe_tu_anamw_upload(const void *blob, size_t bytes);
int melpe_tu_harm_upload(const void *blob, size_t bytes);
int melpe_tu_dec_upload(const void *blob, size_t bytes);
int melpe_tu_r24_upload(const void *blob, size_t bytes);
int melpe_tu_r24_prof(uint64_t *acc);
int melpe_tu_npp_prof(uint64_t *acc);
int melpe_tu_ana_prof(uint64_t *acc);
int melpe_tu_anamw_prof(uint64_t *acc);
int melpe_tu_harm_prof(uint64_t *acc);
int melpe_tu_dec_prof(uint64_t *acc);
int kl_npp(EncState *enc, int16_t *sp, int frames, int stride, const uint8_t *active, int n,
	   int rate1200, hipStream_t s);
int kl_enc_npp(EncState *enc, int16_t *sp, const uint8_t *active, int n, hipStream_t s);
int kl_enc_ana(EncState *enc, const int16_t *sp, uint8_t *bits, const uint8_t *active, int n,
	       const int *perm, const int *nlive, int16_t *res, AnaGate gate, hipStream_t s);
int kl_enc_harm(EncState *enc, const int16_t *res, const uint8_t *active, int n, const int *perm,
		const int *nlive, AnaGate gate, hipStream_t s);
int kl_enc_tail(EncState *enc, uint8_t *bits, const uint8_t *active, int n, const int *perm,
		const int *nlive, AnaGate gate, hipStream_t s);
int kl_enc_ana_mw(EncState *enc, const int16_t *sp, uint8_t *bits, const uint8_t *active, int n,
		  const int *perm, const int *nlive, int nw, uint32_t *lqbuf, AnaGate gate, hipStream_t s);
size_t kl_enc_ana_mw_lq_words(int n);
int kl_enc_ana_dbg(EncState *enc, const int16_t *sp, int n, int upto, hipStream_t s);
int kl_npp_warm(int n, hipStream_t s);
int kl_ana_warm(int n, hipStream_t s);
int kl_harm_warm(int n, hipStream_t s);
int kl_ana_mw_warm(int n, hipStream_t s);
int kl_dec_warm(int n, hipStream_t s);
int kl_dec2_warm(int n, hipStream_t s);
size_t kl_ana_private(void);
size_t kl_ana_mw_private(void);
size_t kl_harm_private(void);
size_t kl_harm_wave_private(void);
size_t kl_npp_private(void);
size_t kl_dec_private(void);
size_t kl_dec2_private(void);
size_t kl_decode2_hb_words(int n);
int kl_decode2(DecState *dec, int16_t *sp, const uint8_t *bits, const uint8_t *active, int n,
	       const int *perm, const int *nlive, uint32_t *hbuf, hipStream_t s);
int kl_decode(DecState *dec, int16_t *sp, const uint8_t *bits, const uint8_t *active, int n,
	      const int *perm, const int *nlive,
	      hipStream_t s);
int kl_enc24(EncState *enc, const int16_t *sp, uint8_t *bits, const uint8_t *active, int n,
	     hipStream_t s);
int kl_dec24(DecState *dec, int16_t *sp, const uint8_t *bits, const uint8_t *active, int n,
	     hipStream_t s);
}

/* ------------------------------------------------------------------ */
/* small kernels: reset, init, parameter sharing, test-signal synth   */
/* ------------------------------------------------------------------ */

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

/* melpe_i on channel 0 of the single-stream engine: melp_ana_init +
 * melp_syn_init (melpe/melpe.c:72-88) */
__global__ void k_melpe_i(EncState *enc, DecState *dec)
{
	if (threadIdx.x == 0) {
		enc_melpe_i(&enc->a);
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
	EncAna *a = &enc->a;
	if (dir == 0) {
		for (int i = 0; i < NF; i++)
			dec->par[i] = a->par[i];
		dec->qpar = a->qpar;
	} else {
		for (int i = 0; i < NF; i++)
			a->par[i] = dec->par[i];
		a->qpar = dec->qpar;
		for (int k = 0; k < 11; k++)
			a->chbuf[k] = dec->chbuf[k];
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


/* VoiceEnc / VoiceDec (crp.c:986-1027, voice_crypt.h), one lane per packet:
 * packet k of channel c is pkts[(c*K + k)*11 ..], its counter counters[c] + k
 * (cnt_out / cnt_in advance by one per packet, crp.c:805), its key the
 * channel's 16 bytes keys[c*16 ..] */
__global__ __launch_bounds__(256) void k_voice_crypt(unsigned char *pkts, const uint32_t *counters,
						     const uint4 *keys, const uint8_t *invert,
						     int channels, int packets, int dir)
{
	long i = blockIdx.x * (long) blockDim.x + threadIdx.x;
	if (i >= (long) channels * packets)
		return;
	int c = (int) (i / packets), k = (int) (i - (long) c * packets);
	uint4 kv = keys[c];
	uint32_t key[4] = {kv.x, kv.y, kv.z, kv.w};
	unsigned char *p = pkts + i * VC_PKT_BYTES;
	unsigned char b[VC_PKT_BYTES];
#pragma unroll
	for (int j = 0; j < VC_PKT_BYTES; j++)
		b[j] = p[j];
	vc_apply(b, counters[c] + (uint32_t) k, key, dir, invert ? invert[c] : 0);
#pragma unroll
	for (int j = 0; j < VC_PKT_BYTES; j++)
		p[j] = b[j];
}


/* VAD of one superframe per channel (vad.h): the six vad2 windows of
 * tx.c:234-239 on the channel's 540 samples; votes[c] = their sum */
__global__ __launch_bounds__(WAVE) void k_vad(VadState *st, const int16_t *sp, uint8_t *votes,
					      uint8_t *gate, const uint8_t *active, int channels)
{
	int c = blockIdx.x * blockDim.x + threadIdx.x;
	if (c >= channels)
		return;
	if (active && !active[c]) {
		if (gate)
			gate[c] = 0;
		return;
	}
	VadState s = st[c];
	int n = va_superframe(sp + (size_t) c * MELPE_SF_SAMPLES, &s);
	st[c] = s;
	votes[c] = (uint8_t) n;
	if (gate)	/* tx.c:242-244: encoded when any window voted */
		gate[c] = n > 0;
}

__global__ __launch_bounds__(WAVE) void k_vad_reset(VadState *st, const uint8_t *mask, int channels)
{
	int c = blockIdx.x * blockDim.x + threadIdx.x;
	if (c >= channels || (mask && !mask[c]))
		return;
	VadState z;
	memset(&z, 0, sizeof z);
	st[c] = z;
}

/* Modulate (modem.h, modem/modem.c:136): one wave per (channel, packet).
 * The packet's starting state follows from the channel's state at launch:
 * the previous bit is the last bit of the previous packet (its parity bit
 * 89) and the muting flag alternates per packet.  Lane pairs of samples are
 * stored as dwords: coalesced 6,480-byte rows per packet. */
__global__ __launch_bounds__(256) void k_modulate(ModemState *st, const uint8_t *pkts, int16_t *pcm,
						  int channels, int packets, const uint8_t *active)
{
	long w = blockIdx.x * 4L + threadIdx.x / WAVE;
	int lane = threadIdx.x % WAVE;
	if (w >= (long) channels * packets)
		return;
	int c = (int) (w / packets), k = (int) (w - (long) c * packets);
	if (active && !active[c])
		return;
	const uint8_t *d = pkts + w * 11;
	int prev0 = k ? modem_tx_bit(d - 11, MODEM_BITS - 1) : st[c].lastb;
	int vad = st[c].vadtr ^ (k & 1);
	uint32_t *o = (uint32_t *) (pcm + w * MODEM_PKT_SAMPLES);
	for (int q = lane; q < MODEM_PKT_SAMPLES / 2; q += WAVE) {
		int s0 = 2 * q, t = s0 / 36, ii = s0 - 36 * t;
		int b = modem_tx_bit(d, t);
		int prev = t ? modem_tx_bit(d, t - 1) : prev0;
		uint32_t lo = (uint16_t) modem_sample(b, prev, vad, ii);
		uint32_t hi = (uint16_t) modem_sample(b, prev, vad, ii + 1);
		o[q] = lo | (hi << 16);
	}
}

/* the state update of a whole modulate launch, after k_modulate has read it */
__global__ __launch_bounds__(WAVE) void k_modulate_state(ModemState *st, const uint8_t *pkts,
							 int channels, int packets, const uint8_t *active)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= channels || (active && !active[c]))
		return;
	st[c].lastb = modem_tx_bit(pkts + ((long) c * packets + packets - 1) * 11, MODEM_BITS - 1);
	st[c].vadtr ^= packets & 1;
}

/* Demodulate (modem.h, modem/modem.c:186): one lane per channel, `calls`
 * successive calls as rx.c:294-297 makes them (pos advances by the return
 * value, data persists); a call that would read past the channel's stride
 * returns -1 and stops the channel.
 *
 * Each lane reads its own row, so a direct read of the stream is a 2-byte
 * load whose 64 lanes touch 64 different rows -- ~1,900 of them per call.
 * Instead the samples of up to DEMOD_CALLS calls are staged once into the
 * lane's private segment with 16-byte loads, and the calls read them from
 * there, where the hardware interleaves the 64 lanes' copies per dword: the
 * same-index reads of a wave are one contiguous 256-byte access. */
#define DEMOD_CALLS 15	/* calls per staged window (one packet time) */
#define DEMOD_ADV_MAX (MODEM_BLOCK_SAMPLES + 8)	/* a call's largest return (q <= 8) */
#define DEMOD_WIN (((DEMOD_CALLS - 1) * DEMOD_ADV_MAX + MODEM_LOOKAHEAD + 8 + 7) & ~7)

struct DemodLane {
	uint8_t guard[FLAT_GUARD_BYTES];
	ModemState S;
	alignas(16) int16_t w[DEMOD_WIN];
};

/* w[sh + i] = src[i], i < n, where sh = the samples before src in its
 * 16-byte line: whole lines by dwordx4 (each starts at or after the line
 * that holds src[0], and ends at or before src[n]), the last partial line
 * sample by sample, so nothing past src[n - 1] is read */
__device__ __forceinline__ int demod_stage(int16_t *w, const int16_t *src, int n)
{
	const int sh = (int) (((uintptr_t) src & 15) >> 1);
	/* pointer arithmetic on src (not an integer cast) keeps the global
	 * address space, so these are global_ loads, not FLAT */
	const v4u32 *g = (const v4u32 *) (src - sh);
	v4u32 *d = (v4u32 *) w;
	const int full = (sh + n) >> 3;
	int k = 0;
	for (; k + 8 <= full; k += 8) {	/* eight loads in flight, then the stores */
		v4u32 t[8];
#pragma unroll
		for (int j = 0; j < 8; j++)
			t[j] = g[k + j];
#pragma unroll
		for (int j = 0; j < 8; j++)
			d[k + j] = t[j];
	}
	for (; k < full; k++)
		d[k] = g[k];
	for (int i = full * 8 - sh; i < n; i++)
		w[sh + i] = src[i];
	return sh;
}

__global__ __launch_bounds__(WAVE) void k_demodulate(ModemState *st, const int16_t *pcm, long stride,
						     int32_t *pos, uint8_t *data, uint8_t *out,
						     int32_t *ret, int channels, int calls,
						     const uint8_t *active)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= channels || (active && !active[c]))
		return;
	DemodLane L;
	PIN_FRAME(L);
	L.S = st[c];
	uint8_t d[12];
	for (int i = 0; i < 12; i++)
		d[i] = data[12L * c + i];
	int32_t p = pos[c];
	const int16_t *x = pcm + (long) c * stride;
	int32_t r = 0;
	for (int k0 = 0; k0 < calls && r >= 0; k0 += DEMOD_CALLS) {
		const int nk = calls - k0 < DEMOD_CALLS ? calls - k0 : DEMOD_CALLS;
		/* the window: from p, the lookahead of the chunk's last call at
		 * the largest advance per call, never past the row */
		long base = 0;
		if (p >= 0 && p + MODEM_LOOKAHEAD <= stride) {
			long end = (long) p + (long) (nk - 1) * DEMOD_ADV_MAX + MODEM_LOOKAHEAD;
			if (end > stride)
				end = stride;
			base = p - demod_stage(L.w, x + p, (int) (end - p));
		}
		for (int k = k0; k < k0 + nk; k++) {
			r = -1;
			if (p >= 0 && p + MODEM_LOOKAHEAD <= stride) {
				r = modem_demod(&L.S, L.w + (p - base), d);
				p += r;
			}
			if (out)
				for (int i = 0; i < 12; i++)
					out[((long) c * calls + k) * 12 + i] = d[i];
			if (ret)
				ret[(long) c * calls + k] = r;
			if (r < 0)
				break;
		}
	}
	st[c] = L.S;
	pos[c] = p;
	for (int i = 0; i < 12; i++)
		data[12L * c + i] = d[i];
}

__global__ __launch_bounds__(WAVE) void k_modem_reset(ModemState *st, const uint8_t *mask, int channels)
{
	int c = blockIdx.x * WAVE + threadIdx.x;
	if (c >= channels || (mask && !mask[c]))
		return;
	ModemState z;
	modem_reset(&z);
	st[c] = z;
}

/* device basic-op parity test: out[i] = op(a[i], b[i], c[i]) with the
 * device build of ops.h (ops_eval.h) */
__global__ __launch_bounds__(256) void k_ops_eval(int op, const int64_t *A, const int32_t *B,
						  const int32_t *C, int64_t *out, long n)
{
	long i = blockIdx.x * (long) blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	int64_t a = A[i];
	int32_t b = B ? B[i] : 0, c = C ? C[i] : 0;
	int64_t r = 0;
	switch (op) {
#define OPS_CASE(id, name, call) case id: r = (int64_t) (call); break;
	MELPE_OPS_EVAL_LIST(OPS_CASE)
#undef OPS_CASE
	default: r = 0;
	}
	out[i] = r;
}

/* divide_s over its whole domain, 0 <= num <= den < 2^15 (den >= 1): one
 * thread per denominator sums q(num) * (num * 0x9E3779B97F4A7C15 + 1) over
 * every numerator in uint64 arithmetic -- a digest that any wrong quotient
 * changes (tests/test_device_ops.py forms the same sums from the
 * reference's divide_s) */
__global__ __launch_bounds__(256) void k_divide_s_sweep(uint64_t *digest)
{
	const int den = blockIdx.x * blockDim.x + threadIdx.x + 1;
	if (den > 32767)
		return;
	uint64_t h = 0;
	for (int num = 0; num <= den; num++)
		h += (uint64_t) (uint16_t) divide_s((Word16) num, (Word16) den) *
		     ((uint64_t) num * 0x9E3779B97F4A7C15ull + 1u);
	digest[den - 1] = h;
}

/* device helper self-test (helpers_eval.h): lane i copies its HE_N
 * samples into a private array -- the codec's streams read the private
 * segment, at per-lane alignments -- and runs helper `mode` on it with
 * (a, b, len) = args[4i .. 4i+2], HE_OUT int32 results per lane */
__global__ __launch_bounds__(WAVE) void k_helpers_eval(int mode, const int16_t *src, const int32_t *args,
						       int32_t *out, int n)
{
	int i = blockIdx.x * WAVE + threadIdx.x;
	if (i >= n)
		return;
	struct {
		uint8_t guard[FLAT_GUARD_BYTES];
		int16_t buf[HE_N];
		int32_t o[HE_OUT];
	} L;
	PIN_FRAME(L);
	for (int k = 0; k < HE_N; k++)
		L.buf[k] = src[(size_t) i * HE_N + k];
	for (int k = 0; k < HE_OUT; k++)
		L.o[k] = 0;
	he_eval(mode, L.buf, args[4 * i], args[4 * i + 1], args[4 * i + 2], L.o);
	for (int k = 0; k < HE_OUT; k++)
		out[(size_t) i * HE_OUT + k] = L.o[k];
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

/* Every entry point that selects a device restores the caller's current
 * device on return, so a multi-GPU host process (or torch's default device)
 * never sees its current device move under it. */
struct DevGuard {
	int prev = -1;
	hipError_t err = hipSuccess;
	explicit DevGuard(int dev)
	{
		int cur = -1;
		if (hipGetDevice(&cur) == hipSuccess && cur == dev)
			return;
		err = hipSetDevice(dev);
		prev = cur;
	}
	~DevGuard()
	{
		if (prev >= 0)
			hipSetDevice(prev);
	}
};
#define DEVGUARD(dev) DevGuard _dg(dev); HIPCHK(_dg.err)

/* device staging of the engine-less *_host calls (VAD, voice crypt): one
 * buffer per device, grown on demand and kept, instead of a hipMalloc /
 * hipFree pair per call */
struct HostStage {
	std::mutex mu;
	void *p = nullptr;
	size_t n = 0;
};
static HostStage g_stage[64];

static int stage_get(int dev, size_t bytes, void **out)
{
	if (dev < 0 || dev >= 64)
		return fail_msg("bad device index");
	HostStage &h = g_stage[dev];
	if (h.n < bytes) {
		if (h.p)
			HIPCHK(hipFree(h.p));
		h.p = nullptr;
		h.n = 0;
		HIPCHK(hipMalloc(&h.p, bytes));
		h.n = bytes;
	}
	*out = h.p;
	return 0;
}

/*
 * Lane order by pitch class (MELPE_BIN, default on).
 *
 * k_enc_ana and k_decode run one channel per lane, and their loops follow
 * each channel's own pitch period and voicing: a synthesis period costs
 * O(L^2) in realIDFT and a frame holds 180/L of them, the analysis windows
 * and harmonic counts follow the pitch, and unvoiced frames take other
 * branches.  A wave pays the slowest of its 64 channels in every such loop.
 * So before each launch the live channels are counting-sorted into 128
 * classes -- voiced frames of the channel's last superframe (0..3) x its last
 * pitch in 3-sample steps -- and lane g of the kernel runs channel perm[g];
 * lanes at or past the live count exit at once, so a ragged mask also packs
 * the live channels into the fewest waves.  Each channel's arithmetic is
 * untouched (the order only decides which channels share a wave), so the
 * output is the same bit for bit; the order within a class follows the
 * atomics and is not reproducible, which nothing depends on.
 */
#define NBIN 640	/* the largest class count of any key (MELPE_BIN_KEY 3: 4 x 141) */
#define NOT_LIVE 0xffff	/* the key of a channel that is not live */
static_assert(NBIN < NOT_LIVE, "class ids and the not-live mark must fit the uint16 keys");
struct BinBuf {
	int *perm = nullptr;	/* [C] lane -> channel */
	uint16_t *key = nullptr;	/* [C] class of each channel (NOT_LIVE: not live) */
	/* [0, NBIN) counts, [NBIN, 2 NBIN) next slot of each class, [2 NBIN]
	 * the live count, [2 NBIN + 1] the mapping the last analysis launch ran
	 * (AnaGate tag: 1 lane, 4 four-wave; 0 none yet), [2 NBIN + 2] the
	 * launch's progress counter (k_ana.hip ana_ckpt) */
	unsigned *ctl = nullptr;
	/* The buffers are one per engine and direction, but *_dev calls may
	 * come on different streams: the sort of a call waits for the kernel
	 * that read the previous call's order (its stream recorded `done`). */
	hipEvent_t done = nullptr;
	hipStream_t last = nullptr;
	bool used = false;
};

static hipError_t bin_alloc(BinBuf *b, int channels)
{
	size_t pb = sizeof(int) * (size_t) channels, cb = sizeof(unsigned) * (2 * NBIN + 4);
	const size_t kb = sizeof(uint16_t) * (size_t) channels;
	char *p = nullptr;
	hipError_t er = hipMalloc(&p, pb + cb + kb);
	if (er != hipSuccess)
		return er;
	er = hipEventCreateWithFlags(&b->done, hipEventDisableTiming);
	if (er != hipSuccess) {
		hipFree(p);
		return er;
	}
	b->perm = (int *) p;
	b->ctl = (unsigned *) (p + pb);
	b->key = (uint16_t *) (p + pb + cb);
	return hipMemset(b->ctl, 0, cb);
}

/* the class of one record, from its last superframe: the voiced frames
 * (quant_par uv_flag, 0 = voiced) and the pitch (Q7) of its frames.
 * MELPE_BIN_KEY: 3 (default) = voiced count x last pitch in 1-sample steps
 * (568 classes), 4 = the same in 2-sample steps, 0 = in 3-sample steps (the
 * round-2 key), 1 = mean pitch in 2-sample steps, 2 = voiced count x last
 * pitch in 5-sample steps.  Round 5, MI355X, 262,144 channels, two runs
 * each (profiles/r05_s_keys.txt): k_decode 8.52 -> 8.39 ms and the analysis
 * 31.11 -> 31.01 ms from key 0 to key 3. */
__device__ __forceinline__ int bin_class(const char *rec, int off_par, int off_uv, int mode)
{
	const int16_t *uv = (const int16_t *) (rec + off_uv);
	int nv = (uv[0] == 0) + (uv[1] == 0) + (uv[2] == 0);
	int p[NF];
	for (int k = 0; k < NF; k++)
		p[k] = *(const int16_t *) (rec + off_par + k * sizeof(MelpParam)) >> 7;
	int b;
	if (mode == 1) {
		b = ((p[0] + p[1] + p[2]) / 3 - 20) / 2;
		return b < 0 ? 0 : (b > 127 ? 127 : b);
	}
	if (mode == 3 || mode == 4) {	/* voiced count x last pitch in 1- / 2-sample steps */
		const int step = mode == 3 ? 1 : 2, nc = 141 / step + 1;
		b = (p[NF - 1] - 20) / step;
		b = b < 0 ? 0 : (b > nc - 1 ? nc - 1 : b);
		return nv * nc + b;
	}
	if (mode == 2) {
		b = (p[NF - 1] - 20) / 5;
		b = b < 0 ? 0 : (b > 15 ? 15 : b);
		return nv * 16 + b;
	}
	b = (p[NF - 1] - 20) / 3;
	b = b < 0 ? 0 : (b > 31 ? 31 : b);
	return nv * 32 + b;
}

__global__ __launch_bounds__(256) void k_bin_count(const char *rec, size_t stride, int off_par,
						   int off_uv, const uint8_t *active, int n, BinBuf b,
						   int mode)
{
	__shared__ unsigned cnt[NBIN];
	for (int k = threadIdx.x; k < NBIN; k += blockDim.x)
		cnt[k] = 0;
	__syncthreads();
	int c = blockIdx.x * blockDim.x + threadIdx.x;
	if (c < n) {
		int k = NOT_LIVE;
		if (!active || active[c]) {
			k = bin_class(rec + (size_t) c * stride, off_par, off_uv, mode);
			atomicAdd(&cnt[k], 1u);
		}
		b.key[c] = (uint16_t) k;
	}
	__syncthreads();
	for (int k = threadIdx.x; k < NBIN; k += blockDim.x)
		if (cnt[k])
			atomicAdd(&b.ctl[k], cnt[k]);
}

__global__ void k_bin_scan(BinBuf b)
{
	if (threadIdx.x == 0) {
		unsigned acc = 0;
		for (int k = 0; k < NBIN; k++) {
			b.ctl[NBIN + k] = acc;
			acc += b.ctl[k];
		}
		b.ctl[2 * NBIN] = acc;
		b.ctl[2 * NBIN + 1] = 0;	/* the mapping tag: the launch that runs sets it */
		b.ctl[2 * NBIN + 2] = 0;	/* the lane kernels' progress counter (k_ana.hip ana_ckpt) */
	}
}

__global__ __launch_bounds__(256) void k_bin_scatter(int n, BinBuf b)
{
	__shared__ unsigned cnt[NBIN], base[NBIN];
	for (int k = threadIdx.x; k < NBIN; k += blockDim.x)
		cnt[k] = 0;
	__syncthreads();
	int c = blockIdx.x * blockDim.x + threadIdx.x;
	int k = c < n ? b.key[c] : NOT_LIVE;
	unsigned r = 0;
	if (k != NOT_LIVE)
		r = atomicAdd(&cnt[k], 1u);
	__syncthreads();
	for (int j = threadIdx.x; j < NBIN; j += blockDim.x)
		if (cnt[j])
			base[j] = atomicAdd(&b.ctl[NBIN + j], cnt[j]);
	__syncthreads();
	if (k != NOT_LIVE)
		b.perm[base[k] + r] = c;
}

static bool bin_enabled(void)
{
	static int v = -1;
	if (v < 0) {
		const char *s = getenv("MELPE_BIN");
		v = !(s && s[0] == '0');
	}
	return v != 0;
}

/* sorts the live channels of `rec` (records of `stride` bytes) into b.perm on
 * stream s; false when the order is off (identity lanes + mask) */
static int bin_key_mode(void)
{
	static int v = -1;
	if (v < 0) {
		const char *s = getenv("MELPE_BIN_KEY");
		v = s ? atoi(s) : 3;
	}
	return v;
}

/* *on: whether the order is used (false: identity lanes + mask) */
static hipError_t bin_launch(int order, BinBuf &b, const void *rec, size_t stride, int off_par,
			     int off_uv, const uint8_t *active, int n, hipStream_t s, bool *on)
{
	*on = !(order == 0 || (order < 0 && !bin_enabled()));
	if (!*on)
		return hipSuccess;
	hipError_t er;
	if (b.used && b.last != s && (er = hipStreamWaitEvent(s, b.done, 0)) != hipSuccess)
		return er;
	unsigned g = (unsigned) ((n + 255) / 256);
	if ((er = hipMemsetAsync(b.ctl, 0, sizeof(unsigned) * NBIN, s)) != hipSuccess)
		return er;
	k_bin_count<<<g, 256, 0, s>>>((const char *) rec, stride, off_par, off_uv, active, n, b,
				      bin_key_mode());
	if ((er = hipGetLastError()) != hipSuccess)
		return er;
	k_bin_scan<<<1, WAVE, 0, s>>>(b);
	if ((er = hipGetLastError()) != hipSuccess)
		return er;
	k_bin_scatter<<<g, 256, 0, s>>>(n, b);
	return hipGetLastError();
}

/* after the kernel that reads b's order, on the same stream */
static hipError_t bin_release(BinBuf &b, hipStream_t s)
{
	b.last = s;
	b.used = true;
	return hipEventRecord(b.done, s);
}

/* k_enc_ana_mw holds two workgroups (of 4 waves, 64 channels) per CU, so it
 * keeps every workgroup resident up to 512 of them */
#define MW_MAX_CHANNELS (512 * WAVE)
/* the two-wave decoder (k_decode2) by default up to this many channels per
 * engine: 2,048 waves (two per SIMD) at 65,536 channels, where the lane
 * decoder has one wave per SIMD */
#define DEC2_MAX_CHANNELS (1024 * WAVE)

struct melpe_engine {
	int device = 0;
	int channels = 0;
	hipStream_t stream = nullptr;	/* the device's engine stream (g_dev_stream), shared */
	hipEvent_t ev0 = nullptr, ev1 = nullptr;
	hipEvent_t ev_in = nullptr, ev_out = nullptr;	/* EngineCall's hops to and from the engine stream */
	hipEvent_t ev_host = nullptr;	/* host_finish: the end of a host call's own work */
	hipEvent_t ev_pin = nullptr, ev_npp = nullptr;	/* melpe_encode_pipe_dev's hops to / from the NPP stream */
	EncState *d_enc = nullptr;
	DecState *d_dec = nullptr;
	synth_state *d_syn = nullptr;
	int16_t *d_pcm = nullptr;	/* staging for *_host calls */
	unsigned char *d_bits = nullptr;
	uint8_t *d_mask = nullptr;
	int16_t *d_npp = nullptr;	/* staging of melpe_npp_host, grown on demand */
	BinBuf bin_enc, bin_dec;	/* pitch-class lane order of k_enc_ana / k_decode */
	int lane_order = -1;	/* 1 on, 0 off, -1 the MELPE_BIN default */
	int ana_waves = 0;	/* waves per 64 channels in k_enc_ana(_mw); 0: by channel count */
	uint32_t *d_lq = nullptr;	/* k_enc_ana_mw's lsf_vq score rows (engine_reserve) */
	int dec_waves = 0;	/* waves per 64 channels of the decoder; 0: by channel count */
	uint32_t *d_hb = nullptr;	/* k_decode2's hand-over buffers (engine_reserve) */
	/* the live-count mapping (ana_launch): a superframe with at most this
	 * many live channels runs the multi-wave kernel (0: off) */
	int mw_live_max = MW_MAX_CHANNELS;
	size_t scratch_need = 0;	/* bytes of scratch the largest launch takes */
	int16_t *d_res = nullptr;	/* the split lane analysis' windowed residuals (C x NF x LPC_FRAME) */
	/* one event per stream this engine's *_dev calls have used, recorded
	 * after each call: the host-side calls wait on these (engine_wait)
	 * instead of the whole device */
	std::vector<std::pair<hipStream_t, hipEvent_t>> marks;
	std::recursive_mutex mu;	/* guards marks and the BinBuf bookkeeping */
	size_t npp_bytes = 0;
	float last_ms = 0.f;
	/* the host-fed pipeline (melpe_encode_host_async): two device slots;
	 * call k uses slot k & 1 -- its H2D on `cin`, its kernels on the
	 * engine stream, its D2H on `cout`, so superframe k's kernels overlap
	 * the copies of k - 1 and k + 1 */
	struct Slot {
		int16_t *pcm = nullptr;
		unsigned char *bits = nullptr;
		uint8_t *mask = nullptr;
		hipEvent_t loaded = nullptr, done = nullptr, freed = nullptr;
		bool used = false;
	} slot[2];
	hipStream_t cin = nullptr, cout = nullptr;
	/* melpe_duplex_pipe_dev's decoder stream and its hops */
	hipStream_t cdec = nullptr;
	hipEvent_t ev_dec = nullptr;
	long async_calls = 0;
	hipStream_t own = nullptr;	/* melpe_engine_set_own_stream */
};

/*
 * Waves per 64 channels of the analysis kernel.  Lane-per-channel (1) needs
 * about four waves per SIMD to hide its scratch latency; below that the
 * channel count leaves SIMDs idle or alone, and the multi-wave kernel
 * (k_enc_ana_mw, ana_mw.h) spreads each channel's independent chains over
 * 2 or 4 waves instead.  MELPE_ANA_NW overrides the automatic choice
 * (diagnostics), not an explicit melpe_engine_set_ana_waves(1 or 4).
 */
static int ana_nw_env(void)
{
	static int env = -2;
	if (env == -2) {
		const char *v = getenv("MELPE_ANA_NW");
		env = v ? atoi(v) : -1;
	}
	return env;
}

static int ana_waves_for(melpe_engine *e)
{
	const int env = ana_nw_env();
	/* an explicit melpe_engine_set_ana_waves() wins over the environment */
	int nw = e->ana_waves ? e->ana_waves : env;
	if (nw == 1 || nw == 4)
		return nw;
	/* k_enc_ana_mw holds two workgroups (of 4 waves) per CU, so it keeps
	 * every workgroup resident up to 512 of them: 32,768 channels */
	long groups = (e->channels + WAVE - 1) / WAVE;
	return groups <= 512 ? 4 : 1;
}

/* the split lane analysis (k_harm.hip); MELPE_HARM=0 (diagnostics) runs the
 * whole analysis in k_enc_ana */
static bool harm_split(void)
{
	static int v = -1;
	if (v < 0) {
		const char *e = getenv("MELPE_HARM");
		v = !(e && e[0] == '0');
	}
	return v != 0;
}

/* after_sort: recorded on s between the lane-order sort and the analysis
 * kernels (melpe_encode_pipe_dev starts the next superframe's NPP there, so
 * that the analysis' waves are dispatched first and the NPP's fill the
 * slots they free) */
static int ana_launch(melpe_engine *e, const int16_t *d_sp, uint8_t *d_bits, const uint8_t *d_act,
		      hipStream_t s, hipEvent_t after_sort = nullptr)
{
	BinBuf &b = e->bin_enc;
	bool on;
	hipError_t er = bin_launch(e->lane_order, b, e->d_enc, sizeof(EncState),
				   (int) (offsetof(EncState, a) + offsetof(EncAna, par)),
				   (int) (offsetof(EncState, a) + offsetof(EncAna, qpar) + offsetof(QuantParam, uv_flag)),
				   d_act, e->channels, s, &on);
	if (er != hipSuccess)
		return (int) er;
	if (after_sort && (er = hipEventRecord(after_sort, s)) != hipSuccess)
		return (int) er;
	const int *perm = on ? b.perm : nullptr;
	const int *nlive = on ? (const int *) (b.ctl + 2 * NBIN) : nullptr;
	int nw = ana_waves_for(e);
	AnaGate all;
	all.tag = (int *) (b.ctl + 2 * NBIN + 1);
	/* Above MW_MAX_CHANNELS the engine runs the lane kernels -- unless few
	 * channels are live (ragged streams, BASELINE config 5).  The live count
	 * is on the device (the lane-order sort counted it), so the choice is
	 * made there: both mappings are enqueued, each gated on the count, and
	 * the one whose range holds it runs (the other's waves leave at once).
	 * No host readback, so host run-ahead cannot make the choice stale.
	 * Either mapping gives the same bits (the four-wave kernel grid-strides
	 * over every live slot). */
	const bool dual = nw == 1 && on && e->ana_waves == 0 && ana_nw_env() < 0 &&
			  e->mw_live_max > 0 && harm_split();
	AnaGate lane = all, mw = all;
	if (dual) {
		lane.lo = e->mw_live_max;
		mw.hi = e->mw_live_max;
	}
	int rc = 0;
	if (dual || nw == 4)
		rc = kl_enc_ana_mw(e->d_enc, d_sp, d_bits, d_act, e->channels, perm, nlive, 4, e->d_lq, mw, s);
	if (rc == 0 && nw == 1) {
		if (harm_split()) {
			/* lane-per-channel analysis up to the Fourier magnitudes,
			 * the magnitudes with a wave per channel, then the packing
			 * (k_harm.hip) */
			rc = kl_enc_ana(e->d_enc, d_sp, d_bits, d_act, e->channels, perm, nlive, e->d_res, lane, s);
			if (rc == 0)
				rc = kl_enc_harm(e->d_enc, e->d_res, d_act, e->channels, perm, nlive, lane, s);
			if (rc == 0)
				rc = kl_enc_tail(e->d_enc, d_bits, d_act, e->channels, perm, nlive, lane, s);
		} else {
			rc = kl_enc_ana(e->d_enc, d_sp, d_bits, d_act, e->channels, perm, nlive, nullptr, lane, s);
		}
	}
	if (rc == 0 && on)
		rc = (int) bin_release(b, s);
	return rc;
}

/* Waves per 64 channels of the decoder: 1 = one lane per channel
 * (k_decode); 2 = the two-wave decoder (k_decode2), for channel counts that
 * leave SIMDs idle in lane mode.  MELPE_DEC_NW overrides the automatic
 * choice (diagnostics), not an explicit melpe_engine_set_dec_waves. */
static int dec_waves_for(melpe_engine *e)
{
	static int env = -2;
	if (env == -2) {
		const char *v = getenv("MELPE_DEC_NW");
		env = v ? atoi(v) : -1;
	}
	int nw = e->dec_waves ? e->dec_waves : env;
	if (nw != 1 && nw != 2)
		nw = e->channels <= DEC2_MAX_CHANNELS ? 2 : 1;
	return nw == 2 && e->d_hb ? 2 : 1;
}

static int dec_launch(melpe_engine *e, int16_t *d_sp, const uint8_t *d_bits, const uint8_t *d_act,
		      hipStream_t s)
{
	BinBuf &b = e->bin_dec;
	bool on;
	hipError_t er = bin_launch(e->lane_order, b, e->d_dec, sizeof(DecState),
				   (int) offsetof(DecState, par),
				   (int) (offsetof(DecState, qpar) + offsetof(QuantParam, uv_flag)),
				   d_act, e->channels, s, &on);
	if (er != hipSuccess)
		return (int) er;
	const int *perm = on ? b.perm : nullptr;
	const int *nlive = on ? (const int *) (b.ctl + 2 * NBIN) : nullptr;
	int rc = dec_waves_for(e) == 2
			 ? kl_decode2(e->d_dec, d_sp, d_bits, d_act, e->channels, perm, nlive, e->d_hb, s)
			 : kl_decode(e->d_dec, d_sp, d_bits, d_act, e->channels, perm, nlive, s);
	if (rc == 0 && on)
		rc = (int) bin_release(b, s);
	return rc;
}

static std::mutex g_dev_mu;
static bool g_dev_ready[64];
/* One stream per device for every engine's own work (create's warm-ups and
 * the host-buffer calls).  The runtime holds kernel scratch per hardware
 * queue and keeps it between dispatches; engines each on a stream of their
 * own end up on every hardware queue the process has, each holding the
 * scratch of the largest codec launch it ran, and together they can exhaust
 * the device's scratch pool (a later launch then aborts its queue with
 * HSA_STATUS_ERROR_OUT_OF_RESOURCES).  Sharing one stream keeps that to one
 * queue plus the callers' own streams. */
static hipStream_t g_dev_stream[64];

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
	DEVGUARD(dev);
	int (*up[])(const void *, size_t) = {melpe_tu_eng_upload, melpe_tu_npp_upload,
					     melpe_tu_ana_upload, melpe_tu_anamw_upload, melpe_tu_harm_upload,
					     melpe_tu_dec_upload, melpe_tu_r24_upload};
	for (auto f : up)
		if (int rc = f(melpe_tables_blob, bytes))
			return fail("table upload", (hipError_t) rc);
	if (hipError_t er = hipStreamCreateWithFlags(&g_dev_stream[dev], hipStreamNonBlocking))
		return fail("engine stream", er);

	g_dev_ready[dev] = true;
	return 0;
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

/* after enqueueing this engine's work on stream s (EngineCall records it on
 * every exit of a call once the call has started enqueueing, error paths
 * included, so a later host-side wait also covers the work a failed call
 * left in flight).  A stream's event is reused; at most MAX_MARKS streams
 * are tracked, beyond that the oldest mark is waited for and recycled. */
#define MAX_MARKS 16
static int engine_mark(melpe_engine *e, hipStream_t s)
{
	for (auto &m : e->marks)
		if (m.first == s) {
			HIPCHK(hipEventRecord(m.second, s));
			return 0;
		}
	if (e->marks.size() >= MAX_MARKS) {
		auto m = e->marks.front();
		e->marks.erase(e->marks.begin());
		HIPCHK(hipEventSynchronize(m.second));
		HIPCHK(hipEventDestroy(m.second));
	}
	hipEvent_t ev;
	HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
	e->marks.emplace_back(s, ev);
	HIPCHK(hipEventRecord(ev, s));
	return 0;
}

/* the host waits for every call of this engine already enqueued, on any
 * stream (not for other engines or unrelated work on the device).  The
 * engines' shared stream needs no wait of its own: every call that enqueues
 * on it synchronises it before returning. */
static int engine_wait(melpe_engine *e)
{
	std::lock_guard<std::recursive_mutex> lk(e->mu);
	for (auto &m : e->marks)
		HIPCHK(hipEventSynchronize(m.second));
	return 0;
}
#define ENGINE_WAIT(e) do { if (int _r = engine_wait(e)) return _r; } while (0)
/* a host-side call (the *_host calls, reset, export / import, synth_seed)
 * holds the engine's lock for its whole body: it stages data through the
 * engine's shared buffers (d_mask, d_pcm, d_bits, d_npp), which another
 * thread's call on the same engine would otherwise overwrite or reallocate
 * under it.  (The lock is recursive: ENGINE_WAIT and EngineCall take it
 * again inside.) */
#define HOST_LOCK(e) std::lock_guard<std::recursive_mutex> _host_lk((e)->mu)
/* the host waits for the work this call enqueued on the engine stream (an
 * event recorded after it), not for work other engines enqueue later */
static int host_finish(melpe_engine *e)
{
	HIPCHK(hipEventRecord(e->ev_host, e->stream));
	HIPCHK(hipEventSynchronize(e->ev_host));
	return 0;
}
#define HOST_FINISH(e) do { if (int _r = host_finish(e)) return _r; } while (0)
/* one *_dev call of an engine: holds the engine's lock (the host-side
 * bookkeeping -- marks, the lane-order buffers -- is shared by the calls of
 * every thread) and records the stream's mark when it ends */
struct EngineCall {
	melpe_engine *e;
	hipStream_t user, run;
	std::lock_guard<std::recursive_mutex> lk;
	bool finished = false;
	EngineCall(melpe_engine *e_, hipStream_t s_) : e(e_), user(s_), run(s_), lk(e_->mu)
	{
		/* the call's kernels run on the device's engine stream, ordered
		 * after the caller's stream and before its later work (two event
		 * hops).  The runtime holds kernel scratch per hardware queue; the
		 * codec kernels' is reserved on the engine stream's queue at create
		 * (engine_reserve), and a second queue running them would hold its
		 * own -- at 14 GB per queue for the analysis kernels two queues
		 * exceed the runtime's threshold and it reclaims one queue's
		 * scratch to grant the other's, hundreds of ms per launch. */
		if (s_ != e->stream && hipEventRecord(e->ev_in, s_) == hipSuccess &&
		    hipStreamWaitEvent(e->stream, e->ev_in, 0) == hipSuccess)
			run = e->stream;
	}
	/* the hop back to the caller's stream and the call's mark; an entry
	 * point returns its result, so a failed hop (the caller's later work
	 * would not be ordered after the kernels) is reported */
	int finish()
	{
		finished = true;
		if (run != user) {
			HIPCHK(hipEventRecord(e->ev_out, run));
			HIPCHK(hipStreamWaitEvent(user, e->ev_out, 0));
		}
		return engine_mark(e, user);
	}
	/* early error returns: the same steps, best effort */
	~EngineCall()
	{
		if (finished)
			return;
		if (run != user && hipEventRecord(e->ev_out, run) == hipSuccess)
			hipStreamWaitEvent(user, e->ev_out, 0);
		engine_mark(e, user);
	}
};
#define ENGINE_CALL(e, s) EngineCall _call(e, s); s = _call.run

extern "C" {

const char *melpe_last_error(void)
{
	return g_err.c_str();
}

/*
 * What the engine's launches need beyond its records, had at create so a
 * shortage fails here and not mid-stream:
 * - the analysis hand-over buffers (the split lane analysis' residuals; the
 *   multi-wave kernel's score rows up to its 512 resident workgroups);
 * - the private-segment scratch of every codec kernel (the lane kernels
 *   hold ~27 KB per lane): the runtime sizes a queue's scratch by the
 *   dispatches it sees, so each kernel is dispatched once on the engine's
 *   stream with the grid of a real launch over the engine's channels and
 *   no live channel (every lane exits at once), and waited for.  (Scratch
 *   is held per hardware queue: a caller's own stream may map to another
 *   queue, whose first dispatch reserves it again.)
 */
/* every codec kernel dispatched once on the engine's stream with the grid
 * of a real launch and no live channel, and waited for: the runtime sizes
 * that hardware queue's scratch by the dispatches it sees */
static int engine_warm(melpe_engine *e)
{
	hipError_t er;
	const int mw = e->channels < MW_MAX_CHANNELS ? e->channels : MW_MAX_CHANNELS;
	int (*warm[])(int, hipStream_t) = {kl_npp_warm, kl_ana_warm, kl_harm_warm, kl_ana_mw_warm, kl_dec_warm};
	for (auto f : warm)
		if ((er = (hipError_t) f(f == kl_ana_mw_warm ? mw : e->channels, e->stream)) != hipSuccess)
			return fail("melpe_engine: codec kernel scratch could not be reserved", er);
	if (e->d_hb && (er = (hipError_t) kl_dec2_warm(e->channels, e->stream)) != hipSuccess)
		return fail("melpe_engine: codec kernel scratch could not be reserved", er);

	if ((er = hipStreamSynchronize(e->stream)) != hipSuccess)
		return fail("melpe_engine: codec kernel scratch could not be reserved", er);
	return 0;
}

static int engine_reserve(melpe_engine *e)
{
	DEVGUARD(e->device);
	hipError_t er;
	if (harm_split() && (er = hipMalloc(&e->d_res, sizeof(int16_t) * NF * LPC_FRAME *
						     (size_t) e->channels)) != hipSuccess) {
		e->d_res = nullptr;
		return fail("melpe_engine_create: analysis residual buffer", er);
	}
	if ((er = hipMalloc(&e->d_lq, sizeof(uint32_t) * kl_enc_ana_mw_lq_words(e->channels))) != hipSuccess) {
		e->d_lq = nullptr;
		return fail("melpe_engine_create: multi-wave score rows", er);
	}
	if (e->channels <= DEC2_MAX_CHANNELS &&
	    (er = hipMalloc(&e->d_hb, sizeof(uint32_t) * kl_decode2_hb_words(e->channels))) != hipSuccess) {
		e->d_hb = nullptr;
		return fail("melpe_engine_create: two-wave decoder hand-over buffers", er);
	}
	const int mw = e->channels < MW_MAX_CHANNELS ? e->channels : MW_MAX_CHANNELS;
	/* The runtime keeps a queue's scratch between dispatches only below its
	 * scratch limit threshold; above it the allocation is made for the
	 * dispatch and given back.  Raise the threshold (never lower it) to
	 * what this engine's largest launch needs: private bytes per lane x 64
	 * lanes x the waves of the launch that can be resident at once (lane
	 * kernels: one per 64 channels; the four-wave kernel: 4 per group, at
	 * most 512 groups; the wave-per-channel kernels k_enc_npp / k_npp and
	 * k_enc_harm: one per channel, up to the device's resident waves). */
	{
		const size_t lane = kl_ana_private() > kl_harm_private() ? kl_ana_private() : kl_harm_private();
		const size_t per_wave = (lane > kl_dec_private() ? lane : kl_dec_private()) * WAVE;
		const size_t mw_wave = kl_ana_mw_private() * WAVE;
		const size_t ww = kl_npp_private() > kl_harm_wave_private() ? kl_npp_private() : kl_harm_wave_private();
		const size_t waves = (size_t) (e->channels + WAVE - 1) / WAVE;
		const size_t mw_waves = 4 * (size_t) ((mw + WAVE - 1) / WAVE);
		size_t resident = (size_t) e->channels;
		hipDeviceProp_t prop;
		if (hipGetDeviceProperties(&prop, e->device) == hipSuccess) {
			const size_t r = (size_t) prop.multiProcessorCount * (size_t) (prop.maxThreadsPerMultiProcessor / WAVE);
			if (r > 0 && r < resident)
				resident = r;
		}
		size_t need = per_wave * waves;
		if (mw_wave * mw_waves > need)
			need = mw_wave * mw_waves;
		if (e->d_hb && kl_dec2_private() * WAVE * 2 * waves > need)
			need = kl_dec2_private() * WAVE * 2 * waves;
		if (ww * WAVE * resident > need)
			need = ww * WAVE * resident;
		size_t cur = 0, mx = 0;
		if (hipDeviceGetLimit(&cur, hipExtLimitScratchCurrent) == hipSuccess &&
		    hipDeviceGetLimit(&mx, hipExtLimitScratchMax) == hipSuccess && need > cur) {
			if (need > mx)
				return fail_msg("melpe_engine_create: the codec kernels' scratch exceeds the "
						"device's scratch limit (fewer channels per engine)");
			if ((er = hipDeviceSetLimit(hipExtLimitScratchCurrent, need)) != hipSuccess)
				return fail("melpe_engine_create: raising the scratch limit", er);
		}
		e->scratch_need = need;
	}
	return engine_warm(e);
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
	DEVGUARD(device);
	melpe_engine *e = new melpe_engine();
	e->device = device;
	e->channels = channels;
	hipError_t er = hipSuccess;
	const char *what = nullptr;
#define CREATE_STEP(expr) if (er == hipSuccess && (er = (expr)) != hipSuccess) what = #expr
	e->stream = g_dev_stream[device];
	CREATE_STEP(hipEventCreate(&e->ev0));
	CREATE_STEP(hipEventCreate(&e->ev1));
	CREATE_STEP(hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming));
	CREATE_STEP(hipEventCreateWithFlags(&e->ev_out, hipEventDisableTiming));
	CREATE_STEP(hipEventCreateWithFlags(&e->ev_host, hipEventDisableTiming));
	CREATE_STEP(hipEventCreateWithFlags(&e->ev_pin, hipEventDisableTiming));
	CREATE_STEP(hipEventCreateWithFlags(&e->ev_npp, hipEventDisableTiming));
	CREATE_STEP(hipMalloc(&e->d_enc, sizeof(EncState) * (size_t) channels));
	CREATE_STEP(hipMalloc(&e->d_dec, sizeof(DecState) * (size_t) channels));
	CREATE_STEP(hipMalloc(&e->d_syn, sizeof(synth_state) * (size_t) channels));
	CREATE_STEP(hipMalloc(&e->d_pcm, sizeof(int16_t) * MELPE_SF_SAMPLES * (size_t) channels));
	CREATE_STEP(hipMalloc(&e->d_bits, (size_t) MELPE_SF_BYTES * channels));
	CREATE_STEP(hipMalloc(&e->d_mask, (size_t) channels));
	CREATE_STEP(bin_alloc(&e->bin_enc, channels));
	CREATE_STEP(bin_alloc(&e->bin_dec, channels));
#undef CREATE_STEP
	if (er != hipSuccess) {
		int r = fail(what, er);
		melpe_engine_destroy(e);	/* frees whatever was allocated */
		return r;
	}
	int r = melpe_engine_reset(e, nullptr, 3);
	if (r == 0)
		r = engine_reserve(e);
	if (r) {
		std::string m = g_err;
		melpe_engine_destroy(e);
		g_err = m;
		return r;
	}
	*out = e;
	return 0;
}

int melpe_engine_set_own_stream(melpe_engine *e, int on)
{
	if (!e)
		return fail_msg("melpe_engine_set_own_stream: null engine");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	ENGINE_WAIT(e);
	HIPCHK(hipStreamSynchronize(e->stream));
	if (on && !e->own) {
		HIPCHK(hipStreamCreateWithFlags(&e->own, hipStreamNonBlocking));
		e->stream = e->own;
		/* the new queue's scratch, had here and not mid-stream */
		if (int rc = engine_warm(e)) {
			e->stream = g_dev_stream[e->device];
			hipStreamDestroy(e->own);
			e->own = nullptr;
			return rc;
		}
	} else if (!on && e->own) {
		e->stream = g_dev_stream[e->device];
		HIPCHK(hipStreamDestroy(e->own));
		e->own = nullptr;
	}
	return 0;
}

int melpe_engine_set_lane_order(melpe_engine *e, int on)
{
	if (!e)
		return fail_msg("melpe_engine_set_lane_order: null engine");
	e->lane_order = on ? 1 : 0;
	return 0;
}

int melpe_engine_set_mw_live_max(melpe_engine *e, int live_max)
{
	if (!e || live_max < 0)
		return fail_msg("melpe_engine_set_mw_live_max: a live-channel count >= 0");
	std::lock_guard<std::recursive_mutex> lk(e->mu);
	e->mw_live_max = live_max;
	return 0;
}

int melpe_engine_last_ana_waves(melpe_engine *e)
{
	if (!e)
		return fail_msg("melpe_engine_last_ana_waves: no engine");
	DEVGUARD(e->device);
	ENGINE_WAIT(e);
	int v = 0;
	HIPCHK(hipMemcpy(&v, e->bin_enc.ctl + 2 * NBIN + 1, sizeof(int), hipMemcpyDeviceToHost));
	return v;
}

int melpe_engine_set_dec_waves(melpe_engine *e, int waves)
{
	if (!e || !(waves == 0 || waves == 1 || waves == 2))
		return fail_msg("melpe_engine_set_dec_waves: waves must be 0 (auto), 1 or 2");
	if (waves == 2 && !e->d_hb)
		return fail_msg("melpe_engine_set_dec_waves: the two-wave decoder is available up to "
				"65,536 channels per engine");
	std::lock_guard<std::recursive_mutex> lk(e->mu);
	e->dec_waves = waves;
	return 0;
}

int melpe_engine_set_ana_waves(melpe_engine *e, int waves)
{
	if (!e || !(waves == 0 || waves == 1 || waves == 4))
		return fail_msg("melpe_engine_set_ana_waves: waves must be 0 (auto), 1 or 4");
	e->ana_waves = waves;
	return 0;
}

int melpe_engine_destroy(melpe_engine *e)
{
	if (!e)
		return 0;
	DevGuard dg(e->device);
	/* this engine's enqueued calls, not the whole shared stream */
	engine_wait(e);
	hipFree(e->d_npp);
	hipFree(e->d_enc);
	hipFree(e->d_dec);
	hipFree(e->d_syn);
	hipFree(e->d_pcm);
	hipFree(e->d_bits);
	hipFree(e->d_mask);
	hipFree(e->bin_enc.perm);
	hipFree(e->bin_dec.perm);
	hipFree(e->d_lq);
	hipFree(e->d_hb);
	hipFree(e->d_res);
	for (auto &m : e->marks)
		hipEventDestroy(m.second);
	if (e->bin_enc.done)
		hipEventDestroy(e->bin_enc.done);
	if (e->bin_dec.done)
		hipEventDestroy(e->bin_dec.done);
	if (e->ev0)
		hipEventDestroy(e->ev0);
	if (e->ev1)
		hipEventDestroy(e->ev1);
	if (e->ev_in)
		hipEventDestroy(e->ev_in);
	if (e->ev_out)
		hipEventDestroy(e->ev_out);
	if (e->ev_host)
		hipEventDestroy(e->ev_host);
	if (e->ev_pin)
		hipEventDestroy(e->ev_pin);
	if (e->ev_npp)
		hipEventDestroy(e->ev_npp);
	for (auto &sl : e->slot) {
		hipFree(sl.pcm);
		hipFree(sl.bits);
		hipFree(sl.mask);
		for (hipEvent_t ev : {sl.loaded, sl.done, sl.freed})
			if (ev)
				hipEventDestroy(ev);
	}
	if (e->own)
		hipStreamDestroy(e->own);
	if (e->cin)
		hipStreamDestroy(e->cin);
	if (e->cout)
		hipStreamDestroy(e->cout);
	if (e->cdec)
		hipStreamDestroy(e->cdec);
	if (e->ev_dec)
		hipEventDestroy(e->ev_dec);
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

int melpe_engine_reset_dev(melpe_engine *e, const void *d_mask, int which, void *hip_stream)
{
	if (!e || which < 1 || which > 3)
		return fail_msg("melpe_engine_reset_dev: bad arguments");
	DEVGUARD(e->device);
	hipStream_t s = (hipStream_t) hip_stream;
	ENGINE_CALL(e, s);
	k_reset<<<grid_for(e->channels), WAVE, 0, s>>>(
		e->d_enc, e->d_dec, (const uint8_t *) d_mask, e->channels, which);
	HIPCHK(hipGetLastError());
	return _call.finish();
}

int melpe_engine_reset(melpe_engine *e, const uint8_t *mask_host, int which)
{
	if (!e || which < 1 || which > 3)
		return fail_msg("melpe_engine_reset: bad arguments");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	/* ordered after every *_dev call of this engine already enqueued, on
	 * any stream: those read and write the same channel records */
	ENGINE_WAIT(e);
	int rc;
	const uint8_t *m = stage_mask(e, mask_host, &rc);
	if (rc)
		return rc;
	k_reset<<<grid_for(e->channels), WAVE, 0, e->stream>>>(e->d_enc, e->d_dec, m,
								  e->channels, which);
	HIPCHK(hipGetLastError());
	HOST_FINISH(e);
	return 0;
}

static int npp_launch(melpe_engine *e, int16_t *d_sp, int frames, int stride,
		      const uint8_t *d_act, hipStream_t s, bool sync, int rate1200)
{
	if (frames <= 0 || stride < frames * MELPE_FRAME_SAMPLES)
		return fail_msg("melpe_npp: bad frames/stride");
	DEVGUARD(e->device);
	ENGINE_CALL(e, s);
	ev_begin(e, s);
	HIPCHK((hipError_t) kl_npp(e->d_enc, d_sp, frames, stride, d_act, e->channels, rate1200, s));
	ev_end(e, s, sync);
	return _call.finish();
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
	if (!e || !sp || stride <= 0)
		return fail_msg("melpe_npp_host: bad arguments");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	ENGINE_WAIT(e);
	size_t bytes = sizeof(int16_t) * (size_t) stride * e->channels;
	if (e->npp_bytes < bytes) {
		HIPCHK(hipFree(e->d_npp));
		e->d_npp = nullptr;
		e->npp_bytes = 0;
		HIPCHK(hipMalloc(&e->d_npp, bytes));
		e->npp_bytes = bytes;
	}
	int16_t *d = e->d_npp;
	int rc;
	const uint8_t *m = stage_mask(e, active, &rc);
	if (!rc) {
		hipError_t ec = hipMemcpyAsync(d, sp, bytes, hipMemcpyHostToDevice, e->stream);
		rc = ec == hipSuccess ? npp_launch(e, d, frames, stride, m, e->stream, true, 1)
				      : fail("npp copy in", ec);
		if (!rc) {
			hipError_t er = hipMemcpyAsync(sp, d, bytes, hipMemcpyDeviceToHost, e->stream);
			if (er == hipSuccess)
				er = hipEventRecord(e->ev_host, e->stream);
			if (er == hipSuccess)
				er = hipEventSynchronize(e->ev_host);
			if (er != hipSuccess)
				rc = fail("npp copy back", er);
		}
	}
	return rc;
}

static int encode_launch(melpe_engine *e, unsigned char *d_bits, int16_t *d_sp,
			 const uint8_t *d_act, hipStream_t s, bool sync)
{
	DEVGUARD(e->device);
	ENGINE_CALL(e, s);
	ev_begin(e, s);
	HIPCHK((hipError_t) kl_enc_npp(e->d_enc, d_sp, d_act, e->channels, s));
	HIPCHK((hipError_t) ana_launch(e, d_sp, d_bits, d_act, s));
	ev_end(e, s, sync);
	return _call.finish();
}

int melpe_encode_dev(melpe_engine *e, void *d_bits, void *d_sp, const void *d_active,
		     void *hip_stream)
{
	if (!e || !d_bits || !d_sp)
		return fail_msg("melpe_encode_dev: null argument");
	return encode_launch(e, (unsigned char *) d_bits, (int16_t *) d_sp,
			     (const uint8_t *) d_active, (hipStream_t) hip_stream, false);
}

int melpe_encode_npp_dev(melpe_engine *e, void *d_sp, const void *d_active, void *hip_stream)
{
	if (!e || !d_sp)
		return fail_msg("melpe_encode_npp_dev: null argument");
	DEVGUARD(e->device);
	hipStream_t s = (hipStream_t) hip_stream;
	ENGINE_CALL(e, s);
	HIPCHK((hipError_t) kl_enc_npp(e->d_enc, (int16_t *) d_sp, (const uint8_t *) d_active,
				       e->channels, s));
	return _call.finish();
}

int melpe_encode_ana_dev(melpe_engine *e, void *d_bits, const void *d_sp, const void *d_active,
			 void *hip_stream)
{
	if (!e || !d_bits || !d_sp)
		return fail_msg("melpe_encode_ana_dev: null argument");
	DEVGUARD(e->device);
	hipStream_t s = (hipStream_t) hip_stream;
	ENGINE_CALL(e, s);
	HIPCHK((hipError_t) ana_launch(e, (const int16_t *) d_sp, (uint8_t *) d_bits,
				       (const uint8_t *) d_active, s));
	return _call.finish();
}

static int side_streams(melpe_engine *e);

int melpe_encode_pipe_dev(melpe_engine *e, void *d_bits, const void *d_sp, const void *d_active,
			  void *d_sp_next, const void *d_active_next, void *hip_stream)
{
	if (!e || !d_bits || !d_sp)
		return fail_msg("melpe_encode_pipe_dev: null argument");
	if (d_sp_next == d_sp)
		return fail_msg("melpe_encode_pipe_dev: the next superframe's PCM must be another buffer");
	DEVGUARD(e->device);
	if (d_sp_next)
		if (int rc = side_streams(e))
			return rc;
	hipStream_t s = (hipStream_t) hip_stream;
	ENGINE_CALL(e, s);
	/* the analysis on the engine stream; the next superframe's NPP on the
	 * engine's cin stream once the analysis' lane-order sort is done (after the
	 * caller's work, too, which the engine stream waited for).  The NPP
	 * touches only the records' NppState and d_sp_next, the analysis only
	 * their EncAna and d_sp. */
	ev_begin(e, s);
	HIPCHK((hipError_t) ana_launch(e, (const int16_t *) d_sp, (uint8_t *) d_bits, (const uint8_t *) d_active,
				       s, d_sp_next ? e->ev_pin : nullptr));
	ev_end(e, s, false);
	if (d_sp_next) {
		const hipStream_t ns = e->cin;
		HIPCHK(hipStreamWaitEvent(ns, e->ev_pin, 0));
		HIPCHK((hipError_t) kl_enc_npp(e->d_enc, (int16_t *) d_sp_next, (const uint8_t *) d_active_next,
					       e->channels, ns));
		HIPCHK(hipEventRecord(e->ev_npp, ns));
	}
	/* the hop back to the caller covers the NPP too */
	if (d_sp_next)
		HIPCHK(hipStreamWaitEvent(s, e->ev_npp, 0));
	return _call.finish();
}

static int dec_queue(melpe_engine *e);

int melpe_duplex_pipe_dev(melpe_engine *e, void *d_bits, const void *d_sp, const void *d_active,
			  void *d_sp_next, const void *d_active_next, void *d_dec_sp,
			  const void *d_dec_bits, const void *d_dec_active, void *hip_stream)
{
	if (!e || !d_bits || !d_sp || (d_dec_bits && !d_dec_sp))
		return fail_msg("melpe_duplex_pipe_dev: null argument");
	if (d_sp_next == d_sp)
		return fail_msg("melpe_duplex_pipe_dev: the next superframe's PCM must be another buffer");
	if (d_dec_bits && (d_dec_bits == d_bits || d_dec_sp == d_sp || d_dec_sp == d_sp_next))
		return fail_msg("melpe_duplex_pipe_dev: the decode's buffers must differ from the encode's");
	DEVGUARD(e->device);
	if (d_sp_next || d_dec_bits)
		if (int rc = d_dec_bits ? dec_queue(e) : side_streams(e))
			return rc;
	hipStream_t s = (hipStream_t) hip_stream;
	ENGINE_CALL(e, s);
	/* three queues: the analysis of this superframe on the engine stream, and
	 * once its lane-order sort is done (so that the analysis' waves, the
	 * longest, are dispatched first) the next superframe's NPP on cin
	 * (melpe_encode_pipe_dev) and the decode on cdec.  The encoder and
	 * decoder halves of a record and their lane-order buffers (bin_enc,
	 * bin_dec) are disjoint. */
	ev_begin(e, s);
	HIPCHK((hipError_t) ana_launch(e, (const int16_t *) d_sp, (uint8_t *) d_bits, (const uint8_t *) d_active,
				       s, (d_sp_next || d_dec_bits) ? e->ev_pin : nullptr));
	ev_end(e, s, false);
	if (d_dec_bits) {
		HIPCHK(hipStreamWaitEvent(e->cdec, e->ev_pin, 0));
		HIPCHK((hipError_t) dec_launch(e, (int16_t *) d_dec_sp, (const uint8_t *) d_dec_bits,
					       (const uint8_t *) d_dec_active, e->cdec));
		HIPCHK(hipEventRecord(e->ev_dec, e->cdec));
	}
	if (d_sp_next) {
		HIPCHK(hipStreamWaitEvent(e->cin, e->ev_pin, 0));
		HIPCHK((hipError_t) kl_enc_npp(e->d_enc, (int16_t *) d_sp_next, (const uint8_t *) d_active_next,
					       e->channels, e->cin));
		HIPCHK(hipEventRecord(e->ev_npp, e->cin));
		HIPCHK(hipStreamWaitEvent(s, e->ev_npp, 0));
	}
	/* the hop back to the caller covers the decode too */
	if (d_dec_bits)
		HIPCHK(hipStreamWaitEvent(s, e->ev_dec, 0));
	return _call.finish();
}

int melpe_encode_host(melpe_engine *e, unsigned char *bits, int16_t *sp, const uint8_t *active)
{
	if (!e || !bits || !sp)
		return fail_msg("melpe_encode_host: null argument");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	ENGINE_WAIT(e);
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
	HOST_FINISH(e);
	return 0;
}

/* The engine's two side streams, made at the first call that needs them
 * (the host-fed pipeline's copies; the pipelined encode's NPP runs on cin).
 * The runtime spreads streams over the process's hardware queues in the
 * order they are made, so they are made in one place, cout then cin.  The
 * NPP kernel's scratch is reserved on cin's queue here (only that kernel
 * runs there besides copies). */
static int side_streams(melpe_engine *e)
{
	if (e->cin)
		return 0;
	HIPCHK(hipStreamCreateWithFlags(&e->cout, hipStreamNonBlocking));
	HIPCHK(hipStreamCreateWithFlags(&e->cin, hipStreamNonBlocking));
	HIPCHK((hipError_t) kl_npp_warm(e->channels, e->cin));
	HIPCHK(hipStreamSynchronize(e->cin));
	return 0;
}

/* melpe_duplex_pipe_dev's decoder stream, made after the two side streams
 * (so the three land on hardware queues in a fixed order), with the
 * decoder kernels' scratch reserved on its queue as engine_warm does on the
 * engine stream's */
static int dec_queue(melpe_engine *e)
{
	if (e->cdec)
		return 0;
	if (int rc = side_streams(e))
		return rc;
	if (!e->ev_dec)
		HIPCHK(hipEventCreateWithFlags(&e->ev_dec, hipEventDisableTiming));
	HIPCHK(hipStreamCreateWithFlags(&e->cdec, hipStreamNonBlocking));
	HIPCHK((hipError_t) kl_dec_warm(e->channels, e->cdec));
	if (e->d_hb)
		HIPCHK((hipError_t) kl_dec2_warm(e->channels, e->cdec));
	HIPCHK(hipStreamSynchronize(e->cdec));
	return 0;
}

/* the host-fed pipeline's buffers, made at its first call */
static int async_setup(melpe_engine *e)
{
	if (e->slot[0].pcm)
		return 0;
	const size_t pb = sizeof(int16_t) * BLOCK * (size_t) e->channels, bb = (size_t) 11 * e->channels;
	for (auto &sl : e->slot) {
		HIPCHK(hipMalloc(&sl.pcm, pb));
		HIPCHK(hipMalloc(&sl.bits, bb));
		HIPCHK(hipMalloc(&sl.mask, (size_t) e->channels));
		for (hipEvent_t *ev : {&sl.loaded, &sl.done, &sl.freed})
			HIPCHK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
	}
	return side_streams(e);
}

int melpe_encode_host_async(melpe_engine *e, unsigned char *bits, int16_t *sp, const uint8_t *active)
{
	if (!e || !bits || !sp)
		return fail_msg("melpe_encode_host_async: null argument");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	if (int rc = async_setup(e))
		return rc;
	const size_t pb = sizeof(int16_t) * BLOCK * (size_t) e->channels, bb = (size_t) 11 * e->channels;
	melpe_engine::Slot &sl = e->slot[e->async_calls & 1];
	/* the slot's previous superframe has left the device (its D2H) */
	if (sl.used)
		HIPCHK(hipStreamWaitEvent(e->cin, sl.freed, 0));
	/* (the copies touch only the slot; the kernels below are ordered after
	 * the engine's earlier calls by the engine stream itself) */
	if (active)
		HIPCHK(hipMemcpyAsync(sl.mask, active, (size_t) e->channels, hipMemcpyHostToDevice, e->cin));
	HIPCHK(hipMemcpyAsync(sl.pcm, sp, pb, hipMemcpyHostToDevice, e->cin));
	if (active)	/* inactive channels keep the caller's bits */
		HIPCHK(hipMemcpyAsync(sl.bits, bits, bb, hipMemcpyHostToDevice, e->cin));
	HIPCHK(hipEventRecord(sl.loaded, e->cin));
	/* the kernels on the engine stream, after the slot's H2D */
	HIPCHK(hipStreamWaitEvent(e->stream, sl.loaded, 0));
	HIPCHK((hipError_t) kl_enc_npp(e->d_enc, sl.pcm, active ? sl.mask : nullptr, e->channels, e->stream));
	HIPCHK((hipError_t) ana_launch(e, sl.pcm, sl.bits, active ? sl.mask : nullptr, e->stream));
	HIPCHK(hipEventRecord(sl.done, e->stream));
	/* the NPP output (melpe_a's in-place side effect) and the bits back */
	HIPCHK(hipStreamWaitEvent(e->cout, sl.done, 0));
	HIPCHK(hipMemcpyAsync(sp, sl.pcm, pb, hipMemcpyDeviceToHost, e->cout));
	HIPCHK(hipMemcpyAsync(bits, sl.bits, bb, hipMemcpyDeviceToHost, e->cout));
	HIPCHK(hipEventRecord(sl.freed, e->cout));
	sl.used = true;
	e->async_calls++;
	/* later calls of this engine (and engine_wait) are ordered after this
	 * one's last copy */
	return engine_mark(e, e->cout);
}

int melpe_encode_host_wait(melpe_engine *e)
{
	if (!e)
		return fail_msg("melpe_encode_host_wait: null argument");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	for (auto &sl : e->slot)
		if (sl.used)
			HIPCHK(hipEventSynchronize(sl.freed));
	return 0;
}

static int decode_launch(melpe_engine *e, int16_t *d_sp, const unsigned char *d_bits,
			 const uint8_t *d_act, hipStream_t s, bool sync)
{
	DEVGUARD(e->device);
	ENGINE_CALL(e, s);
	ev_begin(e, s);
	HIPCHK((hipError_t) dec_launch(e, d_sp, d_bits, d_act, s));
	ev_end(e, s, sync);
	return _call.finish();
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
	DEVGUARD(e->device);
	HOST_LOCK(e);
	ENGINE_WAIT(e);
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
	HOST_FINISH(e);
	return 0;
}

/* 2400 bps mode (codec2400.h): NPP of one 180-sample frame at RATE2400
 * (k_npp, melpe/npp.c:180-184 first-call branch), then analysis + 54-bit
 * packing (k_enc24); decode = channel read + synthesis of one frame */
static int encode24_launch(melpe_engine *e, unsigned char *d_bits, int16_t *d_sp,
			   const uint8_t *d_act, hipStream_t s, bool sync)
{
	DEVGUARD(e->device);
	ENGINE_CALL(e, s);
	ev_begin(e, s);
	HIPCHK((hipError_t) kl_npp(e->d_enc, d_sp, 1, MELPE_FRAME_SAMPLES, d_act, e->channels, 0, s));
	HIPCHK((hipError_t) kl_enc24(e->d_enc, d_sp, d_bits, d_act, e->channels, s));
	ev_end(e, s, sync);
	return _call.finish();
}

int melpe_encode2400_dev(melpe_engine *e, void *d_bits, void *d_sp, const void *d_active,
			 void *hip_stream)
{
	if (!e || !d_bits || !d_sp)
		return fail_msg("melpe_encode2400_dev: null argument");
	return encode24_launch(e, (unsigned char *) d_bits, (int16_t *) d_sp,
			       (const uint8_t *) d_active, (hipStream_t) hip_stream, false);
}

int melpe_decode2400_dev(melpe_engine *e, void *d_sp, const void *d_bits, const void *d_active,
			 void *hip_stream)
{
	if (!e || !d_sp || !d_bits)
		return fail_msg("melpe_decode2400_dev: null argument");
	DEVGUARD(e->device);
	hipStream_t s = (hipStream_t) hip_stream;
	ENGINE_CALL(e, s);
	ev_begin(e, s);
	HIPCHK((hipError_t) kl_dec24(e->d_dec, (int16_t *) d_sp, (const uint8_t *) d_bits,
				     (const uint8_t *) d_active, e->channels, s));
	ev_end(e, s, false);
	return _call.finish();
}

int melpe_encode2400_host(melpe_engine *e, unsigned char *bits, int16_t *sp, const uint8_t *active)
{
	if (!e || !bits || !sp)
		return fail_msg("melpe_encode2400_host: null argument");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	ENGINE_WAIT(e);
	size_t pb = sizeof(int16_t) * MELPE_FRAME_SAMPLES * (size_t) e->channels;
	size_t bb = (size_t) MELPE_R24_BYTES * e->channels;
	int rc;
	const uint8_t *m = stage_mask(e, active, &rc);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(e->d_pcm, sp, pb, hipMemcpyHostToDevice, e->stream));
	if (active)
		HIPCHK(hipMemcpyAsync(e->d_bits, bits, bb, hipMemcpyHostToDevice, e->stream));
	rc = encode24_launch(e, e->d_bits, e->d_pcm, m, e->stream, true);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(sp, e->d_pcm, pb, hipMemcpyDeviceToHost, e->stream));
	HIPCHK(hipMemcpyAsync(bits, e->d_bits, bb, hipMemcpyDeviceToHost, e->stream));
	HOST_FINISH(e);
	return 0;
}

int melpe_decode2400_host(melpe_engine *e, int16_t *sp, const unsigned char *bits,
			  const uint8_t *active)
{
	if (!e || !bits || !sp)
		return fail_msg("melpe_decode2400_host: null argument");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	ENGINE_WAIT(e);
	size_t pb = sizeof(int16_t) * MELPE_FRAME_SAMPLES * (size_t) e->channels;
	size_t bb = (size_t) MELPE_R24_BYTES * e->channels;
	int rc;
	const uint8_t *m = stage_mask(e, active, &rc);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(e->d_bits, bits, bb, hipMemcpyHostToDevice, e->stream));
	if (active)
		HIPCHK(hipMemcpyAsync(e->d_pcm, sp, pb, hipMemcpyHostToDevice, e->stream));
	HIPCHK((hipError_t) kl_dec24(e->d_dec, e->d_pcm, e->d_bits, m, e->channels, e->stream));
	HIPCHK(hipMemcpyAsync(sp, e->d_pcm, pb, hipMemcpyDeviceToHost, e->stream));
	HOST_FINISH(e);
	return 0;
}

/* per-channel state records (checkpoint / migration between engines) */
static int state_geom(melpe_engine *e, int which, int first, int count, size_t *rec,
		      char **base)
{
	if (!e || (which != 1 && which != 2) || first < 0 || count < 0 ||
	    first + (long) count > e->channels)
		return fail_msg("melpe_engine_state: bad arguments");
	*rec = which == 1 ? sizeof(EncState) : sizeof(DecState);
	*base = which == 1 ? (char *) e->d_enc : (char *) e->d_dec;
	return 0;
}

long melpe_engine_state_bytes(int which)
{
	return which == 1 ? (long) sizeof(EncState) : which == 2 ? (long) sizeof(DecState) : -1;
}

int melpe_engine_export(melpe_engine *e, int which, int first, int count, void *host_out)
{
	size_t rec;
	char *base;
	if (int r = state_geom(e, which, first, count, &rec, &base))
		return r;
	if (!host_out && count)
		return fail_msg("melpe_engine_export: null buffer");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	ENGINE_WAIT(e);
	HIPCHK(hipMemcpy(host_out, base + rec * first, rec * count, hipMemcpyDeviceToHost));
	return 0;
}

int melpe_engine_import(melpe_engine *e, int which, int first, int count, const void *host_in)
{
	size_t rec;
	char *base;
	if (int r = state_geom(e, which, first, count, &rec, &base))
		return r;
	if (!host_in && count)
		return fail_msg("melpe_engine_import: null buffer");
	const uint32_t want = which == 1 ? ENC_REC_FMT : DEC_REC_FMT;
	const size_t tag = which == 1 ? offsetof(EncState, fmt) : offsetof(DecState, fmt);
	for (int k = 0; k < count; k++) {
		uint32_t f;
		memcpy(&f, (const char *) host_in + rec * k + tag, sizeof f);
		if (f != want)
			return fail_msg("melpe_engine_import: record " + std::to_string(k) +
					" is not a state record of this library's layout");
	}
	DEVGUARD(e->device);
	HOST_LOCK(e);
	ENGINE_WAIT(e);
	HIPCHK(hipMemcpy(base + rec * first, host_in, rec * count, hipMemcpyHostToDevice));
	return 0;
}

int melpe_synth_seed(melpe_engine *e, uint32_t run_seed, uint32_t first_channel)
{
	if (!e)
		return fail_msg("null engine");
	DEVGUARD(e->device);
	HOST_LOCK(e);
	k_synth_seed<<<grid_for(e->channels), WAVE, 0, e->stream>>>(e->d_syn, run_seed,
								      first_channel, e->channels);
	HIPCHK(hipGetLastError());
	HOST_FINISH(e);
	return 0;
}

int melpe_synth_dev(melpe_engine *e, void *d_sp, int samples, void *hip_stream)
{
	if (!e || !d_sp || samples <= 0)
		return fail_msg("melpe_synth_dev: bad arguments");
	DEVGUARD(e->device);
	hipStream_t s = (hipStream_t) hip_stream;
	ENGINE_CALL(e, s);
	k_synth<<<grid_for(e->channels), WAVE, 0, s>>>(
		e->d_syn, (int16_t *) d_sp, samples, e->channels);
	HIPCHK(hipGetLastError());
	return _call.finish();
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
	if (!e || !d_sp)
		return fail_msg("melpe_debug_encode_stage: null argument");
	DEVGUARD(e->device);
	HIPCHK((hipError_t) kl_enc_npp(e->d_enc, (int16_t *) d_sp, nullptr, e->channels, e->stream));
	if (upto > 0)
		HIPCHK((hipError_t) kl_enc_ana_dbg(e->d_enc, (int16_t *) d_sp, e->channels, upto,
						   e->stream));
	HIPCHK(hipStreamSynchronize(e->stream));
	return 0;
}

#define MELPE_PROF_SLOTS_ABI 256	/* ops.h MELPE_PROF_SLOTS of the profiling build */

int melpe_prof_read(uint64_t *out, int n)
{
	uint64_t acc[MELPE_PROF_SLOTS_ABI] = {0};
	int (*rd[])(uint64_t *) = {melpe_tu_eng_prof, melpe_tu_npp_prof, melpe_tu_ana_prof, melpe_tu_anamw_prof,
				   melpe_tu_harm_prof,
				   melpe_tu_dec_prof, melpe_tu_r24_prof};
	for (auto f : rd)
		if (f(acc))
			return fail_msg("not a profiling build (-DMELPE_PROF)");
	for (int i = 0; i < n && i < MELPE_PROF_SLOTS_ABI; i++)
		out[i] = acc[i];
	return MELPE_PROF_SLOTS_ABI;
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
static bool g_single_rate2400 = false;	/* melpe_i2 sets rate = RATE2400 */
static bool g_single_npp_started = false;	/* npp's static first_time has fired */

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
	DevGuard dg(e->device);
	/* npp reads 256 samples only on its very first call (from melpe_n or
	 * melpe_a) and only when rate == RATE1200 (melpe/npp.c:176-179);
	 * every other call reads the caller's 180 */
	size_t n = (!g_single_npp_started && g_single_rate1200) ? 256 : 180;
	int16_t *d = e->d_pcm;
	if (dg.err != hipSuccess ||
	    hipMemcpy(d, sp, sizeof(int16_t) * n, hipMemcpyHostToDevice) != hipSuccess ||
	    npp_launch(e, d, 1, 256, nullptr, e->stream, true, g_single_rate1200 ? 1 : 0) ||
	    hipMemcpy(sp, d, sizeof(int16_t) * 180, hipMemcpyDeviceToHost) != hipSuccess) {
		fprintf(stderr, "libmelpe_amd: melpe_n failed: %s\n", g_err.c_str());
		abort();
	}
	g_single_npp_started = true;
}

int melpe_single_reset(void)
{
	melpe_engine *e = single_engine();
	g_single_rate1200 = false;
	g_single_rate2400 = false;
	g_single_npp_started = false;
	return melpe_engine_reset(e, nullptr, 3);
}

void melpe_i(void)
{
	melpe_engine *e = single_engine();
	DevGuard dg(e->device);
	k_melpe_i<<<1, WAVE, 0, e->stream>>>(e->d_enc, e->d_dec);
	if (hipGetLastError() != hipSuccess || hipStreamSynchronize(e->stream) != hipSuccess) {
		fprintf(stderr, "libmelpe_amd: melpe_i failed\n");
		abort();
	}
	g_single_rate1200 = true;
	g_single_rate2400 = false;
}

/* melpe_i2 / melpe_al: the 2400 bps entry points the reference declares
 * (melpe/melpe.c:57-58) but never defines.  melpe_i2 = melpe_i at RATE2400
 * (melp_ana_init + melp_syn_init, one-frame blocks); melpe_al = melpe_a's
 * body for one 180-sample frame: npp in place, analysis, 7 bytes out.
 * After melpe_i2, melpe_s decodes one 7-byte frame into 180 samples (the
 * reference's synthesis() at RATE2400). */
void melpe_i2(void)
{
	melpe_engine *e = single_engine();
	DevGuard dg(e->device);
	k_melpe_i<<<1, WAVE, 0, e->stream>>>(e->d_enc, e->d_dec);
	if (hipGetLastError() != hipSuccess || hipStreamSynchronize(e->stream) != hipSuccess) {
		fprintf(stderr, "libmelpe_amd: melpe_i2 failed\n");
		abort();
	}
	g_single_rate1200 = false;
	g_single_rate2400 = true;
}

void melpe_al(unsigned char *buf, short *sp)
{
	melpe_engine *e = single_engine();
	if (!g_single_rate2400) {
		fprintf(stderr, "libmelpe_amd: melpe_al needs melpe_i2 first\n");
		abort();
	}
	if (melpe_encode2400_host(e, buf, sp, nullptr)) {
		fprintf(stderr, "libmelpe_amd: melpe_al failed: %s\n", g_err.c_str());
		abort();
	}
	g_single_npp_started = true;
}

void melpe_a(unsigned char *buf, short *sp)
{
	melpe_engine *e = single_engine();
	if (melpe_encode_host(e, buf, sp, nullptr)) {
		fprintf(stderr, "libmelpe_amd: melpe_a failed: %s\n", g_err.c_str());
		abort();
	}
	g_single_npp_started = true;
}

void melpe_s(short *sp, unsigned char *buf)
{
	melpe_engine *e = single_engine();
	DevGuard dg(e->device);
	if (g_single_rate2400) {	/* synthesis() at RATE2400: 7 bytes -> 180 samples */
		k_share_params<<<1, WAVE, 0, e->stream>>>(e->d_enc, e->d_dec, 0);
		int rc = hipGetLastError() != hipSuccess || melpe_decode2400_host(e, sp, buf, nullptr);
		if (!rc) {
			k_share_params<<<1, WAVE, 0, e->stream>>>(e->d_enc, e->d_dec, 1);
			rc = hipGetLastError() != hipSuccess ||
			     hipStreamSynchronize(e->stream) != hipSuccess;
		}
		if (rc) {
			fprintf(stderr, "libmelpe_amd: melpe_s (2400) failed: %s\n", g_err.c_str());
			abort();
		}
		return;
	}
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


int melpe_modem_state_bytes(void)
{
	return (int) sizeof(ModemState);
}

static int modem_state_ok(const void *d_state, int channels)
{
	if (!d_state || channels <= 0)
		return fail_msg("modem: bad arguments");
	if ((uintptr_t) d_state & 3)
		return fail_msg("modem: state must be 4-byte aligned");
	return 0;
}

int melpe_modem_reset_dev(void *d_state, int channels, const void *d_mask, void *hip_stream)
{
	if (int r = modem_state_ok(d_state, channels))
		return r;
	k_modem_reset<<<grid_for(channels), WAVE, 0, (hipStream_t) hip_stream>>>(
		(ModemState *) d_state, (const uint8_t *) d_mask, channels);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_modulate_dev(void *d_state, const void *d_pkts, void *d_pcm, int channels, int packets,
		       const void *d_active, void *hip_stream)
{
	if (int r = modem_state_ok(d_state, channels))
		return r;
	if (!d_pkts || !d_pcm || packets <= 0 || ((uintptr_t) d_pcm & 3))
		return fail_msg("melpe_modulate_dev: bad arguments (pcm must be 4-byte aligned)");
	long waves = (long) channels * packets;
	if ((waves + 3) / 4 > 0x7fffffffL)
		return fail_msg("melpe_modulate_dev: too many packets");
	hipStream_t s = (hipStream_t) hip_stream;
	k_modulate<<<(unsigned) ((waves + 3) / 4), 256, 0, s>>>(
		(ModemState *) d_state, (const uint8_t *) d_pkts, (int16_t *) d_pcm, channels, packets,
		(const uint8_t *) d_active);
	HIPCHK(hipGetLastError());
	k_modulate_state<<<grid_for(channels), WAVE, 0, s>>>(
		(ModemState *) d_state, (const uint8_t *) d_pkts, channels, packets,
		(const uint8_t *) d_active);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_demodulate_dev(void *d_state, const void *d_pcm, long stride, void *d_pos, void *d_data,
			 void *d_out, void *d_ret, int channels, int calls, const void *d_active,
			 void *hip_stream)
{
	if (int r = modem_state_ok(d_state, channels))
		return r;
	if (!d_pcm || !d_pos || !d_data || calls <= 0 || stride < MODEM_LOOKAHEAD ||
	    ((uintptr_t) d_pos & 3) || ((uintptr_t) d_ret & 3))
		return fail_msg("melpe_demodulate_dev: bad arguments");
	k_demodulate<<<grid_for(channels), WAVE, 0, (hipStream_t) hip_stream>>>(
		(ModemState *) d_state, (const int16_t *) d_pcm, stride, (int32_t *) d_pos,
		(uint8_t *) d_data, (uint8_t *) d_out, (int32_t *) d_ret, channels, calls,
		(const uint8_t *) d_active);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_ops_eval_dev(int op, const void *d_a, const void *d_b, const void *d_c, void *d_out,
		       long n, void *hip_stream)
{
	if (op < 0 || op >= MELPE_OPS_EVAL_COUNT || !d_a || !d_out || n <= 0 ||
	    (n + 255) / 256 > 0x7fffffffL)
		return fail_msg("melpe_ops_eval_dev: bad arguments");
	k_ops_eval<<<(unsigned) ((n + 255) / 256), 256, 0, (hipStream_t) hip_stream>>>(
		op, (const int64_t *) d_a, (const int32_t *) d_b, (const int32_t *) d_c,
		(int64_t *) d_out, n);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_divide_s_sweep_dev(void *d_digest, void *hip_stream)
{
	if (!d_digest)
		return fail_msg("melpe_divide_s_sweep_dev: null argument");
	k_divide_s_sweep<<<(32767 + 255) / 256, 256, 0, (hipStream_t) hip_stream>>>((uint64_t *) d_digest);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_helpers_eval_dev(int mode, const void *d_src, const void *d_args, void *d_out, int n,
			   void *hip_stream)
{
	if (!d_src || !d_args || !d_out || n < 0 || mode < 0 || mode > 8)
		return fail_msg("melpe_helpers_eval_dev: bad arguments");
	if (n == 0)
		return 0;
	k_helpers_eval<<<grid_for(n), WAVE, 0, (hipStream_t) hip_stream>>>(
		mode, (const int16_t *) d_src, (const int32_t *) d_args, (int32_t *) d_out, n);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_voice_crypt_dev(void *d_pkts, const void *d_counters, const void *d_keys,
			  const void *d_invert, int channels, int packets, int dir,
			  void *hip_stream)
{
	if (!d_pkts || !d_counters || !d_keys || channels <= 0 || packets <= 0 ||
	    (dir != 0 && dir != 1))
		return fail_msg("melpe_voice_crypt_dev: bad arguments");
	if (((uintptr_t) d_keys & 15) || ((uintptr_t) d_counters & 3))
		return fail_msg("melpe_voice_crypt_dev: keys must be 16-byte and counters "
				"4-byte aligned");
	long n = (long) channels * packets;
	long blocks = (n + 255) / 256;
	if (blocks > 0x7fffffffL)
		return fail_msg("melpe_voice_crypt_dev: too many packets");
	k_voice_crypt<<<(unsigned) blocks, 256, 0, (hipStream_t) hip_stream>>>(
		(unsigned char *) d_pkts, (const uint32_t *) d_counters, (const uint4 *) d_keys,
		(const uint8_t *) d_invert, channels, packets, dir);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_voice_crypt_host(unsigned char *pkts, const uint32_t *counters,
			   const unsigned char *keys, const uint8_t *invert, int channels,
			   int packets, int dir)
{
	if (!pkts || !counters || !keys || channels <= 0 || packets <= 0)
		return fail_msg("melpe_voice_crypt_host: bad arguments");
	size_t pb = (size_t) channels * packets * VC_PKT_BYTES;
	size_t kb = (size_t) channels * VC_KEY_BYTES, cb = (size_t) channels * 4;
	int dev = 0;
	HIPCHK(hipGetDevice(&dev));
	std::lock_guard<std::mutex> lk(g_stage[dev & 63].mu);
	unsigned char *d = nullptr;
	if (int r = stage_get(dev, kb + cb + channels + pb, (void **) &d))
		return r;
	unsigned char *dk = d, *dc = d + kb, *di = dc + cb, *dp = di + channels;
	int rc = 0;
	hipError_t he;
	if ((he = hipMemcpy(dk, keys, kb, hipMemcpyHostToDevice)) != hipSuccess ||
	    (he = hipMemcpy(dc, counters, cb, hipMemcpyHostToDevice)) != hipSuccess ||
	    (invert && (he = hipMemcpy(di, invert, channels, hipMemcpyHostToDevice)) != hipSuccess) ||
	    (he = hipMemcpy(dp, pkts, pb, hipMemcpyHostToDevice)) != hipSuccess)
		rc = fail("melpe_voice_crypt_host: upload", he);
	if (!rc)
		rc = melpe_voice_crypt_dev(dp, dc, dk, invert ? di : nullptr, channels, packets,
					   dir, nullptr);
	if (!rc && (he = hipMemcpy(pkts, dp, pb, hipMemcpyDeviceToHost)) != hipSuccess)
		rc = fail("melpe_voice_crypt_host: download", he);
	return rc;
}


int melpe_vad_state_bytes(void)
{
	return (int) sizeof(VadState);
}

int melpe_vad_reset_dev(void *d_state, int channels, const void *d_mask, void *hip_stream)
{
	if (!d_state || channels <= 0)
		return fail_msg("melpe_vad_reset_dev: bad arguments");
	if ((uintptr_t) d_state & 3)
		return fail_msg("melpe_vad_reset_dev: state must be 4-byte aligned");
	k_vad_reset<<<grid_for(channels), WAVE, 0, (hipStream_t) hip_stream>>>(
		(VadState *) d_state, (const uint8_t *) d_mask, channels);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_vad_dev(void *d_state, const void *d_sp, void *d_votes, int channels,
		  const void *d_active, void *hip_stream)
{
	if (!d_state || !d_sp || !d_votes || channels <= 0)
		return fail_msg("melpe_vad_dev: bad arguments");
	if ((uintptr_t) d_state & 3)
		return fail_msg("melpe_vad_dev: state must be 4-byte aligned");
	k_vad<<<grid_for(channels), WAVE, 0, (hipStream_t) hip_stream>>>(
		(VadState *) d_state, (const int16_t *) d_sp, (uint8_t *) d_votes, nullptr,
		(const uint8_t *) d_active, channels);
	HIPCHK(hipGetLastError());
	return 0;
}

int melpe_vad_host(unsigned char *state, const int16_t *sp, uint8_t *votes, int channels,
		   const uint8_t *active)
{
	if (!state || !sp || !votes || channels <= 0)
		return fail_msg("melpe_vad_host: bad arguments");
	size_t sb = sizeof(VadState) * (size_t) channels;
	size_t pb = sizeof(int16_t) * MELPE_SF_SAMPLES * (size_t) channels;
	int dev = 0;
	HIPCHK(hipGetDevice(&dev));
	std::lock_guard<std::mutex> lk(g_stage[dev & 63].mu);
	unsigned char *d = nullptr;
	if (int r = stage_get(dev, sb + pb + 2 * (size_t) channels, (void **) &d))
		return r;
	unsigned char *ds = d, *dp = d + sb, *dv = dp + pb, *da = dv + channels;
	int rc = 0;
	hipError_t he;
	if ((he = hipMemcpy(ds, state, sb, hipMemcpyHostToDevice)) != hipSuccess ||
	    (he = hipMemcpy(dp, sp, pb, hipMemcpyHostToDevice)) != hipSuccess ||
	    (he = hipMemcpy(dv, votes, channels, hipMemcpyHostToDevice)) != hipSuccess ||
	    (active && (he = hipMemcpy(da, active, channels, hipMemcpyHostToDevice)) != hipSuccess))
		rc = fail("melpe_vad_host: upload", he);
	if (!rc)
		rc = melpe_vad_dev(ds, dp, dv, channels, active ? da : nullptr, nullptr);
	if (!rc && ((he = hipMemcpy(state, ds, sb, hipMemcpyDeviceToHost)) != hipSuccess ||
		    (he = hipMemcpy(votes, dv, channels, hipMemcpyDeviceToHost)) != hipSuccess))
		rc = fail("melpe_vad_host: download", he);
	return rc;
}


int melpe_tx_dev(melpe_engine *e, void *d_vad_state, void *d_bits, void *d_sp, void *d_votes,
		 void *d_gate, const void *d_active, void *hip_stream)
{
	if (!e || !d_vad_state || !d_bits || !d_sp || !d_votes || !d_gate)
		return fail_msg("melpe_tx_dev: bad arguments");
	if ((uintptr_t) d_vad_state & 3)
		return fail_msg("melpe_tx_dev: state must be 4-byte aligned");
	DEVGUARD(e->device);
	k_vad<<<grid_for(e->channels), WAVE, 0, (hipStream_t) hip_stream>>>(
		(VadState *) d_vad_state, (const int16_t *) d_sp, (uint8_t *) d_votes,
		(uint8_t *) d_gate, (const uint8_t *) d_active, e->channels);
	HIPCHK(hipGetLastError());
	return melpe_encode_dev(e, d_bits, d_sp, d_gate, hip_stream);
}

/* the first half of melpe_tx_dev: the VAD gate and the NPP of the channels
 * it opens (the analysis follows in melpe_tx_pipe_dev or
 * melpe_encode_ana_dev with the gate as the mask) */
int melpe_tx_npp_dev(melpe_engine *e, void *d_vad_state, void *d_sp, void *d_votes, void *d_gate,
		     const void *d_active, void *hip_stream)
{
	if (!e || !d_vad_state || !d_sp || !d_votes || !d_gate)
		return fail_msg("melpe_tx_npp_dev: bad arguments");
	if ((uintptr_t) d_vad_state & 3)
		return fail_msg("melpe_tx_npp_dev: state must be 4-byte aligned");
	DEVGUARD(e->device);
	k_vad<<<grid_for(e->channels), WAVE, 0, (hipStream_t) hip_stream>>>(
		(VadState *) d_vad_state, (const int16_t *) d_sp, (uint8_t *) d_votes,
		(uint8_t *) d_gate, (const uint8_t *) d_active, e->channels);
	HIPCHK(hipGetLastError());
	return melpe_encode_npp_dev(e, d_sp, d_gate, hip_stream);
}

/* the TX front end pipelined like melpe_encode_pipe_dev: superframe k's
 * analysis on the engine stream (gated by d_gate, which melpe_tx_npp_dev or
 * the previous call wrote), and once its lane-order sort is done, on cin,
 * superframe k + 1's VAD (votes and gate out) and the NPP of the channels
 * it opens.  The VAD state is the VAD's alone, so a sequence tx_npp(0),
 * tx_pipe(0, 1), ..., tx_pipe(K-1, NULL) gives the bits, votes, gates and
 * NPP output of K melpe_tx_dev calls. */
int melpe_tx_pipe_dev(melpe_engine *e, void *d_vad_state, void *d_bits, const void *d_sp, const void *d_gate,
		      void *d_sp_next, void *d_votes_next, void *d_gate_next, const void *d_active_next,
		      void *hip_stream)
{
	if (!e || !d_vad_state || !d_bits || !d_sp || !d_gate ||
	    (d_sp_next && (!d_votes_next || !d_gate_next)))
		return fail_msg("melpe_tx_pipe_dev: bad arguments");
	if ((uintptr_t) d_vad_state & 3)
		return fail_msg("melpe_tx_pipe_dev: state must be 4-byte aligned");
	if (d_sp_next == d_sp || (d_sp_next && d_gate_next == d_gate))
		return fail_msg("melpe_tx_pipe_dev: the next superframe's buffers must be other buffers");
	DEVGUARD(e->device);
	if (d_sp_next)
		if (int rc = side_streams(e))
			return rc;
	hipStream_t s = (hipStream_t) hip_stream;
	ENGINE_CALL(e, s);
	ev_begin(e, s);
	HIPCHK((hipError_t) ana_launch(e, (const int16_t *) d_sp, (uint8_t *) d_bits, (const uint8_t *) d_gate, s,
				       d_sp_next ? e->ev_pin : nullptr));
	ev_end(e, s, false);
	if (d_sp_next) {
		const hipStream_t ns = e->cin;
		HIPCHK(hipStreamWaitEvent(ns, e->ev_pin, 0));
		k_vad<<<grid_for(e->channels), WAVE, 0, ns>>>((VadState *) d_vad_state, (const int16_t *) d_sp_next,
							      (uint8_t *) d_votes_next, (uint8_t *) d_gate_next,
							      (const uint8_t *) d_active_next, e->channels);
		HIPCHK(hipGetLastError());
		HIPCHK((hipError_t) kl_enc_npp(e->d_enc, (int16_t *) d_sp_next, (const uint8_t *) d_gate_next,
					       e->channels, ns));
		HIPCHK(hipEventRecord(e->ev_npp, ns));
		HIPCHK(hipStreamWaitEvent(s, e->ev_npp, 0));
	}
	return _call.finish();
}


int melpe_stream_pack(const unsigned char *bits, const uint8_t *votes, uint8_t *last,
		      unsigned char *out, uint8_t *lens, int channels, const uint8_t *active)
{
	if (!bits || !votes || !last || !out || !lens || channels <= 0)
		return fail_msg("melpe_stream_pack: bad arguments");
	for (int c = 0; c < channels; c++) {
		const unsigned char *b = bits + (size_t) c * MELPE_SF_BYTES;
		unsigned char *o = out + (size_t) c * MELPE_SF_BYTES;
		if (active && !active[c]) {
			lens[c] = 0;
			continue;
		}
		if (votes[c] == 0) {	/* melpe_enc.c:57-59: VAD flag on the carried txbuf[0] */
			last[c] |= 2;
			o[0] = last[c];
			lens[c] = 1;
		} else {		/* melpe_enc.c:64-70: bytes 0 and 10 swapped */
			memcpy(o, b, MELPE_SF_BYTES);
			o[0] = b[10];
			o[10] = b[0];
			last[c] = o[0];
			lens[c] = MELPE_SF_BYTES;
		}
	}
	return 0;
}

long melpe_stream_unpack(const unsigned char *stream, long nbytes, unsigned char *bits,
			 uint8_t *voiced, long max_sf)
{
	if (!stream || nbytes < 0 || !bits || !voiced || max_sf < 0)
		return fail_msg("melpe_stream_unpack: bad arguments");
	long pos = 0, k = 0;
	while (pos < nbytes && k < max_sf) {	/* melpe_dec.c:33-48 */
		unsigned char *b = bits + (size_t) k * MELPE_SF_BYTES;
		if (stream[pos] & 2) {
			memset(b, 0, MELPE_SF_BYTES);
			voiced[k++] = 0;
			pos += 1;
			continue;
		}
		if (pos + MELPE_SF_BYTES > nbytes)
			return fail_msg("melpe_stream_unpack: truncated voiced frame");
		memcpy(b, stream + pos, MELPE_SF_BYTES);
		b[0] = stream[pos + 10];
		b[10] = stream[pos];
		voiced[k++] = 1;
		pos += MELPE_SF_BYTES;
	}
	return k;
}

}  // extern "C"
