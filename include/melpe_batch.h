/*
 * melpe_batch.h -- batched C ABI of the MI355X MELPe-1200 engine.
 *
 * One engine = C independent channels resident on one GPU.  Each channel has
 * its own encoder and decoder state, equal to a fresh reference process after
 * melpe_engine_reset (the reference has exactly one instance per process:
 * all its state lives in globals and function statics, melpe/global.c:20-53).
 * Every call processes one superframe (540 samples <-> 11 bytes) of every
 * active channel, exactly as melpe_a / melpe_s (melpe/melpe.c:91-107) would
 * in that channel's own process.
 *
 * Process semantics: a channel's encoder and decoder do NOT share
 * melp_par / quant_par / chbuf (the reference process shares them,
 * melpe/global.c:28-37).  A batched channel therefore behaves as the
 * standalone melpe_enc (encode-only process) and melpe_dec (decode-only
 * process) do.  PairPhone's duplex pp, which runs melpe_a and melpe_s in one
 * process, is reproduced by the single-stream drop-in (melpe.h), not by an
 * engine channel that interleaves encode and decode.
 *
 * Buffers: PCM is channel-major, C x 540 int16 (sample s of channel c at
 * [c*540 + s]); bitstreams are C x 11 bytes.  The *_host calls take host
 * pointers and copy; the *_dev calls take device pointers (e.g. from torch)
 * and enqueue on the given HIP stream without synchronising.  `active` is an
 * optional C-byte mask (NULL = all channels): inactive channels are left
 * untouched (state, PCM and bits), which gives ragged streams.
 *
 * All functions return 0 on success and a negative code on error;
 * melpe_last_error() describes the last error of the calling thread.
 *
 * Ordering: a *_dev call is ordered after the work already enqueued on its
 * stream, and later work on that stream after it.  Its kernels run on the
 * device's engine stream (two event hops), so the *_dev calls of all engines
 * on a device execute in the order they were made, whatever streams they
 * name (the pipelined calls, melpe_encode_pipe_dev, melpe_duplex_pipe_dev
 * and melpe_tx_pipe_dev, also run parts on the engine's own side streams,
 * still inside that order).  The
 * *_host calls, melpe_engine_reset and the state export/import first wait
 * for every *_dev call of the same engine already enqueued, on any stream
 * (the engine records an event on each stream it is given), and for nothing
 * else on the device.  To reset channels in stream order (no host sync), use
 * melpe_engine_reset_dev on the stream that carries the encode/decode work.
 * The engines of one process share that internal stream per device for all
 * their kernels (create's scratch reservation, the *_host and the *_dev
 * calls), so the runtime holds the codec kernels' scratch on one hardware
 * queue rather than on every queue a caller's stream maps to.
 * One engine may be called from several host threads: its calls take a
 * per-engine lock while they enqueue (the host side of a call is short; the
 * device work is not serialised by it).  A call that fails after enqueueing
 * part of its work still records its stream's event, so later host-side
 * waits cover that work too.
 * Entry points restore the calling thread's current HIP device on return.
 */
#ifndef MELPE_AMD_BATCH_H
#define MELPE_AMD_BATCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct melpe_engine melpe_engine;

#define MELPE_SF_SAMPLES 540
#define MELPE_SF_BYTES 11
#define MELPE_FRAME_SAMPLES 180
#define MELPE_R24_BYTES 7

/* create an engine of `channels` channels on HIP device `device` */
int melpe_engine_create(melpe_engine **out, int device, int channels);
int melpe_engine_destroy(melpe_engine *e);
int melpe_engine_channels(const melpe_engine *e);

/* fresh-process state for the channels selected by `mask` (NULL = all);
 * which: 1 = encoder (incl. NPP), 2 = decoder, 3 = both */
int melpe_engine_reset(melpe_engine *e, const uint8_t *mask_host, int which);
/* the same, enqueued on `hip_stream` (d_mask: device C-byte mask or NULL) */
int melpe_engine_reset_dev(melpe_engine *e, const void *d_mask, int which, void *hip_stream);

/* Lane order of the lane-per-channel kernels (analysis, synthesis): on (1,
 * the default unless MELPE_BIN=0 is set in the environment), the live
 * channels are sorted by pitch class before each launch so that channels
 * with similar pitch and voicing share a wave; off (0), lane g runs channel g.
 * Either way every channel's bits and PCM are the same; only the speed
 * differs. */
int melpe_engine_set_lane_order(melpe_engine *e, int on);

/* Waves per 64 channels of the analysis kernel: 1 = one lane per channel;
 * 4 = each channel's independent analysis chains (bandpass-voicing bands,
 * LPC/LSF, global pitch, pitch tracking, classification, the LSF and pitch
 * codebook searches) spread over four waves of one workgroup, for channel
 * counts that would leave SIMDs idle; 0 (default) = chosen from the channel
 * count (4 up to 32,768 channels per engine, where every workgroup is
 * resident at once; 1 above).  Bits are the same either way. */
int melpe_engine_set_ana_waves(melpe_engine *e, int waves);

/* Waves per 64 channels of the decoder: 1 = one lane per channel; 2 = the
 * two-wave decoder, wave A reading the channel and synthesising each
 * frame's excitation, wave B running the synthesis filters, dispersion and
 * postfilter one frame behind (for channel counts that would leave SIMDs
 * idle: available up to 65,536 channels per engine); 0 (default) = chosen
 * from the channel count (2 up to 65,536 channels, 1 above).  PCM is the
 * same either way. */
int melpe_engine_set_dec_waves(melpe_engine *e, int waves);

/* The live-count mapping of the automatic choice above 32,768 channels: a
 * superframe with at most live_max live channels (ragged streams, paused
 * channels) runs the four-wave analysis, more run one lane per channel.
 * The choice is made on the device, per launch: both mappings are enqueued,
 * each gated on the live count the lane-order sort counted there (so it
 * needs the lane order on, the default), and the host never reads the
 * count.  live_max >= 0 (default 32,768, where the four-wave kernel holds
 * every live channel resident; 0 = by channel count only).  Bits are the
 * same either way.  Values above 32,768 are for diagnostics only: the
 * four-wave kernel then loops over the extra live channels and is slower
 * than the lane kernel from about 40,960 live (profiles/r05_mw_crossover.jsonl). */
int melpe_engine_set_mw_live_max(melpe_engine *e, int live_max);

/* By default every engine on a device runs its kernels on one internal
 * stream per device (one hardware queue): the runtime holds kernel scratch
 * per queue, sized for the largest private segment it has run at the
 * device's full wave count, and engines each on a queue of their own could
 * exhaust the scratch pool (a later launch then aborts its queue with
 * HSA_STATUS_ERROR_OUT_OF_RESOURCES) or make the runtime reclaim one
 * queue's scratch for another's, hundreds of ms per launch.  With on = 1
 * this engine gets a stream of its own (its kernels can then overlap other
 * engines', e.g. an encoder and a decoder of a duplex link); its scratch is
 * reserved on it here, and the call fails cleanly if it cannot be had.
 * on = 0 returns to the shared stream.  Waits for the engine's calls. */
int melpe_engine_set_own_stream(melpe_engine *e, int on);

/* The mapping the engine's last analysis launch ran, as the device recorded
 * it: 1 = one lane per channel, 4 = four waves per 64 channels, 0 = none
 * (no live channel in the launch since the last lane-order sort).  Waits for
 * the engine's enqueued calls. */
int melpe_engine_last_ana_waves(melpe_engine *e);

/* Per-channel state records, for checkpoint / resume and for moving channels
 * between engines or GPUs (e.g. re-balancing ragged streams).  which: 1 =
 * encoder (EncState), 2 = decoder (DecState).  melpe_engine_state_bytes gives
 * the record size; export copies records [first, first+count) to host memory
 * (count * bytes), import writes them back into any engine of the same
 * library build.  A record is opaque and carries a channel's complete codec
 * state: continuing an imported channel gives the bits / PCM the exporting
 * engine would have produced.  Each record carries a format tag (layout
 * version and size); import rejects a batch holding any record of another
 * layout (e.g. a checkpoint of an older build) and writes nothing. */
long melpe_engine_state_bytes(int which);
int melpe_engine_export(melpe_engine *e, int which, int first, int count, void *host_out);
int melpe_engine_import(melpe_engine *e, int which, int first, int count, const void *host_in);

/* melpe_a on every active channel: sp (C x 540, in/out: overwritten with the
 * NPP output), bits (C x 11, out) */
int melpe_encode_host(melpe_engine *e, unsigned char *bits, int16_t *sp,
		      const uint8_t *active);
int melpe_encode_dev(melpe_engine *e, void *d_bits, void *d_sp,
		     const void *d_active, void *hip_stream);

/* The two halves of melpe_encode_dev, enqueued separately (e.g. to time
 * each kernel): the noise pre-processor on the superframe's three frames,
 * in place (melpe/melpe.c:94-96), then analysis + packing
 * (melpe/melpe.c:97-98).  encode_npp followed by encode_ana on the same
 * buffers and stream is exactly melpe_encode_dev. */
int melpe_encode_npp_dev(melpe_engine *e, void *d_sp, const void *d_active, void *hip_stream);
int melpe_encode_ana_dev(melpe_engine *e, void *d_bits, const void *d_sp, const void *d_active,
			 void *hip_stream);

/* Pipelined encode of a sequence of superframes: the analysis + packing of
 * superframe k (d_sp: its PCM, already through the NPP, as
 * melpe_encode_npp_dev leaves it; d_bits out) and, concurrently, the NPP of
 * superframe k + 1 (d_sp_next, in place; NULL = none), on a second internal
 * stream.  The two touch disjoint parts of every channel's state, so a
 * sequence npp(0), pipe(0, 1), pipe(1, 2), ..., pipe(K-1, NULL) gives the
 * bits and NPP output of K melpe_encode_dev calls; the next superframe's
 * NPP runs in the SIMD slots the analysis leaves as its waves finish.
 * d_sp_next must be another buffer than d_sp.  Ordered on hip_stream like
 * the other *_dev calls (after its earlier work, before its later work). */
int melpe_encode_pipe_dev(melpe_engine *e, void *d_bits, const void *d_sp, const void *d_active,
			  void *d_sp_next, const void *d_active_next, void *hip_stream);

/* melpe_encode_pipe_dev plus a decode (melpe_decode_dev: d_dec_bits in,
 * C x 11; d_dec_sp out, C x 540; NULL d_dec_bits = no decode) on a third
 * internal stream, concurrently with the encode's analysis and next NPP --
 * a round trip or a duplex link, e.g. decoding the bits the previous call
 * encoded (BASELINE config 3).  The decoder touches only the channels'
 * decoder state, so the results are those of the same calls serialised.
 * d_dec_bits must not be d_bits and d_dec_sp none of d_sp, d_sp_next.
 * Ordered on hip_stream like the other *_dev calls: all three parts start
 * after its earlier work and its later work waits for all three. */
int melpe_duplex_pipe_dev(melpe_engine *e, void *d_bits, const void *d_sp, const void *d_active,
			  void *d_sp_next, const void *d_active_next, void *d_dec_sp,
			  const void *d_dec_bits, const void *d_dec_active, void *hip_stream);

/* melpe_s on every active channel: bits (C x 11, in), sp (C x 540, out) */
int melpe_decode_host(melpe_engine *e, int16_t *sp, const unsigned char *bits,
		      const uint8_t *active);
int melpe_decode_dev(melpe_engine *e, void *d_sp, const void *d_bits,
		     const void *d_active, void *hip_stream);

/* The 2400 bps MELP mode (54 bits per 180-sample frame, in 7 bytes), which
 * the reference compiles but cannot reach through melpe_i (melpe/melpe.c:76
 * pins RATE1200): per active channel, encode2400 = npp of the frame at
 * RATE2400 + analysis + melp_chn_write (sp C x 180 in/out, bits C x 7 out);
 * decode2400 = melp_chn_read + synthesis of one frame (bits C x 7 in, sp C x
 * 180 out).  A channel runs either mode from its reset, not both. */
int melpe_encode2400_dev(melpe_engine *e, void *d_bits, void *d_sp, const void *d_active,
			 void *hip_stream);
int melpe_decode2400_dev(melpe_engine *e, void *d_sp, const void *d_bits, const void *d_active,
			 void *hip_stream);
int melpe_encode2400_host(melpe_engine *e, unsigned char *bits, int16_t *sp,
			  const uint8_t *active);
int melpe_decode2400_host(melpe_engine *e, int16_t *sp, const unsigned char *bits,
			  const uint8_t *active);

/* melpe_n on `frames` consecutive 180-sample frames of every active channel.
 * sp is C x stride int16 (stride >= frames*180), in place.  A channel's first
 * frame reads 256 samples (melpe/npp.c:178-179), so stride should be at
 * least frames*180 + 76 with the look-ahead samples supplied. */
int melpe_npp_host(melpe_engine *e, int16_t *sp, int frames, int stride,
		   const uint8_t *active);
int melpe_npp_dev(melpe_engine *e, void *d_sp, int frames, int stride,
		  const void *d_active, void *hip_stream);

/* deterministic integer test signal (pairphone_amd/csrc/synth.h) generated
 * on the device: `samples` samples for each of C channels, continuing each
 * channel's generator state (seeded by melpe_synth_seed). Output C x samples
 * channel-major, device pointer. */
int melpe_synth_seed(melpe_engine *e, uint32_t run_seed, uint32_t first_channel);
int melpe_synth_dev(melpe_engine *e, void *d_sp, int samples, void *hip_stream);

/* same generator on the host, one channel (for tests and tools) */
int melpe_synth_host(uint32_t run_seed, uint32_t channel, int16_t *out, int samples);

/* wall-clock of the last *_dev/_host call's kernel on the engine stream, ms,
 * measured with HIP events (0 if unavailable) */
double melpe_last_kernel_ms(const melpe_engine *e);

/* Voice-frame encryption, the step after melpe_a on TX and before melpe_s on
 * RX: PairPhone's VoiceEnc (dir 0) / VoiceDec (dir 1), crp.c:986-1027,
 * called from MakeCtr (crp.c:819) and ProcessCtr (crp.c:980).  Each 11-byte
 * packet is XORed in place with gamma = Keccak sponge (r 576, c 1024) of
 * counter (4 bytes little-endian) || key (16 bytes), 81 bits.
 * pkts: C x K x 11 bytes (packet k of channel c at (c*K + k)*11).
 * counters: C uint32, packet k uses counters[c] + k (cnt_out / cnt_in, which
 *   advance by one per packet, crp.c:805).
 * keys: C x 16 bytes, the channel's skey[0..15] to encrypt or skey[16..31]
 *   to decrypt (crp.c:995, :1021); device pointer 16-byte aligned.
 * invert: optional C-byte mask (NULL = none), decrypt only: nonzero = the
 *   channel polarity flag finv < 0 (crp.c:1011-1015), the packet's 81 bits
 *   are inverted before decryption. */
int melpe_voice_crypt_dev(void *d_pkts, const void *d_counters, const void *d_keys,
			  const void *d_invert, int channels, int packets, int dir,
			  void *hip_stream);
int melpe_voice_crypt_host(unsigned char *pkts, const uint32_t *counters,
			   const unsigned char *keys, const uint8_t *invert, int channels,
			   int packets, int dir);
/* Voice activity detection, the TX gate in front of melpe_a: PairPhone runs
 * the AMR VAD option 2 (vad/vad2.c:203) on six 80-sample windows of every
 * superframe, at offsets 10, 100, ..., 460 (tx.c:234-239,
 * melpe_enc.c:48-53), and sends the superframe as silence when all six say
 * no.  state: C records of melpe_vad_state_bytes() bytes (device memory,
 * 4-byte aligned), one vadState2 (vad/vad2.h:76-103) per channel;
 * melpe_vad_reset_dev = vad2_reset (vad/vad2.c:876) on the channels of
 * `mask` (NULL = all).  melpe_vad_dev: sp is C x 540 int16, votes[c] (out,
 * uint8) = the sum of the six decisions (0 = silence); inactive channels
 * (active[c] == 0) keep their state and vote.  melpe_vad_host takes host
 * buffers, state included. */
int melpe_vad_state_bytes(void);
int melpe_vad_reset_dev(void *d_state, int channels, const void *d_mask, void *hip_stream);
int melpe_vad_dev(void *d_state, const void *d_sp, void *d_votes, int channels,
		  const void *d_active, void *hip_stream);
int melpe_vad_host(unsigned char *state, const int16_t *sp, uint8_t *votes, int channels,
		   const uint8_t *active);
/* The TX front end of one superframe (BASELINE config 5, tx.c:232-245):
 * the VAD gate above, then melpe_a on the channels it opens.  gate[c]
 * (out) = active[c] && votes[c] > 0; gated-off channels keep their codec
 * state, PCM and bits, exactly as when tx.c skips melpe_a.  d_active NULL =
 * all channels (ragged streams pass their mask). */
int melpe_tx_dev(melpe_engine *e, void *d_vad_state, void *d_bits, void *d_sp, void *d_votes,
		 void *d_gate, const void *d_active, void *hip_stream);
/* melpe_tx_dev in two halves, for the pipelined form: melpe_tx_npp_dev is
 * the VAD gate and the NPP of the channels it opens; melpe_tx_pipe_dev is
 * the analysis of superframe k under its gate (d_gate, written by the
 * previous call) and, concurrently on a second internal stream once the
 * analysis' lane-order sort is done, the VAD of superframe k + 1
 * (d_votes_next, d_gate_next out; d_active_next its mask) and the NPP of
 * the channels that gate opens (d_sp_next NULL = none).  A sequence
 * tx_npp(0), tx_pipe(0, 1), ..., tx_pipe(K-1, NULL) gives the bits, votes,
 * gates and NPP output of K melpe_tx_dev calls.  The next superframe's
 * buffers must be other buffers than this one's. */
int melpe_tx_npp_dev(melpe_engine *e, void *d_vad_state, void *d_sp, void *d_votes, void *d_gate,
		     const void *d_active, void *hip_stream);
int melpe_tx_pipe_dev(melpe_engine *e, void *d_vad_state, void *d_bits, const void *d_sp,
		      const void *d_gate, void *d_sp_next, void *d_votes_next, void *d_gate_next,
		      const void *d_active_next, void *hip_stream);
/* The VAD-framed stream format of melpe_enc.c:55-72 / melpe_dec.c:33-49
 * (host functions, no GPU).  Per superframe a silent channel writes 1 byte,
 * its carried txbuf[0] with bit 1 set; a voiced channel writes its 11 bytes
 * with bytes 0 and 10 swapped, so that the first byte (bit 80 only) never has
 * bit 1 set.  melpe_stream_pack does one superframe for C channels: bits
 * C x 11 and votes C in (melpe_vad_dev), last C bytes in/out (the carried
 * txbuf[0]; zero at the start: melpe_enc.c leaves it uninitialised and
 * melpe_dec.c reads only bit 1 of it), out C x 11 and lens C (1 or 11; 0
 * for channels that active excludes).  melpe_stream_unpack parses one
 * channel's stream: bits (max_sf x 11, swap undone; zeros for silence) and
 * voiced (1 = melpe_s it, 0 = 540 zero samples); returns the number of
 * superframes, or < 0 for a truncated voiced frame. */
int melpe_stream_pack(const unsigned char *bits, const uint8_t *votes, uint8_t *last,
		      unsigned char *out, uint8_t *lens, int channels, const uint8_t *active);
long melpe_stream_unpack(const unsigned char *stream, long nbytes, unsigned char *bits,
			 uint8_t *voiced, long max_sf);
const char *melpe_last_error(void);

/* The pseudo-voice BPSK modem, PairPhone's TX step after the voice-frame
 * crypt (Modulate, modem/modem.c:136, tx.c:271) and its RX step before it
 * (Demodulate, modem/modem.c:186, rx.c:294-297).  state: C records of
 * melpe_modem_state_bytes() (device, 4-byte aligned) = the modem's file
 * statics (modem.c:48-73) per channel; melpe_modem_reset_dev gives a fresh
 * process's values (mask: device C bytes or NULL = all).
 * melpe_modulate_dev: pkts C x K x 11 bytes (81 bits each) -> pcm C x K x
 *   3240 int16 at 48 kHz (4-byte aligned), K packets per channel in order.
 * melpe_demodulate_dev: `calls` successive Demodulate calls per channel, as
 *   rx.c makes them: channel c's samples are pcm[c*stride ...]; pos[c]
 *   (int32, in/out) is the sample offset of its next call and advances by
 *   each call's return value (216 +- 9); data C x 12 (in/out) is the
 *   persistent buf of rx.c (payload bytes 0..10, lag in byte 10's upper bits,
 *   status in byte 11: 0x80 packet ready, 0x40 block locked, 0x20 phase
 *   locked, 0x10 frequency locked, low nibble symbol errors).  Optional
 *   out C x calls x 12 gets data after every call, ret C x calls int32 the
 *   return values.  A call needs 1080 samples from pos (rx.c:246); one that
 *   would read past stride returns -1 and ends that channel's launch. */
int melpe_modem_state_bytes(void);
int melpe_modem_reset_dev(void *d_state, int channels, const void *d_mask, void *hip_stream);
int melpe_modulate_dev(void *d_state, const void *d_pkts, void *d_pcm, int channels, int packets,
		       const void *d_active, void *hip_stream);
int melpe_demodulate_dev(void *d_state, const void *d_pcm, long stride, void *d_pos, void *d_data,
			 void *d_out, void *d_ret, int channels, int calls, const void *d_active,
			 void *hip_stream);

/* Device basic-op self-test: out[i] = op(a[i], b[i], c[i]) evaluated by the
 * device build of the saturating basic operators, op ids of
 * pairphone_amd/csrc/ops_eval.h (a int64, b and c int32 or NULL, out int64,
 * all device pointers).  tests/test_device_ops.py compares it with the
 * reference's operators. */
int melpe_ops_eval_dev(int op, const void *d_a, const void *d_b, const void *d_c, void *d_out,
		       long n, void *hip_stream);
/* Host-fed pipelined encode: melpe_encode_host's work (PCM in, NPP output
 * back into sp, bits out) enqueued without waiting.  The engine keeps two
 * device slots; call k's host-to-device copy, kernels and device-to-host
 * copy run on three streams, so superframe k's kernels overlap the copies
 * of superframes k - 1 and k + 1.  bits, sp and active must stay valid and
 * untouched until melpe_encode_host_wait returns (a slot's reuse two calls
 * later waits on the device only, so the host may not reuse a call's
 * buffers before the wait).  For the copies to overlap the kernels the host
 * buffers must be pinned (hipHostMalloc / hipHostRegister); with pageable
 * memory the runtime stages them and the host call blocks.  Ordered after
 * the engine's earlier calls on any stream. */
int melpe_encode_host_async(melpe_engine *e, unsigned char *bits, int16_t *sp, const uint8_t *active);
/* Waits for every melpe_encode_host_async call enqueued so far. */
int melpe_encode_host_wait(melpe_engine *e);

/* Device divide_s over its whole domain (0 <= num <= den < 2^15): d_digest
 * (32,767 uint64, device) gets, for den = 1 .. 32,767, the sum over every
 * num of q * (num * 0x9E3779B97F4A7C15 + 1) mod 2^64.  tests/
 * test_device_ops.py forms the same digests from the reference's divide_s. */
int melpe_divide_s_sweep_dev(void *d_digest, void *hip_stream);
/* Device self-test of the sample-stream and exact-correlator helpers the
 * codec kernels use (pairphone_amd/csrc/helpers_eval.h): n lanes, lane i on
 * its own 464 int16 of d_src at the offsets / length d_args[4i .. 4i+2],
 * 512 int32 results per lane in d_out.  tests/test_device_helpers.py. */
int melpe_helpers_eval_dev(int mode, const void *d_src, const void *d_args, void *d_out, int n,
			   void *hip_stream);

/* Diagnostics: per-stage wave-cycle totals of a profiling build
 * (libmelpe_amd_prof.so, -DMELPE_PROF; tools/stage_prof.py,
 * tools/mw_prof.py), read and cleared.  Returns the number of slots (256),
 * or an error in a normal build. */
int melpe_prof_read(uint64_t *out, int n);

/* Extension of the single-stream drop-in (include/melpe.h): return its one
 * instance to the state of a freshly started reference process (melpe_i
 * alone re-initialises only what melp_ana_init / melp_syn_init touch, as in
 * the reference).  Lets one process host several independent sessions. */
int melpe_single_reset(void);

#ifdef __cplusplus
}
#endif

#endif
