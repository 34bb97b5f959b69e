"""Host mirror of the engine's C ABI (include/melpe_batch.h, include/melpe.h).

`Melpe` mirrors the reference's single-stream interface (melpe/melpe.h:10-14:
melpe_n / melpe_i / melpe_a / melpe_s) with the same names, argument meaning
and in-place side effect (melpe_a overwrites its input with the NPP output,
melpe/melpe.c:94-96).  `MelpeEngine` is the batched engine: C channels per
GPU, one superframe of every active channel per call.

There is no CPU fallback: if libmelpe_amd.so cannot be loaded or no GPU is
usable, these classes raise.
"""
import ctypes
import os

import numpy as np

SF_SAMPLES = 540
SF_BYTES = 11
FRAME_SAMPLES = 180

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmelpe_amd.so")
_lib = None


def load_library(path=None):
    """Loads libmelpe_amd.so (the HIP build); raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("MELPE_AMD_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise ImportError("libmelpe_amd.so not built (%s): run __graft_entry__.build()" % p)
    lib = ctypes.CDLL(p)
    vp, i32, u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32
    sig = {
        "melpe_engine_create": (i32, [ctypes.POINTER(vp), i32, i32]),
        "melpe_engine_destroy": (i32, [vp]),
        "melpe_engine_channels": (i32, [vp]),
        "melpe_engine_reset": (i32, [vp, vp, i32]),
        "melpe_engine_reset_dev": (i32, [vp, vp, i32, vp]),
        "melpe_engine_set_lane_order": (i32, [vp, i32]),
        "melpe_engine_set_ana_waves": (i32, [vp, i32]),
        "melpe_engine_set_dec_waves": (i32, [vp, i32]),
        "melpe_engine_set_mw_live_max": (i32, [vp, i32]),
        "melpe_engine_last_ana_waves": (i32, [vp]),
        "melpe_engine_set_own_stream": (i32, [vp, i32]),
        "melpe_engine_state_bytes": (ctypes.c_long, [i32]),
        "melpe_engine_export": (i32, [vp, i32, i32, i32, vp]),
        "melpe_engine_import": (i32, [vp, i32, i32, i32, vp]),
        "melpe_modem_state_bytes": (i32, []),
        "melpe_modem_reset_dev": (i32, [vp, i32, vp, vp]),
        "melpe_modulate_dev": (i32, [vp, vp, vp, i32, i32, vp, vp]),
        "melpe_demodulate_dev": (i32, [vp, vp, ctypes.c_long, vp, vp, vp, vp, i32, i32, vp, vp]),
        "melpe_ops_eval_dev": (i32, [i32, vp, vp, vp, vp, ctypes.c_long, vp]),
        "melpe_divide_s_sweep_dev": (i32, [vp, vp]),
        "melpe_encode_host_async": (i32, [vp, vp, vp, vp]),
        "melpe_encode_host_wait": (i32, [vp]),
        "melpe_helpers_eval_dev": (i32, [i32, vp, vp, vp, i32, vp]),
        "melpe_encode_host": (i32, [vp, vp, vp, vp]),
        "melpe_encode_dev": (i32, [vp, vp, vp, vp, vp]),
        "melpe_encode_npp_dev": (i32, [vp, vp, vp, vp]),
        "melpe_encode_ana_dev": (i32, [vp, vp, vp, vp, vp]),
        "melpe_encode_pipe_dev": (i32, [vp, vp, vp, vp, vp, vp, vp]),
        "melpe_duplex_pipe_dev": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "melpe_decode_host": (i32, [vp, vp, vp, vp]),
        "melpe_decode_dev": (i32, [vp, vp, vp, vp, vp]),
        "melpe_npp_host": (i32, [vp, vp, i32, i32, vp]),
        "melpe_npp_dev": (i32, [vp, vp, i32, i32, vp, vp]),
        "melpe_synth_seed": (i32, [vp, u32, u32]),
        "melpe_synth_dev": (i32, [vp, vp, i32, vp]),
        "melpe_synth_host": (i32, [u32, u32, vp, i32]),
        "melpe_last_kernel_ms": (ctypes.c_double, [vp]),
        "melpe_last_error": (ctypes.c_char_p, []),
        "melpe_single_reset": (i32, []),
        "melpe_prof_read": (i32, [vp, i32]),
        "melpe_voice_crypt_dev": (i32, [vp, vp, vp, vp, i32, i32, i32, vp]),
        "melpe_voice_crypt_host": (i32, [vp, vp, vp, vp, i32, i32, i32]),
        "melpe_vad_state_bytes": (i32, []),
        "melpe_vad_reset_dev": (i32, [vp, i32, vp, vp]),
        "melpe_vad_dev": (i32, [vp, vp, vp, i32, vp, vp]),
        "melpe_vad_host": (i32, [vp, vp, vp, i32, vp]),
        "melpe_tx_dev": (i32, [vp, vp, vp, vp, vp, vp, vp, vp]),
        "melpe_tx_npp_dev": (i32, [vp, vp, vp, vp, vp, vp, vp]),
        "melpe_tx_pipe_dev": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "melpe_stream_pack": (i32, [vp, vp, vp, vp, vp, i32, vp]),
        "melpe_stream_unpack": (ctypes.c_long, [vp, ctypes.c_long, vp, vp, ctypes.c_long]),
        "melpe_encode2400_dev": (i32, [vp, vp, vp, vp, vp]),
        "melpe_decode2400_dev": (i32, [vp, vp, vp, vp, vp]),
        "melpe_encode2400_host": (i32, [vp, vp, vp, vp]),
        "melpe_decode2400_host": (i32, [vp, vp, vp, vp]),
        "melpe_i2": (None, []),
        "melpe_al": (None, [vp, vp]),
        "melpe_i": (None, []),
        "melpe_a": (None, [vp, vp]),
        "melpe_s": (None, [vp, vp]),
        "melpe_n": (None, [vp]),
    }
    # an older build named by MELPE_AMD_LIB (A/B measurements) may lack the
    # newest entry points; the product library must export every one
    older = p != LIB_PATH and os.environ.get("MELPE_AMD_LIB") == p
    for name, (res, args) in sig.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if older:
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _check(rc):
    if rc != 0:
        raise RuntimeError("libmelpe_amd: %s" % load_library().melpe_last_error().decode())


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def synth_signal(run_seed, channel, samples):
    """Deterministic integer test signal of one channel (csrc/synth.h)."""
    out = np.zeros(samples, dtype=np.int16)
    _check(load_library().melpe_synth_host(run_seed, channel, _ptr(out), samples))
    return out


def _crypt(pkts, counters, keys, invert, direction):
    pkts = np.ascontiguousarray(pkts, dtype=np.uint8)
    if pkts.ndim == 2:
        pkts = pkts[:, None, :]
    if pkts.ndim != 3 or pkts.shape[2] != SF_BYTES:
        raise ValueError("packets must be C x 11 or C x K x 11 bytes")
    out = pkts.copy()
    C, K = out.shape[:2]
    counters = np.ascontiguousarray(counters, dtype=np.uint32).reshape(C)
    keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(C, 16)
    inv = None if invert is None else np.ascontiguousarray(invert, dtype=np.uint8).reshape(C)
    _check(load_library().melpe_voice_crypt_host(_ptr(out), _ptr(counters), _ptr(keys),
                                                  _ptr(inv), C, K, direction))
    return out


def VoiceEnc(pkts, counters, keys):
    """crp.c:986-1000 on C channels x K packets: each 11-byte packet XORed
    with the 81-bit sponge keystream of (counters[c] + k, keys[c]), keys =
    the channel's skey[0..15].  Returns the encrypted copy."""
    return _crypt(pkts, counters, keys, None, 0)


def VoiceDec(pkts, counters, keys, invert=None):
    """crp.c:1004-1027: `invert[c]` nonzero = polarity flag finv < 0 (the
    81 bits are inverted first); keys = skey[16..31]."""
    return _crypt(pkts, counters, keys, invert, 1)


def stream_pack(bits, votes):
    """melpe_enc.c:55-72 framing of one channel: bits (nsf x 11) and VAD
    votes (nsf) -> the framed byte stream (1 byte per silent superframe, 11
    swapped bytes per voiced one)."""
    lib = load_library()
    bits = np.ascontiguousarray(bits, np.uint8).reshape(-1, SF_BYTES)
    votes = np.ascontiguousarray(votes, np.uint8).reshape(-1)
    last = np.zeros(1, np.uint8)
    out = np.zeros(SF_BYTES, np.uint8)
    n = np.zeros(1, np.uint8)
    chunks = []
    for k in range(bits.shape[0]):
        _check(lib.melpe_stream_pack(_ptr(bits[k]), _ptr(votes[k:k + 1]), _ptr(last), _ptr(out),
                                     _ptr(n), 1, None))
        chunks.append(out[:n[0]].tobytes())
    return b"".join(chunks)


def stream_unpack(stream, max_sf=None):
    """melpe_dec.c:33-49: framed bytes -> (bits nsf x 11, voiced nsf)"""
    lib = load_library()
    buf = np.frombuffer(bytes(stream), np.uint8)
    max_sf = len(buf) if max_sf is None else max_sf
    bits = np.zeros((max(max_sf, 1), SF_BYTES), np.uint8)
    voiced = np.zeros(max(max_sf, 1), np.uint8)
    k = lib.melpe_stream_unpack(_ptr(buf), len(buf), _ptr(bits), _ptr(voiced), max_sf)
    if k < 0:
        raise RuntimeError("libmelpe_amd: %s" % lib.melpe_last_error().decode())
    return bits[:k], voiced[:k]


class Vad:
    """PairPhone's TX voice-activity gate on C channels (vad/vad2.c run on six
    windows per superframe, tx.c:234-239); state per channel = a fresh
    vad2_reset vadState2.  `superframe(sp)` returns the C votes (0..6);
    0 means the superframe is sent as silence."""

    def __init__(self, channels):
        self.lib = load_library()
        self.C = channels
        self.state = np.zeros(channels * self.lib.melpe_vad_state_bytes(), np.uint8)

    def reset(self):
        self.state[:] = 0

    def superframe(self, sp, active=None):
        sp = np.ascontiguousarray(sp, dtype=np.int16).reshape(self.C, SF_SAMPLES)
        votes = np.zeros(self.C, np.uint8)
        act = None if active is None else np.ascontiguousarray(active, np.uint8)
        _check(self.lib.melpe_vad_host(_ptr(self.state), _ptr(sp), _ptr(votes), self.C,
                                       _ptr(act)))
        return votes


class MelpeEngine:
    """C independent MELPe-1200 channels on one GPU (include/melpe_batch.h)."""

    def __init__(self, channels, device=0):
        self.lib = load_library()
        self.h = ctypes.c_void_p()
        _check(self.lib.melpe_engine_create(ctypes.byref(self.h), device, channels))
        self.channels = channels

    def close(self):
        if self.h:
            self.lib.melpe_engine_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, mask=None, which=3):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        _check(self.lib.melpe_engine_reset(self.h, _ptr(m), which))

    def set_lane_order(self, on):
        """pitch-class lane order of the analysis / synthesis kernels on or
        off (results are the same either way)"""
        _check(self.lib.melpe_engine_set_lane_order(self.h, 1 if on else 0))

    def set_ana_waves(self, waves):
        """waves per 64 channels of the analysis kernel: 1 lane per channel,
        4 waves per channel group (ana_mw.h), 0 = by channel count (results
        are the same either way)"""
        _check(self.lib.melpe_engine_set_ana_waves(self.h, int(waves)))

    def set_dec_waves(self, waves):
        """waves per 64 channels of the decoder: 1 lane per channel, 2 the
        two-wave decoder (excitation / filters, up to 65,536 channels), 0 =
        by channel count (PCM is the same either way)"""
        _check(self.lib.melpe_engine_set_dec_waves(self.h, int(waves)))

    def set_mw_live_max(self, live_max):
        """above 32,768 channels, superframes with at most live_max live
        channels run the four-wave analysis (0 = off; results are the same
        either way)"""
        _check(self.lib.melpe_engine_set_mw_live_max(self.h, int(live_max)))

    def set_own_stream(self, on):
        """run this engine's kernels on a stream (hardware queue) of its own
        instead of the device's shared engine stream"""
        _check(self.lib.melpe_engine_set_own_stream(self.h, 1 if on else 0))

    def last_ana_waves(self):
        """the mapping the last analysis launch ran, recorded on the device:
        1 lane per channel, 4 four waves per 64 channels, 0 none"""
        r = self.lib.melpe_engine_last_ana_waves(self.h)
        _check(r if r < 0 else 0)
        return r

    def reset_dev(self, d_mask=None, which=3, stream=None):
        """reset enqueued on `stream` (ordered with the *_dev calls on it)"""
        _check(self.lib.melpe_engine_reset_dev(self.h, d_mask, which, stream))

    def export_state(self, which, first=0, count=None):
        """channel records [first, first+count) as a uint8 [count, bytes]
        array (which: 1 encoder, 2 decoder)"""
        count = self.channels - first if count is None else count
        rec = self.lib.melpe_engine_state_bytes(which)
        out = np.zeros((count, rec), np.uint8)
        _check(self.lib.melpe_engine_export(self.h, which, first, count, _ptr(out)))
        return out

    def import_state(self, which, records, first=0):
        rec = np.ascontiguousarray(records, np.uint8)
        assert rec.ndim == 2 and rec.shape[1] == self.lib.melpe_engine_state_bytes(which)
        _check(self.lib.melpe_engine_import(self.h, which, first, rec.shape[0], _ptr(rec)))

    def _mask(self, active):
        if active is None:
            return None
        m = np.ascontiguousarray(active, dtype=np.uint8)
        assert m.shape == (self.channels,)
        return m

    def encode(self, sp, active=None):
        """melpe_a on every channel. sp: int16 [C, 540], overwritten with the
        NPP output (as the reference).  Returns uint8 [C, 11]."""
        assert sp.dtype == np.int16 and sp.shape == (self.channels, SF_SAMPLES)
        assert sp.flags.c_contiguous
        bits = np.zeros((self.channels, SF_BYTES), dtype=np.uint8)
        m = self._mask(active)
        _check(self.lib.melpe_encode_host(self.h, _ptr(bits), _ptr(sp), _ptr(m)))
        return bits

    def encode_host_async(self, bits_ptr, sp_ptr, active_ptr=None):
        """host-fed pipelined encode (melpe_encode_host_async): host
        pointers (pinned for overlap) to uint8 [C, 11] bits and int16
        [C, 540] PCM, valid until encode_host_wait()"""
        _check(self.lib.melpe_encode_host_async(self.h, bits_ptr, sp_ptr, active_ptr))

    def encode_host_wait(self):
        _check(self.lib.melpe_encode_host_wait(self.h))

    def _raw_encode(self, sp, bits, active):
        """encode with caller-provided output bits (kept for inactive lanes)"""
        m = self._mask(active)
        _check(self.lib.melpe_encode_host(self.h, _ptr(bits), _ptr(sp), _ptr(m)))
        return bits

    def decode(self, bits, active=None):
        """melpe_s on every channel. bits: uint8 [C, 11] -> int16 [C, 540]."""
        bits = np.ascontiguousarray(bits, dtype=np.uint8)
        assert bits.shape == (self.channels, SF_BYTES)
        sp = np.zeros((self.channels, SF_SAMPLES), dtype=np.int16)
        m = self._mask(active)
        _check(self.lib.melpe_decode_host(self.h, _ptr(sp), _ptr(bits), _ptr(m)))
        return sp

    def encode2400(self, sp, active=None):
        """2400 bps mode: one 180-sample frame per channel. sp: int16 [C, 180],
        overwritten with the NPP output.  Returns uint8 [C, 7] (54 bits)."""
        assert sp.dtype == np.int16 and sp.shape == (self.channels, FRAME_SAMPLES)
        assert sp.flags.c_contiguous
        bits = np.zeros((self.channels, 7), dtype=np.uint8)
        _check(self.lib.melpe_encode2400_host(self.h, _ptr(bits), _ptr(sp), _ptr(self._mask(active))))
        return bits

    def decode2400(self, bits, active=None):
        """2400 bps mode: uint8 [C, 7] -> int16 [C, 180]."""
        bits = np.ascontiguousarray(bits, dtype=np.uint8)
        assert bits.shape == (self.channels, 7)
        sp = np.zeros((self.channels, FRAME_SAMPLES), dtype=np.int16)
        _check(self.lib.melpe_decode2400_host(self.h, _ptr(sp), _ptr(bits), _ptr(self._mask(active))))
        return sp

    def npp(self, sp, frames, active=None):
        """melpe_n on `frames` frames of every channel, in place.
        sp: int16 [C, stride] with stride >= frames*180 (+76 look-ahead)."""
        assert sp.dtype == np.int16 and sp.ndim == 2 and sp.flags.c_contiguous
        m = self._mask(active)
        _check(self.lib.melpe_npp_host(self.h, _ptr(sp), frames, sp.shape[1], _ptr(m)))
        return sp

    def encode_dev(self, d_bits, d_sp, d_active=None, stream=None):
        _check(self.lib.melpe_encode_dev(self.h, d_bits, d_sp, d_active, stream))

    def encode_npp_dev(self, d_sp, d_active=None, stream=None):
        _check(self.lib.melpe_encode_npp_dev(self.h, d_sp, d_active, stream))

    def encode_pipe_dev(self, d_bits, d_sp, d_sp_next, d_active=None, d_active_next=None, stream=None):
        """analysis of superframe k (d_sp already through the NPP) beside
        the NPP of superframe k + 1 (d_sp_next, or None)"""
        _check(self.lib.melpe_encode_pipe_dev(self.h, d_bits, d_sp, d_active, d_sp_next, d_active_next,
                                              stream))

    def duplex_pipe_dev(self, d_bits, d_sp, d_sp_next, d_dec_sp, d_dec_bits, d_active=None,
                        d_active_next=None, d_dec_active=None, stream=None):
        """encode_pipe_dev plus a decode (d_dec_bits -> d_dec_sp, or None)
        on the engine's decoder stream, beside the encode"""
        _check(self.lib.melpe_duplex_pipe_dev(self.h, d_bits, d_sp, d_active, d_sp_next, d_active_next,
                                              d_dec_sp, d_dec_bits, d_dec_active, stream))

    def encode_ana_dev(self, d_bits, d_sp, d_active=None, stream=None):
        _check(self.lib.melpe_encode_ana_dev(self.h, d_bits, d_sp, d_active, stream))

    def tx_dev(self, d_vad_state, d_bits, d_sp, d_votes, d_gate, d_active=None, stream=None):
        """VAD gate + melpe_a on the channels it opens (tx.c:232-245)"""
        _check(self.lib.melpe_tx_dev(self.h, d_vad_state, d_bits, d_sp, d_votes, d_gate,
                                     d_active, stream))

    def tx_npp_dev(self, d_vad_state, d_sp, d_votes, d_gate, d_active=None, stream=None):
        """the first half of tx_dev: VAD gate + the NPP of the opened channels"""
        _check(self.lib.melpe_tx_npp_dev(self.h, d_vad_state, d_sp, d_votes, d_gate, d_active, stream))

    def tx_pipe_dev(self, d_vad_state, d_bits, d_sp, d_gate, d_sp_next, d_votes_next, d_gate_next,
                    d_active_next=None, stream=None):
        """superframe k's analysis under its gate beside superframe k+1's
        VAD and NPP (d_sp_next None: none)"""
        _check(self.lib.melpe_tx_pipe_dev(self.h, d_vad_state, d_bits, d_sp, d_gate, d_sp_next,
                                          d_votes_next, d_gate_next, d_active_next, stream))

    def decode_dev(self, d_sp, d_bits, d_active=None, stream=None):
        _check(self.lib.melpe_decode_dev(self.h, d_sp, d_bits, d_active, stream))

    def synth_seed(self, run_seed, first_channel=0):
        _check(self.lib.melpe_synth_seed(self.h, run_seed, first_channel))

    def synth_dev(self, d_sp, samples, stream=None):
        _check(self.lib.melpe_synth_dev(self.h, d_sp, samples, stream))

    def last_kernel_ms(self):
        return self.lib.melpe_last_kernel_ms(self.h)


class Melpe:
    """Single-stream drop-in mirror of melpe/melpe.h (process-global state,
    exactly one instance, as the reference)."""

    def __init__(self):
        self.lib = load_library()

    def reset_process_state(self):
        """fresh-process state (melpe_single_reset extension)"""
        _check(self.lib.melpe_single_reset())

    def melpe_i(self):
        self.lib.melpe_i()

    def melpe_a(self, sp):
        """sp: int16[540], overwritten with the NPP output; returns 11 bytes."""
        assert sp.dtype == np.int16 and sp.shape == (SF_SAMPLES,) and sp.flags.c_contiguous
        buf = np.zeros(SF_BYTES, dtype=np.uint8)
        self.lib.melpe_a(_ptr(buf), _ptr(sp))
        return buf

    def melpe_s(self, buf):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        sp = np.zeros(SF_SAMPLES, dtype=np.int16)
        self.lib.melpe_s(_ptr(sp), _ptr(buf))
        return sp

    def melpe_n(self, sp):
        """denoise 180 samples in place; the first call reads 256 samples
        (melpe/npp.c:178-179), so pass at least 256 valid samples."""
        assert sp.dtype == np.int16 and sp.size >= 256 and sp.flags.c_contiguous
        self.lib.melpe_n(_ptr(sp))
        return sp
