"""pairphone_amd -- MI355X-native batched MELPe-1200 engine.

The product is libmelpe_amd.so (HIP kernels for gfx950 behind the C ABI in
include/melpe.h and include/melpe_batch.h).  This package is the Python host
mirror of that ABI (pairphone_amd.codec); it has no compute of its own and
raises if the HIP library is missing.
"""
from .codec import (MelpeEngine, Melpe, load_library, LIB_PATH,  # noqa: F401
                    SF_SAMPLES, SF_BYTES, FRAME_SAMPLES, synth_signal)
from .codec import VoiceEnc, VoiceDec, Vad, stream_pack, stream_unpack  # noqa: F401
