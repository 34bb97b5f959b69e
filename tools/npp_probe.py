"""Quick GPU probe: NPP kernel throughput at several channel counts."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pairphone_amd as pa

for ch in [int(a) for a in (sys.argv[1:] or ["1024", "16384", "65536"])]:
    frames = 3
    eng = pa.MelpeEngine(ch)
    eng.synth_seed(1)
    x = torch.zeros((ch, frames * 180 + 76), dtype=torch.int16, device="cuda")
    eng.synth_dev(x.data_ptr(), x.shape[1], torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    eng.lib.melpe_npp_dev(eng.h, x.data_ptr(), frames, x.shape[1], None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    t = time.perf_counter()
    reps = 3
    for _ in range(reps):
        eng.lib.melpe_npp_dev(eng.h, x.data_ptr(), frames, x.shape[1], None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    print("channels %d: %.2f ms per 3 frames -> %.0f channel-frames/s (%.0f ch-s/s of NPP)" % (ch, dt * 1e3, ch * frames / dt, ch * frames * 0.0225 / dt), flush=True)
    eng.close()
