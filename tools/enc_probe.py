"""GPU probe: encode kernel time per superframe at several channel counts."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pairphone_amd as pa

for ch in [int(a) for a in (sys.argv[1:] or ["1024", "16384", "65536"])]:
    eng = pa.MelpeEngine(ch)
    eng.synth_seed(1)
    s = torch.cuda.current_stream().cuda_stream
    nsf = 6
    x = torch.zeros((nsf, ch, 540), dtype=torch.int16, device="cuda")
    for k in range(nsf):
        eng.synth_dev(x[k].data_ptr(), 540, s)
    bits = torch.zeros((ch, 11), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ts = []
    for k in range(nsf):
        t = time.perf_counter()
        eng.encode_dev(bits.data_ptr(), x[k].data_ptr(), None, s)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    dt = min(ts[2:])
    print("channels %6d: %.2f ms/superframe (first %.1f ms) -> %.0f channel-s/s" %
          (ch, dt * 1e3, ts[0] * 1e3, ch * 0.0675 / dt), flush=True)
    eng.close()
