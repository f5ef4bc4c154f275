"""Time the fixed validate kernel on config 2's batch (1M x 1500 B) a few times, after a settle
phase; checksum of the results to compare libraries.  Usage: python tools/probes/fxrun.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from uflow_amd import synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
n, L = 1_000_000, 1500
eng = FrameCrcEngine(0)
frames = synth.fixed_frames(n, L, synth.SEED_CONFIG2, device="cuda")
eng.seal_fixed(frames, L, n=n)
crc = torch.empty(n, dtype=torch.int32, device="cuda")
valid = torch.empty(n, dtype=torch.uint8, device="cuda")
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.1:
    eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid)
    torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
for a, b in ev:
    a.record()
    eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid)
    b.record()
torch.cuda.synchronize()
t = [a.elapsed_time(b) for a, b in ev]
print(f"median {np.median(t):.4f} ms mean {np.mean(t):.4f} min {min(t):.4f} checksum "
      f"{int(crc.to(torch.int64).sum()) & 0xFFFFFFFFFFFF} valid {int(valid.sum())}", flush=True)
eng.close()
