"""Config 2's batch (1M x 1500 B) through the fixed kernel and through the variable-length kernels
(CSR offsets i * 1500): is the 8-lane layout faster for fixed frames?  Timing probe."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from uflow_amd import _native as N, synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

n, L = 1_000_000, 1500
eng = FrameCrcEngine(0)
frames = synth.fixed_frames(n, L, synth.SEED_CONFIG2, device="cuda")
eng.seal_fixed(frames, L, n=n)
offs = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
crc = torch.empty(n, dtype=torch.int32, device="cuda")
valid = torch.empty(n, dtype=torch.uint8, device="cuda")


def timeit(fn, reps=40):
    import time
    t0 = time.perf_counter()  # settle: clocks ramp up from idle over ~1 s
    while time.perf_counter() - t0 < 1.5:
        fn()
        torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = [a.elapsed_time(b) for a, b in ev]
    return np.median(t), int(valid.sum())


print("fixed", timeit(lambda: eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid)), flush=True)
for name, mode in (("sorted8", N.UFC_VARLEN_SORTED8),):
    eng.set_option(N.UFC_OPT_VARLEN_KERNEL, mode)
    print(name, timeit(lambda: eng.crc_varlen(frames, offs, crc_out=crc, valid_out=valid)), flush=True)
eng.close()
