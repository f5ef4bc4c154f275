"""Per-launch cost against per-byte cost: config 2's gate and the plain read-only stream
(ufc_hbm_read_probe, bench's ceiling) over the first n frames of one 4M x 1500-B buffer, n from
0.25M to 4M; HIP events around groups of 10 back-to-back launches, rounds interleaved.  A least-squares
line per kernel gives the marginal rate (TB/s) and the fixed cost per launch (us).  Tuning probe."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from uflow_amd import synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

eng = FrameCrcEngine(0)
L, NMAX = 1500, 4_000_000
frames = synth.fixed_frames(NMAX, L, synth.SEED_CONFIG2, device="cuda")
eng.seal_fixed(frames, L, n=NMAX)
crc = torch.empty(NMAX, dtype=torch.int32, device="cuda")
valid = torch.empty(NMAX, dtype=torch.uint8, device="cuda")
sink = torch.zeros(1, dtype=torch.int32, device="cuda")
sizes = [250_000, 500_000, 1_000_000, 2_000_000, 4_000_000]
G = 10


def gate(n):
    eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid)


def stream(n):
    eng.hbm_read_probe(frames[: n * L], sink)


def timed(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(G):
        fn(n)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / G


import time  # noqa: E402
t_settle = time.perf_counter()  # settle: clocks ramp up from idle over ~1 s
while time.perf_counter() - t_settle < 1.5:
    for n in sizes:
        gate(n)
        stream(n)
    torch.cuda.synchronize()
res = {k: {n: [] for n in sizes} for k in ("gate", "stream")}
for r in range(5):
    for n in sizes:
        res["gate"][n].append(timed(gate, n))
        res["stream"][n].append(timed(stream, n))
nvalid = int(valid.sum())  # the last launch gated all NMAX frames of the GPU-sealed batch
ok = nvalid == NMAX
for k, d in res.items():
    x = np.array([n * L for n in sizes], dtype=np.float64)
    y = np.array([float(np.median(d[n])) for n in sizes])
    slope, icpt = np.polyfit(x, y, 1)
    print(json.dumps({"kernel": k, "ms_median": {str(n): round(float(np.median(d[n])), 4) for n in sizes},
                      "marginal_TBs": round(1e-9 / slope, 3), "fixed_us_per_launch": round(icpt * 1e3, 2),
                      "frac_at_1M": round(1.505e9 / (float(np.median(d[1_000_000])) * 1e-3) / 8e12, 4),
                      "valid_count": nvalid, "valid_counts_ok": ok}), flush=True)
if not ok:
    sys.exit(f"self-check failed: {nvalid} of {NMAX} sealed frames valid")
