"""Config 2's gate (1M x 1500-B frames) launched back to back on one stream against alternating two
streams (consecutive batches' launches may then overlap: one's ramp with the other's tail), each with
its own output slot; total time of 50 launches, rounds interleaved.  Tuning probe."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch  # noqa: E402

from uflow_amd import synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

eng = FrameCrcEngine(0)
n, L = 1_000_000, 1500
frames = synth.fixed_frames(n, L, synth.SEED_CONFIG2, device="cuda")
eng.seal_fixed(frames, L, n=n)
outs = [(torch.empty(n, dtype=torch.int32, device="cuda"), torch.empty(n, dtype=torch.uint8, device="cuda"))
        for _ in range(2)]
streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
K = 50


def run(ns):
    for i in range(K):
        s = streams[i % ns]
        c, v = outs[i % ns]
        with torch.cuda.stream(s):
            eng.crc_fixed(frames, L, n=n, crc_out=c, valid_out=v)


import time  # noqa: E402
t_settle = time.perf_counter()  # settle: clocks ramp up from idle over ~1 s
while time.perf_counter() - t_settle < 1.5:
    eng.crc_fixed(frames, L, n=n, crc_out=outs[0][0], valid_out=outs[0][1])
    torch.cuda.synchronize()
res = {1: [], 2: []}
for r in range(6):
    for ns in (1, 2):
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(streams[0])
        streams[1].wait_event(e0)
        run(ns)
        streams[0].wait_stream(streams[1])
        e1.record(streams[0])
        e1.synchronize()
        res[ns].append(e0.elapsed_time(e1) / K)
counts = [int(o[1].sum()) for o in outs]
ok = all(c == n for c in counts)  # no flips planted: every GPU-sealed frame is valid
for ns in (1, 2):
    t = sorted(res[ns])
    print(json.dumps({"streams": ns, "ms_per_launch_median": round(t[len(t) // 2], 4), "min": round(t[0], 4),
                      "valid_counts": counts, "valid_counts_ok": ok}), flush=True)
if not ok:
    sys.exit(f"self-check failed: valid counts {counts}, expected {n}")
