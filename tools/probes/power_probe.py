"""Clocks and power while a kernel runs back to back (tuning probe): config 2's gate, the plain
read-only stream over the same buffer, the gate again, each for PP_SECS seconds; `rocm-smi
--showclocks --showpower` sampled from a thread in the middle of each phase while launches go on.
Is the gate's lower marginal rate (against the stream) a clock/power effect?  One JSON line per
phase."""
import json
import os
import re
import subprocess
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch  # noqa: E402

from uflow_amd import synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

secs = float(os.environ.get("PP_SECS", 3.0))
eng = FrameCrcEngine(0)
n, L = 1_000_000, 1500
frames = synth.fixed_frames(n, L, synth.SEED_CONFIG2, device="cuda")
eng.seal_fixed(frames, L, n=n)
crc = torch.empty(n, dtype=torch.int32, device="cuda")
valid = torch.empty(n, dtype=torch.uint8, device="cuda")
sink = torch.zeros(1, dtype=torch.int32, device="cuda")


def smi():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks", "--showpower"], capture_output=True, text=True,
                             timeout=20).stdout
    except (OSError, subprocess.TimeoutExpired) as e:
        return {"error": str(e)}
    r = {}
    for key in ("fclk", "mclk", "sclk", "socclk"):
        m = re.search(key + r" clock level: \d+: \((\d+)Mhz\)", out)
        if m:
            r[key + "_MHz"] = int(m.group(1))
    m = re.search(r"Power \(W\): ([\d.]+)", out)
    if m:
        r["power_W"] = float(m.group(1))
    return r


def phase(name, fn):
    t0 = time.perf_counter()
    launches = 0
    sample = None
    child = None
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    while time.perf_counter() - t0 < secs:
        ev0.record()
        for _ in range(20):
            fn()
        ev1.record()
        ev1.synchronize()
        launches += 20
        if time.perf_counter() - t0 > secs / 3:
            times.append(ev0.elapsed_time(ev1) / 20)
        if child is None and time.perf_counter() - t0 > secs / 2:
            # sample from a thread while launches continue
            import threading
            res = {}
            child = threading.Thread(target=lambda: res.update(smi()))
            child.start()
            sample = res
    if child is not None:
        child.join()
    times.sort()
    print(json.dumps({"phase": name, "launches": launches, "ms_median": round(times[len(times) // 2], 4),
                      **(sample or {})}), flush=True)


phase("gate", lambda: eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid))
phase("stream", lambda: eng.hbm_read_probe(frames, sink))
phase("gate", lambda: eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid))
print(json.dumps({"phase": "idle", **smi()}), flush=True)
