import json, os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
from uflow_amd import synth, _native as N
from uflow_amd.batch import FrameCrcEngine
eng = FrameCrcEngine(0)
n = 10_000_000
data, off = synth.varlen_batch(n, 64, 1500, synth.SEED_CONFIG3, device="cuda")
crc = torch.empty(n, dtype=torch.int32, device="cuda"); val = torch.empty(n, dtype=torch.uint8, device="cuda")
for mode in (N.UFC_VARLEN_STREAM, N.UFC_VARLEN_SORTED8):
    eng.set_option(N.UFC_OPT_VARLEN_KERNEL, mode)
    for _ in range(5): eng.crc_varlen(data, off, crc_out=crc, valid_out=val)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): eng.crc_varlen(data, off, crc_out=crc, valid_out=val)
    e1.record(); e1.synchronize()
    print(json.dumps({"lib": os.environ.get("UFC_LIB", "product"), "mode": mode, "ms": e0.elapsed_time(e1) / 10}), flush=True)
