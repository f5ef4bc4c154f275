"""Per-wave timeline of the 8-lane varlen kernel on config 3 (tuning build): warm launches, then
FX_DUMPS launches with UFC_DBG_WAVES set, each summarised by tools/wave_timeline.py.
    UFC_LIB=uflow_amd/libuflowcrc_tuning.so python tools/probes/vl_wave_dump.py gpurun_out/vlwaves.bin"""
import os
import subprocess
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from uflow_amd import synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

out = sys.argv[1]
n = int(os.environ.get("VL_N", 10_000_000))
eng = FrameCrcEngine(0)
data, offsets = synth.varlen_batch(n, 64, 1500, synth.SEED_CONFIG3, device="cuda:0")
eng.seal_varlen(data, offsets)
crc = torch.empty(n, dtype=torch.int32, device="cuda:0")
valid = torch.empty(n, dtype=torch.uint8, device="cuda:0")
for _ in range(20):
    eng.crc_varlen(data, offsets, crc_out=crc, valid_out=valid)
torch.cuda.synchronize()
reps = int(os.environ.get("FX_DUMPS", 2))
for i in range(reps):
    path = f"{out}.{i}"
    os.environ["UFC_DBG_WAVES"] = path
    eng.crc_varlen(data, offsets, crc_out=crc, valid_out=valid)
    torch.cuda.synchronize()
    del os.environ["UFC_DBG_WAVES"]
    print("valid", int(valid.sum()), "of", n, flush=True)
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "wave_timeline.py"), path], check=True)
