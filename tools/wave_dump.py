"""Per-wave timeline of the fixed-length kernel (tuning build): 30 warm launches, then one with
UFC_DBG_WAVES=<file> set (FX_DUMPS=k: k such launches, <file>.0 ..); summarised by
tools/wave_timeline.py.
    UFC_LIB=uflow_amd/libuflowcrc_tuning.so python tools/wave_dump.py gpurun_out/waves.bin"""
import os
import subprocess
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

out = sys.argv[1]
n, L = int(os.environ.get("FX_N", 1_000_000)), 1500
eng = FrameCrcEngine(0)
g = torch.Generator(device="cuda:0")
g.manual_seed(1)
d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda:0", generator=g)
eng.seal_fixed(d, L, n=n)
crc = torch.empty(n, dtype=torch.int32, device="cuda:0")
valid = torch.empty(n, dtype=torch.uint8, device="cuda:0")
for _ in range(30):
    eng.crc_fixed(d, L, n=n, crc_out=crc, valid_out=valid)
torch.cuda.synchronize()
reps = int(os.environ.get("FX_DUMPS", 1))  # several dumped launches: is the per-XCD spread systematic?
for i in range(reps):
    path = out if reps == 1 else f"{out}.{i}"
    os.environ["UFC_DBG_WAVES"] = path
    eng.crc_fixed(d, L, n=n, crc_out=crc, valid_out=valid)
    torch.cuda.synchronize()
    del os.environ["UFC_DBG_WAVES"]
    print("valid", int(valid.sum()))
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "wave_timeline.py"), path], check=True)
