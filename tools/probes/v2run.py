"""Run the varlen kernel (config 3 batch) a few times with nothing else on the GPU: a target for
rocprofv3 --pmc passes.  Usage: python tools/probes/v2run.py [reps] [kernel option value]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from uflow_amd import _native as N, synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
mode = int(sys.argv[2]) if len(sys.argv) > 2 else N.UFC_VARLEN_AUTO
eng = FrameCrcEngine(0)
eng.set_option(N.UFC_OPT_VARLEN_KERNEL, mode)
data, offsets = synth.varlen_batch(10_000_000, 64, 1500, synth.SEED_CONFIG3, device="cuda")
crc = torch.empty(10_000_000, dtype=torch.int32, device="cuda")
valid = torch.empty(10_000_000, dtype=torch.uint8, device="cuda")
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for i in range(reps):
    s.record()
    eng.crc_varlen(data, offsets, crc_out=crc, valid_out=valid)
    e.record()
    torch.cuda.synchronize()
    print(f"rep {i}: {s.elapsed_time(e):.4f} ms", flush=True)
# checksum of the results, to compare libraries (the product library's is checked by the tests)
print("checksum", int(crc.to(torch.int64).sum()) & 0xFFFFFFFFFFFF, int(valid.sum()), flush=True)
eng.close()
