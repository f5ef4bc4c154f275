"""Config-3 ablations of the lean varlen kernel (tuning library): full / loads only / compute
only, plus the generic kernel, each timed on the same 10M-frame batch.  GPU box:
    UFC_LIB=uflow_amd/libuflowcrc_tuning.so python tools/vl_ablate.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))

import torch  # noqa: E402

from bench_configs import timed  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    eng = FrameCrcEngine(0)
    n = int(os.environ.get("VL_N", 10_000_000))
    lo, hi = int(os.environ.get("VL_LO", 64)), int(os.environ.get("VL_HI", 1501))
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0002)
    lens = torch.randint(lo, hi, (n,), generator=g, device=dev, dtype=torch.int64)
    align = int(os.environ.get("VL_ALIGN", 1))  # round lengths to a multiple (alignment A/B)
    lens = (lens // align) * align
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    offsets[1:] = torch.cumsum(lens, 0)
    total = int(offsets[-1])
    data = torch.randint(0, 256, (total,), generator=g, device=dev, dtype=torch.uint8)
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    fn = lambda: eng.crc_varlen(data, offsets, crc_out=crc, valid_out=valid)  # noqa: E731
    out = {"frames": n, "bytes": total, "lens": [lo, hi - 1], "align": align}
    for name, env in (("full", {}), ("loads_only", {"UFC_VL_ABL": "1"}), ("compute_only", {"UFC_VL_ABL": "2"}),
                      ("generic", {"UFC_VARLEN_KERNEL": "generic"}), ("full2", {})):
        os.environ.update(env)
        fn()
        torch.cuda.synchronize()
        ms = timed(fn, 20, s)
        for k in env:
            del os.environ[k]
        out[name] = round(ms, 4)
        print(name, round(ms, 4), "ms", round(total / ms / 1e-3 / 1e9, 1), "GB/s", flush=True)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
