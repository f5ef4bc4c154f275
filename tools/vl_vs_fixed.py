"""The lean varlen kernel on a batch of equal-length frames vs the lean fixed kernel on the same
bytes (isolates the varlen kernel's mechanics from the length mix).  GPU box:
    UFC_LIB=uflow_amd/libuflowcrc_tuning.so python tools/vl_vs_fixed.py"""
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
    n, L = int(os.environ.get("VL_N", 3_000_000)), int(os.environ.get("VL_LEN", 1500))
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    data = torch.randint(0, 256, (n * L,), generator=g, device=dev, dtype=torch.uint8)
    offsets = torch.arange(0, n + 1, dtype=torch.int64, device=dev) * L
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    out = {"frames": n, "len": L}
    fixed = lambda: eng.crc_fixed(data, L, n=n, crc_out=crc, valid_out=valid)  # noqa: E731
    varlen = lambda: eng.crc_varlen(data, offsets, crc_out=crc, valid_out=valid)  # noqa: E731
    runs = (("fixed", fixed, {}), ("fixed_loads_only", fixed, {"UFC_LEAN_ABL": "1"}),
            ("varlen", varlen, {}), ("varlen_loads_only", varlen, {"UFC_VL_ABL": "1"}),
            ("varlen_compute_only", varlen, {"UFC_VL_ABL": "2"}))
    for name, fn, env in runs:
        os.environ.update(env)
        fn()
        torch.cuda.synchronize()
        ms = timed(fn, 20, s)
        for k in env:
            del os.environ[k]
        out[name] = round(ms, 4)
        print(name, round(ms, 4), "ms", round(n * L / ms / 1e-3 / 1e9, 1), "GB/s", flush=True)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
