"""long_gate.py -- the variable-length gate alone on the parse workloads (tools/bench_configs.py's
test-generator batch: 38 % of frames longer than 13 lines, which take the 8-lane kernel's byte path;
and the MTU-bounded batch), with the default kernel and with the generic one (UFC_VARLEN_GENERIC),
CRC words and flags compared.  Run on the GPU box: python tools/probes/long_gate.py"""
import os
import random
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from oracle import codec as C  # noqa: E402
from uflow_amd import _native as N  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402


def batch(n, mtu):
    rng = random.Random(5)

    def fit(fr):
        while mtu and fr["kind"] == "data" and fr["datagrams"] and len(C.frame_write(fr)) > C.MAX_FRAME_SIZE:
            fr["datagrams"].pop()
        return C.frame_write(fr)
    base = [fit(C.random_data_frame(rng) if i % 3 == 0 else C.receive_side_data_frame(rng)
                if i % 3 == 1 else C.random_ack_frame(rng, 20)) for i in range(600)]
    lens = np.array([len(base[i % 600]) for i in range(n)], dtype=np.int64)
    offsets = np.zeros(n + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(base), dtype=np.uint8)
    data = np.concatenate([blob] * (n // 600 + 1))[: int(offsets[-1])]
    return data, offsets, lens


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    eng = FrameCrcEngine(0)
    dev = torch.device("cuda", 0)
    for mtu in (False, True):
        data, offsets, lens = batch(1_000_000, mtu)
        d = torch.from_numpy(data).to(dev)
        o = torch.from_numpy(offsets).to(dev)
        out = {}
        for name, opt in (("sorted8", N.UFC_VARLEN_AUTO), ("generic", N.UFC_VARLEN_GENERIC)):
            eng.set_option(N.UFC_OPT_VARLEN_KERNEL, opt)
            crc = torch.empty(len(lens), dtype=torch.int32, device=dev)
            valid = torch.empty(len(lens), dtype=torch.uint8, device=dev)
            fn = lambda: eng.crc_varlen(d, o, crc_out=crc, valid_out=valid)  # noqa: E731
            for _ in range(200):
                fn()
            ms = timed(fn, 30)
            out[name] = (ms, crc.clone(), valid.clone())
        eng.set_option(N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_AUTO)
        same = bool(torch.equal(out["sorted8"][1], out["generic"][1]) and torch.equal(out["sorted8"][2], out["generic"][2]))
        long_frac = float((lens > 1532).mean())
        print(f"{'mtu' if mtu else 'test generators'}: {len(lens)} frames, {int(offsets[-1]) / 1e9:.3f} GB, "
              f"{long_frac:.3f} over 1532 B; sorted8 {out['sorted8'][0]:.4f} ms, generic {out['generic'][0]:.4f} ms; "
              f"identical {same}", flush=True)


if __name__ == "__main__":
    main()
