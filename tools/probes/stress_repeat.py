"""stress_repeat.py -- the product kernels run many times on one batch, every launch's outputs compared
with the first launch's (a nondeterministic wrong result, like round 4's 16-byte parse walk, shows
as a mismatch): config 3's gate (10M frames, N_GATE launches), config 2's gate (1M x 1500 B), and the
parse of 1M uflow frames (item records and infos).  Run on the GPU box:
python tools/probes/stress_repeat.py [N_GATE]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from uflow_amd import synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402


def main():
    n_gate = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    eng = FrameCrcEngine(0)
    dev = torch.device("cuda", 0)
    bad = 0
    # config 3
    data, offsets = synth.varlen_batch(10_000_000, 64, 1500, synth.SEED_CONFIG3, device=dev)
    n = offsets.numel() - 1
    eng.seal_varlen(data, offsets)
    c0, v0 = eng.crc_varlen(data, offsets)
    torch.cuda.synchronize()
    ok0 = int(v0.sum())
    crc = torch.empty_like(c0)
    val = torch.empty_like(v0)
    for i in range(n_gate):
        eng.crc_varlen(data, offsets, crc_out=crc, valid_out=val)
        if not (torch.equal(crc, c0) and torch.equal(val, v0)):
            bad += 1
            print(f"config 3 launch {i}: mismatch", flush=True)
        if i % 100 == 0:
            print(f"config 3: {i} launches, {bad} mismatches", flush=True)
    print(f"config 3: {n_gate} launches of {n} frames ({ok0} valid), {bad} mismatching", flush=True)
    del data, offsets
    # config 2
    frames = synth.fixed_frames(1_000_000, 1500, synth.SEED_CONFIG2, device=dev)
    eng.seal_fixed(frames, 1500, n=1_000_000)
    f0, g0 = eng.crc_fixed(frames, 1500, n=1_000_000)
    torch.cuda.synchronize()
    b2 = 0
    for i in range(4 * n_gate):
        f1, g1 = eng.crc_fixed(frames, 1500, n=1_000_000)
        if not (torch.equal(f1, f0) and torch.equal(g1, g0)):
            b2 += 1
            print(f"config 2 launch {i}: mismatch", flush=True)
    print(f"config 2: {4 * n_gate} launches, {b2} mismatching; all valid: {int(g0.sum()) == 1_000_000}", flush=True)
    del frames
    # parse
    from oracle import codec as C  # (the input frames only, as tools/bench_configs.py builds them)
    import random
    rng = random.Random(5)
    base = [C.frame_write(C.random_data_frame(rng) if i % 3 == 0 else C.receive_side_data_frame(rng)
                          if i % 3 == 1 else C.random_ack_frame(rng, 20)) for i in range(600)]
    nf = 1_000_000
    lens = np.array([len(base[i % 600]) for i in range(nf)], dtype=np.int64)
    offs = np.zeros(nf + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(base), dtype=np.uint8)
    d = torch.from_numpy(np.concatenate([blob] * (nf // 600 + 1))[: int(offs[-1])]).to(dev)
    o = torch.from_numpy(offs).to(dev)
    _, valid = eng.crc_varlen(d, o)
    infos0, items0, used0 = eng.parse_varlen(d, o, valid)
    torch.cuda.synchronize()
    k0 = int(used0.cpu()[0])
    i0 = items0[:k0].clone()
    inf0 = infos0.clone()
    b3 = 0
    for i in range(n_gate // 2):
        infos, items, used = eng.parse_varlen(d, o, valid, items_cap=items0.shape[0])
        k = int(used.cpu()[0])
        if k != k0 or not (torch.equal(items[:k], i0) and torch.equal(infos, inf0)):
            b3 += 1
            print(f"parse launch {i}: mismatch", flush=True)
    print(f"parse: {n_gate // 2} launches, {k0} items, {b3} mismatching", flush=True)
    sys.exit(1 if (bad or b2 or b3) else 0)


if __name__ == "__main__":
    main()
