"""Probe: back-to-back batches on one stream vs alternating over S streams (tuning tool).

A launch of the fixed kernel leaves the chip partly idle at both ends (≈7 µs before the first
loads return, ≈5-9 µs of per-XCD finish spread).  Consecutive batches of a
receive loop are independent; on S streams batch k+1's workgroups take the CUs batch k's
finished ones free.  Prints, per mode, the per-batch time (events around groups of G batches).

    python tools/probes/overlap_streams.py [--kinds fixed,seal,varlen] [--streams 1,2,3]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def run(kind, eng, args_for, nstreams, groups, G):
    dev = eng.device
    cur = torch.cuda.current_stream(dev)
    streams = [cur] + [torch.cuda.Stream(dev) for _ in range(nstreams - 1)]
    outs = [args_for(i) for i in range(nstreams)]
    times = []
    for g in range(groups + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        for s in streams[1:]:
            s.wait_event(e0)
        for k in range(G):
            i = k % nstreams
            outs[i](streams[i])
        for s in streams[1:]:
            e = torch.cuda.Event()
            e.record(s)
            cur.wait_event(e)
        e1.record(cur)
        torch.cuda.synchronize(dev)
        if g >= 2:
            times.append(e0.elapsed_time(e1) / G)
    return float(np.median(times)), float(np.min(times))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="fixed,seal,varlen")
    ap.add_argument("--streams", default="1,2,3")
    ap.add_argument("--groups", type=int, default=3)
    ap.add_argument("--G", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from uflow_amd import synth
    from uflow_amd.batch import FrameCrcEngine
    dev = torch.device("cuda", 0)
    eng = FrameCrcEngine(0)
    L, n = 1500, 1_000_000
    frames = synth.fixed_frames(n, L, synth.SEED_CONFIG2, device=dev)
    eng.seal_fixed(frames, L, n=n)
    torch.cuda.synchronize(dev)
    ns = [int(x) for x in a.streams.split(",")]
    res = {}
    for kind in a.kinds.split(","):
        if kind == "fixed":
            def args_for(i):
                c = torch.empty(n, dtype=torch.int32, device=dev)
                v = torch.empty(n, dtype=torch.uint8, device=dev)
                return lambda s: eng.crc_fixed(frames, L, n=n, crc_out=c, valid_out=v, stream=s)
            nbytes = n * (L + 5)
        elif kind == "seal":
            def args_for(i):
                c = torch.empty(n, dtype=torch.int32, device=dev)
                return lambda s: eng.seal_fixed(frames, L, n=n, crc_out=c, stream=s)
            nbytes = n * (L + 4)
        else:
            data, offsets = synth.varlen_batch(10_000_000, 64, 1500, synth.SEED_CONFIG3, device=dev)
            eng.seal_varlen(data, offsets)

            def args_for(i):
                c = torch.empty(10_000_000, dtype=torch.int32, device=dev)
                v = torch.empty(10_000_000, dtype=torch.uint8, device=dev)
                return lambda s: eng.crc_varlen(data, offsets, crc_out=c, valid_out=v, stream=s)
            nbytes = data.numel() + 10_000_000 * (8 + 5)
        for S in ns:
            run(kind, eng, args_for, S, 3, a.G)  # warm (and settle the clocks)
        acc = {S: [] for S in ns}
        for r in range(a.rounds):  # modes interleaved, so drifts hit them alike
            for S in ns:
                acc[S].append(run(kind, eng, args_for, S, a.groups, a.G)[0])
        for S in ns:
            med, mn = float(np.median(acc[S])), float(np.min(acc[S]))
            res[f"{kind}_s{S}"] = {"ms": round(med, 4), "min_ms": round(mn, 4),
                                  "frac": round(nbytes / (med * 1e-3) / 8e12, 4)}
            print(json.dumps({kind: S, **res[f"{kind}_s{S}"]}), flush=True)
        if kind == "varlen":
            del data, offsets
    eng.close()


if __name__ == "__main__":
    main()
