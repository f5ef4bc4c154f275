"""Secondary measurements for DESIGN.md (BASELINE.json configs 3, 4-per-GPU and 5), one JSON line
each.  Not the driver's bench (bench.py is); run on the GPU box:  python tools/bench_configs.py

  varlen   config 3: 10M frames, lengths U[64,1500] (seed 0x5EED0002), CSR offsets, device-resident;
           GiB/s on the sum of frame lengths, kernel time from HIP events.
  shard    config 4, one GPU's shard: 12.5M x 1500-B frames (18.75 GB) device-resident (the
           batch spans several launches of the lean kernel).
  seal     the encode side of config 2: 1M x 1500-B frames sealed in place on the device.
  host     config 5's GPU leg: 1M x 1472-B frames (uflow's MAX_FRAME_SIZE) that start and end in
           host memory -> ufc_validate_host_varlen (H2D + CRC + D2H) from pinned and from pageable
           buffers; GiB/s of frame bytes including the copies.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from uflow_amd.batch import FrameCrcEngine  # noqa: E402


def timed(fn, reps, stream):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in evs:
        e0.record(stream)
        fn()
        e1.record(stream)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


def varlen(eng, dev, n=10_000_000, reps=20):
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0002)
    lens = torch.randint(64, 1501, (n,), generator=g, device=dev, dtype=torch.int64)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    offsets[1:] = torch.cumsum(lens, 0)
    total = int(offsets[-1])
    data = torch.randint(0, 256, (total,), generator=g, device=dev, dtype=torch.uint8)
    eng.seal_varlen(data, offsets)
    data[offsets[:-1:997] + 7] ^= 0x20  # flip one bit in every 997th frame
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    fn = lambda: eng.crc_varlen(data, offsets, crc_out=crc, valid_out=valid)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    expect = n - len(range(0, n, 997))
    ok = int(valid.sum()) == expect
    # bit-exact check of a sample (the first 200k frames) against the CPU oracle
    import oracle
    k = 200_000
    off_h = offsets[: k + 1].cpu().numpy().astype(np.uint64)
    ref_crc, ref_valid = oracle.validate_varlen(data[: int(off_h[-1])].cpu().numpy(), off_h)
    exact = bool(np.array_equal(crc[:k].cpu().numpy().view(np.uint32), ref_crc) and
                 np.array_equal(valid[:k].cpu().numpy(), ref_valid))
    ms = timed(fn, reps, s)
    os.environ["UFC_VARLEN_KERNEL"] = "generic"  # A/B: the generic kernel on the same batch
    ms_generic = timed(fn, reps, s)
    del os.environ["UFC_VARLEN_KERNEL"]
    algo = total + 8 * (n + 1) + 4 * n + n
    return {"config": "3: varlen 10M x U[64,1500] device-resident", "frames": n, "bytes": total,
            "kernel_ms": round(ms, 4), "GiB_s": round(total / ms / 1e-3 / 2**30, 1),
            "algo_GB_s": round(algo / ms / 1e-3 / 1e9, 1), "hbm_frac": round(algo / ms / 1e-3 / 8e12, 4),
            "valid_ok": ok, "sample_bit_exact": exact, "generic_kernel_ms": round(ms_generic, 4)}


def shard(eng, dev, n=12_500_000, L=1500, reps=10):
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0003)
    frames = torch.randint(0, 256, (n * L,), generator=g, device=dev, dtype=torch.uint8)
    eng.seal_fixed(frames, L, n=n)
    frames[torch.arange(0, n, 1000, device=dev) * L + 3] ^= 1
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    fn = lambda: eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    ok = int(valid.sum()) == n - len(range(0, n, 1000))
    ms = timed(fn, reps, torch.cuda.current_stream())
    algo = n * L + 5 * n
    out = {"config": "4 (one GPU's shard): 12.5M x 1500-B device-resident", "frames": n,
           "kernel_ms": round(ms, 4), "GiB_s": round(n * L / ms / 1e-3 / 2**30, 1),
           "algo_GB_s": round(algo / ms / 1e-3 / 1e9, 1), "hbm_frac": round(algo / ms / 1e-3 / 8e12, 4),
           "valid_ok": ok}
    del frames
    torch.cuda.empty_cache()
    return out


def seal(eng, dev, n=1_000_000, L=1500, reps=20):
    """The encode side on config 2's batch: ufc_seal_batch_fixed writes every frame's BE32
    trailer in place (reads 1500 B, writes 4 B per frame); checked by validating afterwards."""
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0004)
    frames = torch.randint(0, 256, (n * L,), generator=g, device=dev, dtype=torch.uint8)
    fn = lambda: eng.seal_fixed(frames, L, n=n)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    crc, valid = eng.crc_fixed(frames, L, n=n)
    ok = int(valid.sum()) == n
    ms = timed(fn, reps, torch.cuda.current_stream())
    algo = n * L + 4 * n
    return {"config": "2 (encode side): seal 1M x 1500-B frames in place, device-resident", "frames": n,
            "kernel_ms": round(ms, 4), "GiB_s": round(n * L / ms / 1e-3 / 2**30, 1),
            "algo_GB_s": round(algo / ms / 1e-3 / 1e9, 1), "hbm_frac": round(algo / ms / 1e-3 / 8e12, 4),
            "valid_after_seal": ok}


def host(eng, n=1_000_000, L=1472, reps=5):
    rng = np.random.default_rng(5)
    res = []
    for kind in ("pinned", "pageable"):
        t = torch.empty(n * L, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        a = t.numpy()
        a[:] = rng.integers(0, 256, size=n * L, dtype=np.uint8)
        offsets = (np.arange(n + 1, dtype=np.uint64) * L)
        # seal on the device (fast), copy back: the host buffer then holds valid frames
        d = t.to("cuda")
        eng.seal_fixed(d, L, n=n)
        torch.cuda.synchronize()
        t.copy_(d.cpu())
        del d
        a[np.arange(0, n, 500) * L + 9] ^= 0x40
        eng.validate_host_varlen(a, offsets)  # warm (staging allocation)
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            crc, valid = eng.validate_host_varlen(a, offsets)
            times.append(time.perf_counter() - t0)
        sec = float(np.median(times))
        ok = int(valid.sum()) == n - len(range(0, n, 500))
        res.append({"config": f"5 (GPU leg): host-resident {n} x {L}-B frames, {kind} buffer, H2D + CRC + D2H",
                    "frames": n, "seconds": round(sec, 5), "GiB_s": round(n * L / sec / 2**30, 2),
                    "frames_per_s": round(n / sec), "valid_ok": ok})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="varlen,shard,seal,host")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = FrameCrcEngine(0)
    out = []
    if "varlen" in a.only:
        out.append(varlen(eng, dev))
        print(json.dumps(out[-1]), flush=True)
        torch.cuda.empty_cache()
    if "shard" in a.only:
        out.append(shard(eng, dev))
        print(json.dumps(out[-1]), flush=True)
    if "seal" in a.only:
        out.append(seal(eng, dev))
        print(json.dumps(out[-1]), flush=True)
        torch.cuda.empty_cache()
    if "host" in a.only:
        for r in host(eng):
            out.append(r)
            print(json.dumps(r), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
