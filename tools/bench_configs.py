"""Secondary measurements for DESIGN.md (BASELINE.json configs 3, 4-per-GPU and 5, the seal and the
parse), one JSON line each.  Not the driver's bench (bench.py is); run on the GPU box:
    python tools/bench_configs.py [--only varlen,shard,seal,seal_varlen,parse,parse_mtu,gate_tg,host] [--reps 20]

  varlen   config 3: 10M frames, lengths U[64,1500] (splitmix64, seed 0x5EED0002), CSR offsets,
           device-resident; every frame checked against the oracle; CPU baseline of the same loop
           (1 thread and all threads) on a sample.
  shard    config 4, one GPU's shard: frames [37.5M, 50M) of the 100M-frame batch (seed 0x5EED0003),
           18.75 GB device-resident (3 launches of the lean kernel).
  seal     the encode side of config 2: 1M x 1500-B frames sealed in place on the device.
  parse    Frame::read past the gate on the device (ufc_parse_batch_varlen): 1M real uflow frames from
           the reference's test generators (38 % longer than MAX_FRAME_SIZE).
  parse_mtu  the same with frames <= MAX_FRAME_SIZE only (what a uflow receiver gets).
  host     config 5's GPU leg: 1M x 1472-B frames (uflow's MAX_FRAME_SIZE) that start and end in
           host memory -> ufc_validate_host_varlen (H2D + CRC + D2H) from pinned and from pageable
           buffers; GiB/s of frame bytes including the copies.
Kernel times: HIP events around groups of 10 back-to-back launches on the current stream (median
over the groups of --reps launches); ceiling_GBs = ufc_hbm_read_probe (a plain read-only stream) over
the same buffer, timed the same way.
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

import oracle  # noqa: E402  (the checker and the CPU baseline only)
from uflow_amd import synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

PEAK = 8e12
CHECK = True  # --no-check: skip the oracle comparisons and CPU baselines


def timed(fn, reps, group=10):
    """HIP events around groups of `group` back-to-back launches on the current stream (as bench.py:
    an event pair around every launch adds ~6 us); returns (median, mean) ms per launch over the
    ceil(reps / group) groups."""
    s = torch.cuda.current_stream()
    ng = max(1, -(-reps // group))
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(ng)]
    for e0, e1 in evs:
        e0.record(s)
        for _ in range(group):
            fn()
        e1.record(s)
    torch.cuda.synchronize()
    t = [a.elapsed_time(b) / group for a, b in evs]
    return float(np.median(t)), float(np.mean(t))


def ceiling(eng, buf, reps):
    """Read-only streaming ceiling over the same bytes (ufc_hbm_read_probe): GB/s."""
    sink = torch.zeros(1, dtype=torch.int32, device=buf.device)
    nbytes = eng.hbm_read_probe(buf, sink)
    settle(lambda: eng.hbm_read_probe(buf, sink), 20)
    med, _ = timed(lambda: eng.hbm_read_probe(buf, sink), reps)
    return round(nbytes / med / 1e-3 / 1e9, 1)


def settle(fn, ms=1000):
    """Launches for `ms` before timing: a GPU out of idle runs at reduced clocks for up to ~1 s."""
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        fn()
        torch.cuda.synchronize()


def threads():
    """The process's effective CPU share (cgroup quota, else the box's declared share, never more
    than the affinity mask): bench.py's cpu_baseline rule."""
    from bench import effective_cpus
    return effective_cpus()[0]


def rates(name, nbytes, algo, med, mean, ceil_gbs=None, **kw):
    r = {"config": name, "kernel_ms": round(med, 4), "kernel_mean_ms": round(mean, 4),
         "GiB_s": round(nbytes / med / 1e-3 / 2**30, 1), "algo_GB_s": round(algo / med / 1e-3 / 1e9, 1),
         "hbm_frac": round(algo / med / 1e-3 / PEAK, 4), "algorithmic_bytes": algo}
    if ceil_gbs:
        r["ceiling_GBs"] = ceil_gbs
        r["frac_of_ceiling"] = round(algo / med / 1e-3 / 1e9 / ceil_gbs, 4)
    r.update(kw)
    return r


def varlen(eng, dev, reps, n=10_000_000):
    data, offsets = synth.varlen_batch(n, 64, 1500, synth.SEED_CONFIG3, device=dev)
    eng.seal_varlen(data, offsets)
    flipped = torch.arange(0, n, 997, device=dev)
    synth.flip_bits(data, offsets[flipped], byte_in_frame=7, mask=0x20)
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    fn = lambda: eng.crc_varlen(data, offsets, crc_out=crc, valid_out=valid)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    total = int(offsets[-1])
    settle(fn)
    med, mean = timed(fn, reps)
    ceil_gbs = ceiling(eng, data, reps)
    algo = total + 8 * (n + 1) + 4 * n + n
    # A/B: the generic kernel on the same batch (the same results, timed beside the product kernel)
    from uflow_amd import _native as N
    other = N.UFC_VARLEN_GENERIC
    saved = eng.get_option(N.UFC_OPT_VARLEN_KERNEL)
    eng.set_option(N.UFC_OPT_VARLEN_KERNEL, other)
    crc2 = torch.empty(n, dtype=torch.int32, device=dev)
    valid2 = torch.empty(n, dtype=torch.uint8, device=dev)
    fn2 = lambda: eng.crc_varlen(data, offsets, crc_out=crc2, valid_out=valid2)  # noqa: E731
    fn2()
    torch.cuda.synchronize()
    same = bool(torch.equal(crc, crc2) and torch.equal(valid, valid2))
    settle(fn2)
    med2, _ = timed(fn2, reps)
    eng.set_option(N.UFC_OPT_VARLEN_KERNEL, saved)
    ab = {"other_kernel": "generic",
          "other_kernel_ms": round(med2, 4),
          "other_equal_results": same}
    if not CHECK:
        return rates("3: varlen 10M x U[64,1500] device-resident (unchecked counter pass)", total, algo, med, mean,
                     ceil_gbs, frames=n, **ab)
    h_data, h_off = data.cpu().numpy(), offsets.cpu().numpy().astype(np.uint64)
    ref_crc, ref_valid = oracle.validate_varlen_mt(h_data, h_off, min(64, threads()))
    exact = bool(np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc) and
                 np.array_equal(valid.cpu().numpy(), ref_valid))
    # CPU baseline: the oracle's bytewise loop (crc.rs:94-100) on the first frames, 1 thread and all
    k1, kn = 50_000, min(n, 50_000 * threads())

    def cpu(k, t):
        o = h_off[: k + 1]
        t0 = time.perf_counter()
        oracle.validate_varlen_mt(h_data, o, t)
        return (int(o[-1]) - int(o[0])) / (time.perf_counter() - t0) / 2**30

    cpu1, cpun = cpu(k1, 1), cpu(kn, threads())
    return rates("3: varlen 10M x U[64,1500] device-resident", total, algo, med, mean, ceil_gbs, frames=n, bytes=total,
                 bit_exact_all_frames=exact, valid_count_ok=int(ref_valid.sum()) == n - flipped.numel(), **ab,
                 cpu_baseline={"unit": "GiB/s", "single_thread": round(cpu1, 4), "all_threads": round(cpun, 3),
                               "threads": threads(), "nproc": os.cpu_count(),
                               "sample": f"first {k1} frames on 1 thread, first {kn} frames on {threads()} threads"})


def shard(eng, dev, reps, world=8, rank=3, total=100_000_000, L=1500):
    lo, hi = total * rank // world, total * (rank + 1) // world
    n = hi - lo
    frames = synth.fixed_frames(n, L, synth.SEED_CONFIG4, first_frame=lo, device=dev)
    eng.seal_fixed(frames, L, n=n)
    frames[torch.arange(0, n, 1000, device=dev) * L + 3] ^= 1
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    fn = lambda: eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    ok = int(valid.sum()) == n - len(range(0, n, 1000))
    settle(fn)
    med, mean = timed(fn, reps)
    out = rates(f"4 (one GPU's shard): frames [{lo}, {hi}) of 100M x 1500 B, device-resident", n * L, n * L + 5 * n,
                med, mean, ceiling(eng, frames, reps), frames=n, valid_ok=ok)
    del frames
    torch.cuda.empty_cache()
    return out


def seal(eng, dev, reps, n=1_000_000, L=1500):
    """The encode side on config 2's batch: ufc_seal_batch_fixed writes every frame's BE32 trailer
    in place (reads 1500 B, writes 4 B per frame); checked by validating afterwards."""
    frames = synth.fixed_frames(n, L, synth.SEED_CONFIG2, device=dev)
    fn = lambda: eng.seal_fixed(frames, L, n=n)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    crc, valid = eng.crc_fixed(frames, L, n=n)
    ok = int(valid.sum()) == n
    settle(fn)
    med, mean = timed(fn, reps)
    # the round-3 shape for comparison: two passes (CRC words, then a non-temporal trailer pass)
    from uflow_amd import _native as N
    eng.set_option(N.UFC_OPT_SEAL_KERNEL, N.UFC_SEAL_TWO_PASS)
    try:
        settle(fn)
        med_two, _ = timed(fn, reps)
    finally:
        eng.set_option(N.UFC_OPT_SEAL_KERNEL, N.UFC_SEAL_INLINE)
    return rates("2 (encode side): seal 1M x 1500-B frames in place, device-resident (one kernel: each "
                 "workgroup's trailers after its reads, non-temporal)", n * L, n * L + 4 * n,
                 med, mean, ceiling(eng, frames, reps), frames=n, valid_after_seal=ok,
                 two_pass_seal_ms=round(med_two, 4))


def seal_varlen(eng, dev, reps, n=10_000_000):
    """The encode side on config 3's batch: ufc_seal_batch_varlen writes every frame's BE32
    trailer in place (from the CRC kernel: a separate trailer pass measured 1.961 against
    1.860 ms here, 10M scattered writes); checked by validating every frame afterwards."""
    data, offsets = synth.varlen_batch(n, 64, 1500, synth.SEED_CONFIG3, device=dev)
    fn = lambda: eng.seal_varlen(data, offsets)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    _, valid = eng.crc_varlen(data, offsets)
    ok = int(valid.sum()) == n
    settle(fn)
    med, mean = timed(fn, reps)
    total = int(offsets[-1])
    return rates("3 (encode side): seal 10M x U[64,1500] frames in place, CSR, device-resident",
                 total, total + 8 * (n + 1) + 4 * n, med, mean, ceiling(eng, data, reps), frames=n,
                 valid_after_seal=ok)


def parse_batch(n, mtu):
    """The parse workloads' batch (host arrays): 600 distinct frames from the codec oracle, tiled (see parse)."""
    import random
    from oracle import codec as C
    rng = random.Random(5)

    def fit(fr):  # (data frames: drop datagrams from the end until the frame fits)
        while mtu and fr["kind"] == "data" and fr["datagrams"] and len(C.frame_write(fr)) > C.MAX_FRAME_SIZE:
            fr["datagrams"].pop()
        return C.frame_write(fr)
    base = [fit(C.random_data_frame(rng) if i % 3 == 0 else C.receive_side_data_frame(rng)
                if i % 3 == 1 else C.random_ack_frame(rng, 20)) for i in range(600)]
    assert not mtu or max(len(f) for f in base) <= C.MAX_FRAME_SIZE
    lens = np.array([len(base[i % 600]) for i in range(n)], dtype=np.int64)
    offsets = np.zeros(n + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(base), dtype=np.uint8)
    data = np.concatenate([blob] * (n // 600 + 1))[: int(offsets[-1])]
    return data, offsets, lens


def gate_tg(eng, dev, reps, n=1_000_000):
    """The variable-length gate alone on the parse workload's test-generator batch (38 % of frames over
    13 lines: the first launch's byte path defers them to frame_crc_long8_kernel), every frame against
    the oracle; the generic kernel timed beside it."""
    data, offsets, lens = parse_batch(n, False)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(offsets).to(dev)
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    fn = lambda: eng.crc_varlen(d, o, crc_out=crc, valid_out=valid)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    settle(fn)
    med, mean = timed(fn, reps)
    total = int(offsets[-1])
    from uflow_amd import _native as N
    saved = eng.get_option(N.UFC_OPT_VARLEN_KERNEL)
    eng.set_option(N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_GENERIC)
    crc2 = torch.empty(n, dtype=torch.int32, device=dev)
    valid2 = torch.empty(n, dtype=torch.uint8, device=dev)
    fn2 = lambda: eng.crc_varlen(d, o, crc_out=crc2, valid_out=valid2)  # noqa: E731
    fn2()
    torch.cuda.synchronize()
    same = bool(torch.equal(crc, crc2) and torch.equal(valid, valid2))
    settle(fn2, 300)
    med2, _ = timed(fn2, reps)
    eng.set_option(N.UFC_OPT_VARLEN_KERNEL, saved)
    extra = {}
    if CHECK:
        ref_crc, ref_valid = oracle.validate_varlen_mt(data, offsets.astype(np.uint64), min(64, threads()))
        extra["bit_exact_all_frames"] = bool(np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc) and
                                             np.array_equal(valid.cpu().numpy(), ref_valid))
    return rates("gate on the parse test-generator batch (1M uflow frames, 38 % over 1532 B)", total,
                 total + 8 * (n + 1) + 5 * n, med, mean, None, frames=n, over_13_lines=float(np.mean(lens > 1532)),
                 other_kernel="generic", other_kernel_ms=round(med2, 4), other_equal_results=same, **extra)


def parse(eng, dev, reps, n=1_000_000, mtu=False):
    """ufc_parse_batch_varlen over n real uflow frames (data frames with datagrams, acks, syncs):
    600 distinct frames from the codec oracle, tiled.  The generators are the reference's test
    generators (random_data_frame, serial/mod.rs:932-992), which ignore the frame size limit: 38 % of
    these frames are longer than MAX_FRAME_SIZE (1472 B, src/lib.rs:291-294), up to 7.5 KB, and take
    the gate's byte path.  mtu=True keeps only frames a uflow receiver can get (<= MAX_FRAME_SIZE: the
    emitters' limit, half_connection/emit.rs:69, and the receive buffer, server/mod.rs:595): each data
    frame keeps the longest prefix of its datagrams that fits, as the emitter packs a frame until the
    next datagram would not fit (emit.rs:69)."""
    data, offsets, lens = parse_batch(n, mtu)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(offsets).to(dev)
    _, valid = eng.crc_varlen(d, o)
    infos, items, used = eng.parse_varlen(d, o, valid)
    torch.cuda.synchronize()
    cap = items.shape[0]
    fn = lambda: eng.parse_varlen(d, o, valid, items_cap=cap)  # noqa: E731
    settle(fn)
    med, mean = timed(fn, reps)
    total = int(offsets[-1])
    k = int(used.cpu()[0])
    # (a checksum of the item records and infos: equal across A/B variants)
    digest = int(items[:k].view(torch.int64).sum()) ^ int(infos.view(torch.int64).sum())
    # the gate and the parse back to back (Frame::read end to end: serial/mod.rs:675-706)
    crc = torch.empty(n, dtype=torch.int32, device=dev)

    def both():
        eng.crc_varlen(d, o, crc_out=crc, valid_out=valid)
        eng.parse_varlen(d, o, valid, items_cap=cap)
    settle(both, 300)
    med2, _ = timed(both, reps)
    # algorithmic bytes of the parse: the frame bytes read once, the offsets and
    # gate flags read, the 24-byte items and 32-byte infos written
    algo = total + 8 * (n + 1) + n + 24 * k + 32 * n
    return {"config": ("f3: device parse of 1M uflow frames <= MAX_FRAME_SIZE after the gate" if mtu else
                       "f3: device parse of 1M uflow frames after the gate (test generators, 38 % over MAX_FRAME_SIZE)"),
            "frames": n,
            "frame_bytes": total, "items": k, "items_digest": digest, "ms": round(med, 4), "mean_ms": round(mean, 4),
            "frames_per_s": round(n / med * 1e3), "GB_s_of_frame_bytes": round(total / med / 1e-3 / 1e9, 1),
            "algorithmic_bytes": algo, "frac_of_8TBs": round(algo / (med * 1e-3) / 8e12, 4),
            "gate_plus_parse_ms": round(med2, 4)}


def parse_mtu(eng, dev, reps):
    return parse(eng, dev, reps, mtu=True)


def host(eng, reps=5, n=1_000_000, L=1472):
    res = []
    for kind in ("pinned", "pageable"):
        t = torch.empty(n * L, dtype=torch.uint8, pin_memory=(kind == "pinned"))
        d = synth.fixed_frames(n, L, synth.SEED_CONFIG2, device="cuda")
        eng.seal_fixed(d, L, n=n)
        torch.cuda.synchronize()
        t.copy_(d.cpu())
        del d
        a = t.numpy()
        a[np.arange(0, n, 500) * L + 9] ^= 0x40
        offsets = (np.arange(n + 1, dtype=np.uint64) * L)
        lens = np.full(n, L, dtype=np.uint32)
        for entry, fn in (("ufc_validate_host_varlen (CSR)", lambda: eng.validate_host_varlen(a, offsets)),
                          ("ufc_validate_host_slots (recvmmsg slots, stride 1472)",
                           lambda: eng.validate_host_slots(a, L, lens))):
            fn()  # warm (staging allocation)
            times = []
            for _ in range(reps):
                t0 = time.perf_counter()
                crc, valid = fn()
                times.append(time.perf_counter() - t0)
            sec = float(np.median(times))
            ok = int(valid.sum()) == n - len(range(0, n, 500))
            res.append({"config": f"5 (GPU leg): host-resident {n} x {L}-B frames, {kind} buffer, H2D + CRC + D2H",
                        "entry": entry, "frames": n, "seconds": round(sec, 5), "GiB_s": round(n * L / sec / 2**30, 2),
                        "frames_per_s": round(n / sec), "valid_ok": ok})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--varlen-kernel", default="auto", choices=["auto", "sorted8"],
                    help="variable-length kernel of the timed runs (the other one is timed beside it)")
    ap.add_argument("--only", default="varlen,shard,seal,seal_varlen,parse,parse_mtu,host")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-check", action="store_true",
                    help="skip the oracle checks and CPU baselines (counter passes of tools/profile_workloads.sh)")
    a = ap.parse_args()
    global CHECK
    CHECK = not a.no_check
    dev = torch.device("cuda", 0)
    eng = FrameCrcEngine(0)
    from uflow_amd import _native as N
    eng.set_option(N.UFC_OPT_VARLEN_KERNEL, {"auto": N.UFC_VARLEN_AUTO, "sorted8": N.UFC_VARLEN_SORTED8}[a.varlen_kernel])
    for what in a.only.split(","):
        if what == "host":
            for r in host(eng):
                print(json.dumps(r), flush=True)
        else:
            print(json.dumps(globals()[what](eng, dev, a.reps)), flush=True)
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
