"""Benchmark: device-resident frame-CRC throughput (BASELINE.json metric) on 1..N MI355X.

One step = one pass of the batched CRC gate (crc + valid per frame, ufc_crc_batch_fixed) over
this rank's shard of synthetic 1500-byte frames already resident in HBM, plus -- for N > 1 --
the RCCL gather of the CRC words and valid flags to rank 0.  Weak scaling: every rank holds
--frames-per-gpu frames (default 1M = config 2 of BASELINE.json at N=1).

Launch:  python bench.py [--gpus 1 --steps 50 --warmup 10]
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md "HBM3E peak BW")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--frames-per-gpu", type=int, default=1_000_000)
    ap.add_argument("--frame-len", type=int, default=1500)
    ap.add_argument("--flip-every", type=int, default=1000)
    ap.add_argument("--settle-ms", type=float, default=50.0,
                    help="untimed back-to-back launches before the warmup steps: the clocks of a GPU "
                         "coming out of idle step through a transient (kernels ~15%% slower for ~5 ms, "
                         "DESIGN.md section 6); the timed steps measure the sustained rate")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU work of the baseline leg")
    return ap.parse_args()


def make_frames(engine, n, frame_len, rank, flip_every, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0001 + rank)
    frames = torch.randint(0, 256, (n * frame_len,), dtype=torch.uint8, device=dev, generator=g)
    engine.seal_fixed(frames, frame_len, n=n)  # valid BE trailers
    if flip_every:
        idx = torch.arange(0, n, flip_every, device=dev, dtype=torch.int64) * frame_len + 17
        frames[idx] ^= 0x04  # one flipped bit per flipped frame -> valid must be 0
    torch.cuda.synchronize(dev)
    return frames


def traffic_from_profile(frames, frame_len):
    """HBM bytes per launch from the committed PMC summary (profiles/pmc_traffic.json), if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            j = json.load(f)
        if j.get("frames") == frames and j.get("frame_len") == frame_len:
            return j.get("hbm_bytes_per_launch"), j.get("source")
    except (OSError, ValueError):
        pass
    return None, None


def cpu_baseline(frames_dev, n, frame_len, crc_dev, valid_dev, target_cpu_s):
    """The oracle (C restatement of crc.rs:94-100, bytewise) on a bounded sample of the same
    frames, frames split contiguously over T threads; checked against the GPU results."""
    import oracle
    sample = min(n, 200_000)
    host = frames_dev[: sample * frame_len].cpu().numpy()
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    t0 = time.perf_counter()
    crc, valid = oracle.validate_fixed_mt(host, frame_len, frame_len, sample, threads)
    t1 = time.perf_counter()
    reps = max(1, int(target_cpu_s / max(threads * (t1 - t0), 1e-3)))
    t2 = time.perf_counter()
    for _ in range(reps):
        oracle.validate_fixed_mt(host, frame_len, frame_len, sample, threads)
    t3 = time.perf_counter()
    gcrc = crc_dev[:sample].cpu().numpy().view(np.uint32)
    gval = valid_dev[:sample].cpu().numpy()
    parity = bool(np.array_equal(gcrc, crc) and np.array_equal(gval, valid))
    gib = sample * frame_len * reps / (t3 - t2) / 2**30
    return {
        "value": round(gib, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
        "sample": f"{sample} x {frame_len}-B frames (first frames of rank 0's shard) x {reps} reps, "
                  f"bytewise table loop of crc.rs:94-100 in C (oracle/crc_oracle.c), frames split over "
                  f"{threads} threads; results bit-equal to the GPU: {parity}",
    }


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            print(f"--gpus {a.gpus} needs torch.distributed.run with {a.gpus} processes", file=sys.stderr)
            sys.exit(2)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)  # RCCL on ROCm

    from uflow_amd.batch import FrameCrcEngine
    from uflow_amd.shard import ShardGatherer

    eng = FrameCrcEngine(local)
    n, L = a.frames_per_gpu, a.frame_len
    total = n * world
    frames = make_frames(eng, n, L, rank, a.flip_every, dev)
    # N > 1: the kernel writes into a ShardGatherer slot and the slot's RCCL gather to rank 0 runs
    # asynchronously, overlapping the next step's kernel (two slots, nothing allocated per step).
    gat = ShardGatherer(n, dev) if world > 1 else None
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    k_step = [0]

    def step(ev=None):
        i = k_step[0] % 2
        k_step[0] += 1
        c_out, v_out = crc, valid
        if gat is not None:
            gat.wait(i)  # the slot's previous gather has finished reading it
            c_out, v_out = gat.outputs(i)
        if ev is not None:
            ev[0].record()
        eng.crc_fixed(frames, L, n=n, crc_out=c_out, valid_out=v_out)
        if ev is not None:
            ev[1].record()
        if gat is not None:
            gat.start(i)
        return i

    # Settle: kernel only (no gather), so that ranks may run different numbers of iterations
    # without mismatching their collectives.
    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < a.settle_ms:
        eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid)
        torch.cuda.synchronize(dev)
    for _ in range(a.warmup):
        step()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    last = 0
    for i in range(a.steps):
        last = step(evs[i])
    if gat is not None:
        gat.wait_all()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_all = np.array([e0.elapsed_time(e1) for e0, e1 in evs])
    kern_ms = float(np.mean(kern_all))

    # correctness of this rank's shard: every flip_every-th frame invalid, all others valid; on
    # rank 0 for N > 1 also the gathered flags of every rank
    if gat is not None:
        crc, valid = gat.outputs(last)
    nvalid = int(valid.sum().item())
    expect = n - ((n + a.flip_every - 1) // a.flip_every if a.flip_every else 0)
    ok = nvalid == expect
    if gat is not None and rank == 0:
        g_crc, g_valid = gat.gathered(last)
        ok = ok and int(g_valid.sum().item()) == world * expect and bool(torch.equal(g_crc[:n], crc))

    result = None
    if rank == 0:
        algo_bytes = n * L + n * 4 + n * 1  # frames read + crc words + valid bytes, per launch
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        traffic, tsrc = traffic_from_profile(n, L)
        value = total * L / elapsed * a.steps / 2**30
        result = {
            "metric": "device-resident frame-CRC GiB/s (1500-B frames, validate: crc+valid per frame)",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "settle_ms": a.settle_ms,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: torch Philox random bytes (seed 0x5EED0001+rank), BE CRC trailers sealed on "
                    f"device, 1 bit flipped in every {a.flip_every}th frame; valid flags checked"
                    f"{' (and the gathered flags of every rank)' if world > 1 else ''}: {ok}",
            "config": {
                "workload": f"config 2 (BASELINE.json configs[1]) per GPU: {n} x {L}-B frames, fixed stride, "
                            f"device-resident; N>1: frame-sharded (weak), RCCL gather of CRC words + valid to rank 0 "
                            f"each step (async, overlapping the next step's kernel)",
                "frames_per_gpu": n, "frame_len": L, "global_frames": total,
                "parallelism": f"frame-sharded x{world}",
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": "ufc_dev::frame_crc_fixed_kernel<6, false, 2, 0, 2, 8> (ufc_crc_batch_fixed)",
                "kernel_avg_ms": round(kern_ms, 4),
                "kernel_median_ms": round(float(np.median(kern_all)), 4),
                "kernel_min_ms": round(float(np.min(kern_all)), 4),
                "algorithmic_bytes_per_launch": algo_bytes,
                **({"traffic_source": tsrc} if tsrc else {}),
            },
        }
        if world == 1 and not a.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(frames, n, L, crc, valid, a.cpu_seconds)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if not ok:
        print(f"rank {rank}: valid count {nvalid} != expected {expect}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
