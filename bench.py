"""Benchmark: device-resident frame-CRC throughput (BASELINE.json metric) on 1..N MI355X.

One step = one pass of the batched CRC gate (CRC word + valid flag per frame) over frames already
resident in HBM:
  N = 1   config 2 (BASELINE.json configs[1]): 1M x 1500-B frames, ufc_crc_batch_fixed.
  N > 1   config 4 (configs[3]): 100M x 1500-B frames sharded over the N GPUs (100M / N each,
          strong scaling), ufc_crc_sharded = the gate on every rank's shard + the RCCL gather of
          every CRC word and valid flag into global frame order on rank 0.  --frames-per-gpu gives
          weak scaling instead.
Frames are splitmix64 of the global byte index (seed 0x5EED0001 / 0x5EED0003, uflow_amd/synth.py),
trailers sealed on the GPU, one bit flipped in every 1000th frame.  Results are checked against
the CPU oracle (N = 1: every frame; N > 1: the valid flags of every frame and a sample of every
rank's CRC words on rank 0); a mismatch makes the run fail.

Launch:  python bench.py [--gpus 1 --steps 50 --warmup 10]
         python bench.py --gpus N ...   (N > 1: starts its N ranks itself with torch.distributed.run,
                                         makes no GPU call, forwards rank 0's JSON line)
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
Rank 0 prints one JSON line.  --one-device puts every rank on cuda:0 (RCCL told the ranks are on
different hosts, NCCL_HOSTID, so it accepts them): a one-GPU rehearsal of the N > 1 send/recv path.
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
CONFIG4_FRAMES = 100_000_000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--frames-per-gpu", type=int, default=None,
                    help="weak scaling: frames per GPU (default: N = 1 -> 1M, config 2)")
    ap.add_argument("--global-frames", type=int, default=None,
                    help="strong scaling: frames of the whole batch (default: N > 1 -> 100M, config 4)")
    ap.add_argument("--frame-len", type=int, default=1500)
    ap.add_argument("--flip-every", type=int, default=1000)
    ap.add_argument("--settle-ms", type=float, default=1000.0,
                    help="untimed back-to-back launches before the warmup steps: a GPU coming out of idle "
                         "runs slower at first, and the first process on a fresh box still ran 4%% slower "
                         "after 50 ms (DESIGN.md section 6); the timed steps measure the sustained rate")
    ap.add_argument("--event-group", type=int, default=10,
                    help="HIP events around each group of k back-to-back timed gates (roofline.kernel_avg_ms = "
                         "group time / k; 1 = events around every gate, which adds ~6 us per step)")
    ap.add_argument("--sharded", action="store_true",
                    help="take the N > 1 path (ufc_crc_sharded over RCCL, gather to rank 0, sampled oracle check) "
                         "even at N = 1: a one-GPU rehearsal of the driver's multi-GPU run")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on cuda:0 (one-GPU rehearsal of the N > 1 path: RCCL over its socket "
                         "transport, each rank told it is on its own host via NCCL_HOSTID)")
    ap.add_argument("--fake-worker", action="store_true",
                    help="launcher test (CPU): each rank joins a gloo group and rank 0 prints the rank count")
    ap.add_argument("--no-ceiling", action="store_true", help="skip the read-only streaming ceiling probe")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="target wall time of each CPU baseline leg")
    ap.add_argument("--no-n1-ref", action="store_true",
                    help="N > 1: skip n1_sharded_ref (rank 0 alone gating the whole batch on its GPU)")
    return ap.parse_args()


class _StdoutToStderr:
    """fd 1 -> fd 2 for the duration (RCCL prints its version banner on stdout at communicator
    creation; the driver reads rank 0's stdout for the one JSON line)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def shard_of(total, rank, world):
    return total * rank // world, total * (rank + 1) // world


def make_frames(eng, first, n, L, seed, flip_every, dev):
    """Frames [first, first + n) of the global batch, sealed on the GPU, global frames
    0, flip_every, 2 flip_every, ... with one bit flipped (byte 17, mask 0x04)."""
    from uflow_amd import synth
    frames = synth.fixed_frames(n, L, seed, first_frame=first, device=dev)
    eng.seal_fixed(frames, L, n=n)
    if flip_every:
        g0 = (first + flip_every - 1) // flip_every * flip_every
        local = torch.arange(g0 - first, n, flip_every, device=dev, dtype=torch.int64)
        synth.flip_bits(frames, local * L)
    torch.cuda.synchronize(dev)
    return frames


def expected_valid(first, n, flip_every):
    v = np.ones(n, np.uint8)
    if flip_every:
        g0 = (first + flip_every - 1) // flip_every * flip_every
        v[np.arange(g0 - first, n, flip_every)] = 0
    return v


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


def affinity_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cgroup_cpu_quota():
    """The CPU bandwidth quota of this process's cgroup in CPUs (quota / period), or None if unlimited
    or unreadable: cgroup v2 cpu.max, else v1 cpu.cfs_quota_us / cpu.cfs_period_us."""
    rel = ""
    try:
        with open("/proc/self/cgroup") as f:
            for line in f:
                parts = line.strip().split(":", 2)
                if len(parts) == 3 and (parts[0] == "0" or "cpu" in parts[1].split(",")):
                    rel = parts[2]
                    if parts[0] == "0":
                        break
    except OSError:
        pass
    cands = []
    for d in ([os.path.join("/sys/fs/cgroup", rel.lstrip("/"))] if rel else []) + ["/sys/fs/cgroup"]:
        cands.append(("v2", os.path.join(d, "cpu.max"), None))
    for d in ([os.path.join("/sys/fs/cgroup/cpu", rel.lstrip("/"))] if rel else []) + ["/sys/fs/cgroup/cpu",
                                                                                       "/sys/fs/cgroup/cpu,cpuacct"]:
        cands.append(("v1", os.path.join(d, "cpu.cfs_quota_us"), os.path.join(d, "cpu.cfs_period_us")))
    for kind, qpath, ppath in cands:
        try:
            if kind == "v2":
                with open(qpath) as f:
                    q, p = f.read().split()[:2]
                if q == "max":
                    return None, qpath
                return int(q) / int(p), qpath
            with open(qpath) as f:
                q = int(f.read().strip())
            with open(ppath) as f:
                p = int(f.read().strip())
            return (None if q <= 0 else q / p), qpath
        except (OSError, ValueError):
            continue
    return None, None


def effective_cpus():
    """(threads to use, how they were chosen): the cgroup CPU quota if there is one, else the box's
    declared CPU share (OMP_NUM_THREADS, set to the per-GPU share on the GPU box), never more than the
    affinity mask."""
    aff = affinity_cpus()
    quota, qsrc = cgroup_cpu_quota()
    if quota is not None:
        return max(1, min(aff, int(quota))), f"cgroup quota {quota:g} CPUs ({qsrc})"
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        return min(aff, int(omp)), f"no cgroup quota; OMP_NUM_THREADS={omp} (the box's CPU share)"
    return aff, "no cgroup quota, no OMP_NUM_THREADS; affinity mask"


def cpu_baseline(host, n, L, target_s):
    """The oracle -- a C restatement of the reference's own loop, crc.rs:94-100 (one table load per
    byte) behind the gate of serial/mod.rs:675-690 -- on the host cores: one thread, then as many
    threads as the process's effective CPU share (cgroup quota, else the box's declared share, never
    more than the affinity mask), frames split contiguously; each leg on a bounded sample of config
    2's frames, repeated for about target_s seconds."""
    import oracle

    def leg(threads, sample):
        buf = host[: sample * L]
        t0 = time.perf_counter()
        oracle.validate_fixed_mt(buf, L, L, sample, threads)
        one = time.perf_counter() - t0
        reps = max(1, int(target_s / max(one, 1e-4)))
        t0 = time.perf_counter()
        for _ in range(reps):
            oracle.validate_fixed_mt(buf, L, L, sample, threads)
        dt = time.perf_counter() - t0
        return sample * L * reps / dt / 2**30, reps

    threads, how = effective_cpus()
    quota, _ = cgroup_cpu_quota()
    s1 = min(n, 20_000)
    v1, r1 = leg(1, s1)
    sn = min(n, max(s1, 20_000 * threads))
    vn, rn = leg(threads, sn)
    return {
        "value": round(vn, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "single_core_value": round(v1, 4), "nproc": os.cpu_count(), "affinity_cpus": affinity_cpus(),
        "effective_cpus": threads, "cgroup_quota_cpus": quota, "cores_source": how,
        "sample": f"config 2 frames (first of the batch): {s1} x {L} B x {r1} reps on 1 thread, {sn} x {L} B x "
                  f"{rn} reps on {threads} threads ({how}; affinity {affinity_cpus()} CPUs, os.cpu_count() = "
                  f"{os.cpu_count()}); bytewise table loop of crc.rs:94-100 in C (oracle/crc_oracle.c), "
                  f"frames split contiguously over the threads",
    }


def shard_reference(frames, n, L, threads, chunk=1 << 20):
    """The oracle's CRC words and valid flags of n fixed frames held on the device (uint8[n * L]),
    copied back and checked chunk by chunk."""
    import oracle
    ref_crc = np.empty(n, np.uint32)
    ref_valid = np.empty(n, np.uint8)
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        c, v = oracle.validate_fixed_mt(frames[c0 * L:(c0 + m) * L].cpu().numpy(), L, L, m, threads)
        ref_crc[c0:c0 + m] = c
        ref_valid[c0:c0 + m] = v
    return ref_crc, ref_valid


def split_result_line(line):
    """(text before, rank 0's JSON result) if the line holds the result object, else (line, None).  Ranks
    share the launcher's stdout, so another rank's unterminated print may precede the object on the same
    line: the object is looked for anywhere in the line."""
    k = line.find('{"metric"')
    if k >= 0:
        try:
            j = json.loads(line[k:])
        except ValueError:
            j = None
        if isinstance(j, dict) and "metric" in j:
            return line[:k], line[k:].strip()
    return line, None


def launch_ranks(a):
    """--gpus N > 1 without a launcher: run N ranks of this script under torch.distributed.run as a
    child process (this process makes no GPU call), forward rank 0's JSON line to stdout (other
    output to stderr) and return the launcher's exit code (non-zero if any rank failed)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print("bench: launching " + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=dict(os.environ))
    lines = []
    for line in p.stdout:
        before, obj = split_result_line(line)
        if obj is not None:
            if before:
                sys.stderr.write(before + "\n")
            lines.append(obj)
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = p.wait()
    for line in lines:
        print(line, flush=True)
    if rc == 0 and len(lines) != 1:
        print(f"bench: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 1
    return rc


def fake_worker(world, rank):
    """The launcher's CPU test: no GPU, one gloo all-reduce over the ranks."""
    dist.init_process_group("gloo")
    t = torch.ones(1)
    dist.all_reduce(t)
    print(f"rank {rank} of {world} alive", flush=True)  # non-JSON output is not forwarded as the line
    if rank == 0:
        print(json.dumps({"metric": "launcher test", "n_gpus": world, "ranks_seen": int(t.item()), "value": 0}),
              flush=True)
    dist.destroy_process_group()


def n1_sharded_reference(eng, total, L, seed, flip_every, dev, steps=5):
    """Config 4 at N = 1 on rank 0's GPU: the whole `total`-frame batch (or, when it does not fit beside
    this rank's shard, the largest multiple of 1M frames that does, said so) gated in one call of
    ufc_crc_batch_fixed -- what the N = 1 sharded path runs, since one rank has nothing to transfer --
    timed with HIP events over `steps` calls; valid flags checked against the planted flips."""
    free, _ = torch.cuda.mem_get_info(dev)
    fit = int(free * 0.85) // (L + 5) // 1_000_000 * 1_000_000
    n_ref = min(total, fit)
    if n_ref <= 0:
        return {"skipped": f"no room on rank 0's GPU ({free} B free)"}
    frames = make_frames(eng, 0, n_ref, L, seed, flip_every, dev)
    crc = torch.empty(n_ref, dtype=torch.int32, device=dev)
    valid = torch.empty(n_ref, dtype=torch.uint8, device=dev)
    eng.crc_fixed(frames, L, n=n_ref, crc_out=crc, valid_out=valid)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        eng.crc_fixed(frames, L, n=n_ref, crc_out=crc, valid_out=valid)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / steps
    ok = bool(np.array_equal(valid.cpu().numpy(), expected_valid(0, n_ref, flip_every)))
    del frames, crc, valid
    torch.cuda.empty_cache()
    return {"value": round(n_ref * L / (ms * 1e-3) / 2**30, 2), "unit": "GiB/s", "ms_per_step": round(ms, 4),
            "frames": n_ref, "whole_batch": n_ref == total, "valid_flags_as_planted": ok,
            "what": f"{n_ref} x {L}-B frames of the same batch gated by rank 0's GPU alone "
                    "(ufc_crc_batch_fixed: the N = 1 sharded path, nothing to transfer), HIP events over "
                    f"{steps} calls, after the timed region"}


def read_ceiling(eng, buf, stream, groups=5, per_group=10):
    """Plain read-only stream of buf (the gate's own frame buffer) timed like the gate: HIP events
    around groups of back-to-back launches.  Returns (GB/s, ms per launch, bytes per launch)."""
    sink = torch.zeros(1, dtype=torch.int32, device=buf.device)
    nbytes = eng.hbm_read_probe(buf, sink, stream=stream)
    for _ in range(20):
        eng.hbm_read_probe(buf, sink, stream=stream)
    ts = []
    for _ in range(groups):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(per_group):
            eng.hbm_read_probe(buf, sink, stream=stream)
        e1.record(stream)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / per_group)
    ms = float(np.mean(ts))
    return nbytes / (ms * 1e-3) / 1e9, ms, nbytes


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N > 1 with torch.distributed.run "
              f"--nproc-per-node {a.gpus}", file=sys.stderr)
        sys.exit(2)
    if a.fake_worker:
        return fake_worker(world, rank)
    sharded = world > 1 or a.sharded
    if sharded and world == 1:  # a one-rank group without a launcher
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29531"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
    if a.one_device:
        # RCCL refuses two ranks on one GPU of one host; ranks on "different hosts" talk over its
        # socket transport (loopback), which runs the same ncclSend/ncclRecv calls of ufc_crc_sharded.
        local = 0
        os.environ["NCCL_HOSTID"] = f"ufc-one-device-rank{rank}"
        # One hardware queue per rank: 8 processes x HIP's default 4 queues oversubscribe the GPU's queue
        # slots, and the scheduler then time-slices even idle queues (round 6: n1_sharded_ref 3980 GiB/s with
        # the default, 5919 with one queue per rank; the 8-rank step 108 against 61 ms).  (Before any HIP call.)
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "1")
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if sharded:
        with _StdoutToStderr():
            dist.init_process_group("nccl", device_id=dev)  # RCCL on ROCm: barriers and the timing max
            # A host-side group for waits that must not put RCCL kernels on the GPU (n1_sharded_ref)
            host_group = dist.new_group(backend="gloo") if world > 1 else None

    from uflow_amd import synth
    from uflow_amd.batch import FrameCrcEngine
    from uflow_amd.shard import ShardedGate, comm_id_create

    eng = FrameCrcEngine(local)
    L = a.frame_len
    if a.frames_per_gpu is not None:
        total, scaling = a.frames_per_gpu * world, "weak"
    elif a.global_frames is not None:
        total, scaling = a.global_frames, "strong"
    elif not sharded:
        total, scaling = 1_000_000, "weak"  # config 2
    else:
        total, scaling = CONFIG4_FRAMES, "strong"  # config 4
    seed = synth.SEED_CONFIG2 if not sharded else synth.SEED_CONFIG4
    lo, hi = shard_of(total, rank, world)
    n = hi - lo
    frames = make_frames(eng, lo, n, L, seed, a.flip_every, dev)

    gate = None
    if sharded:
        idt = torch.zeros(128, dtype=torch.uint8, device=dev)
        if rank == 0:
            idt.copy_(torch.frombuffer(bytearray(comm_id_create()), dtype=torch.uint8))
        with _StdoutToStderr():
            dist.broadcast(idt, src=0)
            gate = ShardedGate(eng, world, rank, bytes(idt.cpu().numpy()))
    # Outputs: two slots (step k writes slot k % 2 while the gather of step k - 1 may still read the
    # other); rank 0's slots hold the whole batch in global order.
    n_out = total if rank == 0 else n
    slots = [(torch.empty(n_out, dtype=torch.int32, device=dev), torch.empty(n_out, dtype=torch.uint8, device=dev))
             for _ in range(2 if sharded else 1)]
    compute = torch.cuda.current_stream(dev)
    gather = torch.cuda.Stream(dev) if sharded else None
    gathered = [None, None]  # event on the gather stream after each slot's last gather
    k_step = [0]
    tails = []  # N > 1, timed steps: (compute-stream end, gather-stream end) timing events per step
    host_call = []  # N > 1, timed steps: host seconds inside ufc_crc_sharded (its blocking status agreement)

    def step(ev=None, tail=None):
        i = k_step[0] % len(slots)
        k_step[0] += 1
        crc, valid = slots[i]
        if gathered[i] is not None:
            compute.wait_event(gathered[i])  # the slot's previous gather has finished with it
        if ev is not None and ev[0] is not None:
            ev[0].record(compute)
        if gate is None:
            eng.crc_fixed(frames, L, n=n, crc_out=crc, valid_out=valid)
        else:
            h0 = time.perf_counter()
            gate.crc_sharded(frames, L, total, crc, valid, root=0, stream=compute, gather_stream=gather)
            if tail is not None:
                host_call.append(time.perf_counter() - h0)
            e = torch.cuda.Event(enable_timing=tail is not None)
            e.record(gather)
            gathered[i] = e
            if tail is not None:
                c_end = torch.cuda.Event(enable_timing=True)
                c_end.record(compute)
                tail.append((c_end, e))
        if ev is not None and ev[1] is not None:
            ev[1].record(compute)
        return i

    # Settle: the gate alone (no collective), so ranks may run different numbers of iterations.
    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < a.settle_ms:
        eng.crc_fixed(frames, L, n=n, crc_out=slots[0][0][:n], valid_out=slots[0][1][:n])
        torch.cuda.synchronize(dev)
    for _ in range(a.warmup):
        step()
    # Events around groups of G consecutive gates (an event pair around every gate costs ~6 us per
    # step on the GPU: measured 0.2448-0.2456 against 0.2380-0.2387 ms per step with G = 10).
    G = max(1, a.event_group)
    groups = [(i, min(i + G, a.steps)) for i in range(0, a.steps, G)]
    gev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in groups]
    evs = [None] * a.steps
    for (g0, g1), (e0, e1) in zip(groups, gev):
        evs[g0] = (e0, None) if g1 - g0 > 1 else (e0, e1)
        if g1 - g0 > 1:
            evs[g1 - 1] = (None, e1)
    if sharded:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    last = 0
    for i in range(a.steps):
        last = step(evs[i], tails if sharded else None)
    torch.cuda.synchronize(dev)
    if sharded:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if sharded:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_all = np.array([e0.elapsed_time(e1) / (g1 - g0) for (g0, g1), (e0, e1) in zip(groups, gev)])
    kern_ms = float(np.mean(kern_all))
    # N > 1: every rank's gate time per step (compute stream) and how far its gather stream ran past
    # its last gate of the step (the transfer the gate did not hide), gathered to rank 0
    split = None
    if sharded:
        tail_ms = float(np.mean([max(0.0, c.elapsed_time(g)) for c, g in tails])) if tails else 0.0
        call_ms = float(np.mean(host_call)) * 1e3 if host_call else 0.0
        mine = torch.tensor([kern_ms, tail_ms, call_ms], dtype=torch.float64, device=dev)
        every = [torch.zeros(3, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(every, mine)
        split = [[float(x) for x in t.cpu()] for t in every]

    # ---- read-only streaming ceiling, after the timed region, on rank 0 ----
    ceiling = None
    if rank == 0 and not a.no_ceiling:
        ceiling = read_ceiling(eng, frames[: min(n, 1 << 22) * L], compute)

    # ---- correctness (after the timed region) ----
    crc, valid = slots[last]
    ok, parity = True, ""
    if not sharded:
        import oracle
        h_valid = valid.cpu().numpy()
        ok = bool(np.array_equal(h_valid, expected_valid(0, total, a.flip_every)))
        h_crc = crc.cpu().numpy().view(np.uint32)
        host = frames.cpu().numpy()
        ref_crc, ref_valid = oracle.validate_fixed_mt(host, L, L, n, effective_cpus()[0])
        exact = bool(np.array_equal(h_crc, ref_crc) and np.array_equal(h_valid, ref_valid))
        parity = f"every frame bit-exact vs the CPU oracle: {exact}"
        ok = ok and exact
    else:
        # Every CRC word that reached the root: each rank runs the oracle over its own shard's frames
        # (the bytes the gate read, copied back in chunks) and sends the words to the root, which
        # compares them with the gathered words at their global positions; every valid flag is
        # compared with the planted flips.
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        threads = max(1, effective_cpus()[0] // max(1, local_world))
        t_chk = time.perf_counter()
        ref_crc, ref_valid = shard_reference(frames, n, L, threads)
        local_ok = bool(np.array_equal(ref_valid, expected_valid(lo, n, a.flip_every)))
        exact = True
        if rank == 0:
            g_valid = valid.cpu().numpy()
            ok = bool(np.array_equal(g_valid, expected_valid(0, total, a.flip_every)))
            for r in range(world):
                rlo, rhi = shard_of(total, r, world)
                if r == 0:
                    ref_r = torch.from_numpy(ref_crc.view(np.int32)).to(dev)
                else:
                    ref_r = torch.empty(rhi - rlo, dtype=torch.int32, device=dev)
                    if rhi > rlo:
                        dist.recv(ref_r, src=r)
                exact = exact and bool(torch.equal(crc[rlo:rhi], ref_r))
        elif n > 0:
            dist.send(torch.from_numpy(ref_crc.view(np.int32)).to(dev), dst=0)
        flag = torch.tensor([0 if local_ok else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        all_local_ok = int(flag.item()) == 0
        parity = (f"all {total} CRC words gathered on rank 0 == the CPU oracle over every rank's shard: {exact}; "
                  f"oracle valid flags == planted flips on every rank: {all_local_ok} "
                  f"({time.perf_counter() - t_chk:.1f} s, {threads} threads per rank)")
        ok = ok and exact and all_local_ok

    # N > 1: config 4's batch gated by rank 0's GPU alone (the N = 1 point of the same workload, no
    # gather), after the timed region: the driver's 1 -> N curve then separates the gate's scaling from
    # the gather's cost and from the batch size.  The other ranks wait on the host (a gloo barrier), not
    # on an RCCL barrier: with --one-device the RCCL barrier's kernels would share rank 0's GPU while it
    # times the reference (2545 GiB/s there against 5940 alone).
    n1_ref = None
    if sharded and world > 1 and not a.no_n1_ref:
        torch.cuda.synchronize(dev)
        dist.barrier(group=host_group)  # every rank idle on the GPU before rank 0 starts timing
        if rank == 0:
            n1_ref = n1_sharded_reference(eng, total, L, seed, a.flip_every, dev)
        dist.barrier(group=host_group)

    result = None
    if rank == 0:
        algo_bytes = n * L + n * 4 + n * 1  # per launch group: frames read + crc words + valid bytes
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        traffic, tsrc = traffic_from_profile(n, L) if not sharded else (None, None)
        value = total * L / elapsed * a.steps / 2**30
        cfg_name = (f"config 2 (BASELINE.json configs[1]): {n} x {L}-B frames, fixed stride, device-resident"
                    if not sharded and total == 1_000_000 else
                    f"config 4 (BASELINE.json configs[3]): {total} x {L}-B frames sharded over {world} GPUs "
                    f"({n} per GPU on rank 0), RCCL gather of every CRC word + valid flag to rank 0 in global "
                    f"order (ufc_crc_sharded)" if total == CONFIG4_FRAMES else
                    f"{total} x {L}-B frames over {world} GPU(s)")
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
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: splitmix64 of the global byte index (seed {seed:#x}), BE CRC trailers sealed on "
                    f"the GPU, 1 bit flipped in every {a.flip_every}th frame; {parity}; valid flags as planted: {ok}",
            "config": {
                "workload": cfg_name,
                "frames_per_gpu": n, "frame_len": L, "global_frames": total,
                "parallelism": f"frame-sharded x{world}",
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": "ufc_dev::frame_crc_fixed_kernel<6, false, 2, 2, 8, 4224> (ufc_crc_batch_fixed"
                          + (", per chunk of ufc_crc_sharded" if sharded else "") + ")",
                "kernel_avg_ms": round(kern_ms, 4),
                "kernel_median_ms": round(float(np.median(kern_all)), 4),
                "kernel_min_ms": round(float(np.min(kern_all)), 4),
                "algorithmic_bytes_per_launch": algo_bytes,
                "timed_on": (f"HIP events on the compute stream around {len(groups)} group(s) of up to "
                             f"{min(G, a.steps)} back-to-back gates (per-launch average, inter-launch gaps "
                             "included)" if G > 1 else
                             "HIP events on the compute stream around each step's gate")
                            + (" (all chunks of this rank's shard)" if sharded else ""),
                **({"traffic_source": tsrc} if tsrc else {}),
            },
        }
        if split is not None:
            result["per_rank_kernel_ms"] = [round(x[0], 4) for x in split]
            result["gather_ms"] = [round(x[1], 4) for x in split]
            result["host_call_ms"] = [round(x[2], 4) for x in split]
            result["gather_ms_meaning"] = ("per rank and step: how long its gather stream ran past its last "
                                           "gate of the step (HIP events; the RCCL transfer the gates did not "
                                           "hide); per_rank_kernel_ms: that rank's gates per step; "
                                           "host_call_ms: host time per step inside ufc_crc_sharded, which "
                                           "blocks until every peer has joined the call's status agreement "
                                           "(the gates and transfers themselves are enqueued asynchronously)")
        if n1_ref is not None:
            result["n1_sharded_ref"] = n1_ref
        if ceiling is not None:
            gbs, probe_ms, probe_bytes = ceiling
            result["roofline"].update({
                "ceiling_GBs": round(gbs, 1), "frac_of_ceiling": round(achieved / gbs, 4),
                "ceiling_source": f"ufc_hbm_read_probe (hbm_probe.hip): a plain read-only stream of {probe_bytes} B "
                                  f"of the same frame buffer, 16 B per lane, 4 KiB per wave in flight, 8 waves per "
                                  f"CU; HIP events around 5 groups of 10 launches, {probe_ms:.4f} ms per launch"})
        if not a.no_cpu_baseline:
            if sharded:  # rank 0's own frames: a bounded sample of the same workload
                host = frames[: min(n, 1_000_000) * L].cpu().numpy()
            result["cpu_baseline"] = cpu_baseline(host, min(n, 1_000_000), L, a.cpu_seconds)
    if gate is not None:
        gate.close()
    if sharded:
        okt = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev)
        dist.broadcast(okt, src=0)
        ok = int(okt.item()) == 0
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if not ok:
        print(f"rank {rank}: results differ from the oracle / planted flips", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
