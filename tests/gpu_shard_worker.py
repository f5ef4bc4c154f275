"""One rank of tests/test_gpu_shard.py::test_ranks_on_one_device (one process per rank, started by the test).

Every rank sits on cuda:0 of the one-GPU test box.  RCCL refuses two ranks on one device of one
host, so each rank is told it is on a host of its own (NCCL_HOSTID) and RCCL connects them through
its socket transport over loopback: the N > 1 branch of ufc_crc_sharded / ufc_crc_sharded_varlen --
the ncclSend of every sender, the root's ncclRecv into global frame order, the chunk pipeline on a
separate gather stream -- runs for real, only over a slower wire than xGMI.  The root checks every
gathered CRC word and valid flag against the CPU oracle over the whole batch and prints one JSON line (the fixed batch's root is the last rank, the variable-length batch's rank 0).
Then a rank-local failure: the last rank passes no shard (NULL frames); every rank must return an
error (that rank UFC_ERR_INVALID_ARG, the others UFC_ERR_PEER) instead of hanging, and the next call
on the same communicator must succeed.

--peer-timeout (world 2): a peer that never makes the call.  Rank 1 creates the communicator and then
never calls ufc_crc_sharded; rank 0 calls it with a 3-s deadline (ufc_comm_set_timeout), must get
UFC_ERR_COMM within the deadline instead of hanging, then UFC_ERR_COMM at once from the stalled
communicator, prints what it saw and exits with status 3 (os._exit: the pending all-reduce is left to
process exit); rank 1 leaves once rank 0 has answered.

--late-peer (world 2): a peer that makes the call only after the other rank's deadline has
passed.  Rank 0 calls with a 3-s deadline and fails (UFC_ERR_COMM, stalled); only then does rank 1 call,
with a 3-s deadline of its own.  Its status round completes against rank 0's pending all-reduce, but the
commit round finds no partner, so rank 1 must fail with UFC_ERR_COMM at its deadline too, not go on to a
gather nobody answers.  Each rank then closes its communicator and its context (ufc_ctx_destroy must
return, not wait for the pending all-reduce) and reports how long that took; rank 0 stays alive until
rank 1 is done and prints both ranks' results.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
os.environ["NCCL_HOSTID"] = f"ufc-test-rank{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle  # noqa: E402
from uflow_amd import synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402
from uflow_amd.shard import ShardedGate, comm_id_create, shard_bounds_fixed, shard_bounds_varlen  # noqa: E402


def peer_timeout():
    from uflow_amd._native import UFC_ERR_COMM, NativeError
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    eng = FrameCrcEngine(0)
    idt = torch.zeros(128, dtype=torch.uint8, device=dev)
    if rank == 0:
        idt.copy_(torch.frombuffer(bytearray(comm_id_create()), dtype=torch.uint8))
    dist.broadcast(idt, src=0)
    gate = ShardedGate(eng, world, rank, bytes(idt.cpu().numpy()))
    torch.cuda.synchronize()
    flag = os.path.join("/tmp", "ufc_peer_timeout_%s.done" % os.environ["MASTER_PORT"])
    if rank != 0:  # the peer that never calls: wait for rank 0's verdict, then leave
        t0 = time.monotonic()
        while not os.path.exists(flag) and time.monotonic() - t0 < 90:
            time.sleep(0.1)
        os._exit(0)
    total, L = 100_000, 64
    b = shard_bounds_fixed(total, world)
    frames = synth.fixed_frames(int(b[1] - b[0]), L, synth.SEED_CONFIG4, device=dev)
    crc = torch.full((total,), -1, dtype=torch.int32, device=dev)
    gate.set_timeout(3000)
    codes = []
    t0 = time.monotonic()
    for _ in range(2):
        try:
            gate.crc_sharded(frames, L, total, crc, None, root=0)
            codes.append(0)
        except NativeError as e:
            codes.append(e.code)
        codes.append(round(time.monotonic() - t0, 3))
    print(json.dumps({"peer_timeout_codes": codes, "UFC_ERR_COMM": UFC_ERR_COMM}), flush=True)
    with open(flag, "w") as f:
        f.write("done")
    os._exit(3 if codes[0] == UFC_ERR_COMM else 4)


def late_peer():
    from uflow_amd._native import UFC_ERR_COMM, NativeError
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    eng = FrameCrcEngine(0)
    idt = torch.zeros(128, dtype=torch.uint8, device=dev)
    if rank == 0:
        idt.copy_(torch.frombuffer(bytearray(comm_id_create()), dtype=torch.uint8))
    dist.broadcast(idt, src=0)
    gate = ShardedGate(eng, world, rank, bytes(idt.cpu().numpy()))
    torch.cuda.synchronize()
    tag = os.environ["MASTER_PORT"]
    flag0 = os.path.join("/tmp", "ufc_late_peer_%s.r0" % tag)
    flag1 = os.path.join("/tmp", "ufc_late_peer_%s.r1" % tag)
    total, L = 100_000, 64
    b = shard_bounds_fixed(total, world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    frames = synth.fixed_frames(hi - lo, L, synth.SEED_CONFIG4, device=dev)
    crc = torch.full((total if rank == 0 else hi - lo,), -1, dtype=torch.int32, device=dev)
    gate.set_timeout(3000)

    def say(what):  # progress on stderr (the test prints each rank's stderr tail on a hang)
        print(f"[late_peer rank {rank} {time.monotonic():.2f}] {what}", file=sys.stderr, flush=True)

    say("comm ready")
    if rank == 1:  # late: only after rank 0 has given up
        t0 = time.monotonic()
        while not os.path.exists(flag0) and time.monotonic() - t0 < 90:
            time.sleep(0.05)
    say("calling crc_sharded")
    t0 = time.monotonic()
    try:
        gate.crc_sharded(frames, L, total, crc, None, root=0)
        code = 0
    except NativeError as e:
        code = e.code
    t_call = round(time.monotonic() - t0, 3)
    say(f"crc_sharded returned {code} after {t_call} s")
    t0 = time.monotonic()
    gate.close()
    say("communicator closed")
    eng.close()  # must return although an all-reduce is pending on the device
    t_close = round(time.monotonic() - t0, 3)
    say(f"context closed ({t_close} s)")
    mine = {"rank": rank, "code": code, "t_call": t_call, "t_close": t_close}
    if rank == 0:
        with open(flag0, "w") as f:
            f.write(json.dumps(mine))
        t0 = time.monotonic()
        while not os.path.exists(flag1) and time.monotonic() - t0 < 90:
            time.sleep(0.05)
        time.sleep(0.2)
        other = json.loads(open(flag1).read()) if os.path.exists(flag1) else None
        print(json.dumps({"late_peer": [mine, other], "UFC_ERR_COMM": UFC_ERR_COMM}), flush=True)
        os._exit(0)
    with open(flag1 + ".tmp", "w") as f:
        f.write(json.dumps(mine))
    os.replace(flag1 + ".tmp", flag1)
    os._exit(0)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    eng = FrameCrcEngine(0)
    idt = torch.zeros(128, dtype=torch.uint8, device=dev)
    if rank == 0:
        idt.copy_(torch.frombuffer(bytearray(comm_id_create()), dtype=torch.uint8))
    dist.broadcast(idt, src=0)
    gate = ShardedGate(eng, world, rank, bytes(idt.cpu().numpy()))
    gs = torch.cuda.Stream(dev)
    result = {"world": world, "rank": rank}

    # ---- fixed length: 9,000,001 x 64 B, more than 2^22 frames per shard at world 2 (2 chunks) ----
    total, L, root = 9_000_001, 64, world - 1
    b = shard_bounds_fixed(total, world)
    lo, hi = int(b[rank]), int(b[rank + 1])

    def fixed_batch(first, n):
        f = synth.fixed_frames(n, L, synth.SEED_CONFIG4, first_frame=first, device=dev)
        eng.seal_fixed(f, L, n=n)
        g0 = (first + 1012) // 1013 * 1013  # global frames 0, 1013, 2026, ... damaged
        synth.flip_bits(f, torch.arange(g0 - first, n, 1013, device=dev) * L, byte_in_frame=L // 2)
        return f

    frames = fixed_batch(lo, hi - lo)
    n_out = total if rank == root else hi - lo
    crc = torch.full((n_out,), -1, dtype=torch.int32, device=dev)
    valid = torch.full((n_out,), 7, dtype=torch.uint8, device=dev)
    gate.crc_sharded(frames, L, total, crc, valid, root=root, gather_stream=gs)
    torch.cuda.synchronize()
    if rank == root:
        host = fixed_batch(0, total).cpu().numpy()
        ref_crc, ref_valid = oracle.validate_fixed_mt(host, L, L, total, 32)
        result["fixed_crc_ok"] = bool(np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc))
        result["fixed_valid_ok"] = bool(np.array_equal(valid.cpu().numpy(), ref_valid))
        result["fixed_invalid"] = int(total - ref_valid.sum())
    del frames

    # ---- variable length: 1,500,001 x U[64, 1500] B, split by bytes, gathered to rank 0 ----
    total, root = 1_500_001, 0
    data, off = synth.varlen_batch(total, 64, 1500, synth.SEED_CONFIG3, device=dev)
    eng.seal_varlen(data, off)
    synth.flip_bits(data, off[:-1][::7], byte_in_frame=3)
    h_off = off.cpu().numpy()
    b = shard_bounds_varlen(h_off.view(np.uint64), world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    sdata = data[int(h_off[lo]):int(h_off[hi])].clone()  # this rank's bytes only
    soff = (off[lo:hi + 1] - off[lo]).contiguous()
    n_out = total if rank == root else hi - lo
    crc = torch.full((n_out,), -1, dtype=torch.int32, device=dev)
    valid = torch.full((n_out,), 7, dtype=torch.uint8, device=dev)
    gate.crc_sharded_varlen(sdata, soff, b, crc, valid, root=root, gather_stream=gs)
    torch.cuda.synchronize()
    if rank == root:
        ref_crc, ref_valid = oracle.validate_varlen_mt(data.cpu().numpy(), h_off.view(np.uint64), 32)
        result["varlen_crc_ok"] = bool(np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc))
        result["varlen_valid_ok"] = bool(np.array_equal(valid.cpu().numpy(), ref_valid))
        result["varlen_invalid"] = int(total - ref_valid.sum())
        result["varlen_bounds"] = [int(x) for x in b]

    # ---- a rank-local failure, agreed before any transfer ----
    from uflow_amd._native import NativeError
    total, L, root = 100_000, 64, 0
    b = shard_bounds_fixed(total, world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    frames = fixed_batch(lo, hi - lo)
    n_out = total if rank == root else hi - lo
    crc = torch.full((n_out,), -1, dtype=torch.int32, device=dev)
    bad = rank == world - 1
    try:
        gate.crc_sharded(None if bad else frames, L, total, crc, None, root=root, gather_stream=gs)
        code = 0
    except NativeError as e:
        code = e.code
    torch.cuda.synchronize()
    codes = torch.zeros(world, dtype=torch.int32, device=dev)
    codes[rank] = code
    dist.all_reduce(codes)
    gate.crc_sharded(frames, L, total, crc, None, root=root, gather_stream=gs)  # the comm still works
    torch.cuda.synchronize()
    if rank == root:
        host = fixed_batch(0, total).cpu().numpy()
        ref_crc, _ = oracle.validate_fixed_mt(host, L, L, total, 16)
        result["fail_codes"] = [int(x) for x in codes.cpu()]
        result["after_fail_crc_ok"] = bool(np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc))

    gate.close()
    dist.barrier()
    dist.destroy_process_group()
    eng.close()
    if len(result) > 2:  # the roots of the two gathers print what they checked
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    if "--peer-timeout" in sys.argv:
        peer_timeout()
    elif "--late-peer" in sys.argv:
        late_peer()
    else:
        main()
