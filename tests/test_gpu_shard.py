"""GPU: the multi-GPU C ABI (ufc_comm_create + ufc_crc_sharded / ufc_crc_sharded_varlen over RCCL).

- World size 1 in this process: the RCCL communicator is created through the library's own
  binding, the shard is gated chunk by chunk (front-readable chunks after the first), results land
  in their global positions, and every frame matches the oracle.
- World sizes 2 and 3 on the one GPU of the test box (tests/gpu_shard_worker.py, one process per
  rank, env:// rendezvous): RCCL's socket transport stands in for xGMI, so the senders' ncclSend and
  the root's ncclRecv into global frame order run for real; every gathered word is checked.
The plan itself is checked in C (tests/c/c_abi_smoke.c) and executed over gloo (test_shard_gloo.py).
"""
import json
import re
import os
import signal
import socket
import subprocess
import time
import tempfile
import sys

import numpy as np
import pytest
import torch

import oracle
from uflow_amd import synth
from uflow_amd.shard import ShardedGate, comm_id_create, shard_chunks

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def gate(engine):
    g = ShardedGate(engine, 1, 0, comm_id_create())
    yield g
    g.close()


@pytest.mark.parametrize("n,L,separate_stream", [(9_000_000, 64, True), (1_000_003, 1500, False),
                                                 (5, 1500, True), (4_194_305, 37, True)])
def test_sharded_world1_vs_oracle(engine, gate, n, L, separate_stream):
    assert len(shard_chunks(n, 0, 1)) == max(1, -(-n // (1 << 22)))
    frames = synth.fixed_frames(n, L, synth.SEED_CONFIG4, device=DEV)
    engine.seal_fixed(frames, L, n=n)
    flips = torch.arange(0, n, 1013, device=DEV)
    synth.flip_bits(frames, flips * L, byte_in_frame=L // 2)
    crc = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    valid = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    gs = torch.cuda.Stream() if separate_stream else None
    gate.crc_sharded(frames, L, n, crc, valid, root=0, gather_stream=gs)
    torch.cuda.synchronize()
    host = frames.cpu().numpy()
    ref_crc, ref_valid = oracle.validate_fixed_mt(host, L, L, n, 16)
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid.cpu().numpy(), ref_valid)
    assert int(ref_valid.sum()) == n - flips.numel()


def test_sharded_rejects_bad_arguments(engine, gate):
    from uflow_amd._native import NativeError
    frames = torch.zeros(100 * 10, dtype=torch.uint8, device=DEV)
    crc = torch.zeros(10, dtype=torch.int32, device=DEV)
    with pytest.raises(NativeError):
        gate.crc_sharded(frames, 100, 10, crc, None, root=1)  # root outside the communicator
    with pytest.raises(ValueError):
        gate.crc_sharded(frames, 100, 11, crc, None)  # outputs shorter than the batch


def test_sharded_varlen_world1_config3(engine, gate):
    """ufc_crc_sharded_varlen at world size 1 on config 3's batch (10M x U[64,1500] B, 3 chunks):
    every frame against the oracle."""
    from uflow_amd.shard import shard_bounds_varlen
    n = 10_000_000
    data, off = synth.varlen_batch(n, 64, 1500, synth.SEED_CONFIG3, device=DEV)
    engine.seal_varlen(data, off)
    synth.flip_bits(data, off[:-1][::1001], byte_in_frame=5)
    h_off = off.cpu().numpy().view(np.uint64)
    b = shard_bounds_varlen(h_off, 1)
    assert list(b) == [0, n]
    crc = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    valid = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    gate.crc_sharded_varlen(data, off, b, crc, valid, root=0, gather_stream=torch.cuda.Stream())
    torch.cuda.synchronize()
    ref_crc, ref_valid = oracle.validate_varlen_mt(data.cpu().numpy(), h_off, 64)
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid.cpu().numpy(), ref_valid)
    assert int(ref_valid.sum()) == n - len(range(0, n, 1001))


def _run_worker(world, args, timeout, extra_env=None):
    """`world` ranks of tests/gpu_shard_worker.py started directly (env:// rendezvous on 127.0.0.1),
    each in a process group of its own with its output in a file: on a timeout every rank's group is
    killed and the output read so far names the step that hung."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_WORLD_SIZE=str(world))
    base.update(extra_env or {})
    cmd = [sys.executable, os.path.join(repo, "tests", "gpu_shard_worker.py")] + args
    procs, files = [], []
    for r in range(world):
        env = dict(base, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0")
        fo, fe = tempfile.TemporaryFile("w+"), tempfile.TemporaryFile("w+")
        files.append((fo, fe))
        procs.append(subprocess.Popen(cmd, stdout=fo, stderr=fe, text=True, env=env, cwd=repo, start_new_session=True))
    deadline = time.monotonic() + timeout
    timed_out = False
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            timed_out = True
            break
    if timed_out:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        for p in procs:
            p.wait()
    outs, errs = [], []
    for fo, fe in files:
        fo.seek(0)
        fe.seek(0)
        outs.append(fo.read())
        errs.append(fe.read())
        fo.close()
        fe.close()
    out, err = "".join(outs), "\n".join(f"--- rank {r} ---\n{e[-2000:]}" for r, e in enumerate(errs))
    if timed_out:
        pytest.fail(f"ranks did not finish in {timeout} s; stdout: {out[-1500:]}; stderr: {err}")
    rc = max((p.returncode for p in procs), key=abs)
    return subprocess.CompletedProcess(cmd, rc, out, err)


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_on_one_device(world):
    """The N > 1 send/recv branch of the C ABI, executed: `world` ranks on cuda:0, RCCL over its
    socket transport (each rank on its own NCCL_HOSTID), fixed and variable-length batches gathered
    to a root and checked frame by frame against the oracle (tests/gpu_shard_worker.py)."""
    p = _run_worker(world, [], 240)
    assert p.returncode == 0, p.stderr[-3000:]
    # one JSON object per root (last rank: fixed; rank 0: varlen); the two processes share the pipe,
    # so their lines may arrive on one line
    objs = re.findall(r"\{[^{}]*\}", p.stdout)
    assert len(objs) == 2, p.stdout[-2000:]
    j = {}
    for o in objs:
        j.update(json.loads(o))
    assert j["world"] == world
    assert j["fixed_crc_ok"] and j["fixed_valid_ok"] and j["fixed_invalid"] == len(range(0, 9_000_001, 1013))
    assert j["varlen_crc_ok"] and j["varlen_valid_ok"] and j["varlen_invalid"] == len(range(0, 1_500_001, 7))
    assert len(j["varlen_bounds"]) == world + 1 and 0 < j["varlen_bounds"][1] < 1_500_001
    # the last rank passed no shard: it gets UFC_ERR_INVALID_ARG (-1), every other rank UFC_ERR_PEER
    # (-6), nobody hangs, and the next call on the same communicators is exact
    assert j["fail_codes"] == [-6] * (world - 1) + [-1]
    assert j["after_fail_crc_ok"]


def test_sharded_peer_timeout():
    """A peer that never makes the call: rank 1 of 2 (both on cuda:0) creates the
    communicator and never calls ufc_crc_sharded; rank 0, with a 3-s deadline, gets UFC_ERR_COMM within
    it instead of hanging (no ncclCommAbort), then UFC_ERR_COMM at once from the stalled communicator,
    and exits non-zero (tests/gpu_shard_worker.py --peer-timeout).  Reference caller:
    /root/reference/src/server/mod.rs:591-602 (a receive loop that must not wait for ever)."""
    p = _run_worker(2, ["--peer-timeout"], 120)
    objs = re.findall(r"\{[^{}]*\}", p.stdout)
    assert len(objs) == 1, (p.stdout[-2000:], p.stderr[-2000:])
    j = json.loads(objs[0])
    code0, t0, code1, t1 = j["peer_timeout_codes"]
    assert code0 == j["UFC_ERR_COMM"] and code1 == j["UFC_ERR_COMM"], j
    assert 2.5 <= t0 <= 30.0, j   # the deadline, not a hang
    assert t1 - t0 < 1.0, j       # a stalled communicator fails at once
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])


def test_sharded_late_peer():
    """A peer that calls only after the other rank's deadline has passed: rank 0 fails with
    UFC_ERR_COMM at its 3-s deadline; rank 1 then calls and must fail with UFC_ERR_COMM at its own 3-s
    deadline (the commit round finds no partner) instead of queueing a gather that hangs.  Both ranks
    then close the communicator and the context: ufc_ctx_destroy returns at once although an
    all-reduce stays pending on the device (tests/gpu_shard_worker.py --late-peer)."""
    p = _run_worker(2, ["--late-peer"], 150, extra_env={"UFC_SHARD_TRACE": "1"})
    objs = re.findall(r"\{\"late_peer\".*\}", p.stdout)
    assert len(objs) == 1, (p.stdout[-2000:], p.stderr[-2000:])
    j = json.loads(objs[0])
    r0, r1 = j["late_peer"]
    assert r1 is not None, j
    for r in (r0, r1):
        assert r["code"] == j["UFC_ERR_COMM"], j
        assert 2.5 <= r["t_call"] <= 30.0, j  # the deadline, not a hang, and not an early success
        assert r["t_close"] < 5.0, j          # teardown does not wait for the pending all-reduce
    assert p.returncode == 0, (p.returncode, p.stderr[-2000:])
