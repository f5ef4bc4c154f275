"""bench.py end to end on the GPU: the single-GPU line (config 2 path) and the N > 1 path rehearsed at
one rank (--sharded: ufc_crc_sharded over RCCL, gather to rank 0, sampled oracle check).  Each run
must print exactly one JSON line on stdout (the driver reads rank 0's stdout) and pass its own
oracle checks."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_single_gpu_line():
    j = _run(["--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--settle-ms", "5"])
    assert j["n_gpus"] == 1 and j["config"]["global_frames"] == 1_000_000
    assert "bit-exact vs the CPU oracle: True" in j["data"] and "valid flags as planted: True" in j["data"]
    r = j["roofline"]
    assert 0 < r["frac"] < 1 and r["kernel_avg_ms"] > 0 and j["ms_per_step"] > 0
    assert 0 < r["ceiling_GBs"] < 8000 and r["frac_of_ceiling"] > 0


def test_bench_sharded_path_one_rank():
    j = _run(["--sharded", "--global-frames", "5000000", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
              "--settle-ms", "5"])
    assert j["scaling"] == "strong" and j["config"]["global_frames"] == 5_000_000
    assert "CRC words gathered on rank 0 == the CPU oracle over every rank's shard: True" in j["data"]
    assert "oracle valid flags == planted flips on every rank: True" in j["data"]
    assert "valid flags as planted: True" in j["data"]
    assert "ufc_crc_sharded" in j["roofline"]["kernel"]


def test_bench_two_ranks_one_device():
    """`bench.py --gpus 2` with no launcher: the bench starts its own two ranks; --one-device puts both
    on cuda:0 (RCCL socket transport), so config 4's N > 1 path -- ufc_crc_sharded's sends and the
    root's receives, two chunks per 5M-frame shard -- runs and is checked by bench's own oracle pass."""
    j = _run(["--gpus", "2", "--one-device", "--global-frames", "10000000", "--steps", "3", "--warmup", "1",
              "--settle-ms", "5", "--cpu-seconds", "0.5"], timeout=300)
    assert j["n_gpus"] == 2 and j["scaling"] == "strong" and j["config"]["global_frames"] == 10_000_000
    assert "all 10000000 CRC words gathered on rank 0 == the CPU oracle over every rank's shard: True" in j["data"]
    assert "oracle valid flags == planted flips on every rank: True" in j["data"]
    assert "valid flags as planted: True" in j["data"]
    assert j["cpu_baseline"]["value"] > 0 and j["roofline"]["ceiling_GBs"] > 0
    # the N > 1 line separates the gates from the gather
    assert len(j["per_rank_kernel_ms"]) == 2 and all(x > 0 for x in j["per_rank_kernel_ms"])
    assert len(j["gather_ms"]) == 2 and all(x >= 0 for x in j["gather_ms"])
    assert len(j["host_call_ms"]) == 2 and all(x > 0 for x in j["host_call_ms"])
    ref = j["n1_sharded_ref"]
    assert ref["value"] > 0 and ref["frames"] > 0 and ref["valid_flags_as_planted"]
