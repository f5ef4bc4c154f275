"""CPU: `bench.py --gpus N` with no launcher starts its own N ranks (torch.distributed.run as a child,
no GPU call in the parent) and forwards exactly one JSON line -- rank 0's -- to stdout.  The ranks
here are the launcher test's fake workers (--fake-worker: a gloo all-reduce, no GPU), so this checks
the launch plumbing the driver's `python bench.py --gpus 8` would take."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--fake-worker"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    return p


def test_bench_launches_its_own_ranks():
    p = _run(2)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["ranks_seen"] == 2
    assert "rank 1 of 2 alive" in p.stderr  # the other ranks' output goes to stderr


def test_bench_launcher_three_ranks():
    p = _run(3)
    assert p.returncode == 0, p.stderr[-2000:]
    j = json.loads(p.stdout.strip())
    assert j["ranks_seen"] == 3


def test_split_result_line_interleaved():
    """Rank 0's JSON line found when another rank's print landed in front of it on the same line."""
    import bench
    obj = '{"metric": "m", "value": 1}'
    assert bench.split_result_line(obj + "\n") == ("", obj)
    assert bench.split_result_line("rank 2 of 3 alive" + obj + "\n") == ("rank 2 of 3 alive", obj)
    assert bench.split_result_line("rank 1 of 3 alive\n") == ("rank 1 of 3 alive\n", None)
    assert bench.split_result_line('{"metric": broken\n')[1] is None
