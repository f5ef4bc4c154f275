"""The loopback harness (tools/loopback/ufc_loopback, BASELINE.json configs 1 and 5): frames built
by the native builders, sent over UDP 127.0.0.1, received in batches (recvmmsg), gated and parsed.
CPU: the echo plumbing (examples/echo_server.rs + echo_client.rs) and a short stream with the CPU
gate; GPU: the same stream with the GPU gate (ufc_validate_host_slots) in the receive path."""
import json
import os
import random
import subprocess

import pytest

from uflow_amd._build import LOOPBACK_BIN, build_tools


def _run(args, timeout=120):
    build_tools()
    port = str(random.randrange(20000, 60000))
    r = subprocess.run([LOOPBACK_BIN, "--port", port] + args, capture_output=True, text=True, timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(lines[-1])


def test_echo_plumbing():
    j = _run(["--echo"])
    assert j["echoes_ok"] == j["messages"] == 10


def _check_stream(j, n, every, max_loss=None):
    assert j["payload_mismatch"] == 0
    assert j["received"] > 0 and j["valid"] + j["invalid"] == j["received"]
    assert j["parsed"] == j["valid"]
    if "lost" in j:
        assert j["lost"] == j["sent"] - j["received"]
    if max_loss is not None:  # paced senders: the gate must keep up (ideal_transfer.rs: all arrives)
        assert j["loss_frac"] <= max_loss, j
    if j["received"] == n:  # nothing dropped by the socket: exactly the corrupted frames fail
        assert j["invalid"] == n // every


def test_stream_cpu_gate():
    n = 100_000
    _check_stream(_run(["--gate", "cpu", "--frames", str(n), "--corrupt-every", "997"]), n, 997)


@pytest.mark.gpu
def test_stream_gpu_gate():
    n = 200_000
    _check_stream(_run(["--gate", "gpu", "--frames", str(n), "--corrupt-every", "997"]), n, 997)


def test_stream_inline_cpu_gate():
    """Inline receive loops (receive + gate + parse per thread, server/mod.rs:591-602) on 2 threads."""
    n = 100_000
    _check_stream(_run(["--gate", "cpu", "--rx-threads", "2", "--frames", str(n), "--corrupt-every", "997"]), n, 997)


def test_stream_inline_cpu_gate_paced():
    """Paced senders (0.1 GB/s offered, a rate this container's CPU gate keeps up with): loss is
    reported (sent - received) and stays under 0.5 %."""
    n = 60_000
    j = _run(["--gate", "cpu", "--rx-threads", "2", "--tx-per-rx", "1", "--frames", str(n), "--corrupt-every", "997",
              "--rate-gbps", "0.1"])
    _check_stream(j, n, 997, max_loss=0.005)


@pytest.mark.gpu
def test_stream_inline_gpu_gate():
    """The same with the asynchronous GPU gate overlapped with the next receive: unpaced (loss
    reported, not bounded) and paced at 0.8 GB/s, where the loss must stay under 0.5 %."""
    n = 200_000
    j = _run(["--gate", "gpu", "--rx-threads", "2", "--frames", str(n), "--corrupt-every", "997"])
    assert j["failed_threads"] == 0
    _check_stream(j, n, 997)
    j = _run(["--gate", "gpu", "--rx-threads", "2", "--tx-per-rx", "1", "--frames", str(n), "--corrupt-every", "997",
              "--rate-gbps", "0.8"])
    assert j["failed_threads"] == 0
    _check_stream(j, n, 997, max_loss=0.005)
