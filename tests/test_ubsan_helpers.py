"""The kernels' mask and shift helpers under UBSan, as host code: fix_word,
front_fix, data_mask, frame_word_mask, rot_nibble_key (uflow_amd/csrc/frame_crc_dev.hpp) and head_byte
(frame_parse.hpp) are __host__ __device__; tests/c/ubsan_helpers.hip sweeps each over its whole argument
range against a byte-wise restatement, built with -fsanitize=undefined -fno-sanitize-recover=all on the
host side (the device side is compiled but never run).  Any out-of-range shift amount, in any arm of a
ternary, selected or not, stops the program.  CPU only."""
import os
import subprocess
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def test_helpers_under_ubsan():
    src = os.path.join(REPO, "tests", "c", "ubsan_helpers.hip")
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "ubsan_helpers")
        cmd = [HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O1", "-std=c++17",
               "-Xarch_host", "-fsanitize=undefined", "-Xarch_host", "-fno-sanitize-recover=all",
               "-fsanitize=undefined", "-fno-gpu-sanitize", src, "-o", exe]
        b = subprocess.run(cmd, capture_output=True, text=True)
        assert b.returncode == 0, b.stderr[-3000:]
        r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
        assert r.stdout.startswith("ok:"), r.stdout
        assert "runtime error" not in r.stderr, r.stderr[-3000:]
