"""A plain C program (gcc, C99) linked against libuflowcrc.so seals and gates 200k frames on the GPU
through the host-buffer entry points (tests/c/c_abi_gpu.c): the boundary as a Rust `extern "C"` caller
would use it, no Python or HIP in the caller.  Its results are compared with the CPU oracle's
(oracle/crc_oracle.c: the seal of serial/mod.rs:463-470 / build.rs:151-159 and the gate of
serial/mod.rs:675-690), which this test computes and writes to a file the C program reads."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle
from uflow_amd import _native

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle_file(path, n=200_000, seed=0x5EED0C0C):
    rng = np.random.default_rng(seed)
    lens = rng.integers(5, 1473, n).astype(np.uint64)  # uflow frames: 5..1472 B (src/lib.rs:294)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    for i in range(n):  # the builders' zero trailers
        data[int(off[i + 1]) - 4:int(off[i + 1])] = 0
    sealed = data.copy()
    oracle.seal_varlen_mt(sealed, off)
    seal_crc, seal_valid = oracle.validate_varlen_mt(sealed, off)
    assert seal_valid.all()
    flip_frames = np.arange(0, n, 7)
    flip_at = (off[flip_frames] + (rng.integers(0, 1 << 30, flip_frames.size) % lens[flip_frames])).astype(np.uint64)
    flip_mask = (1 << rng.integers(0, 8, flip_frames.size)).astype(np.uint8)
    recv = sealed.copy()
    recv[flip_at] ^= flip_mask
    crc, valid = oracle.validate_varlen_mt(recv, off)
    with open(path, "wb") as f:
        np.array([n, int(off[-1]), flip_at.size], np.uint64).tofile(f)
        off.tofile(f)
        data.tofile(f)
        sealed.tofile(f)
        seal_crc.astype(np.uint32).tofile(f)
        flip_at.tofile(f)
        flip_mask.tofile(f)
        crc.astype(np.uint32).tofile(f)
        valid.astype(np.uint8).tofile(f)
    return int(valid.sum())


def test_c_caller_on_gpu(tmp_path):
    gcc = shutil.which("gcc")
    assert gcc, "gcc is part of the image"
    exe = tmp_path / "c_abi_gpu"
    libdir = os.path.dirname(_native.LIB_PATH)
    subprocess.run([gcc, "-std=c99", "-O2", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", os.path.join(REPO, "include"),
                    "-o", str(exe), os.path.join(REPO, "tests", "c", "c_abi_gpu.c"), "-L", libdir, "-luflowcrc",
                    f"-Wl,-rpath,{libdir}"], check=True)
    data = tmp_path / "oracle.bin"
    nvalid = _oracle_file(str(data))
    r = subprocess.run([str(exe), str(data)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c gpu ok" in r.stdout and f"equal to the oracle's; {nvalid} valid" in r.stdout
