"""A plain C program (gcc, C99) linked against libuflowcrc.so seals and gates 200k frames on the GPU
through the host-buffer entry points and checks every frame against the scalar host entry points
(tests/c/c_abi_gpu.c): the boundary as a Rust `extern "C"` caller would use it, no Python or HIP in
the caller."""
import os
import shutil
import subprocess

import pytest

from uflow_amd import _native

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_caller_on_gpu(tmp_path):
    gcc = shutil.which("gcc")
    assert gcc, "gcc is part of the image"
    exe = tmp_path / "c_abi_gpu"
    libdir = os.path.dirname(_native.LIB_PATH)
    subprocess.run([gcc, "-std=c99", "-O2", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", os.path.join(REPO, "include"),
                    "-o", str(exe), os.path.join(REPO, "tests", "c", "c_abi_gpu.c"), "-L", libdir, "-luflowcrc",
                    f"-Wl,-rpath,{libdir}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c gpu ok" in r.stdout
