"""CPU: the C-ABI library (libuflowcrc.so) loads and exports every symbol include/uflow_frame_crc.h
declares; its host entry points (ufc_crc32_compute/extend, ufc_frame_validate/seal -- the scalar
drop-ins for crc::compute / crc::extend and the Frame::read CRC gate) agree with the oracle and the
golden data; argument checking and error codes behave as documented.  No GPU compute here.
"""
import ctypes
import json
import os
import re

import numpy as np
import pytest

import oracle
from uflow_amd import _native, crc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "uflow_frame_crc.h")
GOLDEN = os.path.join(REPO, "tests", "golden")


def header_symbols():
    text = ""
    for h in (HEADER, os.path.join(REPO, "include", "uflow_frame_codec.h")):
        with open(h) as f:
            text += f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ufc_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    syms = header_symbols()
    assert "ufc_crc_batch_fixed" in syms and "ufc_validate_host_varlen" in syms, syms
    l = ctypes.CDLL(_native.LIB_PATH)
    missing = [s for s in syms if not hasattr(l, s)]
    assert not missing, missing
    assert set(syms) == set(_native.SYMBOLS), "header vs ctypes binding differ"


def test_constants_match_header():
    with open(HEADER) as f:
        text = f.read()
    consts = dict(re.findall(r"#define\s+(UFC_\w+)\s+\(?(-?\d+)\)?", text))
    assert int(consts["UFC_FRAME_CRC_SIZE"]) == crc.FRAME_CRC_SIZE == 4
    assert int(consts["UFC_FRAME_OVERHEAD"]) == crc.FRAME_OVERHEAD == 5
    assert int(consts["UFC_MAX_FRAME_SIZE"]) == crc.MAX_FRAME_SIZE == 1472
    assert int(consts["UFC_OK"]) == _native.UFC_OK == 0
    for name in ("UFC_OPT_FIXED_KERNEL", "UFC_OPT_VARLEN_KERNEL", "UFC_OPT_GENERIC_JC", "UFC_OPT_SEAL_KERNEL",
                 "UFC_FIXED_CLAIM16", "UFC_VARLEN_SORTED8", "UFC_VARLEN_STREAM", "UFC_SEAL_TWO_PASS", "UFC_SEAL_INLINE"):
        assert int(consts[name]) == getattr(_native, name), name


def test_host_kat_and_lengths():
    assert crc.compute(b"123456789") == 0x11A6F2A3
    assert crc.extend(0, b"123456789") == 0x11A6F2A3
    assert crc.compute(b"\x00") != 0
    with open(os.path.join(GOLDEN, "crc_lengths.json")) as f:
        g = json.load(f)
    for n, c in g["ramp"]:
        assert crc.compute(bytes(i % 256 for i in range(n))) == int(c, 16)


def test_host_extend_random_inits_vs_oracle():
    rng = np.random.default_rng(8)
    for _ in range(200):
        data = rng.integers(0, 256, size=int(rng.integers(0, 2000)), dtype=np.uint8).tobytes()
        init = int(rng.integers(0, 2**32))
        assert crc.extend(init, data) == oracle.extend_slow(init, data)


def test_host_gate_on_reference_frames():
    with open(os.path.join(GOLDEN, "frames.json")) as f:
        frames = json.load(f)["frames"]
    for fr in frames:
        b = bytes.fromhex(fr["hex"])
        assert crc.frame_validate(b), fr["name"]
        assert not crc.frame_validate(b + b"\x00")
        for i in range(0, len(b)):
            assert not crc.frame_validate(b[:i])
        bb = bytearray(b)
        bb[-4:] = b"\0\0\0\0"
        assert crc.frame_seal(bb) == int(fr["crc"], 16)
        assert bytes(bb) == b


def test_host_gate_random_fixture():
    z = np.load(os.path.join(GOLDEN, "random_frames.npz"))
    data, off = z["data"], z["offsets"]
    for i in range(len(off) - 1):
        fb = data[int(off[i]):int(off[i + 1])].tobytes()
        assert crc.frame_validate(fb) == bool(z["valid"][i])


def test_seal_rejects_short_frames():
    l = _native.lib()
    buf = (ctypes.c_uint8 * 3)()
    assert l.ufc_frame_seal(buf, 3) == _native.UFC_ERR_INVALID_ARG
    assert l.ufc_frame_validate(None, 10) == 0
    assert l.ufc_frame_seal(None, 10) == _native.UFC_ERR_INVALID_ARG


def test_batch_entry_points_reject_bad_args_without_gpu():
    l = _native.lib()
    null = ctypes.c_void_p()
    assert l.ufc_crc_batch_fixed(null, None, 0, 0, 1, None, None, None) == _native.UFC_ERR_INVALID_ARG
    assert l.ufc_crc_batch_varlen(null, None, None, 1, None, None, None) == _native.UFC_ERR_INVALID_ARG
    assert l.ufc_seal_batch_fixed(null, None, 0, 0, 1, None, None) == _native.UFC_ERR_INVALID_ARG
    assert l.ufc_seal_batch_varlen(null, None, None, 1, None, None) == _native.UFC_ERR_INVALID_ARG
    assert l.ufc_ctx_create(None, 0) == _native.UFC_ERR_INVALID_ARG
    assert l.ufc_ctx_destroy(null) == _native.UFC_OK
    for code in (0, -1, -2, -3, -4, -99):
        assert l.ufc_error_string(code)


def test_ctx_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    ctx = ctypes.c_void_p()
    rc = _native.lib().ufc_ctx_create(ctypes.byref(ctx), 0)
    assert rc in (_native.UFC_ERR_NO_DEVICE, _native.UFC_ERR_HIP)
    from uflow_amd.batch import FrameCrcEngine
    with pytest.raises(_native.NativeError):
        FrameCrcEngine(0)


def test_c_caller_links_and_runs(tmp_path):
    """The headers compile as strict C99 and a plain C program linked against libuflowcrc.so gets
    the reference's KAT, gate, seal and builder behaviour (tests/c/c_abi_smoke.c) -- the shape of
    the binding a Rust `extern "C"` block would use.  Host entry points only."""
    import shutil
    import subprocess
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    exe = tmp_path / "c_abi_smoke"
    libdir = os.path.dirname(_native.LIB_PATH)
    subprocess.run([gcc, "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", os.path.join(REPO, "include"),
                    "-o", str(exe), os.path.join(REPO, "tests", "c", "c_abi_smoke.c"), "-L", libdir, "-luflowcrc",
                    f"-Wl,-rpath,{libdir}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "c abi ok" in r.stdout


def _unbound_engine():
    """A FrameCrcEngine with no device context (CPU): argument checks run before any C-ABI call."""
    import torch
    from uflow_amd.batch import FrameCrcEngine
    eng = FrameCrcEngine.__new__(FrameCrcEngine)
    eng.device = torch.device("cpu")
    eng._ctx = ctypes.c_void_p()
    return eng


def test_batch_wrappers_reject_bad_tensors():
    """batch.py checks dtype and size of every tensor before the kernels see its pointer (a short
    crc_out or a non-uint8 frames tensor would otherwise be written or read out of bounds)."""
    import torch
    eng = _unbound_engine()
    frames = torch.zeros(10 * 100, dtype=torch.uint8)
    with pytest.raises(ValueError, match="crc_out"):
        eng.crc_fixed(frames, 100, n=10, crc_out=torch.zeros(9, dtype=torch.int32))
    with pytest.raises(ValueError, match="crc_out"):
        eng.crc_fixed(frames, 100, n=10, crc_out=torch.zeros(10, dtype=torch.int16))
    with pytest.raises(ValueError, match="valid_out"):
        eng.crc_fixed(frames, 100, n=10, valid_out=torch.zeros(10, dtype=torch.int32))
    with pytest.raises(ValueError, match="valid_out"):
        eng.crc_fixed(frames, 100, n=10, valid_out=torch.zeros(5, dtype=torch.uint8))
    with pytest.raises(ValueError, match="frames"):
        eng.crc_fixed(frames.view(torch.int32), 100, n=10)
    with pytest.raises(ValueError, match="frames"):
        eng.crc_fixed(frames, 100, n=11)
    with pytest.raises(ValueError, match="frames"):
        eng.seal_fixed(frames, 100, stride=101, n=10)
    offsets = torch.arange(0, 1001, 100, dtype=torch.int64)
    with pytest.raises(ValueError, match="offsets"):
        eng.crc_varlen(frames, offsets.to(torch.int32))
    with pytest.raises(ValueError, match="crc_out"):
        eng.crc_varlen(frames, offsets, crc_out=torch.zeros(3, dtype=torch.int32))
    with pytest.raises(ValueError, match="data"):
        eng.seal_varlen(frames.view(torch.int16), offsets)
    with pytest.raises(ValueError, match="pairs"):
        eng.crc_pairs(frames, torch.zeros(10, dtype=torch.int64))
    with pytest.raises(ValueError, match="pairs"):
        eng.crc_pairs(frames, torch.zeros((10, 2), dtype=torch.int32))
    with pytest.raises(ValueError, match="valid"):
        eng.parse_varlen(frames, offsets, torch.zeros(4, dtype=torch.uint8))
    # well-formed arguments reach the C ABI, which refuses the missing context (no CPU fallback)
    from uflow_amd._native import NativeError
    import types
    with pytest.raises(NativeError):
        eng.crc_fixed(frames, 100, n=10, stream=types.SimpleNamespace(cuda_stream=0))


def test_ctx_options_reject_without_context():
    l = _native.lib()
    null = ctypes.c_void_p()
    assert l.ufc_ctx_set_option(null, _native.UFC_OPT_FIXED_KERNEL, 0) == _native.UFC_ERR_INVALID_ARG
    assert l.ufc_ctx_get_option(null, 0) == _native.UFC_ERR_INVALID_ARG


def test_seal_host_entry_points_reject_null_buffers():
    l = _native.lib()
    null = ctypes.c_void_p()
    scratch = (ctypes.c_uint32 * 4)()
    # no context: invalid argument (never a crash); zero frames: nothing to do
    assert l.ufc_seal_host_slots(null, None, 1472, None, 4, scratch) == _native.UFC_ERR_INVALID_ARG
    assert l.ufc_seal_host_varlen(null, None, None, 4, scratch) == _native.UFC_ERR_INVALID_ARG


def test_gpu_box_receives_what_gpu_runs_load():
    """.gpurunignore keeps the built library and the PMC summary bench.py reads (roofline.traffic)
    in the snapshot sent to the GPU box (tar-style patterns: a leading ./ anchors at the top)."""
    import fnmatch

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(repo, ".gpurunignore")) as f:
        pats = [l.strip() for l in f if l.strip() and not l.startswith("#")]
    for path in ("profiles/pmc_traffic.json", "uflow_amd/libuflowcrc.so", "oracle/liboracle.so", "bench.py",
                 "tools/loopback/ufc_loopback", "tests/golden/kat.json"):
        for p in pats:
            anchored = p.startswith("./")
            pat = p[2:] if anchored else p
            hit = fnmatch.fnmatch(path, pat) or (not anchored and fnmatch.fnmatch(os.path.basename(path), pat)) \
                or path.startswith(pat.rstrip("/") + "/")
            assert not hit, f"{p} in .gpurunignore drops {path}"
