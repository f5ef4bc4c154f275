"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the C oracle (oracle/crc_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module,
and only as the checker / CPU baseline.  The product (uflow_amd, libuflowcrc.so) never
imports or links it.  See crc_oracle.c for the reference citations and how parity is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_DIR, "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_DIR, "crc_oracle.c")
        if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
            subprocess.run(["make", "-C", _DIR, "-s"], check=True)
        l = ctypes.CDLL(_LIB)
        vp, sz, u32, u8 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint8
        sigs = {
            "ufo_extend_slow": (u32, [u32, vp, sz]),
            "ufo_table": (None, [vp]),
            "ufo_table_matches": (ctypes.c_int, [vp]),
            "ufo_extend": (u32, [u32, vp, sz]),
            "ufo_compute": (u32, [vp, sz]),
            "ufo_frame_validate": (ctypes.c_int, [vp, sz, vp]),
            "ufo_frame_seal": (u32, [vp, sz]),
            "ufo_validate_fixed": (None, [vp, sz, sz, sz, vp, vp]),
            "ufo_validate_varlen": (None, [vp, vp, sz, vp, vp]),
            "ufo_seal_fixed": (None, [vp, sz, sz, sz]),
            "ufo_seal_varlen": (None, [vp, vp, sz]),
            "ufo_validate_fixed_mt": (ctypes.c_int, [vp, sz, sz, sz, vp, vp, ctypes.c_int]),
            "ufo_validate_varlen_mt": (ctypes.c_int, [vp, vp, sz, vp, vp, ctypes.c_int]),
            "ufo_seal_fixed_mt": (ctypes.c_int, [vp, sz, sz, sz, ctypes.c_int]),
            "ufo_seal_varlen_mt": (ctypes.c_int, [vp, vp, sz, ctypes.c_int]),
            "ufo_write_handshake_syn": (sz, [vp, u8, u32, u32, u32, u32]),
            "ufo_write_handshake_syn_ack": (sz, [vp, u32, u32, u32, u32, u32]),
            "ufo_write_handshake_ack": (sz, [vp, u32]),
            "ufo_write_handshake_error": (sz, [vp, u32, u8]),
            "ufo_write_disconnect": (sz, [vp, ctypes.c_int]),
            "ufo_write_sync": (sz, [vp, ctypes.c_int, u32, ctypes.c_int, u32]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _bytes(data):
    return np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data


def extend_slow(initial_crc, data):
    a = _bytes(data)
    return lib().ufo_extend_slow(initial_crc & 0xFFFFFFFF, _p(a), a.size)


def extend(initial_crc, data):
    a = _bytes(data)
    return lib().ufo_extend(initial_crc & 0xFFFFFFFF, _p(a), a.size)


def compute(data):
    a = _bytes(data)
    return lib().ufo_compute(_p(a), a.size)


def table():
    out = np.zeros(256, dtype=np.uint32)
    lib().ufo_table(_p(out))
    return out


def table_matches(literals):
    a = np.ascontiguousarray(literals, dtype=np.uint32)
    return bool(lib().ufo_table_matches(_p(a)))


def frame_validate(frame):
    a = _bytes(frame)
    c = ctypes.c_uint32()
    v = lib().ufo_frame_validate(_p(a), a.size, ctypes.byref(c))
    return bool(v), c.value


def frame_seal(frame: bytearray):
    a = np.frombuffer(frame, dtype=np.uint8)
    return lib().ufo_frame_seal(_p(a), a.size)


def validate_fixed(frames: np.ndarray, stride, frame_len, n):
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    crc = np.zeros(n, dtype=np.uint32)
    valid = np.zeros(n, dtype=np.uint8)
    lib().ufo_validate_fixed(_p(frames), stride, frame_len, n, _p(crc), _p(valid))
    return crc, valid


def validate_fixed_mt(frames: np.ndarray, stride, frame_len, n, nthreads):
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    crc = np.zeros(n, dtype=np.uint32)
    valid = np.zeros(n, dtype=np.uint8)
    rc = lib().ufo_validate_fixed_mt(_p(frames), stride, frame_len, n, _p(crc), _p(valid), int(nthreads))
    if rc != 0:
        raise RuntimeError("ufo_validate_fixed_mt failed")
    return crc, valid


def default_threads():
    """Host threads for the full-size checks: the CPUs this process may run on (the GPU box's
    share; os.cpu_count() there reports the whole machine), capped at 64."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(64, n))


def validate_varlen_mt(data: np.ndarray, offsets: np.ndarray, nthreads=None):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    crc = np.zeros(n, dtype=np.uint32)
    valid = np.zeros(n, dtype=np.uint8)
    lib().ufo_validate_varlen_mt(_p(data), _p(offsets), n, _p(crc), _p(valid), int(nthreads or default_threads()))
    return crc, valid


def seal_fixed_mt(frames: np.ndarray, stride, frame_len, n, nthreads=None):
    assert frames.dtype == np.uint8 and frames.flags.c_contiguous
    lib().ufo_seal_fixed_mt(_p(frames), stride, frame_len, n, int(nthreads or default_threads()))


def seal_varlen_mt(data: np.ndarray, offsets: np.ndarray, nthreads=None):
    assert data.dtype == np.uint8 and data.flags.c_contiguous
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lib().ufo_seal_varlen_mt(_p(data), _p(offsets), offsets.size - 1, int(nthreads or default_threads()))


def validate_varlen(data: np.ndarray, offsets: np.ndarray):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    crc = np.zeros(n, dtype=np.uint32)
    valid = np.zeros(n, dtype=np.uint8)
    lib().ufo_validate_varlen(_p(data), _p(offsets), n, _p(crc), _p(valid))
    return crc, valid


def seal_fixed(frames: np.ndarray, stride, frame_len, n):
    lib().ufo_seal_fixed(_p(frames), stride, frame_len, n)


def seal_varlen(data: np.ndarray, offsets: np.ndarray):
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lib().ufo_seal_varlen(_p(data), _p(offsets), offsets.size - 1)


def _writer(fn, size, *args):
    buf = np.zeros(size, dtype=np.uint8)
    n = getattr(lib(), fn)(_p(buf), *args)
    return bytes(buf[:n])


def write_handshake_syn(version, nonce, max_receive_rate, max_packet_size, max_receive_alloc):
    return _writer("ufo_write_handshake_syn", 1472, version, nonce, max_receive_rate, max_packet_size,
                   max_receive_alloc)


def write_handshake_syn_ack(nonce_ack, nonce, max_receive_rate, max_packet_size, max_receive_alloc):
    return _writer("ufo_write_handshake_syn_ack", 64, nonce_ack, nonce, max_receive_rate, max_packet_size,
                   max_receive_alloc)


def write_handshake_ack(nonce_ack):
    return _writer("ufo_write_handshake_ack", 16, nonce_ack)


def write_handshake_error(nonce_ack, error):
    return _writer("ufo_write_handshake_error", 16, nonce_ack, error)


def write_disconnect(ack=False):
    return _writer("ufo_write_disconnect", 16, 1 if ack else 0)


def write_sync(next_frame_id=None, next_packet_id=None):
    return _writer("ufo_write_sync", 16, next_frame_id is not None, next_frame_id or 0,
                   next_packet_id is not None, next_packet_id or 0)
