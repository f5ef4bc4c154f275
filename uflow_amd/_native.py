"""ctypes binding of libuflowcrc.so (the C ABI in include/uflow_frame_crc.h and
include/uflow_frame_codec.h).

This is the Python-side equivalent of the `extern "C"` block a Rust caller would declare
(see INTEGRATION.md).  Loading fails loudly when the in-tree library is missing: there is no
CPU fallback for the batched entry points.
"""
import ctypes
import os

from ._build import LIB_PATH as _DEFAULT_LIB

# Measurement tools only: with UFC_AB=1 set as well, UFC_LIB names another build of the library to
# load (in-process A/B runs under tools/).  Without the guard the in-tree library is the one loaded,
# whatever UFC_LIB says ("Test-only environment").
LIB_PATH = os.environ["UFC_LIB"] if os.environ.get("UFC_AB") == "1" and os.environ.get("UFC_LIB") else _DEFAULT_LIB

UFC_OK = 0
UFC_ERR_INVALID_ARG = -1
UFC_ERR_NO_DEVICE = -2
UFC_ERR_HIP = -3
UFC_ERR_NOMEM = -4
UFC_ERR_COMM = -5
UFC_ERR_PEER = -6
UFC_COMM_ID_BYTES = 128
UFC_MAX_RANKS = 64
UFC_OP_GATE, UFC_OP_SEND, UFC_OP_RECV = 0, 1, 2

# ufc_ctx_set_option (include/uflow_frame_crc.h)
UFC_OPT_FIXED_KERNEL, UFC_OPT_VARLEN_KERNEL, UFC_OPT_GENERIC_JC = 0, 1, 2
UFC_FIXED_AUTO, UFC_FIXED_GENERIC, UFC_FIXED_CLAIM16 = 0, 1, 2
UFC_VARLEN_AUTO, UFC_VARLEN_GENERIC, UFC_VARLEN_SORTED, UFC_VARLEN_BLOCKED8, UFC_VARLEN_CLAIM16 = 0, 1, 2, 3, 4
UFC_VARLEN_BLOCKSTREAM, UFC_VARLEN_SORTED8, UFC_VARLEN_STREAM = 5, 6, 7
UFC_OPT_SEAL_KERNEL, UFC_SEAL_INLINE, UFC_SEAL_TWO_PASS = 3, 0, 1

# Every symbol the header declares, with its ctypes signature.
_c_u8p = ctypes.POINTER(ctypes.c_uint8)
_SIGNATURES = {
    "ufc_crc32_compute": (ctypes.c_uint32, [ctypes.c_void_p, ctypes.c_size_t]),
    "ufc_crc32_extend": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]),
    "ufc_frame_validate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    "ufc_frame_seal": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    "ufc_device_count": (ctypes.c_int, []),
    "ufc_ctx_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]),
    "ufc_ctx_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "ufc_ctx_release_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "ufc_ctx_last_hip_error": (ctypes.c_int, [ctypes.c_void_p]),
    "ufc_ctx_set_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "ufc_ctx_get_option": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ufc_crc_batch_fixed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_crc_batch_varlen": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_seal_batch_fixed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                            ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_seal_batch_varlen": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_hbm_read_probe": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]),
    "ufc_validate_host_varlen": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_crc_batch_pairs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_validate_host_slots": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                               ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_validate_host_slots_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                     ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_seal_host_slots": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_void_p]),
    "ufc_seal_host_varlen": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.c_void_p]),
    "ufc_shard_range": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                       ctypes.POINTER(ctypes.c_uint64)]),
    "ufc_shard_chunk": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "ufc_shard_bounds_fixed": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]),
    "ufc_shard_bounds_varlen": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]),
    "ufc_shard_nchunks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ufc_shard_gather_plan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_void_p, ctypes.c_int]),
    "ufc_comm_id_create": (ctypes.c_int, [ctypes.c_void_p]),
    "ufc_comm_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p]),
    "ufc_comm_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "ufc_comm_last_error": (ctypes.c_int, [ctypes.c_void_p]),
    "ufc_comm_set_timeout": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ufc_crc_sharded": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_crc_sharded_varlen": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p]),
    # include/uflow_frame_codec.h
    "ufc_frame_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_size_t]),
    "ufc_frame_parse": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_size_t]),
    "ufc_datagram_is_valid": (ctypes.c_int, [ctypes.c_void_p]),
    "ufc_frame_write_fixed": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]),
    "ufc_data_frame_builder_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                                   ctypes.c_int]),
    "ufc_data_frame_builder_add": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "ufc_data_frame_encoded_size": (ctypes.c_size_t, [ctypes.c_void_p]),
    "ufc_ack_frame_builder_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                                  ctypes.c_uint32]),
    "ufc_ack_frame_builder_add": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]),
    "ufc_builder_size": (ctypes.c_size_t, [ctypes.c_void_p]),
    "ufc_builder_build": (ctypes.c_size_t, [ctypes.c_void_p, ctypes.c_int]),
    "ufc_parse_batch_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.POINTER(ctypes.c_size_t), ctypes.c_int]),
    "ufc_parse_batch_varlen": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.c_void_p, ctypes.c_void_p]),
}
SYMBOLS = tuple(_SIGNATURES)


# Structs of include/uflow_frame_codec.h (layouts checked by tests/test_codec_cpu.py).
class FrameInfo(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint8), ("ok", ctypes.c_uint8), ("aux", ctypes.c_uint8), ("crc_ok", ctypes.c_uint8),
                ("f", ctypes.c_uint32 * 5), ("item_count", ctypes.c_uint32), ("item_first", ctypes.c_uint32)]


class Item(ctypes.Structure):
    _fields_ = [("id", ctypes.c_uint32), ("channel_id", ctypes.c_uint8), ("form", ctypes.c_uint8),
                ("window_parent_lead", ctypes.c_uint16), ("channel_parent_lead", ctypes.c_uint16),
                ("fragment_id", ctypes.c_uint16), ("fragment_id_last", ctypes.c_uint16), ("flags", ctypes.c_uint16),
                ("data_offset", ctypes.c_uint32), ("data_len", ctypes.c_uint32)]


class Builder(ctypes.Structure):
    _fields_ = [("buf", ctypes.c_void_p), ("cap", ctypes.c_size_t), ("len", ctypes.c_size_t),
                ("count", ctypes.c_uint32), ("kind", ctypes.c_uint32)]


class Xfer(ctypes.Structure):
    """ufc_xfer: one operation of the multi-GPU gather plan (ufc_shard_gather_plan)."""
    _fields_ = [("op", ctypes.c_int32), ("peer", ctypes.c_int32), ("src", ctypes.c_uint64), ("dst", ctypes.c_uint64),
                ("count", ctypes.c_uint64)]


class DatagramRef(ctypes.Structure):
    _fields_ = [("sequence_id", ctypes.c_uint32), ("channel_id", ctypes.c_uint8), ("reserved", ctypes.c_uint8),
                ("window_parent_lead", ctypes.c_uint16), ("channel_parent_lead", ctypes.c_uint16),
                ("fragment_id", ctypes.c_uint16), ("fragment_id_last", ctypes.c_uint16),
                ("data", ctypes.c_void_p), ("data_len", ctypes.c_size_t)]

_lib = None


class NativeError(RuntimeError):
    def __init__(self, code, what=""):
        msg = _lib.ufc_error_string(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} (code {code})" if what else f"{msg} (code {code})")
        self.code = code


def lib():
    """The loaded library (raises if libuflowcrc.so has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libuflowcrc.so not found at {LIB_PATH}: run `python -m uflow_amd._build` "
                              "(the native library is required; there is no CPU fallback)")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def check(rc, what=""):
    if rc != UFC_OK:
        raise NativeError(rc, what)
    return rc
