"""Batched, device-resident frame CRC on MI355X (the hot path).

`FrameCrcEngine` owns one libuflowcrc context per device and wraps the batched C-ABI entry
points on torch tensors (torch provides device memory and the current HIP stream only).
Per frame i:  crc[i] = compute(frame_i[:-4]),  valid[i] = len_i >= 5 and crc[i] == BE32(frame_i[-4:])
-- the CRC gate of Frame::read (src/frame/serial/mod.rs:675-690) -- and seal writes the trailer
(src/frame/serial/mod.rs:463-470, build.rs:151-159).

CRC words are returned as int32 tensors holding the uint32 bit patterns
(`crc.cpu().numpy().view(numpy.uint32)`).
"""
import ctypes

import numpy as np
import torch

from ._native import lib, check


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class FrameCrcEngine:
    def __init__(self, device=None):
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self._ctx = ctypes.c_void_p()
        check(lib().ufc_ctx_create(ctypes.byref(self._ctx), self.device.index or 0), "ufc_ctx_create")

    def _bytes_ptr(self, t):
        """The frame bytes' pointer for the C ABI, which wants a readable device buffer even when a
        batch holds only empty frames (torch gives an empty tensor a NULL data_ptr): a zeroed 256-B
        buffer of the engine's stands in then."""
        if t.numel():
            return _ptr(t)
        if getattr(self, "_no_bytes", None) is None:
            self._no_bytes = torch.zeros(256, dtype=torch.uint8, device=self.device)
        return _ptr(self._no_bytes)

    def close(self):
        if self._ctx:
            lib().ufc_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def release_stream(self, stream):
        """ufc_ctx_release_stream: free this context's scratch kept for `stream` (a torch.cuda.Stream)
        after the work queued on it; call before the stream goes away."""
        check(lib().ufc_ctx_release_stream(self._ctx, ctypes.c_void_p(stream.cuda_stream)), "ufc_ctx_release_stream")

    def set_option(self, option, value):
        """ufc_ctx_set_option (A/B kernel selection; results never depend on it)."""
        check(lib().ufc_ctx_set_option(self._ctx, int(option), int(value)), "ufc_ctx_set_option")

    def get_option(self, option):
        return lib().ufc_ctx_get_option(self._ctx, int(option))

    def _stream(self, stream):
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return ctypes.c_void_p(s.cuda_stream)

    def _check_dev(self, *ts):
        for t in ts:
            if t is not None and (t.device != self.device or not t.is_contiguous()):
                raise ValueError(f"tensor must be contiguous on {self.device}")

    def _check(self, name, t, dtypes, min_numel):
        """Device, contiguity, dtype and size of an argument, checked before the C ABI sees its
        pointer (the kernels trust the sizes they are given)."""
        if t is None:
            return
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name} must be a torch tensor")
        if t.dtype not in dtypes:
            raise ValueError(f"{name} must be {' or '.join(str(d) for d in dtypes)}, got {t.dtype}")
        self._check_dev(t)
        if t.numel() < min_numel:
            raise ValueError(f"{name} holds {t.numel()} elements, needs at least {min_numel}")

    def _check_outputs(self, n, crc_out=None, valid_out=None):
        self._check("crc_out", crc_out, (torch.int32, torch.uint32), n)
        self._check("valid_out", valid_out, (torch.uint8,), n)

    # ---- fixed-stride batches ----
    def crc_fixed(self, frames, frame_len, stride=None, n=None, crc_out=None, valid_out=None,
                  want_crc=True, want_valid=True, stream=None):
        """frames: uint8 tensor; frame i at byte i*stride (stride defaults to frame_len)."""
        stride = frame_len if stride is None else stride
        if n is None:
            n = (frames.numel() - frame_len) // stride + 1 if frames.numel() >= frame_len else 0
        if crc_out is None and want_crc:
            crc_out = torch.empty(n, dtype=torch.int32, device=self.device)
        if valid_out is None and want_valid:
            valid_out = torch.empty(n, dtype=torch.uint8, device=self.device)
        self._check("frames", frames, (torch.uint8,), (n - 1) * stride + frame_len if n else 0)
        self._check_outputs(n, crc_out, valid_out)
        check(lib().ufc_crc_batch_fixed(self._ctx, self._bytes_ptr(frames), stride, frame_len, n, _ptr(crc_out),
                                        _ptr(valid_out), self._stream(stream)), "ufc_crc_batch_fixed")
        return crc_out, valid_out

    def seal_fixed(self, frames, frame_len, stride=None, n=None, crc_out=None, stream=None):
        stride = frame_len if stride is None else stride
        if n is None:
            n = (frames.numel() - frame_len) // stride + 1 if frames.numel() >= frame_len else 0
        self._check("frames", frames, (torch.uint8,), (n - 1) * stride + frame_len if n else 0)
        self._check_outputs(n, crc_out)
        check(lib().ufc_seal_batch_fixed(self._ctx, self._bytes_ptr(frames), stride, frame_len, n, _ptr(crc_out),
                                         self._stream(stream)), "ufc_seal_batch_fixed")
        return crc_out

    # ---- variable-length (CSR) batches ----
    def crc_varlen(self, data, offsets, crc_out=None, valid_out=None, want_crc=True, want_valid=True,
                   stream=None):
        """data: uint8 tensor; offsets: int64 tensor of n+1 nondecreasing byte offsets."""
        n = offsets.numel() - 1
        if crc_out is None and want_crc:
            crc_out = torch.empty(max(n, 0), dtype=torch.int32, device=self.device)
        if valid_out is None and want_valid:
            valid_out = torch.empty(max(n, 0), dtype=torch.uint8, device=self.device)
        self._check("offsets", offsets, (torch.int64,), 1)
        self._check("data", data, (torch.uint8,), 0)
        self._check_outputs(n, crc_out, valid_out)
        check(lib().ufc_crc_batch_varlen(self._ctx, self._bytes_ptr(data), _ptr(offsets), n, _ptr(crc_out), _ptr(valid_out),
                                         self._stream(stream)), "ufc_crc_batch_varlen")
        return crc_out, valid_out

    def seal_varlen(self, data, offsets, crc_out=None, stream=None):
        n = offsets.numel() - 1
        self._check("offsets", offsets, (torch.int64,), 1)
        self._check("data", data, (torch.uint8,), 0)
        self._check_outputs(n, crc_out)
        check(lib().ufc_seal_batch_varlen(self._ctx, self._bytes_ptr(data), _ptr(offsets), n, _ptr(crc_out),
                                          self._stream(stream)), "ufc_seal_batch_varlen")
        return crc_out

    def crc_pairs(self, data, pairs, crc_out=None, valid_out=None, stream=None):
        """pairs: int64 tensor [n, 2] of (start, end) byte offsets into data (any gapped layout)."""
        if pairs.dim() != 2 or pairs.shape[1] != 2:
            raise ValueError("pairs must have shape [n, 2]")
        n = pairs.shape[0]
        if crc_out is None:
            crc_out = torch.empty(n, dtype=torch.int32, device=self.device)
        if valid_out is None:
            valid_out = torch.empty(n, dtype=torch.uint8, device=self.device)
        self._check("pairs", pairs, (torch.int64,), 2 * n)
        self._check("data", data, (torch.uint8,), 0)
        self._check_outputs(n, crc_out, valid_out)
        check(lib().ufc_crc_batch_pairs(self._ctx, self._bytes_ptr(data), data.numel(), _ptr(pairs), n, _ptr(crc_out),
                                        _ptr(valid_out), self._stream(stream)), "ufc_crc_batch_pairs")
        return crc_out, valid_out

    # ---- measurement context (not the CRC path) ----
    def hbm_read_probe(self, buf, sink, stream=None):
        """ufc_hbm_read_probe: read buf (uint8, device) as one plain stream, XOR into sink (int32[1]);
        returns the bytes read (whole KiB).  The bench's read-only streaming ceiling."""
        self._check("buf", buf, (torch.uint8,), 0)
        self._check("sink", sink, (torch.int32, torch.uint32), 1)
        nread = ctypes.c_size_t()
        check(lib().ufc_hbm_read_probe(self._ctx, _ptr(buf), buf.numel(), _ptr(sink), ctypes.byref(nread),
                                       self._stream(stream)), "ufc_hbm_read_probe")
        return nread.value

    # ---- Frame::read past the gate, on the device (uflow_frame_codec.h) ----
    def parse_varlen(self, data, offsets, valid, items_cap=None, stream=None):
        """Batched Frame::read of a CSR batch after the CRC gate (`valid`, from crc_varlen).
        Returns (infos uint8[n, 32], items uint8[items_cap, 24], items_used int64[1]) device tensors;
        the byte rows are ufc_frame_info / ufc_item records (numpy views: uflow_amd.frame
        FRAME_INFO_DTYPE / ITEM_DTYPE).  items_cap defaults to a bound no batch can exceed."""
        n = offsets.numel() - 1
        self._check("offsets", offsets, (torch.int64,), 1)
        self._check("data", data, (torch.uint8,), 0)
        self._check("valid", valid, (torch.uint8,), n)
        if items_cap is None:  # a datagram takes >= 6 bytes, an ack group 9
            items_cap = max(1, data.numel() // 6)
        infos = torch.empty((max(n, 0), 32), dtype=torch.uint8, device=self.device)
        items = torch.empty((items_cap, 24), dtype=torch.uint8, device=self.device)
        used = torch.zeros(1, dtype=torch.int64, device=self.device)
        check(lib().ufc_parse_batch_varlen(self._ctx, self._bytes_ptr(data), _ptr(offsets), n, _ptr(valid), _ptr(infos),
                                           _ptr(items), items_cap, _ptr(used), self._stream(stream)),
              "ufc_parse_batch_varlen")
        return infos, items, used

    # ---- host buffers (frames received into host memory) ----
    def seal_host_varlen(self, data: np.ndarray, offsets: np.ndarray):
        """Seal every frame of a host CSR batch in place (GPU CRC, host trailer write); returns the CRCs."""
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        crc = np.empty(max(n, 0), dtype=np.uint32)
        check(lib().ufc_seal_host_varlen(self._ctx, data.ctypes.data, offsets.ctypes.data, n, crc.ctypes.data),
              "ufc_seal_host_varlen")
        return crc

    def validate_host_slots(self, slots: np.ndarray, slot_stride: int, lens: np.ndarray):
        """Datagrams received into fixed-size slots (recvmmsg layout) -> (crc uint32[n], valid uint8[n])."""
        slots = np.ascontiguousarray(slots, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = lens.size
        if n and slots.size < (n - 1) * slot_stride + int(lens[-1]):
            raise ValueError("slots must hold slot n - 1 and its datagram")
        crc = np.empty(n, dtype=np.uint32)
        valid = np.empty(n, dtype=np.uint8)
        check(lib().ufc_validate_host_slots(self._ctx, slots.ctypes.data, slot_stride, lens.ctypes.data, n,
                                            crc.ctypes.data, valid.ctypes.data), "ufc_validate_host_slots")
        return crc, valid

    def validate_host_slots_async(self, slots, slot_stride: int, lens, crc_out, valid_out, stream):
        """Queue the slots gate on `stream` (torch.cuda.Stream) and return at once: slots (uint8),
        lens (int32) and the outputs crc_out (int32[n]) / valid_out (uint8[n]) are host
        torch tensors, ideally pinned, that must stay alive and unmodified until the stream is done."""
        n = lens.numel() if isinstance(lens, torch.Tensor) else 0
        need = {"lens": (lens, torch.int32, n), "crc_out": (crc_out, torch.int32, n),
                "valid_out": (valid_out, torch.uint8, n), "slots": (slots, torch.uint8, 0)}
        for name, (t, dt, m) in need.items():
            if not isinstance(t, torch.Tensor) or t.is_cuda or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous host tensor")
            if t.dtype != dt or t.numel() < m:
                raise ValueError(f"{name} must be {dt} with at least {m} elements")
        # The copy reads (n - 1) * slot_stride + lens[n - 1] bytes of slots (ufc_api.cpp).
        m = (n - 1) * slot_stride + int(lens[n - 1]) if n else 0
        if slots.numel() < m:
            raise ValueError(f"slots must hold at least {m} bytes (slot n - 1 and its datagram), got {slots.numel()}")
        check(lib().ufc_validate_host_slots_async(self._ctx, slots.data_ptr(), slot_stride, lens.data_ptr(), n,
                                                  crc_out.data_ptr(), valid_out.data_ptr(), stream.cuda_stream),
              "ufc_validate_host_slots_async")

    def validate_host_varlen(self, data: np.ndarray, offsets: np.ndarray):
        """numpy uint8 bytes + uint64/int64 offsets in host memory -> (crc uint32[n], valid uint8[n])."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        crc = np.empty(max(n, 0), dtype=np.uint32)
        valid = np.empty(max(n, 0), dtype=np.uint8)
        check(lib().ufc_validate_host_varlen(self._ctx, data.ctypes.data_as(ctypes.c_void_p),
                                             offsets.ctypes.data_as(ctypes.c_void_p), n,
                                             crc.ctypes.data_as(ctypes.c_void_p),
                                             valid.ctypes.data_as(ctypes.c_void_p)), "ufc_validate_host_varlen")
        return crc, valid
