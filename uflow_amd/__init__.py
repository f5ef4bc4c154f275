"""uflow_amd -- MI355X-native engine for uflow's per-frame CRC-32 (src/frame).

The hot path (batched frame validate / seal) runs as hand-written gfx950 HIP kernels behind the
C ABI of libuflowcrc.so (include/uflow_frame_crc.h).  Submodules:
    crc     scalar host API mirroring crc::compute / crc::extend and the Frame::read CRC gate
    batch   FrameCrcEngine: batched device-resident validate/seal on torch tensors
    shard   multi-GPU sharding by frame + RCCL gather of the CRC words
"""
from . import crc  # noqa: F401

__all__ = ["crc"]
