"""GPU: the multi-GPU C ABI (ufc_comm_create + ufc_crc_sharded over RCCL) at world size 1 -- the one
GPU of the test box.  The RCCL communicator is created through the library's own binding, the
shard is gated chunk by chunk (front-readable chunks after the first), results land in their
global positions, and every frame matches the oracle.  The point-to-point layout between ranks is
covered on the CPU (tests/test_shard_gloo.py); N > 1 runs in the driver's 8-GPU bench.
"""
import numpy as np
import pytest
import torch

import oracle
from uflow_amd import synth
from uflow_amd.shard import ShardedGate, comm_id_create, shard_chunks

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def gate(engine):
    g = ShardedGate(engine, 1, 0, comm_id_create())
    yield g
    g.close()


@pytest.mark.parametrize("n,L,separate_stream", [(9_000_000, 64, True), (1_000_003, 1500, False),
                                                 (5, 1500, True), (4_194_305, 37, True)])
def test_sharded_world1_vs_oracle(engine, gate, n, L, separate_stream):
    assert len(shard_chunks(n, 0, 1)) == max(1, -(-n // (1 << 22)))
    frames = synth.fixed_frames(n, L, synth.SEED_CONFIG4, device=DEV)
    engine.seal_fixed(frames, L, n=n)
    flips = torch.arange(0, n, 1013, device=DEV)
    synth.flip_bits(frames, flips * L, byte_in_frame=L // 2)
    crc = torch.full((n,), -1, dtype=torch.int32, device=DEV)
    valid = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
    gs = torch.cuda.Stream() if separate_stream else None
    gate.crc_sharded(frames, L, n, crc, valid, root=0, gather_stream=gs)
    torch.cuda.synchronize()
    host = frames.cpu().numpy()
    ref_crc, ref_valid = oracle.validate_fixed_mt(host, L, L, n, 16)
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid.cpu().numpy(), ref_valid)
    assert int(ref_valid.sum()) == n - flips.numel()


def test_sharded_rejects_bad_arguments(engine, gate):
    from uflow_amd._native import NativeError
    frames = torch.zeros(100 * 10, dtype=torch.uint8, device=DEV)
    crc = torch.zeros(10, dtype=torch.int32, device=DEV)
    with pytest.raises(NativeError):
        gate.crc_sharded(frames, 100, 10, crc, None, root=1)  # root outside the communicator
    with pytest.raises(ValueError):
        gate.crc_sharded(frames, 100, 11, crc, None)  # outputs shorter than the batch
