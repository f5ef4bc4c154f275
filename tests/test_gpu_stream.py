"""GPU, tuning builds: the byte-balanced streaming kernel (UFC_VARLEN_STREAM, frame_crc_stream8_kernel) against the
oracle on every variable-length case of test_gpu_parity.py plus the cases its byte split and frame
walk add: batches whose offsets do not start at 0, single-frame and tiny batches, runs of empty
frames at group boundaries and at the batch end, frames far longer than a group's byte range, and the
seal (trailers written by the stream).  Reference: the Frame::read gate, src/frame/serial/mod.rs:675-690,
and the seal, serial/mod.rs:463-470 / build.rs:151-159."""
import numpy as np
import pytest
import torch

import oracle
from uflow_amd import _native as N
from uflow_amd import synth

import test_gpu_parity as P

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture()
def stream(engine):
    """The streaming kernel exists in tuning builds only (measured slower than the default,
    DESIGN.md section 5.2): run with UFC_LIB=uflow_amd/libuflowcrc_tuning.so (tools/gpu_tuning_tests.sh)."""
    if N.lib().ufc_ctx_set_option(engine._ctx, N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_STREAM) != N.UFC_OK:
        pytest.skip("UFC_VARLEN_STREAM: tuning builds only (UFC_LIB=uflow_amd/libuflowcrc_tuning.so)")
    assert engine.get_option(N.UFC_OPT_VARLEN_KERNEL) == N.UFC_VARLEN_STREAM
    yield engine
    engine.set_option(N.UFC_OPT_VARLEN_KERNEL, N.UFC_VARLEN_AUTO)


def _case(eng, data, offsets):
    ref_crc, ref_valid = oracle.validate_varlen(data, offsets.astype(np.uint64))
    crc, valid = eng.crc_varlen(torch.from_numpy(data).to(DEV), torch.from_numpy(offsets.astype(np.int64)).to(DEV))
    torch.cuda.synchronize()
    got = crc.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != ref_crc)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}, lens {np.diff(offsets)[bad[:5]]}"
    assert np.array_equal(valid.cpu().numpy(), ref_valid)
    return ref_valid


def test_stream_mixed(stream):
    P.test_varlen_mixed(stream)


def test_stream_edges(stream):
    P.test_varlen_edges(stream)


def test_stream_uflow_frames(stream):
    P.test_varlen_uflow_frames(stream)


def test_stream_seal(stream):
    P.test_seal_varlen(stream)
    P.test_seal_varlen_large(stream)


@pytest.mark.parametrize("lo,hi,n", [(5, 1473, 200_003), (64, 1501, 131_072), (4, 300, 50_001), (1400, 1533, 40_000)])
def test_stream_large_batches(stream, lo, hi, n):
    P.test_varlen_large_batches(stream, lo, hi, n)


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_stream_misaligned_base(stream, shift):
    P.test_varlen_misaligned_base(stream, shift)


@pytest.mark.parametrize("n", [1, 2, 7, 64, 1000])
def test_stream_tiny_batches(stream, n):
    rng = np.random.default_rng(600 + n)
    lens = rng.integers(0, 3000, size=n)
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(lens)
    data = P._rand_bytes(rng, int(off[-1]))  # exact size: nothing readable past the last frame
    for i in range(n):
        if lens[i] >= 4:
            fr = bytearray(data[off[i]:off[i + 1]].tobytes())
            oracle.frame_seal(fr)
            data[off[i]:off[i + 1]] = np.frombuffer(bytes(fr), np.uint8)
    _case(stream, data, off)


def test_stream_offset_base_and_empty_runs(stream):
    """offsets[0] > 0 (a CSR window into a larger buffer), runs of empty frames everywhere (also at
    the very end, where they start exactly at offsets[n]), and frames of 0..4 bytes."""
    rng = np.random.default_rng(77)
    n = 60_000
    lens = rng.integers(5, 1500, size=n)
    lens[rng.integers(0, n, size=5000)] = 0
    lens[rng.integers(0, n, size=2000)] = rng.integers(1, 5, size=2000)
    lens[-50:] = 0
    lens[:30] = 0
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(lens)
    off += 12345
    data = P._rand_bytes(rng, int(off[-1]))
    for i in range(0, n, 3):
        if lens[i] >= 4:
            fr = bytearray(data[off[i]:off[i + 1]].tobytes())
            oracle.frame_seal(fr)
            data[off[i]:off[i + 1]] = np.frombuffer(bytes(fr), np.uint8)
    valid = _case(stream, data, off)
    assert 0 < valid.sum() < n


def test_stream_long_frames(stream):
    """Frames far longer than a group's byte range (up to 1 MB) between short ones: a group keeps
    walking its last frame past its range; other groups start after it."""
    rng = np.random.default_rng(78)
    lens = np.concatenate([rng.integers(5, 1500, size=20_000), [1 << 20, 300_001, 65_536, 8192, 1533]])
    rng.shuffle(lens)
    off = np.zeros(lens.size + 1, np.int64)
    off[1:] = np.cumsum(lens)
    data = P._rand_bytes(rng, int(off[-1]) + 3)
    oracle.seal_varlen(data, off.astype(np.uint64))
    for i in range(0, lens.size, 37):
        data[off[i] + rng.integers(0, lens[i])] ^= 0x40
    valid = _case(stream, data, off)
    assert valid.sum() == lens.size - len(range(0, lens.size, 37))


def test_stream_config3_full(stream):
    """Config 3's batch (10M x U[64,1500] B, 7.8 GB): every frame against the multithreaded oracle."""
    n = 10_000_000
    data, offsets = synth.varlen_batch(n, 64, 1500, synth.SEED_CONFIG3, device=DEV)
    stream.seal_varlen(data, offsets)
    synth.flip_bits(data, offsets[:-1][::997], byte_in_frame=7, mask=0x20)
    crc, valid = stream.crc_varlen(data, offsets)
    torch.cuda.synchronize()
    h_off = offsets.cpu().numpy().view(np.uint64)
    ref_crc, ref_valid = oracle.validate_varlen_mt(data.cpu().numpy(), h_off, 64)
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert np.array_equal(valid.cpu().numpy(), ref_valid)
    assert int(ref_valid.sum()) == n - len(range(0, n, 997))
