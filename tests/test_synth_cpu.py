"""CPU: the synthetic-batch generator (uflow_amd/synth.py) is splitmix64 of the
global byte index, so a rank's shard equals the same range of the whole batch."""
import numpy as np
import torch

from uflow_amd import synth

M = (1 << 64) - 1


def splitmix64_ref(x):
    z = (x + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


def test_splitmix64_matches_reference_definition():
    xs = [0, 1, 2, 0x5EED0001, (1 << 63) - 1, 1 << 63, M, 123456789123]
    got = synth.splitmix64(torch.tensor([synth._s64(x) for x in xs], dtype=torch.int64))
    assert [int(v) & M for v in got] == [splitmix64_ref(x) for x in xs]


def test_bytes_are_little_endian_words():
    out = synth.fill_bytes(torch.empty(40, dtype=torch.uint8), 0x5EED0001, 0)
    ref = b"".join(splitmix64_ref(0x5EED0001 + w).to_bytes(8, "little") for w in range(5))
    assert bytes(out.numpy()) == ref


def test_shards_equal_slices_of_the_whole():
    whole = synth.fixed_frames(97, 1500, synth.SEED_CONFIG4, device="cpu")
    for lo, hi in [(0, 13), (13, 50), (50, 97), (3, 4)]:
        part = synth.fixed_frames(hi - lo, 1500, synth.SEED_CONFIG4, first_frame=lo, device="cpu")
        assert torch.equal(part, whole[lo * 1500:hi * 1500])
    # odd byte ranges and several chunks
    big = synth.fill_bytes(torch.empty(10_001, dtype=torch.uint8), 7, 5, chunk_words=100)
    ref = synth.fill_bytes(torch.empty(10_006, dtype=torch.uint8), 7, 0)
    assert torch.equal(big, ref[5:])


def test_varlen_lengths_range_and_batch():
    lens = synth.varlen_lengths(100_000, 64, 1500, synth.SEED_CONFIG3, device="cpu")
    assert int(lens.min()) == 64 and int(lens.max()) == 1500
    assert abs(float(lens.float().mean()) - 782) < 5
    data, off = synth.varlen_batch(1000, 64, 1500, synth.SEED_CONFIG3, device="cpu")
    assert off[0] == 0 and int(off[-1]) == data.numel()
    assert np.array_equal(np.diff(off.numpy()), synth.varlen_lengths(1000, 64, 1500, synth.SEED_CONFIG3, "cpu").numpy())
