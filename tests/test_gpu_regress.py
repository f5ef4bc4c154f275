"""GPU regressions the round-3 review asked for, every result against the CPU oracle.

  ramp sequence   tools/probes/ramp_probe.py's shape: the GPU seals 4,000,000 / 4,186,112 (one full
                  launch of the fixed kernel) / 4,186,113 (one launch + a 1-frame second launch)
                  frames x 1500 B in place, then the gate runs over n = 250k .. 4,186,113 of the
                  sealed batch into ONE shared (crc, valid) pair, with the plain read stream in
                  between, as the probe does.  Every sealed byte equals the oracle's seal
                  (serial/mod.rs:463-470) and every CRC word / flag equals the oracle's gate
                  (serial/mod.rs:675-690).
  crc_flips       serial/mod.rs:1054-1080 on the HIP path: 10,000 seeded random data frames
                  (random_data_frame, :932-992, up to 3.4 KB: frames past the 8-lane kernel's fast
                  path included), 5 random bit flips each; CSR and shuffled (start, end) pairs.
                  Every frame must be rejected (as the reference asserts) and every CRC word must
                  equal the oracle's.
"""
import random

import numpy as np
import pytest
import torch

import oracle
from oracle import codec as C
from uflow_amd import synth

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
THREADS = 16  # the GPU box's CPU share
L = 1500
FULL_LAUNCH = 4_186_112  # 256 CUs x 8 waves x 511 sets x 4 frames (ufc_api.cpp launch_lean_fixed)


def _first_diff(a, b, chunk=1 << 28):
    """First index where two equal-length uint8 device tensors differ, or -1 (chunked: one
    nonzero over several GB of bytes overflows its workspace)."""
    for c0 in range(0, a.numel(), chunk):
        x, y = a[c0:c0 + chunk], b[c0:c0 + chunk]
        if not torch.equal(x, y):
            return c0 + int(torch.nonzero(x != y)[0])
    return -1


def test_ramp_sequence_vs_oracle(engine):
    nmax = FULL_LAUNCH + 1
    raw = synth.fixed_frames(nmax, L, synth.SEED_CONFIG2, device=DEV)
    ref_h = raw.cpu().numpy()
    oracle.seal_fixed_mt(ref_h, L, L, nmax, THREADS)
    ref_crc, ref_valid = oracle.validate_fixed_mt(ref_h, L, L, nmax, THREADS)
    assert int(ref_valid.sum()) == nmax
    ref = torch.from_numpy(ref_h).to(DEV)
    del ref_h

    # seal: prefixes of the raw batch, with the scratch CRC path (crc_out=None, as the probe) and
    # with a caller crc_out
    for n in (4_000_000, FULL_LAUNCH, FULL_LAUNCH + 1):
        for with_crc in (False, True):
            d = raw.clone()
            crc_out = torch.full((n,), -1, dtype=torch.int32, device=DEV) if with_crc else None
            engine.seal_fixed(d, L, n=n, crc_out=crc_out)
            torch.cuda.synchronize()
            k = _first_diff(d[:n * L], ref[:n * L])
            assert k < 0, f"seal n={n} crc_out={with_crc}: first differing byte {k} (frame {k // L})"
            assert _first_diff(d[n * L:], raw[n * L:]) < 0, f"seal n={n} wrote past its frames"
            if with_crc:
                got = crc_out.cpu().numpy().view(np.uint32)
                assert np.array_equal(got, ref_crc[:n]), f"seal n={n}: crc_out differs"
            del d
    del raw
    torch.cuda.empty_cache()

    # gate: the probe's order (interleaved with the read stream), one shared output pair
    crc = torch.full((nmax,), -1, dtype=torch.int32, device=DEV)
    valid = torch.full((nmax,), 7, dtype=torch.uint8, device=DEV)
    sink = torch.zeros(1, dtype=torch.int32, device=DEV)
    sizes = [250_000, 500_000, 1_000_000, 2_000_000, 4_000_000, FULL_LAUNCH, FULL_LAUNCH + 1]
    for rnd in range(2):
        for n in sizes:
            crc.fill_(-1)
            valid.fill_(7)
            engine.crc_fixed(ref, L, n=n, crc_out=crc, valid_out=valid)
            engine.hbm_read_probe(ref[:n * L], sink)
            torch.cuda.synchronize()
            got_c = crc[:n].cpu().numpy().view(np.uint32)
            got_v = valid[:n].cpu().numpy()
            bad = np.nonzero((got_c != ref_crc[:n]) | (got_v != ref_valid[:n]))[0]
            assert bad.size == 0, f"gate n={n} round {rnd}: {bad.size} frames differ, first {bad[:8]}"
            assert int((crc[n:] != -1).sum()) == 0 and int((valid[n:] != 7).sum()) == 0, \
                f"gate n={n} wrote past frame n"


def _flipped_frames(seed, rounds):
    """crc_flips (serial/mod.rs:1054-1080): random data frames, 5 random bit flips each."""
    rng = random.Random(seed)
    frames = []
    for _ in range(rounds):
        fb = bytearray(C.frame_write(C.random_data_frame(rng)))
        assert len(fb) <= 8192
        for _ in range(5):
            bit = rng.randrange(len(fb) * 8)
            fb[bit // 8] ^= 1 << (bit % 8)
        frames.append(bytes(fb))
    return frames


def test_crc_flips_gpu(engine):
    frames = _flipped_frames(1054, 10_000)
    lens = np.array([len(f) for f in frames], dtype=np.uint64)
    off = np.zeros(len(frames) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    ref_crc, ref_valid = oracle.validate_varlen(data, off)
    assert not ref_valid.any(), "a 5-bit flip passed the oracle's gate"
    assert (lens > 1532).sum() > 100  # frames past the 8-lane kernel's fast path are exercised
    d = torch.from_numpy(data).to(DEV)
    crc, valid = engine.crc_varlen(d, torch.from_numpy(off.view(np.int64)).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
    assert not valid.cpu().numpy().any(), "the GPU gate accepted a frame with 5 flipped bits"
    perm = np.random.default_rng(1080).permutation(len(frames))
    pairs = np.stack([off[:-1][perm], off[1:][perm]], axis=1).astype(np.int64)
    crc, valid = engine.crc_pairs(d, torch.from_numpy(pairs).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc[perm])
    assert not valid.cpu().numpy().any()
    # the unflipped frames pass: the same frames sealed again by the GPU are all accepted
    engine.seal_varlen(d, torch.from_numpy(off.view(np.int64)).to(DEV))
    crc, valid = engine.crc_varlen(d, torch.from_numpy(off.view(np.int64)).to(DEV))
    torch.cuda.synchronize()
    assert valid.cpu().numpy().all()
    assert np.array_equal(crc.cpu().numpy().view(np.uint32), ref_crc)
