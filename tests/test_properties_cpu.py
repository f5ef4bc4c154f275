"""Property-based checks (hypothesis) of the host entry points against the oracle and against the
algebra the reference's CRC satisfies (crc.rs:94-104; the gate of serial/mod.rs:675-690):
  - compute / extend equal the oracle's for any bytes and any initial value;
  - extend composes: extend(extend(c, x), y) == extend(c, x + y) (the property the kernels' slot
    chains and A^-t shifts rely on), and the byte-at-a-time spec (extend_slow) agrees;
  - seal then gate accepts, and any single flipped bit of a sealed frame is rejected (CRC-32 detects
    every single-bit error), for every frame length >= 5;
  - frames shorter than 5 bytes never pass the gate (mod.rs:676-678).
No GPU: the GPU kernels get the same properties in tests/test_gpu_parity.py."""
import pytest
from hypothesis import given, settings, strategies as st

import oracle
from uflow_amd import crc

BYTES = st.binary(min_size=0, max_size=3000)
U32 = st.integers(min_value=0, max_value=0xFFFFFFFF)


@settings(max_examples=300, deadline=None)
@given(BYTES, U32)
def test_compute_and_extend_match_the_oracle(data, init):
    assert crc.compute(data) == oracle.compute(data)
    assert crc.extend(init, data) == oracle.extend(init, data) == oracle.extend_slow(init, data)


@settings(max_examples=300, deadline=None)
@given(BYTES, BYTES, U32)
def test_extend_composes(x, y, init):
    assert crc.extend(crc.extend(init, x), y) == crc.extend(init, x + y)


@settings(max_examples=200, deadline=None)
@given(st.binary(min_size=5, max_size=2000), st.data())
def test_seal_then_gate_and_single_bit_flips(body, data):
    frame = bytearray(body)
    crc.frame_seal(frame)
    assert crc.frame_validate(bytes(frame))
    assert oracle.frame_validate(bytes(frame))[0]
    bit = data.draw(st.integers(min_value=0, max_value=8 * len(frame) - 1))
    frame[bit // 8] ^= 1 << (bit % 8)
    assert not crc.frame_validate(bytes(frame))
    assert not oracle.frame_validate(bytes(frame))[0]


@settings(max_examples=100, deadline=None)
@given(st.binary(min_size=0, max_size=4))
def test_short_frames_never_pass(frame):
    assert not crc.frame_validate(frame)
    assert not oracle.frame_validate(frame)[0]
