"""Synthetic frame batches of BASELINE.json's configs, generated on the device.

Bytes are a counter-based hash of their GLOBAL byte index, so any shard of a batch can be made by
the rank that owns it and equals the same range of the whole batch:
    word w (8 bytes, little-endian) = splitmix64(seed + w),   byte b = byte (b mod 8) of word b // 8
Config seeds: 2 -> 0x5EED0001 (1M x 1500 B), 3 -> 0x5EED0002 (10M x U[64,1500] B lengths and
bytes), 4 -> 0x5EED0003 (100M x 1500 B, frame-sharded).  Trailers are sealed afterwards (by the
GPU seal in bench.py; tests check them against the oracle).

torch supplies the device memory and int64 arithmetic (wrapping multiplies, masked right shifts
for the unsigned shifts); generation is chunked so the temporaries stay small.
"""
import torch

SEED_CONFIG2 = 0x5EED0001
SEED_CONFIG3 = 0x5EED0002
SEED_CONFIG4 = 0x5EED0003

_M64 = (1 << 64) - 1


def _s64(c):
    """A uint64 constant as the int64 with the same bits."""
    c &= _M64
    return c - (1 << 64) if c >= 1 << 63 else c


_GOLDEN = _s64(0x9E3779B97F4A7C15)
_MIX1 = _s64(0xBF58476D1CE4E5B9)
_MIX2 = _s64(0x94D049BB133111EB)


def _shr(z, k):
    """Logical right shift of int64 lanes (torch's >> is arithmetic)."""
    return (z >> k) & ((1 << (64 - k)) - 1)


def splitmix64(x):
    """splitmix64 finaliser of int64 counters x (the value after the generator's own increment)."""
    z = x + _GOLDEN
    z = (z ^ _shr(z, 30)) * _MIX1
    z = (z ^ _shr(z, 27)) * _MIX2
    return z ^ _shr(z, 31)


def fill_bytes(out, seed, byte0, chunk_words=1 << 25):
    """out (uint8, contiguous, on a device) <- global bytes [byte0, byte0 + out.numel()) of stream `seed`."""
    n = out.numel()
    if n == 0:
        return out
    dev = out.device
    w_lo = byte0 // 8
    w_hi = (byte0 + n + 7) // 8
    pos = 0  # bytes of `out` written
    for w0 in range(w_lo, w_hi, chunk_words):
        w1 = min(w_hi, w0 + chunk_words)
        words = splitmix64(torch.arange(w0, w1, dtype=torch.int64, device=dev) + _s64(seed))
        b = words.view(torch.uint8)  # little-endian bytes of the words = global bytes [8 w0, 8 w1)
        lo = max(byte0, 8 * w0) - 8 * w0
        hi = min(byte0 + n, 8 * w1) - 8 * w0
        out[pos:pos + hi - lo].copy_(b[lo:hi])
        pos += hi - lo
    assert pos == n
    return out


def fixed_frames(n, frame_len, seed, first_frame=0, device="cuda"):
    """Frames [first_frame, first_frame + n) of a fixed-length batch: uint8[n * frame_len]
    (trailers are raw stream bytes until sealed)."""
    out = torch.empty(n * frame_len, dtype=torch.uint8, device=device)
    return fill_bytes(out, seed, first_frame * frame_len)


def varlen_lengths(n, lo, hi, seed, device="cuda"):
    """Lengths U[lo, hi] of frames 0..n-1: lo + splitmix64(~seed + i) mod (hi - lo + 1) (int64)."""
    h = splitmix64(torch.arange(n, dtype=torch.int64, device=device) + _s64(~seed))
    return lo + _shr(h, 1) % (hi - lo + 1)


def varlen_batch(n, lo, hi, seed, device="cuda"):
    """A packed CSR batch (config 3 shape): (bytes uint8[sum len], offsets int64[n + 1])."""
    lens = varlen_lengths(n, lo, hi, seed, device)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=device)
    torch.cumsum(lens, 0, out=offsets[1:])
    total = int(offsets[-1])
    data = torch.empty(total, dtype=torch.uint8, device=device)
    fill_bytes(data, seed, 0)
    return data, offsets


def flip_bits(frames_or_data, starts, byte_in_frame=17, mask=0x04):
    """Flip one bit in each listed frame (frames starting at byte offsets `starts`): every such frame
    must then fail the gate (a single-bit error changes a CRC-32)."""
    idx = starts + byte_in_frame
    frames_or_data[idx] ^= mask
    return frames_or_data
