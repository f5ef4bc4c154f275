"""Diagnostic (round 6, not product code): where a config-3 set's cycles go in the variable-length gate.

Runs a stamp build of the library (var/stamp.so, from tools/probes/stamp_variant.py: tools/build_variant.py with s_memtime stamps at the loop
top, after the next record's fetch, before the finish and at the end of each set; lane 0 stores the low 32
bits of the four clocks per set into a debug array read back by ufc_dbg_read) on config 3's batch and
prints the per-set cycle split: top (geometry, next set's record, run sort once per run), positions (the
line steps with their waits for data), finish (slot constants, A^-t, trailer compare, record), and the gap
to the same wave's next set.  Read the SHARES, not the length: the stamps' waits perturb the kernel.
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "tools"))
from ab_inproc import load, make_ctx  # noqa: E402

NSETS = 1250016


def main():
    lib = load(os.path.join(REPO, sys.argv[1] if len(sys.argv) > 1 else "var/stamp.so"))
    lib.ufc_dbg_read.argtypes = [ctypes.c_void_p]
    ctx = make_ctx(lib, {})
    dev = torch.device("cuda", 0)
    sp = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    n = 10_000_000
    rng = np.random.default_rng(0x5EED0002)
    lens = rng.integers(64, 1501, n).astype(np.uint64)
    o = np.zeros(n + 1, np.uint64)
    o[1:] = np.cumsum(lens)
    offs = torch.from_numpy(o.view(np.int64)).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0001)
    frames = torch.randint(0, 256, (int(o[-1]),), dtype=torch.uint8, device=dev, generator=g)
    assert lib.ufc_seal_batch_varlen(ctx, frames.data_ptr(), offs.data_ptr(), n, None, sp) == 0
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for i in range(40):
        e0.record()
        assert lib.ufc_crc_batch_varlen(ctx, frames.data_ptr(), offs.data_ptr(), n, crc.data_ptr(), valid.data_ptr(), sp) == 0
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    assert int(valid.sum()) == n
    buf = np.zeros(NSETS * 8, np.uint32)
    assert lib.ufc_dbg_read(buf.ctypes.data) == 0
    st = buf.reshape(-1, 8)[: n // 8].astype(np.int64)
    slow = st[:, 5] != 0
    t0, t1, t2, t3, t1b = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4]
    m32 = (1 << 32) - 1
    top = (t1 - t0) & m32
    pos = (t2 - t1) & m32
    first = (t1b - t1) & m32
    fin = (t3 - t2) & m32
    q = np.arange(st.shape[0])
    same = (q % 8) != 7
    gap = np.zeros_like(top)
    gap[:-1] = (t0[1:] - t3[:-1]) & m32
    # Pmax per set from the host geometry (runs of 64 sorted by line count, the kernel's order)
    a = o[:-1]
    r = (a - 4) % 128
    P = ((lens + r + 131) >> 7).astype(np.int64)
    P[P > 13] = 14
    Ps = np.sort(P.reshape(-1, 64), axis=1, kind="stable").reshape(-1, 8).max(axis=1)
    fast = ~slow
    print(f"kernel (stamp build) median {np.median(ts):.4f} ms over {len(ts)} launches; sets {st.shape[0]}, slow {int(slow.sum())}")
    tot = top + pos + fin
    for name, v in (("top (geometry, record, sort)", top), ("positions (steps + waits)", pos),
                    ("  of which entry + first line", first), ("finish + record", fin)):
        print(f"  {name:32s} mean {v[fast].mean():8.0f} cycles  share {v[fast].sum() / tot[fast].sum():.3f}")
    g_ok = same & fast
    print(f"  gap to the next set (same wave) mean {gap[g_ok].mean():8.0f} cycles")
    print(f"  set total (fast) mean {tot[fast].mean():.0f} cycles; Pmax mean {Ps[fast].mean():.2f}")
    for pm in range(1, 14):
        sel = fast & (Ps == pm)
        if sel.sum() > 1000:
            print(f"    Pmax {pm:2d}: sets {int(sel.sum()):7d}  positions {pos[sel].mean():7.0f} (entry+first {first[sel].mean():6.0f}, then {(pos[sel] - first[sel]).mean() / max(pm - 1, 1):5.0f} per line)  finish {fin[sel].mean():6.0f}  top {top[sel].mean():6.0f}")


if __name__ == "__main__":
    main()
