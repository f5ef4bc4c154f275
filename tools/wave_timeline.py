"""Summarise a UFC_DBG_WAVES dump (tuning build): per-wave start / staged / end timestamps
(s_memrealtime, 100 MHz) of the lean fixed-length kernel."""
import sys
import numpy as np

d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4)
t0 = d[:, 0].astype(np.int64)
base = t0.min()
start = (t0 - base) / 100.0           # us
staged = (d[:, 1].astype(np.int64) - base) / 100.0
end = (d[:, 2].astype(np.int64) - base) / 100.0
sets = (d[:, 3] & 0xFFFFFFFF).astype(np.int64)
smid = ((d[:, 3] >> 32) & 0xFFFF).astype(np.int64)
xcc = ((d[:, 3] >> 56) & 0xF).astype(np.int64)
pct = lambda a: " ".join(f"{q}%={np.percentile(a, q):.1f}" for q in (0, 10, 50, 90, 99, 100))
print(f"waves {len(d)}  sets/wave {sets.min()}..{sets.max()}")
print("start  us:", pct(start))
print("staging us (staged-start):", pct(staged - start))
print("end    us:", pct(end))
print("busy   us (end-staged):", pct(end - staged))
for x in range(8):
    m = xcc == x
    if m.any():
        print(f"xcc {x}: waves {m.sum():5d} end p50 {np.percentile(end[m], 50):.1f} max {end[m].max():.1f} "
              f"start max {start[m].max():.1f}")
