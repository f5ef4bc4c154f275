"""Where does the fixed kernel's finish spread come from?  From a UFC_DBG_WAVES dump (tuning build,
tools/wave_dump.py): per-wave end times split into the spread inside a workgroup (its 8 waves),
across the workgroups of one XCD, and across XCDs.
    python tools/wave_spread.py gpurun_out/wd/w.bin.0 [...]"""
import sys

import numpy as np

WAVES = 8

for path in sys.argv[1:]:
    d = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
    t0 = d[:, 0].astype(np.int64).min()
    end = (d[:, 2].astype(np.int64) - t0) / 100.0
    xcc = ((d[:, 3] >> 56) & 0xF).astype(np.int64)
    wg = np.arange(len(d)) // WAVES
    nwg = wg.max() + 1
    wg_end = np.array([end[wg == g].max() for g in range(nwg)])
    wg_first = np.array([end[wg == g].min() for g in range(nwg)])
    wg_xcc = np.array([xcc[wg == g][0] for g in range(nwg)])
    print(f"{path}: kernel end {end.max():.1f} us, wave end median {np.median(end):.1f}")
    print(f"  inside a workgroup (last - first wave): median {np.median(wg_end - wg_first):.2f} "
          f"p90 {np.percentile(wg_end - wg_first, 90):.2f} max {np.max(wg_end - wg_first):.2f} us")
    for x in range(8):
        m = wg_xcc == x
        if m.any():
            e = wg_end[m]
            print(f"  xcc {x}: {m.sum()} workgroups, workgroup end median {np.median(e):.1f} max {e.max():.1f} "
                  f"(max - median {e.max() - np.median(e):.2f}), blockIdx % 8 = {sorted(set((np.nonzero(m)[0] % 8).tolist()))}")
    med = [np.median(wg_end[wg_xcc == x]) for x in range(8) if (wg_xcc == x).any()]
    print(f"  across XCDs: workgroup-end medians {min(med):.1f} .. {max(med):.1f}")
