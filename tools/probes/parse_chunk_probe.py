"""parse_chunk_probe.py -- does the device parse gain when the batch is parsed in chunks that fit the
MI355X's 256-MB Infinity Cache?  (tuning probe for frame_parse.hip; not product code)

The walk reads every item header's line and the emit reads the same lines again; over the whole 1M-frame
batch (1.41 GB) the walk's lines have left every cache before the emit reaches them.  This times the
bench's parse workload (tools/bench_configs.py `parse`) as one call and as consecutive calls over chunks
of C frames on one stream or spread over 2-4 streams (each chunk's walk, scan and emit back to back on
its stream, so one chunk's walk can run beside another's emit; item bases from a first full parse), and checks that the chunked items equal the whole-batch items.  Prints one JSON line per C and
exits non-zero if any chunked result differs.  Run on the GPU box: python tools/probes/parse_chunk_probe.py
"""
import ctypes
import json
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from oracle import codec as C  # noqa: E402  (probe input generation only)
from uflow_amd import _native as N  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402


def main():
    n = 1_000_000
    rng = random.Random(5)  # the bench's parse workload
    base = [C.frame_write(C.random_data_frame(rng) if i % 3 == 0 else C.receive_side_data_frame(rng)
                          if i % 3 == 1 else C.random_ack_frame(rng, 20)) for i in range(600)]
    lens = np.array([len(base[i % 600]) for i in range(n)], dtype=np.int64)
    offsets = np.zeros(n + 1, dtype=np.int64)
    offsets[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(base), dtype=np.uint8)
    data = np.concatenate([blob] * (n // 600 + 1))[: int(offsets[-1])]
    eng = FrameCrcEngine()
    d = torch.from_numpy(data).cuda()
    o = torch.from_numpy(offsets).cuda()
    _, valid = eng.crc_varlen(d, o)
    infos, items, used = eng.parse_varlen(d, o, valid)
    torch.cuda.synchronize()
    total = int(used.cpu()[0])
    from uflow_amd.frame import FRAME_INFO_DTYPE
    fi = infos.cpu().numpy().view(FRAME_INFO_DTYPE).reshape(-1)
    item_first = fi["item_first"].astype(np.int64)
    ref_items = items[:total].clone()
    lib = N.lib()
    out_items = torch.empty_like(items)
    out_infos = torch.empty_like(infos)
    used_k = torch.zeros(1, dtype=torch.int64, device="cuda")

    streams = [torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    ev_done = [torch.cuda.Event() for _ in streams]

    def run(chunk, ns=1):
        if ns > 1:  # chunk c on stream c % ns, all forked from and joined back into the current stream
            ev_start = torch.cuda.Event()
            ev_start.record(streams[0])
            for s in streams[1:ns]:
                s.wait_event(ev_start)
        for ci, c0 in enumerate(range(0, n, chunk)):
            st = streams[ci % ns].cuda_stream
            nk = min(chunk, n - c0)
            b = int(item_first[c0])
            e = int(item_first[c0 + nk]) if c0 + nk < n else total
            rc = lib.ufc_parse_batch_varlen(eng._ctx, ctypes.c_void_p(d.data_ptr()),
                                            ctypes.c_void_p(o.data_ptr() + 8 * c0), nk,
                                            ctypes.c_void_p(valid.data_ptr() + c0),
                                            ctypes.c_void_p(out_infos.data_ptr() + 32 * c0),
                                            ctypes.c_void_p(out_items.data_ptr() + 24 * b), max(e - b, 1),
                                            ctypes.c_void_p(used_k.data_ptr()), ctypes.c_void_p(st))
            if rc != 0:
                raise RuntimeError(f"parse rc {rc}")
        for i in range(1, ns):
            ev_done[i].record(streams[i])
            streams[0].wait_event(ev_done[i])

    # settle: clocks ramp up from idle over ~1 s
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    while True:
        run(n)
        ev1.record()
        ev1.synchronize()
        if ev0.elapsed_time(ev1) > 1500:
            break
    bad = 0
    for rnd in range(2):
        for chunk, ns in ((n, 1), (500_000, 1), (500_000, 2), (250_000, 2), (250_000, 4), (125_000, 4)):
            out_items.fill_(0)
            run(chunk, ns)
            torch.cuda.synchronize()
            same = bool(torch.equal(out_items[:total], ref_items))
            bad += not same
            ts = []
            for _ in range(15):
                ev0.record()
                run(chunk, ns)
                ev1.record()
                ev1.synchronize()
                ts.append(ev0.elapsed_time(ev1))
            ts.sort()
            print(json.dumps({"round": rnd, "chunk_frames": chunk, "streams": ns, "calls": (n + chunk - 1) // chunk,
                              "ms_median": round(ts[len(ts) // 2], 4), "ms_min": round(ts[0], 4),
                              "items_equal": same}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
