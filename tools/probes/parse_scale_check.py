"""parse_scale_check.py -- the device parse against the native host parse on the codec test batch tiled
1, 10 and 340 times (600 to 204k frames), printing the frames whose infos differ; exits non-zero if any
do.  (A stress check used to chase a nondeterministic walk variant, profiles/EXPERIMENTS.md; the same
comparison at 340 tiles is tests/test_gpu_parity.py::test_parse_varlen_vs_host_parse_large.)
Run on the GPU box: python tools/probes/parse_scale_check.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
from test_gpu_parity import _codec_batch  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402
from uflow_amd.frame import FRAME_INFO_DTYPE, parse_batch_host  # noqa: E402


def main():
    eng = FrameCrcEngine(0)
    frames, data, offsets = _codec_batch(10, 600)
    lens = np.diff(offsets)
    total_bad = 0
    for reps in (1, 10, 340):
        big = np.tile(data, reps)
        offs = np.zeros(len(lens) * reps + 1, dtype=np.int64)
        offs[1:] = np.cumsum(np.tile(lens, reps))
        d = torch.from_numpy(big).cuda()
        o = torch.from_numpy(offs).cuda()
        _, valid = eng.crc_varlen(d, o)
        infos, _, _ = eng.parse_varlen(d, o, valid)
        torch.cuda.synchronize()
        gi = infos.cpu().numpy().view(FRAME_INFO_DTYPE).reshape(-1)
        ri, _ = parse_batch_host(big, offs.astype(np.uint64), valid.cpu().numpy(), nthreads=8)
        bad = np.nonzero((gi.view(np.uint8).reshape(len(gi), -1) != ri.view(np.uint8).reshape(len(ri), -1)).any(1))[0]
        print("reps", reps, "frames", len(gi), "bad infos", bad.size, bad[:10], flush=True)
        for b in bad[:3]:
            print(" frame", b, "len", lens[b % 600], "kind", big[offs[b]], "gpu", gi[b], "host", ri[b])
        total_bad += bad.size
    sys.exit(1 if total_bad else 0)


if __name__ == "__main__":
    main()
