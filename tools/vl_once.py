"""Config 3 (10M frames, lengths U[64,1500], seed 0x5EED0002) through ufc_crc_batch_varlen, a few
launches and nothing else: the command profiled by rocprofv3 (kernel trace, PMC passes)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from uflow_amd.batch import FrameCrcEngine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    eng = FrameCrcEngine(0)
    n = int(os.environ.get("VL_N", 10_000_000))
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0002)
    lens = torch.randint(64, 1501, (n,), generator=g, device=dev, dtype=torch.int64)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    offsets[1:] = torch.cumsum(lens, 0)
    data = torch.randint(0, 256, (int(offsets[-1]),), generator=g, device=dev, dtype=torch.uint8)
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    for _ in range(int(os.environ.get("VL_REPS", 5))):
        eng.crc_varlen(data, offsets, crc_out=crc, valid_out=valid)
    torch.cuda.synchronize()
    print("bytes", int(offsets[-1]), "frames", n)
    eng.close()


if __name__ == "__main__":
    main()
