"""A/B of the 8-lane varlen kernel's sort window (UFC_V8_SORTW, tuning build) on config 3.

Every variant's CRC words and valid flags must equal the product window's (64, which the -m gpu
suite checks against the oracle); then rounds of 10 back-to-back launches per variant, interleaved.
Run with UFC_LIB pointing at a tuning build.  Tuning probe, not product code."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch  # noqa: E402

from uflow_amd import synth  # noqa: E402
from uflow_amd.batch import FrameCrcEngine  # noqa: E402

# variants "window:aux" (aux 0: default-policy loads, 2: non-temporal)
WINDOWS = os.environ.get("SORTW_LIST", "64:0,8:0,16:0,32:0").split(",")
SEAL = os.environ.get("SORTW_SEAL", "0") == "1"
ROUNDS = int(os.environ.get("SORTW_ROUNDS", "6"))

eng = FrameCrcEngine(0)
n = 10_000_000
data, off = synth.varlen_batch(n, 64, 1500, synth.SEED_CONFIG3, device="cuda")
crc = torch.empty(n, dtype=torch.int32, device="cuda")
val = torch.empty(n, dtype=torch.uint8, device="cuda")


def run(w):
    sw, aux = w.split(":")
    os.environ["UFC_V8_SORTW"] = sw
    os.environ["UFC_V8_AUX"] = aux
    if SEAL:
        eng.seal_varlen(data, off, crc_out=crc)
    else:
        eng.crc_varlen(data, off, crc_out=crc, valid_out=val)


ref = None
for w in WINDOWS:
    crc.fill_(0)
    val.fill_(7)
    run(w)
    torch.cuda.synchronize()
    got = (crc.clone(), val.clone())
    if ref is None:
        ref = got
    else:
        same = torch.equal(ref[0], got[0]) and (SEAL or torch.equal(ref[1], got[1]))
        print(json.dumps({"window": w, "identical_to": WINDOWS[0], "ok": bool(same)}), flush=True)
        if not same and os.environ.get("SORTW_NOCHECK") != "1":  # (ablation builds compute garbage)
            sys.exit(1)

times = {w: [] for w in WINDOWS}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(ROUNDS):
    for w in WINDOWS:
        for _ in range(3):
            run(w)
        e0.record()
        for _ in range(10):
            run(w)
        e1.record()
        e1.synchronize()
        times[w].append(e0.elapsed_time(e1) / 10)
for w in WINDOWS:
    t = sorted(times[w])
    print(json.dumps({"window": w, "seal": SEAL, "median_ms": round(t[len(t) // 2], 4), "min_ms": round(t[0], 4)}),
          flush=True)
