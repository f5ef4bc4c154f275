"""Config 5 like-for-like: the inline receive loops (server/mod.rs:591-602 on R
threads) with the CPU gate and with the asynchronous GPU gate, fed by PACED senders
(tools/loopback/ufc_loopback --rate-gbps): for each arm the offered rate is raised until the loss
exceeds the bound, and the arm's figure is the highest offered rate it took with loss <= the bound
(the ideal_transfer.rs:60-154 criterion is that everything arrives).  Both arms are thus compared at
equal delivered data.  One JSON line per run, then one summary line per (arm, threads).
Usage: python tools/config5_sweep.py [--threads 1,2] [--rates 0.5,1,...] [--frames-per-gb 700000]
"""
import argparse
import json
import os
import random
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tools", "loopback", "ufc_loopback")


def run(gate, threads, rate, frames, port, txr):
    cmd = [BIN, "--gate", gate, "--rx-threads", str(threads), "--tx-per-rx", str(txr), "--batch", "4096",
           "--frames", str(frames), "--corrupt-every", "997", "--port", str(port), "--rate-gbps", str(rate)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        raise RuntimeError(f"{' '.join(cmd)} failed: {p.stderr[-500:]}")
    return json.loads(lines[-1])


def summarize(runs, bound):
    """Per (arm, threads): the first offered rate whose run lost more than the bound (None: none did),
    and the lossless run with the highest delivered rate below it (paced runs, in sweep order)."""
    out, keys = [], []
    for j in runs:
        k = (j["arm"], j["rx_threads"])
        if k not in keys:
            keys.append(k)
    for arm, th in keys:
        rs = [j for j in runs if j["arm"] == arm and j["rx_threads"] == th]
        first_loss = next((j["offered_GB_s"] for j in rs if j["loss_frac"] > bound), None)
        ok = [j for j in rs if j["loss_frac"] <= bound and j["payload_mismatch"] == 0 and
              (first_loss is None or j["offered_GB_s"] < first_loss)]
        best = max(ok, key=lambda j: j["goodput_GB_s_sender_clock"]) if ok else None
        out.append({"summary": "config 5, paced senders: first offered rate with loss > %.3f and the best delivered "
                               "rate below it" % bound, "arm": arm, "rx_threads": th, "tx_threads": rs[0]["tx_threads"],
                    "first_lossy_offered_GB_s": first_loss,
                    "lossy_runs": sum(1 for j in rs if j["loss_frac"] > bound), "runs": len(rs),
                    "best_lossless_goodput_GB_s": best["goodput_GB_s_sender_clock"] if best else 0.0,
                    "at_offered_GB_s": best["offered_GB_s"] if best else None,
                    "gate_share_of_thread_time": best["gate_share_of_thread_time"] if best else None})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--summarize", help="re-summarize the sweep lines of a config5.jsonl instead of running")
    ap.add_argument("--threads", default="1,2")
    ap.add_argument("--rates", default="0.5,1.0,1.5,2.0,2.5,3.0,3.5,4.0,4.5,5.0,6.0")
    ap.add_argument("--seconds", type=float, default=1.5, help="target length of each run at its offered rate")
    ap.add_argument("--loss-bound", type=float, default=0.005)
    ap.add_argument("--tx-per-rx", type=int, default=2)
    a = ap.parse_args()
    if a.summarize:
        runs = [json.loads(ln) for ln in open(a.summarize) if ln.startswith("{")]
        runs = [j for j in runs if "arm" in j and "summary" not in j and j.get("offered_GB_s", 0) > 0]
        for s in summarize(runs, a.loss_bound):
            print(json.dumps(s), flush=True)
        return 0
    port = random.randrange(20000, 50000)
    runs = []
    for th in [int(x) for x in a.threads.split(",")]:
        for gate in ("cpu", "gpu"):
            best, fails = None, 0
            for rate in [float(x) for x in a.rates.split(",")]:
                frames = max(50_000, int(rate * 1e9 * a.seconds / 1472))
                port += 16
                j = run(gate, th, rate, frames, port, a.tx_per_rx)
                j["arm"] = gate
                runs.append(j)
                print(json.dumps(j), flush=True)
                if j["loss_frac"] <= a.loss_bound and j["payload_mismatch"] == 0:
                    best = j
                    fails = 0
                else:
                    fails += 1
                    if fails >= 2:
                        break
    for s in summarize(runs, a.loss_bound):
        print(json.dumps(s), flush=True)


if __name__ == "__main__":
    sys.exit(main())
