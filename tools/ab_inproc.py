"""In-process A/B of frame-CRC library variants on ONE device buffer (tuning tool).

Separate bench processes differ by several % from allocation to allocation, so variants are
compared here on the same frames, interleaved, many times.  Each variant is a library path plus
environment overrides (tuning builds, -DUFC_TUNING): each variant gets its own context, created
with its overrides set (the kernel selection is read at ufc_ctx_create), and the overrides are
also set around its launches (the few knobs read per launch, e.g. UFC_V8_WAVES):

    python tools/ab_inproc.py [--varlen [--seal]] name=lib.so[,ENV=VAL...] ...

Prints, per variant, the median over rounds of the per-round median kernel time (HIP events on
the launch stream) and the min; validates the results of variants without an ablation.
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    lib.ufc_ctx_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.ufc_crc_batch_fixed.argtypes = [vp, vp, sz, sz, sz, vp, vp, vp]
    lib.ufc_crc_batch_varlen.argtypes = [vp, vp, vp, sz, vp, vp, vp]
    lib.ufc_seal_batch_fixed.argtypes = [vp, vp, sz, sz, sz, vp, vp]
    lib.ufc_seal_batch_varlen.argtypes = [vp, vp, vp, sz, vp, vp]
    return lib


def make_ctx(lib, env):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    ctx = ctypes.c_void_p()
    try:
        assert lib.ufc_ctx_create(ctypes.byref(ctx), 0) == 0
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    return ctx


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    varlen = "--varlen" in sys.argv
    seal = "--seal" in sys.argv  # (with --varlen: time ufc_seal_batch_varlen instead of the gate)
    rounds = int(os.environ.get("AB_ROUNDS", 8))
    reps = int(os.environ.get("AB_REPS", 20))
    variants = []
    for a in args:
        name, spec = a.split("=", 1)
        parts = spec.split(",")
        env = dict(p.split("=", 1) for p in parts[1:])
        variants.append((name, parts[0], env))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    loaded = {path: load(path) for _, path, _ in variants}
    libs = {name: (loaded[path], make_ctx(loaded[path], {k: v for k, v in env.items() if not k.startswith("OPT")}))
            for name, path, env in variants}
    for name, path, env in variants:  # OPT<k>=<v>: ufc_ctx_set_option(ctx, k, v)
        lib, ctx = libs[name]
        for k, v in env.items():
            if k.startswith("OPT"):
                lib.ufc_ctx_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
                assert lib.ufc_ctx_set_option(ctx, int(k[3:]), int(v)) == 0, (name, k, v)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0001)
    crc = valid = offs = None
    if varlen:
        n = int(os.environ.get("VL_N", 10_000_000))
        rng = np.random.default_rng(0x5EED0002)
        lens = rng.integers(int(os.environ.get("VL_MIN", 64)), int(os.environ.get("VL_MAX", 1500)) + 1, n).astype(np.uint64)
        o = np.zeros(n + 1, np.uint64)
        o[1:] = np.cumsum(lens)
        offs = torch.from_numpy(o.view(np.int64)).to(dev)
        frames = torch.randint(0, 256, (int(o[-1]),), dtype=torch.uint8, device=dev, generator=g)
        lib0, ctx0 = libs[variants[0][0]]
        assert lib0.ufc_seal_batch_varlen(ctx0, frames.data_ptr(), offs.data_ptr(), n, None, sp) == 0
        nbytes = int(o[-1])
    else:
        n, L = int(os.environ.get("FX_N", 1_000_000)), int(os.environ.get("FX_LEN", 1500))
        frames = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
        lib0, ctx0 = libs[variants[0][0]]
        assert lib0.ufc_seal_batch_fixed(ctx0, frames.data_ptr(), L, L, n, None, sp) == 0
        nbytes = n * L
    idx = torch.arange(0, n, 1000, device=dev)
    torch.cuda.synchronize()
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    valid = torch.empty(n, dtype=torch.uint8, device=dev)

    skip = int(os.environ.get("AB_SKIP", 0))  # frames skipped at the front (readable pad bytes)

    def launch(lib, ctx):
        if skip:
            r = lib.ufc_crc_batch_fixed(ctx, frames.data_ptr() + skip * L, L, L, n - skip, crc.data_ptr(),
                                        valid.data_ptr(), sp)
            assert r == 0
            return
        if varlen and seal:  # (sealing in place again writes the same trailers)
            r = lib.ufc_seal_batch_varlen(ctx, frames.data_ptr(), offs.data_ptr(), n, crc.data_ptr(), sp)
        elif varlen:
            r = lib.ufc_crc_batch_varlen(ctx, frames.data_ptr(), offs.data_ptr(), n, crc.data_ptr(),
                                         valid.data_ptr(), sp)
        else:
            r = lib.ufc_crc_batch_fixed(ctx, frames.data_ptr(), L, L, n, crc.data_ptr(), valid.data_ptr(), sp)
        assert r == 0

    times = {v[0]: [] for v in variants}
    first_out = [None]
    # settle: a GPU out of idle runs at reduced clocks for up to ~1 s (AB_SETTLE_MS)
    import time
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < float(os.environ.get("AB_SETTLE_MS", 1500)):
        for name, path, env in variants:
            launch(*libs[name])
        torch.cuda.synchronize()
    for rnd in range(rounds):
        for name, path, env in variants:
            saved = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            lib, ctx = libs[name]
            launch(lib, ctx)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for e0, e1 in evs:
                e0.record(stream)
                launch(lib, ctx)
                e1.record(stream)
            torch.cuda.synchronize()
            ts = [a.elapsed_time(b) for a, b in evs]
            times[name].append(float(np.median(ts)))
            if os.environ.get("AB_SEQ"):  # per-launch times of this round (sustained-load behaviour)
                print(f"# {name} round {rnd}: " + " ".join(f"{t:.3f}" for t in ts), flush=True)
            if rnd == 0 and "UFC_LEAN_ABL" not in env and "UFC_VL_ABL" not in env and "UFC_ABLATE" not in env:
                nv = int(valid.sum().item())
                same = ""
                if first_out[0] is None:
                    first_out[0] = (name, crc.clone(), valid.clone())
                else:
                    same = (f"; crc words and flags identical to {first_out[0][0]}'s: "
                            f"{bool(torch.equal(crc, first_out[0][1]) and torch.equal(valid, first_out[0][2]))}")
                print(f"# {name}: valid {nv} of {n}{same}", flush=True)
            for k, v in saved.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
    if varlen and seal:  # every variant sealed the same bytes in place: they must still validate
        lib0, ctx0 = libs[variants[0][0]]
        assert lib0.ufc_crc_batch_varlen(ctx0, frames.data_ptr(), offs.data_ptr(), n, crc.data_ptr(), valid.data_ptr(),
                                         sp) == 0
        torch.cuda.synchronize()
        print(f"# after every variant's seals: {int(valid.sum().item())} of {n} frames valid", flush=True)
    for name, _, _ in variants:
        t = np.array(times[name])
        print(f"{name:24s} median {np.median(t):.4f} ms  min {t.min():.4f}  max {t.max():.4f}  "
              f"{nbytes / np.median(t) / 1e6:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
