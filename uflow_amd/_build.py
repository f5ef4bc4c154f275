"""In-tree build of the native library (libuflowcrc.so) and of the CPU oracle.

The library is compiled for gfx950 only (MI355X): hipcc --offload-arch=gfx950.  The .so lands
next to this file so that it travels with the repository snapshot to the GPU box.
"""
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libuflowcrc.so")
SOURCES = ["frame_crc.hip", "frame_crc_varlen8.hip", "frame_parse.hip", "hbm_probe.hip",
           "ufc_api.cpp", "ufc_shard.cpp", "crc_math.cpp", "frame_codec.cpp"]
HEADERS = ["frame_crc_dev.hpp", "frame_crc_kernels.hpp", "crc_math.hpp", "frame_codec_core.hpp", "frame_parse.hpp",
           "ufc_internal.hpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _digest(paths, extra=()):
    """sha256 over the named files' contents (and extra strings): the build's identity."""
    import hashlib
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.relpath(p, REPO_DIR).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    for x in extra:
        h.update(str(x).encode() + b"\0")
    return h.hexdigest()


def _stamp_ok(target, digest):
    """Whether <target>.sha256 records `digest` (its first line)."""
    try:
        with open(target + ".sha256") as f:
            return os.path.exists(target) and f.readline().strip() == digest
    except OSError:
        return False


def _stamp_defines(target):
    """The -D defines recorded in <target>.sha256 (second line, "defines: A B=1 ..."), or ()."""
    try:
        with open(target + ".sha256") as f:
            f.readline()
            line = f.readline().strip()
    except OSError:
        return ()
    return tuple(line[len("defines:"):].split()) if line.startswith("defines:") else ()


def _native_identity(defines=()):
    """(sources, hipcc flags, digest) of a native build from the sources in this tree."""
    sources = list(SOURCES)
    deps = [os.path.join(CSRC, s) for s in sources + HEADERS]
    deps += [os.path.join(REPO_DIR, "include", h) for h in ("uflow_frame_crc.h", "uflow_frame_codec.h")]
    # No atomic optimizer: the lean kernel's single-lane claim atomics must stay plain
    # global_atomic_add (the optimizer reads the result back at once, forcing a vmcnt(0) wait).
    flags = [HIPCC, "-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-Wall",
             "-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]
    flags += ["-D" + d for d in defines]
    per_source = {s: list(UNSTRUCTURED_FLAGS) for s in UNSTRUCTURED_SOURCES}
    extra = [f"{s}:{' '.join(per_source[s])}" for s in sorted(per_source)]
    return sources, flags, per_source, _digest(deps + [os.path.abspath(__file__)], flags[1:] + extra)


# Uniform branches left unstructured, per source: the variable-length kernel's set-level branches (a
# switch on the set's line count, masked or plain steps) otherwise get "Flow" blocks that copy the
# chain registers at every merge (1.585 against 1.484 ms on config 3, profiles/EXPERIMENTS.md).  The
# fixed kernels of frame_crc.hip were measured with it (round 5: the bench kernel's 224.8 us), so it
# stays there too; the parse (frame_parse.hip) and the probe build without it (a non-default
# option is applied only where it was measured).
UNSTRUCTURED_FLAGS = ("-mllvm", "-structurizecfg-skip-uniform-regions=true")
UNSTRUCTURED_SOURCES = ("frame_crc_varlen8.hip", "frame_crc.hip")


def build_native(force=False, verbose=False, out=None, defines=()):
    """`defines` adds -D flags (an experiment build, meant with `out` pointing away from the product
    library).

    Rebuilds when the sha256 of the sources, headers, flags and this file differs from the one
    recorded beside the library (<lib>.sha256), not by file times: a library copied to another
    machine (the GPU box) with its stamp is rebuilt there only if it does not match the source."""
    sources, flags, per_source, digest = _native_identity(defines)
    target = out or LIB_PATH
    if not force and _stamp_ok(target, digest):
        return target
    # One object per source, compiled in parallel, then one link (every object: the stamp differs).
    objdir = os.path.join(REPO_DIR, "build", "obj_" + os.path.basename(target).replace(".", "_"))
    os.makedirs(objdir, exist_ok=True)
    jobs, objs = [], []
    for src in sources:
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        jobs.append(flags + per_source.get(src, []) + ["-c", os.path.join(CSRC, src), "-o", obj])
    from concurrent.futures import ThreadPoolExecutor

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        return subprocess.run(cmd).returncode

    with ThreadPoolExecutor(max_workers=max(1, min(8, len(jobs)))) as ex:
        rcs = list(ex.map(run, jobs))
    if any(rcs):
        raise subprocess.CalledProcessError(max(rcs), "hipcc")
    link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", target + ".tmp"] + objs + ["-ldl"]
    if verbose:
        print(" ".join(link), file=sys.stderr)
    subprocess.run(link, check=True)
    os.replace(target + ".tmp", target)
    with open(target + ".sha256", "w") as f:
        f.write(digest + "\n")
        if defines:
            f.write("defines: " + " ".join(defines) + "\n")
    return target


LOOPBACK_SRC = os.path.join(REPO_DIR, "tools", "loopback", "ufc_loopback.cpp")
LOOPBACK_BIN = os.path.join(REPO_DIR, "tools", "loopback", "ufc_loopback")


def build_tools(force=False, verbose=False):
    """The loopback harness (BASELINE.json configs 1 and 5), linked against the in-tree library."""
    deps = [LOOPBACK_SRC] + [os.path.join(REPO_DIR, "include", h) for h in ("uflow_frame_crc.h", "uflow_frame_codec.h")]
    cmd = [HIPCC, "-O2", "-std=c++17", "-Wall", "-o", LOOPBACK_BIN + ".tmp", LOOPBACK_SRC,
           "-L" + PKG_DIR, "-luflowcrc", "-Wl,-rpath,$ORIGIN/../../uflow_amd", "-lpthread"]
    digest = _digest(deps + [os.path.abspath(__file__)], cmd[1:])
    if not force and _stamp_ok(LOOPBACK_BIN, digest):
        return LOOPBACK_BIN
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LOOPBACK_BIN + ".tmp", LOOPBACK_BIN)
    with open(LOOPBACK_BIN + ".sha256", "w") as f:
        f.write(digest + "\n")
    return LOOPBACK_BIN


def build_oracle(force=False):
    odir = os.path.join(REPO_DIR, "oracle")
    target = os.path.join(odir, "liboracle.so")
    digest = _digest([os.path.join(odir, "crc_oracle.c"), os.path.join(odir, "Makefile")])
    if force or not _stamp_ok(target, digest):
        subprocess.run(["make", "-C", odir, "-s", "-B"], check=True)
        with open(target + ".sha256", "w") as f:
            f.write(digest + "\n")
    return target


if __name__ == "__main__":
    build_native(force="--force" in sys.argv, verbose=True)
    build_oracle(force="--force" in sys.argv)
    build_tools(force="--force" in sys.argv, verbose=True)
    print(LIB_PATH)
