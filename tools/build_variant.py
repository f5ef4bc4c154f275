"""Build an experiment variant of libuflowcrc.so into var/<name>.so: the product sources copied to a
scratch tree, `file:old=>new` substitutions applied (each must match), compiled with the product's
flags.  A/B measurement only (tools/ab_inproc.py); the product library is never touched.
`file@path` replaces a source file of the copy with another file (e.g. an earlier round's, from git show);
VARIANT_FLAGS (environment) adds hipcc flags; VARIANT_NO_MLLVM drops the named `-mllvm` options.
`--ref <git ref>` first takes uflow_amd/csrc and include/ from that commit instead of the working tree (the
previous round's library, for an A/B against it).
Usage: python tools/build_variant.py <name> [--ref <commit>] 'frame_crc_varlen8.hip:old=>new' 'frame_parse.hip@/tmp/old.hip' ..."""
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from uflow_amd import _build  # noqa: E402


def main():
    name, subs = sys.argv[1], sys.argv[2:]
    d = tempfile.mkdtemp(prefix="ufc_var_")
    if subs[:1] == ["--ref"]:
        ref, subs = subs[1], subs[2:]
        arch = subprocess.run(["git", "-C", REPO, "archive", ref, "uflow_amd/csrc", "include"], check=True,
                              capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", d], input=arch, check=True)
    else:
        shutil.copytree(os.path.join(REPO, "uflow_amd", "csrc"), os.path.join(d, "uflow_amd", "csrc"))
        shutil.copytree(os.path.join(REPO, "include"), os.path.join(d, "include"))
    for sub in subs:
        if "@" in sub and ":" not in sub.split("@", 1)[0]:
            fn, src = sub.split("@", 1)
            shutil.copy(src, os.path.join(d, "uflow_amd", "csrc", fn))
            continue
        fn, rest = sub.split(":", 1)
        old, new = rest.split("=>", 1)
        p = os.path.join(d, "uflow_amd", "csrc", fn)
        s = open(p).read()
        assert old in s, f"{fn}: no match for {old!r}"
        open(p, "w").write(s.replace(old, new))
    sources, flags, per_source, _ = _build._native_identity()
    flags = flags + os.environ.get("VARIANT_FLAGS", "").split()
    drop = os.environ.get("VARIANT_NO_MLLVM", "").split()
    objs = []
    jobs = []
    for src in sources:
        obj = os.path.join(d, src + ".o")
        objs.append(obj)
        f = flags + per_source.get(src, [])
        for opt in drop:
            if opt in f:
                i = f.index(opt)
                assert f[i - 1] == "-mllvm", opt
                del f[i - 1:i + 1]
        jobs.append(f + ["-c", os.path.join(d, "uflow_amd", "csrc", src), "-o", obj])
    with ThreadPoolExecutor(8) as ex:
        rcs = list(ex.map(lambda c: subprocess.run(c).returncode, jobs))
    assert not any(rcs), rcs
    os.makedirs(os.path.join(REPO, "var"), exist_ok=True)
    out = os.path.join(REPO, "var", name + ".so")
    subprocess.run([_build.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs + ["-ldl"], check=True)
    shutil.rmtree(d)
    print(out)


if __name__ == "__main__":
    main()
