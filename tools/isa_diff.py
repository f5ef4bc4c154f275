"""Per-kernel ISA comparison of two gfx950 assembly files (hipcc --cuda-device-only -S).

    python tools/isa_diff.py a.s b.s [substring]      # kernels whose instruction streams differ
    python tools/isa_diff.py --count a.s [substring]  # instruction mix per kernel (VALU/SALU/LDS/VMEM)

Used to check that a build flag or a source change leaves a kernel's code alone (DESIGN.md,
profiles/EXPERIMENTS.md), and to count a loop's instructions by class.  CPU only.
"""
import re
import sys


def kernels(path):
    s = open(path).read()
    out = {}
    for m in re.finditer(r"^(_Z\S+):", s, re.M):
        name = m.group(1)
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]
        lines = []
        for l in body.split("\n"):
            l = l.split(";")[0].strip()
            if not l or l.startswith("."):
                continue
            lines.append(l)
        out[name] = lines
    return out


def classify(ins):
    op = ins.split()[0]
    if op.endswith(":"):
        return None
    if op.startswith(("v_",)):
        return "VALU"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep", "s_setprio", "s_sched")):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "VMEM"
    return "other"


def count(lines):
    c = {}
    for l in lines:
        k = classify(l)
        if k:
            c[k] = c.get(k, 0) + 1
    return c


def main(argv):
    if argv and argv[0] == "--count":
        ks = kernels(argv[1])
        sub = argv[2] if len(argv) > 2 else ""
        for k, v in ks.items():
            if sub in k:
                print(k[:100], count(v))
        return 0
    a, b = kernels(argv[0]), kernels(argv[1])
    sub = argv[2] if len(argv) > 2 else ""
    rc = 0
    for k in a:
        if sub not in k:
            continue
        same = a[k] == b.get(k)
        if not same:
            rc = 1
        print("same" if same else "DIFF", k[:100], len(a[k]), len(b.get(k, [])))
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
