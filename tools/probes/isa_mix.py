"""Static instruction mix of one kernel in a hipcc --save-temps .s file: totals by class and the most
frequent opcodes, and per basic block (label) the VALU / LDS / VMEM counts of the largest blocks.
Usage: python tools/probes/isa_mix.py <file.s> <kernel-symbol substring> [top]"""
import re
import sys
from collections import Counter


def kernel_body(path, sub):
    lines = open(path).read().splitlines()
    start = next(i for i, ln in enumerate(lines) if re.match(r"^_Z\S*:", ln) and sub in ln.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def main():
    body = kernel_body(sys.argv[1], sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    blocks, cur = {}, "entry"
    ops = Counter()
    for ln in body:
        if re.match(r"^\.LBB\S*:", ln):
            cur = ln.split(":")[0]
            continue
        t = ln.strip()
        if not ln.startswith(("\t", " ")) or not t or t.startswith((".", ";")):
            continue
        op = t.split()[0]
        ops[op] += 1
        blocks.setdefault(cur, Counter())[op] += 1

    def cls(c):
        return (sum(v for k, v in c.items() if k.startswith("v_")), sum(v for k, v in c.items() if k.startswith("ds_")),
                sum(v for k, v in c.items() if k.startswith(("buffer_", "global_"))),
                sum(v for k, v in c.items() if k.startswith("s_")))

    va, ds, vm, sa = cls(ops)
    print(f"total {sum(ops.values())}  VALU {va}  LDS {ds}  VMEM {vm}  SALU/branch {sa}")
    for k, v in ops.most_common(top):
        print(f"  {k:28s} {v}")
    print("largest blocks (VALU, LDS, VMEM, SALU):")
    for name, c in sorted(blocks.items(), key=lambda kv: -sum(kv[1].values()))[:top]:
        print(f"  {name:16s} {cls(c)}")


if __name__ == "__main__":
    main()
