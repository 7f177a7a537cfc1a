"""Static instruction counts of K1's main loop (design tool, no GPU needed).

Compiles pk_step.hip for gfx950 to assembly (or reads a given .s), finds the step kernel's outer
loop (the largest depth-1 loop), and counts the instructions laid out between its header and its
back-edge by class.  Rare paths the compiler moved out of line (PK_RARE blocks after the loop) are
not counted; in-line conditional blocks are, so this is an upper bound of the common path.
usage: python tools/isa_count.py [--prio 0|1] [--s file.s] [--blocks] [-- extra hipcc flags]"""
import argparse
import os
import re
import subprocess
import sys
from collections import Counter

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(HERE, "pokegym_amd", "csrc", "pk_step.hip")


def compile_s(extra, out="/tmp/pk_isa/pk_step.s"):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
           "-Wno-unused-command-line-argument", "-o", out, SRC] + extra
    subprocess.run(cmd, check=True)
    return out


def kernel_text(lines, prio):
    name = f"_Z14pk_step_kernelILb{prio}EEv10PkStepArgs:"
    start = next(i for i, l in enumerate(lines) if l.startswith(name))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith("; codeLenInByte") or ".Lfunc_end" in lines[i])
    return lines[start:end]


def classify(ins):
    op = ins.split()[0]
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op == "s_nop":
        return "nop"
    if op.startswith("s_setprio") or op.startswith("s_sleep"):
        return "misc"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_") or op.startswith("scratch_"):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "smem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prio", type=int, default=1)
    ap.add_argument("--s", default=None)
    ap.add_argument("--blocks", action="store_true")
    ap.add_argument("extra", nargs="*")
    a = ap.parse_args()
    path = a.s or compile_s(a.extra)
    lines = open(path).read().splitlines()
    K = kernel_text(lines, a.prio)
    # loops: header labels with "Loop Header: Depth=1"; body ends at the last branch back to it
    best = None
    for i, l in enumerate(K):
        m = re.match(r"^(\.LBB\d+_\d+):.*Loop Header: Depth=1", l)
        if not m:
            continue
        lab = m.group(1)
        back = [j for j in range(i, len(K)) if re.search(r"s_cbranch_\w+\s+" + re.escape(lab) + r"$", K[j].strip())]
        if back and (best is None or back[-1] - i > best[1] - best[0]):
            best = (i, back[-1])
    i0, i1 = best
    cnt, blocks, cur = Counter(), [], None
    for l in K[i0:i1 + 1]:
        s = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", s) or s.startswith("; %bb."):
            cur = [s.split()[0] if s.startswith(".") else s.split(":")[0], Counter()]
            blocks.append(cur)
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        c = classify(s)
        cnt[c] += 1
        if cur:
            cur[1][c] += 1
    tot = sum(v for k, v in cnt.items() if k not in ("waitcnt", "nop"))
    print(f"loop body lines {i0}-{i1}: issued {tot}  " + "  ".join(f"{k} {cnt[k]}" for k in
          ("valu", "salu", "branch", "lds", "vmem", "smem", "waitcnt", "nop", "misc", "other") if cnt[k]))
    if a.blocks:
        for name, c in blocks:
            print(f"  {name:12s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
