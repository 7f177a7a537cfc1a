"""Static instruction counts of K1's main loop (design tool, no GPU needed).

Compiles pk_step.hip for gfx950 to assembly (or reads a given .s), finds the step kernel's outer
loop (the depth-1 loop with the most blocks), and counts by class the instructions on its fall-through
path from the header round to the header again (conditional branches not taken, s_branch followed).
Rare paths the compiler moved out of line (PK_RARE blocks) are not counted; in-line conditional
blocks are, so this is an upper bound of the common path.
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


def kernel_text(lines, prio, all_=0, small=False):
    name = (f"_Z20pk_step_kernel_smallILb{prio}ELb{all_}EEv10PkStepArgs:" if small
            else f"_Z14pk_step_kernelILb{prio}ELb{all_}EEv10PkStepArgs:")
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
    ap.add_argument("--all", type=int, default=0, help="1: the every-bank-staged instance (ALL)")
    ap.add_argument("--small", action="store_true", help="the small-LDS K1 (compiled with -DPK_K1_SMALL)")
    ap.add_argument("--s", default=None)
    ap.add_argument("--blocks", action="store_true")
    ap.add_argument("--dump", default=None, help="write the common path's instructions to this file")
    ap.add_argument("extra", nargs="*")
    a = ap.parse_args()
    path = a.s or compile_s(a.extra + (["-DPK_K1_SMALL"] if a.small else []))
    lines = open(path).read().splitlines()
    K = kernel_text(lines, a.prio, a.all, a.small)
    # the outer loop: the "Loop Header: Depth=1" label with the most blocks annotated as its body
    heads = [(i, re.match(r"^\.LBB(\d+_\d+):", l).group(1)) for i, l in enumerate(K) if "Loop Header: Depth=1" in l]
    i0, hb = max(heads, key=lambda h: sum(f"Header=BB{h[1]} Depth=1" in l for l in K))
    labels = {re.match(r"^(\.LBB\d+_\d+):", l).group(1): i for i, l in enumerate(K) if re.match(r"^\.LBB\d+_\d+:", l)}
    # the common path: from the header, fall through every conditional branch (in-line blocks are
    # taken, rare blocks the compiler moved out of line are skipped) and follow s_branch, until the
    # header comes round again (a rotated loop reaches it through a latch block laid out before it)
    cnt, blocks, cur = Counter(), [], None
    path = []
    i, seen = i0, set()
    while True:
        s = K[i].strip()
        if i == i0 and i in seen:
            break
        if i in seen:
            raise SystemExit(f"walk revisits line {i}")
        seen.add(i)
        if re.match(r"^\.LBB\d+_\d+:", s) or s.startswith("; %bb."):
            cur = [s.split()[0] if s.startswith(".") else s.split(":")[0], Counter()]
            blocks.append(cur)
            i += 1
            continue
        i += 1
        if not s or s.startswith(";") or s.startswith("."):
            continue
        c = classify(s)
        path.append(s)
        cnt[c] += 1
        if cur:
            cur[1][c] += 1
        op = s.split()[0]
        if op == "s_branch" or (op.startswith("s_cbranch") and s.split()[1] == f".LBB{hb}"):
            i = labels[s.split()[1]]   # jumps, and the back-edge of a loop closed by a conditional branch
    i1 = i
    tot = sum(v for k, v in cnt.items() if k not in ("waitcnt", "nop"))
    print(f"loop header line {i0}, common path: issued {tot}  " + "  ".join(f"{k} {cnt[k]}" for k in
          ("valu", "salu", "branch", "lds", "vmem", "smem", "waitcnt", "nop", "misc", "other") if cnt[k]))
    if a.dump:
        open(a.dump, "w").write("\n".join(path) + "\n")
    if a.blocks:
        for name, c in blocks:
            print(f"  {name:12s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
