"""K1's register / scratch / LDS budget and where its spills live (design tool, no GPU needed).

Compiles pk_step.hip for gfx950 both ways build.py does (the default kernel and the small-LDS one,
-DPK_K1_SMALL) with -Rpass-analysis=kernel-resource-usage, then reads the assembly:
  * per kernel instance: VGPRs, SGPRs, SGPR spills, scratch bytes per lane, occupancy, LDS;
  * which functions of the code object issue scratch_* instructions;
  * on the main loop's common path (tools/isa_count.py's walk): scratch_* and SGPR-spill lane
    moves (v_writelane / v_readlane), i.e. whether the spills cost the loop anything.
usage: python tools/k1_resources.py [> profiles/rNN/k1_resource_usage.txt]"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "tools"))
import isa_count as IC  # noqa: E402

SRC = os.path.join(HERE, "pokegym_amd", "csrc", "pk_step.hip")
HIPCC = "/opt/rocm/bin/hipcc"
FIELDS = ("TotalSGPRs", "VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill",
          "VGPRs Spill", "LDS Size [bytes/block]")


def resource_usage(defs, tmp):
    out = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "-Rpass-analysis=kernel-resource-usage",
                          "-o", os.path.join(tmp, "k.o"), SRC] + defs, capture_output=True, text=True, check=True)
    rows, cur = [], None
    for ln in out.stderr.splitlines():
        m = re.search(r"remark: +Function Name: (\S+)", ln)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark: +([^:]+): (\d+)", ln)
        if m and cur is not None and m.group(1).strip() in FIELDS:
            cur[m.group(1).strip()] = int(m.group(2))
    return rows


def asm(defs, tmp):
    path = os.path.join(tmp, "k.s")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    "-Wno-unused-command-line-argument", "-o", path, SRC] + defs, check=True)
    return open(path).read().splitlines()


def scratch_by_function(lines):
    cnt, fn = Counter(), None
    for ln in lines:
        m = re.match(r"^([_A-Za-z][_A-Za-z0-9]*):", ln)
        if m and not ln.startswith(".L"):
            fn = m.group(1)
        s = ln.strip()
        if s.startswith("scratch_"):
            cnt[(fn, "scratch")] += 1
        elif s.startswith("v_writelane_b32") or s.startswith("v_readlane_b32"):
            cnt[(fn, "lane_spill_moves")] += 1
    return cnt


def common_path(lines, prio, all_, small):
    K = IC.kernel_text(lines, prio, all_, small)
    heads = [(i, re.match(r"^\.LBB(\d+_\d+):", l).group(1)) for i, l in enumerate(K) if "Loop Header: Depth=1" in l]
    i0, hb = max(heads, key=lambda h: sum(f"Header=BB{h[1]} Depth=1" in l for l in K))
    labels = {re.match(r"^(\.LBB\d+_\d+):", l).group(1): i for i, l in enumerate(K) if re.match(r"^\.LBB\d+_\d+:", l)}
    path, i, seen = [], i0, set()
    while True:
        if i == i0 and i in seen:
            break
        seen.add(i)
        s = K[i].strip()
        i += 1
        if not s or s.startswith(";") or s.startswith(".") or re.match(r"^\.LBB", s):
            continue
        path.append(s)
        op = s.split()[0]
        if op == "s_branch" or (op.startswith("s_cbranch") and s.split()[1] == f".LBB{hb}"):
            i = labels[s.split()[1]]
    return path


def main():
    with tempfile.TemporaryDirectory() as tmp:
        for small in (False, True):
            defs = ["-DPK_K1_SMALL"] if small else []
            print(f"== {'small-LDS K1 (-DPK_K1_SMALL)' if small else 'default K1'} ==")
            for r in resource_usage(defs, tmp):
                print(f"  {r['name']}: " + ", ".join(f"{k} {r.get(k)}" for k in FIELDS))
            lines = asm(defs, tmp)
            sc = scratch_by_function(lines)
            for (fn, kind), v in sorted(sc.items()):
                print(f"  {kind:17s} instructions in {fn}: {v}")
            for prio in (0, 1):
                for all_ in (0, 1):
                    try:
                        p = common_path(lines, prio, all_, small)
                    except StopIteration:
                        continue
                    ns = sum(s.startswith("scratch_") for s in p)
                    nl = sum(s.startswith("v_writelane") or s.startswith("v_readlane") for s in p)
                    print(f"  common path <PRIO={prio}, ALL={all_}>: {len(p)} instructions, scratch {ns}, "
                          f"SGPR-spill lane moves {nl}")


if __name__ == "__main__":
    main()
