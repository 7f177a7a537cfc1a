"""Summarise tools/gpu_pmc_k1.sh passes for K1 (pk_step_kernel): per-wave cost per emulated
instruction (issued ISA instructions by class, cycles, waits), effective clock.  usage: python tools/pmc_k1.py gpurun_out/pmck_TAG [names...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def kernel_means(d, kernel="pk_step_kernel"):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if kernel not in row["Kernel_Name"]:
                continue
            vals[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    durs = {}
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for row in csv.DictReader(open(f)):
            if kernel in row["Kernel_Name"]:
                durs[row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    # the last dispatch of the run (steady state), counters summed over dimensions
    last = sorted(vals, key=int)[-1]
    return dict(vals[last]), durs.get(last)


def summary(root, name, cus=256):
    a, dur = kernel_means(os.path.join(root, f"{name}_a"))
    b, _ = kernel_means(os.path.join(root, f"{name}_b"))
    c = {**a, **b}
    bench = json.loads(open(os.path.join(root, f"{name}_a.json")).read().strip().splitlines()[-1])
    waves = c["SQ_WAVES"]
    envs = bench["config"]["envs_per_gpu"]
    # per emulated SM83 instruction of a lane: a wave runs its lanes' instructions side by side, so
    # wave instructions / (instructions one env executes per launch).  (Round 2 divided by loop
    # iterations, estimated as 1.09 x instructions; with fused instruction pairs a loop iteration
    # now executes ~1.37 instructions, so the per-instruction figure is the comparable one: round 2's
    # rows x 1.09 ~ per-instruction values.)
    iters = bench["instr_per_env_step"]
    clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / dur if dur else 0
    per = lambda k: c.get(k, 0) / waves / iters
    out = {
        "name": name, "envs": envs, "waves": waves, "k1_ms": round(dur * 1e3, 2) if dur else None,
        "clock_GHz": round(clk / 1e9, 3),
        "per": "emulated instruction",
        "wave_cycles_per_instr": round(4 * per("SQ_WAVE_CYCLES"), 1),
        "active_any": round(4 * per("SQ_ACTIVE_INST_ANY"), 1),
        "wait_any": round(4 * per("SQ_WAIT_ANY"), 1),
        "wait_inst_any": round(4 * per("SQ_WAIT_INST_ANY"), 1),
        "valu": round(per("SQ_INSTS_VALU"), 1), "salu": round(per("SQ_INSTS_SALU"), 1),
        "branch": round(per("SQ_INSTS_BRANCH"), 1), "lds": round(per("SQ_INSTS_LDS"), 1),
        "vmem_rd": round(per("SQ_INSTS_VMEM_RD"), 2), "vmem_wr": round(per("SQ_INSTS_VMEM_WR"), 2),
        "valu_busy_pct": round(100 * c.get("SQ_ACTIVE_INST_VALU", 0) * 4 / (4 * cus) / max(c.get("GRBM_GUI_ACTIVE", 1) / 8, 1), 1),
    }
    return out


if __name__ == "__main__":
    root = sys.argv[1]
    names = sys.argv[2:] or sorted({os.path.basename(p)[:-2] for p in glob.glob(os.path.join(root, "*_a")) if os.path.isdir(p)})
    for n in names:
        print(json.dumps(summary(root, n)))
