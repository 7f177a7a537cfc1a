"""Assemble profiles/pmc_<workload>.json (what bench.py reports as roofline.traffic and pmc_stamp)
from a tools/gpu_round_prof.sh run: K1 HBM bytes per launch (FETCH_SIZE + WRITE_SIZE, units
calibrated on a 1 GiB copy), VALUBusy / VALUUtilization by rocprofv3's derived-counter formulas
(gfx94x fallbacks, MI355X_MICROARCH.md §rocprofv3), the wave-parked (s_waitcnt) share, and the
per-launch K1 time of the stats pass.
usage: python tools/round_pmc.py gpurun_out/rprof_TAG NAME WORKLOAD_KEY > profiles/pmc_<key>.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

CU_NUM, MAX_WAVE = 256, 64


def per_dispatch(d, kernel):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if kernel in row["Kernel_Name"]:
                vals[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
    return vals


def sane(vals):
    """Drop dispatches whose SQ_WAVES is not the pass's median: a launch of fixed geometry has one wave
    count, and rocprofv3 once reported a K1 dispatch of 1,024 waves as 2,048 (profiles/r06q: every
    counter of that row doubled) — such a row would skew the means."""
    w = sorted(v["SQ_WAVES"] for v in vals.values() if "SQ_WAVES" in v)
    if not w:
        return vals
    med = w[len(w) // 2]
    return {k: v for k, v in vals.items() if v.get("SQ_WAVES", med) == med}


def mean(vals, key, skip_first=True):
    ids = sorted(vals)
    if skip_first and len(ids) > 1:
        ids = ids[1:]   # the first launch starts from the post-reset state
    xs = [vals[i][key] for i in ids if key in vals[i]]
    return sum(xs) / len(xs) if xs else None


def main():
    root, name, key = sys.argv[1], sys.argv[2], sys.argv[3]
    D = os.path.join(root, name)
    cf = mean(per_dispatch(os.path.join(root, "cfetch"), "__amd_rocclr_copyBuffer"), "FETCH_SIZE", False)
    cw = mean(per_dispatch(os.path.join(root, "cwrite"), "__amd_rocclr_copyBuffer"), "WRITE_SIZE", False)
    gib = float(1 << 30)
    fs, ws = gib / cf, gib / cw          # bytes per FETCH_SIZE / WRITE_SIZE unit (3 copies averaged)
    f = per_dispatch(os.path.join(D, "fetch"), "pk_step_kernel")
    w = per_dispatch(os.path.join(D, "write"), "pk_step_kernel")
    v = sane(per_dispatch(os.path.join(D, "valu"), "pk_step_kernel"))
    rd, wr = mean(f, "FETCH_SIZE") * fs, mean(w, "WRITE_SIZE") * ws
    # rocprofv3's VALUBusy: 100 * sum(SQ_ACTIVE_INST_VALU) / CU_NUM / max(GRBM_GUI_ACTIVE); the
    # per-dispatch GRBM_GUI_ACTIVE here is summed over the 8 XCDs, so max = sum / 8
    busy = 100.0 * mean(v, "SQ_ACTIVE_INST_VALU") / CU_NUM / (mean(v, "GRBM_GUI_ACTIVE") / 8)
    util = 100.0 * mean(v, "SQ_THREAD_CYCLES_VALU") / (mean(v, "SQ_ACTIVE_INST_VALU") * MAX_WAVE)
    wait = 100.0 * mean(v, "SQ_WAIT_ANY") / mean(v, "SQ_WAVE_CYCLES")
    k1 = []
    for fcsv in glob.glob(os.path.join(D, "stats", "*kernel_stats.csv")):
        for row in csv.DictReader(open(fcsv)):
            if "pk_step_kernel" in row["Name"]:
                k1.append(float(row["AverageNs"]) / 1e6)
    bench = json.loads(open(os.path.join(D, "stats_bench.json")).read().strip().splitlines()[-1])
    # envs one K1 dispatch covers (a VecEnv sub-batch, or the whole shard)
    epl = bench["config"].get("vecenv_batch_size") or bench["config"]["envs_per_gpu"]
    # issue: ISA instructions a wave issues per emulated SM83 instruction of one of its envs
    # (SQ_INSTS_* / SQ_WAVES / the instructions one env executes in the launch)
    issue = None
    if os.path.isdir(os.path.join(D, "issue")):
        q = sane(per_dispatch(os.path.join(D, "issue"), "pk_step_kernel"))
        ib = json.loads(open(os.path.join(D, "issue_bench.json")).read().strip().splitlines()[-1])
        ipe = ib["instr_per_env_step"]
        waves = mean(q, "SQ_WAVES")
        per = {k.replace("SQ_INSTS_", "").lower(): round(mean(q, k) / waves / ipe, 1)
               for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                         "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM")}
        per["total"] = round(sum(per.values()), 1)
        issue = {"isa_per_emulated_instr": per, "instr_per_env_step": ipe,
                 "method": "rocprofv3 --pmc SQ_INSTS_* of the K1 launches after the first: wave instructions / "
                           "SQ_WAVES / emulated instructions per env (the device's instruction counter)"}
    out = {
        "workload": bench["config"]["workload"],
        "envs_per_gpu": bench["config"]["envs_per_gpu"],
        "rom": bench["config"]["rom"],
        "source": f"{os.path.relpath(root)}/{name} (tools/gpu_round_prof.sh; summarised by tools/round_pmc.py)",
        "method": "rocprofv3 --kernel-trace --pmc, one pass per counter group; per-dispatch means over the K1 launches "
                  "after the first; FETCH_SIZE / WRITE_SIZE units calibrated on a 1 GiB device copy (FETCH_SIZE "
                  "counts half of a wide read on gfx950; the calibration carries that factor)",
        "calibration": {"FETCH_SIZE_per_GiB": cf, "WRITE_SIZE_per_GiB": cw},
        "k1_read_bytes": int(rd), "k1_write_bytes": int(wr),
        "hbm_bytes_per_launch_k1": int(rd + wr),
        "envs_per_launch": epl,
        "hbm_bytes_per_env_step_k1": round((rd + wr) / epl, 1),
        "traffic_level": "FETCH_SIZE / WRITE_SIZE = the L2's memory-side (fabric) requests (TCC_EA0_RDREQ / _WRREQ): "
                         "L2 misses, served by the Infinity Cache (MALL) or HBM — MALL hits are counted",
        "valu_busy_pct": round(busy, 2),
        "valu_busy_formula": "100*sum(SQ_ACTIVE_INST_VALU)/CU_NUM/max(GRBM_GUI_ACTIVE) (rocprofv3 VALUBusy, gfx94x form)",
        "valu_utilization_pct": round(util, 2),
        "valu_utilization_formula": "100*sum(SQ_THREAD_CYCLES_VALU)/(sum(SQ_ACTIVE_INST_VALU)*64): active lanes per VALU "
                                    "instruction, out of 64 (a wave carries wave_lanes envs: 16, 32 or 64 by launch "
                                    "size, so at most wave_lanes/64)",
        "wait_any_pct": round(wait, 2),
        "issue": issue,
        "waves_per_launch": mean(v, "SQ_WAVES"),
        "k1_avg_ms_rocprof_stats": round(k1[0], 3) if k1 else None,
        "bench_under_rocprof": {"value": bench["value"], "k1_ms": bench["roofline"]["k1_ms"],
                                "span_ms": bench["roofline"]["span_ms"]},
        "note": "K1 loads/stores single bytes from divergent lanes (lane-interleaved images), an access width the "
                "1 GiB-copy calibration does not cover: the byte totals are request-granular upper estimates",
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
