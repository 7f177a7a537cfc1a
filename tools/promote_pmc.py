"""Promote a round profile run to profiles/pmc_<w>.json (the file bench.py cites for roofline.traffic,
roofline.issue and pmc_stamp), with its source line.

usage: python tools/promote_pmc.py TAG WORKLOAD...
For a VecEnv workload (config3/4/5) whose profiles/TAG/pmc_<w>_2wps.json exists, the promoted record
is that one — the K1 counters at the occupancy the timed steps run (two small-LDS workgroups per CU,
two waves per SIMD: the whole handle through the small-LDS kernel as one launch) — and the
serialised per-sub-batch record (rocprofv3 --pmc serialises the bench's two concurrent sub-batch
launches: one wave per SIMD, half the working set) is nested beside it as `serialised_record`."""
import json
import os
import sys

KEYS = ("hbm_bytes_per_env_step_k1", "k1_read_bytes", "k1_write_bytes", "envs_per_launch", "valu_busy_pct",
        "valu_utilization_pct", "wait_any_pct", "waves_per_launch", "k1_avg_ms_rocprof_stats", "issue", "bench_under_rocprof")


def main():
    tag, names = sys.argv[1], sys.argv[2:]
    for w in names:
        ser_path = f"profiles/{tag}/pmc_{w}.json"
        conc_path = f"profiles/{tag}/pmc_{w}_2wps.json"
        ser = json.load(open(ser_path))
        ser["source"] = (f"{ser_path} + profiles/{tag}/{w}_kernel_stats.csv (rocprofv3 run {tag}: tools/gpu_round_prof.sh, "
                         "tools/round_pmc.py)")
        json.dump(ser, open(ser_path, "w"), indent=1)
        d = ser
        if os.path.exists(conc_path):
            d = json.load(open(conc_path))
            d["source"] = (f"{conc_path} + profiles/{tag}/{w}_2wps_kernel_stats.csv (rocprofv3 run {tag}: "
                           "tools/gpu_round_final.sh conc, tools/round_pmc.py)")
            d["regime"] = ("two waves per SIMD, the occupancy of the bench's timed steps: the whole handle through the "
                           "small-LDS K1 as ONE launch (PK_K1_SMALL=1, VecEnv batch = all envs), two 256-thread "
                           "workgroups per CU — what the two concurrent sub-batch launches of the timed steps hold "
                           "together; rocprofv3 --pmc serialises those launches, so they cannot be counted as they run")
            d["serialised_record"] = {**{k: ser[k] for k in KEYS if k in ser}, "source": ser["source"],
                                      "regime": "one sub-batch launch alone (rocprofv3 --pmc serialises dispatches): one "
                                                "wave per SIMD, half the working set"}
            json.dump(d, open(conc_path, "w"), indent=1)
        json.dump(d, open(f"profiles/pmc_{w}.json", "w"), indent=1)
        print(w, d["k1_avg_ms_rocprof_stats"], d.get("regime", "")[:40])


if __name__ == "__main__":
    main()
