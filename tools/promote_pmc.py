"""Promote a round profile run: profiles/<tag>/pmc_<w>.json -> profiles/pmc_<w>.json (the file bench.py cites),
with its source line.  usage: python tools/promote_pmc.py TAG WORKLOAD..."""
import json, sys
tag, names = sys.argv[1], sys.argv[2:]
for w in names:
    d = json.load(open(f"profiles/{tag}/pmc_{w}.json"))
    d["source"] = (f"profiles/{tag}/pmc_{w}.json + profiles/{tag}/{w}_kernel_stats.csv (rocprofv3 run {tag}, the round's "
                   "final kernel: tools/gpu_round_prof.sh, tools/round_pmc.py)")
    json.dump(d, open(f"profiles/{tag}/pmc_{w}.json", "w"), indent=1)
    json.dump(d, open(f"profiles/pmc_{w}.json", "w"), indent=1)
    print(w, d["k1_avg_ms_rocprof_stats"])
