"""Print per-wave, per-emulated-instruction PMC counts of K1 from tools/gpu_pmc_mix.sh output."""
import json
import subprocess
import sys

for tag in sys.argv[1:]:
    d = json.loads(subprocess.check_output(["python3", "tools/pmc_summary.py", f"gpurun_out/pmc_{tag}"]))["pk_step_kernel"]
    js = json.load(open(f"gpurun_out/pmc_{tag}/a.json"))
    ipe, w = js["instr_per_env_step"], d["SQ_WAVES"]
    keys = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
            "SQ_INSTS_SMEM", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"]
    print(tag, "ms/step", js["ms_per_step"], " ".join(f"{k.replace('SQ_', '').replace('INSTS_', '')}={d[k] / w / ipe:.1f}" for k in keys if k in d))
