import json, subprocess, sys
for tag in sys.argv[1:]:
    d = json.loads(subprocess.check_output(['python3', 'tools/pmc_summary.py', f'gpurun_out/pmc_{tag}']))
    k = d['pk_step_kernel']
    js = json.load(open(f'gpurun_out/pmc_{tag}/p1.json'))
    ipe = js['instr_per_env_step']; w = k['SQ_WAVES']
    row = {c.replace('SQ_INSTS_', ''): round(k[c] / w / ipe, 1) for c in sorted(k) if c != 'SQ_WAVES'}
    print(tag, 'ms/step', js['ms_per_step'], row)
