import json, sys
for f in sys.argv[1:]:
    try:
        d = json.load(open(f))
        print(f"{f}: value={d['value']:.0f} ms/step={d['ms_per_step']} k1_ms={d['roofline']['k1_ms']} k2_ms={d['roofline']['k2_render_ms']} "
              f"instr/step={d['instr_per_env_step']} Ginstr/s={d['emulated_instr_per_s']/1e9:.2f} cpu={d.get('cpu_baseline', {}).get('value')}")
    except Exception as e:  # noqa: BLE001
        print(f, "ERR", e)
