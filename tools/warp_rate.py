"""How often pkbench's door warp (multi-frame LCD-off map load) runs under bench.py's random actions:
the C oracle's workload intensity (oracle/gbcore.c gb_intensity) over a large sample, one process per
seed.  bench.py's per-line `workload_intensity` covers 256 env-steps, too few to see a warp.
usage: python tools/warp_rate.py [procs] [envs_per_proc] [steps]"""
import json
import multiprocessing as mp
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def one(seed, n, steps):
    from oracle import oracle
    from pokegym_amd.testrom.game import game_rom
    return oracle.intensity(game_rom(), None, n, 3, steps, seed)


def main():
    procs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.starmap(one, [(1000 + p, n, steps) for p in range(procs)])
    env_steps = procs * n * steps
    cyc = sum(r["cycles_per_frame"] for r in res) / procs
    lcd = sum(r["lcd_off_frac"] for r in res) / procs
    out = {"env_steps": env_steps, "lcd_off_frac": round(lcd, 7),
           "lcd_off_frames_per_1k_env_steps": round(lcd * 24 * 1000, 3),
           "halted_frac": round(sum(r["halted_frac"] for r in res) / procs, 4),
           "instr_per_env_step": round(sum(r["instr_per_env_step"] for r in res) / procs, 1),
           "cycles_per_frame": cyc}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
