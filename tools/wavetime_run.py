"""Per-wave K1 timing from a -DPK_WAVETIME diagnostic build: start/end (s_memrealtime, 100 MHz),
loop iterations, hardware slot (HW_ID, XCC_ID) and the wave's largest per-lane instruction count,
for each timed step.  Shows how much of a launch is the tail (the slowest waves) rather than the
mean wave.  Build: python tools/build_variant.py wt -- -DPK_WAVETIME (here); on the GPU box:
PK_LIB=pokegym_amd/lib/libpokegym_amd_wt.so python tools/wavetime_run.py --workload config4"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
REC = 6
NW = 16384


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="config4")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--rom-banks", type=int, default=4)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    from bench import WORKLOADS
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    W = WORKLOADS[args.workload]
    n = W["envs"]
    emu = BatchedEmulator(game_rom(args.rom_banks), n, render=W["render"])
    L = emu._L
    L.pk_debug_counters.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    g = torch.Generator(device=emu.device)
    g.manual_seed(5)
    words = 64 + REC * NW
    out = (ctypes.c_uint64 * words)()
    steps = []
    for t in range(2 + args.steps):
        if W["actions"] == "random":
            a = torch.randint(0, 8, (n,), generator=g, device=emu.device).to(torch.uint8)
        else:
            a = torch.full((n,), [0, 3, 1, 2][t % 4], dtype=torch.uint8, device=emu.device)
        L.pk_debug_counters(emu._h, out, words)      # clears the records
        emu.step(a)
        torch.cuda.synchronize()
        L.pk_debug_counters(emu._h, out, words)
        if t < 2:
            continue
        r = np.frombuffer(out, dtype=np.uint64)[64:].reshape(NW, REC).copy()
        r = r[r[:, 1] > 0]
        steps.append(r)
    emu.close()
    res = {"workload": args.workload, "envs": n, "steps": []}
    for r in steps:
        t0 = r[:, 0].astype(np.int64)
        t1 = r[:, 1].astype(np.int64)
        base = t0.min()
        dur_us = (t1 - t0) / 100.0        # 100 MHz ticks -> us
        end_us = (t1 - base) / 100.0
        kern_us = end_us.max()
        it = r[:, 2].astype(np.float64)
        icnt = r[:, 5].astype(np.float64)
        # hardware SIMD slot: XCC, SE, SH, CU, SIMD from HW_ID (gfx9 layout)
        hw = r[:, 3].astype(np.int64)
        simd = (hw >> 4) & 3
        cu = (hw >> 8) & 15
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 7
        xcc = r[:, 4].astype(np.int64) & 15
        slot = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
        uniq, inv = np.unique(slot, return_inverse=True)
        simd_end = np.zeros(len(uniq))
        np.maximum.at(simd_end, inv, end_us)
        busy_frac = float(simd_end.mean() / kern_us)
        q = lambda v, p: float(np.percentile(v, p))
        res["steps"].append({
            "waves": int(len(r)), "kernel_us": round(float(kern_us), 1),
            "wave_us": {"mean": round(float(dur_us.mean()), 1), "p50": round(q(dur_us, 50), 1), "p90": round(q(dur_us, 90), 1),
                        "p99": round(q(dur_us, 99), 1), "max": round(float(dur_us.max()), 1)},
            "start_spread_us": round(float((t0.max() - t0.min()) / 100.0), 1),
            "iters": {"mean": round(float(it.mean()), 1), "max": int(it.max())},
            "wave_max_instr": {"mean": round(float(icnt.mean()), 1), "max": int(icnt.max())},
            "ns_per_iter": {"mean": round(float((dur_us * 1000 / np.maximum(it, 1)).mean()), 1),
                            "slowest_wave": round(float(dur_us[np.argmax(dur_us)] * 1000 / max(it[np.argmax(dur_us)], 1)), 1)},
            "corr_dur_iters": round(float(np.corrcoef(dur_us, it)[0, 1]), 3),
            "simd_slots": int(len(uniq)), "simd_busy_frac": round(busy_frac, 3),
            "waves_done_at_50pct": round(float((end_us <= 0.5 * kern_us).mean()), 3),
            "waves_done_at_75pct": round(float((end_us <= 0.75 * kern_us).mean()), 3),
        })
    print(json.dumps(res))
    if args.out:
        np.savez_compressed(args.out, *steps)


if __name__ == "__main__":
    main()
