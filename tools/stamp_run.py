"""K1 phase-cycle breakdown from a -DPK_STAMP diagnostic build (s_memtime at the loop's wait
points, summed per wave).  Build: python tools/stamp_run.py --build (here); run on the GPU box:
PK_LIB=pokegym_amd/lib/libpokegym_amd_stamp.so python tools/stamp_run.py --workload config4"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
STAMP_LIB = os.path.join(HERE, "pokegym_amd", "lib", "libpokegym_amd_stamp.so")
PHASES = ["front+fetch+read to the read's wait (excl. rare fetch/read)", "rare read block", "datapath+control+fast write",
          "rare write block", "prefetch (LDS)", "ucode issue", "HALT block", "timer+LCD+latch", "frame end + loop",
          "rare fetch block", "flush_lines call", "pending-lines check"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--workload", default="config3")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--rom-banks", type=int, default=4)
    args = ap.parse_args()
    if args.build:
        from pokegym_amd import build
        print(build.build(out=STAMP_LIB, extra=["-DPK_STAMP"]))
        return
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
    out = (ctypes.c_uint64 * 16)()
    for t in range(2 + args.steps):
        if W["actions"] == "random":
            a = torch.randint(0, 8, (n,), generator=g, device=emu.device).to(torch.uint8)
        else:
            a = torch.full((n,), [0, 3, 1, 2][t % 4], dtype=torch.uint8, device=emu.device)
        if t == 2:
            L.pk_debug_counters(emu._h, out, 16)     # drop the warmup steps
        emu.step(a)
    torch.cuda.synchronize()
    L.pk_debug_counters(emu._h, out, 16)
    it, waves = out[12], max(out[13], 1)
    res = {"workload": args.workload, "waves": waves, "iterations_per_wave_step": it / waves,
           "cycles_per_iteration": {p: round(out[k] / max(it, 1), 1) for k, p in enumerate(PHASES)},
           "total_per_iteration": round(sum(out[k] for k in range(12)) / max(it, 1), 1)}
    print(json.dumps(res))
    emu.close()


if __name__ == "__main__":
    main()
