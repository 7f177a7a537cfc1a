"""Wave-level iteration statistics of K1 from the host-simulation build (design tool).

SIMT: iteration k of every lane of a wave executes together, so a code path is paid by the wave
at iteration k if ANY lane takes it.  Records per-lane event bits (pk_kernels.hip PK_EV_*) with
tests/hostsim and reports, per 64-lane group, the fraction of wave iterations executing each path
and the lane fraction that wanted it.
usage: python tools/iter_stats.py [steps] [warmup] [wave_lanes]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.hostsim import sim  # noqa: E402
from pokegym_amd.testrom.game import game_rom  # noqa: E402

NAMES = ["EXEC", "F_LDS", "F_ROM16", "F_BUS", "INT", "IDLE", "RD", "RD_ROMLDS", "RD_ROMG", "RD_RAM", "RD_IO",
         "RD2", "WR", "WR_SLOW", "WR2", "LCD", "TIMER", "FRAME", "FLUSH", "HRAM", "JUMP", "CB",
         "FUSE", "FAM_ALU", "FAM_BITROT", "FAM_16", "FAM_CTRL", "FAM_MISC", "RD_WRAM", "WR_WRAM", "WR_VRAM", "WR_HI"]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    wl = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    n = 64
    L = sim.lib()
    L.pk_sim_iter_enable.argtypes = [ctypes.c_uint32, ctypes.c_int]
    L.pk_sim_iter_get.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
    L.pk_sim_iter_get.restype = ctypes.c_uint64
    emu = sim.SimEmulator(game_rom(), n, render=True)
    rng = np.random.default_rng(0)
    for _ in range(warm):
        emu.step(rng.integers(0, 8, n).astype(np.uint8))
    tot_wave = np.zeros(32)
    tot_lane = np.zeros(32)
    iters = lane_iters = 0
    for _ in range(steps):
        L.pk_sim_iter_enable(n, 1)
        emu.step(rng.integers(0, 8, n).astype(np.uint8))
        evs = []
        for e in range(n):
            k = L.pk_sim_iter_get(e, None, 0)
            buf = np.zeros(k, np.uint32)
            L.pk_sim_iter_get(e, buf.ctypes.data, k)
            evs.append(buf)
        L.pk_sim_iter_enable(0, 0)
        for g0 in range(0, n, wl):
            grp = evs[g0:g0 + wl]
            m = max(len(x) for x in grp)
            M = np.zeros((len(grp), m), np.uint32)
            act = np.zeros((len(grp), m), bool)
            for i, x in enumerate(grp):
                M[i, :len(x)] = x
                act[i, :len(x)] = True
            wave_or = np.bitwise_or.reduce(M, axis=0)
            bits = (wave_or[:, None] >> np.arange(32)) & 1
            tot_wave += bits.sum(0)
            lb = (M[..., None] >> np.arange(32)) & 1
            tot_lane += lb.sum((0, 1))
            iters += m
            lane_iters += act.sum()
    ninstr = tot_lane[0]
    print(f"wave iterations {iters}, lane-iterations {lane_iters}, instructions {int(ninstr)}, "
          f"lane occupancy {lane_iters / (iters * wl):.3f}, wave iters per lane instr {iters * wl / ninstr:.3f}")
    print(f"{'path':12s} {'wave%':>7s} {'lane%':>7s}")
    for b, name in enumerate(NAMES):
        print(f"{name:12s} {100 * tot_wave[b] / iters:7.1f} {100 * tot_lane[b] / lane_iters:7.2f}")


if __name__ == "__main__":
    main()
