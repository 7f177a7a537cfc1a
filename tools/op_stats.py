"""Opcode statistics of K1 from the host-simulation build (design tool).

Per wave iteration (SIMT: iteration k of every lane of a wave executes together): how many
distinct microcode entries the active lanes hold (1 = a wave-uniform iteration), and the
instruction-class histogram per lane and per wave (a class is paid by the wave when ANY lane
holds it).  usage: python tools/op_stats.py [steps] [warmup] [wave_lanes] [rom_banks] [mode]
mode: random (default, configs[2..4]) | cycle (configs[1]: every env the same [0,3,1,2] cycle)"""
import ctypes
import os
import sys
from collections import Counter

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.hostsim import sim  # noqa: E402
from pokegym_amd.testrom.game import game_rom  # noqa: E402


def op_class(di):
    if di >= 512:
        return "pseudo"
    if di >= 256:
        o = di - 256
        return "cb_rot" if o < 0x40 else ("cb_bit" if o < 0x80 else "cb_resset")
    o = di
    if 0x40 <= o < 0x80 and o != 0x76:
        return "ld_r_r" if (o & 7) != 6 and ((o >> 3) & 7) != 6 else "ld_hl_mem"
    if 0x80 <= o < 0xC0:
        return "alu_r" if (o & 7) != 6 else "alu_hl"
    if o in (0x07, 0x0F, 0x17, 0x1F):
        return "rot_a"
    if o in (0x27,):
        return "daa"
    if (o & 0xC7) == 0xC6:
        return "alu_n"
    if o in (0x18, 0x20, 0x28, 0x30, 0x38):
        return "jr"
    if o in (0xC3, 0xC2, 0xCA, 0xD2, 0xDA, 0xE9):
        return "jp"
    if o in (0xCD, 0xC4, 0xCC, 0xD4, 0xDC) or (o & 0xC7) == 0xC7:
        return "call_rst"
    if o in (0xC9, 0xD9, 0xC0, 0xC8, 0xD0, 0xD8):
        return "ret"
    if (o & 0xCF) in (0xC1, 0xC5):
        return "push_pop"
    if (o & 0xC7) in (0x04, 0x05):
        return "inc_dec8"
    if (o & 0xC7) == 0x06:
        return "ld_r_n"
    if (o & 0xCF) in (0x03, 0x0B, 0x09):
        return "r16_arith"
    if (o & 0xCF) == 0x01:
        return "ld_rr_nn"
    if (o & 0xC7) == 0x02:
        return "ld_ind_a"
    if o in (0xE0, 0xF0, 0xE2, 0xF2, 0xEA, 0xFA):
        return "ldh_abs"
    if o == 0x76:
        return "halt"
    return "misc"


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    wl = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    banks = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    mode = sys.argv[5] if len(sys.argv) > 5 else "random"
    n = 64
    L = sim.lib()
    L.pk_sim_iter_enable.argtypes = [ctypes.c_uint32, ctypes.c_int]
    L.pk_sim_iter_op_get.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
    L.pk_sim_iter_op_get.restype = ctypes.c_uint64
    emu = sim.SimEmulator(game_rom(banks=banks), n, render=True)
    rng = np.random.default_rng(0)
    cyc = [0, 3, 1, 2]

    def acts(t):
        if mode == "cycle":
            return np.full(n, cyc[t % 4], np.uint8)
        return rng.integers(0, 8, n).astype(np.uint8)

    for t in range(warm):
        emu.step(acts(t))
    distinct = Counter()
    lane_cls, wave_cls = Counter(), Counter()
    lane_ops = Counter()
    iters = 0
    for t in range(steps):
        L.pk_sim_iter_enable(n, 1)
        emu.step(acts(warm + t))
        ops = []
        for e in range(n):
            k = L.pk_sim_iter_op_get(e, None, 0)
            buf = np.zeros(k, np.uint32)
            L.pk_sim_iter_op_get(e, buf.ctypes.data, k)
            ops.append(buf)
        L.pk_sim_iter_enable(0, 0)
        for g0 in range(0, n, wl):
            grp = ops[g0:g0 + wl]
            m = max(len(x) for x in grp)
            for k in range(m):
                col = [int(x[k]) for x in grp if k < len(x)]
                distinct[len(set(col))] += 1
                cl = [op_class(d) for d in col]
                for c in cl:
                    lane_cls[c] += 1
                for c in set(cl):
                    wave_cls[c] += 1
                for d in col:
                    lane_ops[d] += 1
            iters += m
    tot_lanes = sum(lane_cls.values())
    print(f"wave iterations {iters}, lane-iterations {tot_lanes}, wave lanes {wl}, mode {mode}, banks {banks}")
    acc = 0
    for k in sorted(distinct):
        acc += distinct[k]
        print(f"  distinct entries {k:3d}: {100 * distinct[k] / iters:6.2f} %  (cum {100 * acc / iters:6.2f} %)")
    print(f"{'class':12s} {'lane%':>7s} {'wave%':>7s}")
    for c, v in sorted(lane_cls.items(), key=lambda kv: -kv[1]):
        print(f"{c:12s} {100 * v / tot_lanes:7.2f} {100 * wave_cls[c] / iters:7.2f}")
    print("top opcodes:", ", ".join(f"{d:03x}:{100 * v / tot_lanes:.1f}" for d, v in lane_ops.most_common(24)))


if __name__ == "__main__":
    main()
