"""Attribute K1's RAM-image traffic to guest regions (design tool, host simulation).

Runs pkbench in the host-simulation build with K1's fast-path image accesses recorded
(PK_MEMREF: operand reads and writes; the rare bus paths, OAM DMA and the block copy are not
counted) and reports, per guest region and per env-step: accesses, the distinct 128-byte lines of
the lane-interleaved image an env touches (W envs per interleave: a line holds 128 / W guest bytes
of W envs), and per wave iteration the lines a wave's lanes touch together (what one load or store
instruction of the wave costs the memory pipe).
usage: python tools/mem_stats.py [wave_lanes=16] [steps=4] [n=256] [--warp] [--writes]
(--writes: stores only, as bounds on the L2's write-back bytes per env-step)"""
import ctypes
import os
import sys
from collections import Counter, defaultdict

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def region(phys):
    if phys < 0x2000:
        return "VRAM 8000-9FFF"
    if phys < 0x4000:
        g = 0xC000 + phys - 0x2000
        if g >= 0xDF00:
            return "WRAM DF00-DFFF (stack page)"
        if 0xC300 <= g < 0xC400:
            return "WRAM C300-C3FF (OAM buffer)"
        return "WRAM other"
    if phys < 0x4100:
        return "OAM FE00-FEFF"
    if phys < 0x4180:
        return "IO FF00-FF7F"
    if phys < 0x4200:
        return "HRAM FF80-FFFE"
    return "SRAM"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    wl = int(args[0]) if len(args) > 0 else 16
    steps = int(args[1]) if len(args) > 1 else 4
    n = int(args[2]) if len(args) > 2 else 256
    warp = "--warp" in sys.argv
    os.environ["PK_WAVE_LANES"] = str(wl)
    from tests.hostsim import sim
    from pokegym_amd.testrom.game import game_rom
    L = sim.lib()
    L.pk_sim_iter_enable.argtypes = [ctypes.c_uint32, ctypes.c_int]
    L.pk_sim_mem_enable.argtypes = [ctypes.c_uint32, ctypes.c_int]
    L.pk_sim_mem_get.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint64]
    L.pk_sim_mem_get.restype = ctypes.c_uint64
    state = bytes(np.load(os.path.join(HERE, "tests", "golden", "warp_state.npz"))["state"]) if warp else None
    emu = sim.SimEmulator(game_rom(), n, state=state)
    rng = np.random.default_rng(1)
    for _ in range(0 if warp else 3):
        emu.step(rng.integers(0, 8, n).astype(np.uint8))
    L.pk_sim_iter_enable(n, 1)
    L.pk_sim_mem_enable(n, 1)
    for _ in range(steps):
        emu.step(rng.integers(0, 8, n).astype(np.uint8))
    per_line = 128 // wl                       # guest bytes of one env in a 128-byte line
    acc = Counter()                            # (region, kind) -> accesses
    lines_env = Counter()                      # region -> distinct lines per env (summed over envs)
    wave_lines = Counter()                     # region -> sum over wave iterations of distinct lines
    wave_iters = 0
    recs, io_recs = {}, {}
    for e in range(n):
        k = L.pk_sim_mem_get(e, None, 0)
        buf = np.zeros(k, np.uint64)
        L.pk_sim_mem_get(e, buf.ctypes.data, k)
        io_recs[e] = buf[((buf >> 16) & 3) >= 2]
        kind_all = ((buf >> 16) & 3).astype(np.int64)
        buf = buf[kind_all < 2]                      # kinds 2/3: IO reads / slow writes (io_stats below)
        recs[e] = buf
        phys = (buf & 0xFFFF).astype(np.int64)
        kind = ((buf >> 16) & 1).astype(np.int64)
        for p, kd in zip(phys.tolist(), kind.tolist()):
            acc[(region(p), kd)] += 1
        seen = defaultdict(set)
        for p in phys.tolist():
            seen[region(p)].add(p // per_line)
        for r, s in seen.items():
            lines_env[r] += len(s)
    # wave iterations: lanes of one wave (wl consecutive envs) at the same iteration index
    for w0 in range(0, n, wl):
        by_it = defaultdict(set)
        for e in range(w0, min(n, w0 + wl)):
            b = recs[e]
            it = (b >> 20).astype(np.int64)
            phys = (b & 0xFFFF).astype(np.int64)
            sub = e // wl                          # one sub-block per wave (interleave = wave width)
            for i, p in zip(it.tolist(), phys.tolist()):
                by_it[i].add((region(p), sub, p // per_line))
        wave_iters += len(by_it)
        for s in by_it.values():
            for r, _, _ in s:
                wave_lines[r] += 1
    es = n * steps
    if "--writes" in sys.argv:
        # stores only: per region, the env-step's distinct 128-byte lines written (each written back
        # once per step at best: the lower bound of the L2's write-backs) and the wave-level store
        # line touches (each written back on its own: the upper bound when a dirty line is evicted
        # between two stores to it), both in bytes per env-step of the 32-byte sectors written
        wl_lines, wl_env = Counter(), Counter()
        for w0 in range(0, n, wl):
            by_it = defaultdict(set)
            envlines = defaultdict(set)
            for e in range(w0, min(n, w0 + wl)):
                b = recs[e]
                b = b[((b >> 16) & 1) == 1]
                for i, p in zip((b >> 20).astype(np.int64).tolist(), (b & 0xFFFF).astype(np.int64).tolist()):
                    by_it[i].add((region(p), p // per_line))
                    envlines[region(p)].add(p // per_line)
            for st in by_it.values():
                for r, _ in st:
                    wl_lines[r] += 1
            for r, st in envlines.items():
                wl_env[r] += len(st)
        print(f"stores, wave_lanes {wl}, {n} envs x {steps} env-steps: bytes per env-step if each written line is "
              f"written back once per step (lower) / once per wave-iteration store (upper), 32-byte sectors of "
              f"{wl} envs x {per_line} guest bytes")
        print(f"{'region':30s} {'stores/es':>9s} {'lines/step/wave':>16s} {'lower B/es':>11s} {'upper B/es':>11s}")
        lo_t = up_t = 0.0
        for r in sorted(wl_lines, key=lambda r: -wl_lines[r]):
            lo = wl_env[r] * 128 / steps / n            # whole lines, once per step, per env
            up = wl_lines[r] * 32 / steps / n           # one 32-byte sector per line a wave's store touches
            lo_t += lo
            up_t += up
            print(f"{r:30s} {acc[(r, 1)] / es:9.1f} {wl_env[r] / steps / (n // wl):16.1f} {lo:11.1f} {up:11.1f}")
        print(f"{'total':30s} {'':9s} {'':16s} {lo_t:11.1f} {up_t:11.1f}")
        return
    tot_acc = sum(acc.values())
    print(f"wave_lanes {wl}, {n} envs x {steps} env-steps{' (door-warp state)' if warp else ''}: "
          f"{tot_acc / es:.0f} fast-path image accesses per env-step; wave iterations with an access: "
          f"{wave_iters / (n // wl) / steps:.0f} per wave-step")
    print(f"{'region':30s} {'reads/es':>9s} {'writes/es':>9s} {'lines/env-step':>15s} {'wave-iter lines/wave-step':>26s}")
    regs = sorted({r for r, _ in acc}, key=lambda r: -(acc[(r, 0)] + acc[(r, 1)]))
    for r in regs:
        print(f"{r:30s} {acc[(r, 0)] / es:9.1f} {acc[(r, 1)] / es:9.1f} {lines_env[r] / es:15.1f} "
              f"{wave_lines[r] / (n // wl) / steps:26.1f}")
    # finer: the 256-byte guest pages with the most wave-iteration line touches
    page = Counter()
    for w0 in range(0, n, wl):
        by_it = defaultdict(set)
        for e in range(w0, min(n, w0 + wl)):
            b = recs[e]
            for i, p in zip((b >> 20).astype(np.int64).tolist(), (b & 0xFFFF).astype(np.int64).tolist()):
                by_it[i].add(p // per_line * per_line)
        for s in by_it.values():
            for p in s:
                page[p >> 8] += 1
    def guest(pg):
        p = pg << 8
        return (0x8000 + p if p < 0x2000 else 0xC000 + p - 0x2000 if p < 0x4000 else 0xFE00 + p - 0x4000 if p < 0x4100
                else 0xFF00 + p - 0x4100)
    # IO register reads (io_read) and slow-path writes (IO/MBC/DMA): per wave, the iterations in
    # which ANY lane takes that path for that address
    io_w, io_l = Counter(), Counter()
    for w0 in range(0, n, wl):
        by_it = defaultdict(set)
        for e in range(w0, min(n, w0 + wl)):
            b = io_recs[e]
            for i, kd, a in zip((b >> 20).astype(np.int64).tolist(), ((b >> 16) & 3).astype(np.int64).tolist(),
                                (b & 0xFFFF).astype(np.int64).tolist()):
                by_it[i].add((kd, a))
                io_l[(kd, a)] += 1
        for s_ in by_it.values():
            for ka in s_:
                io_w[ka] += 1
        io_w["any"] += len(by_it)
    nw = (n // wl) * steps
    print(f"IO paths: wave iterations with any IO read / slow write: {io_w['any'] / nw:.0f} per wave-step")
    for (kd, a), c in sorted(((k, v) for k, v in io_w.items() if k != "any"), key=lambda kv: -kv[1])[:16]:
        print(f"  {'read ' if kd == 2 else 'write'} {a:04X}  {c / nw:9.1f} wave-iterations per wave-step, "
              f"{io_l[(kd, a)] / es:8.1f} per env-step")
    tot = sum(page.values())
    print("top guest pages by wave-iteration line touches:")
    for pg, c in page.most_common(12):
        print(f"  {guest(pg):04X}-{guest(pg) + 0xFF:04X}  {c / (n // wl) / steps:10.1f} per wave-step  ({100 * c / tot:.1f} %)")


if __name__ == "__main__":
    main()
