"""Estimate K1 loop iterations per emulated instruction under different fusion rules (design tool).

Traces one env's executed instructions with the host-simulation build (tests/hostsim) and groups
them greedily like K1's fused secondary op does: a fusable primary followed by register-only
successors inside the fetched bytes.  Compares the current rule (one successor, 4 fetched bytes)
with two successors and with an 8-byte fetch.  Timing conditions (LCD event, timer) are ignored,
so the counts are lower bounds for every rule alike.
usage: python tools/fuse_est.py [env] [steps] [--warp]"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from tests.hostsim import sim  # noqa: E402
from pokegym_amd.testrom.game import game_rom  # noqa: E402

L2 = {0x06, 0x0E, 0x16, 0x1E, 0x26, 0x2E, 0x36, 0x3E, 0x18, 0x20, 0x28, 0x30, 0x38, 0xC6, 0xCE, 0xD6, 0xDE,
      0xE6, 0xEE, 0xF6, 0xFE, 0xE0, 0xF0, 0xE8, 0xF8, 0xCB, 0x10}
L3 = {0x01, 0x11, 0x21, 0x31, 0x08, 0xC2, 0xC3, 0xCA, 0xD2, 0xDA, 0xC4, 0xCC, 0xCD, 0xD4, 0xDC, 0xEA, 0xFA}


def ilen(op):
    return 3 if op in L3 else 2 if op in L2 else 1


def secondary(op):
    if op in (0x18, 0x20, 0x28, 0x30, 0x38, 0x00, 0x2F, 0x37):
        return True
    if 0x40 <= op < 0x80:
        return op != 0x76 and (op & 7) != 6 and ((op >> 3) & 7) != 6
    if op < 0x40 and (op & 7) == 6:          # LD r,n
        return op != 0x36
    if op < 0x40 and (op & 7) in (4, 5):     # INC/DEC r
        return op not in (0x34, 0x35)
    if op in (0x03, 0x0B, 0x13, 0x1B, 0x23, 0x2B):
        return True
    if 0x80 <= op < 0xC0:
        return (op & 7) != 6
    return op in (0xC6, 0xCE, 0xD6, 0xDE, 0xE6, 0xEE, 0xF6, 0xFE)


MEMW = {0x02, 0x12, 0x22, 0x32, 0x70, 0x71, 0x72, 0x73, 0x74, 0x75, 0x77}   # ld (rr),a / ld (hl),r


def writes_mem(op):
    return op in MEMW or op in (0x34, 0x35, 0x36, 0xE0, 0xE2, 0xEA, 0x08) or op in (0xC5, 0xD5, 0xE5, 0xF5, 0xCD, 0xC4,
                                                                             0xCC, 0xD4, 0xDC)


def primary_fusable(op):
    ctrl = {0x18, 0x20, 0x28, 0x30, 0x38, 0xC0, 0xC2, 0xC3, 0xC4, 0xC7, 0xC8, 0xC9, 0xCA, 0xCC, 0xCD, 0xCF, 0xD0,
            0xD2, 0xD4, 0xD7, 0xD8, 0xD9, 0xDA, 0xDC, 0xDF, 0xE7, 0xE9, 0xEF, 0xF7, 0xFF, 0xF3, 0xFB, 0x76, 0x10,
            0x27}
    return op not in ctrl


MEMR = {0x0A, 0x1A, 0x2A, 0x3A, 0x46, 0x4E, 0x56, 0x5E, 0x66, 0x6E, 0x7E, 0xF0, 0xFA, 0xF2,
        0x86, 0x8E, 0x96, 0x9E, 0xA6, 0xAE, 0xB6, 0xBE}   # ld r,(rr) / ld a,(hl+-) / ldh / ld a,(nn) / alu a,(hl)


def groups(tr, slots, fetch, memw=False, memr=False):
    """tr: list of (pc, op); returns the number of loop iterations"""
    n, i, it = len(tr), 0, 0
    while i < n:
        pc, op = tr[i]
        used = ilen(op)
        j = i + 1
        if primary_fusable(op):
            k = 0
            while k < slots - 1 and j < n:
                pc2, op2 = tr[j]
                ok2 = secondary(op2) or (memw and op2 in MEMW and not writes_mem(op)) or (memr and op2 in MEMR)
                if pc2 != (tr[j - 1][0] + ilen(tr[j - 1][1])) & 0xFFFF or not ok2:
                    break
                if used + ilen(op2) > fetch or pc >= 0x8000:
                    break
                used += ilen(op2)
                j += 1
                k += 1
                # a taken JR ends the group (its successor is not in the fetched bytes)
                if j < n and op2 in (0x18, 0x20, 0x28, 0x30, 0x38) and tr[j][0] != (pc2 + 2) & 0xFFFF:
                    break
        it += 1
        i = j
    return it


def main():
    env = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else 4
    warp = "--warp" in sys.argv
    L = sim.lib()
    L.pk_sim_trace_enable.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    L.pk_sim_trace_get.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    L.pk_sim_trace_get.restype = ctypes.c_uint64
    state = None
    if warp:
        state = bytes(np.load(os.path.join(HERE, "tests", "golden", "warp_state.npz"))["state"])
    n = 64
    emu = sim.SimEmulator(game_rom(), n, state=state)
    rng = np.random.default_rng(env)
    for _ in range(0 if warp else 3):
        emu.step(rng.integers(0, 8, n).astype(np.uint8))
    cap = 4_000_000
    L.pk_sim_trace_enable(env, cap)
    for _ in range(steps):
        emu.step(rng.integers(0, 8, n).astype(np.uint8))
    buf = (ctypes.c_uint32 * (6 * cap))()
    m = L.pk_sim_trace_get(buf, cap)
    a = np.frombuffer(buf, dtype=np.uint32, count=6 * m).reshape(m, 6)
    tr = [(int(r[0]), int(r[4]) & 0xFF) for r in a if not (int(r[4]) & 0x1000)]   # drop loop fast-path markers
    emu.close()
    print(f"env {env} {'warp ' if warp else ''}{steps} steps: {len(tr)} instructions")
    for slots, fetch in ((1, 4), (2, 4), (3, 4), (2, 8), (3, 8), (4, 8)):
        it = groups(tr, slots, fetch)
        print(f"  slots={slots} fetch={fetch}B: iterations {it}  ({it / max(len(tr), 1):.3f} per instruction)")
    it = groups(tr, 2, 4, memr=True)
    print(f"  slots=2 fetch=4B + memory-read secondaries (ld r,(rr) / ldh a,(n) / ld a,(nn) / alu a,(hl)): "
          f"iterations {it}  ({it / max(len(tr), 1):.3f} per instruction)")
    it = groups(tr, 2, 4, memw=True)
    print(f"  slots=2 fetch=4B + memory-write secondaries (ld (rr),a / ld (hl),r after a non-writing primary): "
          f"iterations {it}  ({it / max(len(tr), 1):.3f} per instruction)")


if __name__ == "__main__":
    main()
