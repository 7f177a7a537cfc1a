"""First instruction where the host-simulated K1 and the oracle disagree (debugging tool).

usage: python tools/trace_diff.py fuzzSEED|game [env] [steps] [n] [actions-seed]
Runs n envs for `steps` env-steps with the actions of tests/hostsim/check.py, tracing env `env` on
both sides (pc, BC|DE<<16 / registers, SP, opcode per executed instruction), and prints the first
differing record with some context."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from tests.hostsim import sim  # noqa: E402
from pokegym_amd.testrom.fuzz import fuzz_rom  # noqa: E402
from pokegym_amd.testrom.game import game_rom  # noqa: E402


def main():
    name = sys.argv[1]
    env = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    aseed = int(sys.argv[5]) if len(sys.argv) > 5 else int(name[4:]) if name.startswith("fuzz") else 3
    rom = game_rom() if name == "game" else fuzz_rom(int(name[4:]))
    acts = np.random.default_rng(aseed).integers(0, 9, size=(steps, n), dtype=np.uint8)
    cap = 4_000_000
    L = sim.lib()
    L.pk_sim_trace_enable.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    L.pk_sim_trace_get.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    L.pk_sim_trace_get.restype = ctypes.c_uint64
    L.pk_sim_trace_enable(env, cap)
    emu = sim.SimEmulator(rom, n)
    for s in range(steps):
        emu.step(acts[s])
    buf = np.zeros((cap, 6), np.uint32)
    k = L.pk_sim_trace_get(buf.ctypes.data, cap)
    dev = buf[:k]
    O = oracle.lib()
    O.gb_trace_enable.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    O.gb_trace_count.restype = ctypes.c_uint64
    obuf = np.zeros((cap, 6), np.uint32)
    gb = oracle.GB(rom)
    O.gb_trace_enable(obuf.ctypes.data, cap)
    for s in range(steps):
        gb.run_action(int(acts[s, env]) if acts[s, env] < 8 else 99)
    m = O.gb_trace_count()
    O.gb_trace_enable(None, 0)
    ref = obuf[:m]
    # fold the loop fast paths: a device marker (op 0x1000 | loop length, w0 = passes) stands for
    # passes x length oracle records right after the traced instruction (pk_copy_loop/pk_poll_loop
    # run whole passes inside one iteration and trace none of their instructions)
    keep_d, keep_r, j = [], [], 0
    for i in range(len(dev)):
        if dev[i, 4] & 0x1000:
            j += int(dev[i, 1]) * int(dev[i, 4] & 0xFFF)
            continue
        keep_d.append(i)
        keep_r.append(j)
        j += 1
    nn = sum(1 for r in keep_r if r < len(ref))
    dev, ref = dev[keep_d[:nn]], ref[keep_r[:nn]]
    print(f"device {len(dev)} records, oracle {len(ref)} (after folding loop fast-path passes)")
    cols = ["pc", "w0", "w1", "sp", "op"]
    nn = min(len(dev), len(ref))
    d = np.nonzero((dev[:nn, :5] != ref[:nn, :5]).any(1))[0]
    if not len(d):
        print("traces agree over", nn, "records")
        return
    i = int(d[0])
    print("first difference at record", i)
    for j in range(max(0, i - 6), min(nn, i + 3)):
        print(j, "dev", " ".join(f"{c}={dev[j, q]:08x}" for q, c in enumerate(cols)))
        print(j, "ref", " ".join(f"{c}={ref[j, q]:08x}" for q, c in enumerate(cols)))


if __name__ == "__main__":
    main()
