"""CLI: host-sim kernel vs oracle on fuzz/game ROMs (whole-state v9 compare)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from tests.hostsim.sim import SimEmulator
from oracle import oracle
from pokegym_amd.testrom.fuzz import fuzz_rom
from pokegym_amd.testrom.game import game_rom

def check(rom, n, steps, seed, state=None):
    acts = np.random.default_rng(seed).integers(0, 9, size=(steps, n), dtype=np.uint8)
    emu = SimEmulator(rom, n, state=state)
    for s in range(steps):
        emu.step(acts[s])
    ref, scr = oracle.batch_run(rom, state, acts)
    grey = np.array([0xFF, 0x99, 0x55, 0x00], np.uint8)
    sims = emu.screen()
    bad = []
    for e in range(n):
        a = np.frombuffer(emu.snapshot(e), np.uint8)
        idx = np.nonzero(a != ref[e])[0]
        if len(idx) or not np.array_equal(sims[e], grey[scr[e]]):
            bad.append((e, idx[:8].tolist()))
    emu.close()
    return bad

if __name__ == "__main__":
    for spec in sys.argv[1:]:
        name, n, steps = spec.split(":")
        rom = game_rom() if name == "game" else fuzz_rom(int(name[4:]))
        print(spec, check(rom, int(n), int(steps), 7)[:4], flush=True)
