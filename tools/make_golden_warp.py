"""Fixture for the map-load (LCD-off warp) parity tests -> tests/golden/warp_state.npz.

Runs the oracle on pkbench with seeded random actions until an env walks through a door
(testrom/game.py map_warp: LCD off for ~5 frames of bulk VRAM/WRAM copies), and saves the v9
state two env-steps before that step plus the actions of the next 6 env-steps.  The tests load
the state into the host-simulated and the MI355X kernels and compare them with the oracle."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
from oracle import oracle  # noqa: E402
from pokegym_amd.testrom.game import game_rom  # noqa: E402


def main():
    rom = game_rom()
    rng = np.random.default_rng(1)
    for env in range(16):
        acts = rng.integers(0, 8, 600).astype(np.uint8)
        gb = oracle.GB(rom)
        states = []
        for t in range(600):
            states.append(gb.save_state())
            before = gb.read(0xD4A1)
            gb.run_action(int(acts[t]))
            if t > 4 and gb.read(0xD4A1) != before:   # wMapSeed changed: this step warped
                k = t - 2
                out = os.path.join(REPO, "tests", "golden", "warp_state.npz")
                np.savez_compressed(out, state=np.frombuffer(states[k], np.uint8), actions=acts[k:k + 6],
                                    warp_step=np.int32(2))
                print(f"env {env}: warp at step {t}; saved state of step {k} -> {out}")
                return
    raise SystemExit("no warp found")


if __name__ == "__main__":
    main()
