"""Generate PPU / savestate golden fixtures from the reference's savestate corpus.

Run in the build container only (needs /root/reference).  Writes:
  tests/golden/ppu_states.npz   prefix[264, 9125] (header, CPU, VRAM, OAM, LCD regs, per-line
                                params) and frames[264, 144, 160] — the shade ids (0..3) decoded
                                from the 144x160x4 screen buffer PyBoy embedded in each state
                                (bytes [w,R,G,B], grey FF/99/55/00).
  tests/golden/states.npz       a few complete v9 states (start states for parity runs).
  pokegym_amd/states/Bulbasaur.state   the reference's default start state (environment.py:119-120).
The savestates are DATA files of the reference (no source is copied).
"""
import glob
import os
import shutil
import sys

import numpy as np

REF = "/root/reference/pokegym"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZE = 142610
GREY = {0xFF: 0, 0x99: 1, 0x55: 2, 0x00: 3}


def corpus():
    fs = sorted(f for f in glob.glob(REF + "/**/*", recursive=True)
                if os.path.isfile(f) and os.path.getsize(f) == SIZE)
    out = []
    for f in fs:
        d = open(f, "rb").read()
        if d[0] == 9:
            out.append((os.path.relpath(f, REF), d))
    return out


def main():
    states = corpus()
    names = np.array([n for n, _ in states])
    prefix = np.stack([np.frombuffer(d[:9125], np.uint8) for _, d in states])
    frames = []
    for _, d in states:
        scr = np.frombuffer(d[9125:101285], np.uint8).reshape(144, 160, 4)
        lut = np.zeros(256, np.uint8)
        for k, v in GREY.items():
            lut[k] = v
        frames.append(lut[scr[..., 1]])
    frames = np.stack(frames)
    os.makedirs(os.path.join(REPO, "tests", "golden"), exist_ok=True)
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "ppu_states.npz"),
                        names=names, prefix=prefix, frames=frames)
    keep = ["current_state/Bulbasaur.state", "unused_states/cerulean_gym.state",
            "unused_states/viridian_forest.state", "unused_states/outside_mt_moon.state"]
    # plus a couple of in-battle states (D057 != 0: WRAM offset 0x1057)
    battle = [n for n, d in states if d[101285 + 0x1057] != 0][:2]
    keep += battle
    full = {n: d for n, d in states}
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "states.npz"),
                        names=np.array(keep),
                        states=np.stack([np.frombuffer(full[k], np.uint8) for k in keep]))
    os.makedirs(os.path.join(REPO, "pokegym_amd", "states"), exist_ok=True)
    shutil.copyfile(os.path.join(REF, "current_state", "Bulbasaur.state"),
                    os.path.join(REPO, "pokegym_amd", "states", "Bulbasaur.state"))
    print(len(states), "states;", "kept", keep)


if __name__ == "__main__":
    sys.exit(main())
