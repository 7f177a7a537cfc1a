"""Oracle PPU vs the 264 frames PyBoy embedded in the reference's savestates.

The fixture (tests/golden/ppu_states.npz) was produced by tools/make_golden_ppu.py from the
reference's savestate DATA files; the expected frames are PyBoy's own rendered output."""
import os

import numpy as np

from oracle import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ppu_states.npz")


def test_ppu_matches_all_264_pyboy_frames():
    z = np.load(GOLD)
    prefix, frames, names = z["prefix"], z["frames"], z["names"]
    assert len(prefix) == 264
    bad = []
    for i in range(len(prefix)):
        out = oracle.render_from_state(prefix[i].tobytes())
        if not np.array_equal(out, frames[i]):
            bad.append((str(names[i]), int((out != frames[i]).sum())))
    assert not bad, bad[:10]


def test_savestate_roundtrip_is_identity():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "states.npz"))
    rom = bytes(0x8000)  # ROM-only dummy; no code is executed
    rom = bytearray(rom)
    rom[0x147] = 0x13  # MBC3+RAM+BATTERY like pokemon_red.gb
    for st in z["states"]:
        g = oracle.GB(bytes(rom), st.tobytes())
        assert g.save_state() == st.tobytes()
