"""K2 (the HIP scanline renderer) vs the 264 frames PyBoy rendered into the reference's savestates.

Each savestate's VRAM, OAM, LCD registers and per-line SCX/SCY/WX/WY/tile-data latches are
loaded into one env through the C ABI (pk_load_env), K2 rasterises the latched lines
(pk_render_latched) and the device screen must equal PyBoy's saved frame in the grey palette of
screen.screen_ndarray() (environment.py:268).  The fixture holds the reference's own frames
(tests/golden/ppu_states.npz, tools/make_golden_ppu.py); this pins the HIP renderer directly to
reference-held data, not only to the oracle.  The same check runs on the CPU through the
host-simulation build (unmodified kernel source) and on the MI355X (gfx950 build)."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ppu_states.npz")
GREY = np.array([0xFF, 0x99, 0x55, 0x00], np.uint8)
V9 = 142610


def _dummy_rom() -> bytes:
    rom = bytearray(0x8000)
    rom[0x147] = 0x13   # MBC3+RAM+BATTERY like pokemon_red.gb; no code runs
    return bytes(rom)


def _states():
    z = np.load(GOLD)
    prefix, frames, names = z["prefix"], z["frames"], z["names"]
    full = np.zeros((len(prefix), V9), np.uint8)
    full[:, :prefix.shape[1]] = prefix          # the renderer needs only the state prefix
    return full, frames, names


def _compare(screens, frames, names):
    bad = []
    for i in range(len(frames)):
        want = GREY[frames[i]]
        if not np.array_equal(screens[i], want):
            bad.append((str(names[i]), int((screens[i] != want).sum())))
    return bad


def test_hostsim_k2_matches_264_pyboy_frames():
    from tests.hostsim.sim import SimEmulator
    full, frames, names = _states()
    emu = SimEmulator(_dummy_rom(), len(full), render=True)
    for i, st in enumerate(full):
        emu.load_env(i, st.tobytes())
    emu.render_latched()
    bad = _compare(emu.screen(), frames, names)
    emu.close()
    assert not bad, bad[:10]


@pytest.mark.gpu
def test_gpu_k2_matches_264_pyboy_frames():
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    full, frames, names = _states()
    emu = BatchedEmulator(_dummy_rom(), len(full), render=True)
    for i, st in enumerate(full):
        emu.load_env(i, st.tobytes())
    emu.render_latched()
    torch.cuda.synchronize()
    bad = _compare(emu.screen.cpu().numpy(), frames, names)
    emu.close()
    assert not bad, bad[:10]
