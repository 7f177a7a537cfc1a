"""Trajectory parity against PyBoy itself — for a machine that has both.

PyBoy 1.x and pokemon_red.gb are absent from this container and from the GPU pool, so the
emulator's CPU trajectories are pinned to the C restatement (oracle/gbcore.c) only ("parity
unpinned" vs PyBoy).  These tests close that gap wherever both exist: set
POKEGYM_ROM=/path/to/pokemon_red.gb (and have `pyboy<2` importable, as the reference's
setup.py:12 pins) and they run; otherwise they skip.

PyBoy is driven exactly as the reference drives it: make_env (pyboy_binding.py:42-56:
headless window), load_pyboy_state (:59-69) of the shipped start state, and per env-step
run_action_on_emulator (:71-91): send_input(press), _rendering(False), 24 ticks with the
release sent before tick 8 and _rendering(True) before the last tick.  The same state and action
scripts — a_t = 0 as in test.py:20-25, the [0,3,1,2] cycle of configs[1], seeded random presses
— run through the C oracle (CPU test) and through pokegym_amd's HIP emulator (GPU test).  WRAM
(0xC000-0xDFFF, the north_star's bit-exact criterion) is compared every EVERY env-steps and the
rendered screen (screen_ndarray()[..., 0], the grey shades of environment.py:268) at the end.
POKEGYM_PARITY_STEPS sets the horizon (default 1,000; the north_star's is 10,000)."""
from __future__ import annotations

import io
import os

import numpy as np
import pytest

ROM_PATH = os.environ.get("POKEGYM_ROM", "")
STEPS = int(os.environ.get("POKEGYM_PARITY_STEPS", "1000"))
EVERY = 100
GREY = np.array([0xFF, 0x99, 0x55, 0x00], np.uint8)
STATE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pokegym_amd", "states",
                     "Bulbasaur.state")


def _scripts(steps: int) -> np.ndarray:
    """(steps, 3) actions: Down every step, the [0,3,1,2] cycle, seeded random presses 0..7."""
    a = np.empty((steps, 3), np.uint8)
    a[:, 0] = 0
    a[:, 1] = np.array([0, 3, 1, 2], np.uint8)[np.arange(steps) % 4]
    a[:, 2] = np.random.default_rng(1234).integers(0, 8, steps, dtype=np.uint8)
    return a


def _need_pyboy():
    if not ROM_PATH or not os.path.exists(ROM_PATH):
        pytest.skip("POKEGYM_ROM (pokemon_red.gb) not set: PyBoy trajectory parity needs the cartridge")
    pyboy = pytest.importorskip("pyboy")
    if int(str(getattr(pyboy, "__version__", "1")).split(".")[0]) >= 2:
        pytest.skip("the reference pins pyboy<2.0.0 (setup.py:12)")
    with open(ROM_PATH, "rb") as f:
        rom = f.read()
    with open(STATE, "rb") as f:
        state = f.read()
    return rom, state


def pyboy_trajectory(actions: np.ndarray, every: int = EVERY):
    """The reference's emulator loop on PyBoy: WRAM every `every` env-steps, final grey screen."""
    from pyboy import PyBoy
    from pyboy.utils import WindowEvent
    W = WindowEvent
    # pyboy_binding.py:7-40 ACTIONS order: Down Left Right Up A B Start Select
    table = [(W.PRESS_ARROW_DOWN, W.RELEASE_ARROW_DOWN), (W.PRESS_ARROW_LEFT, W.RELEASE_ARROW_LEFT),
             (W.PRESS_ARROW_RIGHT, W.RELEASE_ARROW_RIGHT), (W.PRESS_ARROW_UP, W.RELEASE_ARROW_UP),
             (W.PRESS_BUTTON_A, W.RELEASE_BUTTON_A), (W.PRESS_BUTTON_B, W.RELEASE_BUTTON_B),
             (W.PRESS_BUTTON_START, W.RELEASE_BUTTON_START), (W.PRESS_BUTTON_SELECT, W.RELEASE_BUTTON_SELECT)]
    with open(STATE, "rb") as f:
        state = io.BytesIO(f.read())
    game = PyBoy(ROM_PATH, debugging=False, window_type="headless", hide_window=True)
    screen = game.botsupport_manager().screen()
    state.seek(0)
    game.load_state(state)
    wram = []
    for t, a in enumerate(actions):
        press, release = table[int(a)]
        game.send_input(press)
        game._rendering(False)
        for i in range(24):
            if i == 8:
                game.send_input(release)
            if i == 23:
                game._rendering(True)
            game.tick()
        if (t + 1) % every == 0:
            wram.append(bytes(game.get_memory_value(x) for x in range(0xC000, 0xE000)))
    final = np.asarray(screen.screen_ndarray())[..., 0].copy()
    game.stop(save=False)
    return wram, final


def _first_diff(want: list, got: list, every: int):
    for k, (w, g) in enumerate(zip(want, got)):
        if w != g:
            wa, ga = np.frombuffer(w, np.uint8), np.frombuffer(g, np.uint8)
            i = int(np.nonzero(wa != ga)[0][0])
            return f"step {(k + 1) * every}: WRAM {0xC000 + i:#06x} PyBoy {wa[i]:#04x} vs {ga[i]:#04x} ({int((wa != ga).sum())} bytes differ)"
    return None


def test_oracle_matches_pyboy_trajectories():
    """C restatement (oracle/gbcore.c) vs PyBoy on the reference's start state."""
    rom, state = _need_pyboy()
    from oracle import oracle
    acts = _scripts(STEPS)
    for j in range(acts.shape[1]):
        want, want_screen = pyboy_trajectory(acts[:, j])
        g = oracle.GB(rom, state)
        got = []
        for t, a in enumerate(acts[:, j]):
            g.run_action(int(a))
            if (t + 1) % EVERY == 0:
                got.append(g.wram().tobytes())
        diff = _first_diff(want, got, EVERY)
        assert diff is None, f"trajectory {j}: {diff}"
        assert np.array_equal(GREY[g.screen()], want_screen), f"trajectory {j}: final screen differs"


@pytest.mark.gpu
def test_gpu_matches_pyboy_trajectories():
    """pokegym_amd's HIP emulator (one lane per trajectory) vs PyBoy on the reference's start state."""
    rom, state = _need_pyboy()
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    acts = _scripts(STEPS)
    n = acts.shape[1]
    emu = BatchedEmulator(rom, n, state=state, render=True)
    dev = torch.from_numpy(acts).to(emu.device)
    got = [[] for _ in range(n)]
    for t in range(STEPS):
        emu.step(dev[t])
        if (t + 1) % EVERY == 0:
            for j in range(n):
                got[j].append(emu.peek(j, 0xC000, 0x2000))
    screens = emu.screen.cpu().numpy()
    emu.close()
    for j in range(n):
        want, want_screen = pyboy_trajectory(acts[:, j])
        diff = _first_diff(want, got[j], EVERY)
        assert diff is None, f"trajectory {j}: {diff}"
        assert np.array_equal(screens[j], want_screen), f"trajectory {j}: final screen differs"
