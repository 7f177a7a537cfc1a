"""Import the REFERENCE pokegym Environment in this container, for golden-fixture generation only.

The reference's reward/obs code (pokegym/environment.py, ram_map.py, ram_map_leanke.py,
game_map.py, bin/ram_reader/red_ram_api.py) is pure Python over `get_memory_value` /
`set_memory_value`.  Its import-time dependencies that are absent from this image (pyboy,
gymnasium, skimage, mediapy) are given minimal module stubs that expose only the names the
reference touches at import/construction time; the emulator itself is replaced by `FakePyBoy`,
a 64 KiB byte array that the fixture generator fills with WRAM/HRAM images between steps.

Never imported by tests, smoke() or bench.py; /root/reference does not exist on the GPU box.
Run with `python3 -B` so no __pycache__ is written into the read-only reference.
"""
from __future__ import annotations

import enum
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference/pokegym"

# PyBoy 1.x `pyboy.utils.WindowEvent` ids (QUIT = 0, then the PRESS_* events, then RELEASE_*).
# Only the ordering of the PRESS_* ids is observable by the reference's step(): it compares the
# integer action with WindowEvent.PRESS_BUTTON_A (environment.py:691).  [external, unverifiable here]
WINDOW_EVENTS = ["QUIT", "PRESS_ARROW_UP", "PRESS_ARROW_DOWN", "PRESS_ARROW_RIGHT", "PRESS_ARROW_LEFT",
                 "PRESS_BUTTON_A", "PRESS_BUTTON_B", "PRESS_BUTTON_SELECT", "PRESS_BUTTON_START",
                 "RELEASE_ARROW_UP", "RELEASE_ARROW_DOWN", "RELEASE_ARROW_RIGHT", "RELEASE_ARROW_LEFT",
                 "RELEASE_BUTTON_A", "RELEASE_BUTTON_B", "RELEASE_BUTTON_SELECT", "RELEASE_BUTTON_START"]


class FakeScreen:
    def __init__(self):
        self.frame = np.zeros((144, 160, 3), np.uint8)

    def raw_screen_buffer_dims(self):
        return (144, 160)

    def screen_ndarray(self):
        return self.frame


class FakePyBoy:
    """Byte-addressed memory standing in for PyBoy's bus (get/set_memory_value)."""

    def __init__(self):
        self.mem = np.zeros(0x10000, np.uint8)
        self.writes = []

    def get_memory_value(self, addr):
        return int(self.mem[addr])

    def set_memory_value(self, addr, value):
        self.mem[addr] = value & 0xFF
        self.writes.append((addr, value & 0xFF))

    def load_state(self, f):  # the generator installs images itself
        pass

    def stop(self, save=False):
        pass

    def send_input(self, ev):
        pass


def _install_stubs():
    pk = types.ModuleType("pokegym")
    pk.__path__ = [REF]
    sys.modules["pokegym"] = pk

    pyboy = types.ModuleType("pyboy")
    utils = types.ModuleType("pyboy.utils")
    WE = type("WindowEvent", (), {n: i for i, n in enumerate(WINDOW_EVENTS)})
    utils.WindowEvent = WE
    pyboy.WindowEvent = WE
    pyboy.PyBoy = FakePyBoy
    pyboy.utils = utils
    sys.modules["pyboy"] = pyboy
    sys.modules["pyboy.utils"] = utils

    gym = types.ModuleType("gymnasium")

    class Env:
        pass

    spaces = types.ModuleType("gymnasium.spaces")

    class Box:
        def __init__(self, low=None, high=None, dtype=None, shape=None):
            self.low, self.high, self.dtype, self.shape = low, high, dtype, tuple(shape)

    class Discrete:
        def __init__(self, n):
            self.n = n

    spaces.Box, spaces.Discrete = Box, Discrete
    gym.Env, gym.spaces = Env, spaces
    sys.modules["gymnasium"] = gym
    sys.modules["gymnasium.spaces"] = spaces

    sk = types.ModuleType("skimage")
    skt = types.ModuleType("skimage.transform")
    skt.resize = lambda *a, **k: None
    sk.transform = skt
    sys.modules["skimage"] = sk
    sys.modules["skimage.transform"] = skt

    mp = types.ModuleType("mediapy")
    mp.VideoWriter = object
    sys.modules["mediapy"] = mp


_ENV_MOD = None


def env_module():
    """Import pokegym.environment once (in a scratch cwd: its constructor makes directories)."""
    global _ENV_MOD
    if _ENV_MOD is None:
        sys.dont_write_bytecode = True
        _install_stubs()
        old = os.getcwd()
        os.chdir(tempfile.mkdtemp(prefix="pkref_"))
        try:
            import pokegym.environment as E  # noqa: PLC0415
        finally:
            os.chdir(old)
        _ENV_MOD = E
    return _ENV_MOD


class ReplayEnv:
    """The reference Environment driven by memory images instead of an emulator.

    step(action, wram, hram, screen) installs the images (as if run_action_on_emulator had just
    produced them), then runs the reference's own Environment.step."""

    def __init__(self, wram0, hram0, screen0=None):
        E = env_module()
        self.E = E
        self.game = FakePyBoy()
        self.screen = FakeScreen()
        self._pending = (wram0, hram0, screen0)
        E.make_env = lambda *a, **k: (self.game, self.screen)
        E.load_pyboy_state = lambda pyboy, state: self._install(*self._pending)
        E.run_action_on_emulator = lambda *a, **k: self._install(*self._pending)
        old = os.getcwd()
        os.chdir(tempfile.mkdtemp(prefix="pkref_"))
        try:
            self.env = E.Environment(rom_path="none.gb", state_path=os.path.join(REF, "current_state", "Bulbasaur.state"))
        finally:
            os.chdir(old)

    def _install(self, wram, hram, screen):
        self.game.mem[0xC000:0xE000] = wram
        self.game.mem[0xE000:0xFE00] = wram[:0x1E00]
        self.game.mem[0xFF80:0xFFFF] = hram
        if screen is not None:
            self.screen.frame = np.repeat(screen[:, :, None], 3, axis=2)

    def reset(self, wram=None, hram=None, screen=None):
        if wram is not None:
            self._pending = (wram, hram, screen)
        self.game.writes = []
        obs, info = self.env.reset()
        return obs

    def step(self, action, wram, hram, screen):
        self._pending = (wram, hram, screen)
        self.game.writes = []
        return self.env.step(int(action))
