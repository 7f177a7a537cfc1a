"""BatchedEmulator over the host-simulation build (TEST INFRASTRUCTURE ONLY).

The unmodified kernels + C ABI compiled with g++ (tests/hostsim) keep every "device" buffer in
host memory, so the product's BatchedEmulator runs on CPU tensors wrapped around those buffers.
Used by the CPU tests of the multi-rank benchmark flow (tests/test_dist.py): the product path
itself has no CPU fallback (pokegym_amd/emulator.py refuses to start without a GPU)."""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

import sim  # noqa: E402
from pokegym_amd import _native  # noqa: E402
from pokegym_amd.emulator import BatchedEmulator  # noqa: E402
from pokegym_amd.info import NFIELDS  # noqa: E402


def _host(ptr: int, shape, dtype) -> torch.Tensor:
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    buf = (ctypes.c_uint8 * nbytes).from_address(ptr)
    return torch.from_numpy(np.frombuffer(buf, dtype=dtype).reshape(shape))


class HostsimEmulator(BatchedEmulator):
    def __init__(self, rom: bytes, n_envs: int, state: bytes | None = None, frame_skip: int = 24,
                 release_frame: int = 8, render: bool = True, max_episode_steps: int = 20480, reward: bool = False,
                 reload_on_reset: bool = False, reward_scale: float = 4.0, device=None):
        L = sim.lib()
        _native.bind(L)
        self._L = L
        self.device = torch.device("cpu")
        self.n = int(n_envs)
        self._rom = np.frombuffer(rom, np.uint8).copy()
        cfg = _native.PkConfig()
        cfg.n_envs = self.n
        cfg.rom = self._rom.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        cfg.rom_len = len(self._rom)
        if state is not None:
            self._state = np.frombuffer(state, np.uint8).copy()
            cfg.state = self._state.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
            cfg.state_len = len(self._state)
        cfg.frame_skip, cfg.release_frame = frame_skip, release_frame
        cfg.flags = ((_native.PK_F_RENDER if render else 0) | (_native.PK_F_REWARD if reward else 0)
                     | (_native.PK_F_RELOAD_ON_RESET if reload_on_reset else 0))
        cfg.max_episode_steps, cfg.reward_scale = max_episode_steps, reward_scale
        h = ctypes.c_void_p()
        _native.check(L.pk_create(ctypes.byref(cfg), ctypes.byref(h)), "pk_create")
        self._h = h
        self.render, self.reward = render, reward
        self.max_episode_steps, self.reward_scale = int(max_episode_steps), float(reward_scale)
        self.screen = _host(L.pk_screen_ptr(h), (self.n, _native.ROWS, _native.COLS), np.uint8)
        self.obs = self.errors = self.heatmap = self.info_bits = self.info = self.info_flag = None
        if reward:
            self.obs = _host(L.pk_obs_ptr(h), (self.n,) + _native.OBS_SHAPE, np.uint8)
            self.errors = _host(L.pk_error_ptr(h), (self.n,), np.int32)
            stride = int(L.pk_info_stride(h))
            self.info = _host(L.pk_info_ptr(h), (NFIELDS, stride), np.float64)[:, :self.n]
            self.info_bits = _host(L.pk_info_bits_ptr(h), (5, stride), np.int32)[:, :self.n]
            self.info_flag = _host(L.pk_info_flag_ptr(h), (self.n,), np.uint8)
        self.rewards = torch.zeros(self.n, dtype=torch.float64)
        self.terminals = torch.zeros(self.n, dtype=torch.uint8)
        self.truncations = torch.zeros(self.n, dtype=torch.uint8)
        self.actions = torch.full((self.n,), 8, dtype=torch.uint8)

    def _stream(self):
        return None

    def close(self):
        if getattr(self, "_h", None):
            self.screen = self.obs = self.errors = None
            self.info = self.info_flag = self.heatmap = self.info_bits = None
            self._L.pk_destroy(self._h)
            self._h = None
