"""Host-simulation backend for tests/reward_replay.run_replay (TEST INFRASTRUCTURE ONLY)."""
from __future__ import annotations

import ctypes

import numpy as np

from pokegym_amd._native import PK_F_REWARD, PkConfig, bind_v2
from pokegym_amd.info import NFIELDS as PK_INFO_NFIELDS

import sim


class HostsimRewardBackend:
    def __init__(self, rom: bytes):
        self.L = sim.lib()
        bind_v2(self.L)
        self.rom = np.frombuffer(rom, np.uint8).copy()
        self._keep = {}

    def _chk(self, rc, what):
        if rc:
            raise RuntimeError(f"{what}: {self.L.pk_last_error().decode()}")

    def create(self, state: bytes, max_steps: int):
        st = np.frombuffer(state, np.uint8).copy()
        cfg = PkConfig()
        cfg.n_envs = 1
        cfg.rom = self.rom.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        cfg.rom_len = len(self.rom)
        cfg.state = st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        cfg.state_len = len(st)
        cfg.frame_skip, cfg.release_frame, cfg.flags, cfg.max_episode_steps = 0, 8, PK_F_REWARD | 8, max_steps
        cfg.reward_scale = 4.0
        h = ctypes.c_void_p()
        self._chk(self.L.pk_create(ctypes.byref(cfg), ctypes.byref(h)), "pk_create")
        self._keep[h.value] = (st, np.zeros(1, np.float64), np.zeros(1, np.uint8), np.zeros(1, np.uint8))
        return h

    def destroy(self, h):
        self.L.pk_destroy(h)
        self._keep.pop(h.value, None)

    def reset(self, h):
        self._chk(self.L.pk_reset(h, None, None), "pk_reset")

    def step(self, h, action):
        _, rew, term, trunc = self._keep[h.value]
        a = np.array([action], np.uint8)
        self._chk(self.L.pk_step(h, a.ctypes.data, None, rew.ctypes.data, term.ctypes.data, trunc.ctypes.data, None), "pk_step")
        return float(rew[0]), bool(term[0])

    def error(self, h):
        p = self.L.pk_error_ptr(h)
        return int(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32))[0])

    def obs(self, h):
        p = self.L.pk_obs_ptr(h)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(72, 80, 4)).copy()

    def set_ram(self, h, w, hr):
        w = np.ascontiguousarray(w, np.uint8)
        hr = np.ascontiguousarray(hr, np.uint8)
        self._chk(self.L.pk_set_ram(h, 0xC000, 8192, w.ctypes.data, None), "pk_set_ram")
        self._chk(self.L.pk_set_ram(h, 0xFF80, 127, hr.ctypes.data, None), "pk_set_ram")

    def get_ram(self, h):
        w = np.zeros(8192, np.uint8)
        hr = np.zeros(127, np.uint8)
        self._chk(self.L.pk_get_ram(h, 0xC000, 8192, w.ctypes.data, None), "pk_get_ram")
        self._chk(self.L.pk_get_ram(h, 0xFF80, 127, hr.ctypes.data, None), "pk_get_ram")
        return w, hr

    def set_screen(self, h, screen):
        p = self.L.pk_screen_ptr(h)
        ctypes.memmove(p, np.ascontiguousarray(screen, np.uint8).ctypes.data, 144 * 160)

    def info(self, h):
        """The step's info record (pokegym_amd/info.py FIELDS) or None (pk_info_ptr / pk_info_flag_ptr)."""
        f = ctypes.cast(self.L.pk_info_flag_ptr(h), ctypes.POINTER(ctypes.c_uint8))[0]
        if not f:
            return None
        stride = int(self.L.pk_info_stride(h))
        p = ctypes.cast(self.L.pk_info_ptr(h), ctypes.POINTER(ctypes.c_double))
        return [p[i * stride] for i in range(PK_INFO_NFIELDS)]

    def heat(self, h):
        """The env's counts_map, flat float64 (pk_heatmap_ptr)."""
        p = ctypes.cast(self.L.pk_heatmap_ptr(h), ctypes.POINTER(ctypes.c_int32))
        return np.ctypeslib.as_array(p, shape=(444 * 436,)).astype(np.float64)

    def events(self, h):
        """The info step's 130 monitor values (pk_info_bits_ptr -> pokegym_amd.info.event_values)."""
        from pokegym_amd.info import event_values
        stride = int(self.L.pk_info_stride(h))
        p = ctypes.cast(self.L.pk_info_bits_ptr(h), ctypes.POINTER(ctypes.c_uint32))
        return event_values([p[j * stride] for j in range(5)])
