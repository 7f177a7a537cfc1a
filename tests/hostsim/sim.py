"""Drive the host-simulation build of the C ABI (tests/hostsim) with numpy buffers.
TEST INFRASTRUCTURE ONLY: checks the HIP kernels' logic against the oracle on the CPU."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from pokegym_amd._native import PkConfig

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libpk_hostsim.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.pk_create.argtypes = [ctypes.POINTER(PkConfig), ctypes.POINTER(vp)]
        L.pk_destroy.argtypes = [vp]
        L.pk_last_error.restype = ctypes.c_char_p
        L.pk_step.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.pk_snapshot.argtypes = [vp, ctypes.c_uint32, u8p, ctypes.c_uint64]
        L.pk_load_env.argtypes = [vp, ctypes.c_uint32, u8p, ctypes.c_uint64]
        L.pk_screen_ptr.argtypes = [vp]
        L.pk_screen_ptr.restype = vp
        L.pk_snapshot_range.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_uint64]
        L.pk_render_latched.argtypes = [vp, vp]
        _lib = L
    return _lib


class SimEmulator:
    def __init__(self, rom: bytes, n: int, state: bytes | None = None, render: bool = True):
        L = lib()
        self._rom = np.frombuffer(rom, np.uint8).copy()
        cfg = PkConfig()
        cfg.n_envs = n
        cfg.rom = self._rom.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
        cfg.rom_len = len(self._rom)
        if state is not None:
            self._st = np.frombuffer(state, np.uint8).copy()
            cfg.state = self._st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
            cfg.state_len = len(self._st)
        cfg.frame_skip, cfg.release_frame, cfg.flags, cfg.max_episode_steps = 24, 8, 1 if render else 0, 20480
        h = ctypes.c_void_p()
        rc = L.pk_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc:
            raise RuntimeError(L.pk_last_error().decode())
        self.h, self.n = h, n

    def step(self, actions: np.ndarray):
        a = np.ascontiguousarray(actions, np.uint8)
        rc = lib().pk_step(self.h, a.ctypes.data, None, None, None, None, None)
        if rc:
            raise RuntimeError(lib().pk_last_error().decode())

    def last_instr_count(self) -> int:
        v = ctypes.c_uint64()
        lib().pk_last_instr_count(self.h, ctypes.byref(v))
        return int(v.value)

    def snapshot(self, e: int) -> bytes:
        out = np.zeros(142610, np.uint8)
        lib().pk_snapshot(self.h, e, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(out))
        return out.tobytes()

    def snapshot_range(self, e0: int, count: int) -> np.ndarray:
        out = np.zeros((count, 142610), np.uint8)
        rc = lib().pk_snapshot_range(self.h, e0, count, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), out.size)
        if rc:
            raise RuntimeError(lib().pk_last_error().decode())
        return out

    def load_env(self, e: int, state: bytes):
        a = np.frombuffer(state, np.uint8).copy()
        rc = lib().pk_load_env(self.h, e, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(a))
        if rc:
            raise RuntimeError(lib().pk_last_error().decode())

    def render_latched(self):
        rc = lib().pk_render_latched(self.h, None)
        if rc:
            raise RuntimeError(lib().pk_last_error().decode())

    def screen(self) -> np.ndarray:
        p = lib().pk_screen_ptr(self.h)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(self.n, 144, 160)).copy()

    def close(self):
        if self.h:
            lib().pk_destroy(self.h)
            self.h = None
