"""BatchedEmulator — N Game Boys on one MI355X behind the C ABI (include/pokegym_amd.h).

This is the device-side replacement of pokegym's per-process PyBoy instance
(pokegym/pyboy_binding.py:42-91): one call to `step(actions)` advances every env by one
env-step (press, 24 frames, release before frame 8, rasterise frame 24) inside one HIP launch.
With `reward=True` the same call also runs pokegym's reward stack and builds the (72, 80, 4)
observation (environment.py:1338-1612, :256-274) on the device.  Device buffers are
PyTorch-ROCm tensors; the kernels run on the caller's current HIP stream.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native
from .info import NFIELDS, event_dicts, info_dict
from ._native import (COLS, ERR_EXCEPTIONS, OBS_SHAPE, PK_F_RELOAD_ON_RESET, PK_F_RENDER, PK_F_REWARD, ROWS,
                      STATE_V9_BYTES, check)


class _CudaArray:
    """__cuda_array_interface__ shim to wrap a handle-owned device buffer without a copy."""

    def __init__(self, ptr: int, shape, typestr: str):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr,
                                         "data": (ptr, False), "version": 2, "strides": None}


def _u8p(buf: bytes | bytearray | np.ndarray):
    a = np.frombuffer(bytes(buf), dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


class BatchedEmulator:
    def __init__(self, rom: bytes, n_envs: int, state: bytes | None = None, device: int = 0,
                 frame_skip: int = 24, release_frame: int = 8, render: bool = True,
                 max_episode_steps: int = 20480, reward: bool = False, reload_on_reset: bool = False,
                 reward_scale: float = 4.0, heatmap: bool = False):
        self._L = _native.load()
        if not torch.cuda.is_available():
            raise _native.PkError("no ROCm GPU visible: the HIP path has no CPU fallback")
        self.device = torch.device("cuda", device)
        self.n = int(n_envs)
        self._rom, rom_p = _u8p(rom)
        cfg = _native.PkConfig()
        cfg.n_envs = self.n
        cfg.device = device
        cfg.rom = rom_p
        cfg.rom_len = len(self._rom)
        if state is not None:
            self._state, st_p = _u8p(state)
            cfg.state = st_p
            cfg.state_len = len(self._state)
        cfg.frame_skip = frame_skip
        cfg.release_frame = release_frame
        cfg.flags = ((PK_F_RENDER if render else 0) | (PK_F_REWARD if reward else 0)
                     | (PK_F_RELOAD_ON_RESET if reload_on_reset else 0)
                     | (_native.PK_F_HEATMAP if (heatmap and reward) else 0))
        cfg.max_episode_steps = max_episode_steps
        cfg.reward_scale = reward_scale
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self._L.pk_create(ctypes.byref(cfg), ctypes.byref(h)), "pk_create")
        self._h = h
        self.render = render
        self.reward = reward
        self.max_episode_steps, self.reward_scale = int(max_episode_steps), float(reward_scale)
        ptr = self._L.pk_screen_ptr(self._h)
        self.screen = torch.as_tensor(_CudaArray(ptr, (self.n, ROWS, COLS), "|u1"), device=self.device)
        self.obs = None
        self.errors = None
        self.heatmap = None     # int32 (n, 444, 436) with heatmap=True
        self.info_bits = None
        self.info = None        # f64 (PK_INFO_NFIELDS, n) view, field-major (pokegym_amd/info.py FIELDS)
        self.info_flag = None   # u8 (n,): 1 where the last step built the reference's info dict
        if reward:
            self.obs = torch.as_tensor(_CudaArray(self._L.pk_obs_ptr(self._h), (self.n,) + OBS_SHAPE, "|u1"),
                                       device=self.device)
            self.errors = torch.as_tensor(_CudaArray(self._L.pk_error_ptr(self._h), (self.n,), "<i4"),
                                          device=self.device)
            stride = int(self._L.pk_info_stride(self._h))
            full = torch.as_tensor(_CudaArray(self._L.pk_info_ptr(self._h), (NFIELDS, stride), "<f8"),
                                   device=self.device)
            self.info = full[:, :self.n]
            bits = torch.as_tensor(_CudaArray(self._L.pk_info_bits_ptr(self._h), (5, stride), "<i4"), device=self.device)
            self.info_bits = bits[:, :self.n]   # event-monitor bits (int32 words; pokegym_amd/info.py event_dicts)
            self.info_flag = torch.as_tensor(_CudaArray(self._L.pk_info_flag_ptr(self._h), (self.n,), "|u1"),
                                             device=self.device)
            hp = self._L.pk_heatmap_ptr(self._h)
            if hp:   # int32 (n, 444, 436) counts_map of every env (environment.py:448, :648-679)
                self.heatmap = torch.as_tensor(_CudaArray(hp, (self.n,) + _native.HEAT_SHAPE, "<i4"), device=self.device)
        self.rewards = torch.zeros(self.n, dtype=torch.float64, device=self.device)
        self.terminals = torch.zeros(self.n, dtype=torch.uint8, device=self.device)
        self.truncations = torch.zeros(self.n, dtype=torch.uint8, device=self.device)
        self.actions = torch.full((self.n,), 8, dtype=torch.uint8, device=self.device)  # sub-batch staging

    # -- stream helpers -----------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # -- hot path -----------------------------------------------------------------------
    def step(self, actions: torch.Tensor):
        """actions: uint8[n] on this device.  Returns (obs, rewards, terminals, truncations) where
        obs is the (n, 72, 80, 4) observation with reward=True, else the (n, 144, 160) screen."""
        if actions.dtype != torch.uint8 or actions.device != self.device or actions.numel() != self.n:
            raise ValueError("actions must be a uint8 tensor of n_envs elements on the emulator's device")
        actions = actions.contiguous()
        check(self._L.pk_step(self._h, ctypes.c_void_p(actions.data_ptr()), None,
                              ctypes.c_void_p(self.rewards.data_ptr()),
                              ctypes.c_void_p(self.terminals.data_ptr()),
                              ctypes.c_void_p(self.truncations.data_ptr()), self._stream()), "pk_step")
        return (self.obs if self.reward else self.screen), self.rewards, self.terminals, self.truncations

    def step_range(self, env0: int, actions: torch.Tensor):
        """One env-step of the sub-batch [env0, env0 + len(actions)) only (pk_step_range), on the
        current stream: env0 is a multiple of 64, the end anywhere up to n.  Returns views of
        the sub-batch's (obs, rewards, terminals, truncations)."""
        count = actions.numel()
        sl = slice(env0, env0 + count)
        self.actions[sl].copy_(actions.reshape(-1))
        check(self._L.pk_step_range(self._h, env0, count, ctypes.c_void_p(self.actions.data_ptr()),
                                    ctypes.c_void_p(self.rewards.data_ptr()), ctypes.c_void_p(self.terminals.data_ptr()),
                                    ctypes.c_void_p(self.truncations.data_ptr()), self._stream()), "pk_step_range")
        obs = self.obs if self.reward else self.screen
        return obs[sl], self.rewards[sl], self.terminals[sl], self.truncations[sl]

    def reset_range(self, env0: int, count: int, mask: torch.Tensor | None = None):
        """Reset the envs of [env0, env0 + count) — all of them, or those with mask[e] != 0 where
        mask is a FULL-size (n) device u8 tensor (e.g. `terminals`; only the range is read) —
        pk_reset_range on the current stream."""
        mp = None
        if mask is not None:
            if mask.dtype != torch.uint8 or mask.device != self.device or mask.numel() != self.n or not mask.is_contiguous():
                raise ValueError("reset_range mask must be a contiguous uint8 tensor of n_envs elements on the device")
            mp = ctypes.c_void_p(mask.data_ptr())
        check(self._L.pk_reset_range(self._h, env0, count, mp, self._stream()), "pk_reset_range")
        obs = self.obs if self.reward else self.screen
        return obs[env0:env0 + count]

    def reset(self, mask: torch.Tensor | None = None):
        """Reset all envs (mask None) or those with mask[e] != 0 (device tensor).  Returns the obs."""
        mp = None
        if mask is not None:
            mask = mask.to(device=self.device, dtype=torch.uint8).contiguous()
            mp = ctypes.c_void_p(mask.data_ptr())
        check(self._L.pk_reset(self._h, mp, self._stream()), "pk_reset")
        return self.obs if self.reward else self.screen

    def set_episode_params(self, max_episode_steps: int, reward_scale: float):
        """Episode length and reward scale of the following steps (Environment.reset's arguments,
        environment.py:1233, :1258-1259); call before the reset they belong to."""
        check(self._L.pk_set_episode_params(self._h, int(max_episode_steps), float(reward_scale)), "pk_set_episode_params")
        self.max_episode_steps, self.reward_scale = int(max_episode_steps), float(reward_scale)

    def raise_if_failed(self, env: int | None = None):
        """Raise the exception the reference would have raised for a failed env (PK_ERR_*)."""
        if self.errors is None:
            return
        err = self.errors if env is None else self.errors[env:env + 1]
        bad = torch.nonzero(err).flatten()
        if bad.numel():
            e = int(bad[0]) + (0 if env is None else env)
            code = int(self.errors[e])
            raise ERR_EXCEPTIONS.get(code, RuntimeError)(f"env {e}: reference reward stack raises here (PK_ERR {code})")

    def info_dicts(self, envs=None) -> dict:
        """{env: info dict} for the envs whose last step built one (host sync; environment.py:1621-1704)."""
        if self.info_flag is None:
            return {}
        flag = self.info_flag if envs is None else self.info_flag[envs]
        ids = torch.nonzero(flag).flatten()
        if envs is not None:
            ids = torch.as_tensor(envs, device=self.device).reshape(-1)[ids]
        if not ids.numel():
            return {}
        rec = self.info[:, ids].t().cpu().numpy()
        bits = (self.info_bits[:, ids].t().cpu().numpy().astype(np.int64) & 0xFFFFFFFF)
        return {int(e): {**info_dict(r), **event_dicts(b)} for e, r, b in zip(ids.tolist(), rec, bits)}

    # -- bulk RAM views (stream-ordered) ------------------------------------------------
    def get_ram(self, addr: int, length: int, out: torch.Tensor | None = None) -> torch.Tensor:
        if out is None:
            out = torch.empty((self.n, length), dtype=torch.uint8, device=self.device)
        check(self._L.pk_get_ram(self._h, addr, length, ctypes.c_void_p(out.data_ptr()), self._stream()), "pk_get_ram")
        return out

    def set_ram(self, addr: int, data: torch.Tensor):
        data = data.to(device=self.device, dtype=torch.uint8).contiguous()
        length = data.numel() // self.n
        check(self._L.pk_set_ram(self._h, addr, length, ctypes.c_void_p(data.data_ptr()), self._stream()), "pk_set_ram")

    # -- host-side accessors (synchronous) --------------------------------------------
    def snapshot(self, env: int) -> bytes:
        out = np.zeros(STATE_V9_BYTES, np.uint8)
        check(self._L.pk_snapshot(self._h, env, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(out)),
              "pk_snapshot")
        return out.tobytes()

    def snapshot_range(self, env0: int, count: int) -> np.ndarray:
        """v9 savestates of envs [env0, env0 + count) as a (count, 142610) uint8 array (bulk pk_snapshot)."""
        out = np.zeros((count, STATE_V9_BYTES), np.uint8)
        check(self._L.pk_snapshot_range(self._h, env0, count, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                        out.size), "pk_snapshot_range")
        return out

    def render_latched(self):
        """Rasterise every env's latched scanlines into `screen` (K2 over a loaded state)."""
        check(self._L.pk_render_latched(self._h, self._stream()), "pk_render_latched")
        return self.screen

    def load_env(self, env: int, state: bytes):
        a, p = _u8p(state)
        check(self._L.pk_load_env(self._h, env, p, len(a)), "pk_load_env")

    def peek(self, env: int, addr: int, n: int = 1) -> bytes:
        out = np.zeros(n, np.uint8)
        check(self._L.pk_peek(self._h, env, addr, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))), "pk_peek")
        return out.tobytes()

    def poke(self, env: int, addr: int, data: bytes):
        a, p = _u8p(data)
        check(self._L.pk_poke(self._h, env, addr, len(a), p), "pk_poke")

    def last_instr_count(self) -> int:
        v = ctypes.c_uint64()
        check(self._L.pk_last_instr_count(self._h, ctypes.byref(v)), "pk_last_instr_count")
        return int(v.value)

    def launch_shape(self, env0: int = 0, count: int | None = None) -> dict:
        """The K1 launch pk_step_range(env0, count) takes (pk_launch_shape; host-side, no GPU work)."""
        out = (ctypes.c_uint32 * 5)()
        count = self.n - env0 if count is None else count
        check(self._L.pk_launch_shape(self._h, env0, count, out), "pk_launch_shape")
        return {"small": bool(out[0]), "wave_lanes": int(out[1]), "block": int(out[2]), "prio": bool(out[3]),
                "all_staged": bool(out[4])}

    def profile_enable(self, on: bool = True):
        check(self._L.pk_profile_enable(self._h, 1 if on else 0), "pk_profile_enable")

    def profile_read(self):
        """(emulate_ms, render_ms, reward_ms, steps) summed since the last read (synchronous)."""
        a, b, c, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
        check(self._L.pk_profile_read(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(n)),
              "pk_profile_read")
        return a.value, b.value, c.value, int(n.value)

    def close(self):
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            self.screen = None
            self.obs = None
            self.errors = None
            self.info = self.info_flag = self.heatmap = self.info_bits = None
            self._L.pk_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
