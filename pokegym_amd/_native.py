"""ctypes binding of the C ABI in include/pokegym_amd.h (libpokegym_amd.so, built in-tree).

This is the reference-side binding a maintainer would add.  There is no
CPU fallback: if the HIP library is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# PK_LIB selects an alternative in-tree build (A/B kernel experiments); default: lib/libpokegym_amd.so
LIB_PATH = os.environ.get("PK_LIB") or os.path.join(HERE, "lib", "libpokegym_amd.so")

ABI_VERSION = 6
PK_F_RENDER = 1
PK_F_REWARD = 2
PK_F_RELOAD_ON_RESET = 4
PK_F_HEATMAP = 8
HEAT_SHAPE = (444, 436)
OBS_SHAPE = (72, 80, 4)
# PK_ERR_* -> the exception the reference raises at that point (include/pokegym_amd.h)
ERR_EXCEPTIONS = {1: KeyError, 2: AttributeError, 3: IndexError, 4: UnboundLocalError, 5: IndexError,
                  6: IndexError, 7: MemoryError, 8: ValueError}
STATE_V9_BYTES = 142610
ROWS, COLS = 144, 160

# the exported symbols declared in include/pokegym_amd.h
EXPORTS = ("pk_create", "pk_destroy", "pk_last_error", "pk_abi_version", "pk_reset", "pk_step",
           "pk_screen_ptr", "pk_num_envs", "pk_peek", "pk_poke", "pk_snapshot", "pk_load_env",
           "pk_last_instr_count", "pk_profile_enable", "pk_profile_read", "pk_obs_ptr", "pk_error_ptr",
           "pk_get_ram", "pk_set_ram", "pk_info_ptr", "pk_info_flag_ptr", "pk_info_stride", "pk_heatmap_ptr", "pk_info_bits_ptr",
           "pk_snapshot_range", "pk_render_latched", "pk_step_range", "pk_reset_range",
           "pk_set_episode_params", "pk_launch_shape")


class PkConfig(ctypes.Structure):
    _fields_ = [
        ("n_envs", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("rom", ctypes.POINTER(ctypes.c_uint8)),
        ("rom_len", ctypes.c_uint64),
        ("state", ctypes.POINTER(ctypes.c_uint8)),
        ("state_len", ctypes.c_uint64),
        ("frame_skip", ctypes.c_uint32),
        ("release_frame", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("max_episode_steps", ctypes.c_uint32),
        ("reward_scale", ctypes.c_double),
    ]


class PkError(RuntimeError):
    pass


_lib = None


def load(path: str = LIB_PATH):
    """Load the HIP library; raise loudly if it is absent (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise PkError(f"{path} not found: build it with `python -m pokegym_amd.build` "
                      "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = ctypes.CDLL(path)
    bind(L)
    _lib = L
    return L


def bind(L):
    """argtypes of every entry point of include/pokegym_amd.h (shared with the host-simulation
    test build, tests/hostsim)."""
    u8p = ctypes.POINTER(ctypes.c_uint8)
    vp = ctypes.c_void_p
    L.pk_create.argtypes = [ctypes.POINTER(PkConfig), ctypes.POINTER(vp)]
    L.pk_destroy.argtypes = [vp]
    L.pk_destroy.restype = None
    L.pk_last_error.restype = ctypes.c_char_p
    L.pk_reset.argtypes = [vp, vp, vp]
    L.pk_step.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.pk_screen_ptr.argtypes = [vp]
    L.pk_screen_ptr.restype = vp
    L.pk_num_envs.argtypes = [vp]
    L.pk_num_envs.restype = ctypes.c_uint32
    L.pk_peek.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_uint32, u8p]
    L.pk_poke.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_uint32, u8p]
    L.pk_snapshot.argtypes = [vp, ctypes.c_uint32, u8p, ctypes.c_uint64]
    L.pk_load_env.argtypes = [vp, ctypes.c_uint32, u8p, ctypes.c_uint64]
    L.pk_snapshot_range.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, u8p, ctypes.c_uint64]
    L.pk_render_latched.argtypes = [vp, vp]
    L.pk_last_instr_count.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    L.pk_launch_shape.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    L.pk_profile_enable.argtypes = [vp, ctypes.c_int]
    dp = ctypes.POINTER(ctypes.c_double)
    L.pk_profile_read.argtypes = [vp, dp, dp, dp, ctypes.POINTER(ctypes.c_uint64)]
    bind_v2(L)


def bind_v2(L):
    """argtypes of the ABI-v2 entry points (shared with the host-simulation test build)."""
    vp = ctypes.c_void_p
    L.pk_obs_ptr.argtypes = [vp]
    L.pk_obs_ptr.restype = vp
    L.pk_error_ptr.argtypes = [vp]
    L.pk_error_ptr.restype = vp
    L.pk_info_ptr.argtypes = [vp]
    L.pk_info_ptr.restype = vp
    L.pk_info_flag_ptr.argtypes = [vp]
    L.pk_info_flag_ptr.restype = vp
    L.pk_info_stride.argtypes = [vp]
    L.pk_info_stride.restype = ctypes.c_uint32
    L.pk_heatmap_ptr.argtypes = [vp]
    L.pk_heatmap_ptr.restype = vp
    L.pk_info_bits_ptr.argtypes = [vp]
    L.pk_info_bits_ptr.restype = vp
    L.pk_get_ram.argtypes = [vp, ctypes.c_uint16, ctypes.c_uint32, vp, vp]
    L.pk_set_ram.argtypes = [vp, ctypes.c_uint16, ctypes.c_uint32, vp, vp]
    L.pk_reset.argtypes = [vp, vp, vp]
    L.pk_step_range.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp, vp]
    L.pk_reset_range.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, vp, vp]
    L.pk_set_episode_params.argtypes = [vp, ctypes.c_uint32, ctypes.c_double]


def check(rc: int, what: str):
    if rc != 0:
        msg = load().pk_last_error().decode(errors="replace")
        raise PkError(f"{what} failed ({rc}): {msg}")
