"""ctypes wrapper for the CPU oracle (oracle/gbcore.c). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module;
the product path (pokegym_amd) never does.  See gbcore.h for what the oracle restates and its
parity status (PPU/savestate pinned on the reference's 264 savestates; CPU trajectories vs
PyBoy unpinned).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libgbcore.so")
STATE_SIZE = 142610
ROWS, COLS = 144, 160

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.gb_new.restype = ctypes.c_void_p
        L.gb_new.argtypes = [u8p, ctypes.c_uint32]
        L.gb_free.argtypes = [ctypes.c_void_p]
        L.gb_clone.restype = ctypes.c_void_p
        L.gb_clone.argtypes = [ctypes.c_void_p]
        L.gb_power_on.argtypes = [ctypes.c_void_p]
        L.gb_load_state.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint32]
        L.gb_save_state.argtypes = [ctypes.c_void_p, u8p, ctypes.c_uint32]
        L.gb_button.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.gb_set_rendering.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.gb_tick.argtypes = [ctypes.c_void_p]
        L.gb_run_action.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.gb_read.restype = ctypes.c_uint8
        L.gb_read.argtypes = [ctypes.c_void_p, ctypes.c_uint16]
        L.gb_write.argtypes = [ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint8]
        L.gb_screen_shades.restype = u8p
        L.gb_screen_shades.argtypes = [ctypes.c_void_p]
        L.gb_wram.restype = u8p
        L.gb_wram.argtypes = [ctypes.c_void_p]
        L.gb_instr_count.restype = ctypes.c_uint64
        L.gb_instr_count.argtypes = [ctypes.c_void_p]
        L.gb_frame_count.restype = ctypes.c_uint64
        L.gb_frame_count.argtypes = [ctypes.c_void_p]
        L.gb_crashed.argtypes = [ctypes.c_void_p]
        L.gb_render_from_state.argtypes = [u8p, ctypes.c_uint32, u8p]
        L.gb_batch_run.argtypes = [u8p, ctypes.c_uint32, u8p, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_uint32, u8p, ctypes.c_int, u8p, u8p]
        L.gb_bench.restype = ctypes.c_double
        L.gb_bench.argtypes = [u8p, ctypes.c_uint32, u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def render_from_state(state: bytes) -> np.ndarray:
    """PPU restatement: render 144x160 shade ids from a v9 state's VRAM/OAM/regs/line params."""
    s = np.frombuffer(state, dtype=np.uint8).copy()
    out = np.zeros((ROWS, COLS), np.uint8)
    rc = lib().gb_render_from_state(_ptr(s), len(s), _ptr(out))
    if rc:
        raise ValueError(f"gb_render_from_state failed: {rc}")
    return out


class GB:
    """One oracle emulator (PyBoy-1.x-shaped)."""

    def __init__(self, rom: bytes, state: bytes | None = None, _handle=None):
        self._rom = np.frombuffer(rom, dtype=np.uint8).copy()  # keep alive: gbcore borrows it
        L = lib()
        self.h = _handle if _handle is not None else L.gb_new(_ptr(self._rom), len(self._rom))
        if not self.h:
            raise ValueError("unsupported ROM (size/MBC)")
        if state is not None:
            self.load_state(state)

    def __del__(self):
        if getattr(self, "h", None):
            lib().gb_free(self.h)
            self.h = None

    def clone(self) -> "GB":
        g = GB.__new__(GB)
        g._rom = self._rom
        g.h = lib().gb_clone(self.h)
        return g

    def load_state(self, state: bytes):
        s = np.frombuffer(state, dtype=np.uint8).copy()
        if lib().gb_load_state(self.h, _ptr(s), len(s)):
            raise ValueError("bad v9 savestate")

    def save_state(self) -> bytes:
        out = np.zeros(STATE_SIZE, np.uint8)
        lib().gb_save_state(self.h, _ptr(out), STATE_SIZE)
        return out.tobytes()

    def power_on(self):
        lib().gb_power_on(self.h)

    def tick(self):
        lib().gb_tick(self.h)

    def button(self, b: int, pressed: bool):
        lib().gb_button(self.h, b, 1 if pressed else 0)

    def set_rendering(self, on: bool):
        lib().gb_set_rendering(self.h, 1 if on else 0)

    def run_action(self, action: int, frame_skip: int = 24, release_frame: int = 8):
        lib().gb_run_action(self.h, int(action), frame_skip, release_frame)

    def read(self, addr: int) -> int:
        return lib().gb_read(self.h, addr)

    def write(self, addr: int, v: int):
        lib().gb_write(self.h, addr, v)

    def screen(self) -> np.ndarray:
        p = lib().gb_screen_shades(self.h)
        return np.ctypeslib.as_array(p, shape=(ROWS, COLS)).copy()

    def wram(self) -> np.ndarray:
        p = lib().gb_wram(self.h)
        return np.ctypeslib.as_array(p, shape=(8192,)).copy()

    @property
    def instr_count(self) -> int:
        return lib().gb_instr_count(self.h)

    @property
    def crashed(self) -> bool:
        return bool(lib().gb_crashed(self.h))


def threads() -> int:
    """Oracle threads for a batch: the host's CPU share, at most 16 (the GPU box allots 16 cores to
    one GPU; os.cpu_count() there shows the whole machine).  PK_ORACLE_PROCS overrides."""
    return max(1, min(16, os.cpu_count() or 1, int(os.environ.get("PK_ORACLE_PROCS", "16"))))


def batch_run(rom: bytes, state: bytes | None, actions: np.ndarray, want_states=True, want_screens=True,
              nthreads: int | None = None):
    """Run n envs x steps env-steps; actions shape (steps, n) uint8. Returns (states, screens).
    Envs are independent, so contiguous env chunks run on threads (ctypes drops the GIL around the
    re-entrant C call; each chunk clones its own template)."""
    actions = np.ascontiguousarray(actions, dtype=np.uint8)
    steps, n = actions.shape
    r = np.frombuffer(rom, dtype=np.uint8).copy()
    st = np.frombuffer(state, dtype=np.uint8).copy() if state is not None else None
    so = np.zeros((n, STATE_SIZE), np.uint8) if want_states else None
    sc = np.zeros((n, ROWS, COLS), np.uint8) if want_screens else None
    L = lib()

    def run(e0, e1):
        a = np.ascontiguousarray(actions[:, e0:e1])
        rc = L.gb_batch_run(_ptr(r), len(r), _ptr(st) if st is not None else None,
                            len(st) if st is not None else 0, e1 - e0, steps, _ptr(a), 1,
                            _ptr(so[e0:e1]) if so is not None else None, _ptr(sc[e0:e1]) if sc is not None else None)
        if rc:
            raise ValueError(f"gb_batch_run failed: {rc}")

    k = max(1, min(nthreads or threads(), n // 8 or 1))
    if k == 1:
        run(0, n)
    else:
        from concurrent.futures import ThreadPoolExecutor
        cuts = [n * i // k for i in range(k + 1)]
        with ThreadPoolExecutor(k) as ex:
            for f in [ex.submit(run, cuts[i], cuts[i + 1]) for i in range(k)]:
                f.result()
    return so, sc


def intensity(rom: bytes, state: bytes | None, n: int, warmup: int, steps: int, seed: int) -> dict:
    """Workload intensity of gb_bench's action stream (oracle/gbcore.c gb_intensity)."""
    r = np.frombuffer(rom, dtype=np.uint8).copy()
    st = np.frombuffer(state, dtype=np.uint8).copy() if state is not None else None
    out = np.zeros(6, np.uint64)
    L = lib()
    L.gb_intensity.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    rc = L.gb_intensity(_ptr(r), len(r), _ptr(st) if st is not None else None, len(st) if st is not None else 0,
                        n, warmup, steps, seed, out.ctypes.data)
    if rc:
        raise ValueError(f"gb_intensity failed: {rc}")
    instr, ticks, cyc, halted, lcdoff, frames = (int(x) for x in out)
    return {"instr_per_env_step": instr / (n * steps), "ticks_per_env_step": ticks / (n * steps),
            "halted_frac": halted / max(cyc, 1), "lcd_off_frac": lcdoff / max(cyc, 1),
            "busy_cycles_per_frame": (cyc - halted) / max(frames, 1), "cycles_per_frame": cyc / max(frames, 1)}


def bench(rom: bytes, state: bytes | None, n: int, warmup: int, steps: int, seed: int):
    """Single-thread CPU timing of the oracle: returns (seconds, emulated_instructions)."""
    r = np.frombuffer(rom, dtype=np.uint8).copy()
    st = np.frombuffer(state, dtype=np.uint8).copy() if state is not None else None
    ic = ctypes.c_uint64()
    sec = lib().gb_bench(_ptr(r), len(r), _ptr(st) if st is not None else None,
                         len(st) if st is not None else 0, n, warmup, steps, seed, ctypes.byref(ic))
    if sec < 0:
        raise ValueError("gb_bench failed")
    return sec, int(ic.value)


# ---------------------------------------------------------------------------------------------
# Whole-batch parity helpers (tests only).  States are compared as 64-bit xxh3 digests of the v9
# bytes so that 65,536-env batches fit in memory; `headless` leaves out the per-line scroll
# parameters and the screen, which a render=False device run does not produce (the oracle always
# renders the last frame, as pyboy_binding.py:86-87 does).
V9_SCAN, V9_WRAM = 8405, 101285


def state_digests(states: np.ndarray, headless: bool = False) -> np.ndarray:
    import xxhash
    out = np.zeros(len(states), np.uint64)
    for i, s in enumerate(states):
        if headless:
            h = xxhash.xxh3_64(s[:V9_SCAN].tobytes())
            h.update(s[V9_WRAM:].tobytes())
            out[i] = h.intdigest()
        else:
            out[i] = xxhash.xxh3_64_intdigest(s.tobytes())
    return out


def batch_digests(rom: bytes, state, actions: np.ndarray, headless: bool = False, chunk: int = 256) -> np.ndarray:
    """Digests of every env's v9 state after running actions (steps, n) from the template."""
    steps, n = actions.shape
    out = np.zeros(n, np.uint64)
    for e0 in range(0, n, chunk):
        st, _ = batch_run(rom, state, actions[:, e0:e0 + chunk], want_screens=False)
        out[e0:e0 + chunk] = state_digests(st, headless)
    return out


def trajectory(rom: bytes, state, actions: np.ndarray, every: int, keep_every: int):
    """Run each env of actions (steps, n) from the template; returns (digests (steps//every, n),
    {(k, env): v9 bytes} at every keep_every steps) — checkpoints for long-horizon parity."""
    import xxhash
    steps, n = actions.shape
    dig = np.zeros((steps // every, n), np.uint64)
    keep = {}
    for e in range(n):
        gb = GB(rom, state)
        if state is None:
            gb.power_on()
        for t in range(steps):
            gb.run_action(int(actions[t, e]))
            if (t + 1) % every == 0:
                s = gb.save_state()
                dig[(t + 1) // every - 1, e] = xxhash.xxh3_64_intdigest(s)
                if (t + 1) % keep_every == 0:
                    keep[((t + 1) // keep_every, e)] = s
    return dig, keep
