"""Process pool for oracle runs beside a GPU test (TEST INFRASTRUCTURE ONLY).

Workers are started with the "spawn" method (a fresh interpreter per worker, never a fork of a
process that holds the GPU) and only load the CPU oracle.  Worker count follows the host share:
at most 16 (the GPU box's CPU share; os.cpu_count() there shows the whole machine)."""
from __future__ import annotations

import multiprocessing as mp
import os
from concurrent.futures import ProcessPoolExecutor

import numpy as np


def workers() -> int:
    return max(1, min(16, os.cpu_count() or 1, int(os.environ.get("PK_ORACLE_PROCS", "16"))))


def pool() -> ProcessPoolExecutor:
    return ProcessPoolExecutor(max_workers=workers(), mp_context=mp.get_context("spawn"))


def _digests(rom, state, actions, headless):
    from oracle import oracle
    return oracle.batch_digests(rom, state, actions, headless)


def _trajectory(rom, state, actions, every, keep_every):
    from oracle import oracle
    return oracle.trajectory(rom, state, actions, every, keep_every)


def batch_digests(ex: ProcessPoolExecutor, rom: bytes, state, actions: np.ndarray, headless=False, chunk=512):
    """Future-like list of (e0, future) covering all envs of actions (steps, n)."""
    n = actions.shape[1]
    return [(e0, ex.submit(_digests, rom, state, np.ascontiguousarray(actions[:, e0:e0 + chunk]), headless))
            for e0 in range(0, n, chunk)]


def gather_digests(futs, n: int) -> np.ndarray:
    out = np.zeros(n, np.uint64)
    for e0, f in futs:
        d = f.result()
        out[e0:e0 + len(d)] = d
    return out


def trajectories(ex: ProcessPoolExecutor, rom: bytes, state, actions: np.ndarray, every: int, keep_every: int, chunk=4):
    """(digests (steps//every, n), {(k, env): v9}) over worker chunks of `chunk` envs."""
    steps, n = actions.shape
    futs = [(e0, ex.submit(_trajectory, rom, state, np.ascontiguousarray(actions[:, e0:e0 + chunk]), every, keep_every))
            for e0 in range(0, n, chunk)]
    dig = np.zeros((steps // every, n), np.uint64)
    keep = {}
    for e0, f in futs:
        d, k = f.result()
        dig[:, e0:e0 + d.shape[1]] = d
        keep.update({(kk, e0 + e): v for (kk, e), v in k.items()})
    return dig, keep


def _reward_run(rom, state, actions, max_steps):
    """Full step (oracle emulator + oracle/reward.py) with a template reload on every reset
    (PK_F_RELOAD_ON_RESET) for actions (steps, m): rewards, dones, errors and digests of the
    (72,80,4) obs and of WRAM after each step (reset obs first)."""
    import xxhash

    from oracle import oracle as O
    from oracle import reward as R
    grey = np.array([0xFF, 0x99, 0x55, 0x00], np.uint8)
    steps, m = actions.shape
    rew = np.zeros((steps, m), np.float64)
    done = np.zeros((steps, m), np.uint8)
    err = np.zeros((steps, m), np.uint32)
    obs_d = np.zeros((steps + 1, m), np.uint64)
    wram_d = np.zeros((steps, m), np.uint64)

    class Bus:
        def __init__(self, gb):
            self.gb = gb

        def r(self, a):
            if a > 0xFFFF:
                raise IndexError(a)
            return self.gb.read(a)

        def w(self, a, v):
            self.gb.write(a, v & 0xFF)

    for e in range(m):
        gb = O.GB(rom, state)
        if state is None:
            gb.power_on()
        bus, st = Bus(gb), R.EnvState()
        reload = (lambda gb=gb: gb.load_state(state)) if state is not None else (lambda gb=gb: gb.power_on())
        scr = (lambda gb=gb: grey[gb.screen()])
        o = R.reset(st, bus, scr, reload=reload, max_episode_steps=max_steps, reload_always=True)
        obs_d[0, e] = xxhash.xxh3_64_intdigest(np.ascontiguousarray(o).tobytes())
        for t in range(steps):
            gb.run_action(int(actions[t, e]))
            o, r, d = R.step(st, bus, int(actions[t, e]), grey[gb.screen()])
            err[t, e] = st.err
            if st.err:
                break
            rew[t, e], done[t, e] = r, d
            wram_d[t, e] = xxhash.xxh3_64_intdigest(gb.wram().tobytes())
            if d:
                o = R.reset(st, bus, scr, reload=reload, max_episode_steps=max_steps, reload_always=True)
            obs_d[t + 1, e] = xxhash.xxh3_64_intdigest(np.ascontiguousarray(o).tobytes())
    return rew, done, err, obs_d, wram_d


def _reset_flow(rom, state, actions, max_steps, check_at):
    """The configs[3] VecEnv flow without the reward stack (reward=False): every env runs its actions
    (steps, m) from the template, `time` counts env-steps and an env whose time reaches max_steps is
    reset to the template after that step (done = time >= max_episode_steps, environment.py:1612-1613;
    the auto-reset of VecEnv: the template reload every reset does when PK_F_REWARD is off).  Returns
    (v9 digests after each step t in check_at (len(check_at), m), dones (steps, m))."""
    import xxhash

    from oracle import oracle as O
    steps, m = actions.shape
    dig = np.zeros((len(check_at), m), np.uint64)
    done = np.zeros((steps, m), np.uint8)
    at = {t: k for k, t in enumerate(check_at)}
    base = O.GB(rom, state)
    if state is None:
        base.power_on()
    for e in range(m):
        gb, time = base.clone(), 0
        for t in range(steps):
            gb.run_action(int(actions[t, e]))
            time += 1
            if time >= max_steps:
                done[t, e] = 1
                gb, time = base.clone(), 0
            if t in at:
                dig[at[t], e] = xxhash.xxh3_64_intdigest(gb.save_state())
    return dig, done


def reset_flows(ex: ProcessPoolExecutor, rom: bytes, state, actions: np.ndarray, max_steps: int, check_at, chunk=512):
    """(digests (len(check_at), n), dones (steps, n)) of _reset_flow over worker chunks."""
    steps, n = actions.shape
    futs = [(e0, ex.submit(_reset_flow, rom, state, np.ascontiguousarray(actions[:, e0:e0 + chunk]), max_steps,
                           list(check_at))) for e0 in range(0, n, chunk)]
    return futs


def gather_reset_flows(futs, n_check: int, steps: int, n: int):
    dig = np.zeros((n_check, n), np.uint64)
    done = np.zeros((steps, n), np.uint8)
    for e0, f in futs:
        d, dn = f.result()
        dig[:, e0:e0 + d.shape[1]] = d
        done[:, e0:e0 + dn.shape[1]] = dn
    return dig, done


def reward_runs_async(ex: ProcessPoolExecutor, rom: bytes, state, actions: np.ndarray, max_steps: int, chunk=256):
    n = actions.shape[1]
    return [(e0, ex.submit(_reward_run, rom, state, np.ascontiguousarray(actions[:, e0:e0 + chunk]), max_steps))
            for e0 in range(0, n, chunk)]


def gather_reward_runs(futs, steps: int, n: int):
    """(rewards, dones, errors, obs digests, WRAM digests) of reward_runs_async over all envs."""
    out = [np.zeros((steps, n), np.float64), np.zeros((steps, n), np.uint8), np.zeros((steps, n), np.uint32),
           np.zeros((steps + 1, n), np.uint64), np.zeros((steps, n), np.uint64)]
    for e0, f in futs:
        for a, r in zip(out, f.result()):
            a[:, e0:e0 + r.shape[1]] = r
    return out


def instr_counts(rom, acts):
    """Per env-step instructions the oracle executes (summed over envs), one gb per env."""
    import ctypes
    import numpy as np
    from oracle import oracle
    L = oracle.lib()
    r = np.frombuffer(rom, np.uint8).copy()
    gs = []
    for _ in range(acts.shape[1]):
        g = L.gb_new(r.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), len(r))
        L.gb_power_on(g)
        gs.append(g)
    out = []
    for t in range(acts.shape[0]):
        tot = 0
        for e, g in enumerate(gs):
            i0 = L.gb_instr_count(g)
            L.gb_run_action(g, int(acts[t, e]), 24, 8)
            tot += L.gb_instr_count(g) - i0
        out.append(tot)
    for g in gs:
        L.gb_free(g)
    return out
