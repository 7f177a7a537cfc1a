"""Shared driver: replay the golden reward sequences through an implementation and compare.

An implementation is driven per sequence with the protocol the golden fixtures were recorded
with (tools/make_golden_reward.py): before every step the sequence's image replaces WRAM, echo
RAM and HRAM; resets happen at t=0 and after a `done` step.
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import replay_gen  # noqa: E402

from pokegym_amd import reward_tables as T  # noqa: E402


def load_golden():
    d = np.load(os.path.join(HERE, "golden", "reward_replay.npz"))
    return {k: d[k] for k in d.files}


def sequences():
    """-> list of (seq_index, (seed, steps, max_steps, allow_err), W, H, S, A, golden rows)."""
    g = load_golden()
    bw, bh = replay_gen.load_bank()
    dims = dict(T.MAP_DIMS)
    out = []
    for si, (seed, steps, max_steps, allow_err, scen) in enumerate(g["seqs"].tolist()):
        W, H, S, A = replay_gen.make_sequence(bw, bh, seed, steps, dims, bool(allow_err), scen, T.MAP_COORD)
        rows = np.nonzero(g["seq"] == si)[0]
        out.append((si, (seed, steps, max_steps, allow_err), W, H, S, A, rows))
    return g, out


def install(mem, w, h):
    mem[0xC000:0xE000] = w
    mem[0xE000:0xFE00] = w[:0x1E00]
    mem[0xFF80:0xFFFF] = h


def obs_hash(o):
    return hashlib.sha1(np.ascontiguousarray(o, np.uint8).tobytes()).hexdigest()


def writes_of(g, row):
    a, b = g["diff_ptr"][row], g["diff_ptr"][row + 1]
    return list(zip(g["diff_addr"][a:b].tolist(), g["diff_val"][a:b].tolist()))


# ---------------------------------------------------------------------------------------------
# driving a C-ABI implementation (host-simulation build or the real HIP library)
STATE_WRAM, STATE_HRAM, STATE_SCREEN = 101285, 109649, 9125


def template_state(base_state: bytes, w, h, screen):
    """A v9 state = base_state with WRAM/HRAM/screen replaced (the reload source of pk_reset)."""
    s = np.frombuffer(base_state, np.uint8).copy()
    s[STATE_WRAM:STATE_WRAM + 8192] = w
    s[STATE_HRAM:STATE_HRAM + 127] = h
    px = s[STATE_SCREEN:STATE_SCREEN + 144 * 160 * 4].reshape(144 * 160, 4)
    g = screen.reshape(-1)
    px[:, 0] = (g == 0xFF)
    px[:, 1] = px[:, 2] = px[:, 3] = g
    return s.tobytes()


def run_replay(backend, base_state: bytes, g, seqs):
    """Replay every golden sequence through `backend` (one 1-env handle per sequence).
    Returns the number of events checked; raises AssertionError on the first mismatch."""
    from oracle.reward import ERR_NAMES
    n_checked = 0
    for si, (seed, steps, max_steps, allow_err), W, H, S, A, rows in seqs:
        h = backend.create(template_state(base_state, W[0], H[0], S[0]), int(max_steps))
        try:
            t = 0
            first = True
            for row in rows:
                kind, gt = int(g["kind"][row]), int(g["t"][row])
                err = str(g["err"][row])
                if kind == 0:
                    if first:
                        bw, bh = W[0], H[0]
                    else:
                        bw, bh = backend.get_ram(h)
                    first = False
                    backend.reset(h)
                    e = backend.error(h)
                    if err:
                        assert e and ERR_NAMES.get(e) == err, (si, "reset", gt, err, e)
                        break
                    assert e == 0, (si, "reset", gt, e)
                    assert obs_hash(backend.obs(h)) == str(g["obs_sha1"][row]), (si, "reset obs", gt)
                else:
                    t = gt
                    backend.set_ram(h, W[t], H[t])
                    backend.set_screen(h, S[t])
                    bw, bh = W[t], H[t]
                    r, d = backend.step(h, int(A[t - 1]))
                    e = backend.error(h)
                    if err:
                        assert e and ERR_NAMES.get(e) == err, (si, t, err, e)
                        break
                    assert e == 0, (si, t, e)
                    assert r == float(g["reward"][row]), (si, t, r, float(g["reward"][row]))
                    assert int(d) == int(g["done"][row]), (si, t)
                    assert obs_hash(backend.obs(h)) == str(g["obs_sha1"][row]), (si, "step obs", t)
                w2, h2 = backend.get_ram(h)
                got = {0xC000 + int(a): int(w2[a]) for a in np.nonzero(w2 != bw)[0]}
                got.update({0xFF80 + int(a): int(h2[a]) for a in np.nonzero(h2 != bh)[0]})
                a0, a1 = g["diff_ptr"][row], g["diff_ptr"][row + 1]
                exp = dict(zip(g["diff_addr"][a0:a1].tolist(), g["diff_val"][a0:a1].tolist()))
                assert got == exp, (si, gt, {hex(a): v for a, v in got.items()}, {hex(a): v for a, v in exp.items()})
                n_checked += 1
        finally:
            backend.destroy(h)
    return n_checked


# ---------------------------------------------------------------------------------------------
# info telemetry (tests/golden/info_stats.npz, tools/make_golden_info.py): short episodes, the
# record of every step whose info dict was non-empty (done or time % 10000 == 0)
def info_sequences():
    """-> (golden dict, list of (seq_index, max_steps, W, H, S, A))."""
    d = np.load(os.path.join(HERE, "golden", "info_stats.npz"))
    g = {k: d[k] for k in d.files}
    bw, bh = replay_gen.load_bank()
    dims = dict(T.MAP_DIMS)
    out = []
    for si, (seed, steps, max_steps, allow_err, scen) in enumerate(g["seqs"].tolist()):
        W, H, S, A = replay_gen.make_sequence(bw, bh, seed, steps, dims, bool(allow_err), scen, T.MAP_COORD)
        out.append((si, int(max_steps), W, H, S, A))
    return g, out


def check_info(g, got):
    """got: {(seq, t): record} -> asserts it equals the golden records (same steps, same values)."""
    exp = {(int(s), int(t)): v for s, t, v in zip(g["seq"], g["t"], g["values"])}
    assert sorted(got) == sorted(exp), (sorted(set(got) ^ set(exp))[:8])
    fields = [str(f) for f in g["fields"]]
    for k, v in exp.items():
        bad = [(fields[i], float(got[k][i]), float(v[i])) for i in range(len(v)) if float(got[k][i]) != float(v[i])]
        assert not bad, (k, bad[:6])
    return len(exp)


def golden_heat(g, si):
    """The reference's final counts_map of info sequence si (444*436 flat, float64)."""
    m = np.zeros(444 * 436, np.float64)
    k = g["heat_seq"] == si
    m[g["heat_idx"][k]] = g["heat_val"][k]
    return m


def check_events(g, got):
    """got: {(seq, t): 130 monitor values (weight * bit)} -> equals the reference's aggregates."""
    exp = {(int(s), int(t)): v for s, t, v in zip(g["seq"], g["t"], g["event_values"])}
    assert sorted(got) == sorted(exp)
    for k, v in exp.items():
        assert [float(x) for x in got[k]] == v.tolist(), k


class _Records(dict):
    """{(seq, t): info record}; .events = {(seq, t): monitor values}."""

    def __init__(self):
        super().__init__()
        self.events = {}


def run_info_replay(backend, base_state: bytes):
    """The info records `backend` emits over the info golden sequences (1-env handle per sequence;
    a sequence ends at its first error, as the reference raised there).  Also checks each
    sequence's final counts_map against the reference's when the backend keeps one."""
    g, seqs = info_sequences()
    got = _Records()
    for si, max_steps, W, H, S, A in seqs:
        h = backend.create(template_state(base_state, W[0], H[0], S[0]), max_steps)
        try:
            backend.reset(h)
            if backend.error(h):
                continue
            for t in range(1, len(A) + 1):
                backend.set_ram(h, W[t], H[t])
                backend.set_screen(h, S[t])
                _, d = backend.step(h, int(A[t - 1]))
                if backend.error(h):
                    break
                rec = backend.info(h)
                if rec is not None:
                    got[(si, t)] = np.asarray(rec, np.float64)
                    got.events[(si, t)] = backend.events(h)
                if d:
                    backend.reset(h)
                    if backend.error(h):
                        break
            if hasattr(backend, "heat"):
                assert np.array_equal(backend.heat(h), golden_heat(g, si)), ("counts_map", si)
        finally:
            backend.destroy(h)
    return g, got
