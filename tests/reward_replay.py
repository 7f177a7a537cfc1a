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


# ---------------------------------------------------------------------------------------------
# the golden sequences at width: many envs of one handle (GPU: tests/test_gpu_reward.py at 4,096
# envs; host simulation: tests/test_hostsim_reward.py)
def _rows_by_event(g, rows):
    """{("reset"|"step", t): golden row} of one sequence (a reset after a done step has that step's t)."""
    return {("reset" if int(g["kind"][r]) == 0 else "step", int(g["t"][r])): int(r) for r in rows}


def run_replay_batched(make_emu, n: int, base_state: bytes) -> dict:
    """Replay every golden sequence as envs of batched handles and compare with the reference.

    One handle per max_episode_steps value (20480, 17, 12, 13: the episode length is a handle
    parameter), `n` envs each, env e playing sequence e % S — neighbouring lanes of a wave hold
    different sequences.  make_emu(template_state, n, max_steps) builds a BatchedEmulator-shaped
    handle with frame_skip 0 (the reward stack and the obs only).  Every tick every env installs its
    sequence's WRAM/HRAM/screen (set_ram / screen), the handle steps, and the envs whose golden step
    was done reset (masked reset).  Checked per env while its sequence is live: reward (exact f64),
    done, the PK_ERR code (the reference's exception), and — replicas equal on the device, one
    replica against the golden — obs sha1 and the RAM writes.  A sequence's first reset runs as a
    second reset without the template reload (a handle has one template): the golden one reloads
    the template, which is that sequence's own start image, so the only difference is the D778 flag
    write of get_base_event_flags (environment.py:1137-1138) that the reload overwrote.  The reset
    before it (the template's) raises KeyError before it touches any state that survives a reset,
    so every env reaches its first real reset as fresh as the reference's.  Returns the counts of
    checked events."""
    import torch
    from oracle.reward import ERR_MAP_KEY, ERR_NAMES

    g, seqs = sequences()
    groups = {}
    for sq in seqs:
        groups.setdefault(int(sq[1][2]), []).append(sq)
    checked = {"step": 0, "reset": 0, "err": 0}
    for max_steps, grp in sorted(groups.items()):
        S = len(grp)
        T = max(len(sq[5]) for sq in grp)
        ev = [_rows_by_event(g, sq[6]) for sq in grp]

        def pad(a, k):
            return np.pad(a, ((0, k - len(a)),) + ((0, 0),) * (a.ndim - 1), mode="edge")

        # the handle's template: sequence 0's start image on a map the reference's MAP_ID_REF lacks
        # (248), so the template reset below raises KeyError inside update_seen_map_dict before it
        # can set anything that survives a reset (stuck_cnt, :733-753) — every env leaves it as
        # fresh as the golden's envs are at their first reset, apart from reset_count
        w_t = grp[0][2][0].copy()
        w_t[0x135E] = 248
        emu = make_emu(template_state(base_state, w_t, grp[0][3][0], grp[0][4][0]), n, max_steps)
        dev = emu.device
        W = torch.from_numpy(np.stack([pad(sq[2], T + 1) for sq in grp])).to(dev)
        H = torch.from_numpy(np.stack([pad(sq[3], T + 1) for sq in grp])).to(dev)
        SC = torch.from_numpy(np.stack([pad(sq[4], T + 1) for sq in grp])).to(dev)
        A = torch.from_numpy(np.stack([np.pad(sq[5], (0, T - len(sq[5]))) for sq in grp]).astype(np.uint8)).to(dev)
        seq_of = torch.arange(n, device=dev) % S
        live = np.ones(S, bool)

        def install(t):
            ti = torch.full((n,), t, dtype=torch.int64, device=dev)
            w, h = W[seq_of, ti].contiguous(), H[seq_of, ti].contiguous()
            emu.set_ram(0xC000, w)
            emu.set_ram(0xFF80, h)
            emu.screen.copy_(SC[seq_of, ti])
            return w, h

        def per_seq(x):
            """rows of the first S envs, after asserting every replica equals its sequence's first."""
            x = x.reshape(n, -1)
            full = n - n % S
            v = x[:full].reshape(full // S, S, -1)
            assert bool((v == v[:1]).all()), "replicas of a sequence disagree"
            if full < n:
                assert torch.equal(x[full:], x[:n - full]), "replicas of a sequence disagree"
            return x[:S].cpu().numpy()

        def ram():
            return per_seq(emu.get_ram(0xC000, 8192)), per_seq(emu.get_ram(0xFF80, 127))

        def compare(kind, t, k, row, err, obs, w_got, h_got, w_base, h_base, extra=None):
            name = ERR_NAMES.get(int(err[k]), str(int(err[k]))) if int(err[k]) else ""
            assert name == str(g["err"][row]), (grp[k][0], kind, t, name, str(g["err"][row]))
            if name:
                checked["err"] += 1
                return False
            assert obs_hash(obs[k].reshape(72, 80, 4)) == str(g["obs_sha1"][row]), (grp[k][0], kind, t, "obs")
            got = {0xC000 + int(a): int(w_got[k][a]) for a in np.nonzero(w_got[k] != w_base[k])[0]}
            got.update({0xFF80 + int(a): int(h_got[k][a]) for a in np.nonzero(h_got[k] != h_base[k])[0]})
            a0, a1 = g["diff_ptr"][row], g["diff_ptr"][row + 1]
            exp = dict(zip(g["diff_addr"][a0:a1].tolist(), g["diff_val"][a0:a1].tolist()))
            if extra:
                exp.update(extra(k))
                exp = {a: v for a, v in exp.items() if v is not None}
            assert got == exp, (grp[k][0], kind, t, {hex(a): v for a, v in got.items()},
                                {hex(a): v for a, v in exp.items()})
            checked[kind] += 1
            return True

        # first reset: one clean template reset (the reload), then each env's own start image and a
        # reset that does not reload
        emu.reset()
        assert bool((emu.errors == ERR_MAP_KEY).all())
        w0, h0 = install(0)
        w0h, h0h = per_seq(w0), per_seq(h0)
        emu.reset()
        err, obs = per_seq(emu.errors)[:, 0], per_seq(emu.obs)
        wg, hg = ram()

        def d778(k):   # the flag write the golden first reset's reload overwrote
            v = int(w0h[k][0x1778]) | 0x10
            return {0xD778: v if v != int(w0h[k][0x1778]) else None}

        for k in range(S):
            live[k] = compare("reset", 0, k, ev[k][("reset", 0)], err, obs, wg, hg, w0h, h0h, extra=d778)
        for t in range(1, T + 1):
            wi, hi = install(t)
            wih, hih = per_seq(wi), per_seq(hi)
            _, rew, term, _ = emu.step(A[seq_of, t - 1].contiguous())
            err, rw, dn, obs = per_seq(emu.errors)[:, 0], per_seq(rew)[:, 0], per_seq(term)[:, 0], per_seq(emu.obs)
            wg, hg = ram()
            reset_mask = np.zeros(S, np.uint8)
            for k in range(S):
                if not live[k] or ("step", t) not in ev[k]:
                    live[k] = False
                    continue
                row = ev[k][("step", t)]
                if not compare("step", t, k, row, err, obs, wg, hg, wih, hih):
                    live[k] = False
                    continue
                assert rw[k] == float(g["reward"][row]), (grp[k][0], t, rw[k], float(g["reward"][row]))
                assert int(dn[k]) == int(g["done"][row]), (grp[k][0], t)
                reset_mask[k] = int(dn[k])
            if reset_mask.any():
                emu.reset(torch.from_numpy(reset_mask).to(dev)[seq_of].contiguous())
                err, obs = per_seq(emu.errors)[:, 0], per_seq(emu.obs)
                wr, hr = ram()
                for k in np.nonzero(reset_mask)[0]:
                    live[k] = compare("reset", t, k, ev[k][("reset", t)], err, obs, wr, hr, wg, hg)
        emu.close()
    return checked
