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
