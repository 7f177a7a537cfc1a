"""Deterministic WRAM/HRAM image sequences for reward-stack parity (no reference code inside).

Shared by tools/make_golden_reward.py (which feeds them to the imported reference Environment to
record tests/golden/reward_replay.npz) and by the parity tests (which feed the same sequences to
the oracle and to the HIP reward kernel).  A sequence starts from one of the 264 savestate WRAM
images (tests/golden/wram_bank.npz) and mutates the bytes the reward stack reads, step by step,
so that every branch of environment.py:1338-1612 is exercised: map changes (incl. the
victory-road maps and the tree maps), party levels/HP (healing, death), badges, event flags,
bag items, party/box moves (HM01 Cut), the cut-tile sequences, menu bytes, CD4D==61 and the
process_game_states battle/menu bytes.
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
W0 = 0xC000


def load_bank():
    d = np.load(os.path.join(HERE, "wram_bank.npz"))
    return d["wram"], d["hram"]


GREY = np.array([0xFF, 0x99, 0x55, 0x00], np.uint8)
CUT_ROWS = [(0x3D, 1, 1, 0, 4, 1), (0x3D, 1, 1, 0, 1, 1), (0x50, 1, 1, 0, 4, 1), (0x50, 1, 1, 0, 1, 1),
            (0x52, 255, 1, 0, 1, 1), (0x52, 1, 1, 0, 1, 1), (0x11, 255, 0, 0, 4, 1), (0x22, 255, 0, 0, 1, 1)]
CUT_ADDRS = (0xCFC6, 0xCFCB, 0xCD6A, 0xD367, 0xD125, 0xCD3D)
TREE_MAPS = [6, 134, 13, 1, 5, 36, 20, 21]
VR_MAPS = [0x6C, 0xC2, 0xC6, 0x22]
MENU_KEYS = [(0x00, 0x00), (0xd3, 0xc3), (0xfB, 0xc3), (0xC1, 0xC4), (0xA9, 0xC4), (0x41, 0xC4), (0x9A, 0xC4),
             (0xC2, 0xC4), (0x4C, 0xC4), (0xB5, 0xC3)]


def _set(w, a, v):
    w[a - W0] = v & 0xFF


def _get(w, a):
    return int(w[a - W0])


def mutate(w, h, rng, dims, allow_errors):
    """One step of mutations of the WRAM image w (8192) and HRAM image h (127), in place."""
    u = rng.random
    # --- position / map
    m = _get(w, 0xD35E)
    if u() < 0.06:
        pool = TREE_MAPS + VR_MAPS + [0, 1, 12, 13, 40, 51, 59, 0xF5, 0x71, int(rng.integers(0, 248))]
        m = int(pool[rng.integers(len(pool))])
        _set(w, 0xD35E, m)
        if m in dims:
            hh, ww = dims[m]
            _set(w, 0xD361, int(rng.integers(0, max(hh, 1))))
            _set(w, 0xD362, int(rng.integers(0, max(ww, 1))))
    if u() < 0.6:
        hh, ww = dims.get(m, (1, 1))
        y = _get(w, 0xD361) + int(rng.integers(-1, 2))
        x = _get(w, 0xD362) + int(rng.integers(-1, 2))
        _set(w, 0xD361, min(max(y, 0), max(hh - 1, 0)))
        _set(w, 0xD362, min(max(x, 0), max(ww - 1, 0)))
    if allow_errors and u() < 0.01:
        _set(w, 0xD361, 250)
    # --- party
    if u() < 0.05:
        k = int(rng.integers(6))
        _set(w, 0xD18C + 44 * k, int(rng.integers(0, 100)))
    if u() < 0.02:
        _set(w, 0xD163, int(rng.integers(0, 7)))
    if u() < 0.15:
        k = int(rng.integers(6))
        mx = int(rng.integers(0, 300))
        hp = int(rng.integers(0, mx + 1)) if u() < 0.8 else 0
        _set(w, 0xD18D + 44 * k, mx >> 8)
        _set(w, 0xD18E + 44 * k, mx)
        _set(w, 0xD16C + 44 * k, hp >> 8)
        _set(w, 0xD16D + 44 * k, hp)
    if u() < 0.03:
        for k in range(6):
            _set(w, 0xD16C + 44 * k, 0)
            _set(w, 0xD16D + 44 * k, 0)
    if u() < 0.02:
        for k in range(6):
            _set(w, 0xD18D + 44 * k, 0)
            _set(w, 0xD18E + 44 * k, 0)
    if u() < 0.05:
        k = int(rng.integers(6))
        _set(w, 0xD8C5 + 44 * k, int(rng.integers(0, 80)))
    # --- badges / events / pokedex
    if u() < 0.03:
        _set(w, 0xD356, _get(w, 0xD356) | (1 << int(rng.integers(8))))
    if u() < 0.2:
        for _ in range(int(rng.integers(1, 6))):
            a = int(rng.integers(0xD747, 0xD886))
            _set(w, a, _get(w, a) ^ (1 << int(rng.integers(8))))
    if u() < 0.1:
        a = int(rng.choice([0xD7B1, 0xD825, 0xD826, 0xD815, 0xD81B, 0xD765, 0xD768, 0xD773, 0xD77C, 0xD792,
                            0xD7B3, 0xD7F1, 0xD7F2, 0xD803, 0xD754, 0xD77E, 0xD838, 0xD7B9]))
        _set(w, a, int(rng.integers(0, 256)))
    if u() < 0.05:
        a = int(rng.integers(0xD2F7, 0xD31D))
        _set(w, a, int(rng.integers(0, 256)))
    # --- bag items
    if u() < 0.06:
        i = int(rng.integers(20))
        pool = [0xC4, 0xC5, 0xC6, 0xC7, 0xC8, 0x3E, 0x48, 0x4A, 0x33, 0x06, 0x04, 0xFF, 0x00, int(rng.integers(256))]
        _set(w, 0xD31E + 2 * i, int(pool[rng.integers(len(pool))]))
    # --- moves (party + box)
    if u() < 0.05:
        k = int(rng.integers(6))
        _set(w, 0xD16B + 44 * k, int(rng.integers(0, 3)) * 0x55)
        mv = 15 if u() < 0.3 else int(rng.integers(0, 0xA5 if not allow_errors or u() < 0.9 else 256))
        _set(w, 0xD173 + 44 * k + int(rng.integers(4)), mv)
    if u() < 0.03:
        _set(w, 0xDA80, int(rng.integers(0, 45 if not allow_errors or u() < 0.8 else 60)))
        for i in range(3):
            off = 0xDA96 + 200 * int(rng.integers(0, 7))
            _set(w, off, int(rng.integers(0, 2)) * 0x20)
            _set(w, off + 8 + i, int(rng.integers(0, 0xA5)))
    # --- cut machinery
    if u() < 0.35:
        row = CUT_ROWS[rng.integers(len(CUT_ROWS))]
        for a, v in zip(CUT_ADDRS, row):
            _set(w, a, v)
    if u() < 0.1:
        _set(w, 0xC109, int(rng.choice([0, 4, 8, 0xC] + ([2] if allow_errors else []))))
    if u() < 0.05:
        _set(w, 0xCD4D, 61 if u() < 0.6 else int(rng.integers(256)))
    if u() < 0.1:
        _set(w, 0xD057, int(rng.choice([0, 0, 0, 1, 2, 255])))
    if u() < 0.05:
        _set(w, 0xD059, int(rng.choice([0, 0, 1, 200])))
    if u() < 0.2:
        _set(w, 0xCFC4, int(rng.choice([0, 0, 1])))
    if u() < 0.05:
        _set(w, 0xCD38, int(rng.choice([0, 0, 0, 1])))
    if u() < 0.15:
        key = MENU_KEYS[rng.integers(len(MENU_KEYS))]
        _set(w, 0xCC30, key[0])
        _set(w, 0xCC31, key[1])
    if u() < 0.1:
        a = int(rng.choice([0xCF13, 0xCF94, 0xD31D, 0xCC36, 0xCC26, 0xCC3A, 0xD125, 0xD730, 0xCC52, 0xC48F, 0xD778]))
        _set(w, a, int(rng.choice([0, 1, 2, 3, 6, 0x40, 0x7E, 0xED, 0xF0, int(rng.integers(256))])))
    if u() < 0.1:
        h[0xFF8C - 0xFF80] = int(rng.choice([6, 6, 0, 1]))
    if u() < 0.1:
        _set(w, 0xD803, _get(w, 0xD803) | 1)


SC_NONE, SC_KEYERROR, SC_STUCK, SC_CUTCOORDS, SC_HEATMAP, SC_EMPTYPARTY = 0, 1, 2, 3, 4, 5


def _scenario(w, t, k, scenario, coords):
    """Targeted mutations that drive the reference into each of its exception paths."""
    if scenario == SC_KEYERROR and t == k:
        _set(w, 0xD35E, 250)                       # MAP_ID_REF has no 248..254
    elif scenario == SC_STUCK and t == 0:
        _set(w, 0xD361, 250)                       # first-ever bounds check fails
    elif scenario == SC_CUTCOORDS:
        if t == 1:                                 # teach Cut: self.cut = 1 after this step
            _set(w, 0xD16B, 0x99)
            _set(w, 0xD173, 15)
            _set(w, 0xD057, 0)
        if t >= 2:
            _set(w, 0xC109, 2)                     # facing not in {0, 4, 8, 0xC}
            _set(w, 0xD057, 0)
            if k <= t < k + 3:
                row = [(0x52, 255, 1, 0, 1, 1), (0x52, 255, 1, 0, 1, 1), (0x52, 1, 1, 0, 1, 1)][t - k]
                for a, v in zip(CUT_ADDRS, row):
                    _set(w, a, v)
    elif scenario == SC_EMPTYPARTY and t >= k:
        for j in range(6):                         # every party level 0 from step k on: the info
            _set(w, 0xD18C + 44 * j, 0)            # dict of the next done step takes max([])
    elif scenario == SC_HEATMAP and t == k:
        m = max((m for m in coords if m <= 247), key=lambda m: coords[m][1])
        _set(w, 0xD35E, m)
        _set(w, 0xD361, 255)


def make_sequence(bank_w, bank_h, seed, steps, dims, allow_errors=False, scenario=SC_NONE, coords=None):
    """-> (wram[steps+1, 8192], hram[steps+1, 127], screens[steps+1, 144, 160], actions[steps])."""
    rng = np.random.default_rng(seed)
    b = int(rng.integers(len(bank_w)))
    w = bank_w[b].copy()
    h = bank_h[b].copy()
    m = _get(w, 0xD35E)
    if m in dims:  # start in bounds
        hh, ww = dims[m]
        _set(w, 0xD361, min(_get(w, 0xD361), max(hh - 1, 0)))
        _set(w, 0xD362, min(_get(w, 0xD362), max(ww - 1, 0)))
    W = np.zeros((steps + 1, 8192), np.uint8)
    H = np.zeros((steps + 1, 127), np.uint8)
    S = np.zeros((steps + 1, 144, 160), np.uint8)
    k = steps // 2
    _scenario(w, 0, k, scenario, coords)
    W[0], H[0] = w, h
    S[0] = GREY[rng.integers(0, 4, (144, 160))]
    for t in range(1, steps + 1):
        mutate(w, h, rng, dims, allow_errors)
        _scenario(w, t, k, scenario, coords)
        W[t], H[t] = w, h
        S[t] = GREY[rng.integers(0, 4, (144, 160))]
    actions = rng.integers(0, 8, steps).astype(np.uint8)
    return W, H, S, actions
