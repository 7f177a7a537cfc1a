"""Record the REFERENCE reward stack's outputs on replayed RAM images -> tests/golden/.

Run in the build container only:  python3 -B tools/make_golden_reward.py
Writes
  tests/golden/wram_bank.npz      WRAM (C000-DFFF) and HRAM (FF80-FFFE) of the reference's 264 v9
                                  savestates (data files of the reference; no source)
  tests/golden/reward_replay.npz  per event (reset / step) of every sequence: reward (f64), done,
                                  error name, sha1 of the (72,80,4) obs, and the RAM bytes the
                                  reference wrote (addr, value)
The reference Environment (environment.py) is imported with tools/ref_env.py; its emulator is
replaced by the images of tests/golden/replay_gen.py (each step's image fully replaces WRAM,
echo RAM and HRAM, as if run_action_on_emulator had produced it).
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)

import ref_env  # noqa: E402
import replay_gen  # noqa: E402
from make_golden_ppu import corpus  # noqa: E402
from pokegym_amd import reward_tables as T  # noqa: E402

# (seed, steps, max_episode_steps, allow_errors, scenario)
SEQUENCES = ([(s, 60, 20480, 0, 0) for s in range(40)]
             + [(100 + s, 50, 17, 0, 0) for s in range(8)]
             + [(200 + s, 60, 20480, 1, 0) for s in range(16)]
             + [(300 + s, 20, 20480, 0, sc) for s in range(2) for sc in (1, 2, 3, 4)]
             + [(400 + s, 20, 12 + s, 0, 5) for s in range(2)])


def obs_hash(o):
    return hashlib.sha1(np.ascontiguousarray(o, np.uint8).tobytes()).hexdigest()


def main():
    st = corpus()
    wram = np.stack([np.frombuffer(d[101285:101285 + 8192], np.uint8) for _, d in st])
    hram = np.stack([np.frombuffer(d[109649:109649 + 127], np.uint8) for _, d in st])
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "wram_bank.npz"), wram=wram, hram=hram)

    dims = dict(T.MAP_DIMS)
    rows = []     # (seq, kind, t, reward, done, err, hash)
    diffs = []    # per row: list of (addr, value)
    for si, (seed, steps, max_steps, allow_err, scen) in enumerate(SEQUENCES):
        W, H, S, A = replay_gen.make_sequence(wram, hram, seed, steps, dims, bool(allow_err), scen, T.MAP_COORD)
        env = ref_env.ReplayEnv(W[0], H[0], S[0])
        env.env.reset_default_max = max_steps

        def ram_diff(base_w, base_h):
            m = env.game.mem
            d = [(0xC000 + int(a), int(m[0xC000 + a])) for a in np.nonzero(m[0xC000:0xE000] != base_w)[0]]
            d += [(0xFF80 + int(a), int(m[0xFF80 + a])) for a in np.nonzero(m[0xFF80:0xFFFF] != base_h)[0]]
            return d

        def do_reset(t):
            if env.env.reset_count == 0:
                bw, bh = W[0], H[0]
            else:
                bw, bh = env.game.mem[0xC000:0xE000].copy(), env.game.mem[0xFF80:0xFFFF].copy()
            try:
                o, _ = env.env.reset(max_episode_steps=max_steps)
                rows.append((si, 0, t, 0.0, 0, "", obs_hash(o)))
            except Exception as e:  # noqa: BLE001
                rows.append((si, 0, t, 0.0, 0, type(e).__name__, ""))
                return False
            diffs.append(ram_diff(bw, bh))
            return True

        if not do_reset(0):
            diffs.append([])
            continue
        for t in range(1, steps + 1):
            try:
                o, r, te, tr, _ = env.step(A[t - 1], W[t], H[t], S[t])
            except Exception as e:  # noqa: BLE001
                rows.append((si, 1, t, 0.0, 0, type(e).__name__, ""))
                diffs.append([])
                break
            rows.append((si, 1, t, float(r), int(te), "", obs_hash(o)))
            diffs.append(ram_diff(W[t], H[t]))
            if te:
                if not do_reset(t):
                    diffs.append([])
                    break
    ptr = np.zeros(len(diffs) + 1, np.int64)
    for i, d in enumerate(diffs):
        ptr[i + 1] = ptr[i] + len(d)
    flat = [x for d in diffs for x in d]
    np.savez_compressed(
        os.path.join(REPO, "tests", "golden", "reward_replay.npz"),
        seqs=np.array(SEQUENCES, np.int64),
        seq=np.array([r[0] for r in rows], np.int32), kind=np.array([r[1] for r in rows], np.int8),
        t=np.array([r[2] for r in rows], np.int32), reward=np.array([r[3] for r in rows], np.float64),
        done=np.array([r[4] for r in rows], np.int8), err=np.array([r[5] for r in rows]),
        obs_sha1=np.array([r[6] for r in rows]),
        diff_ptr=ptr, diff_addr=np.array([a for a, _ in flat], np.int32), diff_val=np.array([v for _, v in flat], np.uint8))
    errs = [r for r in rows if r[5]]
    print(f"{len(rows)} events, {len(errs)} errors: {sorted(set(r[5] for r in errs))}; "
          f"nonzero rewards {sum(1 for r in rows if r[3] != 0)}; writes {len(flat)}")


if __name__ == "__main__":
    main()
