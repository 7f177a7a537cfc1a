"""Record the REFERENCE Environment's `info` telemetry at episode ends -> tests/golden/info_stats.npz.

Run in the build container only:  python3 -B tools/make_golden_info.py
Drives the reference Environment (tools/ref_env.py) over replayed RAM images
(tests/golden/replay_gen.py) with short episodes, so `done` — and with it the info dict of
environment.py:1621-1810 — comes up several times per sequence.  Records the scalar entries of
info["stats"] and info["reward"] listed in STATS_FIELDS / REWARD_FIELDS (float64), per done step.
"""
from __future__ import annotations

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
from pokegym_amd import reward_tables as T  # noqa: E402
from pokegym_amd.info import REWARD_FIELDS, STATS_FIELDS, reference_value  # noqa: E402

# the reference info dict's event-monitor entries, in the order of reward_tables.MONITORS
EVENT_KEYS = ("dojo_events_aggregate", "silph_co_events_aggregate", "hideout_events_aggregate",
              "poke_tower_events_aggregate")
DETAIL_KEYS = ("detailed_rewards_dojo", "detailed_rewards_silph_co", "detailed_rewards_hideout",
               "detailed_rewards_poke_tower")

# (seed, steps, max_episode_steps, allow_errors, scenario)
SEQUENCES = [(500 + s, 24, 3 + (s % 6), 0, (0, 0, 1, 2, 3, 4)[s % 6]) for s in range(64)]


def main():
    bw, bh = replay_gen.load_bank()
    dims = dict(T.MAP_DIMS)
    seqs, ts, vals, errs = [], [], [], []
    heat_seq, heat_idx, heat_val = [], [], []   # each sequence's final counts_map (nonzero cells)
    ev_names, ev_vals, det_vals = None, [], []     # the nine *_events_aggregate / detailed_rewards_* dicts
    for si, (seed, steps, max_steps, allow_err, scen) in enumerate(SEQUENCES):
        W, H, S, A = replay_gen.make_sequence(bw, bh, seed, steps, dims, bool(allow_err), scen, T.MAP_COORD)
        env = ref_env.ReplayEnv(W[0], H[0], S[0])
        env.env.reset_default_max = max_steps
        try:
            env.env.reset(max_episode_steps=max_steps)
        except Exception:  # noqa: BLE001
            continue
        for t in range(1, steps + 1):
            try:
                _, _, done, _, info = env.step(A[t - 1], W[t], H[t], S[t])
            except Exception as ex:  # noqa: BLE001
                errs.append((si, t, type(ex).__name__, str(ex)[:60]))
                break
            if info:
                st, rw = info["stats"], info["reward"]
                row = [float(reference_value(st, k)) for k in STATS_FIELDS] + [float(rw[k]) for k in REWARD_FIELDS]
                seqs.append(si)
                ts.append(t)
                vals.append(row)
                agg = [info[k] for k in EVENT_KEYS[:4]] + [info["gym_events"][f"gym_{g}_events"] for g in range(3, 8)]
                det = [info[k] for k in DETAIL_KEYS[:4]] + [info["detailed_rewards_gyms"][f"gym_{g}_detailed_rewards"]
                                                            for g in range(3, 8)]
                names = [f"{i}:{n}" for i, d in enumerate(agg) for n in d]
                assert ev_names is None or names == ev_names
                ev_names = names
                ev_vals.append([float(v) for d in agg for v in d.values()])
                det_vals.append([float(v) for d in det for v in d.values()])
            if done:
                try:
                    env.env.reset(max_episode_steps=max_steps)
                except Exception:  # noqa: BLE001
                    break
        cm = np.asarray(env.env.counts_map, np.float64).reshape(-1)
        nz = np.nonzero(cm)[0]
        heat_seq += [si] * len(nz)
        heat_idx += nz.tolist()
        heat_val += cm[nz].tolist()
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "info_stats.npz"),
                        seqs=np.array(SEQUENCES, np.int64), seq=np.array(seqs, np.int32), t=np.array(ts, np.int32),
                        values=np.array(vals, np.float64), fields=np.array(list(STATS_FIELDS) + list(REWARD_FIELDS)),
                        heat_seq=np.array(heat_seq, np.int32), heat_idx=np.array(heat_idx, np.int32),
                        heat_val=np.array(heat_val, np.float64), event_names=np.array(ev_names),
                        event_values=np.array(ev_vals, np.float64), detail_values=np.array(det_vals, np.float64))
    print(f"{len(vals)} info records over {len(SEQUENCES)} sequences; step errors: {errs}")


if __name__ == "__main__":
    main()
