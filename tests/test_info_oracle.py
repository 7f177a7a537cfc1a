"""The info telemetry restatement (oracle/reward.py step -> st.info) against the reference's
own info dicts (tests/golden/info_stats.npz, tools/make_golden_info.py: every numeric scalar of
info["stats"] / info["reward"], environment.py:1621-1704, at each done step of short episodes)."""
import numpy as np

from oracle import reward as R
from pokegym_amd import info as I
from reward_replay import check_events, check_info, golden_heat, info_sequences, install


def test_info_fields_match_golden_layout():
    g, _ = info_sequences()
    assert [str(f) for f in g["fields"]] == list(I.STATS_FIELDS) + list(I.REWARD_FIELDS)
    assert I.NFIELDS == len(g["fields"]) and len(g["values"]) > 100


def test_oracle_info_matches_reference():
    g, seqs = info_sequences()
    got, events = {}, {}
    for si, max_steps, W, H, S, A in seqs:
        mem = np.zeros(0x10000, np.uint8)
        bus = R.Bus(mem)
        st = R.EnvState()
        install(mem, W[0], H[0])
        R.reset(st, bus, S[0], reload=lambda: install(mem, W[0], H[0]), max_episode_steps=max_steps)
        if st.err:
            continue
        for t in range(1, len(A) + 1):
            install(mem, W[t], H[t])
            _, _, done = R.step(st, bus, int(A[t - 1]), S[t])
            if st.err:
                break
            if st.info is not None:
                got[(si, t)] = st.info
                events[(si, t)] = st.info_events
            if done:
                R.reset(st, bus, S[t], max_episode_steps=max_steps)
                if st.err:
                    break
    assert check_info(g, got) > 100
    check_events(g, events)


def test_event_dicts_from_bits():
    """info.event_dicts rebuilds the reference's nested dicts from the monitor bits."""
    g, _ = info_sequences()
    for row in range(len(g["event_values"])):
        vals = g["event_values"][row].astype(int).tolist()
        bits = [0] * 5
        for i, v in enumerate(vals):
            bits[i >> 5] |= (1 if v != 0 else 0) << (i & 31)
        d = I.event_dicts(bits)
        flat = [v for k in ("dojo_events_aggregate", "silph_co_events_aggregate", "hideout_events_aggregate",
                            "poke_tower_events_aggregate") for v in d[k].values()]
        flat += [v for gk in range(3, 8) for v in d["gym_events"][f"gym_{gk}_events"].values()]
        assert flat == vals
        det = [v for k in ("detailed_rewards_dojo", "detailed_rewards_silph_co", "detailed_rewards_hideout",
                           "detailed_rewards_poke_tower") for v in d[k].values()]
        det += [v for gk in range(3, 8) for v in d["detailed_rewards_gyms"][f"gym_{gk}_detailed_rewards"].values()]
        assert det == g["detail_values"][row].tolist()


def test_info_dict_shape():
    rec = np.arange(I.NFIELDS, dtype=np.float64)
    d = I.info_dict(rec)
    assert d["stats"]["levels"] == [5, 6, 7, 8, 9, 10] and d["stats"]["step"] == 0
    assert d["reward"]["has_bicycle_in_bag_reward"] == float(I.NFIELDS - 1)
    assert isinstance(d["stats"]["badges"], float) and isinstance(d["stats"]["money"], int)


def test_oracle_heat_map_matches_reference():
    """counts_map (environment.py:648-679) after each sequence: +1 per step on the same map,
    -1 at the entry cell of a new map, persists across resets."""
    g, seqs = info_sequences()
    for si, max_steps, W, H, S, A in seqs:
        mem = np.zeros(0x10000, np.uint8)
        bus = R.Bus(mem)
        st = R.EnvState()
        install(mem, W[0], H[0])
        R.reset(st, bus, S[0], reload=lambda: install(mem, W[0], H[0]), max_episode_steps=max_steps)
        for t in range(1, len(A) + 1):
            if st.err:
                break
            install(mem, W[t], H[t])
            _, _, done = R.step(st, bus, int(A[t - 1]), S[t])
            if not st.err and done:
                R.reset(st, bus, S[t], max_episode_steps=max_steps)
        assert np.array_equal(st.heat.reshape(-1).astype(np.float64), golden_heat(g, si)), si
