"""The reward-stack oracle (oracle/reward.py) against the reference's own outputs.

tests/golden/reward_replay.npz was recorded by running the reference Environment
(environment.py:1233-1612, imported in the build container) on the image sequences of
tests/golden/replay_gen.py.  Checked per event: reward (bit-exact f64), done, the (72,80,4)
observation (sha1), the RAM bytes written (CC30/CC31/CF7C-CF85, victory-road bits, CD4D, D778),
and the step at which the reference raised (and which exception)."""
import numpy as np
import pytest

from oracle import reward as R
from reward_replay import install, obs_hash, sequences


@pytest.fixture(scope="module")
def replay():
    return sequences()


def test_battle_state_table_shapes():
    from pokegym_amd import reward_tables as T
    assert T.GS_UNKNOWN == 115 and T.SV_UNKNOWN == 115 and T.MV_UNKNOWN == 20
    assert sum(len(v) for v in T.MONITORS.values()) == 130


def test_oracle_matches_reference_replay(replay):
    g, seqs = replay
    n_checked = 0
    for si, (seed, steps, max_steps, allow_err), W, H, S, A, rows in seqs:
        mem = np.zeros(0x10000, np.uint8)
        bus = R.Bus(mem)
        st = R.EnvState()
        install(mem, W[0], H[0])
        t = 0
        for row in rows:
            kind, gt = int(g["kind"][row]), int(g["t"][row])
            err = str(g["err"][row])
            if kind == 0:
                if st.reset_count == 0:
                    install(mem, W[0], H[0])
                before = mem.copy()
                o = R.reset(st, bus, S[t], reload=(lambda: install(mem, W[0], H[0])) if st.reset_count == 0 else None,
                            max_episode_steps=max_steps)
                if err:
                    assert st.err and R.ERR_NAMES[st.err] == err, (si, gt, err, st.err)
                    break
                assert not st.err, (si, gt, st.err)
                assert obs_hash(o) == str(g["obs_sha1"][row]), (si, "reset", gt)
            else:
                t = gt
                install(mem, W[t], H[t])
                before = mem.copy()
                o, r, done = R.step(st, bus, int(A[t - 1]), S[t])
                if err:
                    assert st.err and R.ERR_NAMES[st.err] == err, (si, t, err, st.err)
                    break
                assert not st.err, (si, t, st.err)
                assert r == float(g["reward"][row]), (si, t, r, float(g["reward"][row]))
                assert int(done) == int(g["done"][row]), (si, t)
                assert obs_hash(o) == str(g["obs_sha1"][row]), (si, "step", t)
            # RAM after the event differs from the image exactly where the reference's did
            a0, a1 = g["diff_ptr"][row], g["diff_ptr"][row + 1]
            exp = dict(zip(g["diff_addr"][a0:a1].tolist(), g["diff_val"][a0:a1].tolist()))
            got = {int(a): int(mem[a]) for a in np.nonzero(mem != before)[0] if 0xC000 <= a < 0xE000 or 0xFF80 <= a < 0xFFFF}
            assert got == exp, (si, gt, {hex(a): v for a, v in got.items()}, {hex(a): v for a, v in exp.items()})
            n_checked += 1
    assert n_checked > 1500
