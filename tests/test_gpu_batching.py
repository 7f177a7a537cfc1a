"""PufferLib-style sub-batches (VecEnv batch_size < num_envs; the reference trains 72 envs 24 at a
time, /root/reference/README.md:116-118) on the MI355X: stepping env ranges on their own streams
(pk_step_range / pk_reset_range) must be bit-identical to stepping the whole batch at once."""
import os

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STATE = os.path.join(REPO, "pokegym_amd", "states", "Bulbasaur.state")


def test_step_range_on_streams_matches_full_batch():
    """4 sub-batches of 64 envs stepped out of order on 4 streams == one 256-env launch (whole
    machine state as v9 digests, and the rendered screens)."""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    rom, n, steps, bs = game_rom(), 256, 6, 64
    acts = torch.from_numpy(np.random.default_rng(11).integers(0, 9, (steps, n), dtype=np.uint8)).cuda()
    full = BatchedEmulator(rom, n)
    sub = BatchedEmulator(rom, n)
    streams = [torch.cuda.Stream() for _ in range(n // bs)]
    order = [2, 0, 3, 1]
    for t in range(steps):
        full.step(acts[t])
        cur = torch.cuda.current_stream()
        for b in order:
            streams[b].wait_stream(cur)
            with torch.cuda.stream(streams[b]):
                sub.step_range(b * bs, acts[t, b * bs:(b + 1) * bs])
        for st in streams:
            cur.wait_stream(st)
    torch.cuda.synchronize()
    a = oracle.state_digests(full.snapshot_range(0, n))
    b = oracle.state_digests(sub.snapshot_range(0, n))
    assert np.array_equal(a, b), np.nonzero(a != b)[0][:8]
    assert torch.equal(full.screen, sub.screen)
    full.close()
    sub.close()


@pytest.mark.parametrize("n,bs", [(256, 64), (72, 24)])
def test_vecenv_sub_batches_match_full_batch(n, bs):
    """VecEnv(n, batch_size=bs) driven through async_reset/recv/send with the reward stack,
    template reload on done (max_episode_steps 3) and auto-reset: every sub-batch's rewards,
    dones and observations equal those of the same envs in a full-batch VecEnv.  (72, 24) is the
    reference's own setting (README.md:116-118): sub-batches in padded 64-env slots."""
    import torch
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    rom, state = game_rom(), open(STATE, "rb").read()
    rounds = 7
    acts = torch.from_numpy(np.random.default_rng(12).integers(0, 8, (rounds, n), dtype=np.uint8)).cuda()
    kw = dict(rom=rom, state=state, max_episode_steps=3, reload_on_reset=True, log_interval=0)
    full = VecEnv(n, **kw)
    sub = VecEnv(n, batch_size=bs, **kw)
    full.async_reset()
    sub.async_reset()
    f_obs = full.recv()[0].clone()
    got = {}
    for b in range(n // bs):
        o, r, d, t, infos, ids, m = sub.recv()
        got[int(ids[0])] = o.clone()
        sub.send(acts[0, ids])
    assert torch.equal(torch.cat([got[k] for k in sorted(got)]), f_obs)
    dones = 0
    for rnd in range(rounds):
        full.send(acts[rnd])
        f_obs, f_rew, f_term, f_trunc = [x.clone() for x in full.recv()[:4]]
        dones += int(f_term.sum())
        for b in range(n // bs):
            o, r, d, t, infos, ids, m = sub.recv()
            e0 = int(ids[0])
            sl = slice(e0, e0 + bs)
            assert torch.equal(r, f_rew[sl]), (rnd, e0)
            assert torch.equal(d, f_term[sl]) and torch.equal(t, f_trunc[sl])
            assert torch.equal(o, f_obs[sl]), (rnd, e0)
            sub.send(acts[min(rnd + 1, rounds - 1), ids])
    assert dones == 2 * n   # every episode ended (and was reloaded) twice inside the run
    full.close()
    sub.close()


def test_vecenv_padded_slots_step_and_savestates():
    """VecEnv(72, batch_size=24) (sub-batches in padded 64-env slots): step() over all envs returns
    the envs in env order, equal to an unpadded VecEnv(72); save_state/load_state address envs by
    their env index."""
    import torch
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    rom, state = game_rom(), open(STATE, "rb").read()
    kw = dict(rom=rom, state=state, max_episode_steps=4, reload_on_reset=True, log_interval=0)
    full, sub = VecEnv(72, **kw), VecEnv(72, batch_size=24, **kw)
    assert sub._padded and sub.emu.n == 3 * 64 and not full._padded
    fo, _ = full.reset()
    so, _ = sub.reset()
    assert torch.equal(fo, so)
    acts = torch.from_numpy(np.random.default_rng(13).integers(0, 8, (6, 72), dtype=np.uint8)).cuda()
    for t in range(6):
        f = full.step(acts[t])
        s = sub.step(acts[t])
        for x, y in zip(f[:4], s[:4]):
            assert torch.equal(x, y), t
    torch.cuda.synchronize()
    for e in (0, 23, 24, 47, 71):
        assert full.save_state(e) == sub.save_state(e), e
    st = full.save_state(5)
    sub.load_state(50, st)
    assert sub.save_state(50) == st
    full.close()
    sub.close()


def test_vecenv_sub_batches_log_raises_injected_error():
    """VecEnv(256, batch_size=64) through recv/send with a logging interval: an error
    code a sub-batch step writes on its own stream is not lost to the logging interval's check and
    clear — the reference's exception (KeyError: MAP_ID_REF lookup of an unknown map id,
    environment.py:739) is raised at the first interval after the step that hit it (by the recv()
    that reads the interval's snapshot: VecEnv._read_logs), and the episode statistics of every
    sub-batch are all-reduced in each interval."""
    import torch
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    n, bs, log = 256, 64, 4
    v = VecEnv(n, rom=game_rom(), power_on=True, batch_size=bs, max_episode_steps=3, log_interval=log)
    g = torch.Generator(device=v.device)
    g.manual_seed(7)
    v.async_reset()
    bad_env, raised, infos_seen, sends = 70, None, [], 0
    for rnd in range(3 * log):
        for b in range(n // bs):
            try:
                o, r, d, t, infos, ids, m = v.recv()
                infos_seen += infos
                if rnd == log + 1 and int(ids[0]) == 64:          # env 70 is in the second sub-batch
                    torch.cuda.synchronize()
                    v.emu.poke(v.phys(bad_env), 0xD35E, bytes([0xF8]))   # map id 248: not in MAP_ID_REF
                v.send(torch.randint(0, 8, (bs,), device=v.device, generator=g).to(torch.uint8))
                sends += 1
            except KeyError as e:
                raised = (rnd, str(e))
                break
        if raised:
            break
    v.close()
    assert raised is not None and f"env {bad_env}" in raised[1], raised
    assert raised[0] <= 2 * log + 1, raised            # at the first interval after the poke
    assert infos_seen and all(i["episodes"] > 0 for i in infos_seen)
