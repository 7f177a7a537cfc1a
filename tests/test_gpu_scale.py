"""HIP path vs the CPU oracle at the geometries the benchmark and BASELINE.json's configs run.

The small parity tests (test_gpu_parity.py) run <= 128 envs, where K1 launches 256-thread
workgroups.  These run the real shapes: configs[2] at its full 65,536 envs (512-thread
workgroups, two 32-env waves per SIMD, the 256-env HRAM mirror of a workgroup fully used),
configs[1] at 4,096 envs headless with the fixed [0,3,1,2] action cycle, and a configs[4] per-GPU
shard (32,768 envs) with the reward stack and a template reload on every done.  Every env is
compared: machine states as 64-bit digests of the v9 savestate (oracle.state_digests), rewards
as exact float64, observations and WRAM as digests.  The oracle runs in spawned worker processes
(tests/oracle_pool.py) while the GPU steps."""
import os

import numpy as np
import pytest

from oracle import oracle
from tests import oracle_pool as OP

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def gpu_digests(emu, headless=False, chunk=2048):
    out = np.zeros(emu.n, np.uint64)
    for e0 in range(0, emu.n, chunk):
        st = emu.snapshot_range(e0, min(chunk, emu.n - e0))
        out[e0:e0 + len(st)] = oracle.state_digests(st, headless)
    return out


def _explain(rom, state, actions, emu, env):
    """First differing v9 offsets of one env (diagnostics for a failing digest)."""
    ref, _ = oracle.batch_run(rom, state, np.ascontiguousarray(actions[:, env:env + 1]), want_screens=False)
    a = emu.snapshot_range(env, 1)[0]
    idx = np.nonzero(a != ref[0])[0]
    return env, idx[:10].tolist()


def _check_states(rom, state, actions, emu, futs, headless):
    want = OP.gather_digests(futs, emu.n)
    got = gpu_digests(emu, headless)
    bad = np.nonzero(want != got)[0]
    if len(bad):
        pytest.fail(f"{len(bad)}/{emu.n} envs differ; first: {[_explain(rom, state, actions, emu, int(e)) for e in bad[:3]]}")


def test_config3_geometry_65536_envs():
    """configs[2]'s env count, image interleave (32-env waves) and rendered frame 24 as ONE
    whole-handle launch (pk_step_kernel, 512-thread workgroups, wave priority).  Not the benchmark's
    own launch: bench.py steps configs[2] through VecEnv sub-batches on the small-LDS kernel, which
    test_config3_flow_vs_oracle_per_env checks at this size."""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    rom, n, steps = game_rom(), 65536, 2
    actions = np.random.default_rng(65536).integers(0, 8, (steps, n), dtype=np.uint8)
    with OP.pool() as ex:
        futs = OP.batch_digests(ex, rom, None, actions, chunk=1024)
        emu = BatchedEmulator(rom, n, render=True)
        acts = torch.from_numpy(actions).to(emu.device)
        for t in range(steps):
            emu.step(acts[t])
        torch.cuda.synchronize()
        _check_states(rom, None, actions, emu, futs, headless=False)
        emu.close()


def test_capacity_geometry_131072_envs_sub_batches():
    """131,072 envs in two concurrent 65,536-env sub-batches (pk_step_range on two streams): the
    shape of configs[3] split over two GPUs — 64-env waves, 512-env workgroups, two waves per SIMD
    across the two launches, HRAM mirror columns up to 511 — every env vs the oracle."""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    rom, n, steps, half = game_rom(), 131072, 1, 65536
    actions = np.random.default_rng(131072).integers(0, 9, (steps, n), dtype=np.uint8)
    with OP.pool() as ex:
        futs = OP.batch_digests(ex, rom, None, actions, chunk=2048)
        emu = BatchedEmulator(rom, n, render=True)
        acts = torch.from_numpy(actions).to(emu.device)
        streams = [torch.cuda.Stream() for _ in range(2)]
        cur = torch.cuda.current_stream()
        for t in range(steps):
            for b in (1, 0):
                streams[b].wait_stream(cur)
                with torch.cuda.stream(streams[b]):
                    emu.step_range(b * half, acts[t, b * half:(b + 1) * half])
            for st in streams:
                cur.wait_stream(st)
        torch.cuda.synchronize()
        _check_states(rom, None, actions, emu, futs, headless=False)
        emu.close()


def test_config2_geometry_4096_envs_headless_cycle():
    """configs[1]: 4,096 envs, no PPU render (LCD folding + HALT skip-ahead paths), the fixed
    [0,3,1,2] cycle (half the envs at a per-env phase, half with random presses incl. none)."""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    rom, n, steps = game_rom(), 4096, 8
    cyc = np.array([0, 3, 1, 2], np.uint8)
    actions = cyc[(np.arange(steps)[:, None] + np.arange(n)[None, :]) % 4].astype(np.uint8)
    actions[:, n // 2:] = np.random.default_rng(4096).integers(0, 9, (steps, n // 2), dtype=np.uint8)
    with OP.pool() as ex:
        futs = OP.batch_digests(ex, rom, None, actions, headless=True, chunk=128)
        emu = BatchedEmulator(rom, n, render=False)
        acts = torch.from_numpy(actions).to(emu.device)
        for t in range(steps):
            emu.step(acts[t])
        torch.cuda.synchronize()
        _check_states(rom, None, actions, emu, futs, headless=True)
        emu.close()


def test_config5_shard_32768_envs_reward_reload():
    """configs[4] per-GPU shard: 32,768 envs from pkbench's power-on state (bench.py's config5
    template) with the full reward stack, the (72,80,4) obs and a template reload on EVERY done
    (max_episode_steps 3, so two resets fire inside the run).  Every env: exact f64 rewards, dones,
    error codes, obs and WRAM digests.  (Bulbasaur.state is a Pokémon Red state: under pkbench its
    pc lands in unrelated code that wipes the party, so every env's first info step would raise
    the reference's empty-party ValueError instead of resetting.)"""
    import torch
    import xxhash
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    rom, state = game_rom(), None
    n, steps, max_steps = 32768, 7, 3
    actions = np.random.default_rng(32768).integers(0, 8, (steps, n), dtype=np.uint8)

    def dig(rows):
        return np.array([xxhash.xxh3_64_intdigest(r.tobytes()) for r in rows], np.uint64)

    with OP.pool() as ex:
        parts = OP.reward_runs_async(ex, rom, state, actions, max_steps, chunk=256)
        emu = BatchedEmulator(rom, n, state=state, render=True, reward=True, reload_on_reset=True,
                              max_episode_steps=max_steps)
        got_obs = np.zeros((steps + 1, n), np.uint64)
        got_wram = np.zeros((steps, n), np.uint64)
        got_rew = np.zeros((steps, n), np.float64)
        got_done = np.zeros((steps, n), np.uint8)
        got_err = np.zeros((steps, n), np.uint32)
        got_obs[0] = dig(emu.reset().cpu().numpy())
        acts = torch.from_numpy(actions).to(emu.device)
        for t in range(steps):
            obs, rew, term, trunc = emu.step(acts[t])
            got_rew[t] = rew.cpu().numpy()
            got_done[t] = term.cpu().numpy()
            got_err[t] = emu.errors.cpu().numpy()
            got_wram[t] = dig(emu.get_ram(0xC000, 8192).cpu().numpy())
            obs = emu.reset(term)
            got_obs[t + 1] = dig(obs.cpu().numpy())
        emu.close()
        rew, done, err, obs_d, wram_d = OP.gather_reward_runs(parts, steps, n)
    live = np.cumsum(err != 0, axis=0) == 0          # an env stops being compared after its error step
    assert np.array_equal(got_err[err != 0], err[err != 0])
    assert (got_done[live] == done[live]).all() and done[:, :].sum() > 0
    assert np.array_equal(got_rew[live], rew[live]), np.nonzero(got_rew != rew)
    assert (got_wram[live] == wram_d[live]).all()
    live_obs = np.vstack([np.ones((1, n), bool), live])
    assert (got_obs[live_obs] == obs_d[live_obs]).all()
    # resets fired where the reference's done did: time >= 3 after steps 3 and 6
    assert (done[2][live[2]] == 1).all() and (done[5][live[5]] == 1).all() and live[-1].all()


def test_config4_shard_vecenv_sub_batches():
    """configs[3] per-GPU shard through the PufferLib surface: 32,768 envs, screen obs, stepped as
    2 sub-batches of 16,384 on their own streams (the bench's config4) == the same envs stepped as
    one batch (screens, dones, whole-machine digests of every env)."""
    import torch
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    rom, n, steps = game_rom(), 32768, 4
    acts = torch.from_numpy(np.random.default_rng(3276).integers(0, 8, (steps, n), dtype=np.uint8)).cuda()
    kw = dict(rom=rom, power_on=True, reward=False, max_episode_steps=2, log_interval=0)
    full = VecEnv(n, **kw)
    sub = VecEnv(n, batch_size=n // 2, **kw)
    full.async_reset()
    sub.async_reset()
    for t in range(steps):
        full.recv()
        full.send(acts[t])
        for _ in range(2):
            sub.recv()
            sub.send(acts[t, sub.current_envs()])
    torch.cuda.synchronize()
    assert torch.equal(full.emu.screen, sub.emu.screen)
    assert torch.equal(full.emu.terminals, sub.emu.terminals) and bool(full.emu.terminals.any())
    assert np.array_equal(gpu_digests(full.emu), gpu_digests(sub.emu))
    full.close()
    sub.close()


def test_512_env_workgroups_48_steps(monkeypatch):
    """The >= 131,072-env K1 shape (64-env waves in 512-thread workgroups, HRAM mirror columns up
    to 511) over 48 env-steps of pkbench, 1,024 envs, every env vs the oracle."""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    monkeypatch.setenv("PK_K1_BLOCK", "512")
    monkeypatch.setenv("PK_WAVE_LANES", "64")
    rom, n, steps = game_rom(), 1024, 48
    actions = np.random.default_rng(512).integers(0, 9, (steps, n), dtype=np.uint8)
    with OP.pool() as ex:
        futs = OP.batch_digests(ex, rom, None, actions, chunk=64)
        emu = BatchedEmulator(rom, n, render=True)
        acts = torch.from_numpy(actions).to(emu.device)
        for t in range(steps):
            emu.step(acts[t])
        torch.cuda.synchronize()
        _check_states(rom, None, actions, emu, futs, headless=False)
        emu.close()


def test_config4_flow_vs_oracle_per_env():
    """The benchmarked configs[3] flow itself against the oracle, env by env: VecEnv with 32,768 envs
    in 2 sub-batches of 16,384 (pk_step_range launches on their own streams), recv/send over 7
    env-steps with max_episode_steps 4, so every env auto-resets on the device (pk_reset_range:
    template reload of the done envs of its sub-batch, environment.py:1612-1613 done rule) after its
    4th step.  Whole-machine v9 digests of every env after step 3 (before any reset) and after step
    7 (3 steps into the second episode) == the oracle replaying the same actions with reset-on-done;
    the dones recv() hands back == the oracle's, in both sub-batches."""
    import torch
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    rom, n, steps, max_steps = game_rom(), 32768, 7, 4
    actions = np.random.default_rng(40968).integers(0, 8, (steps, n), dtype=np.uint8)
    check_at = (2, steps - 1)
    with OP.pool() as ex:
        futs = OP.reset_flows(ex, rom, None, actions, max_steps, check_at, chunk=512)
        vec = VecEnv(n, rom=rom, power_on=True, reward=False, max_episode_steps=max_steps, log_interval=0,
                     batch_size=n // 2)
        assert vec.num_batches == 2
        acts = torch.from_numpy(actions).to(vec.device)
        vec.async_reset()
        got_done = np.zeros((steps, n), np.uint8)
        got_dig = []
        for t in range(steps):
            for _ in range(vec.num_batches):
                obs, rew, term, trunc, infos, ids, masks = vec.recv()
                sl = vec.current_envs()
                if t > 0:   # the terminals of this sub-batch's step t-1
                    got_done[t - 1, sl] = term.to(torch.uint8).cpu().numpy()
                vec.send(acts[t, sl])
            if t in check_at:
                # every sub-batch's step t has been sent: wait for both streams, digest every env
                vec._join_streams()
                torch.cuda.synchronize()
                got_dig.append(gpu_digests(vec.emu))
        got_done[steps - 1] = vec.emu.terminals.cpu().numpy()
        want_dig, want_done = OP.gather_reset_flows(futs, len(check_at), steps, n)
        vec.close()
    assert np.array_equal(got_done, want_done), np.argwhere(got_done != want_done)[:5]
    half = n // 2
    assert want_done[:, :half].sum() == half and want_done[:, half:].sum() == half   # one done per env
    for k, t in enumerate(check_at):
        bad = np.nonzero(got_dig[k] != want_dig[k])[0]
        assert not len(bad), f"after step {t + 1}: {len(bad)}/{n} envs differ, first {bad[:8].tolist()}"


def test_config3_flow_vs_oracle_per_env():
    """The benchmarked configs[2] flow itself (bench.py's default command), env by env: VecEnv with
    65,536 envs in 2 sub-batches of 32,768 (PufferLib batch_size, README.md:116-118), each stepped by
    pk_step_range on its own stream — the small-LDS K1 with 32-env waves in 256-thread workgroups, no
    wave priority, sub-batch 1 at env0 = 32,768 of a 65,536-env image interleave (asserted through
    pk_launch_shape) — over 6 recv/send env-steps with max_episode_steps 4, so every env auto-resets
    on the device (pk_reset_range template reload, done = time >= max_episode_steps,
    environment.py:1612-1613) after its 4th step.  Whole-machine v9 digests of every env after step 3
    (before any reset) and after step 6 (2 steps into the second episode), and the dones recv()
    hands back, == the oracle replaying the same actions with reset-on-done."""
    import torch
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    rom, n, steps, max_steps = game_rom(), 65536, 6, 4
    half = n // 2
    actions = np.random.default_rng(65538).integers(0, 8, (steps, n), dtype=np.uint8)
    check_at = (2, steps - 1)
    with OP.pool() as ex:
        futs = OP.reset_flows(ex, rom, None, actions, max_steps, check_at, chunk=1024)
        vec = VecEnv(n, rom=rom, power_on=True, reward=False, max_episode_steps=max_steps, log_interval=0,
                     batch_size=half)
        assert vec.num_batches == 2
        for e0 in (0, half):   # the launch bench.py's configs[2] line times
            assert vec.emu.launch_shape(e0, half) == {"small": True, "wave_lanes": 32, "block": 256, "prio": False,
                                                      "all_staged": False}, vec.emu.launch_shape(e0, half)
        acts = torch.from_numpy(actions).to(vec.device)
        vec.async_reset()
        got_done = np.zeros((steps, n), np.uint8)
        got_dig = []
        for t in range(steps):
            for _ in range(vec.num_batches):
                obs, rew, term, trunc, infos, ids, masks = vec.recv()
                sl = vec.current_envs()
                if t > 0:   # the terminals of this sub-batch's step t-1
                    got_done[t - 1, sl] = term.to(torch.uint8).cpu().numpy()
                vec.send(acts[t, sl])
            if t in check_at:
                vec._join_streams()
                torch.cuda.synchronize()
                got_dig.append(gpu_digests(vec.emu))
        got_done[steps - 1] = vec.emu.terminals.cpu().numpy()
        want_dig, want_done = OP.gather_reset_flows(futs, len(check_at), steps, n)
        vec.close()
    assert np.array_equal(got_done, want_done), np.argwhere(got_done != want_done)[:5]
    assert want_done[:, :half].sum() == half and want_done[:, half:].sum() == half   # one done per env
    for k, t in enumerate(check_at):
        bad = np.nonzero(got_dig[k] != want_dig[k])[0]
        assert not len(bad), f"after step {t + 1}: {len(bad)}/{n} envs differ, first {bad[:8].tolist()}"


@pytest.mark.parametrize("lanes", [16, 32])
def test_small_lds_kernel_48_steps(monkeypatch, lanes):
    """The small-LDS K1 (pk_step.hip built with PK_K1_SMALL: 2 staged banks, 128-env HRAM mirror,
    256-thread workgroups, two per CU), forced on a whole-handle launch, over 48 env-steps of pkbench
    (its banks 2-3 come from the global ROM), 1,024 envs, every env vs the oracle."""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    monkeypatch.setenv("PK_K1_SMALL", "1")
    monkeypatch.setenv("PK_WAVE_LANES", str(lanes))
    monkeypatch.setenv("PK_K1_BLOCK", "256")
    rom, n, steps = game_rom(), 1024, 48
    actions = np.random.default_rng(4800 + lanes).integers(0, 9, (steps, n), dtype=np.uint8)
    with OP.pool() as ex:
        futs = OP.batch_digests(ex, rom, None, actions, chunk=64)
        emu = BatchedEmulator(rom, n, render=True)
        acts = torch.from_numpy(actions).to(emu.device)
        for t in range(steps):
            emu.step(acts[t])
        torch.cuda.synchronize()
        _check_states(rom, None, actions, emu, futs, headless=False)
        emu.close()


def test_config5_flow_vecenv_vs_oracle_per_env():
    """The benchmarked configs[4] flow (bench.py config5 since round 4): VecEnv with the reward stack,
    32,768 envs in 2 sub-batches of 16,384 on their own streams (small-LDS K1, K2, K4, K3 per range),
    a template reload on every done (pk_reset_range with the reset kernels of the reward stack),
    max_episode_steps 3 so two resets fire inside 7 steps.  Per env and step, the rewards (exact
    f64) and dones recv() returns, and the obs of the last step, == the oracle emulator + the reward
    oracle with reload-on-reset (tests/oracle_pool._reward_run); the sticky error codes VecEnv keeps
    == the oracle's first error of each env."""
    import torch
    import xxhash
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    rom, n, steps, max_steps = game_rom(), 32768, 7, 3
    actions = np.random.default_rng(5327).integers(0, 8, (steps, n), dtype=np.uint8)
    with OP.pool() as ex:
        parts = OP.reward_runs_async(ex, rom, None, actions, max_steps, chunk=256)
        vec = VecEnv(n, rom=rom, power_on=True, reward=True, reload_on_reset=True, max_episode_steps=max_steps,
                     log_interval=0, batch_size=n // 2)
        acts = torch.from_numpy(actions).to(vec.device)
        vec.async_reset()
        got_rew = np.zeros((steps, n), np.float64)
        got_done = np.zeros((steps, n), np.uint8)
        for t in range(steps + 1):
            for _ in range(vec.num_batches):
                obs, rew, term, trunc, infos, ids, masks = vec.recv()
                sl = vec.current_envs()
                if t > 0:
                    got_rew[t - 1, sl] = rew.cpu().numpy()
                    got_done[t - 1, sl] = term.to(torch.uint8).cpu().numpy()
                vec.send(acts[min(t, steps - 1), sl])   # the extra send's step is not compared
            if t == steps - 1:
                vec._join_streams()
                torch.cuda.synchronize()
                last_obs = np.array([xxhash.xxh3_64_intdigest(o.tobytes()) for o in vec.emu.obs.cpu().numpy()],
                                    np.uint64)
                sticky = vec.sticky_errors.cpu().numpy().copy()
        torch.cuda.synchronize()
        vec.close()
        rew, done, err, obs_d, wram_d = OP.gather_reward_runs(parts, steps, n)
    live = np.cumsum(err != 0, axis=0) == 0
    first_err = np.where((err != 0).any(axis=0), err[np.argmax(err != 0, axis=0), np.arange(n)], 0)
    assert np.array_equal(sticky.astype(np.uint32), first_err.astype(np.uint32))
    assert np.array_equal(got_rew[live], rew[live]), np.argwhere(got_rew != rew)[:5]
    assert np.array_equal(got_done[live], done[live]) and done[:, :n // 2].sum() > 0 and done[:, n // 2:].sum() > 0
    ok = live[-1]
    assert np.array_equal(last_obs[ok], obs_d[steps][ok])
