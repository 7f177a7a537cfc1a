"""K4/K5r/K3 on the MI355X (through the C ABI) against the reference's recorded reward-stack
outputs, and the full step (K1 emulate -> K2 render -> K4 reward -> K3 obs) against the oracle
emulator + reward oracle end to end."""
import os

import numpy as np
import pytest

from reward_replay import run_replay, sequences

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GREY = np.array([0xFF, 0x99, 0x55, 0x00], np.uint8)


class GpuRewardBackend:
    def __init__(self, rom):
        self.rom = rom

    def create(self, state, max_steps):
        from pokegym_amd.emulator import BatchedEmulator
        return BatchedEmulator(self.rom, 1, state=state, frame_skip=0, render=False, reward=True,
                               max_episode_steps=max_steps, heatmap=True)

    def destroy(self, h):
        h.close()

    def reset(self, h):
        h.reset()

    def step(self, h, action):
        import torch
        h.step(torch.tensor([action], dtype=torch.uint8, device=h.device))
        return float(h.rewards[0].item()), bool(h.terminals[0].item())

    def error(self, h):
        return int(h.errors[0].item())

    def obs(self, h):
        return h.obs[0].cpu().numpy()

    def set_ram(self, h, w, hr):
        import torch
        h.set_ram(0xC000, torch.from_numpy(np.ascontiguousarray(w)))
        h.set_ram(0xFF80, torch.from_numpy(np.ascontiguousarray(hr)))

    def get_ram(self, h):
        return h.get_ram(0xC000, 8192)[0].cpu().numpy(), h.get_ram(0xFF80, 127)[0].cpu().numpy()

    def set_screen(self, h, s):
        import torch
        h.screen[0].copy_(torch.from_numpy(np.ascontiguousarray(s)))

    def info(self, h):
        if not int(h.info_flag[0].item()):
            return None
        return h.info[:, 0].cpu().numpy()

    def events(self, h):
        from pokegym_amd.info import event_values
        return event_values((h.info_bits[:, 0].cpu().numpy().astype(np.int64) & 0xFFFFFFFF).tolist())

    def heat(self, h):
        return h.heatmap[0].reshape(-1).cpu().numpy().astype(np.float64)


@pytest.mark.gpu
def test_gpu_reward_kernels_match_reference_replay():
    from pokegym_amd.testrom.game import game_rom
    g, seqs = sequences()
    base = open(os.path.join(REPO, "pokegym_amd", "states", "Bulbasaur.state"), "rb").read()
    assert run_replay(GpuRewardBackend(game_rom()), base, g, seqs) > 1500


@pytest.mark.gpu
def test_gpu_info_record_matches_reference():
    """K4's info telemetry record (pk_info_ptr) against the reference's info dicts."""
    from reward_replay import check_events, check_info, run_info_replay
    from pokegym_amd.testrom.game import game_rom
    base = open(os.path.join(REPO, "pokegym_amd", "states", "Bulbasaur.state"), "rb").read()
    g, got = run_info_replay(GpuRewardBackend(game_rom()), base)
    assert check_info(g, got) > 100
    check_events(g, got.events)


@pytest.mark.gpu
def test_gpu_environment_info_dict_and_vecenv_info_stats():
    """Environment.step returns the reference-shaped info dict at done; VecEnv all-reduces the
    device-side info sums at its logging interval."""
    import torch
    from pokegym_amd.env import Environment, VecEnv
    from pokegym_amd.info import STATS_FIELDS
    from tests.pkbench_state import pkbench_power_on
    rom, state = pkbench_power_on()
    env = Environment(rom_path=rom, state_path=state, max_episode_steps=3)
    env.reset()
    infos = [env.step(0)[4] for _ in range(3)]
    assert infos[0] == {} and infos[1] == {}
    st = infos[2]["stats"]
    assert set(infos[2]["gym_events"]) == {f"gym_{g}_events" for g in range(3, 8)} and "dojo_events_aggregate" in infos[2]
    assert st["step"] == 3 and len(st["levels"]) == 6 and set(infos[2]["reward"]) >= {"delta", "exploration"}
    assert set(STATS_FIELDS) - set(st) == {f"levels_{i}" for i in range(6)}
    assert st["coord"] == float(infos[2]["pokemon_exploration_map"].sum()) <= 3.0   # +1 per step, -1 on a map change
    env.close()
    v = VecEnv(64, rom=rom, power_on=True, max_episode_steps=2, log_interval=4)
    v.reset()
    out = None
    for _ in range(4):
        out = v.step(torch.zeros(64, dtype=torch.uint8))
    info = out[4][0]
    assert info["info_records"] == 128 and info["stats"]["step"] == 2.0
    assert info["stats"]["coord"] != info["stats"]["coord"]   # NaN: no heat map kept
    v.close()
    v = VecEnv(8, rom=rom, power_on=True, max_episode_steps=2, log_interval=4, heatmap=True)
    v.reset()
    for _ in range(4):
        v.step(torch.zeros(8, dtype=torch.uint8))
    em = v.exploration_map()
    assert em.shape == (444, 436) and int(em.sum()) == int(v.emu.heatmap.sum()) <= 8 * 4
    v.close()


class _GBBus:
    """oracle/reward.py bus over an oracle emulator (PyBoy get/set_memory_value)."""

    def __init__(self, gb):
        self.gb = gb

    def r(self, a):
        if a > 0xFFFF:
            raise IndexError(a)
        return self.gb.read(a)

    def w(self, a, v):
        self.gb.write(a, v & 0xFF)


@pytest.mark.gpu
@pytest.mark.parametrize("state_name", [None, "Bulbasaur"])
def test_gpu_full_step_with_reward_matches_oracle(state_name):
    import torch
    from oracle import oracle as O
    from oracle import reward as R
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    rom = game_rom()
    state = None
    if state_name:
        state = open(os.path.join(REPO, "pokegym_amd", "states", f"{state_name}.state"), "rb").read()
    n, steps = 64, 6
    emu = BatchedEmulator(rom, n, state=state, render=True, reward=True, max_episode_steps=4)
    rng = np.random.default_rng(7)
    acts = rng.integers(0, 8, (steps, n)).astype(np.uint8)
    obs0 = emu.reset().cpu().numpy()
    gbs, sts, buses = [], [], []
    for e in range(n):
        gb = O.GB(rom, state) if state else O.GB(rom)
        if state is None:
            gb.power_on()
        st = R.EnvState()
        bus = _GBBus(gb)
        o = R.reset(st, bus, GREY[gb.screen()], reload=(lambda gb=gb: gb.load_state(state) if state else gb.power_on()),
                    max_episode_steps=4)
        assert np.array_equal(o, obs0[e]), e
        gbs.append(gb), sts.append(st), buses.append(bus)
    for t in range(steps):
        obs, rew, term, trunc = emu.step(torch.from_numpy(acts[t]).to(emu.device))
        obs, rew, term = obs.cpu().numpy(), rew.cpu().numpy(), term.cpu().numpy()
        wram = emu.get_ram(0xC000, 8192).cpu().numpy()
        errs = emu.errors.cpu().numpy()
        done_mask = np.zeros(n, np.uint8)
        for e in range(n):
            gbs[e].run_action(int(acts[t, e]))
            o, r, d = R.step(sts[e], buses[e], int(acts[t, e]), GREY[gbs[e].screen()])
            assert errs[e] == sts[e].err, (t, e)
            if sts[e].err:
                continue
            assert r == rew[e], (t, e, r, rew[e])
            assert bool(d) == bool(term[e]), (t, e)
            assert np.array_equal(o, obs[e]), (t, e)
            assert np.array_equal(gbs[e].wram(), wram[e]), (t, e)
            done_mask[e] = d
        if done_mask.any():
            obs_r = emu.reset(torch.from_numpy(done_mask).to(emu.device)).cpu().numpy()
            for e in np.nonzero(done_mask)[0]:
                o = R.reset(sts[e], buses[e], GREY[gbs[e].screen()], reload=None, max_episode_steps=4)
                assert np.array_equal(o, obs_r[e]), (t, e)
    emu.close()



@pytest.mark.gpu
def test_gpu_reward_replay_at_scale():
    """K4/K5r/K3 at width against the reference's recorded outputs: every golden sequence replicated
    over 4,096-env handles (reward_replay.run_replay_batched)."""
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    from reward_replay import run_replay_batched
    base = open(os.path.join(REPO, "pokegym_amd", "states", "Bulbasaur.state"), "rb").read()
    rom = game_rom()

    def make(state, n, max_steps):
        return BatchedEmulator(rom, n, state=state, frame_skip=0, render=False, reward=True,
                               max_episode_steps=max_steps, heatmap=True)

    checked = run_replay_batched(make, 4096, base)
    assert checked["step"] > 1500 and checked["err"] >= 6 and checked["reset"] > 80, checked
