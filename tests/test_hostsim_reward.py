"""K4/K5r/K3 (pk_reward.hip) compiled for the host (tests/hostsim) against the reference's
recorded reward-stack outputs (tests/golden/reward_replay.npz) — CPU-side check of the exact
kernels the GPU runs (the gfx950 build is checked by tests/test_gpu_reward.py)."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "hostsim"))

from reward_replay import run_replay, sequences  # noqa: E402


@pytest.mark.slow
def test_hostsim_reward_kernels_match_reference_replay():
    from reward_backend import HostsimRewardBackend
    from pokegym_amd.testrom.game import game_rom
    g, seqs = sequences()
    base = open(os.path.join(HERE, "..", "pokegym_amd", "states", "Bulbasaur.state"), "rb").read()
    n = run_replay(HostsimRewardBackend(game_rom()), base, g, seqs)
    assert n > 1500


@pytest.mark.slow
def test_hostsim_info_record_matches_reference():
    """K4's info telemetry (pk_info_ptr / pk_info_flag_ptr) against the reference's info dicts."""
    from reward_backend import HostsimRewardBackend
    from reward_replay import check_events, check_info, run_info_replay
    from pokegym_amd.testrom.game import game_rom
    base = open(os.path.join(HERE, "..", "pokegym_amd", "states", "Bulbasaur.state"), "rb").read()
    g, got = run_info_replay(HostsimRewardBackend(game_rom()), base)
    assert check_info(g, got) > 100
    check_events(g, got.events)


@pytest.mark.slow
def test_hostsim_reward_replay_batched():
    """The golden sequences as envs of batched handles (reward_replay.run_replay_batched: replicas
    side by side, masked resets, one handle per episode length) — the host-compiled kernels at 160
    envs per handle (the GPU test runs 4,096)."""
    from emulator import HostsimEmulator
    from reward_replay import run_replay_batched
    from pokegym_amd.testrom.game import game_rom
    rom = game_rom()
    base = open(os.path.join(HERE, "..", "pokegym_amd", "states", "Bulbasaur.state"), "rb").read()

    def make(state, n, max_steps):
        return HostsimEmulator(rom, n, state=state, frame_skip=0, render=False, reward=True,
                               max_episode_steps=max_steps)

    checked = run_replay_batched(make, 160, base)
    assert checked["step"] > 1500 and checked["err"] >= 6 and checked["reset"] > 80, checked
