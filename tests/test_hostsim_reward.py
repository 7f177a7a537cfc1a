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
