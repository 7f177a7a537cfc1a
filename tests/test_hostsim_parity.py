"""HIP kernel LOGIC vs the oracle on the CPU: the unmodified kernels + C ABI compiled with g++
against a host-simulation HIP shim (tests/hostsim).  Whole-state v9 + screen comparison.
The shipped gfx950 build is compared against the same oracle in test_gpu_parity.py (-m gpu)."""
import os

import numpy as np
import pytest

from pokegym_amd.testrom.fuzz import fuzz_rom
from pokegym_amd.testrom.game import game_rom
from tests.hostsim.check import check

STATE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pokegym_amd", "states",
                     "Bulbasaur.state")


@pytest.mark.parametrize("seed", [0, 1, 3, 5, 11, 21, 33, 47, 58, 71])
def test_hostsim_fuzz(seed):
    assert check(fuzz_rom(seed), 8, 3, seed) == []


def test_hostsim_game():
    assert check(game_rom(), 8, 8, 3) == []


def test_hostsim_bulbasaur_state():
    assert check(fuzz_rom(21), 4, 3, 4, state=open(STATE, "rb").read()) == []


def test_hostsim_region_seams():
    """16-bit accesses across the RAM region seams take the generic bus path (K1 pair rule)."""
    from pokegym_amd.testrom.fuzz import boundary_rom
    assert check(boundary_rom(), 8, 2, 9) == []


@pytest.mark.parametrize("seed", [2, 13, 40])
def test_hostsim_fuzz_64_banks(seed):
    """1 MiB fuzz cartridges: code and data in the 58 switchable banks K1 does not stage in LDS
    (global-ROM fetch and read paths)."""
    assert check(fuzz_rom(seed, n_banks=64), 8, 3, seed) == []


def test_hostsim_game_64_banks():
    """pkbench on the 64-bank layout (overworld engine in 60 banks behind Bankswitch trampolines)."""
    assert check(game_rom(64), 8, 8, 5) == []


def test_hostsim_hram_code():
    """Code fetched from inside, across and outside the LDS-mirrored HRAM bytes, self-modified."""
    from pokegym_amd.testrom.fuzz import hram_code_rom
    assert check(hram_code_rom(), 8, 3, 5) == []


@pytest.mark.parametrize("seed", [0, 3, 21, 58])
def test_hostsim_general_execute_path(seed):
    """The host simulation runs one lane per thread, so by default every iteration takes K1's
    wave-uniform execute path (pk_exec<true>: scalar branches around unused units); this runs the
    general all-units path (pk_exec<false>, what divergent waves execute) against the oracle."""
    from tests.hostsim import sim
    L = sim.lib()
    L.pk_sim_set_uniform(0)
    try:
        assert check(fuzz_rom(seed), 8, 3, seed) == []
        assert check(game_rom(), 4, 4, seed) == []
    finally:
        L.pk_sim_set_uniform(1)
