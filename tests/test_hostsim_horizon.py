"""The segment-continuation premise of tests/test_gpu_horizon.py, checked on the CPU: an env
loaded (pk_load_env) from the oracle's v9 state at step k and stepped on continues the oracle's
own continuous trajectory exactly.  Host-simulation build of the unmodified kernels."""
import numpy as np

from oracle import oracle
from pokegym_amd.testrom.game import game_rom
from tests.hostsim.sim import SimEmulator
from tests.test_gpu_horizon import horizon_actions


def test_hostsim_segment_continuation():
    rom = game_rom()
    every, seg, ntraj = 20, 40, 4
    actions = horizon_actions(total=2 * seg, ntraj=ntraj)
    dig, keep = oracle.trajectory(rom, None, actions, every, seg)
    emu = SimEmulator(rom, 2 * ntraj, render=True)
    for j in range(ntraj):
        emu.load_env(ntraj + j, keep[(1, j)])
    table = np.concatenate([actions[:seg], actions[seg:]], axis=1)
    for t in range(seg):
        emu.step(table[t])
        if (t + 1) % every == 0:
            got = oracle.state_digests(emu.snapshot_range(0, 2 * ntraj))
            assert np.array_equal(got[:ntraj], dig[(t + 1) // every - 1]), t
            assert np.array_equal(got[ntraj:], dig[(seg + t + 1) // every - 1]), t
    emu.close()
