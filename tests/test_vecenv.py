"""VecEnv / Environment host logic (PufferLib-style batching, auto-reset, statistics) with a
stand-in emulator on CPU tensors; the real device path is covered by tests/test_gpu_env.py."""
import torch

from pokegym_amd.env import VecEnv


class FakeEmu:
    def __init__(self, n, done_every=3):
        self.n, self.device, self.done_every = n, torch.device("cpu"), done_every
        self.obs = torch.zeros((n, 72, 80, 4), dtype=torch.uint8)
        self.time = torch.zeros(n, dtype=torch.int64)
        self.resets = []

    def reset(self, mask=None):
        m = torch.ones(self.n, dtype=torch.bool) if mask is None else mask.to(torch.bool)
        self.resets.append(m.clone())
        self.time[m] = 0
        self.obs[m] = 7
        return self.obs

    def step(self, a):
        self.time += 1
        self.obs[:] = a.view(-1, 1, 1, 1)
        rew = a.to(torch.float64)
        term = (self.time % self.done_every == 0).to(torch.uint8)
        return self.obs, rew, term, term.clone()

    def close(self):
        pass


def test_vecenv_autoreset_and_stats():
    emu = FakeEmu(4)
    env = VecEnv(4, emulator=emu, log_interval=3)
    obs, infos = env.reset()
    assert obs.shape == (4, 72, 80, 4) and infos == []
    for t in range(3):
        obs, rew, term, trunc, infos = env.step(torch.tensor([1, 2, 3, 4]))
        assert rew.dtype == torch.float64 and term.dtype == torch.bool
    assert term.all() and trunc.all()
    assert (obs == 7).all()                      # finished envs come back reset
    assert len(emu.resets) == 4 and emu.resets[-1].all() and not emu.resets[1].any()
    s = infos[0]
    assert s["episodes"] == 4 and s["episodic_return_sum"] == 3 * (1 + 2 + 3 + 4)
    assert s["mean_episode_length"] == 3


def test_vecenv_async_api():
    env = VecEnv(2, emulator=FakeEmu(2), env_offset=10)
    env.async_reset(0)
    o, r, d, t, i, ids, m = env.recv()
    assert ids.tolist() == [10, 11] and m.all()
    env.send(torch.tensor([5, 6]))
    o, r, d, t, i, ids, m = env.recv()
    assert r.tolist() == [5.0, 6.0]
    assert env.single_observation_space.shape == (72, 80, 4) and env.single_action_space.n == 8
