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


class FakeEmuErr(FakeEmu):
    """env 1 hits a reference exception at step 2 and finishes (auto-reset clears its error word)."""

    def __init__(self, n):
        super().__init__(n, done_every=2)
        self.errors = torch.zeros(n, dtype=torch.int32)

    def reset(self, mask=None):
        m = torch.ones(self.n, dtype=torch.bool) if mask is None else mask.to(torch.bool)
        self.errors[m] = 0
        return super().reset(mask)

    def step(self, a):
        out = super().step(a)
        if int(self.time[1]) == 2:
            self.errors[1] = 1   # PK_ERR_MAP_KEY -> KeyError
        return out


def test_vecenv_error_survives_autoreset():
    import pytest
    emu = FakeEmuErr(3)
    env = VecEnv(3, emulator=emu, log_interval=4)
    env.reset()
    env.step(torch.zeros(3, dtype=torch.uint8))
    env.step(torch.zeros(3, dtype=torch.uint8))     # error + done: the env is reset, its error word cleared
    assert int(emu.errors[1]) == 0 and int(env.sticky_errors[1]) == 1
    env.step(torch.zeros(3, dtype=torch.uint8))
    with pytest.raises(KeyError):
        env.step(torch.zeros(3, dtype=torch.uint8))   # raised at the logging interval


class FakeRangeEmu(FakeEmu):
    """FakeEmu with the sub-batch entry points (step_range / reset_range on full-size arrays)."""
    reward = True

    def __init__(self, n, done_every=3):
        super().__init__(n, done_every)
        self.rewards = torch.zeros(n, dtype=torch.float64)
        self.terminals = torch.zeros(n, dtype=torch.uint8)
        self.truncations = torch.zeros(n, dtype=torch.uint8)
        self.stepped = torch.zeros(n, dtype=torch.int64)

    def step_range(self, env0, a):
        sl = slice(env0, env0 + a.numel())
        self.time[sl] += 1
        self.stepped[sl] += 1
        self.obs[sl] = a.view(-1, 1, 1, 1)
        self.rewards[sl] = a.to(torch.float64)
        self.terminals[sl] = (self.time[sl] % self.done_every == 0).to(torch.uint8)
        self.truncations[sl] = self.terminals[sl]
        return self.obs[sl], self.rewards[sl], self.terminals[sl], self.truncations[sl]

    def reset_range(self, env0, count, mask=None):
        m = torch.zeros(self.n, dtype=torch.bool)
        m[env0:env0 + count] = True if mask is None else mask[env0:env0 + count].to(torch.bool)
        self.time[m] = 0
        self.obs[m] = 7
        return self.obs[env0:env0 + count]


class _NoStream:
    """CPU stand-in for the HIP streams/events of the sub-batch pipeline."""
    def __init__(self, *a, **k):
        pass

    def wait_stream(self, other):
        pass

    def wait_event(self, ev):
        pass

    def record(self, stream=None):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def test_vecenv_padded_sub_batch_slots(monkeypatch):
    """batch_size 24 (the reference's 72 envs in batches of 24, README.md:116-118): each sub-batch
    sits in its own 64-env slot; step() and recv() address envs by env index, padding never steps."""
    import pytest
    for name in ("Stream", "Event", "current_stream", "stream"):
        monkeypatch.setattr(torch.cuda, name, _NoStream)
    monkeypatch.setattr(torch.Tensor, "record_stream", lambda self, s: None)
    with pytest.raises(ValueError):
        VecEnv(72, emulator=FakeRangeEmu(72), batch_size=24)      # needs 3 slots of 64
    emu = FakeRangeEmu(3 * 64)
    env = VecEnv(72, emulator=emu, batch_size=24, log_interval=0)
    assert env.slot == 64 and [env.phys(e) for e in (0, 23, 24, 47, 48, 71)] == [0, 23, 64, 87, 128, 151]
    obs, _ = env.reset()
    assert obs.shape[0] == 72
    a = torch.arange(72, dtype=torch.uint8)
    obs, rew, term, trunc, _ = env.step(a)
    assert torch.equal(rew, a.to(torch.float64)) and torch.equal(obs[:, 0, 0, 0], a)
    pad = torch.ones(192, dtype=torch.bool)
    pad[[env.phys(e) for e in range(72)]] = False
    assert (emu.stepped[pad] == 0).all() and (emu.stepped[~pad] == 1).all()
    env.async_reset()
    for _ in range(3):
        o, r, d, t, infos, ids, m = env.recv()
        assert o.shape[0] == 24 and ids.numel() == 24
        env.send(ids.to(torch.uint8))
    for _ in range(3):
        o, r, d, t, infos, ids, m = env.recv()
        assert torch.equal(r, ids.to(torch.float64)) and torch.equal(o[:, 0, 0, 0], ids.to(torch.uint8))
        env.send(ids.to(torch.uint8))
    assert (emu.stepped[pad] == 0).all()


def test_vecenv_logging_interval_counted_where_it_fires(monkeypatch):
    """The sub-batch pipeline's logging interval (sticky-error check + statistics all-reduce) fires
    on the send that completes every log_interval-th env-step: VecEnv.logs_fired counts it there,
    and each sub-batch stream snapshots its rows and error codes after that step.  The host reads the
    snapshot — no host sync where it fires, which would drain every stream — num_batches recv()s
    later, when the sub-batch being received is the last one stepped before the interval; its record
    reaches the caller with that recv (bench.py reports both counts)."""
    for name in ("Stream", "Event", "current_stream", "stream"):
        monkeypatch.setattr(torch.cuda, name, _NoStream)
    monkeypatch.setattr(torch.Tensor, "record_stream", lambda self, s: None)
    emu = FakeRangeEmu(128, done_every=1000)
    env = VecEnv(128, emulator=emu, batch_size=64, log_interval=3)
    env.async_reset()
    got = []
    for t in range(1, 7):                       # env-steps 1..6: the interval fires at 3 and 6
        for k in range(env.num_batches):
            o, r, d, tr, infos, ids, m = env.recv()
            got.append((t, k, len(infos)))
            env.send(torch.zeros(64, dtype=torch.uint8))
        assert env.logs_fired == t // 3
    # records handed out: by env-step 4's second recv (its sub-batch was the last stepped at 3)
    assert [(t, k) for t, k, n in got if n] == [(4, 1)]
    assert got[-1][2] == 0
    o, r, d, tr, infos, ids, m = env.recv()
    assert len(infos) == 0
    env.send(torch.zeros(64, dtype=torch.uint8))
    o, r, d, tr, infos, ids, m = env.recv()
    assert len(infos) == 1                     # the interval that fired at env-step 6
    assert infos[0]["episodes"] == 0 and infos[0]["steps"] == 3 * 128


def test_vecenv_step_after_send_reads_the_pending_interval(monkeypatch):
    """An interval that fired on a send() is handed out by step() if the caller switches from
    recv/send to step() before the deferred read (VecEnv._read_logs)."""
    for name in ("Stream", "Event", "current_stream", "stream"):
        monkeypatch.setattr(torch.cuda, name, _NoStream)
    monkeypatch.setattr(torch.Tensor, "record_stream", lambda self, s: None)
    emu = FakeRangeEmu(128, done_every=1000)
    env = VecEnv(128, emulator=emu, batch_size=64, log_interval=1)
    env.async_reset()
    for _ in range(env.num_batches):
        env.recv()
        env.send(torch.zeros(64, dtype=torch.uint8))
    assert env.logs_fired == 1
    obs, r, d, t, infos = env.step(torch.zeros(128, dtype=torch.uint8))
    # the pending interval (env-step 1) and the one step() fires itself (env-step 2)
    assert len(infos) == 2 and infos[0]["steps"] == 128 and infos[1]["steps"] == 128
