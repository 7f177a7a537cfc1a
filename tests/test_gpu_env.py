"""Gymnasium/PufferLib surfaces on the MI355X (through the C ABI)."""
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

from tests.pkbench_state import pkbench_power_on  # noqa: E402



@pytest.mark.gpu
def test_environment_reset_step_shapes(tmp_path):
    from pokegym_amd.env import Environment
    rom_bytes, state = pkbench_power_on()
    rom = tmp_path / "pkbench.gb"
    rom.write_bytes(rom_bytes)
    st = tmp_path / "pkbench.state"
    st.write_bytes(state)
    env = Environment(rom_path=str(rom), state_path=str(st), max_episode_steps=3)
    obs, info = env.reset()
    assert obs.shape == (72, 80, 4) and obs.dtype == np.uint8 and info == {}
    for t in range(3):
        obs, rew, term, trunc, info = env.step(t % 8)
        assert isinstance(rew, float) and term == trunc
    assert term  # time >= max_episode_steps
    assert env.observation_space.shape == (72, 80, 4) and env.action_space.n == 8
    env.close()


@pytest.mark.gpu
def test_environment_200_steps_vs_oracle():
    """configs[0]'s shape (test.py:16-29: one Environment, step(0) repeatedly) on the HIP path, env
    by env against the oracle emulator + the reward oracle (oracle/reward.py): the reset obs, then
    for each of 200 step(0) calls the (72,80,4) obs, the float64 reward, done and WRAM C000-DFFF,
    and the whole v9 machine state at the end."""
    from oracle import oracle as O
    from oracle import reward as R
    from pokegym_amd.env import Environment
    grey = np.array([0xFF, 0x99, 0x55, 0x00], np.uint8)
    rom, state = pkbench_power_on()
    env = Environment(rom_path=rom, state_path=state)
    gb = O.GB(rom, state)

    class Bus:
        def r(self, a):
            return gb.read(a)

        def w(self, a, v):
            gb.write(a, v & 0xFF)

    st, bus = R.EnvState(), Bus()
    want = R.reset(st, bus, lambda: grey[gb.screen()], reload=lambda: gb.load_state(state))
    obs, info = env.reset()
    assert np.array_equal(obs, want)
    for t in range(200):
        obs, rew, term, trunc, info = env.step(0)
        gb.run_action(0)
        o, r, d = R.step(st, bus, 0, grey[gb.screen()])
        assert st.err == 0
        assert np.array_equal(obs, o), f"step {t + 1}: obs differs"
        assert rew == r and term == bool(d), (t + 1, rew, r, term, d)
        assert np.array_equal(env.emu.peek(0, 0xC000, 0x2000), gb.wram().tobytes()), f"step {t + 1}: WRAM differs"
    assert env.emu.snapshot(0) == gb.save_state()
    env.close()


def test_base_and_environment_exports():
    """`from pokegym import Base, Environment` (pokegym/__init__.py): two classes, Environment(Base)
    (environment.py:89, :436), with the reference's Base methods."""
    import pokegym_amd
    from pokegym_amd import env
    assert pokegym_amd.Base is env.Base and pokegym_amd.Environment is env.Environment
    assert issubclass(env.Environment, env.Base) and env.Base is not env.Environment
    for m in ("save_screenshot", "save_state", "load_pokemon_center_state", "load_last_state", "load_first_state",
              "load_random_state", "reset", "render", "step", "video", "close"):
        assert callable(getattr(env.Base, m)), m


def _base_vs_oracle(env, rom, steps):
    """pokegym's Base (environment.py:89-434): the ROM boots (the template state is not loaded,
    :116-122), reset() returns the screen untouched (:228-230), and each step(a) is the action alone —
    no reward stack, so no RAM writes of its own — returning (render(), 0, False, False, {})
    (:404-406), render() the half-size screen beside this map's visited-tile window (:256-272).
    Against the oracle emulator + oracle/reward.render with a fresh per-map memory, for seeded
    actions: obs and WRAM every step, the v9 state at the start and the end.  The test ROMs keep
    no pokered position, so before each step the player's (map, y, x) at D35E / D361 / D362 are set
    in both — walks with jumps, three maps, the window's edges (0, 254, 255) and maps past 247."""
    from oracle import oracle as O
    from oracle import reward as R
    grey = np.array([0xFF, 0x99, 0x55, 0x00], np.uint8)
    gb = O.GB(rom)
    assert env.emu.snapshot(0) == gb.save_state()

    class Bus:
        def r(self, a):
            return gb.read(a)

        def w(self, a, v):
            raise AssertionError("Base.render writes no game memory")

    st, bus = R.EnvState(), Bus()
    scr, info = env.reset()
    assert info == {} and np.array_equal(scr, np.repeat(grey[gb.screen()][..., None], 3, axis=2))
    rng = np.random.default_rng(7)
    maps = set()
    m, y, x = 3, 10, 10
    for t in range(steps):
        a = int(rng.integers(0, 8))
        k = int(rng.integers(0, 10))
        if k == 0:
            m = int(rng.choice([3, 12, 250]))
        elif k == 1:
            y, x = (int(v) for v in rng.choice([0, 1, 36, 200, 218, 219, 254, 255], 2))
        else:
            y, x = (y + int(rng.integers(-1, 2))) & 0xFF, (x + int(rng.integers(-1, 2))) & 0xFF
        for addr, v in ((0xD35E, m), (0xD361, y), (0xD362, x)):
            env.emu.poke(0, addr, bytes([v]))
            gb.write(addr, v)
        obs, rew, term, trunc, info = env.step(a)
        gb.run_action(a)
        want = R.render(st, bus, grey[gb.screen()])
        maps.add(gb.read(0xD35E))
        assert (rew, term, trunc, info) == (0, False, False, {})
        assert obs.shape == (72, 80, 4) and np.array_equal(obs, want), f"step {t + 1}: obs differs"
        assert np.array_equal(env.emu.peek(0, 0xC000, 0x2000), gb.wram().tobytes()), f"step {t + 1}: WRAM differs"
    assert np.array_equal(env.render(), want)     # render() again: same tile, same window
    assert env.emu.snapshot(0) == gb.save_state()
    return maps


def test_hostsim_base_vs_oracle():
    """Base's host logic (boot, reset, step, the device-side render) over the host-simulated kernels."""
    from pokegym_amd.env import Base
    from pokegym_amd.testrom.game import game_rom
    from tests.hostsim.emulator import HostsimEmulator

    class HostBase(Base):
        def _emulator(self, rom, state, device):
            return HostsimEmulator(rom, 1, state=None, render=True)

    rom = game_rom()
    env = HostBase(rom_path=rom)
    _base_vs_oracle(env, rom, 30)
    env.close()


@pytest.mark.gpu
def test_base_steps_vs_oracle():
    """_base_vs_oracle on the HIP path, 120 steps of pkbench."""
    from pokegym_amd.env import Base
    from pokegym_amd.testrom.game import game_rom
    rom = game_rom()
    env = Base(rom_path=rom)
    maps = _base_vs_oracle(env, rom, 120)
    assert len(maps) == 3, maps
    env.close()


@pytest.mark.gpu
def test_vecenv_steps_and_autoresets():
    import torch
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    env = VecEnv(128, rom=game_rom(), power_on=True, max_episode_steps=2, log_interval=4)
    obs, _ = env.reset()
    assert obs.shape == (128, 72, 80, 4) and obs.device.type == "cuda"
    for t in range(4):
        obs, rew, term, trunc, infos = env.step(torch.randint(0, 8, (128,), device=env.device))
    assert term.all()
    assert infos and infos[0]["episodes"] == 256
    env.close()


@pytest.mark.gpu
def test_environment_savestates_round_trip(tmp_path):
    """environment.py:208-227 save_state / load_*_state through the device v9 export/import."""
    from pokegym_amd.env import Environment
    from pokegym_amd.testrom.game import game_rom
    env = Environment(rom_path=game_rom(), max_episode_steps=100)
    env.reset()
    for t in range(3):
        env.step(t % 8)
    env.save_state()
    saved = env.load_pokemon_center_state().getvalue()
    ram0 = env.emu.get_ram(0xC000, 8192)[0].cpu().numpy().copy()
    env.emu.poke(0, 0xC100, bytes([ram0[0x100] ^ 0xFF, ram0[0x101] ^ 0xFF]))
    env.step(3)
    env.emu.poke(0, 0xC100, bytes([ram0[0x100] ^ 0xFF]))
    assert not np.array_equal(env.emu.get_ram(0xC000, 8192)[0].cpu().numpy(), ram0)
    env.load_pyboy_state(env.load_pokemon_center_state())
    assert np.array_equal(env.emu.get_ram(0xC000, 8192)[0].cpu().numpy(), ram0)
    assert env.emu.snapshot(0) == saved
    assert len(env.load_first_state().getvalue()) == len(saved)
    env.close()


@pytest.mark.gpu
def test_load_state_mid_episode_keeps_step_counter():
    """load_pyboy_state leaves self.time alone (pyboy_binding.py:59-62): done fires at the same
    step with or without a state load in the middle of the episode."""
    from pokegym_amd.env import Environment
    rom, state = pkbench_power_on()
    done_at = []
    for load in (False, True):
        env = Environment(rom_path=rom, state_path=state, max_episode_steps=5)
        env.reset()
        first = env.load_first_state()
        for t in range(1, 8):
            if load and t == 3:
                env.load_pyboy_state(first)
            done = env.step(0)[2]
            if done:
                done_at.append(t)
                break
        env.close()
    assert done_at == [5, 5]


@pytest.mark.gpu
def test_environment_reset_takes_episode_params():
    """Environment.reset(max_episode_steps, reward_scale) (environment.py:1233, :1258-1259) equals an
    env built with those values: same rewards, done at the same step; a longer episode grows the
    device's seen-coordinate set."""
    import numpy as np
    from pokegym_amd.env import Environment
    rom, state = pkbench_power_on()
    a = Environment(rom_path=rom, state_path=state)
    b = Environment(rom_path=rom, state_path=state, max_episode_steps=5, reward_scale=2.0)
    oa, _ = a.reset(max_episode_steps=5, reward_scale=2.0)
    ob, _ = b.reset()
    assert np.array_equal(oa, ob)
    for t, act in enumerate([0, 3, 4, 1, 2]):
        ra = a.step(act)
        rb = b.step(act)
        assert np.array_equal(ra[0], rb[0]) and ra[1] == rb[1] and ra[2] == rb[2] == (t == 4)
    a.reset(max_episode_steps=50000)          # > the 20,480-step capacity chosen at construction
    for act in range(3):
        assert not a.step(act)[2]
    a.close()
    b.close()


@pytest.mark.gpu
def test_environment_reset_params_do_not_stick():
    """reset(max_episode_steps=X) then reset(): the reference resets both to their defaults on
    every call (environment.py:1233, :1258-1259), so the second episode has the default length."""
    from pokegym_amd.env import Environment
    rom, state = pkbench_power_on()
    env = Environment(rom_path=rom, state_path=state)
    env.reset(max_episode_steps=2, reward_scale=1.0)
    assert not env.step(0)[2] and env.step(0)[2]
    env.reset()
    assert (env.max_episode_steps, env.reward_scale) == (20480, 4.0)
    for _ in range(4):
        assert not env.step(0)[2]
    env.close()


@pytest.mark.gpu
def test_seen_set_growth_keeps_current_episode():
    """pk_set_episode_params growing the seen-coordinate table re-inserts every env's entries of
    its current episode: an env that is not reset keeps its exploration reward."""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    emu = BatchedEmulator(game_rom(), 64, reward=True, max_episode_steps=100)
    emu.reset()
    g = torch.Generator(device=emu.device)
    g.manual_seed(5)
    acts = torch.randint(0, 8, (6, 64), generator=g, device=emu.device).to(torch.uint8)
    ref = BatchedEmulator(game_rom(), 64, reward=True, max_episode_steps=100)
    ref.reset()
    for t in range(3):
        emu.step(acts[t])
        ref.step(acts[t])
    emu.set_episode_params(100000, 4.0)       # grows the table; no reset follows
    ref.set_episode_params(100, 4.0)
    for t in range(3, 6):
        _, ra, _, _ = emu.step(acts[t])
        _, rb, _, _ = ref.step(acts[t])
        assert torch.equal(ra, rb)
    emu.close()
    ref.close()
