"""Video / screenshot capture (environment.py:200-206, :1244-1249, :1340, :1616)."""
import numpy as np
import pytest
import torch

from pokegym_amd import video


class _Emu:
    def __init__(self):
        self.device = torch.device("cpu")
        self.screen = torch.zeros((3, 144, 160), dtype=torch.uint8)


def test_recorder_spills_and_keeps_order(tmp_path):
    emu = _Emu()
    rec = video.FrameRecorder(emu, [2, 0], capacity=4)
    for t in range(10):
        emu.screen[2].fill_(t)
        emu.screen[0].fill_(100 + t)
        rec.capture()
    f = rec.frames(0)
    assert f.shape == (10, 144, 160) and [int(x[0, 0]) for x in f] == list(range(10))
    assert [int(x[5, 5]) for x in rec.frames(1)] == [100 + t for t in range(10)]
    out = rec.write(tmp_path / "reset_0")
    assert out.exists()
    if out.suffix == ".npz":
        frames = np.load(out)["frames"]
        assert len(frames) == 10 and all((fr == t).all() for t, fr in enumerate(frames))
    rec.clear()
    assert rec.frames(0).shape[0] == 0


def test_screenshot(tmp_path):
    scr = np.full((144, 160), 0x55, np.uint8)
    out = video.save_screenshot(scr, "healing", 40, 3, tmp_path)
    assert out.name.startswith("3_healing_40") and out.exists()


@pytest.mark.gpu
def test_environment_save_video(tmp_path):
    """Environment(save_video=True): one file per episode under s_path, one frame per step, equal
    to the screens the steps produced."""
    from pokegym_amd.env import Environment
    from tests.pkbench_state import pkbench_power_on
    rom, state = pkbench_power_on()
    env = Environment(rom_path=rom, state_path=state, save_video=True, max_episode_steps=4, s_path=str(tmp_path))
    env.reset()
    shots = []
    for a in [0, 3, 4, 1]:
        env.step(a)
        shots.append(env.video()[:, :, 0].copy())
    out = env.last_video
    assert out.exists() and out.stem == "reset_0"
    if out.suffix == ".npz":
        frames = np.load(out)["frames"]
        assert len(frames) == 4 and all(np.array_equal(a, b) for a, b in zip(frames, shots))
    env.close()


GREY = np.array([0xFF, 0x99, 0x55, 0x00], np.uint8)


@pytest.mark.gpu
def test_environment_video_frames_vs_oracle(tmp_path, monkeypatch):
    """environment.py:1244-1249 / :1340 / :1616: the episode file Environment(save_video=True) writes
    holds, frame by frame, the screen the oracle emulator shows after each of the same steps
    (GREY[oracle screen]); the .npz writer is forced (mediapy blocked) so frames are compared
    exactly rather than through a lossy mp4."""
    import sys
    from oracle import oracle as O
    from pokegym_amd.env import Environment
    from tests.pkbench_state import pkbench_power_on
    monkeypatch.setitem(sys.modules, "mediapy", None)   # import mediapy -> ImportError
    rom, state = pkbench_power_on()
    acts = [0, 3, 4, 1, 5, 2, 6, 7, 0, 3]
    env = Environment(rom_path=rom, state_path=state, save_video=True, max_episode_steps=len(acts),
                      s_path=str(tmp_path))
    env.reset()
    for a in acts:
        env.step(a)
    out = env.last_video
    env.close()
    assert out.suffix == ".npz" and out.stem == "reset_0"
    frames = np.load(out)["frames"]
    gb = O.GB(rom, state)
    want = []
    for a in acts:
        gb.run_action(a)
        want.append(GREY[gb.screen()])
    assert frames.shape == (len(acts), 144, 160)
    for t, (f, w) in enumerate(zip(frames, want)):
        assert np.array_equal(f, w), f"frame {t}: {(f != w).sum()} pixels differ from the oracle"


@pytest.mark.gpu
def test_vecenv_video_recorder_vs_oracle(tmp_path, monkeypatch):
    """VecEnv.video_recorder (the reference's per-env save_video on the batched surface): 8 envs of
    a 64-env VecEnv, 6 random-action steps; every recorded frame == GREY[oracle screen] of that env
    after that step, and the episode file written for one of them holds the same frames."""
    import sys
    import torch
    from oracle import oracle as O
    from pokegym_amd.env import VecEnv
    from pokegym_amd.testrom.game import game_rom
    monkeypatch.setitem(sys.modules, "mediapy", None)
    rom, n, steps = game_rom(), 64, 6
    envs = [1, 9, 14, 23, 31, 40, 52, 63]
    acts = np.random.default_rng(6464).integers(0, 9, (steps, n), dtype=np.uint8)
    vec = VecEnv(n, rom=rom, power_on=True, reward=False, max_episode_steps=1000, log_interval=0)
    rec = vec.video_recorder(envs, capacity=4)   # spills to host once: the whole episode is kept
    vec.reset()
    for t in range(steps):
        vec.step(torch.from_numpy(acts[t]).to(vec.device))
        rec.capture()
    got = [rec.frames(k) for k in range(len(envs))]
    out = rec.write(tmp_path / "env23", k=envs.index(23))
    vec.close()
    for k, e in enumerate(envs):
        gb = O.GB(rom, None)
        gb.power_on()
        assert got[k].shape == (steps, 144, 160)
        for t in range(steps):
            gb.run_action(int(acts[t, e]))
            assert np.array_equal(got[k][t], GREY[gb.screen()]), f"env {e} step {t + 1} differs from the oracle"
    assert np.array_equal(np.load(out)["frames"], got[envs.index(23)])
