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
