"""Video and screenshot capture (environment.py:1244-1249, :1340-1341, :1616-1617
and :200-206).

The reference writes every step's screen (screen.screen_ndarray(), (144, 160, 3)) into one mp4 per
episode (`{s_path}/reset_{k}.mp4`, mediapy VideoWriter, 60 fps) and saves JPEG screenshots on
events.  Here frames stay on the device until an episode's file is written: `FrameRecorder`
copies the screens of the recorded envs into a device ring buffer once per step (stream-ordered, no
host sync) and `write()` encodes an episode when it ends — mp4 through mediapy when it is
importable (the reference's writer), else every frame exactly in a compressed .npz (frames, fps)
plus an animated-GIF preview through Pillow (GIF merges repeated frames, so the .npz is the record).
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np
import torch

FPS = 60


def to_rgb(screen: np.ndarray) -> np.ndarray:
    """(144, 160) grey screen -> (144, 160, 3) u8, the shape of screen.screen_ndarray()."""
    return np.repeat(np.asarray(screen, np.uint8)[..., None], 3, axis=2)


def write_frames(path: str | os.PathLike, frames: np.ndarray, fps: int = FPS) -> Path:
    """Encode (T, 144, 160) grey frames; returns the path written (the suffix tells the format)."""
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    frames = np.asarray(frames, np.uint8)
    try:  # the reference's writer (environment.py:1248), when installed
        import mediapy as media  # type: ignore
        out = path.with_suffix(".mp4")
        with media.VideoWriter(out, frames.shape[1:3], fps=fps) as w:
            for f in frames:
                w.add_image(to_rgb(f))
        return out
    except ImportError:
        pass
    out = path.with_suffix(".npz")
    np.savez_compressed(out, frames=frames, fps=np.int32(fps))
    try:
        from PIL import Image
        imgs = [Image.fromarray(f, mode="L") for f in frames]
        if imgs:
            imgs[0].save(path.with_suffix(".gif"), save_all=True, append_images=imgs[1:],
                         duration=max(1, round(1000 / fps)), loop=0)
    except ImportError:
        pass
    return out


def save_screenshot(screen: np.ndarray, event, map_n, counter: int, directory: str | os.PathLike = "screenshots") -> Path:
    """environment.py:200-206: `screenshots/{counter}_{event}_{map_n}.jpeg` of the (144, 160, 3) screen."""
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    out = d / f"{counter}_{event}_{map_n}.jpeg"
    try:
        from PIL import Image
        Image.fromarray(to_rgb(screen)).save(out, quality=95)
    except ImportError:
        out = out.with_suffix(".npy")
        np.save(out, np.asarray(screen, np.uint8))
    return out


class FrameRecorder:
    """Device buffer of the screens of some envs of a BatchedEmulator, one frame per step; a full
    buffer is moved to host memory in one copy (so an episode of any length is kept whole)."""

    def __init__(self, emu, envs, capacity: int = 1024):
        self.emu = emu
        self.envs = torch.as_tensor(list(envs), dtype=torch.long, device=emu.device)
        self.capacity = int(capacity)
        self.buf = torch.zeros((self.capacity, len(self.envs), emu.screen.shape[1], emu.screen.shape[2]),
                               dtype=torch.uint8, device=emu.device)
        self.count = 0          # frames in the device buffer
        self.spilled: list[np.ndarray] = []

    def capture(self):
        """Copy the recorded envs' current screens into the next slot (device, stream-ordered)."""
        if self.count == self.capacity:
            self.spilled.append(self.buf.to("cpu", copy=True).numpy())
            self.count = 0
        torch.index_select(self.emu.screen, 0, self.envs, out=self.buf[self.count])
        self.count += 1

    def frames(self, k: int = 0) -> np.ndarray:
        """All captured frames of the k-th recorded env, oldest first (host sync)."""
        parts = [c[:, k] for c in self.spilled] + [self.buf[:self.count, k].cpu().numpy()]
        return np.concatenate(parts, axis=0)

    def clear(self):
        self.count = 0
        self.spilled = []

    def write(self, path, k: int = 0, fps: int = FPS) -> Path:
        return write_frames(path, self.frames(k), fps)
