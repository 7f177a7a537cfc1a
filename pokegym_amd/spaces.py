"""Observation/action spaces of the reference env (environment.py:164-167).

gymnasium is not a dependency of the hot path: when it is importable its Box/Discrete are used,
otherwise these minimal stand-ins carry the same attributes (shape, dtype, low, high, n)."""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - depends on the environment
    from gymnasium.spaces import Box, Discrete  # type: ignore
except Exception:  # noqa: BLE001
    class Box:  # type: ignore[no-redef]
        def __init__(self, low, high, shape, dtype):
            self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return x.shape == self.shape and x.dtype == self.dtype

        def __repr__(self):
            return f"Box({self.low}, {self.high}, {self.shape}, {self.dtype})"

    class Discrete:  # type: ignore[no-redef]
        def __init__(self, n: int):
            self.n = int(n)
            self.shape = ()
            self.dtype = np.dtype(np.int64)

        def contains(self, x) -> bool:
            return 0 <= int(x) < self.n

        def __repr__(self):
            return f"Discrete({self.n})"


def observation_space():
    return Box(low=0, high=255, shape=(72, 80, 4), dtype=np.uint8)


def action_space():
    return Discrete(8)


def screen_space():
    """The full-resolution grey screen (screen.screen_ndarray()[:, :, 0], environment.py:268) that
    the screen-obs configuration returns instead of the (72, 80, 4) composite."""
    return Box(low=0, high=255, shape=(144, 160), dtype=np.uint8)
