"""pokegym_amd — MI355X-native batched Pokémon Red env.step (drop-in for pokegym's hot path).

Public surface:
  pokegym_amd.emulator.BatchedEmulator   device-resident batch of emulators (C ABI wrapper)
  pokegym_amd.env.Base                   the reference's Base: emulator surface, no reward stack (environment.py:89)
  pokegym_amd.env.Environment            per-env Gymnasium-shaped surface (environment.py:436)
  pokegym_amd.env.VecEnv                 PufferLib-shaped batched surface
"""
__version__ = "0.1.0"


def __getattr__(name):
    """`from pokegym_amd import Environment, Base` as `from pokegym import Base, Environment`
    (pokegym/__init__.py); loaded on first use so importing the package needs no GPU."""
    if name in ("Environment", "Base", "VecEnv"):
        from . import env
        return getattr(env, name)
    raise AttributeError(name)
