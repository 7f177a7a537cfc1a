"""pokegym_amd — MI355X-native batched Pokémon Red env.step (drop-in for pokegym's hot path).

Public surface:
  pokegym_amd.emulator.BatchedEmulator   device-resident batch of emulators (C ABI wrapper)
  pokegym_amd.env.Environment            per-env Gymnasium-shaped surface (environment.py:436)
  pokegym_amd.env.VecEnv                 PufferLib-shaped batched surface
"""
__version__ = "0.1.0"
