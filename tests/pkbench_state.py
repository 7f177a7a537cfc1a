"""pkbench's own start state for single-env surfaces (GPU tests)."""


def pkbench_power_on():
    """(rom, v9 state) of pkbench after its boot: the savestate a pkbench Environment starts from.
    The default template (Bulbasaur.state) is a Pokémon Red state — run on pkbench its pc lands in
    unrelated code that wipes the party, and the reference's info step raises ValueError for an
    empty party (environment.py:1672)."""
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    rom = game_rom()
    emu = BatchedEmulator(rom, 1)
    state = emu.snapshot(0)
    emu.close()
    return rom, state
