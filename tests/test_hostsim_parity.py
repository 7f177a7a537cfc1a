"""HIP kernel LOGIC vs the oracle on the CPU: the unmodified kernels + C ABI compiled with g++
against a host-simulation HIP shim (tests/hostsim).  Whole-state v9 + screen comparison.
The shipped gfx950 build is compared against the same oracle in test_gpu_parity.py (-m gpu)."""
import os

import numpy as np
import pytest

from pokegym_amd.testrom.fuzz import fuzz_rom
from pokegym_amd.testrom.game import game_rom
from tests import oracle_pool as OP
from tests.hostsim.check import check

STATE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pokegym_amd", "states",
                     "Bulbasaur.state")


@pytest.mark.parametrize("seed", [0, 1, 3, 5, 11, 21, 33, 47, 58, 71])
def test_hostsim_fuzz(seed):
    assert check(fuzz_rom(seed), 8, 3, seed) == []


def test_hostsim_game():
    assert check(game_rom(), 8, 8, 3) == []


def test_hostsim_bulbasaur_state():
    assert check(fuzz_rom(21), 4, 3, 4, state=open(STATE, "rb").read()) == []


def test_hostsim_region_seams():
    """16-bit accesses across the RAM region seams take the generic bus path (K1 pair rule)."""
    from pokegym_amd.testrom.fuzz import boundary_rom
    assert check(boundary_rom(), 8, 2, 9) == []


@pytest.mark.parametrize("seed", [2, 13, 40])
def test_hostsim_fuzz_64_banks(seed):
    """1 MiB fuzz cartridges: code and data in the 58 switchable banks K1 does not stage in LDS
    (global-ROM fetch and read paths)."""
    assert check(fuzz_rom(seed, n_banks=64), 8, 3, seed) == []


def test_hostsim_game_64_banks():
    """pkbench on the 64-bank layout (overworld engine in 60 banks behind Bankswitch trampolines)."""
    assert check(game_rom(64), 8, 8, 5) == []


@pytest.mark.parametrize("n_banks", [2, 64])
def test_hostsim_hram_code(n_banks):
    """Code fetched from inside, across and outside the LDS-mirrored HRAM bytes, self-modified by
    8- and 16-bit writes; 64 banks: the unstaged-bank instance (branch-free write stage)."""
    from pokegym_amd.testrom.fuzz import hram_code_rom
    assert check(hram_code_rom(n_banks), 8, 3, 5) == []


@pytest.mark.parametrize("n_banks", [2, 64])
def test_hostsim_io_edges(n_banks):
    """DIV / JOYP reads and sound / JOYP writes — served first inside K1's rare branches — beside
    16-bit and read-modify-write accesses at the same addresses (pokegym_amd/testrom/fuzz.py
    io_edge_rom); 64 banks: the unstaged-bank instance."""
    from pokegym_amd.testrom.fuzz import io_edge_rom
    assert check(io_edge_rom(n_banks), 8, 3, 7) == []


@pytest.mark.parametrize("n_banks", [8, 64])
def test_hostsim_irq_bank(n_banks):
    """IF / IE writes (K1's cached pending-interrupt bit) and ROM-bank switches issued from code in
    the switchable bank (K1's prefetch across a slow write) — pokegym_amd/testrom/fuzz.py
    irq_bank_rom; the loop-top invariant checks (pk_check_lane) run on every iteration."""
    from pokegym_amd.testrom.fuzz import irq_bank_rom
    assert check(irq_bank_rom(n_banks), 8, 3, 13) == []


def test_hostsim_vram_midframe():
    """VRAM / OAM / SCY / LCDC writes in the middle of the visible frame, at rows the pending (latched,
    not yet rasterised) lines show and rows they do not (fuzz.py vram_midframe_rom): K1 flushes only
    before writes that would change a pending line (pk_step.hip pend_hit); screens vs the oracle."""
    from pokegym_amd.testrom.fuzz import vram_midframe_rom
    assert check(vram_midframe_rom(), 32, 6, 17) == []


def test_hostsim_dma_wait_loop():
    """pokered's OAM-DMA wait loop (dec a / jr nz), which K1 runs in whole passes at once
    (pk_step.hip pk_dec_loop): from HRAM and ROM, A = 0 / 1 / any, carry in or out, timer on/off,
    STAT / VBlank / timer interrupts dispatching inside the loop (fuzz.py dma_wait_rom); whole state
    vs the oracle.  The fast path must have run: the host simulation's trace holds its skip records."""
    import ctypes
    import numpy as np
    from pokegym_amd.testrom.fuzz import dma_wait_rom
    from tests.hostsim import sim
    from tests.hostsim.sim import SimEmulator
    rom = dma_wait_rom()
    assert check(rom, 32, 4, 23) == []
    L = sim.lib()
    L.pk_sim_trace_enable.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    L.pk_sim_trace_get.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    L.pk_sim_trace_get.restype = ctypes.c_uint64
    cap = 1 << 20
    L.pk_sim_trace_enable(0, cap)
    emu = SimEmulator(rom, 1)
    for t in range(2):
        emu.step(np.array([t], np.uint8))
    buf = np.zeros((cap, 6), np.uint32)
    k = L.pk_sim_trace_get(buf.ctypes.data, cap)
    L.pk_sim_trace_enable(0xFFFFFFFF, 0)
    skips = buf[:k][(buf[:k, 4] & 0x1FFF) == 0x1002]
    assert len(skips) > 0 and skips[:, 1].sum() > 100


def test_hostsim_frame_watchdog():
    """The frame watchdog: LCD switched off faster than once per frame (its clock restarts, so
    frames end on the budget), joypad-dependent passes, timer stretches with TIMA interrupts
    (pokegym_amd/testrom/fuzz.py lcd_toggle_rom).  K1 folds the budget into its tick limit."""
    from pokegym_amd.testrom.fuzz import lcd_toggle_rom
    assert check(lcd_toggle_rom(), 8, 2, 11) == []


@pytest.mark.parametrize("name", ["game", "fuzz3", "lcdtoggle"])
def test_hostsim_instr_count(name):
    """pk_last_instr_count (K1's per-env instruction counter: fused pairs, skipped CopyData / LY-poll
    passes, interrupt dispatch and idle iterations excluded) == the oracle's executed instructions,
    step by step."""
    import numpy as np
    from pokegym_amd.testrom.fuzz import fuzz_rom, lcd_toggle_rom
    from pokegym_amd.testrom.game import game_rom
    from tests.hostsim.sim import SimEmulator
    rom = {"game": game_rom, "fuzz3": lambda: fuzz_rom(3), "lcdtoggle": lcd_toggle_rom}[name]()
    acts = np.random.default_rng(5).integers(0, 9, size=(3, 8), dtype=np.uint8)
    emu = SimEmulator(rom, 8)
    got = []
    for t in range(acts.shape[0]):
        emu.step(acts[t])
        got.append(emu.last_instr_count())
    emu.close()
    assert got == OP.instr_counts(rom, acts)


def test_hostsim_map_load_warp():
    """pkbench's door warp (LCD off for ~5 frames of bulk VRAM/WRAM copies) from the fixture state
    (tests/golden/warp_state.npz, tools/make_golden_warp.py)."""
    import numpy as np
    from oracle import oracle
    from tests.hostsim.sim import SimEmulator
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "warp_state.npz"))
    state = d["state"].tobytes()
    n = 4
    acts = np.random.default_rng(5).integers(0, 9, size=(len(d["actions"]), n), dtype=np.uint8)
    acts[:, :2] = d["actions"][:, None]
    rom = game_rom()
    emu = SimEmulator(rom, n, state=state)
    for t in range(len(acts)):
        emu.step(acts[t])
    ref, _ = oracle.batch_run(rom, state, acts, want_screens=False)
    bad = [e for e in range(n) if emu.snapshot(e) != ref[e].tobytes()]
    assert not bad, bad
    # the recorded envs did warp: wMapSeed (0xD4A1, v9 WRAM at 101285) moved on from its boot value
    assert ref[0][101285 + 0x14A1] != 0x5A


def test_hostsim_copydata_block_path():
    """CopyData (pokered home/copy.asm) and its B/C twin, which K1 runs in blocks of whole passes:
    ROM/WRAM/VRAM sources, VRAM/WRAM/overlapping/HRAM/OAM destinations, interrupts and the timer
    landing inside copies, LCD-off copies (pokegym_amd/testrom/fuzz.py copydata_rom)."""
    from pokegym_amd.testrom.fuzz import copydata_rom
    assert check(copydata_rom(), 16, 4, 7) == []


@pytest.mark.parametrize("lanes", ["16", "32"])
def test_hostsim_small_lds_kernel(lanes, monkeypatch):
    """The small-LDS K1 (pk_step.hip compiled a second time with PK_K1_SMALL, as build.py does: 2
    staged banks, the HRAM mirror of 128 envs, 256-thread workgroups) forced on the launch: pkbench's
    bank 3 from the global ROM, mirror columns up to 127 (128 envs per workgroup at 32 envs per wave)."""
    monkeypatch.setenv("PK_K1_SMALL", "1")
    monkeypatch.setenv("PK_WAVE_LANES", lanes)
    monkeypatch.setenv("PK_K1_BLOCK", "256")
    assert check(game_rom(), 128, 2, 48 + int(lanes)) == []

