"""SM83 instruction semantics pinned to the documented CPU (tests/sm83_spec.py): the known-answer
ROM (pokegym_amd/testrom/kat.py) runs every block on the oracle and the block checksums must equal
the ones the documentation's statement gives for the same input sequence.  The oracle is what the
HIP kernels are bit-exact against (test_gpu_parity.py, and the same ROM on the device below), so
this pins their per-instruction results — A, F, HL, SP for the 8-bit ALU (exhaustive), DAA, INC /
DEC, the rotates / shifts / SWAP / BIT, CPL / SCF / CCF, ADD HL,rr and the SP-relative adds — to
the published CPU, independently of PyBoy (absent here: trajectories stay unpinned)."""
import sys

import numpy as np

import pytest

from pokegym_amd.testrom import kat
from tests import sm83_spec as S


def expected(name: str, stride: int = 1):
    f = S.Fletcher()
    ds = range(0, 256, stride)
    if name.startswith("alu_"):
        op = name[4:]
        for d in ds:
            for e in range(256):
                for cy in (0, 1):
                    f.add(*S.alu(op, d, e, cy))
    elif name == "incdec":
        for d in ds:
            for op in ("inc", "dec"):
                for cy in (0, 1):
                    f.add(*S.inc_dec(op, d, S.C if cy else 0))
    elif name == "daa":
        for d in ds:
            for n in range(16):
                f.add(*S.daa(d, n << 4))
    elif name == "misc":
        for d in ds:
            for n in range(16):
                for op in kat.MISC_OPS:
                    f.add(*S.misc(op, d, n << 4))
    elif name.startswith("cb_"):
        for d in ds:
            for cy in (0, 1):
                f.add(*S.cb_rot(name[3:], d, cy))
    elif name == "accrot":
        for d in ds:
            for op in kat.ACC_OPS:
                for cy in (0, 1):
                    f.add(*S.acc_rot(op, d, cy))
    elif name == "bit":
        for d in ds:
            for b in range(8):
                for cy in (0, 1):
                    f.add(*S.bit(b, d, S.C if cy else 0))
    elif name == "add_hl":
        for d in ds:
            for e in range(256):
                b = d ^ 0x5A
                hl, fl = S.add_hl((d << 8) | e, (b << 8) | ((3 * e) & 0xFF), S.Z if b == 0 else 0)
                f.add(fl, hl & 0xFF, hl >> 8)
    elif name in ("add_sp", "ld_hl_sp"):
        for sp in kat.SP_VALUES:
            for e in range(256):
                r, fl = S.sp_plus(sp, e)
                f.add(fl, r & 0xFF, r >> 8)
    return f.pair()


def run_oracle(group=None, max_steps=3000):
    from oracle import oracle as O
    gb = O.GB(kat.kat_rom())
    gb.power_on()
    act = 8 if group is None else kat.GROUP_ACTION[group]
    for _ in range(max_steps):
        gb.run_action(act)
        if gb.read(kat.W_DONE):
            break
    assert gb.read(kat.W_DONE), "the known-answer ROM did not finish"
    return bytes(gb.read(kat.W_OUT + i) for i in range(2 * len(kat.BLOCKS)))


@pytest.fixture(scope="module")
def oracle_out():
    return run_oracle()


@pytest.mark.parametrize("k,name", list(enumerate(n for n, _ in kat.BLOCKS)))
def test_oracle_block_matches_documented_cpu(oracle_out, k, name):
    assert tuple(oracle_out[2 * k:2 * k + 2]) == expected(name), name


def test_group_selection():
    """A pressed button runs only its group's blocks (the GPU test splits the work by action)."""
    out = run_oracle(group=3)
    for k, (name, grp) in enumerate(kat.BLOCKS):
        got = tuple(out[2 * k:2 * k + 2])
        assert got == (expected(name) if grp == 3 else (0xFF, 0xFF)) or (grp != 3 and got == (0, 0)), name


# single-rule changes of the documented statement and the block each must show up in: the ROM's
# hash has to tell them apart (a plain byte sum let regularly spaced flag differences cancel)
MUTATIONS = {
    "alu_adc": ("(a & 0xF) + (v & 0xF) + cy > 0xF", "(a & 0xF) + (v & 0xF) > 0xF"),
    "alu_sbc": ("(a & 0xF) < (v & 0xF) + cy, a < v + cy", "(a & 0xF) < (v & 0xF), a < v + cy"),
    "daa": ("if h or (a & 0x0F) > 0x09:", "if h or (a & 0x0F) > 0x0A:"),
    "add_sp": ("(C if (sp & 0xFF) + (e & 0xFF) > 0xFF else 0)", "(C if (sp + (e - 256 if e & 0x80 else e)) > 0xFFFF else 0)"),
    "bit": ("return a, _f(not ((a >> b) & 1), 0, 1, f & C)", "return a, _f(not ((a >> b) & 1), 0, 1, 0)"),
    "incdec": ("(a & 0xF) == 0xF, f & C)", "(a & 0xF) == 0xE, f & C)"),
    "cb_sra": ("r = (a >> 1) | (a & 0x80)", "r = a >> 1"),
    "add_hl": ("(hl & 0xFFF) + (rr & 0xFFF) > 0xFFF", "(hl & 0xFF) + (rr & 0xFF) > 0xFF"),
    "misc": ("return a, (f & Z) | (0 if f & C else C)", "return a, (f & Z) | (0 if f & C else C) | H"),
    "accrot": ("return r, f & ~Z & 0xFF", "return r, f"),
}


@pytest.mark.parametrize("block", sorted(MUTATIONS))
def test_hash_detects_a_changed_rule(block, monkeypatch):
    import inspect
    import types
    src = inspect.getsource(S)
    a, b = MUTATIONS[block]
    assert src.count(a) == 1
    mutated = types.ModuleType("sm83_spec_mutated")
    exec(compile(src.replace(a, b), "sm83_spec_mutated", "exec"), mutated.__dict__)
    want = expected(block)
    monkeypatch.setattr(sys.modules[__name__], "S", mutated)
    assert expected(block) != want, f"{block}: the hash does not see the change"


def kernel_outputs(rom, states):
    """Per env: (done flag, the block hashes) its kernel run stored, read from the env's v9 state."""
    from oracle import oracle as O
    out = []
    for st in states:
        gb = O.GB(rom)
        gb.load_state(bytes(st))
        out.append((gb.read(kat.W_DONE), bytes(gb.read(kat.W_OUT + i) for i in range(2 * len(kat.BLOCKS)))))
    return out


def check_group_outputs(outs, groups, stride):
    assert all(d for d, _ in outs), "the known-answer ROM did not finish"
    bad = []
    for e, ((_, o), g) in enumerate(zip(outs, groups)):
        for k, (name, grp) in enumerate(kat.BLOCKS):
            if grp == g and tuple(o[2 * k:2 * k + 2]) != expected(name, stride):
                bad.append((e, name))
    return bad


def test_hostsim_kernel_kat():
    """K1 (host-simulation build of pk_step.hip) runs the known-answer ROM, one group per env (the
    A values stepping by 15): every block hash == the documented CPU's (sm83_spec)."""
    from tests.hostsim.sim import SimEmulator
    stride, n = 15, 16
    rom = kat.kat_rom(stride)
    groups = [e % 8 for e in range(n)]
    acts = np.array([kat.GROUP_ACTION[g] for g in groups], np.uint8)
    emu = SimEmulator(rom, n)
    for _ in range(10):
        emu.step(acts)
    states = emu.snapshot_range(0, n)
    emu.close()
    assert check_group_outputs(kernel_outputs(rom, states), groups, stride) == []
