"""SM83 (Game Boy CPU) instruction semantics as the published CPU documentation states them (Pan
Docs, "CPU Instruction Set"; the GBCPUman flag tables) — TEST INFRASTRUCTURE ONLY.

An independent statement of what each tested instruction does to A, F (Z N H C in bits 7-4, the low
nibble always 0), HL and SP, written from the documentation, not from PyBoy or from
oracle/gbcore.c.  tests/test_sm83_kat.py runs pokegym_amd/testrom/kat.py's known-answer ROM on the
oracle (and on the HIP kernel) and compares its per-block checksums with the ones computed here, so
the oracle's per-instruction semantics are pinned to the documented CPU, not only to the builder's
own restatement of PyBoy (PyBoy itself is absent, so CPU trajectories stay unpinned).
"""
from __future__ import annotations

Z, N, H, C = 0x80, 0x40, 0x20, 0x10


def _f(z, n, h, c):
    return (Z if z else 0) | (N if n else 0) | (H if h else 0) | (C if c else 0)


def alu(op: str, a: int, v: int, cy: int):
    """8-bit ALU A,v with carry-in cy: (A', F')."""
    if op == "add":
        r = a + v
        return r & 0xFF, _f((r & 0xFF) == 0, 0, (a & 0xF) + (v & 0xF) > 0xF, r > 0xFF)
    if op == "adc":
        r = a + v + cy
        return r & 0xFF, _f((r & 0xFF) == 0, 0, (a & 0xF) + (v & 0xF) + cy > 0xF, r > 0xFF)
    if op in ("sub", "cp"):
        r = a - v
        res = (r & 0xFF, _f((r & 0xFF) == 0, 1, (a & 0xF) < (v & 0xF), a < v))
        return (a, res[1]) if op == "cp" else res
    if op == "sbc":
        r = a - v - cy
        return r & 0xFF, _f((r & 0xFF) == 0, 1, (a & 0xF) < (v & 0xF) + cy, a < v + cy)
    if op == "and":
        r = a & v
        return r, _f(r == 0, 0, 1, 0)
    if op == "xor":
        r = a ^ v
        return r, _f(r == 0, 0, 0, 0)
    if op == "or":
        r = a | v
        return r, _f(r == 0, 0, 0, 0)
    raise ValueError(op)


def inc_dec(op: str, a: int, f: int):
    """INC A / DEC A: carry kept."""
    if op == "inc":
        r = (a + 1) & 0xFF
        return r, _f(r == 0, 0, (a & 0xF) == 0xF, f & C)
    r = (a - 1) & 0xFF
    return r, _f(r == 0, 1, (a & 0xF) == 0, f & C)


def daa(a: int, f: int):
    """DAA after an addition (N clear) or a subtraction (N set), Pan Docs' statement."""
    n, h, c = f & N, f & H, f & C
    if not n:
        if c or a > 0x99:
            a += 0x60
            c = 1
        if h or (a & 0x0F) > 0x09:
            a += 0x06
    else:
        if c:
            a -= 0x60
        if h:
            a -= 0x06
    a &= 0xFF
    return a, _f(a == 0, n, 0, c)


def cb_rot(op: str, a: int, cy: int):
    """CB-prefixed rotate/shift/swap on A: Z from the result, N = H = 0."""
    if op == "rlc":
        c = a >> 7
        r = ((a << 1) | c) & 0xFF
    elif op == "rrc":
        c = a & 1
        r = (a >> 1) | (c << 7)
    elif op == "rl":
        c = a >> 7
        r = ((a << 1) | cy) & 0xFF
    elif op == "rr":
        c = a & 1
        r = (a >> 1) | (cy << 7)
    elif op == "sla":
        c = a >> 7
        r = (a << 1) & 0xFF
    elif op == "sra":
        c = a & 1
        r = (a >> 1) | (a & 0x80)
    elif op == "swap":
        c = 0
        r = ((a << 4) | (a >> 4)) & 0xFF
    elif op == "srl":
        c = a & 1
        r = a >> 1
    else:
        raise ValueError(op)
    return r, _f(r == 0, 0, 0, c)


def acc_rot(op: str, a: int, cy: int):
    """RLCA / RRCA / RLA / RRA: as the CB forms, but Z always clear."""
    r, f = cb_rot({"rlca": "rlc", "rrca": "rrc", "rla": "rl", "rra": "rr"}[op], a, cy)
    return r, f & ~Z & 0xFF


def bit(b: int, a: int, f: int):
    return a, _f(not ((a >> b) & 1), 0, 1, f & C)


def misc(op: str, a: int, f: int):
    """CPL / SCF / CCF: Z kept."""
    if op == "cpl":
        return a ^ 0xFF, (f & (Z | C)) | N | H
    if op == "scf":
        return a, (f & Z) | C
    if op == "ccf":
        return a, (f & Z) | (0 if f & C else C)
    raise ValueError(op)


def add_hl(hl: int, rr: int, f: int):
    """ADD HL,rr: Z kept, N = 0, H from bit 11, C from bit 15."""
    r = hl + rr
    return r & 0xFFFF, (f & Z) | (H if (hl & 0xFFF) + (rr & 0xFFF) > 0xFFF else 0) | (C if r > 0xFFFF else 0)


def sp_plus(sp: int, e: int):
    """ADD SP,e and LD HL,SP+e: result, F = 0 | H / C from the unsigned low-byte sum."""
    se = e - 256 if e & 0x80 else e
    r = (sp + se) & 0xFFFF
    return r, (H if (sp & 0xF) + (e & 0xF) > 0xF else 0) | (C if (sp & 0xFF) + (e & 0xFF) > 0xFF else 0)


class Fletcher:
    """The ROM's running hash (pokegym_amd/testrom/kat.py acc1): h = rotl16(h, 5) + byte, mod 2^16;
    pair() = (low byte, high byte) as the ROM stores them."""

    def __init__(self):
        self.h = 0

    def add(self, *bs):
        for b in bs:
            self.h = ((((self.h << 5) | (self.h >> 11)) & 0xFFFF) + b) & 0xFFFF

    def pair(self):
        return self.h & 0xFF, self.h >> 8
