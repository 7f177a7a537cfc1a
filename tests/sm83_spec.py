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


# ---- instruction timing (T-states, Pan Docs / the opcode tables): (not taken, taken) ----
ILLEGAL = {0xD3, 0xDB, 0xDD, 0xE3, 0xE4, 0xEB, 0xEC, 0xED, 0xF4, 0xFC, 0xFD}


def cycles(op: int):
    """T-states of base opcode op as (cycles, cycles when a condition holds) — equal for the
    unconditional ones; None for the illegal opcodes and the CB prefix (see cb_cycles)."""
    if op in ILLEGAL or op == 0xCB:
        return None
    hi, lo = op >> 6, op & 7
    if 0x40 <= op < 0x80:                       # LD r,r' / LD r,(HL) / LD (HL),r / HALT
        if op == 0x76:
            return (4, 4)
        return (8, 8) if (lo == 6 or (op >> 3) & 7 == 6) else (4, 4)
    if 0x80 <= op < 0xC0:                       # ALU A,r / A,(HL)
        return (8, 8) if lo == 6 else (4, 4)
    fixed = {
        0x00: 4, 0x10: 4, 0x76: 4, 0xF3: 4, 0xFB: 4, 0x27: 4, 0x2F: 4, 0x37: 4, 0x3F: 4,
        0x07: 4, 0x0F: 4, 0x17: 4, 0x1F: 4,
        0x02: 8, 0x12: 8, 0x22: 8, 0x32: 8, 0x0A: 8, 0x1A: 8, 0x2A: 8, 0x3A: 8,
        0x08: 20, 0xE0: 12, 0xF0: 12, 0xE2: 8, 0xF2: 8, 0xEA: 16, 0xFA: 16,
        0xF8: 12, 0xF9: 8, 0xE8: 16, 0x36: 12, 0x34: 12, 0x35: 12,
        0xC3: 16, 0xE9: 4, 0x18: 12, 0xCD: 24, 0xC9: 16, 0xD9: 16,
    }
    if op in fixed:
        return (fixed[op], fixed[op])
    if hi == 0:
        if lo == 1:
            return (12, 12) if op & 0x08 == 0 else (8, 8)          # LD rr,nn / ADD HL,rr
        if lo == 3:
            return (8, 8)                                           # INC / DEC rr
        if lo in (4, 5):
            return (4, 4)                                           # INC / DEC r
        if lo == 6:
            return (8, 8)                                           # LD r,n
        if lo == 0 and op in (0x20, 0x28, 0x30, 0x38):
            return (8, 12)                                          # JR cc,e
    if hi == 3:
        if lo == 6:
            return (8, 8)                                           # ALU A,n
        if lo == 7:
            return (16, 16)                                         # RST
        if lo == 5:
            return (16, 16)                                         # PUSH
        if lo == 1:
            return (12, 12)                                         # POP
        if op in (0xC2, 0xCA, 0xD2, 0xDA):
            return (12, 16)                                         # JP cc,nn
        if op in (0xC4, 0xCC, 0xD4, 0xDC):
            return (12, 24)                                         # CALL cc,nn
        if op in (0xC0, 0xC8, 0xD0, 0xD8):
            return (8, 20)                                          # RET cc
    raise KeyError(f"no documented timing for {op:02X}")


def cb_cycles(op: int) -> int:
    """T-states of CB-prefixed op: 8 on a register, 16 on (HL), BIT n,(HL) 12."""
    if op & 7 != 6:
        return 8
    return 12 if 0x40 <= op < 0x80 else 16
