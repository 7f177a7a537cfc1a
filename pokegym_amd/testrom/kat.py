"""Known-answer ROM for SM83 instruction semantics (TEST CONTENT).

Each block runs one instruction (or one family) over exhaustive or tabulated inputs — every A and
operand with carry clear and set for the eight 8-bit ALU ops, every A x flag nibble for DAA / CPL /
SCF / CCF, every A x carry for INC / DEC and the rotates / shifts / SWAP / BIT, 65,536 HL x BC pairs
for ADD HL,BC, 16 SP values x every e for ADD SP,e and LD HL,SP+e — and folds every result (A, F,
HL or SP) into a running 16-bit hash (h = rotl16(h, 5) + byte), stored at wOut + 2 * block.
tests/sm83_spec.py states what the documented CPU produces for the same sequence; the tests
compare the two for the oracle (tests/test_sm83_kat.py) and for the HIP kernel.

At boot the ROM reads the joypad: a pressed button selects one group of blocks (group = the JOYP
bit of that button, GROUP_ACTION maps it to a pokegym action), none runs them all.  wDone is set
when the selected blocks are finished; the CPU then spins."""
from __future__ import annotations

from .sm83asm import build_rom

ALU_OPS = ("add", "adc", "sub", "sbc", "and", "xor", "or", "cp")
CB_OPS = ("rlc", "rrc", "rl", "rr", "sla", "sra", "swap", "srl")
ACC_OPS = ("rlca", "rrca", "rla", "rra")
MISC_OPS = ("cpl", "scf", "ccf")
SP_VALUES = (0x0000, 0x000F, 0x00F0, 0x00FF, 0x0F0F, 0x7FFF, 0x8000, 0xFFF0, 0xFFFF, 0x1234, 0xFEDC, 0x00F8,
             0x0008, 0x0088, 0xFF80, 0xC0FF)
W_S1, W_S2, W_GRP, W_DONE, W_SP, W_OUT = 0xC000, 0xC001, 0xC003, 0xC002, 0xC004, 0xC010
# JOYP bit of a pressed button (ROM's group bit) -> pokegym action (pyboy_binding.py ACTIONS order:
# Down Left Right Up A B Start Select)
GROUP_ACTION = {0: 2, 1: 1, 2: 3, 3: 0, 4: 4, 5: 5, 6: 7, 7: 6}

# (block name, group bit); names are what tests/sm83_spec.py computes expectations for
BLOCKS = ([(f"alu_{op}", g) for g, op in enumerate(ALU_OPS)]
          + [("incdec", 0), ("daa", 1), ("bit", 2), ("misc", 3), ("accrot", 4), ("add_hl", 5)]
          + [(f"cb_{op}", 2 + (k % 6)) for k, op in enumerate(CB_OPS)]
          + [("add_sp", 6), ("ld_hl_sp", 7)])


def _next_d(stride: int) -> list[str]:
    """d += stride while it stays below 256 (stride 1: every value)"""
    return ["inc d", "jr nz, .la"] if stride == 1 else ["ld a, d", f"add a, {stride}", "ld d, a", "jr nc, .la"]


def _block(k: int, name: str, grp: int, stride: int = 1) -> list[str]:
    out = W_OUT + 2 * k
    L = [f"blk_{k}:", f"ld a, [${W_GRP:04x}]", "and a", f"jr z, .run", f"and ${1 << grp:02x}", f"jp z, blk_{k + 1}",
         ".run:", "xor a", f"ld [${W_S1:04x}], a", f"ld [${W_S2:04x}], a"]
    if name.startswith("alu_"):
        op = name[4:]
        L += ["ld d, 0", ".la:", "ld e, 0", ".lb:",
              "ld a, d", "scf", "ccf", f"{op} a, e", "call accaf",
              "ld a, d", "scf", f"{op} a, e", "call accaf",
              "inc e", "jr nz, .lb"] + _next_d(stride)
    elif name == "incdec":
        L += ["ld d, 0", ".la:"]
        for op in ("inc", "dec"):
            L += ["ld a, d", "scf", "ccf", f"{op} a", "call accaf", "ld a, d", "scf", f"{op} a", "call accaf"]
        L += _next_d(stride)
    elif name in ("daa", "misc"):
        ops = ["daa"] if name == "daa" else list(MISC_OPS)
        L += ["ld d, 0", ".la:", "ld e, 0", ".lb:"]
        for op in ops:
            L += ["ld a, e", "swap a", "ld l, a", "ld h, d", "push hl", "pop af", op, "call accaf"]
        L += ["inc e", "ld a, e", "cp 16", "jr nz, .lb"] + _next_d(stride)
    elif name.startswith("cb_") or name == "accrot":
        ops = [name[3:]] if name.startswith("cb_") else list(ACC_OPS)
        L += ["ld d, 0", ".la:"]
        for op in ops:
            src = f"{op} a" if name.startswith("cb_") else op
            L += ["ld a, d", "scf", "ccf", src, "call accaf", "ld a, d", "scf", src, "call accaf"]
        L += _next_d(stride)
    elif name == "bit":
        L += ["ld d, 0", ".la:"]
        for b in range(8):
            L += ["ld a, d", "scf", "ccf", f"bit {b}, a", "call accaf", "ld a, d", "scf", f"bit {b}, a", "call accaf"]
        L += _next_d(stride)
    elif name == "add_hl":
        # H = d, L = e, B = d ^ $5a, C = 3e; the xor leaves Z = (B == 0), N = H = C = 0
        L += ["ld d, 0", ".la:", "ld e, 0", ".lb:",
              "ld a, e", "add a, a", "add a, e", "ld c, a", "ld a, d", "xor $5a", "ld b, a",
              "ld h, d", "ld l, e", "add hl, bc", "call acchlf",
              "inc e", "jr nz, .lb"] + _next_d(stride)
    elif name in ("add_sp", "ld_hl_sp"):
        L += [f"call sp_{name}"]
    L += [f"ld a, [${W_S1:04x}]", f"ld [${out:04x}], a", f"ld a, [${W_S2:04x}]", f"ld [${out + 1:04x}], a"]
    return L


def _sp_routine(name: str) -> list[str]:
    # for each SP value (table), each e unrolled: SP = value; op; result and F into the checksum.
    # The real stack is at $dfea here (below $dff0: the routine's return address and the two pushes
    # below), restored after every test.
    L = [f"sp_{name}:", "ld hl, sp_table", "ld b, 16", ".ls:", "ld a, [hl+]", "ld e, a", "ld a, [hl+]", "ld d, a",
         "push hl", "push bc"]
    for e in range(256):
        if name == "add_sp":
            L += ["ld h, d", "ld l, e", "ld sp, hl", f"add sp, {e}", f"ld [${W_SP:04x}], sp", "ld sp, $dfea",
                  "call accspf"]
        else:
            L += ["ld h, d", "ld l, e", "ld sp, hl", f"ld hl, sp+{e}", "ld sp, $dfea", "call acchlf"]
    L += ["pop bc", "pop hl", "dec b", "jp nz, .ls", "ret"]
    return L


def kat_rom(stride: int = 1) -> bytes:
    """stride > 1: the A / H values of the looped blocks step by `stride` (0, stride, ... < 256) — a
    shorter run for the kernels' own checks (the oracle test runs stride 1: every value)."""
    L = [f"wS1 equ ${W_S1:04x}", f"wS2 equ ${W_S2:04x}",
         "section 0", "org $0040", "reti", "org $0048", "reti", "org $0050", "reti", "org $0058", "reti", "org $0060", "reti",
         "org $0100", "nop", "jp start", "org $0150",
         "start:", "di", "ld sp, $dff0", "xor a", "ldh [$ff], a", f"ld [${W_DONE:04x}], a",
         # the pressed button's JOYP bit: directions in bits 0-3, buttons in bits 4-7 (1 = pressed)
         "ld a, $20", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]", "cpl", "and $0f", "ld b, a",
         "ld a, $10", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]", "cpl", "and $0f", "swap a", "or b",
         f"ld [${W_GRP:04x}], a"]
    for k, (name, grp) in enumerate(BLOCKS):
        L += _block(k, name, grp, stride)
    L += [f"blk_{len(BLOCKS)}:", "ld a, 1", f"ld [${W_DONE:04x}], a", "spin:", "jr spin",
          # hash helpers (d, e, b, c kept)
          # acc1: h = rotl16(h, 5) + a over the 16-bit state wS2:wS1 (a plain byte sum, or h * 33 + a,
          # lets the same flag-bit difference in thousands of regularly spaced cases cancel out;
          # tests/test_sm83_kat.py checks that ten single-rule changes of the statement each change it)
          "acc1:", "push bc", "push hl", "ld c, a", "ld a, [wS1]", "ld l, a", "ld a, [wS2]", "ld h, a"]
    L += ["add hl, hl", "ld a, l", "adc a, 0", "ld l, a"] * 5
    L += ["ld b, 0", "add hl, bc", "ld a, l", "ld [wS1], a", "ld a, h", "ld [wS2], a", "pop hl", "pop bc", "ret",
          "accaf:", "push af", "pop hl", "ld a, h", "call acc1", "ld a, l", "call acc1", "ret",          # A, F
          "acchlf:", "push hl", "push af", "pop hl", "ld a, l", "call acc1", "pop hl", "ld a, l", "call acc1",
          "ld a, h", "call acc1", "ret",                                                              # F, L, H
          "accspf:", "push af", "pop hl", "ld a, l", "call acc1", f"ld a, [${W_SP:04x}]", "call acc1",
          f"ld a, [${W_SP + 1:04x}]", "call acc1", "ret",                                              # F, SP lo, hi
          "section 1", "org $4000", "sp_table:", "dw " + ", ".join(f"${v:04x}" for v in SP_VALUES)]
    L += _sp_routine("add_sp") + _sp_routine("ld_hl_sp")
    return build_rom("\n".join(L), n_banks=2, title="SM83KAT")
