"""Seeded random SM83 programs for kernel-vs-oracle parity ("fuzz ROMs").

Each ROM boots (post-boot state, PC=0x100), installs interrupt handlers for VBlank, STAT, timer
and joypad, enables a random IE subset / TAC / STAT sources, copies an OAM-DMA stub to HRAM, and
then loops forever over a few hundred random instruction blocks.  The blocks cover every legal
opcode class: 8/16-bit loads (all addressing modes), ALU (reg, (HL), imm), INC/DEC, all CB ops,
rotates, DAA/CPL/SCF/CCF, PUSH/POP, ADD SP,e / LD HL,SP+e / LD (nn),SP, JR/JP/CALL/RET/RST
(conditional and not), RETI via the handlers, HALT, DI/EI, MBC3 ROM/SRAM bank switching, OAM DMA,
LCD on/off, scroll/palette/window writes (visible in the rendered frame), joypad reads (so each
env's action stream changes its control flow), DIV/TIMA/LY/STAT reads.
"""
from __future__ import annotations

import random

from .sm83asm import build_rom

R8 = ["b", "c", "d", "e", "h", "l", "a"]
ALU = ["add", "adc", "sub", "sbc", "and", "xor", "or", "cp"]
CB = ["rlc", "rrc", "rl", "rr", "sla", "sra", "swap", "srl"]
CC = ["nz", "z", "nc", "c"]
IO_W = [0x42, 0x43, 0x47, 0x48, 0x49, 0x4A, 0x4B, 0x45, 0x41, 0x05, 0x06, 0x01, 0x02, 0x90]
IO_R = [0x44, 0x41, 0x04, 0x05, 0x0F, 0x40, 0x42, 0x00, 0x47, 0x4A, 0xFF, 0x10, 0x26, 0x07]


def _hl_anchor(rng: random.Random) -> str:
    return f"ld hl, ${0xC000 + rng.randrange(0x0800, 0x1800):04x}"


def _block(rng: random.Random, idx: int, n_banks: int, max_n: int = 14) -> list[str]:
    out = []
    for _ in range(rng.randint(min(4, max_n), max_n)):
        k = rng.random()
        r = rng.choice(R8)
        if k < 0.10:
            out.append(f"ld {r}, ${rng.randrange(256):02x}")
        elif k < 0.17:
            out.append(f"ld {rng.choice(R8)}, {rng.choice(R8)}")
        elif k < 0.27:
            op = rng.choice(ALU)
            src = rng.choice(R8 + ["imm", "[hl]"])
            if src == "imm":
                out.append(f"{op} a, ${rng.randrange(256):02x}")
            elif src == "[hl]":
                out += [_hl_anchor(rng), f"{op} a, [hl]"]
            else:
                out.append(f"{op} a, {src}")
        elif k < 0.32:
            out.append(f"{rng.choice(['inc', 'dec'])} {rng.choice(R8)}")
        elif k < 0.36:
            out += [_hl_anchor(rng), f"{rng.choice(['inc', 'dec'])} [hl]"]
        elif k < 0.42:
            t = rng.choice(R8 + ["[hl]"])
            pre = [_hl_anchor(rng)] if t == "[hl]" else []
            g = rng.random()
            if g < 0.4:
                out += pre + [f"{rng.choice(CB)} {t}"]
            else:
                out += pre + [f"{rng.choice(['bit', 'res', 'set'])} {rng.randrange(8)}, {t}"]
        elif k < 0.45:
            out.append(rng.choice(["rlca", "rla", "rrca", "rra", "daa", "cpl", "scf", "ccf"]))
        elif k < 0.48:
            out += ["add a, $19" if rng.random() < 0.5 else "sub $27", "daa"]
        elif k < 0.53:
            out += [_hl_anchor(rng), rng.choice(["ld [hl+], a", "ld [hl-], a", "ld a, [hl+]", "ld a, [hl-]",
                                               f"ld [hl], ${rng.randrange(256):02x}", f"ld [hl], {rng.choice(R8[:4] + ['a'])}",
                                               f"ld {rng.choice(R8[:4] + ['a'])}, [hl]"])]
        elif k < 0.56:
            p = rng.choice(["bc", "de"])
            out += [f"ld {p}, ${0xC000 + rng.randrange(0x800, 0x1800):04x}", f"ld [{p}], a" if rng.random() < 0.5 else f"ld a, [{p}]"]
        elif k < 0.59:
            a = 0xC000 + rng.randrange(0x800, 0x1800)
            out.append(f"ld [${a:04x}], a" if rng.random() < 0.5 else f"ld a, [${a:04x}]")
        elif k < 0.62:
            p = rng.choice(["bc", "de", "hl"])
            out.append(rng.choice([f"ld {p}, ${rng.randrange(65536):04x}", f"inc {p}", f"dec {p}", f"add hl, {p}"]))
        elif k < 0.64:
            out += ["add hl, sp", f"ld hl, sp+{rng.randrange(-128, 128)}", "inc sp", "dec sp"]
        elif k < 0.66:
            e = rng.randrange(1, 100)
            out += [f"add sp, {e}", f"add sp, {-e}"]
        elif k < 0.67:
            out.append(f"ld [${0xC000 + rng.randrange(0x800, 0x1800):04x}], sp")
        elif k < 0.71:
            p1, p2 = rng.choice(["bc", "de", "hl", "af"]), rng.choice(["bc", "de", "hl", "af"])
            out += [f"push {p1}", f"pop {p2}"]
        elif k < 0.74:
            out.append(f"call {'' if rng.random() < 0.5 else rng.choice(CC) + ', '}sub{rng.randrange(8)}")
        elif k < 0.76:
            out.append(f"rst ${rng.choice([0x08, 0x10, 0x18, 0x20, 0x28, 0x30]):02x}")
        elif k < 0.79:
            lbl = f"skip_{idx}_{len(out)}"
            out += [f"jr {rng.choice(CC)}, {lbl}", f"inc {rng.choice(R8)}", f"{lbl}:"]
        elif k < 0.81:
            lbl = f"skip_{idx}_{len(out)}"
            out += [f"jp {rng.choice(CC)}, {lbl}", f"dec {rng.choice(R8)}", f"{lbl}:"]
        elif k < 0.84:
            io = rng.choice(IO_W)
            v = rng.randrange(256)
            if io == 0x41:
                v &= 0x78
            out += [f"ld a, ${v:02x}", f"ldh [${io:02x}], a"]
        elif k < 0.88:
            io = rng.choice(IO_R)
            if io == 0x00:
                out += [f"ld a, ${rng.choice([0x10, 0x20, 0x30, 0x00]):02x}", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]"]
            else:
                out.append(f"ldh a, [${io:02x}]")
            if rng.random() < 0.5:
                lbl = f"jj_{idx}_{len(out)}"
                out += [f"bit {rng.randrange(8)}, a", f"jr z, {lbl}", f"inc {rng.choice(['b', 'c', 'd', 'e'])}", f"{lbl}:"]
        elif k < 0.89:
            out += [f"ld c, ${rng.choice(IO_R):02x}", "ld a, [c]" if rng.random() < 0.5 else "ld [c], a"]
            if out[-1] == "ld [c], a":
                out[-2] = f"ld c, ${rng.choice([0x42, 0x43, 0x47, 0x4a, 0x90]):02x}"
        elif k < 0.905:
            out.append("halt")
        elif k < 0.915:
            out.append(rng.choice(["di", "ei", "ei"]))
        elif k < 0.93:
            b = rng.randrange(1, n_banks)
            out += [f"ld a, ${b:02x}", "ld [$2100], a", f"call ${0x4000 + 0x10 * rng.randrange(4):04x}"]
        elif k < 0.945:
            out += ["ld a, $0a", "ld [$0000], a", f"ld a, ${rng.randrange(4):02x}", "ld [$4000], a",
                    f"ld hl, ${0xA000 + rng.randrange(0x2000):04x}", rng.choice(["ld [hl], b", "ld a, [hl]", "inc [hl]"])]
            if rng.random() < 0.3:
                out += ["xor a", "ld [$0000], a", "ld a, [hl]"]
        elif k < 0.955:
            out += [f"ld a, ${rng.choice([0xC1, 0xC2, 0xC0, 0x80, 0x00, 0xFE]):02x}", "call $ff80"]
        elif k < 0.96:
            out.append("nop")
        elif k < 0.975:
            out += [f"ld a, ${rng.randrange(256):02x}", f"ldh [${rng.choice([0x07, 0x06, 0x05, 0x04]):02x}], a"]
        else:
            out.append(f"ld {rng.choice(['bc', 'de'])}, ${rng.randrange(65536):04x}")
    return out


def fuzz_source(seed: int, n_blocks: int = 160, n_banks: int = 8) -> str:
    rng = random.Random(seed)
    L = ["section 0"]
    for v in range(8):
        L += [f"org ${v * 8:04x}", "inc e" if v else "nop", "ret"]
    L += ["org $0040", "jp vblank", "org $0048", "jp stat", "org $0050", "jp timer",
          "org $0058", "reti", "org $0060", "jp joyp"]
    L += ["org $0100", "nop", "jp start", "org $0150"]
    L += ["start:", "di", "ld sp, $dff0",
          # copy the DMA stub to HRAM (pokered's WriteDMACodeToHRAM)
          "ld hl, dma_stub", "ld de, $ff80", "ld b, 10", ".cp:", "ld a, [hl+]", "ld [de], a", "inc de",
          "dec b", "jr nz, .cp",
          f"ld a, ${rng.choice([0x01, 0x03, 0x05, 0x07, 0x11, 0x15, 0x17, 0x1F]):02x}", "ldh [$ff], a",
          f"ld a, ${rng.choice([0x00, 0x04, 0x05, 0x06, 0x07]):02x}", "ldh [$07], a",
          f"ld a, ${rng.randrange(154):02x}", "ldh [$45], a",
          f"ld a, ${rng.choice([0x00, 0x08, 0x20, 0x40, 0x48, 0x10]):02x}", "ldh [$41], a",
          "ld a, $e3", "ldh [$40], a", "ld a, $e4", "ldh [$47], a", "ld a, $d0", "ldh [$48], a",
          # tiles / map / OAM buffer with some non-zero content so the PPU has work
          "ld hl, $8000", "ld bc, $1800", ".t:", "ld a, l", "xor h", "ld [hl+], a", "dec bc", "ld a, b",
          "or c", "jr nz, .t",
          "ld hl, $c100", "ld b, 160", ".o:", "ld a, l", "add a, b", "ld [hl+], a", "dec b", "jr nz, .o",
          "ei", "main:"]
    for i in range(n_blocks):
        L += _block(rng, i, n_banks)
    L += ["jp main"]
    for s in range(8):
        L += [f"sub{s}:"] + _block(rng, 1000 + s, n_banks, max_n=5) + ["ret"]
    L += ["vblank:", "push af", "push hl", "ld hl, $c0f0", "inc [hl]", "ldh a, [$44]", "ld [$c0f1], a",
          "ld a, $c1", "call $ff80",
          # every 32nd vblank: LCD off for a short while (pokered's DisableLCD/EnableLCD pattern)
          "ld a, [$c0f0]", "and $1f", "jr nz, vb_done", "ldh a, [$40]", "and $7f", "ldh [$40], a",
          "ld h, $20", "vb_wait:", "dec h", "jr nz, vb_wait", "ldh a, [$40]", "or $80", "ldh [$40], a",
          "vb_done:", "pop hl", "pop af", "reti",
          "stat:", "push af", "ldh a, [$41]", "ld [$c0f2], a", "ldh a, [$04]", "ldh [$43], a", "pop af", "reti",
          "timer:", "push af", "ld a, [$c0f3]", "inc a", "ld [$c0f3], a", "pop af", "reti",
          "joyp:", "push af", "ld a, $10", "ldh [$00], a", "ldh a, [$00]", "ld [$c0f4], a", "pop af", "reti",
          "dma_stub:", "db $3e, $c3, $e0, $46, $3e, $28, $3d, $20, $fd, $c9"]
    # the stub writes a fixed page; patch: use A as the page (ld a,N removed): ldh [$46],a ; wait ; ret
    L[-1] = "db $e0, $46, $3e, $28, $3d, $20, $fd, $c9, $00, $00"
    for b in range(1, n_banks):
        L += [f"section {b}"]
        for j in range(4):
            L += [f"org ${0x4000 + 0x10 * j:04x}", f"ld a, ${b:02x}", f"add a, {rng.choice(R8)}", f"ld [${0xC080 + b:04x}], a",
                  "ld a, $01", "ld [$2100], a", "ret"]
    return "\n".join(L)


def fuzz_rom(seed: int, n_blocks: int = 160, n_banks: int = 8) -> bytes:
    return build_rom(fuzz_source(seed, n_blocks, n_banks), n_banks=n_banks, title=f"FUZZ{seed}")


def boundary_rom() -> bytes:
    """16-bit accesses straddling the RAM region seams (WRAM/echo at 0xE000, echo/OAM at 0xFE00,
    IO/HRAM at 0xFF80, VRAM/SRAM at 0xA000): PUSH/POP/CALL/RET with SP at the seams, LD (nn),SP
    and LD A,[HL+]/LD [HL-],A over them, with values that change every pass (joypad-dependent)."""
    L = ["section 0"]
    L += ["org $0040", "reti", "org $0048", "reti", "org $0050", "reti", "org $0058", "reti", "org $0060", "reti"]
    L += ["org $0100", "nop", "jp start", "org $0150"]
    L += ["start:", "di", "ld sp, $dff0", "ld a, $e3", "ldh [$40], a", "ld bc, $1234", "ld de, $5678",
          "main:",
          # joypad bits feed the values, so each env's action stream changes them
          "ld a, $10", "ldh [$00], a", "ldh a, [$00]", "add a, c", "ld c, a", "inc b", "inc d", "dec e",
          # SP at the seams: PUSH writes [SP-1], [SP-2]; POP reads [SP], [SP+1]
          "ld hl, $0000", "add hl, sp", "ld sp, $e001", "push bc", "pop de", "push de",
          "ld sp, $fe01", "push bc", "pop hl", "push hl",
          "ld sp, $e000", "call sub_seam",
          "ld sp, $dfff", "pop af", "push af",
          "ld sp, $fdff", "pop bc", "push bc",
          # LD (nn),SP across the seams
          "ld sp, $1357", "ld [$dfff], sp", "ld sp, $2468", "ld [$fdff], sp", "ld sp, $9abc", "ld [$9fff], sp",
          "ld sp, $dff0",
          # [HL+] / [HL-] walking over the seams
          "ld hl, $dffe", "ld a, c", "ld [hl+], a", "ld [hl+], a", "ld [hl+], a",
          "ld hl, $fdfe", "ld a, e", "ld [hl+], a", "ld [hl+], a", "ld a, [hl-]", "ld a, [hl-]", "ld c, a",
          "ld hl, $ff7f", "ld a, [hl+]", "ld a, b", "ld [hl-], a", "ld a, [hl]",
          "ld hl, $c000", "ld a, [$dfff]", "ld [hl+], a", "ld a, [$e000]", "ld [hl+], a",
          "ld a, [$fdff]", "ld [hl+], a", "ld a, [$fe00]", "ld [hl+], a", "ld a, [$ff80]", "ld [hl+], a",
          "jp main",
          "sub_seam:", "ld a, d", "ld [$dffd], a", "ret"]
    return build_rom("\n".join(L), n_banks=2, title="SEAMS")


def hram_code_rom(n_banks: int = 2) -> bytes:
    """Code run from all over HRAM: K1 fetches HRAM code from an LDS mirror of 0xFF80-0xFF9F only
    (where games keep the OAM-DMA routine) and from the RAM image elsewhere.  Routines sit inside
    the mirror (0xFF90), across its end (0xFF98-0xFF9F: the RET is fetched from the image),
    outside it (0xFFB0, 0xFFC0) and at the top of HRAM (0xFFF6: the RET's fetch reaches IE at
    0xFFFF); two of them are rewritten every pass with joypad-dependent immediates, and the
    mirrored loop's jr offset by a push (self-modifying HRAM code: the mirror must follow 8- and
    16-bit writes).  n_banks = 64: the same code on a cartridge K1 cannot stage whole (the
    unstaged-bank instance and its branch-free write stage)."""
    loop = "$04, $78, $81, $4f, $15, $20, $f9, $c9"        # inc b; ld a,b; add a,c; ld c,a; dec d; jr nz,-7; ret
    imm = "$3e, $00, $80, $47, $c9"                          # ld a,N; add a,b; ld b,a; ret
    L = ["section 0", "org $0040", "reti", "org $0048", "reti", "org $0050", "reti", "org $0058", "reti",
         "org $0060", "reti", "org $0100", "nop", "jp start", "org $0150",
         "start:", "di", "ld sp, $dff0"]
    for src, dst, n in (("r_imm", 0xFF90, 5), ("r_loop", 0xFF98, 8), ("r_loop", 0xFFB0, 8), ("r_imm", 0xFFC0, 5),
                        ("r_loop", 0xFFF6, 8)):
        lbl = f"cp_{dst:04x}"
        L += [f"ld hl, {src}", f"ld de, ${dst:04x}", f"ld b, {n}", f"{lbl}:", "ld a, [hl+]", "ld [de], a", "inc de",
              "dec b", f"jr nz, {lbl}"]
    L += ["ld a, $e3", "ldh [$40], a", "ld bc, $0102",
          "main:",
          "ld a, $10", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]", "add a, c", "ld e, a",
          "ldh [$91], a",                        # rewrite the mirrored routine's immediate
          "and $01", "add a, $f9", "ld h, a", "ld l, $20",   # and the loop's jr nz + offset (-7 / -6)
          "ld sp, $ff9f", "push hl", "ld sp, $dff0",          # by a push (the offset is its 2nd byte)
          "ld a, e",
          "xor $5a", "ldh [$c1], a",             # and the unmirrored one's
          "call $ff90", "ld d, 3", "call $ff98", "call $ffc0", "ld d, 2", "call $ffb0",
          "ld a, e", "and $03", "inc a", "ld d, a", "call $fff6",
          "ld a, b", "ld [$c000], a", "ld a, c", "ld [$c001], a",
          "jp main",
          "r_loop:", f"db {loop}", "r_imm:", f"db {imm}"]
    return build_rom("\n".join(L), n_banks=n_banks, title="HRAMCODE")


def io_edge_rom(n_banks: int = 2) -> bytes:
    """The IO accesses K1 serves first inside its rare branches (pk_step.hip: one-byte DIV and JOYP
    reads, one-byte sound and JOYP writes) beside the forms that must still take the general bus:
    16-bit reads and writes at the same addresses (pop / push / ld [a16],sp, one of each across
    the sound block's end into LCDC), read-modify-write instructions on DIV, JOYP and NR52,
    [c]-relative and absolute addressing, a JOYP select that changes every pass and a DIV reset
    every 8th pass.  Every value read is summed into WRAM each pass (so a wrong read in any pass
    shows in the final image), and the last pass's values stay at 0xC010-0xC022."""
    L = ["section 0", "org $0040", "reti", "org $0048", "reti", "org $0050", "reti", "org $0058", "reti",
         "org $0060", "reti", "org $0100", "nop", "jp start", "org $0150",
         "start:", "di", "ld sp, $dff0", "ld a, $e3", "ldh [$40], a", "ld b, 0",
         "ld a, $05", "ldh [$07], a",                               # the timer runs (TIMA next to DIV)
         "main:",
         # JOYP: the select bits change per pass; one-byte reads by ldh, [c] and through HL
         "ld a, b", "swap a", "and $30", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]", "ld e, a",
         "ld [$c010], a", "call acc",
         "ld a, b", "or $a5", "ldh [$01], a",                      # SB: JOYP's neighbour in a 16-bit read
         "ld a, $20", "ldh [$00], a", "ld c, $00", "ldh a, [c]", "ld [$c011], a", "call acc",
         "ld hl, $ff00", "set 4, [hl]", "ld a, [hl]", "ld [$c012], a", "call acc",
         # DIV: ldh, absolute and HL reads; a reset by a read-modify-write every 8th pass
         "ldh a, [$04]", "ld [$c013], a", "call acc",
         "ld a, [$ff04]", "ld [$c014], a", "call acc",
         "ld hl, $ff04", "ld a, [hl]", "ld [$c015], a", "call acc",
         "ld a, b", "and $07", "jr nz, .nodiv", "inc [hl]", ".nodiv:",
         # sound (not emulated): one-byte writes and reads, a read-modify-write of NR52
         "ld a, e", "ldh [$24], a", "ldh [$25], a", "ld [$ff30], a", "ldh [$3f], a",
         "ldh a, [$25]", "ld [$c016], a", "call acc",
         "ldh a, [$30]", "ld [$c017], a", "call acc",
         "ld hl, $ff26", "inc [hl]", "ld a, [hl]", "ld [$c018], a", "call acc",
         # 16-bit accesses: a push into NR10/NR11, pops across FF03/DIV and DIV/TIMA, JOYP/SB and NR52's block end
         # into LCDC, and ld [a16],sp across FF3F/LCDC (SP's high byte lands in LCDC, read back, restored)
         "ld d, b", "ld sp, $ff12", "push de", "ld sp, $ff03", "pop hl", "ld sp, $ff00", "pop de",
         "ld sp, $ff3f", "pop bc", "ld sp, $e7e0", "ld [$ff3f], sp", "ld sp, $dff0",
         "ldh a, [$40]", "ld [$c01e], a", "call acc", "ld a, $e3", "ldh [$40], a",
         "ld a, l", "ld [$c019], a", "call acc", "ld a, h", "ld [$c01a], a", "call acc",
         "ld a, e", "ld [$c01b], a", "call acc", "ld a, d", "ld [$c01c], a", "call acc",
         "ld a, c", "ld [$c01d], a", "call acc", "ld a, b", "call acc",
         "ld sp, $ff04", "pop hl", "ld sp, $dff0",                 # DIV + TIMA as one 16-bit read
         "ld a, l", "ld [$c021], a", "call acc", "ld a, h", "ld [$c022], a", "call acc",
         "ld a, [$c020]", "inc a", "ld [$c020], a", "ld b, a",
         "jp main",
         "acc:", "push hl", "ld hl, $c01f", "add a, [hl]", "ld [hl], a", "pop hl", "ret"]
    return build_rom("\n".join(L), n_banks=n_banks, title="IOEDGE")


def irq_bank_rom(n_banks: int = 8) -> bytes:
    """Two paths whose effect K1 caches in lane state instead of re-deriving it every iteration
    (pk_step.hip pk_check_lane): (1) IF and IE writes — K1 keeps "an interrupt is pending" as a bit
    of its cpu word, updated wherever IE or IF change — with IME off, read back, then a short IME-on
    window (ei / nop / nop / di) in which whatever the writes left pending dispatches, the timer
    raising its own IF bit meanwhile in half of the passes; (2) ROM-bank switches issued from code IN the switchable bank:
    every bank holds the same routine at 0x4000 that writes the next bank number to the MBC and
    continues at the next address — fetched from the NEW bank, whose immediate differs — so a fetch
    prefetched from the old bank before the switch would show in WRAM (K1 refetches after a slow
    write).  n_banks 8: the switch goes between LDS-staged banks and (small-LDS kernel) global-ROM
    ones; 64: mostly between unstaged banks.  Handler counts, IF read-backs and the per-bank sums
    stay in WRAM 0xC020-0xC04F."""
    L = ["section 0",
         "org $0040", "jp h_0", "org $0048", "jp h_1", "org $0050", "jp h_2", "org $0058", "jp h_3", "org $0060", "jp h_4",
         "org $0100", "nop", "jp start", "org $0150",
         "start:", "di", "ld sp, $dff0", "ld a, $e3", "ldh [$40], a",
         "main:",
         "ld a, [$c030]", "inc a", "ld [$c030], a", "ld b, a",
         # the timer runs in every other stretch of 8 passes (TAC 5 / 1): with it on, K1 takes its
         # timer stage — which re-derives the pending bit — every iteration
         "and $08", "rrca", "or $01", "ldh [$07], a",
         # the joypad mixes into the masks, so envs differ
         "ld a, $10", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]", "xor b", "ld e, a",
         "and $1f", "ldh [$ff], a",                       # IE
         "ld a, e", "rrca", "and $1f", "ldh [$0f], a",    # IF (IME off: nothing dispatches yet)
         "ldh a, [$0f]", "ld [$c031], a",
         "ld hl, $ff0f", "set 2, [hl]", "res 0, [hl]",    # read-modify-writes of IF
         "ldh a, [$0f]", "ld [$c032], a",
         "ei", "nop", "nop", "di",                        # the pending ones dispatch here
         "ld a, e", "and $03", "jr nz, .keep", "xor a", "ldh [$0f], a", ".keep:",
         "ld a, $1f", "ldh [$ff], a", "xor a", "ldh [$ff], a",  # IE on and off again with IF as it is
         "ld a, 1", "ld [$2000], a", "ld a, e", "and $07", "inc a", "ld c, a", "call $4000",
         "jp main"]
    for k in range(5):
        L += [f"h_{k}:", "push af", f"ld a, [${0xC040 + k:04x}]", "inc a", f"ld [${0xC040 + k:04x}], a", "pop af", "reti"]
    for k in range(1, n_banks):
        nxt = (k * 5) % (n_banks - 1) + 1
        L += [f"section {k}", "org $4000", f"hop_{k}:",
              "ld hl, $c020", "ld a, [hl]", f"add a, ${(k * 13) & 0xFF:02x}", "ld [hl], a",
              f"ld a, {nxt}", "ld [$2000], a",            # switch from inside the switchable bank
              f"ld b, ${(k * 29 + 7) & 0xFF:02x}",        # fetched from bank `nxt`: its own immediate
              "ld a, [$c021]", "add a, b", "ld [$c021], a",
              "dec c", f"jr nz, hop_{k}", "ret"]
    return build_rom("\n".join(L), n_banks=n_banks, title="IRQBANK")


def dma_wait_rom() -> bytes:
    """pokered's OAM-DMA wait loop (`dec a / jr nz,-3`), which K1 runs in whole passes at once
    (pk_step.hip pk_dec_loop): from HRAM (where pokered's hDMARoutine runs it) and from ROM, with A
    from the joypad and a pass counter (0 = 256 passes and 1 = none to skip included), carry set or
    clear on entry (the loop keeps it), the timer on in half of the stretches, STAT mode-0 and
    VBlank interrupts enabled or not and IME on or off — interrupts dispatch inside the loop, their
    handlers keep A and F.  After each loop A, F and the handler counts go into WRAM 0xC030-0xC04F."""
    L = ["section 0",
         "org $0040", "jp h_0", "org $0048", "jp h_1", "org $0050", "jp h_2",
         "org $0100", "nop", "jp start", "org $0150",
         "start:", "di", "ld sp, $dff0", "ld a, $e3", "ldh [$40], a",
         "ld hl, rom_wait", "ld de, $ff80", "ld b, 4",
         ".cp:", "ld a, [hl+]", "ld [de], a", "inc de", "dec b", "jr nz, .cp",
         "main:",
         "ld a, [$c030]", "inc a", "ld [$c030], a", "ld b, a",
         "and $08", "rrca", "or $01", "ldh [$07], a",            # timer on (TAC 5) / off (TAC 1)
         "ld a, b", "and $10", "rrca", "ldh [$41], a",           # STAT mode-0 interrupt on / off
         "ld a, b", "and $07", "or $01", "ldh [$ff], a",         # IE: VBlank, + STAT, + timer
         "ld a, $10", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]", "xor b", "ld c, a",
         "ld a, b", "and $20", "jr z, .di", "ei", "jr .go", ".di:", "di", ".go:",
         "ld a, b", "and $07", "jr nz, .ab",
         "ld a, b", "and $08", "jr .set",                         # A = 0 (256 passes) or 8
         ".ab:", "ld a, c", "swap a", "xor b",
         ".set:", "ld d, a",
         "ld a, b", "rrca", "jr c, .sc", "and a", "ld a, d", "jr .call", ".sc:", "ld a, d", "scf",
         ".call:", "bit 6, b", "jr z, .hram",
         "call rom_wait", "jr .done",
         ".hram:", "call $ff80",
         ".done:", "push af", "pop hl", "di",
         "ld a, h", "ld [$c031], a", "ld a, l", "ld [$c032], a",
         "ld a, [$c033]", "add a, l", "ld [$c033], a",
         "ld a, d", "ld [$c034], a",
         "jp main",
         "rom_wait:", "db $3d, $20, $fd, $c9"]
    for k in range(3):
        L += [f"h_{k}:", "push af", f"ld a, [${0xC040 + k:04x}]", "inc a", f"ld [${0xC040 + k:04x}], a", "pop af", "reti"]
    return build_rom("\n".join(L), n_banks=2, title="DMAWAIT")


def vram_midframe_rom() -> bytes:
    """VRAM and OAM writes in the middle of the visible frame — what K1's deferred rasteriser must
    get right: a line is latched at its mode-0 event and rasterised later (K2 at the step's end, or
    flush_lines before a write that would change it: pk_step.hip pend_hit).  Each pass waits (LY
    poll) for a joypad- and pass-dependent line T, then writes one of: a BG-map byte in the row the
    line just above T shows (pending: must flush) or in a row further down (not yet latched: no
    flush; about ten writes a frame), a window-map byte in the window's current row or another, a tile-data byte of a tile the
    maps use, an OAM byte of a visible sprite, SCY (later lines show other rows), LCDC's BG-map
    select (the other map's rows), or a BG-map byte of the map not shown; BG, window (WY 72, WX 47)
    and ten 8x8 sprites are on, so every kind of read a line makes is covered."""
    L = ["wPass equ $c0f0", "wT equ $c0f1",
         "section 0", "org $0040", "reti", "org $0048", "reti", "org $0050", "reti", "org $0058", "reti", "org $0060", "reti",
         "org $0100", "nop", "jp start", "org $0150",
         "start:", "di", "ld sp, $dff0", "xor a", "ldh [$40], a",
         # tiles 0-15: byte k of tile t = t * 17 ^ k * 29; BG map 9800: (row * 3 + col) & 15; map 9C00: (row + 5 * col) & 15
         "ld hl, $8000", "ld b, 0", ".t:", "ld a, b", "swap a", "add a, b", "ld c, a", "ld a, l", "and $0f", "ld e, a",
         "add a, a", "add a, e", "ld e, a", "add a, a", "add a, a", "add a, a", "add a, e", "sub e", "xor c", "ld [hl+], a",
         "ld a, l", "and $0f", "jr nz, .t", "inc b", "ld a, b", "cp 16", "jr nz, .t",
         "ld hl, $9800", ".m:", "ld a, h", "sub $98", "ld d, a", "ld a, l", "and $1f", "ld e, a",
         "ld a, l", "swap a", "rrca", "and $07", "ld c, a", "ld a, d", "add a, a", "add a, a", "add a, a", "add a, c",
         "ld c, a", "add a, a", "add a, c", "add a, e", "and $0f", "ld [hl+], a", "ld a, h", "cp $9c", "jr nz, .m",
         ".w9c:", "ld a, l", "and $1f", "ld e, a", "add a, a", "add a, a", "add a, e", "ld e, a", "ld a, l", "swap a",
         "rrca", "and $07", "add a, e", "add a, h", "and $0f", "ld [hl+], a", "ld a, h", "cp $a0", "jr nz, .w9c",
         # OAM: sprite n at y = 16 + 13 n, x = 8 + 15 n, tile n, attribute 0 / $20 / $80 by n
         "ld hl, $fe00", "ld b, 0", ".o:", "ld a, b", "add a, a", "add a, a", "add a, a", "add a, b", "add a, b",
         "add a, b", "add a, b", "add a, b", "add a, 16", "ld [hl+], a", "ld a, b", "swap a", "sub b", "add a, 8",
         "ld [hl+], a", "ld a, b", "ld [hl+], a", "ld a, b", "and $03", "rrca", "rrca", "rrca", "ld [hl+], a",
         "inc b", "ld a, b", "cp 10", "jr nz, .o",
         ".oz:", "xor a", "ld [hl+], a", "ld a, l", "cp $a0", "jr nz, .oz",
         "ld a, 72", "ldh [$4a], a", "ld a, 47", "ldh [$4b], a", "ld a, $e4", "ldh [$47], a", "ld a, $d2", "ldh [$48], a",
         "ld a, $f3", "ldh [$40], a",                         # LCD on, window map 9C00, tile data 8000, BG map 9800
         "main:",
         "ld a, $10", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]", "and $0f", "ld e, a",
         "ld a, [wPass]", "inc a", "ld [wPass], a", "ld b, a",
         # the next line: 5..20 lines after the last one (about ten writes a frame), wrapping below 140
         "ld a, e", "and $07", "add a, a", "add a, 5", "ld d, a", "ld a, [wT]", "add a, d", "cp 140", "jr c, .tok",
         "sub 131", ".tok:", "ld [wT], a", "ld d, a",
         ".ly:", "ldh a, [$44]", "cp d", "jr nz, .ly",
         # the row (T + SCY) / 8 of the line at T
         "ldh a, [$42]", "add a, d", "srl a", "srl a", "srl a", "ld c, a",
         "ld a, b", "and $07", "jr z, .k0", "dec a", "jr z, .k1", "dec a", "jr z, .k2", "dec a", "jr z, .k3",
         "dec a", "jr z, .k4", "dec a", "jr z, .k5", "dec a", "jr z, .k6", "jp .k7",
         ".k0:", "ld a, c", "dec a", "jr .bgrow",                     # the row the line above shows: pending
         ".k1:", "ld a, c", "add a, 3",                               # a row further down: not latched yet
         ".bgrow:", "and $1f", "ld l, a", "ld h, 0", "add hl, hl", "add hl, hl", "add hl, hl", "add hl, hl", "add hl, hl",
         "ld a, b", "and $1f", "add a, l", "ld l, a", "ld a, h", "add a, $98", "ld h, a", "ld a, b", "and $0f", "ld [hl], a",
         "jp main",
         ".k2:", "ld a, d", "sub 72", "jr c, .k2b", "srl a", "srl a", "srl a", "jr .wrow",   # the window's current row
         ".k2b:", "ld a, b", "and $07",
         ".wrow:", "ld l, a", "ld h, 0", "add hl, hl", "add hl, hl", "add hl, hl", "add hl, hl", "add hl, hl",
         "ld a, b", "and $07", "add a, l", "ld l, a", "ld a, h", "add a, $9c", "ld h, a", "ld a, b", "and $0f", "ld [hl], a",
         "jp main",
         ".k3:", "ld a, b", "and $0f", "swap a", "ld l, a", "ld h, $80", "ld a, e", "xor b", "ld [hl], a", "jp main",  # tile data
         ".k4:", "ld a, b", "rrca", "rrca", "rrca", "and $07", "add a, a", "add a, a", "ld l, a", "ld h, $fe",  # OAM y / x
         "ld a, b", "rlca", "rlca", "and $01", "add a, l", "ld l, a", "ld a, [hl]", "xor $05", "ld [hl], a", "jp main",
         ".k5:", "ld a, b", "and $0f", "ldh [$42], a", "jp main",                                   # SCY
         ".k6:", "ldh a, [$40]", "xor $08", "ldh [$40], a", "jp main",                              # BG map select
         ".k7:", "ld a, c", "and $1f", "ld l, a", "ld h, 0", "add hl, hl", "add hl, hl", "add hl, hl", "add hl, hl",
         "add hl, hl", "ld a, h", "add a, $9c", "ld h, a", "ld a, b", "and $0f", "ld [hl], a", "jp main"]   # the other map
    return build_rom("\n".join(L), n_banks=2, title="VRAMMID")


def copydata_rom() -> bytes:
    """pokered's CopyData loop (home/copy.asm) and its B/C-swapped twin — which K1 runs in blocks of
    whole passes (pk_step.hip pk_copy_loop) — called with per-env parameters from the joypad and an
    LFSR: sources in ROM bank 0, the switchable bank, WRAM and VRAM; destinations in VRAM and WRAM,
    overlapping the source either way, and — where the block path must step aside — HRAM and OAM;
    lengths 1..512; the LCD on with the VBlank, STAT (HBlank, some passes) and timer interrupts
    enabled, so interrupts land inside copies; the timer switched on and off; every 16th pass a
    1 KiB ROM-to-VRAM copy with the LCD off (pokered's DisableLCD regime)."""
    L = ["wSeed equ $c0f0", "wPass equ $c0f1", "wVbl equ $c0f2", "wStat equ $c0f3", "wR0 equ $c0f4", "wR1 equ $c0f5",
         "section 0",
         "org $0040", "jp h_vbl", "org $0048", "jp h_stat", "org $0050", "reti", "org $0058", "reti", "org $0060", "reti",
         "org $0100", "nop", "jp start", "org $0150",
         "start:", "di", "ld sp, $dff0",
         "ld a, 1", "ld [$2000], a",                          # MBC3: bank 1 switchable
         "ld a, $5a", "ld [wSeed], a", "xor a", "ld [wPass], a",
         "ld a, $07", "ldh [$ff], a",                         # IE: VBlank, STAT, timer
         "ld a, $e3", "ldh [$40], a", "ei",
         "main:",
         # two LFSR bytes, the joypad mixed in
         "ld a, $20", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]", "ld b, a",
         "ld a, [wSeed]", "xor b", "add a, a", "jr nc, .n1", "xor $1d", ".n1:", "ld [wR0], a",
         "add a, a", "jr nc, .n2", "xor $1d", ".n2:", "ld [wR1], a", "ld [wSeed], a",
         "ld a, [wPass]", "inc a", "ld [wPass], a", "ld d, a",
         # every 8th pass: the timer on or off (TAC 5 / 0); STAT HBlank interrupt on some passes
         "and $07", "jr nz, .t1", "ld a, d", "and $08", "rrca", "or $01", "and $05", "ldh [$07], a", ".t1:",
         "ld a, [wR1]", "and $08", "ldh [$41], a",
         # every 16th pass: 1 KiB ROM -> VRAM with the LCD off
         "ld a, d", "and $0f", "jr nz, .nolcd",
         "xor a", "ldh [$0f], a", "ldh a, [$ff]", "push af", "res 0, a", "ldh [$ff], a",
         ".wly:", "ldh a, [$44]", "cp 145", "jr nz, .wly",
         "ldh a, [$40]", "and $7f", "ldh [$40], a",
         "ld hl, $0000", "ld de, $8800", "ld bc, $0400", "call copy_a",
         "ldh a, [$40]", "or $80", "ldh [$40], a", "xor a", "ldh [$0f], a", "pop af", "ldh [$ff], a",
         ".nolcd:",
         # length: BC = 1..512
         "ld a, [wR0]", "and $01", "ld b, a", "ld a, [wR1]", "ld c, a", "or b", "jr nz, .len", "inc c", ".len:",
         # source (wR0 bits 7-6): ROM bank 0 / bank 1 / WRAM / VRAM, + 8 * (wR1 & $3f)
         "ld a, [wR1]", "and $3f", "ld l, a", "ld h, 0", "add hl, hl", "add hl, hl", "add hl, hl",
         "ld a, [wR0]", "and $c0", "jr nz, .s1", "ld a, $02", "jr .sh", ".s1:",
         "cp $40", "jr nz, .s2", "ld a, $40", "jr .sh", ".s2:",
         "cp $80", "jr nz, .s3", "ld a, $c4", "jr .sh", ".s3:", "ld a, $80", ".sh:",
         "add a, h", "ld h, a",
         # destination (wR0 bits 5-3)
         "ld a, [wR0]", "and $38", "rrca", "rrca", "rrca", "ld e, a",
         "cp 2", "jr nc, .d2", "ld d, $90", "jr .dlow", ".d2:",
         "cp 4", "jr nc, .d4", "ld d, $d0", "jr .dlow", ".d4:",
         "cp 5", "jr nc, .d5", "ld a, l", "add a, 5", "ld e, a", "ld a, h", "adc a, 0", "ld d, a", "jr .dgo", ".d5:",
         "cp 6", "jr nc, .d6", "ld a, l", "sub 7", "ld e, a", "ld a, h", "sbc a, 0", "ld d, a", "jr .dgo", ".d6:",
         # HRAM / OAM: short copies only
         "ld b, 0", "ld a, c", "and $1f", "inc a", "ld c, a",
         "ld a, e", "cp 6", "jr nz, .d7", "ld de, $ff90", "jr .dgo", ".d7:", "ld de, $fe10", "jr .dgo",
         ".dlow:", "ld a, [wR1]", "and $3f", "rlca", "rlca", "ld e, a",
         ".dgo:",
         "ld a, [wR1]", "and $01", "jr nz, .vb", "call copy_a", "jp main", ".vb:", "call copy_b", "jp main",
         "h_vbl:", "push af", "ld a, [wVbl]", "inc a", "ld [wVbl], a", "pop af", "reti",
         "h_stat:", "push af", "ld a, [wStat]", "inc a", "ld [wStat], a", "pop af", "reti",
         "copy_a:", "ld a, [hl+]", "ld [de], a", "inc de", "dec bc", "ld a, c", "or b", "jr nz, copy_a", "ret",
         "copy_b:", "ld a, [hl+]", "ld [de], a", "inc de", "dec bc", "ld a, b", "or c", "jr nz, copy_b", "ret"]
    return build_rom("\n".join(L), n_banks=2, title="COPYDATA")


def lcd_toggle_rom() -> bytes:
    """The frame watchdog (oracle/gbcore.c PK_FRAME_BUDGET; K1 folds it into its tick limit): a
    main loop that switches the LCD on, spins a joypad-dependent count, writes WRAM and switches the
    LCD off again — faster than once per frame, so the LCD clock restarts and no frame ever ends by
    itself; every frame is ended by the budget.  A pass whose joypad read shows Select pressed (bit 2
    low) skips the LCD-off write, and the timer runs in every fourth 256-pass
    stretch (a TIMA interrupt handler counts), so the budget's end meets LCD events, the timer and
    interrupts."""
    L = ["section 0", "org $0040", "reti", "org $0048", "reti",
         "org $0050", "jp timer_isr",
         "org $0058", "reti", "org $0060", "reti", "org $0100", "nop", "jp start", "org $0150",
         "start:", "di", "ld sp, $dff0", "ld a, $04", "ldh [$ff], a", "xor a", "ldh [$06], a", "ei",
         "ld b, 1",
         "main:",
         "ld a, $91", "ldh [$40], a",
         "ld a, $10", "ldh [$00], a", "ldh a, [$00]", "ldh a, [$00]", "ld d, a", "and $0f", "add a, b", "ld c, a",
         ".w:", "dec c", "jr nz, .w",
         "ld a, b", "ld [$c000], a", "ld hl, $c001", "inc [hl]",
         "ld a, d", "and $04", "jr z, .keep",
         "xor a", "ldh [$40], a",
         ".keep:",
         "inc b", "ld a, b", "and a", "jr nz, main",
         # every 256 passes: the timer on for one stretch in four
         "ld hl, $c002", "inc [hl]", "ld a, [hl]", "and $03", "jr nz, .toff",
         "ld a, $05", "ldh [$07], a", "jp main",
         ".toff:", "xor a", "ldh [$07], a", "jp main",
         "timer_isr:", "push af", "ld a, [$c010]", "inc a", "ld [$c010], a", "pop af", "reti"]
    return build_rom("\n".join(L), n_banks=2, title="LCDTOGGLE")
