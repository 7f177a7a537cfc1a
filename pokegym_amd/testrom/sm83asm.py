"""A small two-pass SM83 (Game Boy CPU) assembler.

Used to build the synthetic ROMs the tests and bench run (the real pokemon_red.gb is not part
of this repository).  Syntax (one statement per line, ';' comments):

    section N            ; switch to ROM bank N (bank 0 = 0x0000-0x3FFF, N>0 = 0x4000-0x7FFF)
    org $0150            ; set the address inside the current bank
    label:               ; global label;  .loop: local label (scoped to the last global label)
    NAME equ expr        ; constant
    db 1, $02, "txt"     ; bytes;  dw $1234  ; words;  ds 16 [, fill]
    ld a, [hl+]          ; instructions in RGBDS-like syntax ([...] = memory operand)

Expressions are Python expressions over symbols with `$hex`, `%bin` and `0x..` literals.
"""
from __future__ import annotations

import re

R8 = {"b": 0, "c": 1, "d": 2, "e": 3, "h": 4, "l": 5, "[hl]": 6, "a": 7}
R16 = {"bc": 0, "de": 1, "hl": 2, "sp": 3}
R16STK = {"bc": 0, "de": 1, "hl": 2, "af": 3}
CC = {"nz": 0, "z": 1, "nc": 2, "c": 3}
ALU = {"add": 0, "adc": 1, "sub": 2, "sbc": 3, "and": 4, "xor": 5, "or": 6, "cp": 7}
CBROT = {"rlc": 0, "rrc": 1, "rl": 2, "rr": 3, "sla": 4, "sra": 5, "swap": 6, "srl": 7}
SIMPLE = {"nop": 0x00, "halt": 0x76, "di": 0xF3, "ei": 0xFB, "daa": 0x27, "cpl": 0x2F,
          "scf": 0x37, "ccf": 0x3F, "rlca": 0x07, "rla": 0x17, "rrca": 0x0F, "rra": 0x1F,
          "reti": 0xD9}


class AsmError(Exception):
    pass


def _split_operands(s: str):
    out, depth, cur, q = [], 0, "", False
    for ch in s:
        if ch == '"':
            q = not q
        if not q and ch in "([":
            depth += 1
        if not q and ch in ")]":
            depth -= 1
        if ch == "," and depth == 0 and not q:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


class Assembler:
    def __init__(self, n_banks: int = 2):
        self.n_banks = n_banks
        self.rom = bytearray(b"\xff" * (0x4000 * n_banks))
        self.symbols: dict[str, int] = {}
        self.consts: dict[str, int] = {}

    # -- expressions --------------------------------------------------------------------
    def _expr(self, e: str, final: bool, scope: str) -> int:
        e = e.strip()
        e = re.sub(r"\$([0-9a-fA-F]+)", r"0x\1", e)
        e = re.sub(r"%([01]+)", r"0b\1", e)

        def loc(m):
            return scope + m.group(0)

        e = re.sub(r"(?<![\w.])\.[A-Za-z_]\w*", loc, e)
        names = dict(self.consts)
        names.update(self.symbols)
        tokens = re.findall(r"(?<![\w.])[A-Za-z_][\w.]*", e)
        env = {}
        for t in tokens:
            if t in names:
                env[t.replace(".", "__dot__")] = names[t]
            elif not final:
                env[t.replace(".", "__dot__")] = 0
            else:
                raise AsmError(f"undefined symbol {t!r} in {e!r}")
        e2 = re.sub(r"(?<![\w.])[A-Za-z_][\w.]*", lambda m: m.group(0).replace(".", "__dot__"), e)
        try:
            return int(eval(e2, {"__builtins__": {}}, env))
        except Exception as exc:  # noqa: BLE001
            raise AsmError(f"bad expression {e!r}: {exc}") from exc

    # -- encoding -----------------------------------------------------------------------
    def _encode(self, mn: str, ops: list[str], pc: int, final: bool, scope: str) -> bytes:
        lo = [o.lower().replace(" ", "") for o in ops]
        X = lambda s: self._expr(s, final, scope)  # noqa: E731

        def mem(o):
            return o.startswith("[") and o.endswith("]")

        def n8(v):
            if final and not (-128 <= v <= 255):
                raise AsmError(f"byte out of range: {v}")
            return v & 0xFF

        def n16(v):
            if final and not (-32768 <= v <= 0xFFFF):
                raise AsmError(f"word out of range: {v}")
            return bytes([v & 0xFF, (v >> 8) & 0xFF])

        if mn in SIMPLE and not ops:
            return bytes([SIMPLE[mn]])
        if mn == "stop":
            return b"\x10\x00"
        if mn == "ret":
            if not ops:
                return b"\xc9"
            return bytes([0xC0 | (CC[lo[0]] << 3)])
        if mn == "jp":
            if lo == ["hl"] or lo == ["[hl]"]:
                return b"\xe9"
            if len(ops) == 2:
                return bytes([0xC2 | (CC[lo[0]] << 3)]) + n16(X(ops[1]))
            return b"\xc3" + n16(X(ops[0]))
        if mn == "jr":
            tgt = X(ops[-1])
            off = tgt - (pc + 2)
            if final and not (-128 <= off <= 127):
                raise AsmError(f"jr out of range ({off})")
            if len(ops) == 2:
                return bytes([0x20 | (CC[lo[0]] << 3), off & 0xFF])
            return bytes([0x18, off & 0xFF])
        if mn == "call":
            if len(ops) == 2:
                return bytes([0xC4 | (CC[lo[0]] << 3)]) + n16(X(ops[1]))
            return b"\xcd" + n16(X(ops[0]))
        if mn == "rst":
            v = X(ops[0])
            return bytes([0xC7 | (v & 0x38)])
        if mn in ("push", "pop"):
            base = 0xC5 if mn == "push" else 0xC1
            return bytes([base | (R16STK[lo[0]] << 4)])
        if mn in ("inc", "dec"):
            o = lo[0]
            if o in R16:
                return bytes([(0x03 if mn == "inc" else 0x0B) | (R16[o] << 4)])
            return bytes([(0x04 if mn == "inc" else 0x05) | (R8[o] << 3)])
        if mn in ALU:
            if mn == "add" and lo[0] == "hl":
                return bytes([0x09 | (R16[lo[1]] << 4)])
            if mn == "add" and lo[0] == "sp":
                return bytes([0xE8, n8(X(ops[1]))])
            src = lo[-1]
            if len(lo) == 2 and lo[0] != "a":
                raise AsmError(f"bad {mn} operands {ops}")
            if src in R8:
                return bytes([0x80 | (ALU[mn] << 3) | R8[src]])
            return bytes([0xC6 | (ALU[mn] << 3), n8(X(ops[-1]))])
        if mn in CBROT:
            return bytes([0xCB, (CBROT[mn] << 3) | R8[lo[0]]])
        if mn in ("bit", "res", "set"):
            b = X(ops[0])
            base = {"bit": 0x40, "res": 0x80, "set": 0xC0}[mn]
            return bytes([0xCB, base | ((b & 7) << 3) | R8[lo[1]]])
        if mn == "ldh":
            d, s = lo
            if d == "[c]" or d == "[$ff00+c]":
                return b"\xe2"
            if s == "[c]" or s == "[$ff00+c]":
                return b"\xf2"
            if mem(d) and s == "a":
                v = X(ops[0][1:-1])
                return bytes([0xE0, v & 0xFF])
            if d == "a" and mem(s):
                v = X(ops[1][1:-1])
                return bytes([0xF0, v & 0xFF])
            raise AsmError(f"bad ldh {ops}")
        if mn in ("ld", "ldi", "ldd"):
            d, s = lo
            if mn == "ldi":
                d = "[hl+]" if d == "[hl]" else d
                s = "[hl+]" if s == "[hl]" else s
            if mn == "ldd":
                d = "[hl-]" if d == "[hl]" else d
                s = "[hl-]" if s == "[hl]" else s
            d = {"[hli]": "[hl+]", "[hld]": "[hl-]"}.get(d, d)
            s = {"[hli]": "[hl+]", "[hld]": "[hl-]"}.get(s, s)
            if d in R8 and s in R8:
                if d == "[hl]" and s == "[hl]":
                    raise AsmError("ld [hl],[hl] is halt")
                return bytes([0x40 | (R8[d] << 3) | R8[s]])
            if d == "a" and s in ("[bc]", "[de]", "[hl+]", "[hl-]"):
                return bytes([{"[bc]": 0x0A, "[de]": 0x1A, "[hl+]": 0x2A, "[hl-]": 0x3A}[s]])
            if s == "a" and d in ("[bc]", "[de]", "[hl+]", "[hl-]"):
                return bytes([{"[bc]": 0x02, "[de]": 0x12, "[hl+]": 0x22, "[hl-]": 0x32}[d]])
            if d == "[c]":
                return b"\xe2"
            if s == "[c]":
                return b"\xf2"
            if d == "sp" and s == "hl":
                return b"\xf9"
            if d == "hl" and s.startswith("sp+") or d == "hl" and s.startswith("sp-"):
                return bytes([0xF8, n8(X(ops[1].replace(" ", "")[2:]))])
            if d in R16 and not mem(s):
                return bytes([0x01 | (R16[d] << 4)]) + n16(X(ops[1]))
            if mem(d) and s == "sp":
                return b"\x08" + n16(X(ops[0][1:-1]))
            if mem(d) and s == "a":
                return b"\xea" + n16(X(ops[0][1:-1]))
            if d == "a" and mem(s):
                return b"\xfa" + n16(X(ops[1][1:-1]))
            if d in R8 and not mem(s) or d == "[hl]":
                return bytes([0x06 | (R8[d] << 3), n8(X(ops[1]))])
            raise AsmError(f"bad ld {ops}")
        raise AsmError(f"unknown instruction {mn} {ops}")

    # -- driver -------------------------------------------------------------------------
    def _pass(self, lines: list[str], final: bool):
        bank, addr = 0, 0
        scope = ""
        for lineno, raw in enumerate(lines, 1):
            line = raw.split(";", 1)[0].rstrip()
            if not line.strip():
                continue
            try:
                m = re.match(r"^\s*([.A-Za-z_][\w.]*):(.*)$", line)
                if m:
                    name = m.group(1)
                    if name.startswith("."):
                        name = scope + name
                    else:
                        scope = name
                    base = 0 if bank == 0 else 0x4000
                    val = base + addr
                    if not final and name in self.symbols and self._seen.get(name):
                        raise AsmError(f"duplicate label {name}")
                    self.symbols[name] = val
                    self._seen[name] = True
                    line = m.group(2)
                    if not line.strip():
                        continue
                m = re.match(r"^\s*([A-Za-z_]\w*)\s+equ\s+(.*)$", line, re.I)
                if m:
                    self.consts[m.group(1)] = self._expr(m.group(2), final, scope)
                    continue
                parts = line.strip().split(None, 1)
                mn = parts[0].lower()
                rest = parts[1] if len(parts) > 1 else ""
                ops = _split_operands(rest)
                if mn == "section":
                    bank, addr = self._expr(ops[0], True, scope), 0
                    continue
                if mn == "org":
                    a = self._expr(ops[0], True, scope)
                    addr = a if bank == 0 else a - 0x4000
                    continue
                if mn == "db":
                    data = bytearray()
                    for o in ops:
                        if o.startswith('"'):
                            data += o[1:-1].encode("latin-1")
                        else:
                            data.append(self._expr(o, final, scope) & 0xFF)
                elif mn == "dw":
                    data = bytearray()
                    for o in ops:
                        v = self._expr(o, final, scope)
                        data += bytes([v & 0xFF, (v >> 8) & 0xFF])
                elif mn == "ds":
                    n = self._expr(ops[0], True, scope)
                    fill = self._expr(ops[1], True, scope) if len(ops) > 1 else 0
                    data = bytes([fill & 0xFF]) * n
                else:
                    pc = (0 if bank == 0 else 0x4000) + addr
                    data = self._encode(mn, ops, pc, final, scope)
                if addr + len(data) > 0x4000:
                    raise AsmError("bank overflow")
                if final:
                    off = bank * 0x4000 + addr
                    self.rom[off:off + len(data)] = data
                addr += len(data)
            except AsmError as e:
                raise AsmError(f"line {lineno}: {raw.strip()!r}: {e}") from None

    def assemble(self, src: str) -> bytearray:
        lines = src.splitlines()
        self._seen = {}
        self._pass(lines, final=False)
        self._seen = {}
        self._pass(lines, final=True)
        return self.rom


def build_rom(src: str, n_banks: int = 4, title: str = "PKGPU", cart_type: int = 0x13) -> bytes:
    """Assemble `src` and fill in a cartridge header (MBC3+RAM+BATTERY by default, like Red)."""
    a = Assembler(n_banks)
    rom = a.assemble(src)
    t = title.encode()[:15]
    rom[0x134:0x134 + len(t)] = t
    rom[0x147] = cart_type
    rom[0x148] = {2: 0, 4: 1, 8: 2, 16: 3, 32: 4, 64: 5, 128: 6}[n_banks]
    rom[0x149] = 0x03  # 32 KiB SRAM
    chk = 0
    for i in range(0x134, 0x14D):
        chk = (chk - rom[i] - 1) & 0xFF
    rom[0x14D] = chk
    g = sum(rom) - rom[0x14E] - rom[0x14F]
    rom[0x14E], rom[0x14F] = (g >> 8) & 0xFF, g & 0xFF
    rom_bytes = bytes(rom)
    build_rom.symbols = dict(a.symbols)
    return rom_bytes
