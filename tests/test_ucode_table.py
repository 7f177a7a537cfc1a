"""The microcode tables K1 reads (pk_ucode.h), checked on the host: compiled with g++ from the
unmodified header, no GPU.  The secondary-op table has one entry per opcode; PK_U2_NONE = 0xFF is
both RST 38h's entry and the index every primary that may not fuse selects for its successor, so
K1's correctness rests on that entry being empty (length 0: no secondary op) and on every
PK_DB_NOFUSE primary's successor selector producing 0xFF whatever its instruction bytes."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "pokegym_amd", "csrc")

PROG = r"""
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include "pk_ucode.h"
// v_perm_b32 semantics for the selector bytes the tables use: 0-7 pick a byte of hi:lo, 12 = 0x00,
// 13 and up = 0xFF
static uint32_t vperm(uint32_t hi, uint32_t lo, uint32_t s) {
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int k = 0; k < 4; k++) {
        const uint32_t b = (s >> (8 * k)) & 0xFFu;
        const uint32_t x = b < 8 ? (uint32_t)((v >> (8 * b)) & 0xFFu) : b == 12 ? 0u : b >= 13 ? 0xFFu : 0xEEu;
        r |= x << (8 * k);
    }
    return r;
}
int main() {
    std::vector<uint32_t> t(PK_UC_WORDS);
    pk_build_ucode(t.data());
    const uint32_t* none = t.data() + PK_UC_U2 + (size_t)PK_U2_NONE * PK_U2_WORDS;
    printf("none_len %u\n", none[1] & 3u);
    unsigned nofuse = 0, bad = 0;
    for (int i = 0; i < 512; i++) {
        const uint32_t* e = t.data() + (size_t)i * PK_UE_WORDS;
        if (!(e[PK_UE_D] & (1u << PK_DB_NOFUSE))) continue;
        nofuse++;
        const uint32_t probes[3] = {0x12345678u, 0x00000000u, 0xFFFFFFFEu};
        for (uint32_t b : probes) bad += (vperm(b, b, e[PK_UE_V]) & 0xFFu) != PK_U2_NONE;
    }
    printf("nofuse %u bad %u\n", nofuse, bad);
    // cycles: base and extra-when-taken of every primary entry (V word, T-states), then the
    // secondary-op table's length and cycles per opcode
    for (int i = 0; i < 512; i++) {
        const uint32_t v = t[(size_t)i * PK_UE_WORDS + PK_UE_V];
        printf("cyc%d %u\n", i, ((v >> 16) & 0xFFu) | (((v >> 24) & 0xFFu) << 8));
    }
    for (int op = 0; op < 256; op++) {
        const uint32_t y = t[PK_UC_U2 + (size_t)op * PK_U2_WORDS + 1];
        printf("u2_%d %u\n", op, (y & 3u) | (((y >> PK_U2B_CYC) & 15u) << 8));
    }
    return 0;
}
"""


@pytest.fixture(scope="module")
def table_report(tmp_path_factory):
    d = tmp_path_factory.mktemp("ucode")
    src, exe = d / "t.cpp", d / "t"
    src.write_text(PROG)
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", CSRC, "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    return dict(zip(out[0::2], map(int, out[1::2])))


def test_u2_none_entry_is_empty(table_report):
    assert table_report["none_len"] == 0


def test_nofuse_primaries_select_the_empty_entry(table_report):
    assert table_report["nofuse"] >= 40 and table_report["bad"] == 0


def test_cycles_match_the_documented_cpu(table_report):
    """Every primary microcode entry's cycles (V word: base, + extra when the condition holds) and
    every secondary op's cycles (the fused successor; JR not taken — taken adds 4 in pk_step.hip)
    == the published opcode timing (tests/sm83_spec.py cycles / cb_cycles)."""
    from tests import sm83_spec as S
    bad = []
    for op in range(256):
        doc = S.cycles(op)
        if doc is None:
            continue
        v = table_report[f"cyc{op}"]
        base, extra = v & 0xFF, v >> 8
        if (base, base + extra) != doc:
            bad.append((f"{op:02X}", (base, base + extra), doc))
        u2 = table_report[f"u2_{op}"]
        if u2 & 3:
            c2 = u2 >> 8
            # a fused JR: the table holds the not-taken cycles, a taken one (JR e always) adds 4
            jr = op in (0x18, 0x20, 0x28, 0x30, 0x38)
            if (jr and (c2 + 4 != doc[1] or (op != 0x18 and c2 != doc[0]))) or (not jr and c2 != doc[0]):
                bad.append((f"u2 {op:02X}", c2, doc))
    for op in range(256):
        v = table_report[f"cyc{256 + op}"]
        if (v & 0xFF, v >> 8) != (S.cb_cycles(op), 0):
            bad.append((f"CB {op:02X}", (v & 0xFF, v >> 8), S.cb_cycles(op)))
    assert not bad, bad[:10]
