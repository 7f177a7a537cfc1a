// pk_decode.h — builds the 512-entry SM83 decode table (256 base + 256 CB-prefixed opcodes)
// consumed by the step kernel's uniform datapath.  Each descriptor says which memory reads and
// writes the instruction performs and which datapath class computes its result, so every lane
// of a wave runs the same fetch → read → compute → write → tick sequence no matter which
// opcode it holds (divergence is confined to the small class bodies).
//
// Instruction semantics/cycle counts follow the SM83 as PyBoy 1.x's generated opcodes.py
// implements them (restated in the oracle, oracle/gbcore.c:cpu_execute / exec_cb).
#pragma once
#include <stdint.h>

#include "pk_layout.h"

static inline uint32_t pk_desc(uint32_t cls, uint32_t len, uint32_t rd, uint32_t wr, uint32_t a,
                               uint32_t b, uint32_t op, uint32_t cyc, uint32_t xcyc) {
    return cls | (len << 6) | (rd << 8) | (wr << 12) | (a << 16) | (b << 20) | (op << 24) |
           ((cyc / 4) << 27) | ((xcyc / 4) << 30);
}

static inline void pk_build_decode(uint32_t* t /* 512 */) {
    for (int i = 0; i < 512; i++) t[i] = pk_desc(PK_C_ILLEGAL, 1, 0, 0, 0, 0, 0, 4, 0);
    const uint32_t N = PK_M_NONE;
    // ---- 0x00-0x3F ----
    t[0x00] = pk_desc(PK_C_NOP, 1, N, N, 0, 0, 0, 4, 0);
    t[0x10] = pk_desc(PK_C_NOP, 2, N, N, 0, 0, 0, 4, 0);  // STOP: 2-byte no-op on DMG
    for (int p = 0; p < 4; p++) {
        t[0x01 | (p << 4)] = pk_desc(PK_C_LD16, 3, N, N, p, 0, 0, 12, 0);
        t[0x03 | (p << 4)] = pk_desc(PK_C_INC16, 1, N, N, p, 0, 0, 8, 0);
        t[0x0B | (p << 4)] = pk_desc(PK_C_DEC16, 1, N, N, p, 0, 0, 8, 0);
        t[0x09 | (p << 4)] = pk_desc(PK_C_ADDHL, 1, N, N, p, 0, 0, 8, 0);
    }
    t[0x02] = pk_desc(PK_C_LD8, 1, N, PK_M_BC, 6, 7, 0, 8, 0);
    t[0x12] = pk_desc(PK_C_LD8, 1, N, PK_M_DE, 6, 7, 0, 8, 0);
    t[0x22] = pk_desc(PK_C_LD8, 1, N, PK_M_HLI, 6, 7, 0, 8, 0);
    t[0x32] = pk_desc(PK_C_LD8, 1, N, PK_M_HLD, 6, 7, 0, 8, 0);
    t[0x0A] = pk_desc(PK_C_LD8, 1, PK_M_BC, N, 7, 6, 0, 8, 0);
    t[0x1A] = pk_desc(PK_C_LD8, 1, PK_M_DE, N, 7, 6, 0, 8, 0);
    t[0x2A] = pk_desc(PK_C_LD8, 1, PK_M_HLI, N, 7, 6, 0, 8, 0);
    t[0x3A] = pk_desc(PK_C_LD8, 1, PK_M_HLD, N, 7, 6, 0, 8, 0);
    for (int r = 0; r < 8; r++) {
        uint32_t m = (r == 6);
        t[0x04 | (r << 3)] = pk_desc(PK_C_INC8, 1, m ? PK_M_HL : N, m ? PK_M_HL : N, r, 0, 0, m ? 12 : 4, 0);
        t[0x05 | (r << 3)] = pk_desc(PK_C_DEC8, 1, m ? PK_M_HL : N, m ? PK_M_HL : N, r, 0, 0, m ? 12 : 4, 0);
        t[0x06 | (r << 3)] = pk_desc(PK_C_LD8, 2, N, m ? PK_M_HL : N, r, PK_SRC_IMM, 0, m ? 12 : 8, 0);
    }
    t[0x07] = pk_desc(PK_C_ROTA, 1, N, N, 0, 0, 0, 4, 0);  // RLCA
    t[0x0F] = pk_desc(PK_C_ROTA, 1, N, N, 0, 0, 1, 4, 0);  // RRCA
    t[0x17] = pk_desc(PK_C_ROTA, 1, N, N, 0, 0, 2, 4, 0);  // RLA
    t[0x1F] = pk_desc(PK_C_ROTA, 1, N, N, 0, 0, 3, 4, 0);  // RRA
    t[0x08] = pk_desc(PK_C_LDNNSP, 3, N, PK_M_NN2, 0, 0, 0, 20, 0);
    t[0x18] = pk_desc(PK_C_JR, 2, N, N, PK_COND_ALWAYS, 0, 0, 12, 0);
    for (int cc = 0; cc < 4; cc++) {
        t[0x20 | (cc << 3)] = pk_desc(PK_C_JR, 2, N, N, PK_COND_FLAG | cc, 0, 0, 8, 4);
        t[0xC2 | (cc << 3)] = pk_desc(PK_C_JP, 3, N, N, PK_COND_FLAG | cc, 0, 0, 12, 4);
        t[0xC4 | (cc << 3)] = pk_desc(PK_C_CALL, 3, N, PK_M_PUSH2, PK_COND_FLAG | cc, 0, 0, 12, 12);
        t[0xC0 | (cc << 3)] = pk_desc(PK_C_RET, 1, PK_M_SP2, N, PK_COND_FLAG | cc, 0, 0, 8, 12);
    }
    t[0x27] = pk_desc(PK_C_DAA, 1, N, N, 0, 0, 0, 4, 0);
    t[0x2F] = pk_desc(PK_C_CPL, 1, N, N, 0, 0, 0, 4, 0);
    t[0x37] = pk_desc(PK_C_SCF, 1, N, N, 0, 0, 0, 4, 0);
    t[0x3F] = pk_desc(PK_C_CCF, 1, N, N, 0, 0, 0, 4, 0);
    // ---- 0x40-0x7F: LD r,r' ----
    for (int d = 0; d < 8; d++)
        for (int s = 0; s < 8; s++) {
            int op = 0x40 | (d << 3) | s;
            if (op == 0x76) {
                t[op] = pk_desc(PK_C_HALT, 1, N, N, 0, 0, 0, 4, 0);
                continue;
            }
            uint32_t rd = (s == 6) ? PK_M_HL : N, wr = (d == 6) ? PK_M_HL : N;
            t[op] = pk_desc(PK_C_LD8, 1, rd, wr, d, s, 0, (d == 6 || s == 6) ? 8 : 4, 0);
        }
    // ---- 0x80-0xBF: ALU A,r ----
    for (int o = 0; o < 8; o++)
        for (int s = 0; s < 8; s++)
            t[0x80 | (o << 3) | s] = pk_desc(PK_C_ALU, 1, s == 6 ? PK_M_HL : N, N, 7, s, o, s == 6 ? 8 : 4, 0);
    // ---- 0xC0-0xFF ----
    t[0xC9] = pk_desc(PK_C_RET, 1, PK_M_SP2, N, PK_COND_ALWAYS, 0, 0, 16, 0);
    t[0xD9] = pk_desc(PK_C_RETI, 1, PK_M_SP2, N, 0, 0, 0, 16, 0);
    t[0xC3] = pk_desc(PK_C_JP, 3, N, N, PK_COND_ALWAYS, 0, 0, 16, 0);
    t[0xE9] = pk_desc(PK_C_JPHL, 1, N, N, 0, 0, 0, 4, 0);
    t[0xCD] = pk_desc(PK_C_CALL, 3, N, PK_M_PUSH2, PK_COND_ALWAYS, 0, 0, 24, 0);
    for (int p = 0; p < 4; p++) {
        t[0xC1 | (p << 4)] = pk_desc(PK_C_POP, 1, PK_M_SP2, N, p, 0, 0, 12, 0);
        t[0xC5 | (p << 4)] = pk_desc(PK_C_PUSH, 1, N, PK_M_PUSH2, p, 0, 0, 16, 0);
    }
    for (int v = 0; v < 8; v++) t[0xC7 | (v << 3)] = pk_desc(PK_C_RST, 1, N, PK_M_PUSH2, v, 0, 0, 16, 0);
    for (int o = 0; o < 8; o++) t[0xC6 | (o << 3)] = pk_desc(PK_C_ALU, 2, N, N, 7, PK_SRC_IMM, o, 8, 0);
    t[0xE0] = pk_desc(PK_C_LD8, 2, N, PK_M_HN, 6, 7, 0, 12, 0);
    t[0xF0] = pk_desc(PK_C_LD8, 2, PK_M_HN, N, 7, 6, 0, 12, 0);
    t[0xE2] = pk_desc(PK_C_LD8, 1, N, PK_M_HC, 6, 7, 0, 8, 0);
    t[0xF2] = pk_desc(PK_C_LD8, 1, PK_M_HC, N, 7, 6, 0, 8, 0);
    t[0xEA] = pk_desc(PK_C_LD8, 3, N, PK_M_NN, 6, 7, 0, 16, 0);
    t[0xFA] = pk_desc(PK_C_LD8, 3, PK_M_NN, N, 7, 6, 0, 16, 0);
    t[0xE8] = pk_desc(PK_C_ADDSP, 2, N, N, 0, 0, 0, 16, 0);
    t[0xF8] = pk_desc(PK_C_LDHLSP, 2, N, N, 0, 0, 0, 12, 0);
    t[0xF9] = pk_desc(PK_C_LDSPHL, 1, N, N, 0, 0, 0, 8, 0);
    t[0xF3] = pk_desc(PK_C_DI, 1, N, N, 0, 0, 0, 4, 0);
    t[0xFB] = pk_desc(PK_C_EI, 1, N, N, 0, 0, 0, 4, 0);
    // 0xCB prefix itself is never looked up (the kernel indexes 256 + second byte)
    // ---- CB-prefixed ----
    for (int i = 0; i < 256; i++) {
        int r = i & 7, y = (i >> 3) & 7, grp = i >> 6;
        uint32_t m = (r == 6);
        uint32_t rd = m ? PK_M_HL : N, wr = m ? PK_M_HL : N;
        uint32_t d;
        switch (grp) {
            case 0: d = pk_desc(PK_C_CBROT, 2, rd, wr, r, 0, y, m ? 16 : 8, 0); break;
            case 1: d = pk_desc(PK_C_BIT, 2, rd, N, r, y, 0, m ? 12 : 8, 0); break;
            case 2: d = pk_desc(PK_C_RES, 2, rd, wr, r, y, 0, m ? 16 : 8, 0); break;
            default: d = pk_desc(PK_C_SET, 2, rd, wr, r, y, 0, m ? 16 : 8, 0); break;
        }
        t[256 + i] = d;
    }
}
