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
        t[0x03 | (p << 4)] = pk_desc(PK_C_INCDEC16, 1, N, N, p, 0, 0, 8, 0);
        t[0x0B | (p << 4)] = pk_desc(PK_C_INCDEC16, 1, N, N, p, 0, 1, 8, 0);
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
    t[0x37] = pk_desc(PK_C_SCFCCF, 1, N, N, 0, 0, 0, 4, 0);
    t[0x3F] = pk_desc(PK_C_SCFCCF, 1, N, N, 0, 0, 1, 4, 0);
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
    t[0xE8] = pk_desc(PK_C_ADDSPE, 2, N, N, 0, 0, 0, 16, 0);
    t[0xF8] = pk_desc(PK_C_ADDSPE, 2, N, N, 0, 0, 1, 12, 0);
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

static inline uint32_t pk_ucode(uint32_t r8sel, uint32_t dst8, uint32_t xtgt, uint32_t yone, uint32_t arith,
                                uint32_t fmode, uint32_t op16, uint32_t ctrl, uint32_t wsrc, uint32_t ime) {
    return r8sel | (dst8 << 4) | (xtgt << 6) | (yone << 7) | (arith << 8) | (fmode << 10) | (op16 << 14) |
           (ctrl << 18) | (wsrc << 22) | (ime << 24);
}

// Microcode word for a descriptor (the second half of each decode entry): which result the fused
// datapath selects, where it is written, which flags rule applies, the 16-bit op and the control
// transfer.  Derived from the datapath class so the two words can never disagree.
static inline uint32_t pk_ucode_for(uint32_t d) {
    const uint32_t cls = PK_D_CLS(d), sub = PK_D_OP(d), fa = PK_D_A(d);
    switch (cls) {
        case PK_C_LD8: return pk_ucode(1, 2, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_ALU:
            if (sub >= 4 && sub <= 6) return pk_ucode(3, 1, 0, 0, 0, PK_F_ALU, PK_O_NONE, PK_K_SEQ, 0, 0);
            return pk_ucode(2, sub == 7 ? 0 : 1, 0, 0, 0, PK_F_ALU, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_INC8: return pk_ucode(2, 2, 1, 1, 1, PK_F_INCDEC, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_DEC8: return pk_ucode(2, 2, 1, 1, 2, PK_F_INCDEC, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_ROTA: return pk_ucode(4, 1, 0, 0, 0, PK_F_ROTA, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_CBROT: return pk_ucode(4, 2, 1, 0, 0, PK_F_CBROT, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_BIT: return pk_ucode(0, 0, 1, 0, 0, PK_F_BIT, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_RES: return pk_ucode(5, 2, 1, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_SET: return pk_ucode(6, 2, 1, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_DAA: return pk_ucode(7, 1, 0, 0, 0, PK_F_DAA, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_CPL: return pk_ucode(8, 1, 0, 0, 0, PK_F_CPL, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_SCFCCF: return pk_ucode(0, 0, 0, 0, 0, sub ? PK_F_CCF : PK_F_SCF, PK_O_NONE, PK_K_SEQ, 0, 0);
        case PK_C_LD16: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_LD16, PK_K_SEQ, 0, 0);
        case PK_C_INCDEC16: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, sub ? PK_O_DEC16 : PK_O_INC16, PK_K_SEQ, 0, 0);
        case PK_C_ADDHL: return pk_ucode(0, 0, 0, 0, 0, PK_F_ADDHL, PK_O_ADDHL, PK_K_SEQ, 0, 0);
        case PK_C_ADDSPE: return pk_ucode(0, 0, 0, 0, 0, PK_F_ADDSPE, sub ? PK_O_SPE_HL : PK_O_SPE_SP, PK_K_SEQ, 0, 0);
        case PK_C_LDSPHL: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_SPHL, PK_K_SEQ, 0, 0);
        case PK_C_LDNNSP: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_SEQ, 3, 0);
        case PK_C_PUSH: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_SEQ, 2, 0);
        case PK_C_POP: return pk_ucode(0, 0, 0, 0, 0, fa == 3 ? PK_F_POPAF : PK_F_KEEP, fa == 3 ? PK_O_POPAF : PK_O_POP, PK_K_SEQ, 0, 0);
        case PK_C_JP: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_JP, 0, 0);
        case PK_C_JPHL: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_JPHL, 0, 0);
        case PK_C_JR: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_JR, 0, 0);
        case PK_C_CALL: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_CALL, 1, 0);
        case PK_C_RET: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_RET, 0, 0);
        case PK_C_RETI: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_RETI, 0, 2);
        case PK_C_RST: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_RST, 1, 0);
        case PK_C_INT: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_INT, 1, 1);
        case PK_C_DI: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_SEQ, 0, 1);
        case PK_C_EI: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_SEQ, 0, 2);
        case PK_C_HALT: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_HALT, 0, 0);
        case PK_C_ILLEGAL: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_ILLEGAL, 0, 0);
        default: return pk_ucode(0, 0, 0, 0, 0, PK_F_KEEP, PK_O_NONE, PK_K_SEQ, 0, 0);  // NOP/STOP
    }
}

// full decode table for the kernel's slow (RAM-code) path: [0,512) descriptors, [512,1024) ucode
static inline void pk_build_dtab(uint32_t* t /* 1024 */) {
    pk_build_decode(t);
    for (int i = 0; i < 512; i++) t[512 + i] = pk_ucode_for(t[i]);
}

// Pre-decoded ROM: for every ROM byte position p (bank * 0x4000 + offset) the descriptor and
// microcode of the instruction that would start there plus its raw bytes, so the kernel's fetch
// + decode is ONE 16-byte load.  Positions whose operand bytes would cross the end of their
// 16 KiB bank are flagged slow (fetched through the memory bus instead).
static inline void pk_build_rom16(const uint8_t* rom, uint32_t rom_len, const uint32_t* dtab, pk_rom_entry* out) {
    for (uint32_t p = 0; p < rom_len; p++) {
        uint32_t off = p & 0x3FFFu;
        uint8_t op = rom[p];
        uint8_t b1 = off + 1 < 0x4000u ? rom[p + 1] : 0;
        uint8_t b2 = off + 2 < 0x4000u ? rom[p + 2] : 0;
        uint32_t slow = off >= 0x3FFEu ? 1u : 0u;
        uint32_t di = op == 0xCB ? 256u + b1 : op;
        out[p].desc = dtab[di];
        out[p].ucode = dtab[512 + di];
        out[p].bytes = (uint32_t)op | ((uint32_t)b1 << 8) | ((uint32_t)b2 << 16) | (slow << 24);
        out[p].pad = 0;
    }
}
