// pk_ucode.h — SM83 microcode for the K1 step kernel (pk_step.hip), built on the host and staged
// in LDS.  One 48-byte entry per opcode (256 base + 256 CB-prefixed + 3 pseudo-ops) drives ONE
// fused datapath that every lane runs each iteration, whatever opcode it holds:
//
//   X = perm(w1:w0, XR) | perm(ext, XE)     Y = perm(w1:w0, YR) | perm(ext, YE) | yconst
//   (ext = the instruction bytes op|n|n2 and m0|m1|SP: immediates, memory operands, SP and the
//   sign of n all come out of one v_perm with a per-opcode selector)
//   adder  r = X + (sub ? ~Y : Y) + cin;   carries = X ^ Y' ^ r  ->  H, C at bit 4/8 or 12/16
//   logic  X & Y | X ^ Y | X | Y           rotate/shift unit on X
//   val    = res16 | F' << 16 | res8 << 24;  w0 = perm(val, w0, S0);  w1 = perm(val, w1, S1)
//
// so an 8-bit write, a 16-bit pair write, the flags, POP AF and (HL+)/(HL-) are all the same two
// v_perm_b32.  Register layout inside the kernel: w0 = C|B<<8|E<<16|D<<24,
// w1 = L|H<<8|F<<16|A<<24 (bytes 0..7 of the perm source pair w1:w0: C B E D L H F A).
//
// Instruction semantics and cycle counts are those of PyBoy 1.x's generated opcodes.py as the
// oracle restates them (oracle/gbcore.c cpu_execute / exec_cb / cpu_check_interrupts).
#pragma once
#include <stdint.h>

// ---- entry layout: 16 dwords (four ds_read_b128) ----
enum { PK_UE_D = 0, PK_UE_U, PK_UE_K, PK_UE_V, PK_UE_XR, PK_UE_XE, PK_UE_YR, PK_UE_YE, PK_UE_AR, PK_UE_AE,
       PK_UE_S0, PK_UE_S1, PK_UE_YC, PK_UE_YX, PK_UE_CW, PK_UE_CI, PK_UE_WORDS };
// stored words (what the kernel reads; the builder below works in the PK_UB_/PK_KB_ form):
//   U  datapath control bits PK_US_*          K  FC | FK << 8 | FM << 16 | CPUAND << 24 | CPUOR << 28
//   V  the successor selector: bytes 0-1 = a v_perm selector taking the fetched bytes' successor
//      opcode and operand (bytes len, len + 1), or 0xFF (0x0D: RST 38h, no secondary op) for a
//      primary that may not fuse; | cycles << 16 | extra cycles when the condition holds << 24 (the D
//      fields CYC/XCYC times 4: one add and one select in the kernel)
//   YC Y constant (INC/DEC, CPL, BIT/RES/SET masks, RST vector); bits 16-31: 0xFFFF for JR (target =
//      pc + len + Y; Y's bits above 16 reach no result)                YX 0x1FFFF when the adder subtracts
//   CW/CI carry-in (adder) / shifted-in bit (right-shift unit) = bit CW of (X | F << 16) ^ CI:
//         bit 20 = F.C, bit 7/bit 0 = X's top/bottom bit, bit 16 = constant 0 (with CI: constant 1)
#define PK_US_LOGIC 0     // result8 from the logic unit (loads: X = 0xFF AND Y), else adder / right unit
#define PK_US_RIGHT 1     // result8 and C from the right-shift unit
#define PK_US_SWAP 2      // right-shift unit: nibble swap
#define PK_US_HSH8 3      // H/C from carry bits 12/16 (ADD HL,rr), else 4/8 (at bit 3: U & 8 is the shift)
#define PK_US_JUMP 4      // control transfer to X + Y (+ pc + len for JR) when the condition holds
#define PK_US_WPC 5       // 16-bit write value = return PC (else X)
#define PK_US_W16 6       // write value 16-bit (else result8)
#define PK_US_HIFIRST 7   // a 16-bit push: the slow bus path writes the high address first (PyBoy order)
#define PK_US_FPOP 8      // F = m0 & 0xF0 (POP AF)
#define PK_US_R16HL 9     // res16 = HL +- 1 (else adder)
#define PK_US_SPW 10      // SP = res16
#define PK_US_LAND 12     // logic result includes X & Y (AND, OR)
#define PK_US_LXOR 13     // logic result includes X ^ Y (XOR, OR)
#define PK_US_HLINC 22    // 2 bits signed HL increment for (HL+)/(HL-)
#define PK_US_SPD 26      // 3 bits signed SP delta (PUSH/POP family), applied when the condition holds
#define PK_UC_ENTRIES 515u
#define PK_UC_INT 512u    // pseudo-op: interrupt dispatch (push PC, jump to the vector)
#define PK_UC_IDLE 513u   // pseudo-op: halted / crashed CPU, 4 cycles
#define PK_UC_NOP0 514u   // pseudo-op: interrupt pending with IME off (queued), 0 cycles
// secondary-op table (fused pairs, see pk_u2_entry): 256 entries x 8 dwords after the main table
#define PK_U2_WORDS 8u
#define PK_U2_NONE 0xFFu   // RST 38h: never a secondary op (the index of every primary that may not fuse)
#define PK_UC_U2 (PK_UC_ENTRIES * PK_UE_WORDS)
#define PK_UC_WORDS (PK_UC_U2 + (PK_U2_NONE + 1u) * PK_U2_WORDS)

// D word: memory, timing, control
#define PK_DB_LEN 0       // 2 bits  instruction length
#define PK_DB_RD 2        // read m0 at addr0
#define PK_DB_RD2 3       // read m1 at addr1
#define PK_DB_WR 4        // write wv0 at addr0
#define PK_DB_WR2 5       // write wv1 at addr1
#define PK_DB_ASP 6       // (builder only) address source SP        -> AE selector
#define PK_DB_RD1 6       // (stored word) a one-byte read (RD, not RD2): the LDS-staged ROM path
#define PK_DB_NOFUSE 8    // (stored word) no secondary op may follow in the same iteration (pk_u2_entry)
#define PK_DB_AIMM 7      // (builder only) address source immediate -> AE selector
#define PK_DB_AHN 8       // (builder only) immediate address 0xFF00|n
#define PK_DB_AOFF 9      // 2 bits signed: addr0 = src + aoff
#define PK_DB_ADIR 11     // 2 bits signed: addr1 = addr0 + adir
#define PK_DB_CYC 13      // 3 bits cycles/4 (the kernel reads them pre-scaled from the V word)
#define PK_DB_XCYC 16     // 2 bits extra cycles/4 when the condition holds (likewise)
#define PK_DB_CPOS 18     // 4 bits: condition = bit cpos of (F | 0x100)
#define PK_DB_CINV 22     //         ^ cinv
#define PK_DB_TSRC 23     // 3 bits jump target (builder: PK_T_*; stored: 0 none, 1 X|Y, 2 JR)
#define PK_DB_IME 26      // 2 bits: 0 keep 1 clear 2 set
#define PK_DB_HALT 28     // set HALT
#define PK_DB_CRASH 29    // set CRASH|HALT (illegal opcode)
#define PK_DB_DAA 30      // DAA (the rare read block: its microcode reads 0xFFFF twice)
#define PK_DB_YSP 31      // (builder only) Y = SP
enum { PK_T_NONE = 0, PK_T_IMM, PK_T_HL, PK_T_JR, PK_T_M16, PK_T_RST };
enum { PK_J_NONE = 0, PK_J_XY = 1, PK_J_JR = 2 };  // stored: target = X | Y (operands chosen below) or pc+2+e

// U word: datapath
// bits 0-5 are builder-only operand flags, turned into the XE/YE selectors by pk_build_ucode
#define PK_UB_XSP 0       // X = SP
#define PK_UB_XMEM 1      // X = m0
#define PK_UB_YIMM 2      // Y = immediate
#define PK_UB_IMM8 3      // immediate = n (else nn)
#define PK_UB_SEXT 4      // immediate = sign-extended n (16-bit)
#define PK_UB_YMEM 5      // Y = m16
#define PK_UB_SUB 6       // adder subtracts
#define PK_UB_USEC 7      // adder carry-in from F.C (ADC/SBC)
#define PK_UB_HC16 8      // H/C from bits 12/16 (else 4/8)
#define PK_UB_R8 9        // 2 bits result8: 0 Y 1 adder 2 logic 3 rotate
#define PK_UB_LOP 11      // 2 bits logic: 0 AND 1 XOR 2 OR
// V word (derived from U by pk_store_uop)
#define PK_VB_R8SH 0      // 5 bits: result8 byte offset in the [Y, adder, logic, rotate] pool (8 * R8)
#define PK_VB_LAND 8      // logic result includes X & Y (AND, OR)
#define PK_VB_LXOR 9      // logic result includes X ^ Y (XOR, OR); OR = AND | XOR
#define PK_UB_RDIR 13     // rotate right (else left)
#define PK_UB_RBIN 14     // 2 bits rotate-in bit: 0 zero 1 F.C 2 rotated-out bit 3 bit 7 (SRA)
#define PK_UB_SWAP 16     // SWAP
#define PK_UB_FZ 17       // Z from result8
#define PK_UB_FH 18       // H from adder
#define PK_UB_FC 19       // 2 bits C: 0 none 1 adder 2 rotate 3 !F.C
#define PK_UB_FPOP 21     // F = m0 & 0xF0 (POP AF)
#define PK_UB_HLINC 22    // 2 bits signed HL increment for (HL+)/(HL-)
#define PK_UB_R16HL 24    // res16 = HL +- 1 (else adder)
#define PK_UB_SPW 25      // SP = res16
#define PK_UB_SPD 26      // 3 bits signed SP delta (PUSH/POP family), applied when the condition holds
#define PK_UB_W16 29      // write value is 16-bit (else result8)
#define PK_UB_WPC 30      // 16-bit write value = return PC
#define PK_UB_WSP 31      // 16-bit write value = SP

// K word: constants
#define PK_KB_YCONST 0    // 8 bits ORed into Y
#define PK_KB_FKEEP 8     // 8 bits: F bits kept
#define PK_KB_FCONST 16   // 8 bits: F bits set
#define PK_KB_CPUAND 24   // 4 bits: CPU state bits (IME HALT QUEUED CRASH) kept
#define PK_KB_CPUOR 28    // 4 bits: CPU state bits set

// perm selectors over (w1:w0) = bytes C B E D L H F A ; 0x0C = 0x00, 0x0D = 0xFF
#define PK_PZERO 0x0C0C0C0Cu
// perm selectors over the ext pool (q1:q0): q0 = op | n<<8 | n2<<16, q1 = m0 | m1<<8 | SP<<16;
// 0x08 = the sign of n replicated
#define PK_E_SP 0x0C0C0706u
// the address pool is (SP : q0) (the kernel's first stage has no m0|m1 yet): SP at bytes 4-5
#define PK_A_SP 0x0C0C0504u
#define PK_E_M0 0x0C0C0C04u
#define PK_E_M16 0x0C0C0504u
#define PK_E_N 0x0C0C0C01u
#define PK_E_NN 0x0C0C0201u
#define PK_E_SEXTN 0x0C0C0801u
#define PK_E_HN 0x0C0C0D01u

static inline uint32_t pk_r8_byte(int r) {  // SM83 r8 index (B C D E H L (HL) A) -> byte in w1:w0
    static const uint8_t b[8] = {1, 0, 3, 2, 5, 4, 0xFF, 7};
    return b[r & 7];
}
static inline uint32_t pk_sel8(int r) { return 0x0C0C0C00u | pk_r8_byte(r); }
static inline uint32_t pk_sel16(int p) {  // BC DE HL AF -> 16-bit (lo | hi<<8)
    static const uint32_t s[4] = {0x0C0C0100u, 0x0C0C0302u, 0x0C0C0504u, 0x0C0C0706u};
    return s[p & 3];
}

struct PkUop {
    uint32_t d, u, px, py, s0, s1, pa, k;
};

// writeback selectors: identity, F always from val byte 2 (F' = kept bits | computed bits)
#define PK_S0_ID 0x03020100u
#define PK_S1_ID 0x03060100u
static inline void pk_wb_r8(PkUop& o, int r) {  // dest r8 <- val byte 3 (result8)
    uint32_t b = pk_r8_byte(r);
    if (b < 4) o.s0 = (o.s0 & ~(0xFFu << (8 * b))) | (0x07u << (8 * b));
    else o.s1 = (o.s1 & ~(0xFFu << (8 * (b - 4)))) | (0x07u << (8 * (b - 4)));
}
static inline void pk_wb_r16(PkUop& o, int p) {  // dest pair BC DE HL <- val bytes 0,1 (res16)
    if (p == 0) o.s0 = (o.s0 & 0xFFFF0000u) | 0x0504u;
    else if (p == 1) o.s0 = (o.s0 & 0x0000FFFFu) | 0x05040000u;
    else if (p == 2) o.s1 = (o.s1 & 0xFFFF0000u) | 0x0504u;
}

static inline uint32_t pk_fld(uint32_t v, int pos) { return v << pos; }
static inline uint32_t pk_sfld(int v, int pos, int bits) { return ((uint32_t)v & ((1u << bits) - 1u)) << pos; }

// adder / flag helpers
#define PK_F_Z 0x80u
#define PK_F_N 0x40u
#define PK_F_H 0x20u
#define PK_F_C 0x10u

static inline PkUop pk_uop_base(int len, int cyc) {
    PkUop o;
    o.d = pk_fld((uint32_t)len, PK_DB_LEN) | pk_fld((uint32_t)cyc / 4u, PK_DB_CYC) | pk_fld(8u, PK_DB_CPOS);
    o.u = 0;
    o.px = PK_PZERO;
    o.py = PK_PZERO;
    o.s0 = PK_S0_ID;
    o.s1 = PK_S1_ID;
    o.pa = PK_PZERO;
    o.k = pk_fld(0xF0u, PK_KB_FKEEP);  // keep every flag unless the op says otherwise
    return o;
}
static inline void pk_flags(PkUop& o, uint32_t keep, uint32_t cst) {
    o.k = (o.k & ~(0xFFFFu << PK_KB_FKEEP)) | pk_fld(keep, PK_KB_FKEEP) | pk_fld(cst, PK_KB_FCONST);
}
static inline void pk_cond(PkUop& o, int cc) {  // NZ Z NC C
    static const uint32_t pos[4] = {7, 7, 4, 4}, inv[4] = {1, 0, 1, 0};
    o.d = (o.d & ~(15u << PK_DB_CPOS)) | pk_fld(pos[cc & 3], PK_DB_CPOS) | pk_fld(inv[cc & 3], PK_DB_CINV);
}
// memory operand through a register pair / (C) / SP / immediate
static inline void pk_mem_pair(PkUop& o, int p) { o.pa = pk_sel16(p); }
static inline void pk_mem_hc(PkUop& o) { o.pa = 0x0C0C0D00u; }  // 0xFF00 | C

// 8-bit operation on A (or a register target) with source r / (HL) / n
static inline void pk_alu(PkUop& o, int aop, int src) {
    // src: 0..7 register (6 = (HL)), 8 = immediate n
    o.px = pk_sel8(7);
    if (src == 8) o.u |= pk_fld(1, PK_UB_YIMM) | pk_fld(1, PK_UB_IMM8);
    else if (src == 6) o.u |= pk_fld(1, PK_UB_YMEM);
    else o.py = pk_sel8(src);
    o.u |= pk_fld(1, PK_UB_FZ);
    if (aop <= 3 || aop == 7) {  // ADD ADC SUB SBC CP
        o.u |= pk_fld(1, PK_UB_R8) | pk_fld(1, PK_UB_FH) | pk_fld(1, PK_UB_FC);
        if (aop >= 2) o.u |= pk_fld(1, PK_UB_SUB);
        if (aop == 1 || aop == 3) o.u |= pk_fld(1, PK_UB_USEC);
        pk_flags(o, 0, aop >= 2 ? PK_F_N : 0);
        if (aop != 7) pk_wb_r8(o, 7);
    } else {  // AND XOR OR
        o.u |= pk_fld(2, PK_UB_R8) | pk_fld((uint32_t)(aop - 4), PK_UB_LOP);
        pk_flags(o, 0, aop == 4 ? PK_F_H : 0);
        pk_wb_r8(o, 7);
    }
}

static inline PkUop pk_uop(int op) {
    PkUop o = pk_uop_base(1, 4);
    const int N = 0;
    (void)N;
    if (op >= 0x40 && op < 0x80 && op != 0x76) {  // LD r, r'
        int d = (op >> 3) & 7, s = op & 7;
        o = pk_uop_base(1, (d == 6 || s == 6) ? 8 : 4);
        if (s == 6) { o.u |= pk_fld(1, PK_UB_YMEM); o.d |= pk_fld(1, PK_DB_RD); pk_mem_pair(o, 2); }
        else o.py = pk_sel8(s);
        if (d == 6) { o.d |= pk_fld(1, PK_DB_WR); pk_mem_pair(o, 2); }
        else pk_wb_r8(o, d);
        return o;
    }
    if (op >= 0x80 && op < 0xC0) {  // ALU A, r
        int s = op & 7;
        o = pk_uop_base(1, s == 6 ? 8 : 4);
        if (s == 6) { o.d |= pk_fld(1, PK_DB_RD); pk_mem_pair(o, 2); }
        pk_alu(o, (op >> 3) & 7, s);
        return o;
    }
    switch (op) {
        case 0x00: return pk_uop_base(1, 4);
        case 0x10: return pk_uop_base(2, 4);  // STOP: 2-byte no-op on DMG
        case 0x76: o = pk_uop_base(0, 4); o.d |= pk_fld(1, PK_DB_HALT); return o;  // HALT: PC stays
        case 0xF3: o.d |= pk_fld(1, PK_DB_IME); return o;
        case 0xFB: o.d |= pk_fld(2, PK_DB_IME); return o;
        case 0x27:  // DAA: computed in the kernel's rare read block, delivered as m1|m0 (A, F) like POP AF
            o.d |= pk_fld(1, PK_DB_DAA) | pk_fld(1, PK_DB_RD) | pk_fld(1, PK_DB_RD2) | pk_sfld(-1, PK_DB_AOFF, 2);
            o.u |= pk_fld(1, PK_UB_YMEM) | pk_fld(1, PK_UB_FPOP);
            o.s1 = (o.s1 & 0x00FFFFFFu) | 0x05000000u;
            return o;
        case 0x2F:  // CPL = A ^ 0xFF
            o.px = pk_sel8(7); o.k |= pk_fld(0xFF, PK_KB_YCONST);
            o.u |= pk_fld(2, PK_UB_R8) | pk_fld(1, PK_UB_LOP);
            pk_flags(o, PK_F_Z | PK_F_C, PK_F_N | PK_F_H); pk_wb_r8(o, 7); return o;
        case 0x37: pk_flags(o, PK_F_Z, PK_F_C); return o;                                  // SCF
        case 0x3F: pk_flags(o, PK_F_Z, 0); o.u |= pk_fld(3, PK_UB_FC); return o;          // CCF
        case 0x07: case 0x0F: case 0x17: case 0x1F: {  // RLCA RRCA RLA RRA
            int y = (op >> 3) & 3;
            o.px = pk_sel8(7);
            o.u |= pk_fld(3, PK_UB_R8) | pk_fld(2, PK_UB_FC) | pk_fld((uint32_t)(y & 1), PK_UB_RDIR)
                 | pk_fld(y >= 2 ? 1u : 2u, PK_UB_RBIN);
            pk_flags(o, 0, 0); pk_wb_r8(o, 7); return o;
        }
        case 0x08:  // LD (nn), SP
            o = pk_uop_base(3, 20);
            o.d |= pk_fld(1, PK_DB_WR) | pk_fld(1, PK_DB_WR2) | pk_fld(1, PK_DB_AIMM) | pk_sfld(1, PK_DB_ADIR, 2);
            o.u |= pk_fld(1, PK_UB_W16) | pk_fld(1, PK_UB_WSP);
            return o;
        case 0x18: o = pk_uop_base(2, 12); o.d |= pk_fld(PK_T_JR, PK_DB_TSRC); return o;
        case 0xC3: o = pk_uop_base(3, 16); o.d |= pk_fld(PK_T_IMM, PK_DB_TSRC); return o;
        case 0xE9: o = pk_uop_base(1, 4); o.d |= pk_fld(PK_T_HL, PK_DB_TSRC); return o;
        case 0xCD: case 0xC4: case 0xCC: case 0xD4: case 0xDC: {  // CALL (cc,) nn
            o = pk_uop_base(3, op == 0xCD ? 24 : 12);
            o.d |= pk_fld(PK_T_IMM, PK_DB_TSRC) | pk_fld(1, PK_DB_WR) | pk_fld(1, PK_DB_WR2) | pk_fld(1, PK_DB_ASP)
                 | pk_sfld(-1, PK_DB_AOFF, 2) | pk_sfld(-1, PK_DB_ADIR, 2);
            o.u |= pk_fld(1, PK_UB_W16) | pk_fld(1, PK_UB_WPC) | pk_sfld(-2, PK_UB_SPD, 3);
            if (op != 0xCD) { pk_cond(o, (op >> 3) & 3); o.d |= pk_fld(3, PK_DB_XCYC); }
            return o;
        }
        case 0xC9: case 0xD9: case 0xC0: case 0xC8: case 0xD0: case 0xD8: {  // RET / RETI / RET cc
            o = pk_uop_base(1, (op == 0xC9 || op == 0xD9) ? 16 : 8);
            o.d |= pk_fld(PK_T_M16, PK_DB_TSRC) | pk_fld(1, PK_DB_RD) | pk_fld(1, PK_DB_RD2) | pk_fld(1, PK_DB_ASP)
                 | pk_sfld(1, PK_DB_ADIR, 2);
            o.u |= pk_sfld(2, PK_UB_SPD, 3);
            if (op == 0xD9) o.d |= pk_fld(2, PK_DB_IME);
            if ((op & 0x0F) == 0x00 || (op & 0x0F) == 0x08) { pk_cond(o, (op >> 3) & 3); o.d |= pk_fld(3, PK_DB_XCYC); }
            return o;
        }
        case 0xE0: case 0xF0: case 0xEA: case 0xFA: {  // LDH (n),A / LDH A,(n) / LD (nn),A / LD A,(nn)
            int hn = (op & 0x0F) == 0x00;
            o = pk_uop_base(hn ? 2 : 3, hn ? 12 : 16);
            o.d |= pk_fld(1, PK_DB_AIMM) | pk_fld((uint32_t)hn, PK_DB_AHN);
            if (op >= 0xF0) { o.d |= pk_fld(1, PK_DB_RD); o.u |= pk_fld(1, PK_UB_YMEM); pk_wb_r8(o, 7); }
            else { o.d |= pk_fld(1, PK_DB_WR); o.py = pk_sel8(7); }
            return o;
        }
        case 0xE2: case 0xF2:  // LD (C),A / LD A,(C)
            o = pk_uop_base(1, 8);
            pk_mem_hc(o);
            if (op == 0xF2) { o.d |= pk_fld(1, PK_DB_RD); o.u |= pk_fld(1, PK_UB_YMEM); pk_wb_r8(o, 7); }
            else { o.d |= pk_fld(1, PK_DB_WR); o.py = pk_sel8(7); }
            return o;
        case 0xE8: case 0xF8:  // ADD SP,e / LD HL,SP+e : X = SP, Y = sext(e), H/C from the low byte
            o = pk_uop_base(2, op == 0xE8 ? 16 : 12);
            o.u |= pk_fld(1, PK_UB_XSP) | pk_fld(1, PK_UB_YIMM) | pk_fld(1, PK_UB_SEXT) | pk_fld(1, PK_UB_FH) | pk_fld(1, PK_UB_FC);
            pk_flags(o, 0, 0);
            if (op == 0xE8) o.u |= pk_fld(1, PK_UB_SPW);
            else pk_wb_r16(o, 2);
            return o;
        case 0xF9: o = pk_uop_base(1, 8); o.px = pk_sel16(2); o.u |= pk_fld(1, PK_UB_SPW); return o;  // LD SP,HL
    }
    // LD rr,nn / INC rr / DEC rr / ADD HL,rr / (BC|DE|HL+|HL-) loads and stores
    if ((op & 0xC0) == 0x00) {
        int p = (op >> 4) & 3, lo = op & 0x0F;
        switch (lo) {
            case 0x01:  // LD rr, nn
                o = pk_uop_base(3, 12);
                o.u |= pk_fld(1, PK_UB_YIMM);
                if (p == 3) o.u |= pk_fld(1, PK_UB_SPW); else pk_wb_r16(o, p);
                return o;
            case 0x03: case 0x0B:  // INC rr / DEC rr
                o = pk_uop_base(1, 8);
                if (p == 3) o.u |= pk_fld(1, PK_UB_XSP) | pk_fld(1, PK_UB_SPW);
                else { o.px = pk_sel16(p); pk_wb_r16(o, p); }
                o.k |= pk_fld(1, PK_KB_YCONST);
                if (lo == 0x0B) o.u |= pk_fld(1, PK_UB_SUB);
                return o;
            case 0x09:  // ADD HL, rr
                o = pk_uop_base(1, 8);
                o.px = pk_sel16(2);
                if (p == 3) o.d |= pk_fld(1, PK_DB_YSP); else o.py = pk_sel16(p);
                o.u |= pk_fld(1, PK_UB_HC16) | pk_fld(1, PK_UB_FH) | pk_fld(1, PK_UB_FC);
                pk_flags(o, PK_F_Z, 0);
                pk_wb_r16(o, 2);
                return o;
            case 0x02: case 0x0A: {  // LD (BC|DE|HL+|HL-), A  /  LD A, (...)
                o = pk_uop_base(1, 8);
                if (p < 2) pk_mem_pair(o, p);
                else {
                    pk_mem_pair(o, 2);
                    o.u |= pk_sfld(p == 2 ? 1 : -1, PK_UB_HLINC, 2) | pk_fld(1, PK_UB_R16HL);
                    pk_wb_r16(o, 2);
                }
                if (lo == 0x0A) { o.d |= pk_fld(1, PK_DB_RD); o.u |= pk_fld(1, PK_UB_YMEM); pk_wb_r8(o, 7); }
                else { o.d |= pk_fld(1, PK_DB_WR); o.py = pk_sel8(7); }
                return o;
            }
        }
        int r = (op >> 3) & 7, low3 = op & 7;
        if (low3 == 4 || low3 == 5) {  // INC r / DEC r
            o = pk_uop_base(1, r == 6 ? 12 : 4);
            if (r == 6) { o.d |= pk_fld(1, PK_DB_RD) | pk_fld(1, PK_DB_WR); pk_mem_pair(o, 2); o.u |= pk_fld(1, PK_UB_XMEM); }
            else { o.px = pk_sel8(r); pk_wb_r8(o, r); }
            o.k |= pk_fld(1, PK_KB_YCONST);
            o.u |= pk_fld(1, PK_UB_R8) | pk_fld(1, PK_UB_FZ) | pk_fld(1, PK_UB_FH);
            if (low3 == 5) o.u |= pk_fld(1, PK_UB_SUB);
            pk_flags(o, PK_F_C, low3 == 5 ? PK_F_N : 0);
            return o;
        }
        if (low3 == 6) {  // LD r, n
            o = pk_uop_base(2, r == 6 ? 12 : 8);
            o.u |= pk_fld(1, PK_UB_YIMM) | pk_fld(1, PK_UB_IMM8);
            if (r == 6) { o.d |= pk_fld(1, PK_DB_WR); pk_mem_pair(o, 2); }
            else pk_wb_r8(o, r);
            return o;
        }
        if (low3 == 0 && op >= 0x20) {  // JR cc, e
            o = pk_uop_base(2, 8);
            o.d |= pk_fld(PK_T_JR, PK_DB_TSRC) | pk_fld(1, PK_DB_XCYC);
            pk_cond(o, (op >> 3) & 3);
            return o;
        }
    }
    if ((op & 0xC0) == 0xC0) {
        int p = (op >> 4) & 3, lo = op & 0x0F;
        if (lo == 0x01) {  // POP rr
            o = pk_uop_base(1, 12);
            o.d |= pk_fld(1, PK_DB_RD) | pk_fld(1, PK_DB_RD2) | pk_fld(1, PK_DB_ASP) | pk_sfld(1, PK_DB_ADIR, 2);
            o.u |= pk_fld(1, PK_UB_YMEM) | pk_sfld(2, PK_UB_SPD, 3);
            if (p == 3) {  // POP AF: A <- m1, F <- m0 & 0xF0
                o.u |= pk_fld(1, PK_UB_FPOP);
                o.s1 = (o.s1 & 0x00FFFFFFu) | 0x05000000u;
            } else pk_wb_r16(o, p);
            return o;
        }
        if (lo == 0x05) {  // PUSH rr
            o = pk_uop_base(1, 16);
            o.d |= pk_fld(1, PK_DB_WR) | pk_fld(1, PK_DB_WR2) | pk_fld(1, PK_DB_ASP) | pk_sfld(-1, PK_DB_AOFF, 2)
                 | pk_sfld(-1, PK_DB_ADIR, 2);
            o.u |= pk_fld(1, PK_UB_W16) | pk_sfld(-2, PK_UB_SPD, 3);
            o.py = pk_sel16(p);  // AF: F | A << 8
            return o;
        }
        if ((op & 7) == 7) {  // RST
            o = pk_uop_base(1, 16);
            o.k |= pk_fld((uint32_t)op & 0x38u, PK_KB_YCONST);  // vector rides in Y
            o.d |= pk_fld(PK_T_RST, PK_DB_TSRC) | pk_fld(1, PK_DB_WR) | pk_fld(1, PK_DB_WR2) | pk_fld(1, PK_DB_ASP)
                 | pk_sfld(-1, PK_DB_AOFF, 2) | pk_sfld(-1, PK_DB_ADIR, 2);
            o.u |= pk_fld(1, PK_UB_W16) | pk_fld(1, PK_UB_WPC) | pk_sfld(-2, PK_UB_SPD, 3);
            return o;
        }
        if ((op & 7) == 6) {  // ALU A, n
            o = pk_uop_base(2, 8);
            pk_alu(o, (op >> 3) & 7, 8);
            return o;
        }
        if ((op & 0xE7) == 0xC2) {  // JP cc, nn
            o = pk_uop_base(3, 12);
            o.d |= pk_fld(PK_T_IMM, PK_DB_TSRC) | pk_fld(1, PK_DB_XCYC);
            pk_cond(o, (op >> 3) & 3);
            return o;
        }
    }
    // illegal opcode: freeze the CPU (documented extension; PyBoy raises)
    o = pk_uop_base(0, 4);
    o.d |= pk_fld(1, PK_DB_CRASH);
    return o;
}

static inline PkUop pk_uop_cb(int op) {
    int r = op & 7, y = (op >> 3) & 7, grp = op >> 6;
    PkUop o = pk_uop_base(2, r == 6 ? (grp == 1 ? 12 : 16) : 8);
    if (r == 6) {
        pk_mem_pair(o, 2);
        o.d |= pk_fld(1, PK_DB_RD);
        if (grp != 1) o.d |= pk_fld(1, PK_DB_WR);
        o.u |= pk_fld(1, PK_UB_XMEM);
    } else {
        o.px = pk_sel8(r);
        if (grp != 1) pk_wb_r8(o, r);
    }
    switch (grp) {
        case 0: {  // RLC RRC RL RR SLA SRA SWAP SRL
            static const uint8_t dir[8] = {0, 1, 0, 1, 0, 1, 0, 1}, bin[8] = {2, 2, 1, 1, 0, 3, 0, 0};
            o.u |= pk_fld(3, PK_UB_R8) | pk_fld(1, PK_UB_FZ) | pk_fld(dir[y], PK_UB_RDIR) | pk_fld(bin[y], PK_UB_RBIN);
            if (y == 6) o.u |= pk_fld(1, PK_UB_SWAP);
            else o.u |= pk_fld(2, PK_UB_FC);
            pk_flags(o, 0, 0);
            break;
        }
        case 1:  // BIT: Z = !(X & bit), H = 1, C kept
            o.k |= pk_fld(1u << y, PK_KB_YCONST);
            o.u |= pk_fld(2, PK_UB_R8) | pk_fld(0, PK_UB_LOP) | pk_fld(1, PK_UB_FZ);
            pk_flags(o, PK_F_C, PK_F_H);
            break;
        case 2:  // RES = X & ~bit
            o.k |= pk_fld(0xFFu & ~(1u << y), PK_KB_YCONST);
            o.u |= pk_fld(2, PK_UB_R8) | pk_fld(0, PK_UB_LOP);
            break;
        default:  // SET = X | bit
            o.k |= pk_fld(1u << y, PK_KB_YCONST);
            o.u |= pk_fld(2, PK_UB_R8) | pk_fld(2, PK_UB_LOP);
            break;
    }
    return o;
}

// the whole table: [0,256) base, [256,512) CB-prefixed, then the three pseudo-ops
static inline uint32_t pk_has_res8(uint32_t s) {   // a writeback selector taking val byte 3 (result8)
    for (int b = 0; b < 4; b++)
        if (((s >> (8 * b)) & 0xFFu) == 0x07u) return 1u;
    return 0u;
}
static inline void pk_store_uop(uint32_t* e, PkUop o, bool real) {
    for (int w = 0; w < (int)PK_UE_WORDS; w++) e[w] = 0;
    // CPU state update as (cpu & keep) | set: IME from DI/EI/RETI/INT, HALT, CRASH; an executed
    // instruction clears QUEUED (pyboy cpu.tick), the pseudo-ops keep it
    uint32_t cpu_keep = 0xFu, cpu_set = 0u;
    {
        const uint32_t ime = (o.d >> PK_DB_IME) & 3u;
        if (real) cpu_keep &= ~4u;
        if (ime == 1u) cpu_keep &= ~1u;
        if (ime == 2u) cpu_set |= 1u;
        if (o.d & pk_fld(1, PK_DB_HALT)) cpu_set |= 2u;
        if (o.d & pk_fld(1, PK_DB_CRASH)) cpu_set |= 2u | 8u;
    }
    uint32_t us = 0, jrm = 0;
    uint32_t yc = o.k & 0xFFu, yx = 0, cw = 0, ci = 0;
    const uint32_t r8 = (o.u >> PK_UB_R8) & 3u, lop = (o.u >> PK_UB_LOP) & 3u, fcs = (o.u >> PK_UB_FC) & 3u;
    const bool sub = (o.u & pk_fld(1, PK_UB_SUB)) != 0u, usec = (o.u & pk_fld(1, PK_UB_USEC)) != 0u;
    const bool w16 = (o.u & pk_fld(1, PK_UB_W16)) != 0u, wr = (o.d & pk_fld(1, PK_DB_WR)) != 0u;
    // jump targets through the operand pools: JP/CALL/INT nn -> Y = nn, JP HL -> X = HL,
    // RET -> Y = m16, RST -> Y = yconst (the vector), JR -> pc + len + (Y = sign-extended e)
    const uint32_t ts = (o.d >> PK_DB_TSRC) & 7u;
    if (ts != PK_T_NONE) {
        us |= pk_fld(1, PK_US_JUMP);
        o.u &= ~(pk_fld(1, PK_UB_XSP) | pk_fld(1, PK_UB_XMEM) | pk_fld(1, PK_UB_YIMM) | pk_fld(1, PK_UB_IMM8) |
                 pk_fld(1, PK_UB_SEXT) | pk_fld(1, PK_UB_YMEM));
        o.px = PK_PZERO;
        o.py = PK_PZERO;
        if (ts == PK_T_IMM) o.u |= pk_fld(1, PK_UB_YIMM);
        if (ts == PK_T_HL) o.px = pk_sel16(2);
        if (ts == PK_T_M16) o.u |= pk_fld(1, PK_UB_YMEM);
        if (ts == PK_T_JR) { o.u |= pk_fld(1, PK_UB_YIMM) | pk_fld(1, PK_UB_SEXT); jrm = 0xFFFFu; }
        if (ts != PK_T_RST) yc = 0;
    }
    o.d &= ~(7u << PK_DB_TSRC);
    // 16-bit writes: the value is X (PUSH: the pair, LD (nn),SP: SP) or the return PC; pushes go to
    // SP-2 (low byte) and SP-1 (high byte), the slow path writes the high byte first as PyBoy does
    bool push = false;
    if (w16) {
        us |= pk_fld(1, PK_US_W16);
        if (o.u & pk_fld(1, PK_UB_WPC)) us |= pk_fld(1, PK_US_WPC);
        else if (o.u & pk_fld(1, PK_UB_WSP)) o.u |= pk_fld(1, PK_UB_XSP);
        else { o.px = o.py; o.py = PK_PZERO; }   // PUSH rr: X = the pair
        if (((o.d >> PK_DB_ADIR) & 3u) == 3u) {   // adir -1: a push
            push = true;
            o.d = (o.d & ~(15u << PK_DB_AOFF)) | pk_sfld(-2, PK_DB_AOFF, 2) | pk_sfld(1, PK_DB_ADIR, 2);
            us |= pk_fld(1, PK_US_HIFIRST);
        }
    }
    (void)push;
    // result8: loads (builder R8 = 0, Y) go through the logic unit as 0xFF AND Y when result8 is used
    if (r8 == 0u && (pk_has_res8(o.s0) || pk_has_res8(o.s1) || (wr && !w16))) {
        o.px = 0x0C0C0C0Du;
        o.u &= ~(pk_fld(1, PK_UB_XSP) | pk_fld(1, PK_UB_XMEM));
        us |= pk_fld(1, PK_US_LOGIC) | pk_fld(1, PK_US_LAND);
    }
    if (r8 == 2u) {
        us |= pk_fld(1, PK_US_LOGIC) | pk_fld(lop != 1u ? 1u : 0u, PK_US_LAND) | pk_fld(lop != 0u ? 1u : 0u, PK_US_LXOR);
    }
    if (sub) yx = 0x1FFFFu;
    // carry-in of the adder: SUB ^ (USEC & F.C)
    if (usec) { cw = 1u << 20; ci = sub ? (1u << 20) : 0u; }
    else if (sub) { cw = 1u << 16; ci = 1u << 16; }
    const uint32_t rbin = (o.u >> PK_UB_RBIN) & 3u;
    if (r8 == 3u) {
        const bool rdir = (o.u & pk_fld(1, PK_UB_RDIR)) != 0u;
        if (o.u & pk_fld(1, PK_UB_SWAP)) {
            us |= pk_fld(1, PK_US_RIGHT) | pk_fld(1, PK_US_SWAP);
        } else if (rdir) {   // RRC RRCA RR RRA SRA SRL: shifted-in bit 0 / F.C / bit 0 (rotated out) / bit 7
            static const uint32_t rb[4] = {0u, 1u << 20, 1u << 0, 1u << 7};
            us |= pk_fld(1, PK_US_RIGHT);
            cw = rb[rbin];
        } else {             // RLC RLCA RL RLA SLA: the adder, X + X + (0 / F.C / bit 7)
            static const uint32_t lb[4] = {0u, 1u << 20, 1u << 7, 0u};
            o.py = o.px;
            if (o.u & pk_fld(1, PK_UB_XMEM)) o.u |= pk_fld(1, PK_UB_YMEM);
            cw = lb[rbin];
            ci = 0;
        }
    }
    if (fcs == 3u) {   // CCF: C = !F.C through the adder, 0xFF + 0 + !F.C
        o.px = 0x0C0C0C0Du;
        cw = 1u << 20;
        ci = 1u << 20;
    }
    if (o.u & pk_fld(1, PK_UB_HC16)) us |= pk_fld(1, PK_US_HSH8);
    if (o.u & pk_fld(1, PK_UB_FPOP)) us |= pk_fld(1, PK_US_FPOP);
    if (o.u & pk_fld(1, PK_UB_R16HL)) us |= pk_fld(1, PK_US_R16HL);
    if (o.u & pk_fld(1, PK_UB_SPW)) us |= pk_fld(1, PK_US_SPW);
    us |= o.u & ((3u << PK_UB_HLINC) | (7u << PK_UB_SPD));   // same positions as PK_US_HLINC / PK_US_SPD
    // flags: F' = (F & FK) | ((Z | H | C | FC) & FM)
    const uint32_t fkeep = (o.k >> PK_KB_FKEEP) & 0xFFu, fconst = (o.k >> PK_KB_FCONST) & 0xFFu;
    uint32_t fm = fconst;
    if (o.u & pk_fld(1, PK_UB_FZ)) fm |= 0x80u;
    if (o.u & pk_fld(1, PK_UB_FH)) fm |= 0x20u;
    if (fcs != 0u) fm |= 0x10u;
    // operand sources -> ext-pool selectors (the register-pool selector is zeroed when unused);
    // a memory operand is m0 for one-byte reads, m0|m1 for two
    const bool rd2 = (o.d & pk_fld(1, PK_DB_RD2)) != 0u;
    uint32_t xe = PK_PZERO, ye = PK_PZERO, ae = PK_PZERO;
    if (o.u & pk_fld(1, PK_UB_XSP)) xe = PK_E_SP;
    else if (o.u & pk_fld(1, PK_UB_XMEM)) xe = PK_E_M0;
    if (o.u & pk_fld(1, PK_UB_YIMM)) ye = (o.u & pk_fld(1, PK_UB_SEXT)) ? PK_E_SEXTN : (o.u & pk_fld(1, PK_UB_IMM8)) ? PK_E_N : PK_E_NN;
    else if (o.u & pk_fld(1, PK_UB_YMEM)) ye = rd2 ? PK_E_M16 : PK_E_M0;
    else if (o.d & pk_fld(1, PK_DB_YSP)) ye = PK_E_SP;
    if (o.d & pk_fld(1, PK_DB_ASP)) ae = PK_A_SP;
    else if (o.d & pk_fld(1, PK_DB_AIMM)) ae = (o.d & pk_fld(1, PK_DB_AHN)) ? PK_E_HN : PK_E_NN;
    e[PK_UE_D] = o.d & ~(pk_fld(1, PK_DB_ASP) | pk_fld(1, PK_DB_AIMM) | pk_fld(1, PK_DB_AHN) | pk_fld(1, PK_DB_YSP));
    if ((o.d & pk_fld(1, PK_DB_RD)) && !rd2) e[PK_UE_D] |= pk_fld(1, PK_DB_RD1);
    // a secondary op may be fused after this one: executed instructions without control transfer,
    // IME/HALT/STOP changes or the rare DAA path (pk_u2_entry states the remaining conditions)
    if (!(real && ts == PK_T_NONE && !(o.d & (pk_fld(3, PK_DB_IME) | pk_fld(1, PK_DB_HALT) | pk_fld(1, PK_DB_CRASH) |
                                              pk_fld(1, PK_DB_DAA))) && (o.d & 3u) != 0u))
        e[PK_UE_D] |= pk_fld(1, PK_DB_NOFUSE);
    e[PK_UE_U] = us;
    e[PK_UE_K] = fconst | (fkeep << 8) | (fm << 16) | (cpu_keep << 24) | (cpu_set << 28);
    const uint32_t len = o.d & 3u;
    const uint32_t succ = (e[PK_UE_D] & pk_fld(1, PK_DB_NOFUSE)) ? 0x0C0Du : (len | ((len + 1u) << 8));
    e[PK_UE_V] = succ | ((((o.d >> PK_DB_CYC) & 7u) * 4u) << 16) | ((((o.d >> PK_DB_XCYC) & 3u) * 4u) << 24);
    e[PK_UE_XR] = xe != PK_PZERO ? PK_PZERO : o.px;
    e[PK_UE_XE] = xe;
    e[PK_UE_YR] = ye != PK_PZERO ? PK_PZERO : o.py;
    e[PK_UE_YE] = ye;
    e[PK_UE_AR] = ae != PK_PZERO ? PK_PZERO : o.pa;
    e[PK_UE_AE] = ae;
    e[PK_UE_S0] = o.s0;
    e[PK_UE_S1] = o.s1;
    e[PK_UE_YC] = yc | (jrm << 16);
    e[PK_UE_YX] = yx;
    e[PK_UE_CW] = cw;
    e[PK_UE_CI] = ci;
}

// ---- secondary ops: fused into the iteration of the instruction before them ----
// The SIMT loop pays for one iteration per emulated instruction whatever the instruction, so the
// cheap register-only successors of an instruction run in the same iteration: a JR (cc), LD r,r',
// LD r,n, INC/DEC r, INC/DEC BC/DE/HL, an 8-bit ALU op on A with a register or immediate operand
// (ADD ADC SUB SBC AND XOR OR CP), CPL, SCF or NOP right after a fusable instruction executes on
// the registers and flags that instruction left, exactly as the next cpu.tick would, when nothing
// can happen in between (pk_step.hip states the test).  Index = the successor's opcode (256
// entries).  A primary with PK_DB_NOFUSE selects index PK_U2_NONE = 0xFF for its successor
// whatever the bytes (its V word's successor selector yields 0xFF): that index is also RST 38h's
// own entry, which must therefore stay empty (length 0) — RST is a control transfer, never a
// secondary op; tests/test_ucode_table.py checks both.  Entry, two uint4:
//   a.x  X selector over w1:w0 (the pair, or a register into byte 0; JR: the F mask at F's byte)
//   a.y  misc: length, cycles, delta, JR condition value, mask of the F bits the op writes
//   a.z/a.w  writeback selectors of val2 = res16 | F' << 16 | res8 << 24 (as S0/S1)
//   b.x  Y selector over w1:w0 (register operand), b.y immediate mask (Y |= n & b.y), b.z Y xor
//        mask (0xFF: subtract), b.w control (PK_U2C_*)
// datapath: r = X + (Y ^ b.z) + delta + carry-in; res = r, or the logic unit's X&Y / X^Y / X|Y;
// flags Z from res, H/C from the adder's carry vector (^ flip, & mask), constants ORed in.
#define PK_U2B_LEN 0      // 2 bits length (0: no secondary op)
#define PK_U2B_ONE 2      // 1: counts as an executed instruction
#define PK_U2B_CYC 4      // 4 bits cycles (JR: not taken; at most 8)
#define PK_U2B_DELTA 8    // 8 bits signed: added to Y (INC/DEC)
#define PK_U2B_CV 16      // 8 bits: JR taken when (F & mask) == cv, the mask in byte 2 of the x word;
                          //         1 for every other entry (F's low nibble is 0: never)
#define PK_U2B_FM 24      // 8 bits: F bits the op writes, the rest kept
#define PK_U2_NONE_Y (1u << PK_U2B_CV)
#define PK_U2C_USEC 0     // carry-in F.C (ADC, SBC)
#define PK_U2C_SUBC 1     // carry-in ^ 1 (SUB, SBC, CP: X + ~Y + 1 [- C])
#define PK_U2C_LOGIC 2    // res = logic unit
#define PK_U2C_LA 3       // logic includes X & Y (AND, OR)
#define PK_U2C_LX 4       // logic includes X ^ Y (XOR, OR, CPL)
#define PK_U2C_FCONST 8   // 8 bits: F bits set (N of SUB/DEC/CP, H of AND, CPL/SCF constants)
#define PK_U2C_HCM 16     // 8 bits: F bits taken from the adder (H 0x20, C 0x10)
#define PK_U2C_FLIP 24    // 8 bits: adder flags inverted (borrow = !carry)
static inline void pk_u2_entry(uint32_t* e, int op) {
    uint32_t len = 0, cyc = 0, cv = 1, fm = 0, ysel = PK_PZERO, imm = 0, ysm = 0, ctl = 0;
    int delta = 0;
    PkUop o = pk_uop_base(1, 4);   // identity writeback selectors (F from val2 = F' = F unless fm)
    uint32_t sel = PK_PZERO;
    const int src = op & 7, dst = (op >> 3) & 7;
    if (op < 256) {
        if (op == 0x00) {
            len = 1; cyc = 4;
        } else if (op >= 0x40 && op < 0x80 && op != 0x76 && src != 6 && dst != 6) {  // LD r, r'
            len = 1; cyc = 4;
            sel = pk_sel8(src);
            pk_wb_r8(o, dst);
        } else if ((op & 0xC7) == 0x06 && dst != 6) {  // LD r, n
            len = 2; cyc = 8;
            imm = 0xFFu;
            pk_wb_r8(o, dst);
        } else if ((op & 0xC6) == 0x04 && dst != 6) {  // INC r / DEC r: Z N H, C kept
            len = 1; cyc = 4; fm = 0xE0;
            sel = pk_sel8(dst);
            delta = (op & 1) ? -1 : 1;
            ctl = pk_fld(PK_F_H, PK_U2C_HCM) | ((op & 1) ? pk_fld(PK_F_H, PK_U2C_FLIP) | pk_fld(PK_F_N, PK_U2C_FCONST) : 0u);
            pk_wb_r8(o, dst);
        } else if ((op & 0xC7) == 0x03 && ((op >> 4) & 3) != 3) {  // INC rr / DEC rr (BC DE HL), no flags
            const int p = (op >> 4) & 3;
            len = 1; cyc = 8;
            sel = pk_sel16(p);
            delta = (op & 8) ? -1 : 1;
            pk_wb_r16(o, p);
        } else if ((op >= 0x80 && op < 0xC0 && src != 6) || (op & 0xC7) == 0xC6) {  // ALU A, r / ALU A, n
            const int f = dst;   // ADD ADC SUB SBC AND XOR OR CP
            const bool immop = op >= 0xC0;
            len = immop ? 2 : 1; cyc = immop ? 8 : 4; fm = 0xF0;
            sel = pk_sel8(7);
            if (immop) imm = 0xFFu;
            else ysel = pk_sel8(src);
            if (f < 4 || f == 7) {   // adder: Z N H C
                const bool sub = f == 2 || f == 3 || f == 7;
                ysm = sub ? 0xFFu : 0u;
                ctl = pk_fld(PK_F_H | PK_F_C, PK_U2C_HCM) | ((f == 1 || f == 3) ? pk_fld(1, PK_U2C_USEC) : 0u)
                    | (sub ? pk_fld(1, PK_U2C_SUBC) | pk_fld(PK_F_H | PK_F_C, PK_U2C_FLIP) | pk_fld(PK_F_N, PK_U2C_FCONST) : 0u);
            } else {                 // logic: Z 0 H(AND) 0
                ctl = pk_fld(1, PK_U2C_LOGIC) | (f != 5 ? pk_fld(1, PK_U2C_LA) : 0u) | (f != 4 ? pk_fld(1, PK_U2C_LX) : 0u)
                    | (f == 4 ? pk_fld(PK_F_H, PK_U2C_FCONST) : 0u);
            }
            if (f != 7) pk_wb_r8(o, 7);
        } else if (op == 0x2F) {  // CPL: A ^ 0xFF, N H set
            len = 1; cyc = 4; fm = PK_F_N | PK_F_H;
            sel = pk_sel8(7);
            ysm = 0xFFu;
            ctl = pk_fld(1, PK_U2C_LOGIC) | pk_fld(1, PK_U2C_LX) | pk_fld(PK_F_N | PK_F_H, PK_U2C_FCONST);
            pk_wb_r8(o, 7);
        } else if (op == 0x37) {  // SCF: N H cleared, C set
            len = 1; cyc = 4; fm = PK_F_N | PK_F_H | PK_F_C;
            ctl = pk_fld(PK_F_C, PK_U2C_FCONST);
        } else if (op == 0x18 || op == 0x20 || op == 0x28 || op == 0x30 || op == 0x38) {  // JR (cc,) e
            static const uint32_t msk[4] = {0x80, 0x80, 0x10, 0x10}, val[4] = {0, 0x80, 0, 0x10};  // NZ Z NC C
            len = 2; cyc = 8;   // + 4 when taken
            sel = op == 0x18 ? 0u : msk[(op >> 3) & 3] << 16;   // JR e: mask 0 -> always taken
            cv = op == 0x18 ? 0u : val[(op >> 3) & 3];
        }
    }
    e[0] = sel;
    e[1] = (len << PK_U2B_LEN) | ((len ? 1u : 0u) << PK_U2B_ONE) | (cyc << PK_U2B_CYC)
         | (((uint32_t)delta & 0xFFu) << PK_U2B_DELTA) | (cv << PK_U2B_CV) | (fm << PK_U2B_FM);
    e[2] = o.s0;
    e[3] = o.s1;
    e[4] = ysel;
    e[5] = imm;
    e[6] = ysm;
    e[7] = ctl;
}

static inline void pk_build_ucode(uint32_t* t /* PK_UC_WORDS */) {
    for (int i = 0; i < 512; i++) {
        PkUop o = i < 256 ? pk_uop(i) : pk_uop_cb(i - 256);
        if (i == 0xCB) o = pk_uop_base(2, 8);  // never executed: the kernel indexes 256 + second byte
        pk_store_uop(t + (size_t)i * PK_UE_WORDS, o, true);
    }
    // INT: push PC (len 0: the current PC), jump to the vector the front-end puts in imm16, IME off
    PkUop it = pk_uop_base(0, 0);
    it.d |= pk_fld(PK_T_IMM, PK_DB_TSRC) | pk_fld(1, PK_DB_WR) | pk_fld(1, PK_DB_WR2) | pk_fld(1, PK_DB_ASP)
          | pk_sfld(-1, PK_DB_AOFF, 2) | pk_sfld(-1, PK_DB_ADIR, 2) | pk_fld(1, PK_DB_IME);
    it.u |= pk_fld(1, PK_UB_W16) | pk_fld(1, PK_UB_WPC) | pk_sfld(-2, PK_UB_SPD, 3);
    PkUop idle = pk_uop_base(0, 4), nop0 = pk_uop_base(0, 0);
    const PkUop ps[3] = {it, idle, nop0};
    for (int j = 0; j < 3; j++) pk_store_uop(t + (size_t)(512 + j) * PK_UE_WORDS, ps[j], false);
    for (int op = 0; op <= (int)PK_U2_NONE; op++) pk_u2_entry(t + PK_UC_U2 + (size_t)op * PK_U2_WORDS, op);
}
