// pk_layout.h — device data layout shared by the HIP kernels and the host C-ABI.
//
// One wavefront lane = one emulator ("env").  Envs are grouped 64 to a "group" (= one wave).
//
// Per-env RAM image ("phys" address space, PK_PHYS bytes), stored LANE-INTERLEAVED per group:
//     byte(env, phys) = mem[group(env) * PK_GROUP_STRIDE + phys * 64 + lane(env)]
// so the 64 lanes of a wave touching the same guest address (the common case while they run
// the same code) hit 64 consecutive bytes — one coalesced access — and a group's whole state is
// one contiguous 3.0 MiB block of HBM.
//
//   phys 0x0000-0x1FFF  VRAM   (guest 0x8000-0x9FFF)
//   phys 0x2000-0x3FFF  WRAM   (guest 0xC000-0xDFFF, echo 0xE000-0xFDFF)
//   phys 0x4000-0x409F  OAM    (guest 0xFE00-0xFE9F)
//   phys 0x40A0-0x40FF  unusable RAM (guest 0xFEA0-0xFEFF)
//   phys 0x4100-0x414B  IO ports backing store (guest 0xFF00-0xFF4B; special regs live in lane regs)
//   phys 0x414C-0x417F  non-IO RAM (guest 0xFF4C-0xFF7F)
//   phys 0x4180-0x41FE  HRAM   (guest 0xFF80-0xFFFE); 0x41FF unused (IE lives in lane regs)
//   phys 0x4200-0xC1FF  cartridge SRAM, 4 banks x 8 KiB (guest 0xA000-0xBFFF)
//
// Per-env lane registers: SoA u32 arrays regs[field * npad + env] (coalesced load/store at
// kernel entry/exit; inside the kernel they live in VGPRs).
#pragma once
#include <stdint.h>

typedef struct { uint32_t x, y; } uint2_t;
typedef struct { uint32_t desc, ucode, bytes, pad; } pk_rom_entry;  // 16-byte pre-decoded ROM entry

#define PK_LANES 64u
#define PK_PHYS 0xC200u
#define PK_GROUP_STRIDE (PK_PHYS * PK_LANES)

#define PK_P_VRAM 0x0000u
#define PK_P_WRAM 0x2000u
#define PK_P_OAM 0x4000u
#define PK_P_IO 0x4100u
#define PK_P_HRAM 0x4180u
#define PK_P_SRAM 0x4200u

#define PK_ROWS 144u
#define PK_COLS 160u
#define PK_SCREEN (PK_ROWS * PK_COLS)

// lane register fields
enum {
    PK_R_W0 = 0,     // C | B<<8 | E<<16 | D<<24
    PK_R_W1,         // L | H<<8 | A<<16 | F<<24
    PK_R_SP,
    PK_R_PC,
    PK_R_CPU,        // ime | halted<<1 | queued<<2 | crashed<<3 | stopped<<4 | IE<<8 | IF<<16
    PK_R_CLOCK,      // PyBoy lcd.clock (always < 2^18 after the frame-wrap reduction)
    PK_R_TARGET,     // lcd.clock_target
    PK_R_LCD0,       // LCDC | STAT<<8 | LY<<16 | LYC<<24
    PK_R_LCD1,       // SCY | SCX<<8 | WY<<16 | WX<<24
    PK_R_LCD2,       // BGP | OBP0<<8 | OBP1<<16 | next_stat_mode<<24
    PK_R_TIM0,       // DIV | TIMA<<8 | TMA<<16 | TAC<<24
    PK_R_TIM1,       // DIV_counter | TIMA_counter<<16
    PK_R_MBC,        // rombank | rambank<<8 | ram_enabled<<16 | memorymodel<<24
    PK_R_MISC,       // joypad directional | standard<<8 | (ly_window+1)<<16 (u8)
    PK_R_TIME,       // env-steps since reset (pokegym `self.time`, environment.py:1338)
    PK_R_ICOUNT,     // emulated instructions in the last pk_step (perf counter)
    PK_R_RFLAGS,     // render bookkeeping of the last step: blank<<0 | pending-lines<<8
    PK_NREGS
};

// decode-table descriptor (u32), built on the host (pk_decode.h), staged in LDS by the kernel.
//   [0:6)  class           [6:8)  length          [8:12)  read mode     [12:16) write mode
//   [16:20) field a        [20:24) field b         [24:27) sub-op        [27:30) cycles/4
//   [30:32) extra cycles/4 when a condition is taken
#define PK_D_CLS(d) ((d) & 63u)
#define PK_D_LEN(d) (((d) >> 6) & 3u)
#define PK_D_RD(d) (((d) >> 8) & 15u)
#define PK_D_WR(d) (((d) >> 12) & 15u)
#define PK_D_A(d) (((d) >> 16) & 15u)
#define PK_D_B(d) (((d) >> 20) & 15u)
#define PK_D_OP(d) (((d) >> 24) & 7u)
#define PK_D_CYC(d) ((((d) >> 27) & 7u) * 4u)
#define PK_D_XCYC(d) ((((d) >> 30) & 3u) * 4u)

enum {  // memory addressing modes (read and write)
    PK_M_NONE = 0, PK_M_HL, PK_M_BC, PK_M_DE, PK_M_HLI, PK_M_HLD, PK_M_NN, PK_M_HN, PK_M_HC,
    PK_M_SP2,    // read:  [SP], [SP+1]          (POP/RET)
    PK_M_PUSH2,  // write: [SP-1]=hi, [SP-2]=lo  (PUSH/CALL/RST/interrupt)
    PK_M_NN2     // write: [nn]=lo, [nn+1]=hi    (LD (nn),SP)
};

// datapath classes: class = family << 3 | index, so the kernel dispatches on 6 families and
// computes the classes inside a family with selects (no per-opcode branches).
enum {
    PK_C_LD8 = 0x00,                                                     // family 0: loads
    PK_C_ALU = 0x08, PK_C_INC8, PK_C_DEC8,                               // family 1: 8-bit arithmetic
    PK_C_ROTA = 0x10, PK_C_CBROT, PK_C_BIT, PK_C_RES, PK_C_SET, PK_C_DAA, PK_C_CPL,
    PK_C_SCFCCF,                                                         // family 2: bit/rotate/misc 8-bit
    PK_C_LD16 = 0x18, PK_C_INCDEC16, PK_C_ADDHL, PK_C_ADDSPE, PK_C_LDSPHL, PK_C_LDNNSP, PK_C_PUSH,
    PK_C_POP,                                                            // family 3: 16-bit
    PK_C_JP = 0x20, PK_C_JPHL, PK_C_JR, PK_C_CALL, PK_C_RET, PK_C_RETI, PK_C_RST,
    PK_C_INT,                                                            // family 4: control flow
    PK_C_NOP = 0x28, PK_C_DI, PK_C_EI, PK_C_HALT, PK_C_ILLEGAL           // family 5: misc
};
#define PK_FAMILY(cls) ((cls) >> 3)

// second descriptor word: microcode controlling the fused (branch-free) datapath
#define PK_U_R8SEL(u) ((u) & 15u)           // result8: 0 keep 1 Y 2 ADD 3 LOGIC 4 ROT 5 RES 6 SET 7 DAA 8 CPL
#define PK_U_DST8(u) (((u) >> 4) & 3u)      // 0 none, 1 A, 2 r[fa] (mem if fa==6)
#define PK_U_XTGT(u) (((u) >> 6) & 1u)      // X = tgt (r[fa]/m0) instead of A
#define PK_U_YONE(u) (((u) >> 7) & 1u)      // Y = 1 (INC/DEC)
#define PK_U_ARITH(u) (((u) >> 8) & 3u)     // adder: 0 from ALU sub-op, 1 INC, 2 DEC
#define PK_U_FMODE(u) (((u) >> 10) & 15u)   // flags: see PK_F_*
#define PK_U_OP16(u) (((u) >> 14) & 15u)    // 16-bit op: see PK_O_*
#define PK_U_CTRL(u) (((u) >> 18) & 15u)    // control: see PK_K_*
#define PK_U_WSRC(u) (((u) >> 22) & 3u)     // write data: 0 res8, 1 push PC, 2 push pair, 3 SP lo/hi
#define PK_U_IME(u) (((u) >> 24) & 3u)      // 0 keep, 1 clear, 2 set
enum { PK_F_KEEP = 0, PK_F_ALU, PK_F_INCDEC, PK_F_ROTA, PK_F_CBROT, PK_F_BIT, PK_F_DAA, PK_F_CPL, PK_F_SCF,
       PK_F_CCF, PK_F_ADDHL, PK_F_ADDSPE, PK_F_POPAF };
enum { PK_O_NONE = 0, PK_O_LD16, PK_O_INC16, PK_O_DEC16, PK_O_ADDHL, PK_O_SPE_SP, PK_O_SPE_HL, PK_O_SPHL,
       PK_O_POP, PK_O_POPAF };
enum { PK_K_SEQ = 0, PK_K_JP, PK_K_JPHL, PK_K_JR, PK_K_CALL, PK_K_RET, PK_K_RETI, PK_K_RST, PK_K_INT,
       PK_K_HALT, PK_K_ILLEGAL };

#define PK_SRC_IMM 8u
#define PK_LDS_SLOTS 6u  // ROM banks (16 KiB each) staged in LDS by the step kernel  // field b of LD8/ALU: source is the immediate byte
#define PK_COND_ALWAYS 0u
#define PK_COND_FLAG 4u  // field a bit 2 set: conditional; bits 0..1 = nz,z,nc,c

// kernel argument blocks (passed by value)
struct PkStepArgs {
    uint8_t* mem;             // lane-interleaved RAM images
    const uint8_t* rom;       // whole ROM
    const pk_rom_entry* rom16; // pre-decoded ROM: per ROM byte {desc, ucode, op|b1<<8|b2<<16|slow<<24, 0}
    uint32_t* regs;           // SoA lane registers [PK_NREGS][npad]
    const uint32_t* dtab;     // 512 decode descriptors + 512 microcode words
    const uint8_t* actions;   // [n] action ids (0..7; >=8 = no button)
    uint32_t* lat;            // [3][ngroups*144*64] per-line render latches
    uint8_t* screen;          // [n][144][160] persistent grey screen
    uint32_t n, npad;
    uint32_t rom_bank_mask;
    uint32_t mbc;             // 0 = ROM only, 3 = MBC3
    uint32_t frames;          // frame_skip (24)
    uint32_t release_frame;   // 8
    uint32_t render_last;     // rasterise the last frame
    uint32_t lat_stride;      // ngroups*144*64
    uint32_t nslots;          // ROM banks staged in LDS (slot 0 = bank 0)
    const int8_t* bank_slot;  // [128] LDS slot of each ROM bank, -1 = not staged
    const uint8_t* slot_bank; // [PK_LDS_SLOTS] bank held by each slot
};

struct PkResetArgs {
    uint8_t* mem;
    uint32_t* regs;
    uint32_t* lat;
    uint8_t* screen;
    const uint8_t* tmpl_mem;     // PK_PHYS bytes
    const uint32_t* tmpl_regs;   // PK_NREGS
    const uint32_t* tmpl_lat;    // 3*144
    const uint8_t* tmpl_screen;  // 144*160
    const uint8_t* mask;         // [n] or null = all
    uint32_t n, npad, lat_stride;
};
