// pk_layout.h — device data layout shared by the HIP kernels and the host C-ABI.
//
// One wavefront lane = one emulator ("env").  Envs are grouped 64 to a "group".
//
// Per-env RAM image ("phys" address space, PK_PHYS bytes), stored LANE-INTERLEAVED per group, with
// an interleave W = 1 << sh (sh <= 6) chosen per handle = K1's envs per wave (16, 32 or 64): a
// group's PK_GROUP_STRIDE bytes hold 64 / W sub-blocks of W envs, and inside a sub-block
//     byte(env, phys) = sub-block base[phys * W + env % W]          (pk_img_off)
// so the W lanes of a wave touching the same guest address (the common case while they run the
// same code) hit W consecutive bytes — one coalesced access — no 64-byte line is shared by two
// waves, and a 128-byte line holds 128 / W consecutive guest bytes of the wave's envs.  (W = 64 is
// the round-1/2 layout.)
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
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef struct { uint32_t x, y; } uint2_t;

#define PK_LANES 64u
#define PK_PHYS 0xC200u
// sub-block skew: every sub-block starts PK_SKEW bytes after the end of the previous one, so the
// same guest byte of consecutive sub-blocks (waves) is not at the same offset modulo the memory
// channel interleave (PK_PHYS << sh is a multiple of 16 KiB for sh >= 5)
#ifndef PK_SKEW
#define PK_SKEW 0u
#endif
// bytes of one 64-env group: the largest over the interleaves (sh = 0: 64 sub-blocks)
#define PK_GROUP_STRIDE (PK_PHYS * PK_LANES + PK_SKEW * PK_LANES)

// sub-block stride and group stride of interleave 1 << sh
__host__ __device__ static inline uint64_t pk_sub_stride(uint32_t sh) { return ((uint64_t)PK_PHYS << sh) + PK_SKEW; }
__host__ __device__ static inline uint64_t pk_group_stride(uint32_t sh) { return (uint64_t)(PK_LANES >> sh) * pk_sub_stride(sh); }

// byte offset of (env, phys) in the image array, interleave 1 << sh
__host__ __device__ static inline uint64_t pk_img_off(uint32_t env, uint32_t phys, uint32_t sh) {
    const uint32_t l = env & (PK_LANES - 1u);
    return (uint64_t)(env / PK_LANES) * pk_group_stride(sh) + (uint64_t)(l >> sh) * pk_sub_stride(sh)
         + ((uint64_t)phys << sh) + (l & ((1u << sh) - 1u));
}

#define PK_P_VRAM 0x0000u
#define PK_P_WRAM 0x2000u
#define PK_P_OAM 0x4000u
#define PK_P_IO 0x4100u
#define PK_P_HRAM 0x4180u
#define PK_P_SRAM 0x4200u
#define PK_P_UNUSED 0x41FFu   // no guest byte (IE lives in lane regs): K1's dummy store target.
                              // K1's branch-free write stage stores a changing byte here every
                              // iteration, so nothing may read it: the v9 export/import and every
                              // image digest cover HRAM as 0x4180-0x41FE only (127 bytes) and take
                              // IE from the cpu register (pk_capi.cpp export_v9 / import_v9).
                              // The 64-bank parity tests (test_hostsim_game_64_banks,
                              // test_game_rom_64_banks_parity) would fail if an export read it: that
                              // instance stores unmodelled values here in every iteration

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
    PK_R_RFLAGS,     // render bookkeeping of the last step: blank<<0 | (lines left for K2)<<8
    PK_NREGS
};

// diagnostic buffer (-DPK_STAMP phase counters; -DPK_WAVETIME adds one PK_WT_REC-word record per K1 wave)
#ifdef PK_WAVETIME
#define PK_WT_REC 6u
#define PK_DBG_WORDS (64u + PK_WT_REC * 16384u)
#else
#define PK_DBG_WORDS 64u
#endif

// K1's LDS budget.  The default kernel stages PK_LDS_SLOTS ROM banks (16 KiB each, slot 0 = bank 0)
// and the HRAM code mirror of up to PK_WG_ENVS envs: 158 KB, one workgroup per CU, 512 threads =
// 8 waves, two per SIMD at ~233 VGPRs.  The small-LDS kernel (pk_step.hip compiled a second time
// with PK_K1_SMALL) stages 2 banks and the mirror of 128 envs in 256-thread workgroups: 78.7 KB, so
// two workgroups fit on a CU.  pk_capi.cpp launches it for the ranges of concurrent sub-batches
// (VecEnv), whose workgroups can then start on a CU where the other sub-batch is still in its tail.
#define PK_SMALL_LDS_SLOTS 2u
#define PK_SMALL_WG_ENVS 128u
#define PK_SMALL_MAX_THREADS 256
#ifdef PK_K1_SMALL
#define PK_WG_ENVS PK_SMALL_WG_ENVS
#define PK_LDS_SLOTS PK_SMALL_LDS_SLOTS
#define PK_K1_MAX_THREADS PK_SMALL_MAX_THREADS
#endif
#ifndef PK_K1_MAX_THREADS
#define PK_K1_MAX_THREADS 512
#endif
#ifndef PK_WG_ENVS
#define PK_WG_ENVS 512u
#endif
#ifndef PK_LDS_SLOTS
#define PK_LDS_SLOTS 6u
#endif

// kernel argument blocks (passed by value)
struct PkStepArgs {
    uint8_t* mem;             // lane-interleaved RAM images
    const uint8_t* rom;       // whole ROM (+16 bytes of padding: dword fetches may overrun the end)
    const uint32_t* romw;     // the same, as dwords
    uint32_t* regs;           // SoA lane registers [PK_NREGS][npad]
    const uint32_t* ucode;    // microcode table (pk_ucode.h), PK_UC_ENTRIES x 8 dwords
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
    uint32_t wave_lanes;      // envs per 64-lane wave in K1 (64, 32 or 16): fewer lanes = more waves/SIMD
    uint32_t simds;           // SIMDs of the device: K1 uses 256-thread workgroups while waves <= simds
    uint32_t block;           // K1 workgroup size override (0 = by geometry; PK_K1_BLOCK, tests)
    uint32_t prio;            // K1 wave-priority variant (two waves per SIMD; PK_K1_PRIO overrides)
    unsigned long long* dbg;  // diagnostic counters (-DPK_STAMP builds only), else null
    uint32_t env0, env1;      // env range of this launch: [env0, env1), env0 % 64 == 0 (sub-batches)
    uint32_t ilv_sh;          // image interleave: 1 << ilv_sh envs (pk_img_off)
    uint32_t small;           // launch the small-LDS K1 (pk_launch_step_small)
    uint32_t all_staged;      // every ROM bank is staged in this kernel's LDS slots (the ALL instance)
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
    const uint32_t* cnt;         // envs to reset: count (device memory) ...
    const uint32_t* ids;         // ... and their ids (pk_list_kernel)
    uint32_t n, npad, lat_stride;
    uint32_t env0, env1;         // env range the list was built over
    uint32_t ilv_sh;             // image interleave (pk_img_off)
};
