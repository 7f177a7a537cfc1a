// pk_step.hip — K1, the MI355X (gfx950) env.step kernel: 24 emulated DMG frames per env-step, one
// wavefront lane per emulator.  Replaces PyBoy's tick() loop as pokegym drives it in
// pokegym/pyboy_binding.py:71-91 (run_action_on_emulator: press, 24 ticks, release before tick 8,
// render only tick 24).  Semantics are pinned bit-exactly to the CPU oracle (oracle/gbcore.c,
// a restatement of PyBoy 1.x): cpu_tick / cpu_check_interrupts, cpu_execute, bus_read/bus_write,
// lcd_tick, timer_tick, the HALT fast-forward of gb_tick.
//
// SIMT design (one wave = 64 independent emulators that drift apart within a few frames, so any
// path a lane takes more than ~1 % of the time is executed by the wave almost every iteration):
//   * every lane runs the SAME straight-line sequence per emulated instruction: front-end
//     (interrupts/HALT) -> fetch (LDS-staged ROM) -> microcode entry (LDS, pk_ucode.h) -> address
//     -> read -> fused datapath -> register writeback (two v_perm_b32) -> write -> timer/LCD.
//     Selections are sel() on precomputed values (v_cndmask, not branch trees), and the hot loop
//     has only single-level `if`s without `else`: LLVM's structurizer turns else-if chains into
//     exec-mask bookkeeping that spilled SGPRs into VGPR lanes (measured: ~450 VALU per iteration).
//   * paths a lane takes rarely (code outside the staged ROM, IO registers, MBC, OAM DMA, SRAM,
//     deferred-line flush) sit in their own single-level `if`s and work on a copy of the lane
//     state.  (Out-of-line calls were tried: the call convention moved the loop's uniform pointers
//     into callee-saved VGPRs and turned the hot RAM accesses into flat loads — slower.)
//   * a halted CPU that nothing can wake before VBlank jumps there in one iteration (HALT
//     skip-ahead below) instead of one iteration per LCD mode event.
//   * ROM bank 0 + the hottest switchable banks and the microcode table live in LDS; the RAM
//     images are lane-interleaved in HBM (pk_layout.h) so lanes at the same guest address coalesce.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pk_layout.h"
#include "pk_render.h"
#include "pk_ucode.h"

#define FRAME_CYCLES 70224u
#define CPU_IME 1u
#define CPU_HALT 2u
#define CPU_QUEUED 4u
#define CPU_CRASH 8u
// kernel-internal: IE & IF & 0x1F != 0 (an interrupt is pending), kept in step by cpu_sync_pend
// wherever IE or IF change (all on rare paths) and cleared before the word is stored, so the loop
// top's rare test is one mask test of the word
#define CPU_PEND 0x20u
#define PK_NO_BANK 0xFFFFFFFFu


// debug hooks: the host-simulation build (tests/hostsim) records an instruction trace and
// per-iteration event bits; the gfx950 build compiles them away.
#ifndef PK_TRACE
#define PK_TRACE(env, pc, w0, w1, sp, op) ((void)0)
#endif
// a loop fast path ran `passes` whole passes of a `len`-instruction loop after the traced
// instruction (tools/trace_diff.py drops the oracle's records of those passes)
#ifndef PK_TRACE_SKIP
#define PK_TRACE_SKIP(env, pc, passes, len) ((void)0)
#endif
#ifndef PK_ITER
#define PK_ITER(env, ev) ((void)(ev))
#endif
// a fast-path RAM-image access (kind 0 read, 1 write) at image offset phys (host simulation:
// tools/mem_stats.py attributes K1's memory traffic to guest regions)
#ifndef PK_MEMREF
#define PK_MEMREF(env, kind, phys) ((void)0)
#endif
#ifndef PK_ITER_OP
#define PK_ITER_OP(env, di) ((void)0)
#endif
// invariants of the lane-cached derived state (pk_check_lane, run at every loop top): the host-
// simulation build defines PK_CHECK to record a failure; the gfx950 build compiles the checks away
#ifdef PK_CHECK
#define PK_CHECK_ON 1
#else
#define PK_CHECK_ON 0
#define PK_CHECK(env, cond, what) ((void)0)
#endif
// diagnostic build only (-DPK_STAMP, tools/stamp_build.py): per-phase wave cycles of the loop,
// read with s_memtime at points where the loop already waits, summed per wave into A.dbg
#ifdef PK_STAMP
#define PK_NSTAMP 12
#define PK_STAMP_AT(k)                                          \
    do {                                                        \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();       \
        st_acc[k] += (uint64_t)(t_ - st_prev);                  \
        st_prev = t_;                                           \
    } while (0)
// the stage functions take the accumulators as extra arguments
#define PK_STAMP_PARAMS , uint64_t* st_acc, uint64_t& st_prev
#define PK_STAMP_ARGS , st_acc, st_prev
#else
#define PK_STAMP_AT(k) ((void)0)
#define PK_STAMP_PARAMS
#define PK_STAMP_ARGS
#endif
enum {
    PK_EV_EXEC = 1u << 0, PK_EV_F_LDS = 1u << 1, PK_EV_F_ROM16 = 1u << 2, PK_EV_F_BUS = 1u << 3,
    PK_EV_INT = 1u << 4, PK_EV_IDLE = 1u << 5, PK_EV_RD = 1u << 6, PK_EV_RD_ROMLDS = 1u << 7,
    PK_EV_RD_ROMG = 1u << 8, PK_EV_RD_RAM = 1u << 9, PK_EV_RD_IO = 1u << 10, PK_EV_RD2 = 1u << 11,
    PK_EV_WR = 1u << 12, PK_EV_WR_SLOW = 1u << 13, PK_EV_WR2 = 1u << 14, PK_EV_LCD = 1u << 15,
    PK_EV_TIMER = 1u << 16, PK_EV_FRAME = 1u << 17, PK_EV_FLUSH = 1u << 18, PK_EV_HRAM = 1u << 19,
    PK_EV_JUMP = 1u << 20, PK_EV_CB = 1u << 21, PK_EV_FUSE = 1u << 22 /* 23..27: unused here */,
    PK_EV_RD_WRAM = 1u << 28, PK_EV_WR_WRAM = 1u << 29, PK_EV_WR_VRAM = 1u << 30, PK_EV_WR_HI = 1u << 31
};

// LDS, staged by each workgroup at kernel entry: one struct, so the layout is fixed — the ROM bytes
// first, at LDS address 0, so the fetch's ds_read2_b32 (8-bit dword offsets) takes the byte index
// as its address with no base add; the microcode reads fold the ROM array's size into their 16-bit
// offsets (small-LDS kernel; the whole-CU kernel's ROM is larger than the offset field)
// ROM banks (+ fetch overrun pad), then the HRAM code mirror (below): one byte array, so the
// next instruction's bytes come from one ds_read2_b32 whichever of the two holds them.
// Fetch-only mirror of the first PK_HC_ROWS bytes of HRAM (0xFF80-0xFF9F: where games put the
// OAM-DMA routine, pokered's hDMARoutine included), PK_HC_STRIDE bytes per env of the workgroup
// at PK_HC_BASE + local env * PK_HC_STRIDE, + one dummy byte: the OAM-DMA wait loop runs from HRAM,
// and fetching it from the HBM image put a second dependent HBM round trip (fetch, then data) into
// ~30 % of wave iterations.  Code elsewhere in HRAM is fetched from the image.  Data reads/writes
// stay on the image (authoritative); a plain-RAM write near the mirrored bytes also updates the
// mirror (near_hcode, a rare branch; the second byte of a one-byte write goes to the dummy byte).
// Up to 512 envs per workgroup: 64-env waves two per SIMD when a launch has the envs for it
// (>= 131,072).
#define PK_HC_ROWS 32u
#define PK_HC_STRIDE 36u
#define PK_HC_BASE (PK_LDS_SLOTS * 0x4000u + 16u)
struct PkLds {
    u8 rom[PK_HC_BASE + PK_WG_ENVS * PK_HC_STRIDE];   // ROM slots, then the HRAM mirror (a multiple of 16 B)
    u32 u2[PK_UC_WORDS - PK_UC_U2];                   // secondary ops (small-LDS kernel: base in the 16-bit offset)
    u32 uc[PK_UC_U2];                                 // microcode
    int8_t slot[128];                                 // bank -> slot
};
__shared__ __attribute__((aligned(16))) PkLds pk_lds;
#define lds_rom pk_lds.rom
#define lds_uc pk_lds.uc
#define lds_u2 pk_lds.u2
#define lds_slot pk_lds.slot

// ---------------------------------------------------------------------------------------------
// branch-free helpers: arguments are evaluated unconditionally, so ?: on them is a v_cndmask
__device__ __forceinline__ u32 sel(bool c, u32 a, u32 b) { return c ? a : b; }
__device__ __forceinline__ u32 cpu_sync_pend(u32 cpu) {
    return (cpu & ~CPU_PEND) | sel(((cpu >> 8) & (cpu >> 16) & 0x1Fu) != 0u, CPU_PEND, 0u);
}
// rare-path hint: the block is laid out away from the hot instruction stream (instruction fetch)
#define PK_RARE(x) __builtin_expect(!!(x), 0)
// keep three lane values materialised in VGPRs at this point (an empty asm that reads and
// rewrites them): stops LLVM from sinking their computation further down the loop body
#ifndef PK_PIN3
#define PK_PIN3(a, b, c) asm volatile("" : "+v"(a), "+v"(b), "+v"(c))
#endif
// make a lane value opaque to LLVM at this point (an empty asm that rewrites it in place)
#ifndef PK_OPAQUE
#define PK_OPAQUE(x) asm("" : "+v"(x))
#endif
// Drain the vector-memory counter (s_waitcnt vmcnt(0); expcnt/lgkmcnt untouched) at the end of a
// rare block.  gfx950 counts loads and stores on one in-order counter, and LLVM's wait insertion
// merges the paths into a loop header conservatively: a load left outstanding on a rare path (the
// block copy's batch loads past the copy's end, whose stores are skipped) made the common path wait
// for vmcnt(0) — i.e. for the previous iteration's byte stores — before issuing its operand read,
// every iteration.  Draining on the rare path keeps the store acknowledgements off the common path.
#ifndef PK_BF
#define PK_BF 1      // branch-free image stores in the unstaged-bank instance (pk_write)
#endif
#ifndef PK_NO_DRAIN
#define PK_VM_DRAIN() __builtin_amdgcn_s_waitcnt(0x0F70)
#else
#define PK_VM_DRAIN() ((void)0)
#endif
// TIMA input clock divider as a shift: TAC & 3 = 0/1/2/3 -> 1024/16/64/256 cycles
__device__ __forceinline__ u32 timer_shift(u32 tac) { return (0x0806040Au >> (8u * (tac & 3u))) & 0xFFu; }
__device__ __forceinline__ u32 bit(u32 w, int pos) { return (w >> pos) & 1u; }
__device__ __forceinline__ int sfield(u32 w, int pos, int bits) { return ((int)(w << (32 - pos - bits))) >> (32 - bits); }
__device__ __forceinline__ u32 perm(u32 hi, u32 lo, u32 s) { return __builtin_amdgcn_perm(hi, lo, s); }
// Lane selects on a microcode bit as masks: bmask = all ones / all zeros from bit pos of w (one
// v_bfe_i32), msel = m ? a : b for such a mask (one v_bfi_b32 / v_bitop3_b32) — one VALU less per
// condition than a compare into a lane mask + v_cndmask.  The empty asm keeps the mask opaque:
// LLVM would otherwise see a sign-extended bit and turn msel back into compare + select.
__device__ __forceinline__ u32 bmask(u32 w, int pos) {
    u32 m = (u32)((int)(w << (31 - pos)) >> 31);
    PK_OPAQUE(m);
    return m;
}
__device__ __forceinline__ u32 msel(u32 m, u32 a, u32 b) { return (a & m) | (b & ~m); }
// The initial value of a register that a divergent branch writes and that lanes outside the
// branch never read: any defined value will do, and a constant would cost a move per iteration.
// PK_UNREAD names a value that dies at that point, so the register allocator gives both one
// register and no instruction is issued (a reminder at the use site, not an operation).
#define PK_UNREAD(v) (v)

// lane state (VGPRs for the whole launch).  Never select between two fields by reference: that
// makes LLVM take field addresses and spill the struct to scratch.
struct St {
    u32 w0, w1, sp, pc;   // w0 = C|B<<8|E<<16|D<<24, w1 = L|H<<8|F<<16|A<<24 (kernel-internal order)
    u32 cpu;              // ime | halted<<1 | queued<<2 | crashed<<3 | stopped<<4 | IE<<8 | IF<<16
    u32 clock, target;    // lcd.clock, lcd.clock_target
    u32 lcd0, lcd1, lcd2; // LCDC|STAT<<8|LY<<16|LYC<<24, SCY|SCX<<8|WY<<16|WX<<24, BGP|OBP0<<8|OBP1<<16|next_mode<<24
    u32 tim0;             // (DIV stale) | TIMA<<8 | TMA<<16 | TAC<<24
    u32 divacc;           // DIV<<8 | DIV_counter: its low 16 bits (every reader takes a byte of them, so
                          // the sums need no mask)
    u32 timac;            // TIMA_counter
    u32 mbc;              // rombank | rambank<<8 | ram_enabled<<16 | memorymodel<<24
    u32 misc;             // joypad directional | standard<<8 | (ly_window+1)<<16
    u32 rb;               // LDS byte offset of the switchable ROM bank - 0x4000 (index = address + rb)
    u32 rlim;             // ROM addresses below it are staged: 0x8000, or 0x4000 when the bank is not
    u32 lim;              // tick_lim(): clock below it = no LCD event, no LCD-off frame end, timer off,
                          // no frame watchdog
    u32 npend;            // latched, not yet rasterised lines: 0 = none, else the range (pk_render.h pend_add)
    u32 prow;             // tile-map rows those lines read, either map: bit r = row r (pend_hit)
    u32 render, blank, frame_done;
};

// where this lane's emulator lives
struct Ctx {
    const PkStepArgs* A;
    u8* g;                // this env's image sub-block (pk_layout.h: byte(phys) = g[phys << sh | lane])
    u32 lane, sh;         // lane within the sub-block, interleave shift
    u32 glane, env, gid;  // lane within the 64-env group (render latches), env, group
    u32 loc;              // env index within the workgroup (HRAM mirror column)
};

__device__ __forceinline__ u32 ld_img(const Ctx& c, u32 phys) { return c.g[(phys << c.sh) + c.lane]; }
__device__ __forceinline__ void st_img(const Ctx& c, u32 phys, u32 v) { c.g[(phys << c.sh) + c.lane] = (u8)v; }
// keep the HRAM fetch mirror in step with a RAM write at guest address a (row PK_HC_ROWS = dummy)
__device__ __forceinline__ void hcode_st(const Ctx& c, u32 a, u32 v) {
    const u32 row = sel(a - 0xFF80u < PK_HC_ROWS, a - 0xFF80u, PK_HC_ROWS);
    lds_rom[PK_HC_BASE + c.loc * PK_HC_STRIDE + row] = (u8)v;
}
// a plain-RAM write at a (and a +- 1 for 16-bit writes) that may touch the mirrored HRAM bytes:
// only those writes update the mirror (a rare branch on the common path: code and the few HRAM
// variables there are written seldom)
__device__ __forceinline__ bool near_hcode(u32 a) { return a - 0xFF7Fu < PK_HC_ROWS + 2u; }

// fast RAM: VRAM, WRAM, echo, OAM/unusable, HRAM — plain bytes of the image with no side effects
__device__ __forceinline__ bool ram_region(u32 a) { return __builtin_amdgcn_ubfe(0xD0u, a >> 13, 1u) != 0u; }  // 0x8000, 0xC000, 0xE000
// IO registers FF00-FF7F and IE (FFFF): a ^ 0x7F maps exactly those to the range FF00-FF80
__device__ __forceinline__ bool io_addr(u32 a) { return ((a ^ 0x7Fu) - 0xFF00u) <= 0x80u; }
__device__ __forceinline__ bool fast_ram(u32 a) { return ram_region(a) && !io_addr(a); }
__device__ __forceinline__ u32 fast_phys(u32 a) {
    const u32 p = (a & 0x1FFFu) + sel(a < 0xA000u, PK_P_VRAM, PK_P_WRAM);
    return sel(a >= 0xFE00u, PK_P_OAM + (a & 0x1FFu), p);
}
__device__ __forceinline__ bool vram_or_oam(u32 a) { return (a >= 0x8000u && a < 0xA000u) || (a >= 0xFE00u && a < 0xFEA0u); }
// Would a write at a change a pending (latched, not yet rasterised) line?  A pending line reads the
// tile data, the OAM and at most two tile-map rows — its BG row (y + SCY) / 8 and its window row
// lw / 8, recorded in St.prow at its latch (the bulk latch of the HALT skip-ahead sets every bit).
// A map write to a row no pending line reads leaves every pending line's pixels as they were at its
// latch, so the lines stay pending (K2 or a later flush rasterises them from the same bytes); tile
// data and OAM writes always flush.  pkbench's rendered frames write map rows the pending lines do
// not show ~12 times per env-step (host simulation), each a flush before
__device__ __forceinline__ bool pend_hit(u32 prow, u32 a) {
    return (a - 0x8000u < 0x1800u) | (a - 0xFE00u < 0xA0u) | ((a - 0x9800u < 0x800u) & (((prow >> ((a >> 5) & 31u)) & 1u) != 0u));
}
// ROM address staged in LDS?  and its LDS byte index
__device__ __forceinline__ bool rom_staged(const St& s, u32 a) { return a < s.rlim; }
__device__ __forceinline__ u32 rom_lds_index(const St& s, u32 a) { return a + sel(a < 0x4000u, 0u, s.rb); }
// byte index in the global ROM of a switchable-bank address (0x4000-0x7FFF)
__device__ __forceinline__ u32 rom_global_index(const PkStepArgs& A, const St& s, u32 a) {
    return (((s.mbc & 0xFFu) & A.rom_bank_mask) << 14) | (a & 0x3FFFu);
}
// The clock the next LCD event (LCD on) or the LCD-off frame end happens at, or 0 while the timer
// runs: clock + cycles < lim is "the timer/LCD stage has nothing to do" (fused pairs, the common
// tick).  Kept in St.lim and recomputed wherever target, LCDC, TAC, the clock or the watchdog
// budget change outside the common path: kernel entry and the ends of the rare loop-top, write and
// timer/LCD stages.
// The frame watchdog fires when cycles + 1 > slack, i.e. clock + cycles >= clock + slack; the
// common path lowers clock + slack by one per instruction only (cycles move both), and lim is
// recomputed at least once per frame (every LCD event, the LCD-off frame end), so bounding lim by
// clock + slack - PK_SLACK_MARGIN (two fused instructions per iteration, at most 70224 / 4 per
// frame) makes clock + cycles < lim imply the watchdog cannot fire: the common path needs no
// budget test of its own.  Near the budget's end lim is 0 and every iteration takes the rare stage,
// which tests the budget exactly.
#define PK_SLACK_MARGIN (2u * (FRAME_CYCLES / 4u) + 64u)
__device__ __forceinline__ u32 tick_lim(const St& s, int slack) {
    const int e = (int)s.clock + slack - (int)PK_SLACK_MARGIN;
    // 0 also while the CPU is halted (the HALT instruction's microcode zeroes it: pk_exec)
    const u32 lim = sel((s.tim0 & (4u << 24)) | (s.cpu & CPU_HALT), 0u, sel(s.lcd0 & 0x80u, s.target, FRAME_CYCLES));
    return min(lim, e > 0 ? (u32)e : 0u);
}
__device__ __forceinline__ u32 slot_base(u32 bank) {
    const int sl = lds_slot[bank & 127u];
    return sl >= 0 ? (u32)sl * 0x4000u : PK_NO_BANK;
}
// the switchable bank's LDS slot (slot_base), or PK_NO_BANK: rb and the staged-address limit
__device__ __forceinline__ void set_rom_bank(St& s, u32 base) {
    s.rb = base - 0x4000u;   // (unused when the bank is not staged: rom_lds_index is behind rom_staged)
    s.rlim = sel(base != PK_NO_BANK, 0x8000u, 0x4000u);
}

// ---------------------------------------------------------------------------------------------
// LCD helpers (pyboy lcd.py) — oracle: gbcore.c lcd_set_lcdc
// Folded line: when no STAT mode interrupt is enabled and the frame is not rendered, a visible
// line's mode-3 and mode-0 events change nothing but the STAT mode bits, so the mode-2 event
// schedules the line-end event directly (one LCD event per line instead of three) and marks the
// line folded.  The mode bits are derived from the clock whenever they are observed (STAT read),
// and the exact unfolded state is restored before anything else depends on it (STAT write, kernel
// exit).  The event at the line end sees the same state as in the unfolded sequence except the
// stored mode 2 instead of 0, which only feeds the mode-change interrupt test (disabled here).
// Folded frame: when in addition the LY=LYC interrupt is off, a visible line's mode-2 event
// schedules the VBlank event (line 144) directly; LY and the coincidence bit are then derived
// from the clock too (LY/STAT read), and restored exactly on LCDC/STAT/LYC writes and at exit.
#define PK_LCD_FOLD (1u << 26)   // lcd2 bit: current line folded (next-mode field = bits 24-25)
#define PK_LCD_FFOLD (1u << 27)  // lcd2 bit: folded run of lines: the rest of the visible frame
                                 // (next mode 1: VBlank event) or of VBlank (next mode 2: line 0)
__device__ __forceinline__ u32 lcd_fold_off(const St& s) { return s.clock - (s.target - 456u); }
__device__ __forceinline__ u32 lcd_fold_mode(u32 off) { return sel(off < 80u, 2u, sel(off < 250u, 3u, 0u)); }
__device__ __forceinline__ void lcd_unfold(St& s) {
    if (s.lcd2 & PK_LCD_FFOLD) {  // -> the current line (a folded visible line, or a VBlank line)
        const bool vis = ((s.lcd2 >> 24) & 3u) == 1u;
        const u32 k = (s.target - s.clock - 1u) / 456u;  // whole lines left after the current one
        const u32 ly = sel(vis, 143u, 153u) - k, lyc = s.lcd0 >> 24;
        const u32 stat = (bfe8(s.lcd0, 8) & 0xFBu) | sel(ly == lyc, 4u, 0u);  // its line-start LYC test
        s.lcd0 = (s.lcd0 & 0xFF0000FFu) | (stat << 8) | (ly << 16);
        s.target -= 456u * k;
        const u32 nm = sel(vis, sel(ly < 143u, 2u, 1u), sel(ly == 153u, 2u, 1u));
        s.lcd2 = (s.lcd2 & 0x00FFFFFFu) | (nm << 24) | sel(vis, PK_LCD_FOLD, 0u);
    }
    if (s.lcd2 & PK_LCD_FOLD) {
        const u32 off = lcd_fold_off(s);
        s.lcd0 = (s.lcd0 & ~0x300u) | (lcd_fold_mode(off) << 8);
        s.target = sel(off < 80u, s.target - 376u, sel(off < 250u, s.target - 206u, s.target));
        const u32 nm = sel(off < 80u, 3u, sel(off < 250u, 0u, (s.lcd2 >> 24) & 3u));
        s.lcd2 = (s.lcd2 & 0x00FFFFFFu) | (nm << 24);
    }
}

__device__ __forceinline__ void lcd_set_lcdc(St& s, u32 v) {
    s.lcd0 = setb8(s.lcd0, 0, v);
    if (!(v & 0x80u)) {
        s.clock = 0;
        s.target = FRAME_CYCLES;
        s.lcd0 = (s.lcd0 & 0xFF0000FFu) | ((bfe8(s.lcd0, 8) & 0xFCu) << 8);  // set_mode(0), LY = 0
        s.lcd2 = setb8(s.lcd2, 24, 2u);
    }
}

// joypad (pyboy interaction.py) — oracle: gbcore.c gb_button / joy_pull
__device__ __forceinline__ void key_event(St& s, u32 button, bool pressed) {
    const u32 od = bfe8(s.misc, 0), os = bfe8(s.misc, 8);
    u32 nd = od, ns = os;
    const u32 b = 1u << (button & 3u);
    if (button < 4u) nd = pressed ? (nd & ~b) : (nd | b);
    else ns = pressed ? (ns & ~b) : (ns | b);
    s.misc = (s.misc & 0xFFFF0000u) | nd | (ns << 8);
    if (((od ^ nd) & od) || ((os ^ ns) & os)) s.cpu = cpu_sync_pend(s.cpu | 0x10u << 16);
}

// ---------------------------------------------------------------------------------------------
// generic memory bus (rare paths only)
__device__ __forceinline__ u32 rom_read(const Ctx& c, const St& s, u32 a) {
    if (rom_staged(s, a)) return lds_rom[rom_lds_index(s, a)];
    const u32 bank = (s.mbc & 0xFFu) & c.A->rom_bank_mask;
    return c.A->rom[bank * 0x4000u + (a & 0x3FFFu)];
}

// IO register read (FF00-FF7F, FFFF) — oracle: gbcore.c bus_read
__device__ __forceinline__ u32 io_read(const Ctx& c, const St& s, u32 a) {
    if (a == 0xFFFFu) return bfe8(s.cpu, 8);
    const u32 lo = a & 0xFFu;
    u32 v = ld_img(c, PK_P_IO + lo);  // plain IO / FF4C-FF7F backing bytes
    v = sel(lo >= 0x10u && lo < 0x40u, 0u, v);  // sound: not emulated
    v = sel(lo == 0x04u, bfe8(s.divacc, 8), v);
    v = sel(lo == 0x05u, bfe8(s.tim0, 8), v);
    v = sel(lo == 0x06u, bfe8(s.tim0, 16), v);
    v = sel(lo == 0x07u, bfe8(s.tim0, 24), v);
    v = sel(lo == 0x0Fu, bfe8(s.cpu, 16), v);
    // FF40-FF4B: LCDC STAT SCY SCX LY LYC DMA BGP OBP0 OBP1 WY WX
    const u32 k = lo - 0x40u;
    if (k < 12u) {
        // per register: word (0 lcd0, 1 lcd1, 2 lcd2, 3 zero) << 2 | byte, 4 bits each
        const uint64_t tab = 0x76A98C325410ull;
        const u32 e = (u32)(tab >> (4u * k)) & 15u;
        const u32 w = sel((e >> 2) == 0u, s.lcd0, sel((e >> 2) == 1u, s.lcd1, sel((e >> 2) == 2u, s.lcd2, 0u)));
        v = bfe8(w, 8u * (e & 3u));
        if ((k == 1u || k == 4u) && (s.lcd2 & (PK_LCD_FOLD | PK_LCD_FFOLD))) {  // STAT / LY of a folded line or frame
            St t = s;
            lcd_unfold(t);
            v = bfe8(t.lcd0, sel(k == 1u, 8u, 16u));
        }
    }
    return v;
}

// pyboy mb.getitem for any address
__device__ __forceinline__ u32 bus_read_any(const Ctx& c, const St& s, u32 a) {
    if (a < 0x8000u) return rom_read(c, s, a);
    if ((a & 0xE000u) == 0xA000u) {  // cartridge SRAM
        if (c.A->mbc == 0u || !bfe8(s.mbc, 16)) return 0xFFu;
        return ld_img(c, PK_P_SRAM + (bfe8(s.mbc, 8) & 3u) * 0x2000u + (a - 0xA000u));
    }
    if (a >= 0xFF00u && (a < 0xFF80u || a == 0xFFFFu)) return io_read(c, s, a);
    return ld_img(c, fast_phys(a));
}

// joypad select (FF00): the register reads back the pulled lines
__device__ __forceinline__ void joyp_write(const Ctx& c, const St& s, u32 v) {
    const u32 p14 = (v >> 4) & 1u, p15 = (v >> 5) & 1u;
    u32 r = (v | 0xCFu) & 0xFFu;
    if (p14 != p15) r &= (!p14) ? bfe8(s.misc, 0) : bfe8(s.misc, 8);
    st_img(c, PK_P_IO, r);
}

// pyboy mb.setitem for any address: MBC3 registers, SRAM, IO registers, OAM DMA, IE, and plain
// RAM (with the deferred-line flush before VRAM/OAM changes)
__device__ __forceinline__ void bus_write_any(const Ctx& c, St& s, u32 a, u32 v) {
    const PkStepArgs& A = *c.A;
    if (a < 0x8000u) {  // MBC3.setitem
        if (A.mbc == 0u) return;
        if (a < 0x2000u) {
            s.mbc = setb8(s.mbc, 16, ((v & 0x0Fu) == 0x0Au) ? 1u : 0u);
        } else if (a < 0x4000u) {
            v &= 0x7Fu;
            s.mbc = setb8(s.mbc, 0, v == 0u ? 1u : v);
            set_rom_bank(s, slot_base((s.mbc & 0xFFu) & A.rom_bank_mask));
        } else if (a < 0x6000u) {
            s.mbc = setb8(s.mbc, 8, v);
        }
        return;
    }
    if ((a & 0xE000u) == 0xA000u) {
        if (A.mbc != 0u && bfe8(s.mbc, 16)) st_img(c, PK_P_SRAM + (bfe8(s.mbc, 8) & 3u) * 0x2000u + (a - 0xA000u), v);
        return;
    }
    if (a >= 0xFF00u && (a < 0xFF80u || a == 0xFFFFu)) {
        switch (a) {
            case 0xFF00: joyp_write(c, s, v); break;
            case 0xFF04: s.divacc = 0; s.timac = 0; break;
            case 0xFF05: s.tim0 = setb8(s.tim0, 8, v); break;
            case 0xFF06: s.tim0 = setb8(s.tim0, 16, v); break;
            case 0xFF07: s.tim0 = setb8(s.tim0, 24, v & 7u); break;
            case 0xFF0F: s.cpu = cpu_sync_pend(setb8(s.cpu, 16, v)); break;
            case 0xFF40:
                lcd_unfold(s);
                lcd_set_lcdc(s, v);
                break;
            case 0xFF41:
                lcd_unfold(s);
                s.lcd0 = setb8(s.lcd0, 8, (bfe8(s.lcd0, 8) & 0x87u) | (v & 0x78u));
                break;
            case 0xFF42: s.lcd1 = setb8(s.lcd1, 0, v); break;
            case 0xFF43: s.lcd1 = setb8(s.lcd1, 8, v); break;
            case 0xFF44: break;  // LY is read-only
            case 0xFF45:
                lcd_unfold(s);
                s.lcd0 = setb8(s.lcd0, 24, v);
                break;
            case 0xFF46: {  // OAM DMA: instantaneous 160-byte copy (pyboy mb.transfer_DMA)
#ifdef PK_ABLATE_DMA
                break;      // (diagnostic ablation build: what the copy costs, profiles/r06/ab_dma; breaks parity)
#endif
                if (s.npend) {
                    flush_lines(A.lat, A.lat_stride, A.screen, c.g, c.lane, c.sh, c.glane, c.env, c.gid, s.npend);
                    s.npend = 0;
                    s.prow = 0;
                }
                const u32 src = v << 8;
                if (fast_ram(src) && src < 0xFE00u) {
                    // plain RAM page (VRAM, WRAM, echo: the OAM buffers games use): the page is
                    // linear in the image, so copy in batches of 32 independent loads — the
                    // byte-by-byte bus loop waited one memory round trip per byte, and one lane
                    // in DMA held its whole wave for ~160 of them
                    const u32 sp = fast_phys(src);
                    for (u32 n0 = 0; n0 < 0xA0u; n0 += 32u) {
                        u32 b[32];
#pragma unroll
                        for (u32 k = 0; k < 32u; k++) b[k] = ld_img(c, sp + n0 + k);
#pragma unroll
                        for (u32 k = 0; k < 32u; k++) st_img(c, PK_P_OAM + n0 + k, b[k]);
                    }
                } else {
                    for (u32 n = 0; n < 0xA0u; n++) st_img(c, PK_P_OAM + n, bus_read_any(c, s, (src + n) & 0xFFFFu));
                }
                break;
            }
            case 0xFF47: s.lcd2 = setb8(s.lcd2, 0, v); break;
            case 0xFF48: s.lcd2 = setb8(s.lcd2, 8, v); break;
            case 0xFF49: s.lcd2 = setb8(s.lcd2, 16, v); break;
            case 0xFF4A: s.lcd1 = setb8(s.lcd1, 16, v); break;
            case 0xFF4B: s.lcd1 = setb8(s.lcd1, 24, v); break;
            case 0xFFFF: s.cpu = cpu_sync_pend(setb8(s.cpu, 8, v)); break;
            default:
                if (a >= 0xFF10u && a < 0xFF40u) break;  // sound: not emulated
                st_img(c, PK_P_IO + (a & 0xFFu), v);
                break;
        }
        return;
    }
    if (s.npend && pend_hit(s.prow, a)) {
        flush_lines(A.lat, A.lat_stride, A.screen, c.g, c.lane, c.sh, c.glane, c.env, c.gid, s.npend);
        s.npend = 0;
        s.prow = 0;
    }
    st_img(c, fast_phys(a), v);
    hcode_st(c, a, v);
}

// ---- rare paths (operate on a copy of the lane state) ----
__device__ __forceinline__ u32 pk_fetch_slow(const PkStepArgs* A, u8* g, u32 lane, u32 loc, const St* sp, u32 pc) {
    Ctx c;
    c.A = A; c.g = g; c.lane = lane; c.sh = A->ilv_sh; c.glane = 0; c.env = 0; c.gid = 0; c.loc = loc;
    const St s = *sp;
    return bus_read_any(c, s, pc) | (bus_read_any(c, s, (pc + 1u) & 0xFFFFu) << 8)
         | (bus_read_any(c, s, (pc + 2u) & 0xFFFFu) << 16);
}
__device__ __forceinline__ u32 pk_read_slow(const PkStepArgs* A, u8* g, u32 lane, u32 loc, const St* sp, u32 a0, u32 a1, u32 two) {
    Ctx c;
    c.A = A; c.g = g; c.lane = lane; c.sh = A->ilv_sh; c.glane = 0; c.env = 0; c.gid = 0; c.loc = loc;
    const St s = *sp;
    const u32 m0 = bus_read_any(c, s, a0);
    const u32 m1 = two ? bus_read_any(c, s, a1) : 0u;
    return m0 | (m1 << 8);
}
__device__ __forceinline__ void pk_write_slow(const PkStepArgs* A, u8* g, u32 lane, u32 loc, u32 env, u32 gid, St* sp,
                                                  u32 a0, u32 v0, u32 a1, u32 v1, u32 two, u32 hifirst) {
    Ctx c;
    c.A = A; c.g = g; c.lane = lane; c.sh = A->ilv_sh; c.glane = env & (PK_LANES - 1u); c.env = env; c.gid = gid; c.loc = loc;
    St s = *sp;
    // a push writes SP-1 (high byte) before SP-2 (low byte), as PyBoy's push does
    if (two && hifirst) bus_write_any(c, s, a1, v1);
    bus_write_any(c, s, a0, v0);
    if (two && !hifirst) bus_write_any(c, s, a1, v1);
    *sp = s;
}

// ---------------------------------------------------------------------------------------------
// Block copy.  pokered's CopyData (home/copy.asm: copy BC bytes from HL to DE) and the same loop
// with B and C swapped in the zero test,
//     ld a,[hli] / ld [de],a / inc de / dec bc / ld a,c (ld a,b) / or b (or c) / jr nz,-8
// is the bulk of a map load with the LCD off (tileset graphics into VRAM).  K1 runs it one
// instruction (or two, fused) per loop iteration, 7 instructions per byte; here up to PK_COPY_CAP
// whole passes run at the top of one iteration — their bytes copied in batches; registers, flags,
// cycles, watchdog budget and instruction count set as the 7k instructions set them — and the
// iteration goes on to execute the next pass's first instruction (pc is unchanged: at least one
// pass is left).  Only when nothing can happen inside the passes: CPU running with no interrupt
// pending, timer off, their cycles (and the next instruction's) below the next LCD event (LCD off:
// the frame end) and inside the watchdog budget; code in staged ROM; source in staged ROM, VRAM
// or WRAM, destination in VRAM or WRAM (no echo, OAM, HRAM or IO), disjoint; VRAM only with no
// rendered lines pending.  Returns the passes run.
#define PK_COPY_W0 0x0B13122Au          // 2A 12 13 0B: ld a,[hli] / ld [de],a / inc de / dec bc
#define PK_COPY_W1A 0xF820B079u         // 79 B0 20 F8: ld a,c / or b / jr nz,-8 (pokered)
#define PK_COPY_W1B 0xF820B178u         // 78 B1 20 F8: ld a,b / or c / jr nz,-8
#define PK_COPY_CAP 64u
// advance a running CPU by `cyc` cycles of `ninstr` instructions inside one LCD event window:
// DIV, clock, watchdog budget (cycles + 1 per instruction) and the instruction count
__device__ __forceinline__ void pk_skip(St& s, int& slack, u32& icount, u32 cyc, u32 ninstr) {
    s.divacc += cyc;
    s.clock += cyc;
    slack -= (int)(cyc + ninstr);
    icount += ninstr;
}
__device__ __forceinline__ bool copy_ram(u32 a) { return (a - 0x8000u < 0x2000u) | (a - 0xC000u < 0x2000u); }
__device__ __forceinline__ u32 pk_copy_loop(St& s, const Ctx& c, u32 pc, int& slack, u32& icount) {
    const u32 cpu = s.cpu;
    if ((cpu & (CPU_CRASH | CPU_HALT | CPU_QUEUED)) | ((cpu >> 8) & (cpu >> 16) & 0x1Fu)) return 0;
    if (s.tim0 & (4u << 24)) return 0;
    if (!rom_staged(s, pc) || (pc & 0x3FFFu) > 0x3FF8u) return 0;
    const u32 li = rom_lds_index(s, pc) + 4u;
    const u32* romw = reinterpret_cast<const u32*>(lds_rom);
    const u32 w1 = __builtin_amdgcn_alignbyte(romw[(li >> 2) + 1u], romw[li >> 2], li & 3u);
    if (w1 != PK_COPY_W1A && w1 != PK_COPY_W1B) return 0;
    const u32 bc = s.w0 & 0xFFFFu, de = s.w0 >> 16, hl = s.w1 & 0xFFFFu;
    // latched lines waiting for rasterisation: a copy into VRAM goes the instruction-by-instruction
    // way (its writes decide the flushes, pend_hit); a copy into WRAM changes nothing they read
    if (s.npend && de < 0xA000u) return 0;
    u32 k = (bc == 0u ? 0x10000u : bc) - 1u;          // passes before the last one
    k = min(k, PK_COPY_CAP);
    // 52 cycles and 59 watchdog units per pass; the iteration's own ld a,[hli]: 8 and 9
    const u32 lim = sel(s.lcd0 & 0x80u, s.target, FRAME_CYCLES);
    if (lim < s.clock + 9u || slack < 9) return 0;
    k = min(k, (lim - s.clock - 9u) / 52u);
    k = min(k, (u32)(slack - 9) / 59u);
    // destination: inside one VRAM or WRAM region
    if (!copy_ram(de)) return 0;
    k = min(k, ((de | 0x1FFFu) + 1u) - de);
    // source: staged ROM (inside its bank) or VRAM / WRAM (inside its region, disjoint from the
    // destination)
    const bool srom = hl < 0x8000u;
    if (srom) {
        if (!rom_staged(s, hl)) return 0;
        k = min(k, ((hl | 0x3FFFu) + 1u) - hl);
    } else {
        if (!copy_ram(hl)) return 0;
        k = min(k, ((hl | 0x1FFFu) + 1u) - hl);
        k = min(k, hl > de ? hl - de : de - hl);
    }
    if (k == 0u) return 0;
    const u32 sb = srom ? rom_lds_index(s, hl) : fast_phys(hl);
    const u32 db = fast_phys(de);
    for (u32 i0 = 0; i0 < k; i0 += 16u) {
        u32 b[16];
#pragma unroll
        for (u32 j = 0; j < 16u; j++) {
            const u32 i = min(i0 + j, k - 1u);
            b[j] = srom ? (u32)lds_rom[sb + i] : ld_img(c, sb + i);
        }
#pragma unroll
        for (u32 j = 0; j < 16u; j++)
            if (i0 + j < k) st_img(c, db + i0 + j, b[j]);
    }
    PK_VM_DRAIN();
    const u32 nbc = (bc - k) & 0xFFFFu;                // >= 1: the loop goes on
    const u32 a = (nbc >> 8) | (nbc & 0xFFu);
    s.w0 = nbc | (((de + k) & 0xFFFFu) << 16);
    s.w1 = ((hl + k) & 0xFFFFu) | (sel(a == 0u, 0x80u, 0u) << 16) | (a << 24);
    pk_skip(s, slack, icount, 52u * k, 7u * k);
    return k;
}

// The LY poll: pokered's DisableLCD waits for the VBlank line with
//     ldh a,[rLY] / cp N / jr nz,-6
// (pkbench's door warp too).  LY changes only at an LCD event or, in a folded frame (see
// lcd_unfold), every 456 cycles of the clock; while it stays unequal to N every pass reads the
// same value and sets the same A and flags, so the passes up to the next change (or PK_POLL_CAP)
// run here in one step; the iteration then executes the next pass's ldh at the advanced clock.
// Same conditions as the block copy (CPU running, nothing pending, timer off, inside the watchdog
// budget); staged-ROM code.  Returns the passes skipped.
#define PK_POLL_W0 0x00FE44F0u          // F0 44 FE: ldh a,[rLY] / cp N (N in the fourth byte)
#define PK_POLL_W1 0xFA20u              // 20 FA: jr nz,-6
#define PK_POLL_CAP 256u
__device__ __forceinline__ u32 pk_poll_loop(St& s, const Ctx& c, u32 pc, u32 bytes, int& slack, u32& icount) {
    const u32 cpu = s.cpu;
    if ((cpu & (CPU_CRASH | CPU_HALT | CPU_QUEUED)) | ((cpu >> 8) & (cpu >> 16) & 0x1Fu)) return 0;
    if (s.tim0 & (4u << 24)) return 0;
    if (!rom_staged(s, pc) || (pc & 0x3FFFu) > 0x3FFAu) return 0;
    const u32 li = rom_lds_index(s, pc) + 4u;
    if ((lds_rom[li] | ((u32)lds_rom[li + 1u] << 8)) != PK_POLL_W1) return 0;
    const u32 n = bytes >> 24, v = io_read(c, s, 0xFF44u);
    if (v == n) return 0;
    // the clock of the first read; LY holds until `chg`, no event before `lim`
    const u32 c0 = s.clock, lim = sel(s.lcd0 & 0x80u, s.target, FRAME_CYCLES);
    u32 chg = lim;
    if (s.lcd2 & PK_LCD_FFOLD) chg = min(chg, s.target - 456u * ((s.target - c0 - 1u) / 456u));
    if (chg <= c0 || slack < 16) return 0;
    u32 k = min(PK_POLL_CAP, (chg - c0 - 1u) / 32u + 1u);   // reads at c0 + 32p < chg
    k = min(k, (lim - c0 - 1u) / 32u);                        // passes end before the event
    k = min(k, (u32)(slack - 16) / 35u);                      // 32 cycles + 3 instructions each
    if (k == 0u) return 0;
    const u32 f = 0x40u | sel((v & 0xFu) < (n & 0xFu), 0x20u, 0u) | sel(v < n, 0x10u, 0u);
    s.w1 = (s.w1 & 0xFFFFu) | (f << 16) | (v << 24);
    pk_skip(s, slack, icount, 32u * k, 3u * k);
    return k;
}

// The OAM-DMA wait: pokered's hDMARoutine (copied to HRAM, run from the VBlank handler every frame)
// starts the DMA and waits 160 us with
//     ld a,$28 / dec a / jr nz,-3
// — 40 passes of 16 cycles that change only A, F and the clock.  The passes that jump back (A stays
// nonzero) run here in one step, up to the next LCD event, under the block copy's conditions (CPU
// running with nothing pending, timer off, inside the watchdog budget); the iteration then executes
// the next pass as usual.  The code may be anywhere (the prefetched bytes identify it: HRAM here).
// Returns the passes skipped.
#define PK_DEC_W0 0x00FD203Du           // 3D 20 FD: dec a / jr nz,-3
__device__ __forceinline__ u32 pk_dec_loop(St& s, int& slack, u32& icount) {
    const u32 cpu = s.cpu;
    if ((cpu & (CPU_CRASH | CPU_HALT | CPU_QUEUED)) | ((cpu >> 8) & (cpu >> 16) & 0x1Fu)) return 0;
    if (s.tim0 & (4u << 24)) return 0;
    const u32 a = s.w1 >> 24, c0 = s.clock, lim = sel(s.lcd0 & 0x80u, s.target, FRAME_CYCLES);
    if (lim <= c0 || slack < 18) return 0;
    u32 k = (a == 0u ? 256u : a) - 1u;             // passes whose dec leaves A != 0 (jr taken)
    k = min(k, (lim - c0 - 1u) / 16u);             // passes end before the event
    k = min(k, (u32)(slack - 18) / 18u);           // 16 cycles + 2 instructions each
    if (k == 0u) return 0;
    const u32 na = (a - k) & 0xFFu;                // != 0
    // the last dec's flags: Z 0, N 1, H from the borrow out of bit 4 (the old low nibble was 0), C kept
    const u32 f = (bfe8(s.w1, 16) & 0x10u) | 0x40u | sel(((na + 1u) & 0xFu) == 0u, 0x20u, 0u);
    s.w1 = (s.w1 & 0xFFFFu) | (f << 16) | (na << 24);
    pk_skip(s, slack, icount, 16u * k, 2u * k);
    return k;
}

// ---------------------------------------------------------------------------------------------
// One emulated instruction's execution: address, operand reads, fused datapath, control
// (pk_exec) and memory writes (pk_write), the same straight-line all-units sequence in every lane.
// (A wave-uniform variant — scalar branches around the units an instruction does not use when
// every lane holds the same microcode entry — measured slower on every workload, configs[1]'s
// lockstep envs included: profiles/r03_ab/uniform/.)
struct Mc {   // a microcode entry (pk_ucode.h), one VGPR per word
    u32 D, U, K, V, XR, XE, YR, YE, AR, AE, S0, S1, YC, YX, CW, CI;
};
struct Ex {   // what the rest of the iteration needs from the instruction
    u32 addr0, addr1, o0, o1, wv0, wv1, cycles;
    bool wr, wr2, wram, slow;   // slow: a write the generic bus path takes (wr & !wram)
};
template <bool PRIO, bool ALL>
__device__ __forceinline__ void pk_exec(St& s, const Ctx& c, u32 pc, u32 bytes, const Mc& m, u32& ev, Ex& x PK_STAMP_PARAMS) {
    const PkStepArgs& A = *c.A;
    const u32 D = m.D, U = m.U, K = m.K;
    // ---------------- operands, condition, memory address ----------------
    const u32 w0 = s.w0, w1 = s.w1, sp = s.sp;
    const u32 F = (w1 >> 16) & 0xFFu;
    const u32 pcn = (pc + (D & 3u)) & 0xFFFFu;
    // the condition as a lane mask: bit CPOS of (F | 0x100) ^ CINV, sign-extended
    const u32 tkm = (u32)__builtin_amdgcn_sbfe((int)(F | 0x100u), (D >> PK_DB_CPOS) & 15u, 1u) ^ bmask(D, PK_DB_CINV);
    u32 addr0 = 0, addr1 = 0, o0 = 0, o1 = 0;
    bool pair = false, fast01 = false;
    // operand pools: registers (w1:w0) and ext (q1:q0) = instruction bytes, m0|m1 and SP; the
    // address's ext pool is (SP : instruction bytes) (pk_ucode.h PK_A_SP)
    const u32 asrc = perm(w1, w0, m.AR) | perm(sp, bytes, m.AE);
    {
        addr0 = (asrc + (u32)sfield(D, PK_DB_AOFF, 2)) & 0xFFFFu;
        addr1 = (addr0 + (u32)sfield(D, PK_DB_ADIR, 2)) & 0xFFFFu;
        // image offsets of both addresses, shared by the fast read and write paths
        // The fast paths take a pair (addr1 = addr0 + ADIR, ADIR in -1/0/+1) only inside one
        // 512-byte block of plain RAM, where fast_phys is linear: o1 follows from o0.  A pair that
        // crosses a block boundary (incl. WRAM/echo at 0xE000 and echo/OAM at 0xFE00) is rare
        // and goes through the generic bus paths.
        o0 = (fast_phys(addr0) << c.sh) + c.lane;
        o1 = o0 + ((u32)sfield(D, PK_DB_ADIR, 2) << c.sh);
        pair = ((addr0 ^ addr1) & 0xFE00u) == 0u;  // both in one 512-byte block
        // inside one 512-byte block both addresses share a region; only IO/IE can differ
        fast01 = ram_region(addr0) & pair & !io_addr(addr0) & !io_addr(addr1);
    }

    // ---------------- memory reads (m0 at addr0, m1 at addr1) ----------------
    const bool rd = bit(D, PK_DB_RD) != 0u, rd2 = bit(D, PK_DB_RD2) != 0u;
    u32 m16 = 0;
    {
        const bool rram = rd & fast01;  // addr1 == addr0 for 1-byte reads
        // one-byte reads of staged ROM (a two-byte read there — POP/RET with SP in ROM — takes the
        // rare path); ALL: every ROM bank is staged in LDS (a cartridge of <= the kernel's slots), so
        // the switchable bank is staged whatever it is
        const bool rrom = (bit(D, PK_DB_RD1) != 0u) & (ALL ? addr0 < 0x8000u : rom_staged(s, addr0));
        // The image loads and the LDS ROM read have registers of their own (sharing one would make
        // the LDS read wait for the image loads of other lanes: write-after-write); the rare paths
        // write the LDS read's register, after it.  A lane reads only the source it loaded: the
        // initial values are never read, and are values that die here (PK_UNREAD), so the
        // registers need no zeroing moves.  (m16 is unspecified for an instruction without a read:
        // no selector takes it.)
        u32 rm0 = PK_UNREAD(m.AR), rm1 = PK_UNREAD(m.AE), om = PK_UNREAD(asrc);
        if (rram) {
            // a one-byte read has o1 == o0 (ADIR 0): its second load hits the same line, and m1 is
            // not taken for it, so the load needs no test of its own
            rm0 = c.g[o0];
            rm1 = c.g[o1];
            PK_MEMREF(c.env, 0u, fast_phys(addr0));
            if (rd2) PK_MEMREF(c.env, 0u, fast_phys(addr1));
        }
        if (rrom) om = lds_rom[rom_lds_index(s, addr0)];
        if (PK_RARE(rd & !rram & !rrom)) {  // rare: IO registers (LY, STAT, joypad, ...), SRAM, unstaged ROM, DAA
            PK_STAMP_AT(0);
            // DIV first, on its own: the RNG's source (pokered's Random; pkbench reads it in a quarter
            // of all wave iterations) — a wave whose rare lanes all read DIV skips the bus dispatch
            if ((addr0 == 0xFF04u) & !rd2) {
                om = bfe8(s.divacc, 8);
                PK_MEMREF(c.env, 2u, addr0);
                ev |= PK_EV_RD_IO;
            } else if ((addr0 == 0xFF00u) & !rd2) {   // JOYP, next (its image byte: o0 = PK_P_IO)
                om = c.g[o0];
                PK_MEMREF(c.env, 2u, addr0);
                ev |= PK_EV_RD_IO;
            } else if (bit(D, PK_DB_DAA)) {
                // DAA (opcodes.py DAA_27): its microcode reads two bytes at 0xFFFF (IE: never a fast
                // or staged read) to land here, and takes the result as POP AF takes m1|m0: A = m1,
                // F = m0 & 0xF0 — so the common path carries no DAA test of its own
                const u32 a = w1 >> 24;
                u32 corr = sel(F & 0x20u, 0x06u, 0u) | sel(F & 0x10u, 0x60u, 0u);
                corr |= sel(F & 0x40u, 0u, sel((a & 0x0Fu) > 0x09u, 0x06u, 0u) | sel(a > 0x99u, 0x60u, 0u));
                const u32 res = sel(F & 0x40u, a - corr, a + corr) & 0xFFu;
                om = (F & 0x40u) | sel(res == 0u, 0x80u, 0u) | sel(corr & 0x60u, 0x10u, 0u) | (res << 8);
            } else if (!rd2 & (addr0 >= 0xFF00u) & ((addr0 < 0xFF80u) | (addr0 == 0xFFFFu))) {
                om = io_read(c, s, addr0);
                PK_MEMREF(c.env, 2u, addr0);
                ev |= PK_EV_RD_IO;
            } else if ((addr0 - 0x4000u < 0x4000u) & pair) {  // unstaged switchable bank: the global ROM
                const u32 ga = rom_global_index(A, s, addr0);
                om = A.rom[ga] | sel(rd2, (u32)A.rom[ga + (u32)sfield(D, PK_DB_ADIR, 2)] << 8, 0u);
                ev |= PK_EV_RD_ROMG;
            } else {
                const St t = s;
                om = pk_read_slow(&A, c.g, c.lane, c.loc, &t, addr0, addr1, rd2 ? 1u : 0u);
                ev |= PK_EV_RD_ROMG;
            }
            PK_STAMP_AT(1);
        }
        // m0 | m1 << 8 (m1 is only meaningful for two-byte reads: one-byte operands select m0 alone)
        // (the byte pairs by v_perm: a shift would be pushed into the load branches, each then
        // waiting there for its own loads)
        m16 = sel(rram, perm(rm1, rm0, 0x0C0C0400u), om);
        ev |= sel(rd, PK_EV_RD | sel(rd2, PK_EV_RD2, 0u) | sel(rram, PK_EV_RD_RAM, 0u) | sel(rrom, PK_EV_RD_ROMLDS, 0u)
                      | sel(addr0 >= 0xFF80u && addr0 < 0xFFFFu, PK_EV_HRAM, 0u)
                      | sel(addr0 >= 0xC000u && addr0 < 0xFE00u, PK_EV_RD_WRAM, 0u), 0u);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);   // operand read issued: the SIMD's other wave first
    PK_STAMP_AT(0);

    // ---------------- fused datapath ----------------
    const u32 q1 = perm(sp, m16, 0x05040100u);   // m0 | m1 << 8 | SP << 16
    const u32 X = perm(w1, w0, m.XR) | perm(q1, bytes, m.XE);
    const u32 Y = perm(w1, w0, m.YR) | perm(q1, bytes, m.YE) | m.YC;
    const u32 right = bmask(U, PK_US_RIGHT);
    u32 cin = 0, r = 0, cvx = 0, rs = 0, lres = 0;
    // carry-in of the adder, or the bit shifted in by the right-shift unit: bit CW of
    // (X | F << 16) ^ CI (F.C at bit 20, X's bits 7/0, bit 16 = 0 for the constants)
    cin = min((((X & 0xFFFFu) | (w1 & 0xFFFF0000u)) ^ m.CI) & m.CW, 1u);
    // adder: r = X + Y ^ YX + cin (YX = 0x1FFFF subtracts); X ^ Y ^ r = the carry (borrow) into
    // each bit.  Left rotates and shifts are X + X + (0 / F.C / bit 7): bit 8 is the carry out
    r = X + (Y ^ m.YX) + cin;
    cvx = X ^ Y ^ r;
    // right-shift unit: RRC RRA RR SRA SRL ((X | in << 8 | X.0 << 9) >> 1: bit 8 = the bit
    // shifted out) and SWAP ((X | X << 8) >> 4)
    {
        const u32 swap = bmask(U, PK_US_SWAP);
        rs = (X | (msel(swap, X, cin | ((X & 1u) << 1)) << 8)) >> msel(swap, 4u, 1u);
    }
    // logic: (X & Y) and/or (X ^ Y) (OR = both); loads are 0xFF AND Y
    lres = ((X & Y) & (u32)sfield(U, PK_US_LAND, 1)) | ((X ^ Y) & (u32)sfield(U, PK_US_LXOR, 1));
    const u32 res8 = msel(bmask(U, PK_US_LOGIC), lres, msel(right, rs, r)) & 0xFFu;
    // flags: F' = (F & FK) | ((Z | H | C | FC) & FM), H/C = carry bits 4/8 (12/16 for ADD HL) or
    // the right unit's shifted-out bit 8
    u32 nf = F;
    {
        const u32 cs = msel(right, rs, cvx) >> (U & (1u << PK_US_HSH8));   // >> 8 for ADD HL
        const u32 fv = sel(res8 == 0u, 0x80u, 0u) | ((cs << 1) & 0x20u) | ((cs >> 4) & 0x10u) | K;
        nf = ((F & (K >> 8)) | (fv & (K >> 16))) & 0xFFu;
        nf = msel(bmask(U, PK_US_FPOP), m16 & 0xF0u, nf);
    }
    // register writeback: val = res16 | F' << 16 | res8 << 24 through the per-op byte selectors
    // (res16: the adder, or HL +- 1 for (HL+)/(HL-); bytes 2-3 of either are not taken)
    const u32 u16 = msel(bmask(U, PK_US_R16HL), w1 + (u32)sfield(U, PK_US_HLINC, 2), r);
    {
        const u32 val = perm(nf | (res8 << 8), u16, 0x05040100u);
        s.w0 = perm(val, w0, m.S0);
        s.w1 = perm(val, w1, m.S1);
    }

    // ---------------- control transfer, SP, IME/HALT ----------------
    // JP/CALL/INT nn, JP HL, RET, RST: X | Y (one of them is 0); JR: pc + 2 + (Y = sext e)
    s.pc = pcn;
    {
        const u32 tgt = (X + Y + (pcn & (m.YC >> 16))) & 0xFFFFu;
        const u32 jump = bmask(U, PK_US_JUMP) & tkm;
        s.pc = msel(jump, tgt, pcn);
        ev |= sel(jump != 0u, PK_EV_JUMP, 0u);
    }
    x.cycles = ((m.V >> 16) & 0xFFu) + ((m.V >> 24) & tkm);   // (pk_ucode.h: V word)
    {
        const u32 sp2 = (sp + ((u32)sfield(U, PK_US_SPD, 3) & tkm)) & 0xFFFFu;
        s.sp = msel(bmask(U, PK_US_SPW), u16 & 0xFFFFu, sp2);
    }
    // IME / HALT / CRASH / QUEUED: (cpu & keep) | set from the microcode
    s.cpu = (s.cpu & (0xFFFFFFF0u | ((K >> 24) & 15u))) | (K >> 28);
    s.lim = msel(bmask(K, 28 + 1), 0u, s.lim);   // HALT (or CRASH) set: the tick stage runs (tick_lim)
    PK_OPAQUE(s.cpu);   // (else LLVM keeps the incoming word live too: a loop-end copy)

    // the write: wv0 at addr0, wv1 at addr1 (16-bit writes: low byte first in memory; pushes
    // SP-2, SP-1); the stage itself (pk_write) runs after the secondary op
    x.wr = (D & tkm & (1u << PK_DB_WR)) != 0u;
    x.wr2 = bit(D, PK_DB_WR2) != 0u;
    x.wram = x.wr & fast01;
    x.slow = x.wr & !fast01;
    const u32 wv = msel(bmask(U, PK_US_W16), msel(bmask(U, PK_US_WPC), pcn, X), res8);
    x.wv0 = wv & 0xFFu;
    x.wv1 = (wv >> 8) & 0xFFu;
    x.addr0 = addr0;
    x.addr1 = addr1;
    x.o0 = o0;
    x.o1 = o1;
}

// BF (branch-free stores, the unstaged-bank instance): both image stores issue in every iteration,
// a lane without a plain-RAM write storing to its image's unused byte (phys 0x41FF, pk_layout.h),
// and the rare write paths drain the memory counter at their end — so the number of memory
// operations between the next-fetch global-ROM loads (issued before this stage) and their use in
// the prefetch stage is fixed, and that use waits for those loads alone (vmcnt(2)) instead of for
// this iteration's store acknowledgements too (vmcnt(0)).
template <bool BF>
__device__ __forceinline__ void pk_write(St& s, const Ctx& c, u32 env, const Mc& m, const Ex& x, int slack, u32& ev PK_STAMP_PARAMS) {
    const PkStepArgs& A = *c.A;
    if constexpr (BF) {
        if (PK_RARE(x.wram & (s.npend != 0u))) {
            if (pend_hit(s.prow, x.addr0) | (x.wr2 & pend_hit(s.prow, x.addr1))) {
                flush_lines(A.lat, A.lat_stride, A.screen, c.g, c.lane, c.sh, c.glane, env, c.gid, s.npend);
                s.npend = 0;
                s.prow = 0;
                ev |= PK_EV_FLUSH;
            }
            PK_VM_DRAIN();
        }
        const u32 dummy = (PK_P_UNUSED << c.sh) + c.lane;
        const bool w2 = x.wram & x.wr2;
        u32 wm = sel(x.wram, ~0u, 0u);   // the store address selects as masks (msel)
        PK_OPAQUE(wm);
        const u32 w2m = wm & bmask(m.D, PK_DB_WR2);
        c.g[msel(wm, x.o0, dummy)] = (u8)x.wv0;
        c.g[msel(w2m, x.o1, dummy)] = (u8)x.wv1;
        if (x.wram) PK_MEMREF(env, 1u, fast_phys(x.addr0));
        if (w2) PK_MEMREF(env, 1u, fast_phys(x.addr1));
        if (PK_RARE(x.wram & near_hcode(x.addr0))) {
            hcode_st(c, x.addr0, x.wv0);
            hcode_st(c, sel(x.wr2, x.addr1, 0u), x.wv1);   // address 0: the mirror's dummy row
        }
    } else if (x.wram) {
        // VRAM / OAM change while rendered lines are pending: rasterise them first (rare)
        // (lines are pending only in the rendered frame: test that first, alone)
        if (PK_RARE(s.npend != 0u)) {
            PK_STAMP_AT(2);
            if (pend_hit(s.prow, x.addr0) | (x.wr2 & pend_hit(s.prow, x.addr1))) {
                PK_STAMP_AT(11);
                flush_lines(A.lat, A.lat_stride, A.screen, c.g, c.lane, c.sh, c.glane, env, c.gid, s.npend);
                PK_STAMP_AT(10);
                s.npend = 0;
                s.prow = 0;
                ev |= PK_EV_FLUSH;
            }
        }
        c.g[x.o0] = (u8)x.wv0;
        PK_MEMREF(env, 1u, fast_phys(x.addr0));
        if (x.wr2) {
            c.g[x.o1] = (u8)x.wv1;
            PK_MEMREF(env, 1u, fast_phys(x.addr1));
        }
        if (PK_RARE(near_hcode(x.addr0))) {
            hcode_st(c, x.addr0, x.wv0);
            hcode_st(c, sel(x.wr2, x.addr1, 0u), x.wv1);   // address 0: the mirror's dummy row
        }
    }
    PK_STAMP_AT(2);
    // rare: IO registers / MBC / SRAM / OAM DMA / IE.  The two most frequent first, each on its own
    // (pkbench: 5 % and 4 % of all wave iterations, tools/mem_stats.py): a one-byte write to a sound
    // register (not emulated: nothing to do) or to the joypad select — a wave whose slow writes are
    // all of those skips the generic bus path and its state round trip
    if (PK_RARE(x.slow)) {
        if (!x.wr2 & (x.addr0 - 0xFF10u < 0x30u)) {
            PK_MEMREF(env, 3u, x.addr0);                      // sound: not emulated
        } else if (!x.wr2 & (x.addr0 == 0xFF00u)) {
            joyp_write(c, s, x.wv0);
            PK_MEMREF(env, 3u, x.addr0);
        } else {
            St t = s;
            pk_write_slow(&A, c.g, c.lane, c.loc, env, c.gid, &t, x.addr0, x.wv0, x.addr1, x.wv1, x.wr2 ? 1u : 0u,
                          bit(m.U, PK_US_HIFIRST));
            PK_MEMREF(env, 3u, x.addr0);
            s = t;
            s.lim = tick_lim(s, slack);
        }
        ev |= PK_EV_WR_SLOW;
        PK_STAMP_AT(3);
        if constexpr (BF) PK_VM_DRAIN();
    }
    ev |= sel(x.wr, PK_EV_WR | sel(x.wr2, PK_EV_WR2, 0u) | sel(x.addr0 >= 0xFF80u && x.addr0 < 0xFFFFu, PK_EV_HRAM, 0u)
                        | sel(x.addr0 >= 0xC000u && x.addr0 < 0xFE00u, PK_EV_WR_WRAM,
                              sel(x.addr0 >= 0x8000u && x.addr0 < 0xA000u, PK_EV_WR_VRAM, 0u)), 0u);
}

#if PK_CHECK_ON
// The lane state K1 caches instead of recomputing — none of it is stored, so the v9 state cannot
// show it directly — checked against a recomputation from the architectural state at the top of
// every iteration (host simulation only; tests/hostsim records the failures and every hostsim run
// fails on one):
//   * the CPU_PEND bit == (IE & IF & 0x1F) != 0 (cpu_sync_pend at every IE/IF change);
//   * lim: 0 while halted or while the timer runs (HALT folded into the tick limit), never past the
//     next LCD event / LCD-off frame end, never past the watchdog budget (clock + slack) — the
//     bounds that let the common path skip the timer/LCD stage and fuse a second instruction;
//   * rb / rlim == the staged slot of the current ROM bank;
//   * the HRAM code mirror == the image's bytes 0xFF80-0xFF9F;
//   * prefetched bytes (pbytes != PK_COPY_W0) == the bytes the bus holds at pc (the ones any use can
//     take: up to the bank end for ROM code, 3 for code in RAM) and p0..p3 == their microcode entry.
static __device__ void pk_check_lane(const St& s, const Ctx& c, int slack, u32 pbytes, const uint4& p0, const uint4& p1,
                              const uint4& p2, const uint4& p3) {
    const u32 env = c.env, cpu = s.cpu;
    PK_CHECK(env, ((cpu & CPU_PEND) != 0u) == (((cpu >> 8) & (cpu >> 16) & 0x1Fu) != 0u), "CPU_PEND != IE & IF");
    PK_CHECK(env, !(cpu & CPU_HALT) || s.lim == 0u, "halted with lim != 0");
    PK_CHECK(env, !(s.tim0 & (4u << 24)) || s.lim == 0u, "timer on with lim != 0");
    PK_CHECK(env, s.lim <= sel(s.lcd0 & 0x80u, s.target, FRAME_CYCLES), "lim past the next LCD event / frame end");
    PK_CHECK(env, (long long)s.lim <= (long long)s.clock + slack, "lim past the watchdog budget");
    const u32 base = slot_base((s.mbc & 0xFFu) & c.A->rom_bank_mask);
    PK_CHECK(env, s.rlim == sel(base != PK_NO_BANK, 0x8000u, 0x4000u), "rlim != staged(bank)");
    PK_CHECK(env, base == PK_NO_BANK || s.rb == base - 0x4000u, "rb != slot(bank)");
    for (u32 i = 0; i < PK_HC_ROWS; i++)
        PK_CHECK(env, lds_rom[PK_HC_BASE + c.loc * PK_HC_STRIDE + i] == ld_img(c, PK_P_HRAM + i), "HRAM code mirror stale");
    if (pbytes != PK_COPY_W0) {
        const u32 pc = s.pc;
        const u32 nb = pc < 0x8000u ? min(4u, 0x4000u - (pc & 0x3FFFu)) : 3u;
        for (u32 k = 0; k < nb; k++)
            PK_CHECK(env, ((pbytes >> (8u * k)) & 0xFFu) == bus_read_any(c, s, (pc + k) & 0xFFFFu), "prefetched bytes stale");
        const u32 op = pbytes & 0xFFu;
        const u32 di = op == 0xCBu ? 256u + ((pbytes >> 8) & 0xFFu) : op;
        const uint4* ucv = reinterpret_cast<const uint4*>(lds_uc);
        const uint4 q[4] = {p0, p1, p2, p3};
        for (u32 k = 0; k < 4u; k++) {
            const uint4 e = ucv[di * 4u + k];
            PK_CHECK(env, e.x == q[k].x && e.y == q[k].y && e.z == q[k].z && e.w == q[k].w, "prefetched microcode stale");
        }
    }
}
#endif

// ---------------------------------------------------------------------------------------------
// K1
// PRIO: the launch runs two waves per SIMD (A.prio, chosen by the host), and K1 raises a wave's
// issue priority over its dependent fetch -> decode -> operand-read chain (see the prefetch stage)
#ifdef PK_K1_SMALL
#define PK_K1_KERNEL pk_step_kernel_small
#define PK_K1_LAUNCH pk_launch_step_small
#else
#define PK_K1_KERNEL pk_step_kernel
#define PK_K1_LAUNCH pk_launch_step
#endif
template <bool PRIO, bool ALL>
__global__ void __launch_bounds__(PK_K1_MAX_THREADS) PK_K1_KERNEL(PkStepArgs A) {
    for (u32 i = threadIdx.x; i < PK_UC_U2; i += blockDim.x) lds_uc[i] = A.ucode[i];
    for (u32 i = threadIdx.x; i < PK_UC_WORDS - PK_UC_U2; i += blockDim.x) lds_u2[i] = A.ucode[PK_UC_U2 + i];
    for (u32 i = threadIdx.x; i < 128u; i += blockDim.x) lds_slot[i] = A.bank_slot[i];
    for (u32 sl = 0; sl < A.nslots; sl++) {
        const uint4* src = reinterpret_cast<const uint4*>(A.rom + (size_t)A.slot_bank[sl] * 0x4000u);
        uint4* dst = reinterpret_cast<uint4*>(lds_rom + sl * 0x4000u);
        for (u32 i = threadIdx.x; i < 0x4000u / 16u; i += blockDim.x) dst[i] = src[i];
    }
    __syncthreads();

    // thread -> env: the first wave_lanes lanes of each wave carry envs (fewer envs per wave =
    // more waves per SIMD for the same env count); the RAM layout is unchanged.
    // XCD-aware workgroup order: the hardware hands workgroup b to XCD b % 8, and each XCD has its
    // own L2.  When a workgroup holds fewer than 64 envs (few envs per wave), one 64-env image
    // group spans several workgroups; numbering them XCD-major keeps those on one XCD, so a
    // group's cache lines live in one L2 instead of bouncing between eight.
    const u32 G = gridDim.x, G8 = G & ~7u;
    const u32 blk = blockIdx.x < G8 ? (blockIdx.x & 7u) * (G8 >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const u32 tid = blk * blockDim.x + threadIdx.x;
    const u32 wl = tid & (PK_LANES - 1u);
    if (wl >= A.wave_lanes) return;
    const u32 env = A.env0 + (tid >> 6) * A.wave_lanes + wl;   // env0: first env of the sub-batch
    if (env >= ((A.env1 + PK_LANES - 1u) & ~(PK_LANES - 1u))) return;
    Ctx c;
    c.A = &A;
    c.glane = env & (PK_LANES - 1u);
    c.env = env;
    c.gid = __builtin_amdgcn_readfirstlane(env / PK_LANES);
    // image sub-block of this env (interleave 1 << ilv_sh >= the wave's envs: one per wave)
    c.sh = A.ilv_sh;
    // c.g is wave-uniform (the sub-block of the wave's first env); an interleave narrower than the
    // wave puts the wave's envs in several sub-blocks, reached through the per-lane offset
    {
        const u32 sub = c.glane >> c.sh, sub0 = __builtin_amdgcn_readfirstlane(sub);
        c.g = A.mem + (size_t)c.gid * pk_group_stride(c.sh) + (size_t)sub0 * pk_sub_stride(c.sh);
        c.lane = (u32)((sub - sub0) * pk_sub_stride(c.sh)) + (c.glane & ((1u << c.sh) - 1u));
    }
    c.loc = (threadIdx.x >> 6) * A.wave_lanes + wl;  // < PK_WG_ENVS envs per workgroup
    for (u32 i = 0; i < PK_HC_ROWS; i++) lds_rom[PK_HC_BASE + c.loc * PK_HC_STRIDE + i] = (u8)ld_img(c, PK_P_HRAM + i);
#ifdef PK_WAVETIME
    // diagnostic build (tools/wavetime_run.py): per-wave start/end (s_memrealtime, 100 MHz), loop
    // iterations of lane 0, hardware slot, and the wave's largest per-lane instruction count
    const uint64_t wt0 = __builtin_amdgcn_s_memrealtime();
    u32 wt_iter = 0;
#endif

    const u32 np = A.npad;
    u32* R = A.regs;
    St s;
    s.w0 = R[PK_R_W0 * np + env];
    s.w1 = perm(R[PK_R_W1 * np + env], R[PK_R_W1 * np + env], 0x02030100u);  // L H A F -> L H F A
    s.sp = R[PK_R_SP * np + env];
    s.pc = R[PK_R_PC * np + env];
    s.cpu = cpu_sync_pend(R[PK_R_CPU * np + env]);
    s.clock = R[PK_R_CLOCK * np + env];
    s.target = R[PK_R_TARGET * np + env];
    s.lcd0 = R[PK_R_LCD0 * np + env];
    s.lcd1 = R[PK_R_LCD1 * np + env];
    s.lcd2 = R[PK_R_LCD2 * np + env];
    {
        const u32 t0 = R[PK_R_TIM0 * np + env], t1 = R[PK_R_TIM1 * np + env];
        s.tim0 = t0;
        s.divacc = ((t0 & 0xFFu) << 8) | (t1 & 0xFFu);
        s.timac = t1 >> 16;
    }
    s.mbc = R[PK_R_MBC * np + env];
    s.misc = R[PK_R_MISC * np + env];
    set_rom_bank(s, slot_base((s.mbc & 0xFFu) & A.rom_bank_mask));
    s.npend = 0;
    s.prow = 0;
    s.blank = 0;
    s.frame_done = 0;
    u32 icount = 0;

    const bool active = env < A.env1;
    u32 frame = active ? 0u : A.frames;
    const u32 action = active ? A.actions[env] : 8u;   // actions: full-size [n] array
    // pyboy_binding.py:7-40 ACTIONS: Down Left Right Up A B Start Select -> interaction buttons
    // (0 Right 1 Left 2 Up 3 Down 4 A 5 B 6 Select 7 Start); 8+ = no button (extension)
    const u32 btn = action == 0u ? 3u : action == 1u ? 1u : action == 2u ? 0u : action == 3u ? 2u
                  : action == 4u ? 4u : action == 5u ? 5u : action == 6u ? 7u : action == 7u ? 6u : 0xFFu;
    if (active && btn != 0xFFu) key_event(s, btn, true);
    if (active && A.frames > 0u && A.release_frame == 0u && btn != 0xFFu) key_event(s, btn, false);
    // (no latch flags to clear for the rendered frame: every consumer of a latched line — K2,
    // flush_lines, K2's blank-screen path — clears its flag)
    s.render = (A.render_last && frame + 1u == A.frames) ? 1u : 0u;
    const uint4* ucv = reinterpret_cast<const uint4*>(lds_uc);
    const uint4* ucv2 = reinterpret_cast<const uint4*>(lds_u2);
    const u32* romw = reinterpret_cast<const u32*>(lds_rom);

    int slack = (int)(16u * FRAME_CYCLES);  // frame watchdog: PK_FRAME_BUDGET - budget (oracle/gbcore.c)
    s.lim = tick_lim(s, slack);
    // software pipeline: the next instruction's bytes and microcode entry, loaded from LDS at the
    // end of the previous iteration (after its writes, so bank switches and HRAM code stores are
    // seen) while the timer/LCD work runs.  pbytes = PK_COPY_W0 means "not prefetched": fetch and
    // decode at the top instead (the block-copy loop's own first bytes, which take the rare loop-top
    // stage anyway, are fetched there again), so the loop top tests one value for both
    u32 pbytes = PK_COPY_W0;
    uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0, p2 = p0, p3 = p0;
#ifdef PK_STAMP
    uint64_t st_acc[PK_NSTAMP] = {}, st_prev = __builtin_amdgcn_s_memtime(), st_iter = 0;
#endif
    while (frame < A.frames) {
        u32 ev = 0;
#if PK_CHECK_ON
        pk_check_lane(s, c, slack, pbytes, p0, p1, p2, p3);
#endif
#ifdef PK_WAVETIME
        wt_iter++;
#endif
        PK_STAMP_AT(8);
#ifdef PK_STAMP
        st_iter++;
#endif
        // ---------------- front-end: cpu.tick / check_interrupts ----------------
        // common case (running, nothing pending): execute at pc; otherwise the full PyBoy order
        const u32 cpu0 = s.cpu;
        bool exec = true, doint = false, dispatch = false;
        u32 pc = s.pc, intflag = 0;
        u32 bytes = pbytes;
        uint4 e0 = p0, e1 = p1, e2 = p2, e3 = p3;
        // the three rare stages of the loop top (interrupts / HALT, a fetch that was not prefetched,
        // a block-copy or LY-poll loop at pc) sit behind one test: the common path pays one branch
        const bool fe_rare = (cpu0 & (CPU_CRASH | CPU_HALT | CPU_QUEUED | CPU_PEND)) != 0u;
        const u32 pb3 = pbytes & 0x00FFFFFFu;
        const bool loop_at = (pbytes == PK_COPY_W0) | (pb3 == PK_POLL_W0) | (pb3 == PK_DEC_W0);
        bool pf = true;   // prefetched (iteration statistics only)
        if (PK_RARE(fe_rare | loop_at)) {
        pf = !fe_rare & (pbytes != PK_COPY_W0);
        if (fe_rare) {
            const u32 pend = (cpu0 >> 8) & (cpu0 >> 16) & 0x1Fu;
            const bool crashed = (cpu0 & CPU_CRASH) != 0u;
            const bool halted = (cpu0 & CPU_HALT) != 0u;
            const bool queued = (cpu0 & CPU_QUEUED) != 0u;
            doint = !crashed && !queued && pend != 0u;
            dispatch = doint && (cpu0 & CPU_IME) != 0u;
            const bool wake = !crashed && !doint && halted && queued;
            exec = !crashed && !doint && (!halted || queued);
            pc = (pc + sel((doint && halted) || wake, 1u, 0u)) & 0xFFFFu;
            intflag = pend & (0u - pend);
            s.cpu = cpu_sync_pend(sel(doint, (cpu0 | CPU_QUEUED) & ~CPU_HALT, sel(wake, cpu0 & ~CPU_HALT, cpu0))
                                  ^ sel(dispatch, intflag << 16, 0u));
        }

        // ---------------- fetch + microcode entry (prefetched, or here when pf = false) ----------------
        if (!pf) {
            PK_STAMP_AT(8);
            const bool flds = rom_staged(s, pc) && (pc & 0x3FFFu) < 0x3FFEu;
            const u32 la = sel(flds, rom_lds_index(s, pc), 0u);
            bytes = __builtin_amdgcn_alignbyte(romw[(la >> 2) + 1u], romw[la >> 2], la & 3u);
            // code outside the staged ROM (rare): RAM code such as the HRAM OAM-DMA wait loop reads the
            // image (three loads when pc..pc+2 stay in one 512-byte block of plain RAM), else the bus
            if (PK_RARE(exec & !flds)) {
                if (pc - 0xFF80u < PK_HC_ROWS - 2u) {  // pc..pc+2 inside the mirrored HRAM bytes
                    const u32 q = PK_HC_BASE + c.loc * PK_HC_STRIDE + (pc - 0xFF80u);
                    bytes = __builtin_amdgcn_alignbyte(romw[(q >> 2) + 1u], romw[q >> 2], q & 3u);
                    ev |= PK_EV_F_BUS | PK_EV_HRAM;
                } else if (fast_ram(pc) & fast_ram((pc + 2u) & 0xFFFFu) & (((pc ^ (pc + 2u)) & 0xFE00u) == 0u)) {
                    const u32 p = fast_phys(pc);
                    bytes = ld_img(c, p) | (ld_img(c, p + 1u) << 8) | (ld_img(c, p + 2u) << 16);
                    ev |= PK_EV_F_BUS | sel(pc >= 0xFF80u, PK_EV_HRAM, 0u);
                } else if (pc - 0x4000u < 0x3FFEu) {
                    // switchable bank not staged in LDS (a 64-bank cartridge runs most banks from
                    // here): two aligned dwords of the global ROM (1 MiB, L2-resident)
                    const u32 ga = rom_global_index(A, s, pc);
                    bytes = __builtin_amdgcn_alignbyte(A.romw[(ga >> 2) + 1u], A.romw[ga >> 2], ga & 3u);
                    ev |= PK_EV_F_ROM16;
                } else {
                    const St t = s;
                    bytes = pk_fetch_slow(&A, c.g, c.lane, c.loc, &t, pc);
                    ev |= PK_EV_F_ROM16;
                }
            }
            const u32 op = bytes & 0xFFu;
            // INT pseudo-op: the vector rides in imm16
            bytes = sel(exec, bytes, (0x40u + 8u * (u32)__builtin_ctz(intflag | 0x20u)) << 8);
            const u32 di = sel(exec, sel(op == 0xCBu, 256u + ((bytes >> 8) & 0xFFu), op),
                               sel(dispatch, PK_UC_INT, sel(doint, PK_UC_NOP0, PK_UC_IDLE)));
            ev |= sel(exec, sel(flds, PK_EV_F_LDS, 0u), 0u);
            e0 = ucv[di * 4u];
            e1 = ucv[di * 4u + 1u];
            e2 = ucv[di * 4u + 2u];
            e3 = ucv[di * 4u + 3u];
            PK_STAMP_AT(9);
        }
        // ---------------- block copy and LY poll (pk_copy_loop, pk_poll_loop) ----------------
        // whole passes of the loop run here; the iteration then executes the next pass's first
        // instruction as usual (the loop's first bytes identify it: no INT pseudo-op has them)
        if ((bytes == PK_COPY_W0) | ((bytes & 0x00FFFFFFu) == PK_POLL_W0) | ((bytes & 0x00FFFFFFu) == PK_DEC_W0)) {
            if (exec) PK_TRACE(env, pc, s.w0, perm(s.w1, s.w1, 0x02030100u), s.sp, bytes & 0xFFu);
            if (bytes == PK_COPY_W0) {
                const u32 k = pk_copy_loop(s, c, pc, slack, icount);
                if (k) PK_TRACE_SKIP(env, pc, k, 7u);
            } else if ((bytes & 0x00FFFFFFu) == PK_DEC_W0) {
                const u32 k = exec ? pk_dec_loop(s, slack, icount) : 0u;
                if (k) PK_TRACE_SKIP(env, pc, k, 2u);
            } else {
                const u32 k = pk_poll_loop(s, c, pc, bytes, slack, icount);
                if (k) PK_TRACE_SKIP(env, pc, k, 3u);
            }
        }
        s.lim = tick_lim(s, slack);   // the loop fast paths moved the clock and the budget
        icount -= sel(exec, 0u, 1u);   // an interrupt dispatch or idle iteration emulates no instruction
        }
        icount += 1u;   // (the rare loop-top stage takes it back for an interrupt dispatch / idle iteration)
        ev |= sel(exec, PK_EV_EXEC | sel((bytes & 0xFFu) == 0xCBu, PK_EV_CB, 0u), 0u) | sel(pf, PK_EV_F_LDS, 0u)
            | sel(dispatch, PK_EV_INT, 0u) | sel(!exec && !dispatch, PK_EV_IDLE, 0u);
        if (exec && !((bytes == PK_COPY_W0) | ((bytes & 0x00FFFFFFu) == PK_POLL_W0) | ((bytes & 0x00FFFFFFu) == PK_DEC_W0)))
            PK_TRACE(env, pc, s.w0, perm(s.w1, s.w1, 0x02030100u), s.sp, bytes & 0xFFu);
        const Mc m = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w, e2.x, e2.y, e2.z, e2.w, e3.x, e3.y, e3.z, e3.w};
        const u32 D = m.D;
        // the successor's secondary-op entry (read now: its LDS latency overlaps the execute stage)
        // (nxt: byte 0 the successor's opcode — 0xFF, never a secondary op, after a primary that may
        // not fuse — byte 1 its operand: one v_perm with the entry's selector, pk_ucode.h V word)
        const u32 nxt = perm(bytes, bytes, m.V);
        const u32 i2 = nxt & 0xFFu;
        const uint4 u2 = ucv2[2u * i2], u2b = ucv2[2u * i2 + 1u];
        // ---------------- execute ----------------
        Ex x;
        pk_exec<PRIO, ALL>(s, c, pc, bytes, m, ev, x PK_STAMP_ARGS);
        u32 cycles = x.cycles;
        const bool wr = x.wr, slow = x.slow;
        // ---------------- fused secondary op (pk_ucode.h pk_u2_entry) ----------------
        // The instruction after this one, if it is a JR (cc), LD r,r', INC/DEC r, INC/DEC BC/DE/HL or
        // NOP, runs in this iteration on the registers and flags just written, as PyBoy's next
        // cpu.tick would, when nothing could happen between the two: this instruction may fuse (its
        // PK_DB_NOFUSE bit clear: executed, no control transfer / IME / HALT / DAA), its cycles raise
        // no LCD event (clock stays below the LCD target and the frame length: covers the LCD-off
        // frame end too) and no watchdog frame end (slack), the timer is off (no TIMA overflow), and
        // it writes no IO/MBC register (slow write).  Code in RAM also needs: no write at all (the
        // fetched bytes stay valid), both instructions within the 3 bytes every fetch path provides
        // (ROM code has 4), and none of them an IO register (DIV and a folded STAT change with the clock).
        {
            const u32 len2 = u2.y & 3u;
            // a secondary op (len2 != 0) and both instructions within the fetched bytes,
            // (D & 3) + len2 <= avail: 4 for ROM code (and inside its 16 KiB bank: the LDS slots of
            // other banks follow it), 3 for code in RAM.  As one compare: len2 - 1 wraps for len2 = 0,
            // and avail - (D & 3) saturates (v_sub clamp) for an instruction at the bank end
            const u32 avail = sel(pc < 0x8000u, min(4u, 0x4000u - (pc & 0x3FFFu)), 3u);
            const bool lenok = len2 - 1u < (avail > (D & 3u) ? avail - (D & 3u) : 0u);
            const bool ramok = (pc < 0x8000u) | (!wr & !(pc - 0xFEFEu < 0x82u));
            // next LCD event / LCD-off frame end, 0 with the timer on (tick_lim)
            // (s.lim also bounds the watchdog: clock + cycles < lim implies cycles < slack)
            const bool fuse = (s.clock + cycles < s.lim) & !slow & ramok & lenok;
            const u32 M2 = sel(fuse, u2.y, PK_U2_NONE_Y);
            // X (pair, or register in byte 0); Y = register | immediate n, ^ the subtract mask, + delta;
            // one adder X + Y + carry-in (ADC/SBC: F.C; SUB/SBC/CP: ^ 1), a logic unit (AND XOR OR),
            // flags Z from the result, H/C from the carry vector; F' replaces F's bits under the
            // entry's mask; val2 = r16 | F' << 16 | r8 << 24 through the selectors
            const u32 ctl = u2b.w;
            const u32 F1 = (s.w1 >> 16) & 0xFFu;
            const u32 x = perm(s.w1, s.w0, u2.x);
            const u32 yv = (perm(s.w1, s.w0, u2b.x) | ((nxt >> 8) & u2b.y)) ^ u2b.z;
            const u32 yy = yv + (u32)sfield(M2, PK_U2B_DELTA, 8);
            const u32 cin = (bit(F1, 4) & ctl) ^ bit(ctl, PK_U2C_SUBC);
            const u32 r = x + yy + cin;
            const u32 cvec = x ^ yy ^ r;
            const u32 hc = ((cvec << 1) & 0x20u) | ((cvec >> 4) & 0x10u);   // H: carry into bit 4, C: into bit 8
            const u32 lr = (x & yv & (0u - bit(ctl, PK_U2C_LA))) | ((x ^ yv) & (0u - bit(ctl, PK_U2C_LX)));
            const u32 res = sel(ctl & (1u << PK_U2C_LOGIC), lr, r);
            const u32 comp = sel((res & 0xFFu) == 0u, 0x80u, 0u) | ((hc ^ (ctl >> PK_U2C_FLIP)) & (ctl >> PK_U2C_HCM))
                           | (ctl >> PK_U2C_FCONST);
            const u32 fm = M2 >> PK_U2B_FM;
            const u32 Fn = (comp & fm) | (F1 & ~fm);
            const u32 val2 = perm(Fn, res, 0x00040100u);
            const u32 w0f = perm(val2, s.w0, sel(fuse, u2.z, PK_S0_ID));
            const u32 w1f = perm(val2, s.w1, sel(fuse, u2.w, PK_S1_ID));
            // JR: taken when (F & mask) == cv (mask at F's byte of the x word, cv at the same byte of
            // the misc word; never for the other entries and when not fused)
            const bool tk2 = (((s.w1 & u2.x) ^ M2) & 0x00FF0000u) == 0u;
            const u32 pc2 = (s.pc + (M2 & 3u) + sel(tk2, (u32)sfield(nxt, 8, 8), 0u)) & 0xFFFFu;
            if (fuse) PK_TRACE(env, s.pc, s.w0, perm(s.w1, s.w1, 0x02030100u), s.sp, nxt & 0xFFu);
            ev |= sel(fuse, PK_EV_FUSE, 0u);
#ifdef PK_DBG_FUSE
            ev |= sel(len2 != 0u, 1u << 23, 0u) | sel((int)cycles < slack, 1u << 24, 0u) | sel(s.clock + cycles < s.lim, 1u << 25, 0u)
                | sel(!slow & ramok, 1u << 27, 0u);
#endif
            s.w0 = w0f;
            s.w1 = w1f;
            s.pc = pc2;
            // materialise the register file here: otherwise LLVM sinks both writebacks (and SP's)
            // past the next instruction's microcode prefetch, which keeps this entry's selector
            // registers live there and costs register copies at the loop end
            PK_PIN3(s.w0, s.w1, s.sp);
            const u32 one = bit(M2, PK_U2B_ONE);
            cycles += ((M2 >> PK_U2B_CYC) & 15u) + sel(tk2, 4u, 0u);
            slack -= (int)one;
            icount += one;
        }

        // priority 2 from here (the writes and the next instruction's address): above a wave in its
        // datapath (0), below one in its fetch -> operand-read chain (3)
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(2);
        // next instruction in an unstaged switchable bank (most of a 64-bank cartridge): its two
        // global-ROM dwords are requested now, so their latency overlaps the write stage (a lane
        // whose write switches the ROM bank refetches at the top of the next iteration)
        u32 ng0 = PK_UNREAD(u2b.x), ng1 = PK_UNREAD(u2b.y), nga = PK_UNREAD(u2b.z);   // read only where loaded (fg)
        const bool nfg = !ALL & !rom_staged(s, s.pc) & (s.pc - 0x4000u < 0x3FFEu)
                       & !(s.pc - 0xFF80u < 0x7Du);
        if (nfg) {
            nga = rom_global_index(A, s, s.pc);
            ng0 = A.romw[nga >> 2];
            ng1 = A.romw[(nga >> 2) + 1u];
        }

        // ---------------- memory writes (wv0 at addr0, wv1 at addr1) ----------------
        pk_write<PK_BF && !ALL>(s, c, env, m, x, slack, ev PK_STAMP_ARGS);

        // ---------------- prefetch the next instruction (LDS-staged ROM or the HRAM mirror) ----------------
        // wave priority (two waves per SIMD): from here through the next iteration's fetch, decode
        // and address to its operand read — a dependent chain of LDS and memory round trips — this
        // wave wins issue over the SIMD's other wave, which is meanwhile in its (long, latency-free)
        // datapath; the read is issued sooner and its latency overlaps the other wave's ALU work
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
        {
            const u32 npc = s.pc;
            const bool fl = (ALL ? npc < 0x8000u : rom_staged(s, npc)) && (npc & 0x3FFFu) < 0x3FFEu;
            // staged ROM or the HRAM code mirror: one LDS byte index, one ds_read2_b32
            const bool fh = npc - 0xFF80u < PK_HC_ROWS - 2u;
            const u32 la = sel(fh, PK_HC_BASE + c.loc * PK_HC_STRIDE + (npc - 0xFF80u), sel(fl, rom_lds_index(s, npc), 0u));
            // (one unaligned ds_read_b32 instead — the LDS runs in unaligned mode — measured ±0.5 %:
            // profiles/r05/ab_diet r05m; not kept, as it would rest on a driver setting)
            const u32 r0 = romw[la >> 2], r1 = romw[(la >> 2) + 1u];
            pbytes = __builtin_amdgcn_alignbyte(r1, r0, la);   // (v_alignbyte_b32 takes the shift's low 2 bits)
            // code in a switchable bank not staged in LDS (most of a 64-bank cartridge's banks): two
            // dwords of the global ROM (L2-resident), so the microcode entry is still prefetched here
            // and its LDS latency overlaps the timer/LCD stage like that of staged code
            const bool fg = nfg & !slow;   // unchanged bank (no slow write) and still unstaged
            pbytes = sel(fg, __builtin_amdgcn_alignbyte(ng1, ng0, nga), pbytes);
            const u32 op = pbytes & 0xFFu;
            PK_STAMP_AT(4);
            const u32 di = sel(op == 0xCBu, 256u + ((pbytes >> 8) & 0xFFu), op);
            p0 = ucv[di * 4u];
            p1 = ucv[di * 4u + 1u];
            p2 = ucv[di * 4u + 2u];
            p3 = ucv[di * 4u + 3u];
            pbytes = sel(fl | fh | fg, pbytes, PK_COPY_W0);
        }


        // ---------------- HALT fast-forward, timer, LCD (pyboy mb.tick) ----------------
        // Common case: a running CPU whose cycles reach neither the next LCD event (nor, LCD off,
        // the frame length), with the timer off and the watchdog budget left — then the whole stage
        // is DIV, clock and watchdog bookkeeping (no interrupt, no latch, no frame end).
        // The common case's bookkeeping is done for every lane before the test (the rare stage below
        // works on the advanced clock, DIV and budget; its HALT block undoes and redoes them around
        // its own cycle count), so the common case is no separate branch with its own copies of them.
        const u32 clk2 = s.clock + cycles;
        // timer on or CPU halted: lim 0; the watchdog (cycles + 1 > slack) is within clk2 >= lim (tick_lim)
        const bool rare = clk2 >= s.lim;
        s.divacc += cycles;
        s.clock = clk2;
        slack -= (int)(cycles + 1u);
        // opaque from here: otherwise LLVM folds the HALT block's undo (clock - cycles) back to the
        // iteration's incoming clock and DIV, which keeps those registers live past the update and
        // costs loop-end register copies on the common path
        PK_PIN3(s.clock, s.divacc, s.cpu);
        if (PK_RARE(rare)) {
            const u32 tac = s.tim0 >> 24;
            // HALT skip-ahead: a halted CPU that nothing can wake before VBlank (no pending or queued
            // interrupt, timer off, STAT HBlank/OAM/LYC interrupts off, frame not rendered) would spend
            // one loop iteration per LCD mode event (3 per scanline) fast-forwarding to it.  Jump to
            // the state right after line 143's mode-0 event in one step instead (exactly the state those
            // iterations would reach: LY, STAT mode and coincidence bit, clock, DIV, watchdog budget),
            // so the VBlank event itself is processed below as usual.
            // Both halted-CPU blocks sit behind one `if`: a wave has a halted lane in only a few % of
            // its iterations, so the others skip their ~50 instructions.
            PK_STAMP_AT(5);
            if (PK_RARE(s.cpu & CPU_HALT)) {
                // a halted CPU fast-forwards to the next LCD event and notices pending interrupts only
                // there, so folded events are observable here: restore the exact event state first
                s.clock -= cycles;
                s.divacc -= cycles;
                slack += (int)(cycles + 1u);
                lcd_unfold(s);
                const u32 cpu = s.cpu, stat = bfe8(s.lcd0, 8), ly = bfe8(s.lcd0, 16), nm = (s.lcd2 >> 24) & 3u;
                const bool cand = !(cpu & CPU_QUEUED) && ((cpu >> 8) & (cpu >> 16) & 0x1Fu) == 0u
                               && (s.lcd0 & 0x80u) && (stat & 0x68u) == 0u && !(tac & 4u) && ly < 143u && nm != 1u && s.clock <= s.target;
                const u32 lines = 143u - ly;
                const u32 vbl = sel(nm == 2u, s.target + 456u * lines, s.target - sel(nm == 3u, 80u, 250u) + 456u * (lines + 1u));
                const u32 nev = sel(nm == 3u, 2u, sel(nm == 0u, 1u, 0u)) + 3u * lines + 1u;  // iterations up to VBlank
                const u32 tnew = vbl - 206u;                                                  // line 143 mode-0 event
                if (cand && (int)((vbl - s.clock) + nev) <= slack) {
                    if (s.render) {
                        // rendered frame: the skipped mode-0 events would latch every remaining line with
                        // the (unchanging, the CPU is halted) scroll/window/palette registers — latch
                        // them here, advancing the window line counter as the per-event latch does
                        const u32 lcdc = s.lcd0 & 0xFFu, wy = bfe8(s.lcd1, 16), wx = bfe8(s.lcd1, 24);
                        const u32 l0 = lcdc | (bfe8(s.lcd1, 8) << 8) | (bfe8(s.lcd1, 0) << 16) | (wx << 24);
                        const u32 l1 = wy | ((s.lcd2 & 0xFFFFFFu) << 8);
                        const bool wline = (lcdc & 0x20u) && (int)wx - 7 < (int)PK_COLS;
                        int lw = (int)bfe8(s.misc, 16) - 1;
                        const u32 y0 = sel(nm == 2u, ly + 1u, ly);   // nm 2: this line's mode-0 event has passed
                        for (u32 y = y0; y < PK_ROWS; y++) {
                            if (wline && wy <= y) lw += 1;
                            const u32 idx = (c.gid * PK_ROWS + y) * PK_LANES + c.glane;
                            A.lat[idx] = l0;
                            A.lat[A.lat_stride + idx] = l1;
                            A.lat[2u * A.lat_stride + idx] = (u32)(lw + 1) | 0x100u;
                        }
                        s.misc = setb8(s.misc, 16, 0u);              // reset after line 143
                        s.npend = pend_add(s.npend, y0, PK_ROWS - 1u);
                        s.prow = ~0u;                                 // (their rows: not worth computing here)
                    }
                    const u32 skipped = tnew - s.clock;
                    s.divacc += skipped;
                    slack -= (int)(skipped + (nev - 1u));
                    s.clock = tnew;
                    s.target = vbl;
                    const u32 st2 = (stat & 0xF8u) | sel((s.lcd0 >> 24) == 143u, 4u, 0u);
                    s.lcd0 = (s.lcd0 & 0xFF0000FFu) | (st2 << 8) | (143u << 16);
                    s.lcd2 = (s.lcd2 & 0x00FFFFFFu) | (1u << 24);
                }
                const u32 dsh = timer_shift(tac);
                const int tb = (int)sel(tac & 4u, ((0x100u - bfe8(s.tim0, 8)) << dsh) - s.timac, 1u << 16);
                const int ta = (int)s.target - (int)s.clock;
                const int mm = ta < tb ? ta : tb;
                cycles = (u32)(mm < 0 ? 0 : mm);
                s.clock += cycles;
                s.divacc += cycles;
                slack -= (int)(cycles + 1u);
                PK_STAMP_AT(6);
            }
            u32 irq = 0;
            if (PK_RARE(tac & 4u)) {  // TAC enabled (timer.py Timer.tick)
                const u32 dsh = timer_shift(tac);
                u32 timac = s.timac + cycles;
                u32 tima = bfe8(s.tim0, 8);
                const u32 mul = timac >> dsh;
                timac -= mul << dsh;
                tima += mul;
                const bool ovf = tima > 0xFFu;
                tima = sel(ovf, (tima - 0x100u + bfe8(s.tim0, 16)) & 0xFFu, tima);
                irq |= sel(ovf, 4u, 0u);
                ev |= sel(ovf, PK_EV_TIMER, 0u);
                s.tim0 = setb8(s.tim0, 8, tima);
                s.timac = timac;
            }
            const u32 lcdc = s.lcd0 & 0xFFu;
            const bool lcdev = (lcdc & 0x80u) && s.clock >= s.target;
            if (lcdev) {  // lcd.tick mode transition
                const u32 nm = (s.lcd2 >> 24) & 3u;
                u32 stat = bfe8(s.lcd0, 8), ly = sel(s.lcd2 & PK_LCD_FFOLD, sel(nm == 1u, 143u, 153u), bfe8(s.lcd0, 16));
                const u32 lyc = s.lcd0 >> 24;
                const bool changed = (stat & 3u) != nm;
                stat = (stat & 0xFCu) | nm;
                irq |= sel(changed && nm != 3u && ((stat >> (nm + 3u)) & 1u), 2u, 0u);
                const bool m2 = nm == 2u, m3 = nm == 3u, m0 = nm == 0u, m1 = nm == 1u;
                const bool wrap = m2 && ly == 153u;  // clock, target < 2 frames: one subtraction
                s.clock -= sel(wrap && s.clock >= FRAME_CYCLES, FRAME_CYCLES, 0u);
                s.target -= sel(wrap && s.target >= FRAME_CYCLES, FRAME_CYCLES, 0u);
                ly = sel(wrap, 0u, sel(m2 || m1, ly + 1u, ly));
                const bool fold = m2 && (stat & 0x38u) == 0u && !s.render;  // see lcd_unfold
                // folded runs: the rest of the visible frame, or VBlank lines 145-153 (from the VBlank event)
                const bool vfold = m1 && ly == 144u && (stat & 0x40u) == 0u;
                const bool ffold = (fold && (stat & 0x40u) == 0u && ly < 143u) || vfold;
                s.target += sel(ffold, 456u * sel(vfold, 10u, 144u - ly), sel(fold, 456u, sel(m2, 80u, sel(m3, 170u, sel(m0, 206u, 456u)))));
                const bool eq = lyc == ly, upd = m2 || m1;
                stat = sel(upd, sel(eq, stat | 4u, stat & 0xFBu), stat);
                irq |= sel(upd && eq && (stat & 0x40u), 2u, 0u);
                const u32 nnext = sel(m2 && !fold, 3u, sel(m3, 0u, sel(m0 || fold, sel(ly < 143u && !ffold, 2u, 1u),
                                                                       sel(ly == 153u || vfold, 2u, 1u))));
                const bool vbl = m1 && ly == 144u;
                irq |= sel(vbl, 1u, 0u);
                s.frame_done |= sel(vbl, 1u, 0u);
                s.lcd0 = (s.lcd0 & 0xFF0000FFu) | (stat << 8) | (ly << 16);
                s.lcd2 = (s.lcd2 & 0x00FFFFFFu) | (nnext << 24) | sel(ffold, PK_LCD_FFOLD, sel(fold, PK_LCD_FOLD, 0u));
            }
            ev |= sel(lcdev, PK_EV_LCD, 0u);
            {
                // latch this scanline's registers at its mode-0 event in the rendered frame; K2 (or
                // flush_lines) rasterises it later
                const u32 ly = bfe8(s.lcd0, 16);
                if (PK_RARE(lcdev && s.render && (s.lcd0 & 0x300u) == 0u && ly < PK_ROWS)) {
                    const u32 wy = bfe8(s.lcd1, 16), wx = bfe8(s.lcd1, 24);
                    int lw = (int)bfe8(s.misc, 16) - 1;
                    const bool wl = (lcdc & 0x20u) && wy <= ly && (int)wx - 7 < (int)PK_COLS;
                    if (wl) lw += 1;
                    const u32 idx = (c.gid * PK_ROWS + ly) * PK_LANES + c.glane;
                    A.lat[idx] = lcdc | (bfe8(s.lcd1, 8) << 8) | (bfe8(s.lcd1, 0) << 16) | (wx << 24);
                    A.lat[A.lat_stride + idx] = wy | ((s.lcd2 & 0xFFFFFFu) << 8);
                    A.lat[2u * A.lat_stride + idx] = (u32)(lw + 1) | 0x100u;
                    if (ly == PK_ROWS - 1u) lw = -1;
                    s.misc = setb8(s.misc, 16, (u32)(lw + 1));
                    s.npend = pend_add(s.npend, ly, ly);
                    // the map rows this line reads: its BG row, and its window row when the window shows
                    s.prow |= sel(lcdc & 0x01u, 1u << (((ly + bfe8(s.lcd1, 0)) >> 3) & 31u), 0u)
                            | sel(wl, 1u << (((u32)lw >> 3) & 31u), 0u);
                }
            }
            if (PK_RARE(!(lcdc & 0x80u) && s.clock >= FRAME_CYCLES)) {  // LCD off: the frame ends on the clock alone
                s.frame_done = 1u;
                s.clock %= FRAME_CYCLES;
                s.blank |= s.render;
            }
            s.cpu = cpu_sync_pend(s.cpu | irq << 16);
            PK_STAMP_AT(7);
            ev |= sel(s.frame_done != 0u || slack < 0, PK_EV_FRAME, 0u);
            if (PK_RARE((s.frame_done != 0u) | (slack < 0))) {  // frame end or watchdog
                s.frame_done = 0;
                slack = (int)(16u * FRAME_CYCLES);
                frame += 1u;
                if (frame == A.release_frame && btn != 0xFFu) key_event(s, btn, false);
                s.render = (A.render_last && frame + 1u == A.frames) ? 1u : 0u;
            }
            s.lim = tick_lim(s, slack);
        }
        PK_ITER(env, ev);
        PK_ITER_OP(env, sel(exec, sel((bytes & 0xFFu) == 0xCBu, 256u + ((bytes >> 8) & 0xFFu), bytes & 0xFFu),
                            sel(dispatch, PK_UC_INT, sel(doint, PK_UC_NOP0, PK_UC_IDLE))));
    }

#ifdef PK_STAMP
    if (A.dbg && wl == 0u) {
        for (int k = 0; k < PK_NSTAMP; k++) atomicAdd(&A.dbg[k], (unsigned long long)st_acc[k]);
        atomicAdd(&A.dbg[PK_NSTAMP], (unsigned long long)st_iter);
        atomicAdd(&A.dbg[PK_NSTAMP + 1], 1ull);
    }
#endif
#ifdef PK_WAVETIME
    {
        const uint64_t wt1 = __builtin_amdgcn_s_memrealtime();
        const u32 w = tid >> 6;
        unsigned long long* rec = A.dbg + 64u + PK_WT_REC * (size_t)w;
        if (A.dbg && w < 16384u) {
            if (wl == 0u) {
                rec[0] = wt0;
                rec[1] = wt1;
                rec[2] = wt_iter;
                rec[3] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));    // HW_ID
                rec[4] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));   // XCC_ID
            }
            atomicMax(&rec[5], (unsigned long long)icount);
        }
    }
#endif
    // lanes past the range's end (in its last 64-env group) ran nothing and write nothing back:
    // those envs may belong to nobody else, but the range does not own them
    if (!active) return;
    lcd_unfold(s);
    R[PK_R_W0 * np + env] = s.w0;
    R[PK_R_W1 * np + env] = perm(s.w1, s.w1, 0x02030100u);
    R[PK_R_SP * np + env] = s.sp;
    R[PK_R_PC * np + env] = s.pc;
    R[PK_R_CPU * np + env] = s.cpu & ~CPU_PEND;
    R[PK_R_CLOCK * np + env] = s.clock;
    R[PK_R_TARGET * np + env] = s.target;
    R[PK_R_LCD0 * np + env] = s.lcd0;
    R[PK_R_LCD1 * np + env] = s.lcd1;
    R[PK_R_LCD2 * np + env] = s.lcd2;
    R[PK_R_TIM0 * np + env] = (s.tim0 & 0xFFFFFF00u) | ((s.divacc >> 8) & 0xFFu);
    R[PK_R_TIM1 * np + env] = (s.divacc & 0xFFu) | (s.timac << 16);
    R[PK_R_MBC * np + env] = s.mbc;
    R[PK_R_MISC * np + env] = s.misc;
    R[PK_R_TIME * np + env] += 1u;
    R[PK_R_ICOUNT * np + env] = icount;
    R[PK_R_RFLAGS * np + env] = s.blank | sel(s.npend != 0u, 0x100u, 0u);   // bit 8: lines left for K2
}

hipError_t PK_K1_LAUNCH(const PkStepArgs& a, hipStream_t s) {
    // one wave per SIMD while the waves fit, else 512-thread workgroups put two waves on each SIMD
    // of a CU (the 158 KB of LDS staging allows one workgroup per CU; the small-LDS build: 256-thread
    // workgroups, two per CU)
    const u32 wl = a.wave_lanes;
    const u32 span = ((a.env1 + PK_LANES - 1u) & ~(PK_LANES - 1u)) - a.env0;
    const u32 threads = span * (PK_LANES / wl);
    const u32 wide = PK_WG_ENVS * PK_LANES / wl < PK_K1_MAX_THREADS ? PK_WG_ENVS * PK_LANES / wl : PK_K1_MAX_THREADS;
    const u32 block = a.block ? a.block : (threads / PK_LANES <= a.simds ? 256u : wide);
    const u32 grid = (threads + block - 1) / block;
    // the shape this build's LDS arrays assume: every env of a workgroup has an HRAM-mirror column
    // (c.loc < PK_WG_ENVS), whole waves, at most PK_K1_MAX_THREADS threads, staged slots that exist
    if (wl == 0u || wl > PK_LANES || (wl & (wl - 1u)) || block % PK_LANES || block > PK_K1_MAX_THREADS ||
        (block / PK_LANES) * wl > PK_WG_ENVS || a.nslots > PK_LDS_SLOTS || (a.env0 % PK_LANES))
        return hipErrorInvalidValue;
    if (a.prio) {
        if (a.all_staged) hipLaunchKernelGGL((PK_K1_KERNEL<true, true>), dim3(grid), dim3(block), 0, s, a);
        else hipLaunchKernelGGL((PK_K1_KERNEL<true, false>), dim3(grid), dim3(block), 0, s, a);
    } else {
        if (a.all_staged) hipLaunchKernelGGL((PK_K1_KERNEL<false, true>), dim3(grid), dim3(block), 0, s, a);
        else hipLaunchKernelGGL((PK_K1_KERNEL<false, false>), dim3(grid), dim3(block), 0, s, a);
    }
    return hipGetLastError();
}
