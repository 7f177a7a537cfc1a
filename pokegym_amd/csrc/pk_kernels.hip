// pk_kernels.hip — MI355X (gfx950) kernels for the batched Pokémon Red env.step hot path.
//
//   K1 pk_step_kernel    24 emulated frames per env-step, one wavefront lane per emulator:
//                        SM83 interpreter (uniform decode-table datapath), memory bus, MBC3,
//                        DIV/TIMA timer, LCD mode/LY/STAT timing, joypad, OAM DMA, HALT fast-
//                        forward.  Replaces PyBoy's tick() loop driven by
//                        pokegym/pyboy_binding.py:71-91 (run_action_on_emulator).
//   K2 pk_render_kernel  rasterises the scanlines latched during the last (rendered) frame into
//                        the persistent 144x160 u8 grey screen (replaces PyBoy's renderer +
//                        screen.screen_ndarray(), pokegym/environment.py:268).
//   K5 pk_reset_kernel   per-env copy of the parsed template savestate (pyboy_binding.py:66-69).
//
// Semantics are pinned bit-exactly to the CPU oracle (oracle/gbcore.c), which restates PyBoy
// 1.x; see DESIGN.md.  Everything here is integer work; no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pk_layout.h"

typedef uint32_t u32;
typedef uint8_t u8;

#define FRAME_CYCLES 70224u

// debug hook: the host-simulation test build (tests/hostsim) defines it to record an instruction
// trace; the gfx950 build compiles it away.
#ifndef PK_TRACE
#define PK_TRACE(env, pc, w0, w1, sp, op) ((void)0)
#endif



// ---------------------------------------------------------------------------------------------
// lane state kept in VGPRs for the whole launch
struct Lane {
    u32 w0, w1, sp, pc;
    u32 cpu;            // ime | halted<<1 | queued<<2 | crashed<<3 | stopped<<4 | IE<<8 | IF<<16
    u32 clock, target;
    u32 lcd0, lcd1, lcd2;
    u32 tim0;           // (DIV byte stale in-kernel) | TIMA<<8 | TMA<<16 | TAC<<24
    u32 divacc;         // DIV<<8 | DIV_counter  (mod 2^16)
    u32 timac;          // TIMA_counter
    u32 mbc;
    u32 misc;
    u32 icount;
    // step-local
    u32 render;         // rasterising this frame
    u32 npend;          // latched, not yet rasterised lines
    u32 blank;          // frame ended with the LCD off while rendering
    u32 frame_done;
};

#define CPU_IME 1u
#define CPU_HALT 2u
#define CPU_QUEUED 4u
#define CPU_CRASH 8u

__device__ __forceinline__ u32 bfe8(u32 v, u32 sh) { return (v >> sh) & 0xFFu; }
__device__ __forceinline__ u32 setb8(u32 v, u32 sh, u32 b) { return (v & ~(0xFFu << sh)) | ((b & 0xFFu) << sh); }

#define G_IE(L) bfe8((L).cpu, 8)
#define G_IF(L) bfe8((L).cpu, 16)
#define S_IF(L, v) ((L).cpu = setb8((L).cpu, 16, (v)))
#define S_IE(L, v) ((L).cpu = setb8((L).cpu, 8, (v)))
#define G_LCDC(L) bfe8((L).lcd0, 0)
#define G_STAT(L) bfe8((L).lcd0, 8)
#define G_LY(L) bfe8((L).lcd0, 16)
#define G_LYC(L) bfe8((L).lcd0, 24)

// per-lane memory context: wave-uniform group base (SGPR) + lane offset
struct Mem {
    u8* g;      // group base (uniform)
    u32 lane;
};

__device__ __forceinline__ u32 ld_phys(const Mem& m, u32 phys) { return m.g[phys * PK_LANES + m.lane]; }
__device__ __forceinline__ void st_phys(const Mem& m, u32 phys, u32 v) { m.g[phys * PK_LANES + m.lane] = (u8)v; }

// ---------------------------------------------------------------------------------------------
// LCD helpers (pyboy lcd.py STATRegister / LCD.tick) — oracle: gbcore.c stat_set_mode etc.
__device__ __forceinline__ u32 stat_set_mode(Lane& L, u32 mode) {
    u32 stat = G_STAT(L);
    if ((stat & 3u) == mode) return 0;
    stat = (stat & 0xFCu) | mode;
    L.lcd0 = setb8(L.lcd0, 8, stat);
    return (mode != 3u && (stat & (1u << (mode + 3u)))) ? 2u : 0u;
}

__device__ __forceinline__ u32 stat_update_lyc(Lane& L) {
    u32 stat = G_STAT(L);
    u32 r = 0;
    if (G_LYC(L) == G_LY(L)) {
        stat |= 4u;
        if (stat & 0x40u) r = 2u;
    } else {
        stat &= 0xFBu;
    }
    L.lcd0 = setb8(L.lcd0, 8, stat);
    return r;
}

// ---------------------------------------------------------------------------------------------
// scanline rasteriser (pyboy renderer.scanline + scanline_sprites, DMG) for ONE lane.
// lat0 = LCDC | SCX<<8 | SCY<<16 | WX<<24 ; lat1 = WY | BGP<<8 | OBP0<<16 | OBP1<<24
// lw = window line counter AFTER this line's increment.  out: 160 grey bytes.
__device__ __constant__ u8 k_grey[4] = {0xFF, 0x99, 0x55, 0x00};

__device__ __forceinline__ u32 tile_px(const Mem& m, u32 tile_addr, u32 row, u32 col) {
    u32 lo = ld_phys(m, PK_P_VRAM + tile_addr + row * 2u), hi = ld_phys(m, PK_P_VRAM + tile_addr + row * 2u + 1u);
    u32 sh = 7u - col;
    return ((lo >> sh) & 1u) | (((hi >> sh) & 1u) << 1);
}

__device__ __forceinline__ u32 bg_tile_addr(u32 lcdc, u32 t) {
    if (lcdc & 0x10u) return t * 16u;
    return (u32)(0x1000 + (int)(int8_t)(u8)t * 16);
}

__device__ void render_line(const Mem& m, u32 y, u32 lat0, u32 lat1, int lw, u8* out) {
    u32 lcdc = lat0 & 0xFFu;
    int bx = (int)bfe8(lat0, 8), by = (int)bfe8(lat0, 16), wx = (int)bfe8(lat0, 24) - 7;
    int wy = (int)(lat1 & 0xFFu);
    u32 bgp = bfe8(lat1, 8), obp0 = bfe8(lat1, 16), obp1 = bfe8(lat1, 24);
    u32 bgmap = (lcdc & 0x08u) ? 0x1C00u : 0x1800u;
    u32 wmap = (lcdc & 0x40u) ? 0x1C00u : 0x1800u;
    bool win = (lcdc & 0x20u) && wy <= (int)y;
    u8 line[PK_COLS];
    // background / window, one 8-pixel tile row at a time
    int x = 0;
    while (x < (int)PK_COLS) {
        u32 lo, hi, sub;
        int run;
        if (win && wx <= x) {
            int wxx = x - wx;
            u32 t = ld_phys(m, PK_P_VRAM + wmap + (u32)(((lw / 8) * 32) % 0x400) + (u32)((wxx / 8) % 32));
            u32 ta = bg_tile_addr(lcdc, t) + (u32)(lw % 8) * 2u;
            lo = ld_phys(m, PK_P_VRAM + ta);
            hi = ld_phys(m, PK_P_VRAM + ta + 1u);
            sub = (u32)(wxx % 8);
            run = 8 - (int)sub;
        } else if (lcdc & 0x01u) {
            int xx = x + bx;
            u32 t = ld_phys(m, PK_P_VRAM + bgmap + (u32)((((y + (u32)by) / 8u) * 32u) % 0x400u) + (u32)((xx / 8) % 32));
            u32 ta = bg_tile_addr(lcdc, t) + ((y + (u32)by) % 8u) * 2u;
            lo = ld_phys(m, PK_P_VRAM + ta);
            hi = ld_phys(m, PK_P_VRAM + ta + 1u);
            sub = (u32)(xx % 8);
            run = 8 - (int)sub;
            // stop the run where the window starts
            if (win && wx > x && wx < x + run) run = wx - x;
        } else {
            line[x] = 0;  // background disabled -> white (shade 0)
            x++;
            continue;
        }
        for (int k = 0; k < run && x < (int)PK_COLS; k++, x++) {
            u32 s = 7u - (sub + (u32)k);
            u32 ci = ((lo >> s) & 1u) | (((hi >> s) & 1u) << 1);
            line[x] = (u8)((bgp >> (2u * ci)) & 3u);
        }
    }
    if (lcdc & 0x02u) {
        int h = (lcdc & 0x04u) ? 16 : 8;
        int sel[10];
        int ns = 0;
        for (int n = 0; n < 40 && ns < 10; n++) {
            int sy = (int)ld_phys(m, PK_P_OAM + (u32)n * 4u) - 16;
            if (sy <= (int)y && (int)y < sy + h) sel[ns++] = n;
        }
        for (int i = 1; i < ns; i++) {
            int k = sel[i], j = i - 1;
            u32 kx = ld_phys(m, PK_P_OAM + (u32)k * 4u + 1u);
            while (j >= 0 && ld_phys(m, PK_P_OAM + (u32)sel[j] * 4u + 1u) > kx) { sel[j + 1] = sel[j]; j--; }
            sel[j + 1] = k;
        }
        u32 bg0 = bgp & 3u;
        for (int i = ns - 1; i >= 0; i--) {
            u32 base = PK_P_OAM + (u32)sel[i] * 4u;
            int sy = (int)ld_phys(m, base) - 16, sx = (int)ld_phys(m, base + 1u) - 8;
            u32 ti = ld_phys(m, base + 2u), at = ld_phys(m, base + 3u);
            if (h == 16) ti &= 0xFEu;
            int dy = (int)y - sy;
            int yy = (at & 0x40u) ? (h - dy - 1) : dy;
            u32 pal = (at & 0x10u) ? obp1 : obp0;
            u32 ta = ti * 16u + (u32)yy * 2u;
            u32 lo = ld_phys(m, PK_P_VRAM + ta), hi = ld_phys(m, PK_P_VRAM + ta + 1u);
            for (int dx = 0; dx < 8; dx++) {
                int px = sx + dx;
                u32 xx = (at & 0x20u) ? (u32)(7 - dx) : (u32)dx;
                u32 s = 7u - xx;
                u32 c = ((lo >> s) & 1u) | (((hi >> s) & 1u) << 1);
                if (px >= 0 && px < (int)PK_COLS && c != 0u) {
                    u32 shade = (pal >> (2u * c)) & 3u;
                    if (at & 0x80u) {
                        if (line[px] == bg0) line[px] = (u8)shade;
                    } else {
                        line[px] = (u8)shade;
                    }
                }
            }
        }
    }
    // grey write, 16 bytes at a time
    for (int q = 0; q < (int)PK_COLS; q += 16) {
        uint4 v;
        u32 w[4];
        for (int j = 0; j < 4; j++) {
            u32 a = 0;
            for (int b = 0; b < 4; b++) a |= (u32)k_grey[line[q + j * 4 + b]] << (8 * b);
            w[j] = a;
        }
        v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3];
        *reinterpret_cast<uint4*>(out + q) = v;
    }
}

// rasterise every latched-but-pending line of this lane now (before VRAM/OAM change).  Rare
// path: kept out of line with by-value arguments so the hot loop's lane state stays in VGPRs.
__device__ __noinline__ void flush_lines(u32* lat, u32 lat_stride, u8* screen, u8* gbase, u32 lane, u32 env, u32 gid) {
    Mem m;
    m.g = gbase;
    m.lane = lane;
    u32* lat0 = lat;
    u32* lat1 = lat + lat_stride;
    u32* lat2 = lat + 2u * lat_stride;
    for (u32 y = 0; y < PK_ROWS; y++) {
        u32 idx = (gid * PK_ROWS + y) * PK_LANES + lane;
        u32 l2 = lat2[idx];
        if (l2 & 0x100u) {
            render_line(m, y, lat0[idx], lat1[idx], (int)(l2 & 0xFFu) - 1, screen + (size_t)env * PK_SCREEN + y * PK_COLS);
            lat2[idx] = l2 & ~0x100u;
        }
    }
}

#define FLUSH_PENDING()                                                                   \
    do {                                                                                  \
        if (L.npend) {                                                                    \
            flush_lines(A.lat, A.lat_stride, A.screen, m.g, m.lane, env, gid);            \
            L.npend = 0;                                                                  \
        }                                                                                 \
    } while (0)

// ---------------------------------------------------------------------------------------------
// LCD tick (pyboy lcd.py LCD.tick) — oracle: gbcore.c lcd_tick.  The mode transition is written
// branch-light: under divergence some lane of the wave transitions on most iterations.
__device__ __forceinline__ u32 lcd_tick(const PkStepArgs& A, Lane& L, u32 gid, u32 lane, u32 cycles) {
    u32 intr = 0;
    L.clock += cycles;
    const u32 lcdc = G_LCDC(L);
    if (lcdc & 0x80u) {
        if (L.clock >= L.target) {
            const u32 nm = bfe8(L.lcd2, 24);
            u32 stat = G_STAT(L);
            const bool changed = (stat & 3u) != nm;
            stat = (stat & 0xFCu) | nm;
            if (changed && nm != 3u && (stat & (1u << (nm + 3u)))) intr |= 2u;
            u32 ly = G_LY(L);
            const bool m2 = nm == 2u, m3 = nm == 3u, m0 = nm == 0u, m1 = nm == 1u;
            const bool wrap = m2 && ly == 153u;
            if (wrap) {
                while (L.clock >= FRAME_CYCLES) L.clock -= FRAME_CYCLES;
                while (L.target >= FRAME_CYCLES) L.target -= FRAME_CYCLES;
            }
            ly = wrap ? 0u : ((m2 || m1) ? ly + 1u : ly);
            L.target += m2 ? 80u : m3 ? 170u : m0 ? 206u : 456u;
            if (m2 || m1) {  // STATRegister.update_LYC
                const bool eq = G_LYC(L) == ly;
                stat = eq ? (stat | 4u) : (stat & 0xFBu);
                if (eq && (stat & 0x40u)) intr |= 2u;
            }
            const u32 nnext = m2 ? 3u : m3 ? 0u : m0 ? (ly < 143u ? 2u : 1u) : (ly == 153u ? 2u : 1u);
            if (m1 && ly == 144u) {
                intr |= 1u;
                L.frame_done = 1u;
            }
            L.lcd0 = (L.lcd0 & 0xFF0000FFu) | (stat << 8) | (ly << 16);
            L.lcd2 = (L.lcd2 & 0x00FFFFFFu) | (nnext << 24);
            if (m0 && L.render && ly < PK_ROWS) {
                // latch this scanline's registers; rasterised by K2 (or flush_lines)
                const u32 lcd1 = L.lcd1;
                const u32 wy = bfe8(lcd1, 16), wx = bfe8(lcd1, 24);
                int lw = (int)bfe8(L.misc, 16) - 1;
                if ((lcdc & 0x20u) && wy <= ly && (int)wx - 7 < (int)PK_COLS) lw += 1;
                const u32 idx = (gid * PK_ROWS + ly) * PK_LANES + lane;
                A.lat[idx] = lcdc | (bfe8(lcd1, 8) << 8) | (bfe8(lcd1, 0) << 16) | (wx << 24);
                A.lat[A.lat_stride + idx] = wy | ((L.lcd2 & 0xFFFFFFu) << 8);
                A.lat[2u * A.lat_stride + idx] = (u32)(lw + 1) | 0x100u;
                if (ly == PK_ROWS - 1u) lw = -1;
                L.misc = setb8(L.misc, 16, (u32)(lw + 1));
                L.npend += 1u;
            }
        }
    } else if (L.clock >= FRAME_CYCLES) {
        L.frame_done = 1u;
        while (L.clock >= FRAME_CYCLES) L.clock -= FRAME_CYCLES;
        if (L.render) L.blank = 1u;
    }
    return intr;
}

// timer (pyboy timer.py Timer.tick) — oracle: gbcore.c timer_tick.
// DIV/DIV_counter are kept as one 16-bit accumulator: DIV_counter += c; DIV += DIV_counter >> 8;
// both masked to 8 bits  ==  (DIV << 8 | DIV_counter) + c  mod 2^16.
__device__ __forceinline__ u32 timer_tick(Lane& L, u32 cycles) {
    L.divacc = (L.divacc + cycles) & 0xFFFFu;
    const u32 tac = bfe8(L.tim0, 24);
    u32 r = 0;
    if (tac & 4u) {
        u32 timac = L.timac + cycles;
        const u32 dsh = ((tac & 3u) == 0u) ? 10u : ((tac & 3u) == 1u) ? 4u : ((tac & 3u) == 2u) ? 6u : 8u;
        u32 tima = bfe8(L.tim0, 8);
        if (timac >= (1u << dsh)) {
            const u32 mul = timac >> dsh;
            timac -= mul << dsh;
            tima += mul;
            if (tima > 0xFFu) {
                tima -= 0x100u;
                tima += bfe8(L.tim0, 16);
                tima &= 0xFFu;
                r = 4u;
            }
        }
        L.tim0 = setb8(L.tim0, 8, tima);
        L.timac = timac;
    }
    return r;
}

__device__ __forceinline__ int timer_cycles_to_interrupt(const Lane& L) {
    const u32 tac = bfe8(L.tim0, 24);
    if (!(tac & 4u)) return 1 << 16;
    const u32 dsh = ((tac & 3u) == 0u) ? 10u : ((tac & 3u) == 1u) ? 4u : ((tac & 3u) == 2u) ? 6u : 8u;
    return (int)((0x100u - bfe8(L.tim0, 8)) << dsh) - (int)L.timac;
}

// joypad (pyboy interaction.py) — oracle: gbcore.c gb_button / joy_pull
__device__ __forceinline__ void key_event(Lane& L, u32 button, bool pressed) {
    const u32 od = bfe8(L.misc, 0), os = bfe8(L.misc, 8);
    u32 nd = od, ns = os;
    const u32 bit = 1u << (button & 3u);
    if (button < 4u) nd = pressed ? (nd & ~bit) : (nd | bit);
    else ns = pressed ? (ns & ~bit) : (ns | bit);
    L.misc = (L.misc & 0xFFFF0000u) | nd | (ns << 8);
    if (((od ^ nd) & od) || ((os ^ ns) & os)) S_IF(L, G_IF(L) | 0x10u);
}

__device__ __forceinline__ u32 joy_pull(const Lane& L, u32 v) {
    const u32 p14 = (v >> 4) & 1u, p15 = (v >> 5) & 1u;
    u32 r = (v | 0xCFu) & 0xFFu;
    if (p14 != p15) r &= (!p14) ? bfe8(L.misc, 0) : bfe8(L.misc, 8);
    return r;
}

// ---------------------------------------------------------------------------------------------
// memory bus (pyboy mb.getitem / setitem) — oracle: gbcore.c bus_read / bus_write.
// Every guest address maps to ONE load: either the ROM (shared, read-only) or the env's
// lane-interleaved RAM image at phys = addr - off(addr).  Special IO registers live in the lane
// registers and take a (rare) branch.
__device__ __forceinline__ bool io_is_special(u32 a) {
    // FF04-FF07, FF0F, FF10-FF4B (sound: not emulated, LCD), FFFF (IE)
    return (a >= 0xFF04u && a <= 0xFF07u) || a == 0xFF0Fu || (a >= 0xFF10u && a <= 0xFF4Bu) || a == 0xFFFFu;
}

__device__ __noinline__ u32 io_read_special(u32 a, u32 cpu, u32 lcd0, u32 lcd1, u32 lcd2, u32 tim0, u32 divacc) {
    switch (a) {
        case 0xFF04: return (divacc >> 8) & 0xFFu;
        case 0xFF05: return bfe8(tim0, 8);
        case 0xFF06: return bfe8(tim0, 16);
        case 0xFF07: return bfe8(tim0, 24);
        case 0xFF0F: return bfe8(cpu, 16);
        case 0xFF40: return bfe8(lcd0, 0);
        case 0xFF41: return bfe8(lcd0, 8);
        case 0xFF42: return bfe8(lcd1, 0);
        case 0xFF43: return bfe8(lcd1, 8);
        case 0xFF44: return bfe8(lcd0, 16);
        case 0xFF45: return bfe8(lcd0, 24);
        case 0xFF47: return bfe8(lcd2, 0);
        case 0xFF48: return bfe8(lcd2, 8);
        case 0xFF49: return bfe8(lcd2, 16);
        case 0xFF4A: return bfe8(lcd1, 16);
        case 0xFF4B: return bfe8(lcd1, 24);
        case 0xFFFF: return bfe8(cpu, 8);
        default: return 0;  // FF46 (DMA) and FF10-FF3F (sound not emulated)
    }
}

// phys offset of a RAM-backed guest address (a >= 0x8000): phys = a - ram_off(a)
__device__ __forceinline__ u32 ram_off(u32 a, u32 mbcreg) {
    const u32 sram_off = 0xA000u - PK_P_SRAM - (bfe8(mbcreg, 8) & 3u) * 0x2000u;
    return a >= 0xFE00u ? 0xBE00u : a >= 0xE000u ? 0xC000u : a >= 0xC000u ? 0xA000u
         : a >= 0xA000u ? sram_off : 0x8000u;
}

// ROM bytes staged in LDS (slot 0 = bank 0, then the hottest banks) + the bank -> slot map
struct RomLds {
    const u8* bytes;     // nslots * 16 KiB
    const int8_t* slot;  // [128]
};

__device__ __forceinline__ u32 bus_read(const PkStepArgs& A, const RomLds& RL, const Mem& m, const Lane& L, u32 a) {
    const bool rom = a < 0x8000u;
    const u32 bank = a < 0x4000u ? 0u : (bfe8(L.mbc, 0) & A.rom_bank_mask);
    const int slot = a < 0x4000u ? 0 : (int)RL.slot[bank & 127u];
    if (rom && slot >= 0) return RL.bytes[(u32)slot * 0x4000u + (a & 0x3FFFu)];
    const u8* p = rom ? (A.rom + bank * 0x4000u + (a & 0x3FFFu)) : (m.g + (size_t)((a - ram_off(a, L.mbc)) * PK_LANES + m.lane));
    u32 v = *p;
    if ((a & 0xE000u) == 0xA000u && (A.mbc == 0u || !bfe8(L.mbc, 16))) v = 0xFFu;
    if (io_is_special(a)) v = io_read_special(a, L.cpu, L.lcd0, L.lcd1, L.lcd2, L.tim0, L.divacc);
    return v;
}

__device__ __forceinline__ void lcd_set_lcdc(Lane& L, u32 v) {
    L.lcd0 = setb8(L.lcd0, 0, v);
    if (!(v & 0x80u)) {
        L.clock = 0;
        L.target = FRAME_CYCLES;
        L.lcd0 = (L.lcd0 & 0xFF0000FFu) | ((G_STAT(L) & 0xFCu) << 8);  // set_mode(0), LY = 0
        L.lcd2 = setb8(L.lcd2, 24, 2u);
    }
}

// rare writes: MBC registers, special IO (incl. OAM DMA), IE, joypad select
__device__ __forceinline__ void bus_write_slow(const PkStepArgs& A, const RomLds& RL, const Mem& m, Lane& L, u32 env, u32 gid, u32 a, u32 v) {
    if (a < 0x8000u) {  // MBC3.setitem
        if (A.mbc == 0u) return;
        if (a < 0x2000u) {
            L.mbc = setb8(L.mbc, 16, ((v & 0x0Fu) == 0x0Au) ? 1u : 0u);
        } else if (a < 0x4000u) {
            v &= 0x7Fu;
            L.mbc = setb8(L.mbc, 0, v == 0u ? 1u : v);
        } else if (a < 0x6000u) {
            L.mbc = setb8(L.mbc, 8, v);
        }
        return;
    }
    switch (a) {
        case 0xFF00: st_phys(m, PK_P_IO, joy_pull(L, v)); break;
        case 0xFF04: L.divacc = 0; L.timac = 0; break;
        case 0xFF05: L.tim0 = setb8(L.tim0, 8, v); break;
        case 0xFF06: L.tim0 = setb8(L.tim0, 16, v); break;
        case 0xFF07: L.tim0 = setb8(L.tim0, 24, v & 7u); break;
        case 0xFF0F: S_IF(L, v); break;
        case 0xFF40: lcd_set_lcdc(L, v); break;
        case 0xFF41: L.lcd0 = setb8(L.lcd0, 8, (G_STAT(L) & 0x87u) | (v & 0x78u)); break;
        case 0xFF42: L.lcd1 = setb8(L.lcd1, 0, v); break;
        case 0xFF43: L.lcd1 = setb8(L.lcd1, 8, v); break;
        case 0xFF45: L.lcd0 = setb8(L.lcd0, 24, v); break;
        case 0xFF46: {  // OAM DMA: instantaneous 160-byte copy (pyboy mb.transfer_DMA)
            if (L.npend) {
                flush_lines(A.lat, A.lat_stride, A.screen, m.g, m.lane, env, gid);
                L.npend = 0;
            }
            const u32 src = v << 8;
            for (u32 n = 0; n < 0xA0u; n++) st_phys(m, PK_P_OAM + n, bus_read(A, RL, m, L, (src + n) & 0xFFFFu));
            break;
        }
        case 0xFF47: L.lcd2 = setb8(L.lcd2, 0, v); break;
        case 0xFF48: L.lcd2 = setb8(L.lcd2, 8, v); break;
        case 0xFF49: L.lcd2 = setb8(L.lcd2, 16, v); break;
        case 0xFF4A: L.lcd1 = setb8(L.lcd1, 16, v); break;
        case 0xFF4B: L.lcd1 = setb8(L.lcd1, 24, v); break;
        case 0xFFFF: S_IE(L, v); break;
        default: break;  // FF44 (LY, read-only) and FF10-FF3F (sound not emulated)
    }
}

__device__ __forceinline__ void bus_write(const PkStepArgs& A, const RomLds& RL, const Mem& m, Lane& L, u32 env, u32 gid, u32 a, u32 v) {
    if (a < 0x8000u || a == 0xFF00u || io_is_special(a)) {
        bus_write_slow(A, RL, m, L, env, gid, a, v);
        return;
    }
    // VRAM / OAM change while rendered lines are pending: rasterise them first
    if (L.npend && (a < 0xA000u || (a >= 0xFE00u && a < 0xFEA0u))) {
        flush_lines(A.lat, A.lat_stride, A.screen, m.g, m.lane, env, gid);
        L.npend = 0;
    }
    if ((a & 0xE000u) == 0xA000u && (A.mbc == 0u || !bfe8(L.mbc, 16))) return;  // SRAM disabled
    m.g[(size_t)((a - ram_off(a, L.mbc)) * PK_LANES + m.lane)] = (u8)v;
}

// ---------------------------------------------------------------------------------------------
// register file helpers (W0 = C|B<<8|E<<16|D<<24, W1 = L|H<<8|A<<16|F<<24).
// NOTE: selections between lane-state fields are written as arithmetic on VALUES. A C++
// `cond ? L.w1 : L.w0` (or an if/else storing to one of two fields) lets LLVM form a select of
// field ADDRESSES, which forces the whole Lane struct into scratch memory.
__device__ __forceinline__ u32 rd8(u32 w0, u32 w1, u32 r) {
    const u32 sel = 0u - ((r >> 2) & 1u);
    const u32 w = (w0 & ~sel) | (w1 & sel);
    return bfe8(w, ((r ^ 1u) & 3u) * 8u);
}
// write r8 (r != 6) into (w0, w1)
__device__ __forceinline__ void wr8(u32& w0, u32& w1, u32 r, u32 v) {
    const u32 sh = ((r ^ 1u) & 3u) * 8u;
    const u32 sel = 0u - ((r >> 2) & 1u);
    const u32 msk = 0xFFu << sh, nv = (v & 0xFFu) << sh;
    w0 = (w0 & ~(msk & ~sel)) | (nv & ~sel);
    w1 = (w1 & ~(msk & sel)) | (nv & sel);
}
__device__ __forceinline__ u32 rd16(u32 w0, u32 w1, u32 sp, u32 p) {  // BC DE HL SP
    const u32 lo = (p & 1u) ? (w0 >> 16) : (w0 & 0xFFFFu);
    const u32 hi = (p & 1u) ? sp : (w1 & 0xFFFFu);
    return (p & 2u) ? hi : lo;
}
__device__ __forceinline__ void wr16(u32& w0, u32& w1, u32& sp, u32 p, u32 v) {
    v &= 0xFFFFu;
    const u32 n0 = p == 0u ? ((w0 & 0xFFFF0000u) | v) : p == 1u ? ((w0 & 0xFFFFu) | (v << 16)) : w0;
    const u32 n1 = p == 2u ? ((w1 & 0xFFFF0000u) | v) : w1;
    const u32 ns = p == 3u ? v : sp;
    w0 = n0;
    w1 = n1;
    sp = ns;
}

__device__ __forceinline__ bool cond_ok(u32 f, u32 a) {
    const u32 cc = a & 3u;
    const bool z = (f & 0x80u) != 0, c = (f & 0x10u) != 0;
    const bool t = cc == 0u ? !z : cc == 1u ? z : cc == 2u ? !c : c;
    return !(a & PK_COND_FLAG) || t;
}

__device__ __forceinline__ u32 sext8(u32 b) { return (u32)(int)(int8_t)(u8)b; }

// ---------------------------------------------------------------------------------------------
// K1: the step kernel (one lane = one emulator; 24 frames per launch)
__global__ void __launch_bounds__(256) pk_step_kernel(PkStepArgs A) {
    __shared__ u32 lds_dtab[1024];
    __shared__ __attribute__((aligned(16))) u8 lds_rom[PK_LDS_SLOTS * 0x4000u];
    __shared__ int8_t lds_slot[128];
    for (u32 i = threadIdx.x; i < 1024u; i += blockDim.x) lds_dtab[i] = A.dtab[i];
    for (u32 i = threadIdx.x; i < 128u; i += blockDim.x) lds_slot[i] = A.bank_slot[i];
    for (u32 s = 0; s < A.nslots; s++) {
        const uint4* src = reinterpret_cast<const uint4*>(A.rom + (size_t)A.slot_bank[s] * 0x4000u);
        uint4* dst = reinterpret_cast<uint4*>(lds_rom + s * 0x4000u);
        for (u32 i = threadIdx.x; i < 0x4000u / 16u; i += blockDim.x) dst[i] = src[i];
    }
    __syncthreads();
    RomLds RL;
    RL.bytes = lds_rom;
    RL.slot = lds_slot;

    const u32 env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= A.npad) return;
    const u32 lane = env & (PK_LANES - 1u);
    const u32 gid = __builtin_amdgcn_readfirstlane(env / PK_LANES);
    Mem m;
    m.g = A.mem + (size_t)gid * PK_GROUP_STRIDE;
    m.lane = lane;

    const u32 np = A.npad;
    u32* R = A.regs;
    Lane L;
    L.w0 = R[PK_R_W0 * np + env];
    L.w1 = R[PK_R_W1 * np + env];
    L.sp = R[PK_R_SP * np + env];
    L.pc = R[PK_R_PC * np + env];
    L.cpu = R[PK_R_CPU * np + env];
    L.clock = R[PK_R_CLOCK * np + env];
    L.target = R[PK_R_TARGET * np + env];
    L.lcd0 = R[PK_R_LCD0 * np + env];
    L.lcd1 = R[PK_R_LCD1 * np + env];
    L.lcd2 = R[PK_R_LCD2 * np + env];
    {
        const u32 t0 = R[PK_R_TIM0 * np + env], t1 = R[PK_R_TIM1 * np + env];
        L.tim0 = t0;
        L.divacc = ((t0 & 0xFFu) << 8) | (t1 & 0xFFu);
        L.timac = t1 >> 16;
    }
    L.mbc = R[PK_R_MBC * np + env];
    L.misc = R[PK_R_MISC * np + env];
    L.icount = 0;
    L.npend = 0;
    L.blank = 0;
    L.frame_done = 0;

    const bool active = env < A.n;
    u32 frame = active ? 0u : A.frames;
    const u32 action = active ? A.actions[env] : 8u;
    // pyboy_binding.py:7-40 ACTIONS: Down Left Right Up A B Start Select -> interaction buttons
    // (0 Right 1 Left 2 Up 3 Down 4 A 5 B 6 Select 7 Start)
    const u32 btn = action == 0u ? 3u : action == 1u ? 1u : action == 2u ? 0u : action == 3u ? 2u
                  : action == 4u ? 4u : action == 5u ? 5u : action == 6u ? 7u : action == 7u ? 6u : 0xFFu;
    if (active && btn != 0xFFu) key_event(L, btn, true);
    if (active && A.frames > 0u && A.release_frame == 0u && btn != 0xFFu) key_event(L, btn, false);
    L.render = (A.render_last && frame + 1u == A.frames) ? 1u : 0u;
    if (L.render) {
        u32* lat2 = A.lat + 2u * A.lat_stride;
        for (u32 y = 0; y < PK_ROWS; y++) lat2[(gid * PK_ROWS + y) * PK_LANES + lane] &= ~0x100u;
    }

    const uint4* rom16 = reinterpret_cast<const uint4*>(A.rom16);
    u32 budget = 0;  // frame watchdog (see oracle/gbcore.c PK_FRAME_BUDGET)
    while (frame < A.frames) {
        // ---------------- cpu.tick: interrupts / HALT (branch-free) ----------------
        const u32 cpu = L.cpu;
        const bool crashed = (cpu & CPU_CRASH) != 0;
        const bool halted = (cpu & CPU_HALT) != 0;
        const bool queued = (cpu & CPU_QUEUED) != 0;
        const u32 pend = G_IF(L) & G_IE(L) & 0x1Fu;
        const bool do_int = !crashed && !queued && pend != 0u;
        const bool dispatch = do_int && (cpu & CPU_IME);
        const bool wake = !crashed && !do_int && halted && queued;
        const bool exec = !crashed && !do_int && (!halted || queued);
        const u32 pc = (L.pc + ((do_int && halted) || wake ? 1u : 0u)) & 0xFFFFu;
        L.cpu = do_int ? ((cpu | CPU_QUEUED) & ~CPU_HALT) : wake ? (cpu & ~CPU_HALT) : cpu;
        const u32 intflag = pend & (~pend + 1u);  // lowest set bit = highest priority
        u32 cycles = (crashed || (halted && !exec && !do_int)) ? 4u : 0u;

        // ---------------- fetch + decode: LDS-staged ROM bank, else ONE 16-byte pre-decoded load ----------------
        u32 d = PK_C_NOP | (1u << 6);
        u32 u = 0;
        u32 bytes = 0;
        if (exec) {
            const u32 bank = pc < 0x4000u ? 0u : (bfe8(L.mbc, 0) & A.rom_bank_mask);
            const int slot = pc < 0x4000u ? 0 : (int)lds_slot[bank & 127u];
            const u32 off = pc & 0x3FFFu;
            if (pc < 0x8000u && slot >= 0 && off < 0x3FFEu) {
                // ROM bank staged in LDS: 3 byte reads + decode-table lookup, all LDS
                const u8* q = lds_rom + (u32)slot * 0x4000u + off;
                const u32 op = q[0], b1 = q[1], b2 = q[2];
                const u32 di = op == 0xCBu ? 256u + b1 : op;
                d = lds_dtab[di];
                u = lds_dtab[512u + di];
                bytes = op | (b1 << 8) | (b2 << 16);
            } else if (pc < 0x8000u && off < 0x3FFEu) {
                // bank not staged: ONE 16-byte load of the pre-decoded ROM
                const uint4 e = rom16[bank * 0x4000u + off];
                d = e.x;
                u = e.y;
                bytes = e.z;
            } else {  // code in RAM / operands across a bank end
                const u32 op = bus_read(A, RL, m, L, pc);
                const u32 b1 = bus_read(A, RL, m, L, (pc + 1u) & 0xFFFFu);
                const u32 b2 = bus_read(A, RL, m, L, (pc + 2u) & 0xFFFFu);
                const u32 di = op == 0xCBu ? 256u + b1 : op;
                d = lds_dtab[di];
                u = lds_dtab[512u + di];
                bytes = op | (b1 << 8) | (b2 << 16);
            }
            cycles = PK_D_CYC(d);
            L.icount += 1u;
            PK_TRACE(env, pc, L.w0, L.w1, L.sp, bytes & 0xFFu);
        } else if (dispatch) {
            d = PK_C_INT | (PK_M_PUSH2 << 12);
            u = (PK_K_INT << 18) | (1u << 22) | (1u << 24);
        }
        const u32 b1 = bfe8(bytes, 8);
        const u32 imm16 = (bytes >> 8) & 0xFFFFu;
        const u32 fa = PK_D_A(d), fb = PK_D_B(d), sub = PK_D_OP(d);
        const u32 ctrl = PK_U_CTRL(u);
        u32 w0 = L.w0, w1 = L.w1;
        const u32 sp_old = L.sp;
        const u32 hl = w1 & 0xFFFFu;
        u32 f = bfe8(w1, 24);
        // field a holds a condition only for JP/JR/CALL/RET (RST uses it for the vector)
        const bool condctl = ctrl == PK_K_JP || ctrl == PK_K_JR || ctrl == PK_K_CALL || ctrl == PK_K_RET;
        const bool taken = !condctl || cond_ok(f, fa);

        // ---------------- memory reads (0, 1 or 2; one load each) ----------------
        u32 rmode = PK_D_RD(d);
        if (ctrl == PK_K_RET && !taken) rmode = PK_M_NONE;
        u32 m0 = 0, m1 = 0;
        if (rmode != PK_M_NONE) {
            const u32 addr = (rmode == PK_M_HL || rmode == PK_M_HLI || rmode == PK_M_HLD) ? hl
                           : rmode == PK_M_BC ? (w0 & 0xFFFFu)
                           : rmode == PK_M_DE ? (w0 >> 16)
                           : rmode == PK_M_NN ? imm16
                           : rmode == PK_M_HN ? (0xFF00u | b1)
                           : rmode == PK_M_HC ? (0xFF00u | (w0 & 0xFFu))
                           : sp_old;
            m0 = bus_read(A, RL, m, L, addr);
            if (rmode == PK_M_SP2) m1 = bus_read(A, RL, m, L, (addr + 1u) & 0xFFFFu);
        }

        // ---------------- compute: ONE fused, branch-free datapath driven by the microcode ----------------
        const u32 a = bfe8(w1, 16);
        const u32 fc = (f >> 4) & 1u;
        const u32 tgt = fa == 6u ? m0 : rd8(w0, w1, fa);
        const u32 src8 = fb == PK_SRC_IMM ? b1 : fb == 6u ? m0 : rd8(w0, w1, fb & 7u);
        const u32 X = PK_U_XTGT(u) ? tgt : a;
        const u32 Y = PK_U_YONE(u) ? 1u : src8;
        // 8-bit adder (ADD ADC SUB SBC CP, INC, DEC)
        const u32 arith = PK_U_ARITH(u);
        const bool isSub = arith == 2u || (arith == 0u && (sub == 2u || sub == 3u || sub == 7u));
        const u32 c_in = (arith == 0u && (sub == 1u || sub == 3u)) ? fc : 0u;
        const u32 yy = isSub ? (~Y & 0xFFu) : Y;
        const u32 cin = isSub ? (1u - c_in) : c_in;
        const u32 r9 = X + yy + cin;
        const u32 hadd = ((((X & 0xFu) + (yy & 0xFu) + cin) >> 4) & 1u) ^ (isSub ? 1u : 0u);
        const u32 cadd = ((r9 >> 8) & 1u) ^ (isSub ? 1u : 0u);
        // logic (AND XOR OR)
        const u32 lres = sub == 4u ? (X & Y) : sub == 5u ? (X ^ Y) : (X | Y);
        // rotate/shift unit (RLC RRC RL RR SLA SRA SWAP SRL; RLCA.. use sub-ops 0..3 on A)
        const u32 rl = ((X << 1) | ((sub & 2u) ? fc : (X >> 7))) & 0xFFu;
        const u32 rr = (X >> 1) | (((sub & 2u) ? fc : (X & 1u)) << 7);
        const u32 rot = sub <= 3u ? ((sub & 1u) ? rr : rl)
                      : sub == 4u ? ((X << 1) & 0xFFu) : sub == 5u ? ((X >> 1) | (X & 0x80u))
                      : sub == 6u ? (((X >> 4) | (X << 4)) & 0xFFu) : (X >> 1);
        const u32 rotc = (sub == 0u || sub == 2u || sub == 4u) ? (X >> 7) : sub == 6u ? 0u : (X & 1u);
        const u32 bm = 1u << (fb & 7u);
        // DAA (opcodes.py DAA_27) on A
        u32 corr = ((f & 0x20u) ? 0x06u : 0u) | ((f & 0x10u) ? 0x60u : 0u);
        corr |= (f & 0x40u) ? 0u : (((a & 0x0Fu) > 0x09u ? 0x06u : 0u) | (a > 0x99u ? 0x60u : 0u));
        const u32 daa = ((f & 0x40u) ? (a - corr) : (a + corr)) & 0xFFu;
        const u32 r8sel = PK_U_R8SEL(u);
        const u32 res8 = r8sel == 1u ? Y : r8sel == 2u ? (r9 & 0xFFu) : r8sel == 3u ? lres : r8sel == 4u ? rot
                       : r8sel == 5u ? (X & ~bm) : r8sel == 6u ? (X | bm) : r8sel == 7u ? daa : r8sel == 8u ? (~a & 0xFFu) : X;
        const u32 zf = res8 == 0u ? 0x80u : 0u;
        // 16-bit unit
        const u32 op16 = PK_U_OP16(u);
        const u32 rp = rd16(w0, w1, sp_old, fa);
        const u32 spe = (sp_old + sext8(b1)) & 0xFFFFu;
        const u32 popv = m0 | (m1 << 8);
        const u32 addhl = hl + rp;
        // flags
        const u32 fmode = PK_U_FMODE(u);
        const bool logic = sub >= 4u && sub <= 6u;
        const u32 f_alu = zf | (isSub ? 0x40u : 0u) | ((logic ? (sub == 4u ? 1u : 0u) : hadd) << 5) | ((logic ? 0u : cadd) << 4);
        const u32 f_spe = ((((sp_old & 0xFu) + (b1 & 0xFu)) > 0xFu) ? 0x20u : 0u) | ((((sp_old & 0xFFu) + b1) > 0xFFu) ? 0x10u : 0u);
        f = fmode == PK_F_ALU ? f_alu
          : fmode == PK_F_INCDEC ? (zf | (isSub ? 0x40u : 0u) | (hadd << 5) | (f & 0x10u))
          : fmode == PK_F_ROTA ? (rotc << 4)
          : fmode == PK_F_CBROT ? (zf | (rotc << 4))
          : fmode == PK_F_BIT ? ((f & 0x10u) | 0x20u | ((X & bm) ? 0u : 0x80u))
          : fmode == PK_F_DAA ? ((f & 0x40u) | zf | ((corr & 0x60u) ? 0x10u : 0u))
          : fmode == PK_F_CPL ? (f | 0x60u)
          : fmode == PK_F_SCF ? ((f & 0x80u) | 0x10u)
          : fmode == PK_F_CCF ? ((f & 0x80u) | ((f & 0x10u) ^ 0x10u))
          : fmode == PK_F_ADDHL ? ((f & 0x80u) | ((((hl & 0xFFFu) + (rp & 0xFFFu)) > 0xFFFu) ? 0x20u : 0u) | ((addhl > 0xFFFFu) ? 0x10u : 0u))
          : fmode == PK_F_ADDSPE ? f_spe
          : fmode == PK_F_POPAF ? (m0 & 0xF0u)
          : f;
        // 8-bit writeback
        const u32 dst8 = PK_U_DST8(u);
        if (dst8 == 1u) w1 = setb8(w1, 16, res8);
        if (dst8 == 2u && fa != 6u) wr8(w0, w1, fa, res8);
        // 16-bit writeback (pair fa: BC DE HL SP; POP AF special)
        u32 sp = sp_old;
        const u32 v16 = op16 == PK_O_LD16 ? imm16 : op16 == PK_O_INC16 ? rp + 1u : op16 == PK_O_DEC16 ? rp - 1u
                      : op16 == PK_O_POP ? popv : op16 == PK_O_ADDHL ? addhl : spe;
        const u32 p16 = (op16 == PK_O_ADDHL || op16 == PK_O_SPE_HL) ? 2u : (op16 == PK_O_SPE_SP || op16 == PK_O_SPHL) ? 3u : fa;
        if (op16 != PK_O_NONE && op16 != PK_O_POPAF) wr16(w0, w1, sp, p16, op16 == PK_O_SPHL ? hl : v16);
        if (op16 == PK_O_POPAF) w1 = setb8(w1, 16, m1);
        w1 = setb8(w1, 24, f);
        // control transfer
        u32 npc = (pc + PK_D_LEN(d)) & 0xFFFFu;
        const u32 push_pc = ctrl == PK_K_INT ? pc : npc;
        const u32 jr_t = (pc + 2u + sext8(b1)) & 0xFFFFu;
        const u32 tgt_pc = ctrl == PK_K_JP || ctrl == PK_K_CALL ? imm16 : ctrl == PK_K_JPHL ? hl : ctrl == PK_K_JR ? jr_t
                         : (ctrl == PK_K_RET || ctrl == PK_K_RETI) ? popv : ctrl == PK_K_RST ? fa * 8u
                         : ctrl == PK_K_INT ? 0x40u + 8u * (u32)__builtin_ctz(intflag | 0x20u) : pc;
        const bool jump = ctrl != PK_K_SEQ && taken;
        npc = jump ? tgt_pc : npc;
        if (jump && ctrl <= PK_K_RETI) cycles += PK_D_XCYC(d);
        u32 cpu2 = L.cpu;
        const u32 ime = PK_U_IME(u);
        cpu2 = ime == 1u ? (cpu2 & ~CPU_IME) : ime == 2u ? (cpu2 | CPU_IME) : cpu2;
        cpu2 |= ctrl == PK_K_HALT ? CPU_HALT : ctrl == PK_K_ILLEGAL ? (CPU_CRASH | CPU_HALT) : 0u;
        if (ctrl == PK_K_INT) cpu2 ^= intflag << 16;   // IF ^= flag
        L.cpu = cpu2;
        // write data
        const u32 wsrc = PK_U_WSRC(u);
        const u32 pushv = wsrc == 1u ? push_pc : (fa == 3u ? ((a << 8) | bfe8(L.w1, 24)) : rp);
        const u32 wv0 = wsrc == 0u ? res8 : wsrc == 3u ? (sp_old & 0xFFu) : (pushv >> 8);
        const u32 wv1 = wsrc == 3u ? (sp_old >> 8) : (pushv & 0xFFu);
        u32 wmode = PK_D_WR(d);
        if (ctrl == PK_K_CALL && !taken) wmode = PK_M_NONE;
        // stack pointer moves of PUSH/CALL/RST/INT (PUSH2) and POP/RET (SP2)
        if (wmode == PK_M_PUSH2) sp = (sp_old - 2u) & 0xFFFFu;
        if (rmode == PK_M_SP2) sp = (sp_old + 2u) & 0xFFFFu;

        // ---------------- memory writes (0, 1 or 2; one store each) ----------------
        L.w0 = w0;
        L.w1 = w1;
        if (wmode != PK_M_NONE) {
            const u32 addr = (wmode == PK_M_HL || wmode == PK_M_HLI || wmode == PK_M_HLD) ? hl
                           : wmode == PK_M_BC ? (w0 & 0xFFFFu)
                           : wmode == PK_M_DE ? (w0 >> 16)
                           : (wmode == PK_M_NN || wmode == PK_M_NN2) ? imm16
                           : wmode == PK_M_HN ? (0xFF00u | b1)
                           : wmode == PK_M_HC ? (0xFF00u | (w0 & 0xFFu))
                           : ((sp_old - 1u) & 0xFFFFu);
            const u32 nw = (wmode == PK_M_PUSH2 || wmode == PK_M_NN2) ? 2u : 1u;
#pragma unroll 1
            for (u32 k = 0; k < nw; k++) {
                const u32 wa = k == 0u ? addr : wmode == PK_M_PUSH2 ? ((addr - 1u) & 0xFFFFu) : ((addr + 1u) & 0xFFFFu);
                bus_write(A, RL, m, L, env, gid, wa, k == 0u ? wv0 : wv1);
            }
        }
        // HL post-increment/decrement ((HL+)/(HL-) forms)
        if (rmode == PK_M_HLI || wmode == PK_M_HLI) L.w1 = (L.w1 & 0xFFFF0000u) | ((hl + 1u) & 0xFFFFu);
        if (rmode == PK_M_HLD || wmode == PK_M_HLD) L.w1 = (L.w1 & 0xFFFF0000u) | ((hl - 1u) & 0xFFFFu);
        if (exec || dispatch) {
            L.pc = npc;
            L.sp = sp;
        } else {
            L.pc = pc;
        }
        if (exec) L.cpu &= ~CPU_QUEUED;

        // ---------------- HALT fast-forward + timer + LCD (pyboy mb.tick) ----------------
        if (L.cpu & CPU_HALT) {
            const int ta = (int)L.target - (int)L.clock;
            const int tb = timer_cycles_to_interrupt(L);
            const int mm = ta < tb ? ta : tb;
            cycles = mm < 0 ? 0u : (u32)mm;
        }
        u32 irq = timer_tick(L, cycles);
        irq |= lcd_tick(A, L, gid, lane, cycles);
        if (irq) S_IF(L, G_IF(L) | irq);
        budget += cycles + 1u;
        if (budget > 16u * FRAME_CYCLES) L.frame_done = 1u;
        if (L.frame_done) {
            L.frame_done = 0;
            budget = 0;
            frame += 1u;
            if (frame == A.release_frame && btn != 0xFFu) key_event(L, btn, false);
            L.render = (A.render_last && frame + 1u == A.frames) ? 1u : 0u;
            if (L.render) {
                u32* lat2 = A.lat + 2u * A.lat_stride;
                for (u32 y = 0; y < PK_ROWS; y++) lat2[(gid * PK_ROWS + y) * PK_LANES + lane] &= ~0x100u;
            }
        }
    }

    if (!active) return;
    R[PK_R_W0 * np + env] = L.w0;
    R[PK_R_W1 * np + env] = L.w1;
    R[PK_R_SP * np + env] = L.sp;
    R[PK_R_PC * np + env] = L.pc;
    R[PK_R_CPU * np + env] = L.cpu;
    R[PK_R_CLOCK * np + env] = L.clock;
    R[PK_R_TARGET * np + env] = L.target;
    R[PK_R_LCD0 * np + env] = L.lcd0;
    R[PK_R_LCD1 * np + env] = L.lcd1;
    R[PK_R_LCD2 * np + env] = L.lcd2;
    R[PK_R_TIM0 * np + env] = (L.tim0 & 0xFFFFFF00u) | ((L.divacc >> 8) & 0xFFu);
    R[PK_R_TIM1 * np + env] = (L.divacc & 0xFFu) | (L.timac << 16);
    R[PK_R_MBC * np + env] = L.mbc;
    R[PK_R_MISC * np + env] = L.misc;
    R[PK_R_TIME * np + env] += 1u;
    R[PK_R_ICOUNT * np + env] = L.icount;
    R[PK_R_RFLAGS * np + env] = L.blank | (L.npend << 8);
}

// ---------------------------------------------------------------------------------------------
// K2: rasterise the latched lines of the rendered frame.  One wave = one (group, scanline),
// lane = env: the 64 lanes read the same VRAM offsets of their interleaved images (coalesced).
__global__ void __launch_bounds__(64) pk_render_kernel(PkStepArgs A) {
    const u32 y = blockIdx.x % PK_ROWS;
    const u32 gid = blockIdx.x / PK_ROWS;
    const u32 lane = threadIdx.x;
    const u32 env = gid * PK_LANES + lane;
    if (env >= A.n) return;
    const u32 rf = A.regs[PK_R_RFLAGS * A.npad + env];
    u8* out = A.screen + (size_t)env * PK_SCREEN + y * PK_COLS;
    if (rf & 1u) {  // frame ended with the LCD off: blank_screen() (white)
        uint4 wv;
        wv.x = wv.y = wv.z = wv.w = 0xFFFFFFFFu;
        for (u32 q = 0; q < PK_COLS; q += 16) *reinterpret_cast<uint4*>(out + q) = wv;
        return;
    }
    const u32 idx = (gid * PK_ROWS + y) * PK_LANES + lane;
    const u32 l2 = A.lat[2u * A.lat_stride + idx];
    if (!(l2 & 0x100u)) return;
    Mem m;
    m.g = A.mem + (size_t)gid * PK_GROUP_STRIDE;
    m.lane = lane;
    render_line(m, y, A.lat[idx], A.lat[A.lat_stride + idx], (int)(l2 & 0xFFu) - 1, out);
    A.lat[2u * A.lat_stride + idx] = l2 & ~0x100u;
}

// ---------------------------------------------------------------------------------------------
// K5: reset selected envs from the template (regs + RAM image + screen + line latches).


__global__ void __launch_bounds__(256) pk_reset_mem_kernel(PkResetArgs A) {
    // grid-stride over (group, phys/16): each thread writes 16 lanes' bytes of one phys row? No:
    // one thread = one (env, 16 consecutive phys bytes)
    const size_t total = (size_t)A.npad * (PK_PHYS / 16u);
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        // t enumerates (gid, row16, lane) with lane fastest so that stores are coalesced
        u32 lane = (u32)(t % PK_LANES);
        size_t r = t / PK_LANES;
        u32 chunk = (u32)(r % (PK_PHYS / 16u));
        u32 gid = (u32)(r / (PK_PHYS / 16u));
        u32 env = gid * PK_LANES + lane;
        if (env >= A.n) continue;
        if (A.mask && !A.mask[env]) continue;
        u8* g = A.mem + (size_t)gid * PK_GROUP_STRIDE;
        const u8* src = A.tmpl_mem + chunk * 16u;
        for (u32 k = 0; k < 16u; k++) g[(chunk * 16u + k) * PK_LANES + lane] = src[k];
    }
}

__global__ void __launch_bounds__(256) pk_reset_regs_kernel(PkResetArgs A) {
    const u32 env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= A.n) return;
    if (A.mask && !A.mask[env]) return;
    for (u32 f = 0; f < PK_NREGS; f++) A.regs[f * A.npad + env] = A.tmpl_regs[f];
    const u32 gid = env / PK_LANES, lane = env % PK_LANES;
    for (u32 k = 0; k < 3u; k++)
        for (u32 y = 0; y < PK_ROWS; y++)
            A.lat[k * A.lat_stride + (gid * PK_ROWS + y) * PK_LANES + lane] = A.tmpl_lat[k * PK_ROWS + y];
    const uint4* s = reinterpret_cast<const uint4*>(A.tmpl_screen);
    uint4* d = reinterpret_cast<uint4*>(A.screen + (size_t)env * PK_SCREEN);
    for (u32 q = 0; q < PK_SCREEN / 16u; q++) d[q] = s[q];
}

// gather one env's RAM image into a compact buffer (for pk_snapshot / pk_peek)
__global__ void pk_gather_env_kernel(const u8* mem, u32 env, u8* out) {
    const u32 gid = env / PK_LANES, lane = env % PK_LANES;
    const u8* g = mem + (size_t)gid * PK_GROUP_STRIDE;
    for (u32 p = blockIdx.x * blockDim.x + threadIdx.x; p < PK_PHYS; p += gridDim.x * blockDim.x)
        out[p] = g[p * PK_LANES + lane];
}

__global__ void pk_scatter_env_kernel(u8* mem, u32 env, const u8* in) {
    const u32 gid = env / PK_LANES, lane = env % PK_LANES;
    u8* g = mem + (size_t)gid * PK_GROUP_STRIDE;
    for (u32 p = blockIdx.x * blockDim.x + threadIdx.x; p < PK_PHYS; p += gridDim.x * blockDim.x)
        g[p * PK_LANES + lane] = in[p];
}

// ---------------------------------------------------------------------------------------------
// host-side launchers (called by the C ABI in pk_capi.cpp)
hipError_t pk_launch_step(const PkStepArgs& a, hipStream_t s) {
    const u32 block = 256;
    const u32 grid = (a.npad + block - 1) / block;
    hipLaunchKernelGGL(pk_step_kernel, dim3(grid), dim3(block), 0, s, a);
    return hipGetLastError();
}

hipError_t pk_launch_render(const PkStepArgs& a, hipStream_t s) {
    const u32 grid = (a.npad / PK_LANES) * PK_ROWS;
    hipLaunchKernelGGL(pk_render_kernel, dim3(grid), dim3(PK_LANES), 0, s, a);
    return hipGetLastError();
}

hipError_t pk_launch_reset(const PkResetArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pk_reset_mem_kernel, dim3(2048), dim3(256), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pk_reset_regs_kernel, dim3((a.npad + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t pk_launch_gather_env(const u8* mem, u32 env, u8* out, hipStream_t s) {
    hipLaunchKernelGGL(pk_gather_env_kernel, dim3(64), dim3(256), 0, s, mem, env, out);
    return hipGetLastError();
}

hipError_t pk_launch_scatter_env(u8* mem, u32 env, const u8* in, hipStream_t s) {
    hipLaunchKernelGGL(pk_scatter_env_kernel, dim3(64), dim3(256), 0, s, mem, env, in);
    return hipGetLastError();
}

__global__ void pk_done_kernel(const u32* time_reg, u32 n, u32 max_steps, u8* term, u8* trunc, double* rew) {
    const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const u8 done = time_reg[e] >= max_steps ? 1 : 0;
    if (term) term[e] = done;
    if (trunc) trunc[e] = done;
    if (rew) rew[e] = 0.0;
}

hipError_t pk_launch_done(const u32* time_reg, u32 n, u32 max_steps, u8* term, u8* trunc, double* rew, hipStream_t s) {
    hipLaunchKernelGGL(pk_done_kernel, dim3((n + 255) / 256), dim3(256), 0, s, time_reg, n, max_steps, term, trunc, rew);
    return hipGetLastError();
}
