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



// ---------------------------------------------------------------------------------------------
// lane state kept in VGPRs for the whole launch
struct Lane {
    u32 w0, w1, sp, pc;
    u32 cpu;            // ime | halted<<1 | queued<<2 | crashed<<3 | stopped<<4 | IE<<8 | IF<<16
    u32 clock, target;
    u32 lcd0, lcd1, lcd2;
    u32 tim0, tim1;
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
// LCD tick (pyboy lcd.py LCD.tick) — oracle: gbcore.c lcd_tick
__device__ __forceinline__ u32 lcd_tick(const PkStepArgs& A, Lane& L, u32 gid, u32 lane, u32 cycles) {
    u32 intr = 0;
    L.clock += cycles;
    u32 lcdc = G_LCDC(L);
    if (lcdc & 0x80u) {
        if (L.clock >= L.target) {
            u32 nmode = bfe8(L.lcd2, 24);
            intr |= stat_set_mode(L, nmode);
            u32 mode = G_STAT(L) & 3u;
            u32 ly = G_LY(L);
            if (mode == 2u) {
                if (ly == 153u) {
                    ly = 0;
                    L.clock %= FRAME_CYCLES;
                    L.target %= FRAME_CYCLES;
                } else {
                    ly += 1u;
                }
                L.lcd0 = setb8(L.lcd0, 16, ly);
                L.target += 80u;
                L.lcd2 = setb8(L.lcd2, 24, 3u);
                intr |= stat_update_lyc(L);
            } else if (mode == 3u) {
                L.target += 170u;
                L.lcd2 = setb8(L.lcd2, 24, 0u);
            } else if (mode == 0u) {
                L.target += 206u;
                if (L.render && ly < PK_ROWS) {
                    // latch this scanline's registers; rasterised by K2 (or flush_lines)
                    u32 lcd1 = L.lcd1;
                    u32 wy = bfe8(lcd1, 16), wx = bfe8(lcd1, 24);
                    int lw = (int)bfe8(L.misc, 16) - 1;
                    if ((lcdc & 0x20u) && wy <= ly && (int)wx - 7 < (int)PK_COLS) lw += 1;
                    u32 idx = (gid * PK_ROWS + ly) * PK_LANES + lane;
                    A.lat[idx] = lcdc | (bfe8(lcd1, 8) << 8) | (bfe8(lcd1, 0) << 16) | (wx << 24);
                    A.lat[A.lat_stride + idx] = wy | ((L.lcd2 & 0xFFFFFFu) << 8);
                    A.lat[2u * A.lat_stride + idx] = (u32)(lw + 1) | 0x100u;
                    if (ly == PK_ROWS - 1u) lw = -1;
                    L.misc = setb8(L.misc, 16, (u32)(lw + 1));
                    L.npend += 1u;
                }
                L.lcd2 = setb8(L.lcd2, 24, (ly < 143u) ? 2u : 1u);
            } else {
                L.target += 456u;
                L.lcd2 = setb8(L.lcd2, 24, 1u);
                ly += 1u;
                L.lcd0 = setb8(L.lcd0, 16, ly);
                intr |= stat_update_lyc(L);
                if (ly == 144u) {
                    intr |= 1u;
                    L.frame_done = 1u;
                }
                if (ly == 153u) L.lcd2 = setb8(L.lcd2, 24, 2u);
            }
        }
    } else {
        if (L.clock >= FRAME_CYCLES) {
            L.frame_done = 1u;
            L.clock %= FRAME_CYCLES;
            if (L.render) L.blank = 1u;
        }
    }
    return intr;
}

// timer (pyboy timer.py Timer.tick) — oracle: gbcore.c timer_tick
__device__ __forceinline__ u32 timer_tick(Lane& L, u32 cycles) {
    u32 divc = (L.tim1 & 0xFFFFu) + cycles;
    u32 div = (bfe8(L.tim0, 0) + (divc >> 8)) & 0xFFu;
    divc &= 0xFFu;
    u32 r = 0;
    u32 tac = bfe8(L.tim0, 24);
    u32 timac = L.tim1 >> 16;
    u32 tima = bfe8(L.tim0, 8);
    if (tac & 4u) {
        timac += cycles;
        u32 dsh = ((tac & 3u) == 0u) ? 10u : ((tac & 3u) == 1u) ? 4u : ((tac & 3u) == 2u) ? 6u : 8u;
        u32 d = 1u << dsh;
        if (timac >= d) {
            u32 mul = timac >> dsh;
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
    }
    L.tim0 = setb8(L.tim0, 0, div);
    L.tim1 = divc | (timac << 16);
    return r;
}

__device__ __forceinline__ int timer_cycles_to_interrupt(const Lane& L) {
    u32 tac = bfe8(L.tim0, 24);
    if (!(tac & 4u)) return 1 << 16;
    u32 dsh = ((tac & 3u) == 0u) ? 10u : ((tac & 3u) == 1u) ? 4u : ((tac & 3u) == 2u) ? 6u : 8u;
    return (int)((0x100u - bfe8(L.tim0, 8)) << dsh) - (int)(L.tim1 >> 16);
}

// joypad (pyboy interaction.py) — oracle: gbcore.c gb_button / joy_pull
__device__ __forceinline__ void key_event(Lane& L, u32 button, bool pressed) {
    u32 od = bfe8(L.misc, 0), os = bfe8(L.misc, 8);
    u32 nd = od, ns = os;
    u32 bit = 1u << (button & 3u);
    if (button < 4u) nd = pressed ? (nd & ~bit) : (nd | bit);
    else ns = pressed ? (ns & ~bit) : (ns | bit);
    L.misc = (L.misc & 0xFFFF0000u) | nd | (ns << 8);
    if (((od ^ nd) & od) || ((os ^ ns) & os)) S_IF(L, G_IF(L) | 0x10u);
}

__device__ __forceinline__ u32 joy_pull(const Lane& L, u32 v) {
    u32 p14 = (v >> 4) & 1u, p15 = (v >> 5) & 1u;
    u32 r = (v | 0xCFu) & 0xFFu;
    if (p14 != p15) r &= (!p14) ? bfe8(L.misc, 0) : bfe8(L.misc, 8);
    return r;
}

// ---------------------------------------------------------------------------------------------
// memory bus (pyboy mb.getitem / setitem) — oracle: gbcore.c bus_read / bus_write
__device__ __forceinline__ u32 rom_read(const PkStepArgs& A, const u8* lds_bank0, const Lane& L, u32 a) {
    if (a < 0x4000u) return lds_bank0[a];
    u32 bank = bfe8(L.mbc, 0) & A.rom_bank_mask;
    return A.rom[bank * 0x4000u + (a - 0x4000u)];
}

__device__ __forceinline__ u32 io_read_special(const Lane& L, u32 a) {
    switch (a) {
        case 0xFF04: return bfe8(L.tim0, 0);
        case 0xFF05: return bfe8(L.tim0, 8);
        case 0xFF06: return bfe8(L.tim0, 16);
        case 0xFF07: return bfe8(L.tim0, 24);
        case 0xFF0F: return G_IF(L);
        case 0xFF40: return G_LCDC(L);
        case 0xFF41: return G_STAT(L);
        case 0xFF42: return bfe8(L.lcd1, 0);
        case 0xFF43: return bfe8(L.lcd1, 8);
        case 0xFF44: return G_LY(L);
        case 0xFF45: return G_LYC(L);
        case 0xFF46: return 0;
        case 0xFF47: return bfe8(L.lcd2, 0);
        case 0xFF48: return bfe8(L.lcd2, 8);
        case 0xFF49: return bfe8(L.lcd2, 16);
        case 0xFF4A: return bfe8(L.lcd1, 16);
        case 0xFF4B: return bfe8(L.lcd1, 24);
        default: return 0;  // FF10-FF3F: sound not emulated
    }
}

__device__ __forceinline__ bool io_is_special(u32 a) {
    // FF04-FF07, FF0F, FF10-FF3F (sound), FF40-FF4B
    return (a >= 0xFF04u && a <= 0xFF07u) || a == 0xFF0Fu || (a >= 0xFF10u && a <= 0xFF4Bu);
}

__device__ __forceinline__ u32 bus_read(const PkStepArgs& A, const u8* lds_bank0, const Mem& m, const Lane& L, u32 a) {
    if (a < 0x8000u) return rom_read(A, lds_bank0, L, a);
    u32 phys;
    if (a < 0xA000u) {
        phys = PK_P_VRAM + (a - 0x8000u);
    } else if (a < 0xC000u) {
        if (A.mbc == 0u || !bfe8(L.mbc, 16)) return 0xFFu;
        phys = PK_P_SRAM + (bfe8(L.mbc, 8) & 3u) * 0x2000u + (a - 0xA000u);
    } else if (a < 0xFE00u) {
        phys = PK_P_WRAM + (a & 0x1FFFu);
    } else if (a < 0xFF00u) {
        phys = PK_P_OAM + (a - 0xFE00u);
    } else if (a >= 0xFF80u) {
        if (a == 0xFFFFu) return G_IE(L);
        phys = PK_P_HRAM + (a - 0xFF80u);
    } else if (io_is_special(a)) {
        return io_read_special(L, a);
    } else {
        phys = PK_P_IO + (a - 0xFF00u);
    }
    return ld_phys(m, phys);
}

__device__ __forceinline__ void lcd_set_lcdc(Lane& L, u32 v) {
    L.lcd0 = setb8(L.lcd0, 0, v);
    if (!(v & 0x80u)) {
        L.clock = 0;
        L.target = FRAME_CYCLES;
        (void)stat_set_mode(L, 0u);
        L.lcd2 = setb8(L.lcd2, 24, 2u);
        L.lcd0 = setb8(L.lcd0, 16, 0u);
    }
}


__device__ __forceinline__ void oam_dma(const PkStepArgs& A, const u8* lds_bank0, const Mem& m, Lane& L, u32 env, u32 gid, u32 v) {
    u32 src = v << 8;
    FLUSH_PENDING();
    for (u32 n = 0; n < 0xA0u; n++) {
        u32 b = bus_read(A, lds_bank0, m, L, (src + n) & 0xFFFFu);
        st_phys(m, PK_P_OAM + n, b);
    }
}

__device__ __forceinline__ void io_write_special(const PkStepArgs& A, const u8* lds_bank0, const Mem& m, Lane& L, u32 env, u32 gid, u32 a, u32 v) {
    switch (a) {
        case 0xFF04: L.tim0 = setb8(L.tim0, 0, 0u); L.tim1 = 0u; break;
        case 0xFF05: L.tim0 = setb8(L.tim0, 8, v); break;
        case 0xFF06: L.tim0 = setb8(L.tim0, 16, v); break;
        case 0xFF07: L.tim0 = setb8(L.tim0, 24, v & 7u); break;
        case 0xFF0F: S_IF(L, v); break;
        case 0xFF40: lcd_set_lcdc(L, v); break;
        case 0xFF41: L.lcd0 = setb8(L.lcd0, 8, (G_STAT(L) & 0x87u) | (v & 0x78u)); break;
        case 0xFF42: L.lcd1 = setb8(L.lcd1, 0, v); break;
        case 0xFF43: L.lcd1 = setb8(L.lcd1, 8, v); break;
        case 0xFF44: break;
        case 0xFF45: L.lcd0 = setb8(L.lcd0, 24, v); break;
        case 0xFF46: oam_dma(A, lds_bank0, m, L, env, gid, v); break;
        case 0xFF47: L.lcd2 = setb8(L.lcd2, 0, v); break;
        case 0xFF48: L.lcd2 = setb8(L.lcd2, 8, v); break;
        case 0xFF49: L.lcd2 = setb8(L.lcd2, 16, v); break;
        case 0xFF4A: L.lcd1 = setb8(L.lcd1, 16, v); break;
        case 0xFF4B: L.lcd1 = setb8(L.lcd1, 24, v); break;
        default: break;  // sound not emulated
    }
}

__device__ __forceinline__ void mbc_write(const PkStepArgs& A, Lane& L, u32 a, u32 v) {
    if (A.mbc == 0u) return;
    if (a < 0x2000u) {
        L.mbc = setb8(L.mbc, 16, ((v & 0x0Fu) == 0x0Au) ? 1u : 0u);
    } else if (a < 0x4000u) {
        v &= 0x7Fu;
        if (v == 0u) v = 1u;
        L.mbc = setb8(L.mbc, 0, v);
    } else if (a < 0x6000u) {
        L.mbc = setb8(L.mbc, 8, v);
    }
}

__device__ __forceinline__ void bus_write(const PkStepArgs& A, const u8* lds_bank0, const Mem& m, Lane& L, u32 env, u32 gid, u32 a, u32 v) {
    if (a < 0x8000u) { mbc_write(A, L, a, v); return; }
    u32 phys;
    if (a < 0xA000u) {
        FLUSH_PENDING();
        phys = PK_P_VRAM + (a - 0x8000u);
    } else if (a < 0xC000u) {
        if (A.mbc == 0u || !bfe8(L.mbc, 16)) return;
        phys = PK_P_SRAM + (bfe8(L.mbc, 8) & 3u) * 0x2000u + (a - 0xA000u);
    } else if (a < 0xFE00u) {
        phys = PK_P_WRAM + (a & 0x1FFFu);
    } else if (a < 0xFF00u) {
        if (a < 0xFEA0u) FLUSH_PENDING();
        phys = PK_P_OAM + (a - 0xFE00u);
    } else if (a >= 0xFF80u) {
        if (a == 0xFFFFu) { S_IE(L, v); return; }
        phys = PK_P_HRAM + (a - 0xFF80u);
    } else if (a == 0xFF00u) {
        v = joy_pull(L, v);
        phys = PK_P_IO;
    } else if (io_is_special(a)) {
        io_write_special(A, lds_bank0, m, L, env, gid, a, v);
        return;
    } else {
        phys = PK_P_IO + (a - 0xFF00u);
    }
    st_phys(m, phys, v);
}

// ---------------------------------------------------------------------------------------------
// register file helpers (W0 = C|B<<8|E<<16|D<<24, W1 = L|H<<8|A<<16|F<<24)
// NOTE: selections between lane-state fields are written as arithmetic on VALUES. A C++
// `cond ? L.w1 : L.w0` (or an if/else storing to one of two fields) lets LLVM form a select of
// field ADDRESSES, which forces the whole Lane struct into scratch memory.
__device__ __forceinline__ u32 rd8(const Lane& L, u32 r) {
    const u32 sel = 0u - ((r >> 2) & 1u);
    const u32 w = (L.w0 & ~sel) | (L.w1 & sel);
    return bfe8(w, ((r ^ 1u) & 3u) * 8u);
}
__device__ __forceinline__ void wr8(Lane& L, u32 r, u32 v) {
    const u32 sh = ((r ^ 1u) & 3u) * 8u;
    const u32 sel = 0u - ((r >> 2) & 1u);
    const u32 msk = 0xFFu << sh, nv = (v & 0xFFu) << sh;
    const u32 w0 = L.w0, w1 = L.w1;
    L.w0 = (w0 & ~(msk & ~sel)) | (nv & ~sel);
    L.w1 = (w1 & ~(msk & sel)) | (nv & sel);
}
__device__ __forceinline__ u32 rd16(const Lane& L, u32 p) {  // BC DE HL SP
    const u32 w0 = L.w0, w1 = L.w1, sp = L.sp;
    const u32 lo = (p & 1u) ? (w0 >> 16) : (w0 & 0xFFFFu);
    const u32 hi = (p & 1u) ? sp : (w1 & 0xFFFFu);
    return (p & 2u) ? hi : lo;
}
__device__ __forceinline__ void wr16(Lane& L, u32 p, u32 v) {
    v &= 0xFFFFu;
    const u32 w0 = L.w0, w1 = L.w1, sp = L.sp;
    const u32 n0 = p == 0u ? ((w0 & 0xFFFF0000u) | v) : p == 1u ? ((w0 & 0xFFFFu) | (v << 16)) : w0;
    const u32 n1 = p == 2u ? ((w1 & 0xFFFF0000u) | v) : w1;
    const u32 ns = p == 3u ? v : sp;
    L.w0 = n0;
    L.w1 = n1;
    L.sp = ns;
}
#define A_(L) bfe8((L).w1, 16)
#define F_(L) bfe8((L).w1, 24)
#define HL_(L) ((L).w1 & 0xFFFFu)
#define SETA(L, v) ((L).w1 = setb8((L).w1, 16, (v)))
#define SETF(L, v) ((L).w1 = setb8((L).w1, 24, (v)))

__device__ __forceinline__ bool cond_ok(const Lane& L, u32 a) {
    if (!(a & PK_COND_FLAG)) return true;
    u32 f = F_(L);
    u32 cc = a & 3u;
    bool z = (f & 0x80u) != 0, c = (f & 0x10u) != 0;
    return cc == 0u ? !z : cc == 1u ? z : cc == 2u ? !c : c;
}

// ---------------------------------------------------------------------------------------------
// K1: the step kernel
__global__ void __launch_bounds__(256) pk_step_kernel(PkStepArgs A) {
    __shared__ u8 lds_bank0[0x4000];
    __shared__ u32 lds_dtab[512];
    // stage ROM bank 0 (home code + vectors) and the decode table in LDS
    {
        const uint4* src = reinterpret_cast<const uint4*>(A.rom);
        uint4* dst = reinterpret_cast<uint4*>(lds_bank0);
        for (u32 i = threadIdx.x; i < 0x4000u / 16u; i += blockDim.x) dst[i] = src[i];
        for (u32 i = threadIdx.x; i < 512u; i += blockDim.x) lds_dtab[i] = A.dtab[i];
    }
    __syncthreads();

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
    L.tim0 = R[PK_R_TIM0 * np + env];
    L.tim1 = R[PK_R_TIM1 * np + env];
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
    L.render = (A.render_last && frame + 1u == A.frames) ? 1u : 0u;
    if (active && A.frames > 0u && A.release_frame == 0u && btn != 0xFFu) key_event(L, btn, false);
    if (L.render) {
        u32* lat2 = A.lat + 2u * A.lat_stride;
        for (u32 y = 0; y < PK_ROWS; y++) {
            u32 idx = (gid * PK_ROWS + y) * PK_LANES + lane;
            lat2[idx] &= ~0x100u;
        }
    }

    u32 budget = 0;  // frame watchdog (see oracle/gbcore.c PK_FRAME_BUDGET)
    while (frame < A.frames) {
        // ---------------- cpu.tick ----------------
        u32 cycles = 0;
        u32 d = (PK_C_NOP) | (1u << 6);  // no-op descriptor
        u32 b1 = 0, b2 = 0;
        bool exec = false;
        u32 cpu = L.cpu;
        u32 intv = 0, intflag = 0;
        if (cpu & CPU_CRASH) {
            cycles = 4u;
        } else {
            u32 pend = G_IF(L) & G_IE(L) & 0x1Fu;
            if (!(cpu & CPU_QUEUED) && pend) {
                if (cpu & CPU_HALT) L.pc = (L.pc + 1u) & 0xFFFFu;
                if (cpu & CPU_IME) {
                    intflag = pend & (~pend + 1u);  // lowest set bit = highest priority
                    intv = 0x40u + 8u * (u32)__builtin_ctz(intflag);
                    d = PK_C_INT | (PK_M_PUSH2 << 12);
                }
                L.cpu = (cpu | CPU_QUEUED) & ~CPU_HALT;
            } else {
                if ((cpu & CPU_HALT) && (cpu & CPU_QUEUED)) {
                    L.cpu = cpu & ~CPU_HALT;
                    L.pc = (L.pc + 1u) & 0xFFFFu;
                    exec = true;
                } else if (cpu & CPU_HALT) {
                    cycles = 4u;
                } else {
                    exec = true;
                }
            }
        }
        const u32 pc = L.pc;
        if (exec) {
            // fetch: opcode + two operand bytes
            u32 op;
            if (pc < 0x3FFEu) {
                op = lds_bank0[pc]; b1 = lds_bank0[pc + 1u]; b2 = lds_bank0[pc + 2u];
            } else if (pc >= 0x4000u && pc < 0x7FFEu) {
                const u8* rb = A.rom + (bfe8(L.mbc, 0) & A.rom_bank_mask) * 0x4000u + (pc - 0x4000u);
                op = rb[0]; b1 = rb[1]; b2 = rb[2];
            } else {
                op = bus_read(A, lds_bank0, m, L, pc);
                b1 = bus_read(A, lds_bank0, m, L, (pc + 1u) & 0xFFFFu);
                b2 = bus_read(A, lds_bank0, m, L, (pc + 2u) & 0xFFFFu);
            }
            u32 di = op;
            if (op == 0xCBu) { di = 256u + b1; }
            d = lds_dtab[di];
            cycles = PK_D_CYC(d);
            L.icount += 1u;
        }
        const u32 cls = PK_D_CLS(d);
        const u32 fa = PK_D_A(d), fb = PK_D_B(d), sub = PK_D_OP(d);
        const u32 hl = HL_(L);
        const u32 imm16 = b1 | (b2 << 8);
        const bool taken = cond_ok(L, fa);

        // ---------------- memory reads ----------------
        u32 rmode = PK_D_RD(d);
        if (cls == PK_C_RET && !taken) rmode = PK_M_NONE;
        u32 m0 = 0, m1 = 0;
        if (rmode != PK_M_NONE) {
            u32 addr = rmode == PK_M_HL || rmode == PK_M_HLI || rmode == PK_M_HLD ? hl
                     : rmode == PK_M_BC ? (L.w0 & 0xFFFFu)
                     : rmode == PK_M_DE ? (L.w0 >> 16)
                     : rmode == PK_M_NN ? imm16
                     : rmode == PK_M_HN ? (0xFF00u | b1)
                     : rmode == PK_M_HC ? (0xFF00u | bfe8(L.w0, 0))
                     : L.sp;
            const u32 nr = rmode == PK_M_SP2 ? 2u : 1u;
            for (u32 k = 0; k < nr; k++) {
                u32 v = bus_read(A, lds_bank0, m, L, (addr + k) & 0xFFFFu);
                if (k == 0) m0 = v; else m1 = v;
            }
        }

        // ---------------- compute ----------------
        u32 src8 = fb == PK_SRC_IMM ? b1 : fb == 6u ? m0 : rd8(L, fb & 7u);
        u32 wv0 = 0, wv1 = 0;
        u32 npc = (pc + PK_D_LEN(d)) & 0xFFFFu;
        u32 nsp = L.sp;
        u32 f = F_(L);
        switch (cls) {
            case PK_C_NOP: break;
            case PK_C_LD8:
                if (fa != 6u) wr8(L, fa, src8);
                wv0 = src8;
                break;
            case PK_C_ALU: {
                u32 a = A_(L), v = src8, c = (f >> 4) & 1u, r = 0;
                switch (sub) {
                    case 0: r = a + v; f = (((r & 0xFFu) == 0) ? 0x80u : 0) | ((((a & 0xFu) + (v & 0xFu)) > 0xFu) ? 0x20u : 0) | ((r > 0xFFu) ? 0x10u : 0); break;
                    case 1: r = a + v + c; f = (((r & 0xFFu) == 0) ? 0x80u : 0) | ((((a & 0xFu) + (v & 0xFu) + c) > 0xFu) ? 0x20u : 0) | ((r > 0xFFu) ? 0x10u : 0); break;
                    case 2:
                    case 7: r = a - v; f = 0x40u | (((r & 0xFFu) == 0) ? 0x80u : 0) | (((a & 0xFu) < (v & 0xFu)) ? 0x20u : 0) | ((a < v) ? 0x10u : 0); if (sub == 7u) r = a; break;
                    case 3: r = a - v - c; f = 0x40u | (((r & 0xFFu) == 0) ? 0x80u : 0) | (((a & 0xFu) < (v & 0xFu) + c) ? 0x20u : 0) | ((a < v + c) ? 0x10u : 0); break;
                    case 4: r = a & v; f = ((r == 0) ? 0x80u : 0) | 0x20u; break;
                    case 5: r = a ^ v; f = (r == 0) ? 0x80u : 0; break;
                    default: r = a | v; f = (r == 0) ? 0x80u : 0; break;
                }
                SETA(L, r & 0xFFu);
                break;
            }
            case PK_C_INC8: {
                u32 v = fa == 6u ? m0 : rd8(L, fa), r = (v + 1u) & 0xFFu;
                f = (f & 0x10u) | (r == 0 ? 0x80u : 0) | (((v & 0xFu) == 0xFu) ? 0x20u : 0);
                if (fa != 6u) wr8(L, fa, r);
                wv0 = r;
                break;
            }
            case PK_C_DEC8: {
                u32 v = fa == 6u ? m0 : rd8(L, fa), r = (v - 1u) & 0xFFu;
                f = (f & 0x10u) | 0x40u | (r == 0 ? 0x80u : 0) | (((v & 0xFu) == 0u) ? 0x20u : 0);
                if (fa != 6u) wr8(L, fa, r);
                wv0 = r;
                break;
            }
            case PK_C_ROTA:
            case PK_C_CBROT: {
                u32 v = cls == PK_C_ROTA ? A_(L) : (fa == 6u ? m0 : rd8(L, fa));
                u32 c, r;
                u32 fc = (f >> 4) & 1u;
                switch (sub) {
                    case 0: c = v >> 7; r = (v << 1) | c; break;
                    case 1: c = v & 1u; r = (v >> 1) | (c << 7); break;
                    case 2: c = v >> 7; r = (v << 1) | fc; break;
                    case 3: c = v & 1u; r = (v >> 1) | (fc << 7); break;
                    case 4: c = v >> 7; r = v << 1; break;
                    case 5: c = v & 1u; r = (v >> 1) | (v & 0x80u); break;
                    case 6: c = 0; r = (v >> 4) | (v << 4); break;
                    default: c = v & 1u; r = v >> 1; break;
                }
                r &= 0xFFu;
                if (cls == PK_C_ROTA) {
                    f = c ? 0x10u : 0u;
                    SETA(L, r);
                } else {
                    f = (r == 0 ? 0x80u : 0) | (c ? 0x10u : 0u);
                    if (fa != 6u) wr8(L, fa, r);
                    wv0 = r;
                }
                break;
            }
            case PK_C_BIT: {
                u32 v = fa == 6u ? m0 : rd8(L, fa);
                f = (f & 0x10u) | 0x20u | ((v & (1u << fb)) ? 0u : 0x80u);
                break;
            }
            case PK_C_RES:
            case PK_C_SET: {
                u32 v = fa == 6u ? m0 : rd8(L, fa);
                u32 r = cls == PK_C_RES ? (v & ~(1u << fb)) : (v | (1u << fb));
                if (fa != 6u) wr8(L, fa, r);
                wv0 = r & 0xFFu;
                break;
            }
            case PK_C_LD16: wr16(L, fa, imm16); nsp = L.sp; break;
            case PK_C_INC16: wr16(L, fa, rd16(L, fa) + 1u); nsp = L.sp; break;
            case PK_C_DEC16: wr16(L, fa, rd16(L, fa) - 1u); nsp = L.sp; break;
            case PK_C_ADDHL: {
                u32 v = rd16(L, fa), r = hl + v;
                f = (f & 0x80u) | ((((hl & 0xFFFu) + (v & 0xFFFu)) > 0xFFFu) ? 0x20u : 0) | ((r > 0xFFFFu) ? 0x10u : 0);
                L.w1 = (L.w1 & 0xFFFF0000u) | (r & 0xFFFFu);
                break;
            }
            case PK_C_ADDSP:
            case PK_C_LDHLSP: {
                u32 sp = L.sp;
                u32 r = (sp + (u32)(int)(int8_t)(u8)b1) & 0xFFFFu;
                f = ((((sp & 0xFu) + (b1 & 0xFu)) > 0xFu) ? 0x20u : 0) | ((((sp & 0xFFu) + b1) > 0xFFu) ? 0x10u : 0);
                if (cls == PK_C_ADDSP) nsp = r;
                else L.w1 = (L.w1 & 0xFFFF0000u) | r;
                break;
            }
            case PK_C_LDSPHL: nsp = hl; break;
            case PK_C_LDNNSP: wv0 = L.sp & 0xFFu; wv1 = L.sp >> 8; break;
            case PK_C_JP: if (taken) { npc = imm16; cycles += PK_D_XCYC(d); } break;
            case PK_C_JPHL: npc = hl; break;
            case PK_C_JR: if (taken) { npc = (pc + 2u + (u32)(int)(int8_t)(u8)b1) & 0xFFFFu; cycles += PK_D_XCYC(d); } break;
            case PK_C_CALL:
                if (taken) {
                    wv0 = npc >> 8; wv1 = npc & 0xFFu;
                    nsp = (L.sp - 2u) & 0xFFFFu;
                    npc = imm16;
                    cycles += PK_D_XCYC(d);
                }
                break;
            case PK_C_RET:
            case PK_C_RETI:
                if (taken) {
                    npc = m0 | (m1 << 8);
                    nsp = (L.sp + 2u) & 0xFFFFu;
                    cycles += PK_D_XCYC(d);
                    if (cls == PK_C_RETI) L.cpu |= CPU_IME;
                }
                break;
            case PK_C_RST:
                wv0 = npc >> 8; wv1 = npc & 0xFFu;
                nsp = (L.sp - 2u) & 0xFFFFu;
                npc = fa * 8u;
                break;
            case PK_C_PUSH: {
                u32 v = fa == 3u ? ((A_(L) << 8) | f) : rd16(L, fa);
                wv0 = v >> 8; wv1 = v & 0xFFu;
                nsp = (L.sp - 2u) & 0xFFFFu;
                break;
            }
            case PK_C_POP: {
                u32 v = m0 | (m1 << 8);
                if (fa == 3u) { SETA(L, v >> 8); f = v & 0xF0u; }
                else wr16(L, fa, v);
                nsp = (L.sp + 2u) & 0xFFFFu;
                break;
            }
            case PK_C_DAA: {
                int t = (int)A_(L);
                u32 corr = 0;
                if (f & 0x20u) corr |= 0x06u;
                if (f & 0x10u) corr |= 0x60u;
                if (f & 0x40u) t -= (int)corr;
                else {
                    if ((t & 0x0F) > 0x09) corr |= 0x06u;
                    if (t > 0x99) corr |= 0x60u;
                    t += (int)corr;
                }
                f = (f & 0x40u) | (((t & 0xFF) == 0) ? 0x80u : 0) | ((corr & 0x60u) ? 0x10u : 0);
                SETA(L, (u32)t & 0xFFu);
                break;
            }
            case PK_C_CPL: SETA(L, (~A_(L)) & 0xFFu); f |= 0x60u; break;
            case PK_C_SCF: f = (f & 0x80u) | 0x10u; break;
            case PK_C_CCF: f = (f & 0x80u) | ((f & 0x10u) ^ 0x10u); break;
            case PK_C_DI: L.cpu &= ~CPU_IME; break;
            case PK_C_EI: L.cpu |= CPU_IME; break;
            case PK_C_HALT: L.cpu |= CPU_HALT; npc = pc; break;
            case PK_C_ILLEGAL: L.cpu |= CPU_CRASH | CPU_HALT; npc = pc; break;
            case PK_C_INT:
                wv0 = pc >> 8; wv1 = pc & 0xFFu;
                nsp = (L.sp - 2u) & 0xFFFFu;
                npc = intv;
                S_IF(L, G_IF(L) ^ intflag);
                L.cpu &= ~CPU_IME;
                break;
            default: break;
        }
        SETF(L, f);

        // ---------------- memory writes ----------------
        u32 wmode = PK_D_WR(d);
        if (cls == PK_C_CALL && !taken) wmode = PK_M_NONE;
        if (wmode != PK_M_NONE) {
            u32 addr = wmode == PK_M_HL || wmode == PK_M_HLI || wmode == PK_M_HLD ? hl
                     : wmode == PK_M_BC ? (L.w0 & 0xFFFFu)
                     : wmode == PK_M_DE ? (L.w0 >> 16)
                     : wmode == PK_M_NN || wmode == PK_M_NN2 ? imm16
                     : wmode == PK_M_HN ? (0xFF00u | b1)
                     : wmode == PK_M_HC ? (0xFF00u | bfe8(L.w0, 0))
                     : ((L.sp - 1u) & 0xFFFFu);
            const u32 nw = (wmode == PK_M_PUSH2 || wmode == PK_M_NN2) ? 2u : 1u;
            for (u32 k = 0; k < nw; k++) {
                u32 wa = wmode == PK_M_PUSH2 ? ((addr - k) & 0xFFFFu) : ((addr + k) & 0xFFFFu);
                bus_write(A, lds_bank0, m, L, env, gid, wa, k == 0 ? wv0 : wv1);
            }
        }
        // HL post-increment/decrement ((HL+)/(HL-) forms)
        if (rmode == PK_M_HLI || wmode == PK_M_HLI) L.w1 = (L.w1 & 0xFFFF0000u) | ((hl + 1u) & 0xFFFFu);
        if (rmode == PK_M_HLD || wmode == PK_M_HLD) L.w1 = (L.w1 & 0xFFFF0000u) | ((hl - 1u) & 0xFFFFu);
        if (exec || cls == PK_C_INT) {
            L.pc = npc;
            L.sp = nsp;
        }
        if (exec) L.cpu &= ~CPU_QUEUED;

        // ---------------- HALT fast-forward + timer + LCD (pyboy mb.tick) ----------------
        if (L.cpu & CPU_HALT) {
            int a = (int)L.target - (int)L.clock;
            int b = timer_cycles_to_interrupt(L);
            int mm = a < b ? a : b;
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
                for (u32 y = 0; y < PK_ROWS; y++) {
                    u32 idx = (gid * PK_ROWS + y) * PK_LANES + lane;
                    lat2[idx] &= ~0x100u;
                }
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
    R[PK_R_TIM0 * np + env] = L.tim0;
    R[PK_R_TIM1 * np + env] = L.tim1;
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
