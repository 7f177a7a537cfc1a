// pk_render.h — device helpers shared by K1 (pk_step.hip: deferred-line flush before a VRAM/OAM
// write) and K2 (pk_kernels.hip: rasterise the latched lines of the rendered frame).
//
// DMG scanline rasteriser = PyBoy 1.x renderer.scanline + scanline_sprites as the oracle restates
// it (oracle/gbcore.c render_scanline), grey palette FF/99/55/00 of screen.screen_ndarray()
// (pokegym/environment.py:268).  Pinned on the reference's 264 savestate frames.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pk_layout.h"

typedef uint32_t u32;
typedef uint8_t u8;

__device__ __forceinline__ u32 bfe8(u32 v, u32 sh) { return (v >> sh) & 0xFFu; }
__device__ __forceinline__ u32 setb8(u32 v, u32 sh, u32 b) { return (v & ~(0xFFu << sh)) | ((b & 0xFFu) << sh); }

// per-lane view of a lane-interleaved RAM image (pk_layout.h): byte(phys) = g[phys << sh | lane]
struct Mem {
    u8* g;      // the env's sub-block base
    u32 lane;   // lane within the sub-block
    u32 sh;     // interleave shift
};
__device__ __forceinline__ u32 ld_phys(const Mem& m, u32 phys) { return m.g[(phys << m.sh) + m.lane]; }
__device__ __forceinline__ void st_phys(const Mem& m, u32 phys, u32 v) { m.g[(phys << m.sh) + m.lane] = (u8)v; }
// the view of env (interleave shift sh)
__device__ __forceinline__ Mem mem_view(u8* mem, u32 env, u32 sh) {
    Mem m;
    m.g = mem + pk_img_off(env, 0u, sh) - (env & (PK_LANES - 1u) & ((1u << sh) - 1u));
    m.lane = env & (PK_LANES - 1u) & ((1u << sh) - 1u);
    m.sh = sh;
    return m;
}

// grey shade of palette index 0..3 (0xFF 0x99 0x55 0x00)
__device__ __forceinline__ u32 grey(u32 shade) { return (0x005599FFu >> (8u * shade)) & 0xFFu; }

__device__ __forceinline__ u32 bg_tile_addr(u32 lcdc, u32 t) {
    if (lcdc & 0x10u) return t * 16u;
    return (u32)(0x1000 + (int)(int8_t)(u8)t * 16);
}

// one scanline of one lane. lat0 = LCDC | SCX<<8 | SCY<<16 | WX<<24 ; lat1 = WY | BGP<<8 |
// OBP0<<16 | OBP1<<24 ; lw = window line counter after this line's increment. out: 160 grey bytes.
__device__ inline void render_line(const Mem& m, u32 y, u32 lat0, u32 lat1, int lw, u8* out) {
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
            if (win && wx > x && wx < x + run) run = wx - x;  // stop the run where the window starts
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
            for (int b = 0; b < 4; b++) a |= grey(line[q + j * 4 + b]) << (8 * b);
            w[j] = a;
        }
        v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3];
        *reinterpret_cast<uint4*>(out + q) = v;
    }
}

// host-simulation hooks (design statistics): a flush_lines call (0) and a line it rasterises (1)
#ifndef PK_FLUSH_STAT
#define PK_FLUSH_STAT(rendered) ((void)0)
#endif

// The pending-lines word K1 keeps per lane (St.npend): 0 = no latched line waits for rasterisation,
// else (highest pending line + 1) | lowest pending line << 16 — lines are latched at mode-0 events
// (and in bulk by the HALT skip-ahead), so flush_lines reads only that range's latch flags
__device__ __forceinline__ u32 pend_add(u32 p, u32 lo, u32 hi) {
    const u32 h1 = hi + 1u;
    return p == 0u ? (h1 | (lo << 16)) : ((((p & 0xFFFFu) > h1) ? (p & 0xFFFFu) : h1) | (((p >> 16) < lo ? (p >> 16) : lo) << 16));
}

// rasterise every latched-but-pending line of this lane now (before VRAM/OAM change); pend = the
// lane's pending-lines word (pend_add).  Rare path: kept out of line with by-value arguments so
// the step loop's state stays in VGPRs.
__device__ __noinline__ static void flush_lines(u32* lat, u32 lat_stride, u8* screen, u8* gbase, u32 il, u32 sh, u32 lane,
                                                u32 env, u32 gid, u32 pend) {
    Mem m;
    m.g = gbase;
    m.lane = il;
    m.sh = sh;
    u32* lat0 = lat;
    u32* lat1 = lat + lat_stride;
    u32* lat2 = lat + 2u * lat_stride;
#ifndef PK_FLUSH_FULL
    const u32 ylo = pend >> 16, yend = pend & 0xFFFFu;   // lines [ylo, yend)
#else
    const u32 ylo = 0u, yend = pend ? PK_ROWS : 0u;       // (A/B diagnostic: every line's flag)
#endif
    // the latch flags of the range are read 16 lines at a time (independent loads: one memory
    // round trip per batch instead of one per line)
    for (u32 y0 = ylo; y0 < yend; y0 += 16u) {
        u32 f[16];
#pragma unroll
        for (u32 k = 0; k < 16u; k++) {
            const u32 y = y0 + k < PK_ROWS ? y0 + k : PK_ROWS - 1u;   // (reads past the range: never used)
            f[k] = lat2[(gid * PK_ROWS + y) * PK_LANES + lane];
        }
        for (u32 k = 0; k < 16u && y0 + k < yend; k++) {
            const u32 y = y0 + k, idx = (gid * PK_ROWS + y) * PK_LANES + lane, l2 = f[k];
            if (l2 & 0x100u) {
                render_line(m, y, lat0[idx], lat1[idx], (int)(l2 & 0xFFu) - 1, screen + (size_t)env * PK_SCREEN + y * PK_COLS);
                lat2[idx] = l2 & ~0x100u;
                PK_FLUSH_STAT(1);
            }
        }
    }
    PK_FLUSH_STAT(0);
}
