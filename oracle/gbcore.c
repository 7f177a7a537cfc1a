/*
 * gbcore.c — CPU ORACLE for the pokegym_amd hot path. TEST INFRASTRUCTURE ONLY.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Restates PyBoy 1.x (pinned `pyboy<2.0.0`, reference setup.py:12; NOT vendored, NOT installed)
 * as driven by pokegym/pyboy_binding.py:71-91. Section comments name the PyBoy 1.x module whose
 * behaviour each block restates. Savestate v9 layout: SURVEY.md §5 (pinned on 264 reference files).
 * Parity of CPU trajectories vs PyBoy is UNPINNED (no PyBoy, no ROM, no recorded trajectories).
 */
#define _POSIX_C_SOURCE 199309L
#include "gbcore.h"
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define FRAME_CYCLES 70224u
#define INTR_VBLANK 0x01
#define INTR_LCDC 0x02
#define INTR_TIMER 0x04
#define INTR_SERIAL 0x08
#define INTR_HIGHTOLOW 0x10
#define FZ 0x80
#define FN 0x40
#define FH 0x20
#define FC 0x10

struct gb {
    /* cartridge (pyboy/core/cartridge) */
    const uint8_t* rom;
    uint32_t rom_banks;  /* power of two */
    uint8_t mbc;         /* 0 = ROM only, 3 = MBC3 */
    uint8_t rombank, rambank, ram_enabled, memorymodel;
    uint8_t sram[4 * 8192];
    /* cpu (pyboy/core/cpu.py) */
    uint8_t A, F, B, C, D, E;
    uint16_t HL, SP, PC;
    uint8_t ime, halted, stopped, IE, queued, IF;
    uint8_t crashed;
    /* lcd (pyboy/core/lcd.py) */
    uint8_t vram[8192], oam[160];
    uint8_t LCDC, BGP, OBP0, OBP1, STAT, LY, LYC, SCY, SCX, WY, WX;
    uint8_t lcd_cgb, lcd_ds;
    uint64_t clock, clock_target;
    uint8_t next_stat_mode, frame_done, render;
    /* renderer */
    uint8_t scan_params[GB_ROWS][5];
    uint8_t screen[GB_ROWS][GB_COLS]; /* shade 0..3 */
    int32_t ly_window;
    /* ram (pyboy/core/ram.py) */
    uint8_t wram[8192], fea0[96], io[76], hram[127], ff4c[52];
    /* timer (pyboy/core/timer.py) */
    uint32_t DIV, TIMA, TMA, TAC, DIV_counter, TIMA_counter;
    /* interaction (pyboy/core/interaction.py) */
    uint8_t directional, standard;
    /* header bytes 1..4 of the state file */
    uint8_t hdr[4];
    uint64_t instr_count, frame_count, iter_count;
    uint64_t cyc_total, cyc_halted, cyc_lcdoff;   /* workload intensity (gb_intensity) */
};

static const uint32_t TIMER_DIVIDERS[4] = {1024, 16, 64, 256};

/* ------------------------------------------------------------------ cartridge ------------- */
gb_t* gb_new(const uint8_t* rom, uint32_t rom_len) {
    if (!rom || rom_len < 0x8000 || (rom_len & 0x3FFF)) return NULL;
    uint32_t banks = rom_len / 0x4000;
    if (banks & (banks - 1)) return NULL;
    uint8_t type = rom[0x147];
    uint8_t mbc;
    if (type == 0x00) mbc = 0;
    else if (type >= 0x0F && type <= 0x13) mbc = 3;
    else return NULL;
    gb_t* gb = (gb_t*)calloc(1, sizeof(gb_t));
    if (!gb) return NULL;
    gb->rom = rom;
    gb->rom_banks = banks;
    gb->mbc = mbc;
    gb_power_on(gb);
    return gb;
}

void gb_free(gb_t* gb) { free(gb); }

gb_t* gb_clone(const gb_t* gb) {
    gb_t* g = (gb_t*)malloc(sizeof(gb_t));
    if (g) memcpy(g, gb, sizeof(gb_t));
    return g;
}

static inline uint8_t rom_read(const gb_t* gb, uint16_t a) {
    if (a < 0x4000) return gb->rom[a];
    uint32_t bank = gb->rombank & (gb->rom_banks - 1);
    return gb->rom[bank * 0x4000u + (a - 0x4000u)];
}

static inline void mbc_write(gb_t* gb, uint16_t a, uint8_t v) {
    if (gb->mbc == 0) return;
    /* MBC3.setitem */
    if (a < 0x2000) {
        gb->ram_enabled = ((v & 0x0F) == 0x0A) ? 1 : 0;
    } else if (a < 0x4000) {
        v &= 0x7F;
        if (v == 0) v = 1;
        gb->rombank = v;
    } else if (a < 0x6000) {
        gb->rambank = v;
    } else {
        /* RTC latch: no RTC on this cartridge -> ignored (pokered issue #155) */
    }
}

/* ------------------------------------------------------------------ lcd / renderer ---------- */
static inline uint8_t stat_set_mode(gb_t* gb, uint8_t mode) {
    if ((gb->STAT & 3) == mode) return 0;
    gb->STAT = (uint8_t)((gb->STAT & 0xFC) | mode);
    if (mode != 3 && (gb->STAT & (1u << (mode + 3)))) return INTR_LCDC;
    return 0;
}

static inline uint8_t stat_update_lyc(gb_t* gb) {
    if (gb->LYC == gb->LY) {
        gb->STAT |= 0x04;
        if (gb->STAT & 0x40) return INTR_LCDC;
    } else {
        gb->STAT &= 0xFB;
    }
    return 0;
}

static inline uint8_t tile_px(const uint8_t* vram, uint32_t tile_addr, uint32_t row, uint32_t col) {
    uint8_t lo = vram[tile_addr + row * 2], hi = vram[tile_addr + row * 2 + 1];
    uint32_t sh = 7 - col;
    return (uint8_t)(((lo >> sh) & 1) | (((hi >> sh) & 1) << 1));
}

static inline uint32_t bg_tile_addr(uint8_t lcdc, uint8_t t) {
    if (lcdc & 0x10) return (uint32_t)t * 16;
    return 0x1000 + (uint32_t)((int32_t)(int8_t)t * 16); /* signed from 0x9000 */
}

/* renderer.scanline + scanline_sprites (DMG path) */
static void render_scanline(gb_t* gb, int y) {
    uint8_t lcdc = gb->LCDC;
    int bx = gb->SCX, by = gb->SCY, wx = (int)gb->WX - 7, wy = gb->WY;
    gb->scan_params[y][0] = gb->SCX;
    gb->scan_params[y][1] = gb->SCY;
    gb->scan_params[y][2] = gb->WX;
    gb->scan_params[y][3] = gb->WY;
    gb->scan_params[y][4] = (lcdc >> 4) & 1;
    uint32_t bgmap = (lcdc & 0x08) ? 0x1C00 : 0x1800;
    uint32_t wmap = (lcdc & 0x40) ? 0x1C00 : 0x1800;
    int win = (lcdc & 0x20) && wy <= y;
    if (win && wx < GB_COLS) gb->ly_window += 1;
    uint8_t* out = gb->screen[y];
    for (int x = 0; x < GB_COLS; x++) {
        uint8_t ci;
        if (win && wx <= x) {
            int lw = gb->ly_window;
            uint8_t t = gb->vram[wmap + ((lw / 8) * 32 % 0x400) + ((x - wx) / 8) % 32];
            ci = tile_px(gb->vram, bg_tile_addr(lcdc, t), (uint32_t)(lw % 8), (uint32_t)((x - wx) % 8));
            out[x] = (gb->BGP >> (2 * ci)) & 3;
        } else if (lcdc & 0x01) {
            uint8_t t = gb->vram[bgmap + (((y + by) / 8) * 32 % 0x400) + ((x + bx) / 8) % 32];
            ci = tile_px(gb->vram, bg_tile_addr(lcdc, t), (uint32_t)((y + by) % 8), (uint32_t)((x + bx) % 8));
            out[x] = (gb->BGP >> (2 * ci)) & 3;
        } else {
            out[x] = 0; /* background disabled -> white */
        }
    }
    if (y == GB_ROWS - 1) gb->ly_window = -1;

    if (!(lcdc & 0x02)) return;
    int h = (lcdc & 0x04) ? 16 : 8;
    int sel[10], ns = 0;
    for (int n = 0; n < 40 && ns < 10; n++) {
        int sy = (int)gb->oam[n * 4] - 16;
        if (sy <= y && y < sy + h) sel[ns++] = n;
    }
    /* DMG priority: smaller X first, ties by OAM index (stable insertion sort) */
    for (int i = 1; i < ns; i++) {
        int k = sel[i], j = i - 1;
        while (j >= 0 && gb->oam[sel[j] * 4 + 1] > gb->oam[k * 4 + 1]) { sel[j + 1] = sel[j]; j--; }
        sel[j + 1] = k;
    }
    uint8_t bg0 = gb->BGP & 3;
    for (int i = ns - 1; i >= 0; i--) {
        int n = sel[i];
        int sy = (int)gb->oam[n * 4] - 16, sx = (int)gb->oam[n * 4 + 1] - 8;
        uint8_t ti = gb->oam[n * 4 + 2], at = gb->oam[n * 4 + 3];
        if (h == 16) ti &= 0xFE;
        int dy = y - sy;
        int yy = (at & 0x40) ? (h - dy - 1) : dy;
        uint8_t pal = (at & 0x10) ? gb->OBP1 : gb->OBP0;
        for (int dx = 0; dx < 8; dx++) {
            int xx = (at & 0x20) ? 7 - dx : dx;
            uint8_t c = tile_px(gb->vram, (uint32_t)ti * 16 + (uint32_t)(yy / 8) * 16, (uint32_t)(yy % 8), (uint32_t)xx);
            int px = sx + dx;
            if (px >= 0 && px < GB_COLS && c != 0) {
                uint8_t shade = (pal >> (2 * c)) & 3;
                if (at & 0x80) {
                    if (out[px] == bg0) out[px] = shade;
                } else {
                    out[px] = shade;
                }
            }
        }
    }
}

/* lcd.set_lcdc */
static void lcd_set_lcdc(gb_t* gb, uint8_t v) {
    gb->LCDC = v;
    if (!(v & 0x80)) {
        gb->clock = 0;
        gb->clock_target = FRAME_CYCLES;
        (void)stat_set_mode(gb, 0);
        gb->next_stat_mode = 2;
        gb->LY = 0;
    }
}

/* lcd.tick */
static uint8_t lcd_tick(gb_t* gb, uint32_t cycles) {
    uint8_t intr = 0;
    gb->clock += cycles;
    if (gb->LCDC & 0x80) {
        if (gb->clock >= gb->clock_target) {
            intr |= stat_set_mode(gb, gb->next_stat_mode);
            uint8_t mode = gb->STAT & 3;
            if (mode == 2) {
                if (gb->LY == 153) {
                    gb->LY = 0;
                    gb->clock %= FRAME_CYCLES;
                    gb->clock_target %= FRAME_CYCLES;
                } else {
                    gb->LY += 1;
                }
                gb->clock_target += 80;
                gb->next_stat_mode = 3;
                intr |= stat_update_lyc(gb);
            } else if (mode == 3) {
                gb->clock_target += 170;
                gb->next_stat_mode = 0;
            } else if (mode == 0) {
                gb->clock_target += 206;
                if (gb->render && gb->LY < GB_ROWS) render_scanline(gb, gb->LY);
                gb->next_stat_mode = (gb->LY < 143) ? 2 : 1;
            } else { /* mode 1 */
                gb->clock_target += 456;
                gb->next_stat_mode = 1;
                gb->LY += 1;
                intr |= stat_update_lyc(gb);
                if (gb->LY == 144) {
                    intr |= INTR_VBLANK;
                    gb->frame_done = 1;
                }
                if (gb->LY == 153) gb->next_stat_mode = 2;
            }
        }
    } else {
        if (gb->clock >= FRAME_CYCLES) {
            gb->frame_done = 1;
            gb->clock %= FRAME_CYCLES;
            if (gb->render) memset(gb->screen, 0, sizeof(gb->screen));
        }
    }
    return intr;
}

static inline int64_t lcd_cycles_to_interrupt(const gb_t* gb) { return (int64_t)gb->clock_target - (int64_t)gb->clock; }

/* ------------------------------------------------------------------ timer ------------------- */
static uint8_t timer_tick(gb_t* gb, uint32_t cycles) {
    gb->DIV_counter += cycles;
    gb->DIV += gb->DIV_counter >> 8;
    gb->DIV_counter &= 0xFF;
    gb->DIV &= 0xFF;
    if (!(gb->TAC & 4)) return 0;
    gb->TIMA_counter += cycles;
    uint32_t div = TIMER_DIVIDERS[gb->TAC & 3];
    if (gb->TIMA_counter >= div) {
        uint32_t mul = gb->TIMA_counter / div;
        gb->TIMA_counter -= div * mul;
        gb->TIMA += mul;
        if (gb->TIMA > 0xFF) {
            gb->TIMA -= 0x100;
            gb->TIMA += gb->TMA;
            gb->TIMA &= 0xFF;
            return 1;
        }
    }
    return 0;
}

static inline int64_t timer_cycles_to_interrupt(const gb_t* gb) {
    if (!(gb->TAC & 4)) return 1 << 16;
    int64_t div = TIMER_DIVIDERS[gb->TAC & 3];
    return (int64_t)(0x100 - (int64_t)gb->TIMA) * div - (int64_t)gb->TIMA_counter;
}

/* ------------------------------------------------------------------ joypad ------------------ */
static uint8_t joy_pull(const gb_t* gb, uint8_t v) {
    uint8_t p14 = (v >> 4) & 1, p15 = (v >> 5) & 1;
    uint8_t r = (uint8_t)(v | 0xCF);
    if (p14 && p15) {
    } else if (!p14 && !p15) {
    } else if (!p14) {
        r &= gb->directional;
    } else {
        r &= gb->standard;
    }
    return r;
}

void gb_button(gb_t* gb, int button, int pressed) {
    uint8_t od = gb->directional, os = gb->standard;
    uint8_t* reg = (button < 4) ? &gb->directional : &gb->standard;
    uint8_t bit = (uint8_t)(1u << (button & 3));
    if (pressed) *reg &= (uint8_t)~bit;
    else *reg |= bit;
    if (((od ^ gb->directional) & od) || ((os ^ gb->standard) & os)) gb->IF |= INTR_HIGHTOLOW;
}

/* ------------------------------------------------------------------ bus --------------------- */
static void bus_write(gb_t* gb, uint16_t a, uint8_t v);

static uint8_t bus_read(gb_t* gb, uint16_t a) {
    if (a < 0x8000) return rom_read(gb, a);
    if (a < 0xA000) return gb->vram[a - 0x8000];
    if (a < 0xC000) {
        if (gb->mbc == 0) return 0xFF;
        if (!gb->ram_enabled) return 0xFF;
        return gb->sram[(gb->rambank & 3) * 8192u + (a - 0xA000u)];
    }
    if (a < 0xE000) return gb->wram[a - 0xC000];
    if (a < 0xFE00) return gb->wram[a - 0xE000];
    if (a < 0xFEA0) return gb->oam[a - 0xFE00];
    if (a < 0xFF00) return gb->fea0[a - 0xFEA0];
    if (a < 0xFF4C) {
        switch (a) {
            case 0xFF04: return (uint8_t)gb->DIV;
            case 0xFF05: return (uint8_t)gb->TIMA;
            case 0xFF06: return (uint8_t)gb->TMA;
            case 0xFF07: return (uint8_t)gb->TAC;
            case 0xFF0F: return gb->IF;
            case 0xFF40: return gb->LCDC;
            case 0xFF41: return gb->STAT;
            case 0xFF42: return gb->SCY;
            case 0xFF43: return gb->SCX;
            case 0xFF44: return gb->LY;
            case 0xFF45: return gb->LYC;
            case 0xFF46: return 0;
            case 0xFF47: return gb->BGP;
            case 0xFF48: return gb->OBP0;
            case 0xFF49: return gb->OBP1;
            case 0xFF4A: return gb->WY;
            case 0xFF4B: return gb->WX;
            default:
                if (a >= 0xFF10 && a < 0xFF40) return 0; /* sound not emulated */
                return gb->io[a - 0xFF00];
        }
    }
    if (a < 0xFF80) return gb->ff4c[a - 0xFF4C];
    if (a < 0xFFFF) return gb->hram[a - 0xFF80];
    return gb->IE;
}

static void bus_write(gb_t* gb, uint16_t a, uint8_t v) {
    if (a < 0x8000) { mbc_write(gb, a, v); return; }
    if (a < 0xA000) { gb->vram[a - 0x8000] = v; return; }
    if (a < 0xC000) {
        if (gb->mbc != 0 && gb->ram_enabled) gb->sram[(gb->rambank & 3) * 8192u + (a - 0xA000u)] = v;
        return;
    }
    if (a < 0xE000) { gb->wram[a - 0xC000] = v; return; }
    if (a < 0xFE00) { gb->wram[a - 0xE000] = v; return; }
    if (a < 0xFEA0) { gb->oam[a - 0xFE00] = v; return; }
    if (a < 0xFF00) { gb->fea0[a - 0xFEA0] = v; return; }
    if (a < 0xFF4C) {
        switch (a) {
            case 0xFF00: gb->io[0] = joy_pull(gb, v); return;
            case 0xFF04: gb->DIV = 0; gb->DIV_counter = 0; gb->TIMA_counter = 0; return;
            case 0xFF05: gb->TIMA = v; return;
            case 0xFF06: gb->TMA = v; return;
            case 0xFF07: gb->TAC = v & 7; return;
            case 0xFF0F: gb->IF = v; return;
            case 0xFF40: lcd_set_lcdc(gb, v); return;
            case 0xFF41: gb->STAT = (uint8_t)((gb->STAT & 0x87) | (v & 0x78)); return;
            case 0xFF42: gb->SCY = v; return;
            case 0xFF43: gb->SCX = v; return;
            case 0xFF44: return;
            case 0xFF45: gb->LYC = v; return;
            case 0xFF46: {
                uint16_t src = (uint16_t)(v << 8);
                for (int n = 0; n < 0xA0; n++) bus_write(gb, (uint16_t)(0xFE00 + n), bus_read(gb, (uint16_t)(src + n)));
                return;
            }
            case 0xFF47: gb->BGP = v; return;
            case 0xFF48: gb->OBP0 = v; return;
            case 0xFF49: gb->OBP1 = v; return;
            case 0xFF4A: gb->WY = v; return;
            case 0xFF4B: gb->WX = v; return;
            default:
                if (a >= 0xFF10 && a < 0xFF40) return; /* sound not emulated */
                gb->io[a - 0xFF00] = v;
                return;
        }
    }
    if (a < 0xFF80) { gb->ff4c[a - 0xFF4C] = v; return; }
    if (a < 0xFFFF) { gb->hram[a - 0xFF80] = v; return; }
    gb->IE = v;
}

uint8_t gb_read(gb_t* gb, uint16_t a) { return bus_read(gb, a); }
void gb_write(gb_t* gb, uint16_t a, uint8_t v) { bus_write(gb, a, v); }

/* ------------------------------------------------------------------ cpu --------------------- */
#define RD(a) bus_read(gb, (uint16_t)(a))
#define WR(a, v) bus_write(gb, (uint16_t)(a), (uint8_t)(v))

static inline uint8_t get_r8(gb_t* gb, int r) {
    switch (r) {
        case 0: return gb->B;
        case 1: return gb->C;
        case 2: return gb->D;
        case 3: return gb->E;
        case 4: return (uint8_t)(gb->HL >> 8);
        case 5: return (uint8_t)gb->HL;
        case 6: return RD(gb->HL);
        default: return gb->A;
    }
}

static inline void set_r8(gb_t* gb, int r, uint8_t v) {
    switch (r) {
        case 0: gb->B = v; break;
        case 1: gb->C = v; break;
        case 2: gb->D = v; break;
        case 3: gb->E = v; break;
        case 4: gb->HL = (uint16_t)((gb->HL & 0x00FF) | (v << 8)); break;
        case 5: gb->HL = (uint16_t)((gb->HL & 0xFF00) | v); break;
        case 6: WR(gb->HL, v); break;
        default: gb->A = v; break;
    }
}

static inline uint16_t get_rr(gb_t* gb, int p) { /* BC DE HL SP */
    switch (p) {
        case 0: return (uint16_t)((gb->B << 8) | gb->C);
        case 1: return (uint16_t)((gb->D << 8) | gb->E);
        case 2: return gb->HL;
        default: return gb->SP;
    }
}

static inline void set_rr(gb_t* gb, int p, uint16_t v) {
    switch (p) {
        case 0: gb->B = (uint8_t)(v >> 8); gb->C = (uint8_t)v; break;
        case 1: gb->D = (uint8_t)(v >> 8); gb->E = (uint8_t)v; break;
        case 2: gb->HL = v; break;
        default: gb->SP = v; break;
    }
}

static inline void alu(gb_t* gb, int op, uint8_t v) {
    uint32_t a = gb->A, c = (gb->F & FC) ? 1 : 0, r;
    uint8_t f;
    switch (op) {
        case 0: /* ADD */
            r = a + v;
            f = (uint8_t)((((r & 0xFF) == 0) ? FZ : 0) | ((((a & 0xF) + (v & 0xF)) > 0xF) ? FH : 0) | ((r > 0xFF) ? FC : 0));
            gb->A = (uint8_t)r; gb->F = f; break;
        case 1: /* ADC */
            r = a + v + c;
            f = (uint8_t)((((r & 0xFF) == 0) ? FZ : 0) | ((((a & 0xF) + (v & 0xF) + c) > 0xF) ? FH : 0) | ((r > 0xFF) ? FC : 0));
            gb->A = (uint8_t)r; gb->F = f; break;
        case 2: /* SUB */
        case 7: /* CP */
            r = a - v;
            f = (uint8_t)(FN | (((r & 0xFF) == 0) ? FZ : 0) | (((a & 0xF) < (v & 0xF)) ? FH : 0) | ((a < v) ? FC : 0));
            if (op == 2) gb->A = (uint8_t)r;
            gb->F = f; break;
        case 3: /* SBC */
            r = a - v - c;
            f = (uint8_t)(FN | (((r & 0xFF) == 0) ? FZ : 0) | (((int)(a & 0xF) - (int)(v & 0xF) - (int)c < 0) ? FH : 0) |
                          (((int)a - (int)v - (int)c < 0) ? FC : 0));
            gb->A = (uint8_t)r; gb->F = f; break;
        case 4: /* AND */
            gb->A = (uint8_t)(a & v); gb->F = (uint8_t)((gb->A == 0 ? FZ : 0) | FH); break;
        case 5: /* XOR */
            gb->A = (uint8_t)(a ^ v); gb->F = (uint8_t)(gb->A == 0 ? FZ : 0); break;
        default: /* OR */
            gb->A = (uint8_t)(a | v); gb->F = (uint8_t)(gb->A == 0 ? FZ : 0); break;
    }
}

static inline int cond(gb_t* gb, int cc) {
    switch (cc) {
        case 0: return !(gb->F & FZ);
        case 1: return (gb->F & FZ) != 0;
        case 2: return !(gb->F & FC);
        default: return (gb->F & FC) != 0;
    }
}

static inline void push16(gb_t* gb, uint16_t v) {
    WR((uint16_t)(gb->SP - 1), v >> 8);
    WR((uint16_t)(gb->SP - 2), v & 0xFF);
    gb->SP = (uint16_t)(gb->SP - 2);
}

static inline uint16_t pop16(gb_t* gb) {
    uint8_t lo = RD(gb->SP);
    uint8_t hi = RD((uint16_t)(gb->SP + 1));
    gb->SP = (uint16_t)(gb->SP + 2);
    return (uint16_t)((hi << 8) | lo);
}

static uint32_t exec_cb(gb_t* gb, uint8_t op) {
    int r = op & 7, y = (op >> 3) & 7;
    uint8_t v = get_r8(gb, r), res = v, f = gb->F;
    uint32_t cyc = (r == 6) ? 16 : 8;
    switch (op >> 6) {
        case 0: {
            uint8_t c = 0;
            switch (y) {
                case 0: c = v >> 7; res = (uint8_t)((v << 1) | c); break;                    /* RLC */
                case 1: c = v & 1; res = (uint8_t)((v >> 1) | (c << 7)); break;              /* RRC */
                case 2: c = v >> 7; res = (uint8_t)((v << 1) | ((f & FC) ? 1 : 0)); break;   /* RL */
                case 3: c = v & 1; res = (uint8_t)((v >> 1) | ((f & FC) ? 0x80 : 0)); break; /* RR */
                case 4: c = v >> 7; res = (uint8_t)(v << 1); break;                          /* SLA */
                case 5: c = v & 1; res = (uint8_t)((v >> 1) | (v & 0x80)); break;            /* SRA */
                case 6: c = 0; res = (uint8_t)((v >> 4) | (v << 4)); break;                  /* SWAP */
                default: c = v & 1; res = (uint8_t)(v >> 1); break;                          /* SRL */
            }
            gb->F = (uint8_t)((res == 0 ? FZ : 0) | (c ? FC : 0));
            set_r8(gb, r, res);
            break;
        }
        case 1: /* BIT */
            gb->F = (uint8_t)((f & FC) | FH | ((v & (1u << y)) ? 0 : FZ));
            if (r == 6) cyc = 12;
            break;
        case 2: set_r8(gb, r, (uint8_t)(v & ~(1u << y))); break; /* RES */
        default: set_r8(gb, r, (uint8_t)(v | (1u << y))); break; /* SET */
    }
    gb->PC = (uint16_t)(gb->PC + 2);
    return cyc;
}

/* optional instruction trace (debugging/tests): pc, BC|DE<<16, HL|A<<16|F<<24, SP, opcode */
static uint32_t* g_trace = NULL;
static uint64_t g_trace_cap = 0, g_trace_n = 0;
void gb_trace_enable(uint32_t* buf, uint64_t cap) { g_trace = buf; g_trace_cap = cap; g_trace_n = 0; }
uint64_t gb_trace_count(void) { return g_trace_n; }

/* cpu.fetch_and_execute + opcodes.py; returns T-cycles */
static uint32_t cpu_execute(gb_t* gb) {
    uint16_t pc = gb->PC;
    uint8_t op = RD(pc);
    gb->instr_count++;
    if (g_trace && g_trace_n < g_trace_cap) {
        uint32_t* r = g_trace + g_trace_n * 6;
        r[0] = pc;
        r[1] = (uint32_t)(gb->C | (gb->B << 8) | (gb->E << 16) | ((uint32_t)gb->D << 24));
        r[2] = (uint32_t)((gb->HL & 0xFF) | ((gb->HL >> 8) << 8) | (gb->A << 16) | ((uint32_t)gb->F << 24));
        r[3] = gb->SP;
        r[4] = op;
        r[5] = 0;
        g_trace_n++;
    }
    if (op == 0xCB) return exec_cb(gb, RD((uint16_t)(pc + 1)));
    uint8_t n8 = 0;
    uint16_t n16 = 0;
    /* immediates are fetched only for instructions that have them (PyBoy reads them eagerly) */
    switch (op) {
        /* ---- 0x40-0x7F: LD r,r' / HALT ---- */
        default:
            if (op >= 0x40 && op < 0x80) {
                if (op == 0x76) { gb->halted = 1; return 4; } /* HALT: PC not advanced */
                int d = (op >> 3) & 7, s = op & 7;
                set_r8(gb, d, get_r8(gb, s));
                gb->PC = (uint16_t)(pc + 1);
                return (d == 6 || s == 6) ? 8 : 4;
            }
            if (op >= 0x80 && op < 0xC0) {
                int s = op & 7;
                alu(gb, (op >> 3) & 7, get_r8(gb, s));
                gb->PC = (uint16_t)(pc + 1);
                return s == 6 ? 8 : 4;
            }
            /* illegal opcode: freeze the CPU (documented extension; PyBoy raises) */
            gb->crashed = 1;
            gb->halted = 1;
            return 4;
        case 0x00: gb->PC = (uint16_t)(pc + 1); return 4;
        case 0x01: case 0x11: case 0x21: case 0x31:
            n16 = (uint16_t)(RD(pc + 1) | (RD(pc + 2) << 8));
            set_rr(gb, op >> 4, n16); gb->PC = (uint16_t)(pc + 3); return 12;
        case 0x02: WR(get_rr(gb, 0), gb->A); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x12: WR(get_rr(gb, 1), gb->A); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x22: WR(gb->HL, gb->A); gb->HL = (uint16_t)(gb->HL + 1); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x32: WR(gb->HL, gb->A); gb->HL = (uint16_t)(gb->HL - 1); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x0A: gb->A = RD(get_rr(gb, 0)); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x1A: gb->A = RD(get_rr(gb, 1)); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x2A: gb->A = RD(gb->HL); gb->HL = (uint16_t)(gb->HL + 1); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x3A: gb->A = RD(gb->HL); gb->HL = (uint16_t)(gb->HL - 1); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x03: case 0x13: case 0x23: case 0x33:
            set_rr(gb, op >> 4, (uint16_t)(get_rr(gb, op >> 4) + 1)); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x0B: case 0x1B: case 0x2B: case 0x3B:
            set_rr(gb, op >> 4, (uint16_t)(get_rr(gb, op >> 4) - 1)); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0x04: case 0x0C: case 0x14: case 0x1C: case 0x24: case 0x2C: case 0x34: case 0x3C: {
            int r = (op >> 3) & 7;
            uint8_t v = get_r8(gb, r), res = (uint8_t)(v + 1);
            gb->F = (uint8_t)((gb->F & FC) | (res == 0 ? FZ : 0) | (((v & 0xF) == 0xF) ? FH : 0));
            set_r8(gb, r, res); gb->PC = (uint16_t)(pc + 1); return r == 6 ? 12 : 4;
        }
        case 0x05: case 0x0D: case 0x15: case 0x1D: case 0x25: case 0x2D: case 0x35: case 0x3D: {
            int r = (op >> 3) & 7;
            uint8_t v = get_r8(gb, r), res = (uint8_t)(v - 1);
            gb->F = (uint8_t)((gb->F & FC) | FN | (res == 0 ? FZ : 0) | (((v & 0xF) == 0) ? FH : 0));
            set_r8(gb, r, res); gb->PC = (uint16_t)(pc + 1); return r == 6 ? 12 : 4;
        }
        case 0x06: case 0x0E: case 0x16: case 0x1E: case 0x26: case 0x2E: case 0x36: case 0x3E: {
            int r = (op >> 3) & 7;
            n8 = RD(pc + 1);
            set_r8(gb, r, n8); gb->PC = (uint16_t)(pc + 2); return r == 6 ? 12 : 8;
        }
        case 0x07: { uint8_t c = gb->A >> 7; gb->A = (uint8_t)((gb->A << 1) | c); gb->F = c ? FC : 0; gb->PC = (uint16_t)(pc + 1); return 4; }
        case 0x0F: { uint8_t c = gb->A & 1; gb->A = (uint8_t)((gb->A >> 1) | (c << 7)); gb->F = c ? FC : 0; gb->PC = (uint16_t)(pc + 1); return 4; }
        case 0x17: { uint8_t c = gb->A >> 7; gb->A = (uint8_t)((gb->A << 1) | ((gb->F & FC) ? 1 : 0)); gb->F = c ? FC : 0; gb->PC = (uint16_t)(pc + 1); return 4; }
        case 0x1F: { uint8_t c = gb->A & 1; gb->A = (uint8_t)((gb->A >> 1) | ((gb->F & FC) ? 0x80 : 0)); gb->F = c ? FC : 0; gb->PC = (uint16_t)(pc + 1); return 4; }
        case 0x08:
            n16 = (uint16_t)(RD(pc + 1) | (RD(pc + 2) << 8));
            WR(n16, gb->SP & 0xFF); WR((uint16_t)(n16 + 1), gb->SP >> 8); gb->PC = (uint16_t)(pc + 3); return 20;
        case 0x09: case 0x19: case 0x29: case 0x39: {
            uint32_t hl = gb->HL, v = get_rr(gb, op >> 4), r = hl + v;
            gb->F = (uint8_t)((gb->F & FZ) | ((((hl & 0xFFF) + (v & 0xFFF)) > 0xFFF) ? FH : 0) | ((r > 0xFFFF) ? FC : 0));
            gb->HL = (uint16_t)r; gb->PC = (uint16_t)(pc + 1); return 8;
        }
        case 0x10: gb->PC = (uint16_t)(pc + 2); return 4; /* STOP (DMG): treated as a 2-byte no-op */
        case 0x18: n8 = RD(pc + 1); gb->PC = (uint16_t)(pc + 2 + (int8_t)n8); return 12;
        case 0x20: case 0x28: case 0x30: case 0x38:
            n8 = RD(pc + 1);
            if (cond(gb, (op >> 3) & 3)) { gb->PC = (uint16_t)(pc + 2 + (int8_t)n8); return 12; }
            gb->PC = (uint16_t)(pc + 2); return 8;
        case 0x27: { /* DAA */
            int t = gb->A, corr = 0;
            if (gb->F & FH) corr |= 0x06;
            if (gb->F & FC) corr |= 0x60;
            if (gb->F & FN) t -= corr;
            else {
                if ((t & 0x0F) > 0x09) corr |= 0x06;
                if (t > 0x99) corr |= 0x60;
                t += corr;
            }
            gb->F = (uint8_t)((gb->F & FN) | (((t & 0xFF) == 0) ? FZ : 0) | ((corr & 0x60) ? FC : 0));
            gb->A = (uint8_t)t; gb->PC = (uint16_t)(pc + 1); return 4;
        }
        case 0x2F: gb->A = (uint8_t)~gb->A; gb->F = (uint8_t)(gb->F | FN | FH); gb->PC = (uint16_t)(pc + 1); return 4;
        case 0x37: gb->F = (uint8_t)((gb->F & FZ) | FC); gb->PC = (uint16_t)(pc + 1); return 4;
        case 0x3F: gb->F = (uint8_t)((gb->F & FZ) | ((gb->F & FC) ? 0 : FC)); gb->PC = (uint16_t)(pc + 1); return 4;
        /* ---- 0xC0-0xFF ---- */
        case 0xC0: case 0xC8: case 0xD0: case 0xD8:
            if (cond(gb, (op >> 3) & 3)) { gb->PC = pop16(gb); return 20; }
            gb->PC = (uint16_t)(pc + 1); return 8;
        case 0xC9: gb->PC = pop16(gb); return 16;
        case 0xD9: gb->PC = pop16(gb); gb->ime = 1; return 16;
        case 0xC1: case 0xD1: case 0xE1: {
            uint16_t v = pop16(gb); set_rr(gb, (op >> 4) & 3, v); gb->PC = (uint16_t)(pc + 1); return 12;
        }
        case 0xF1: { uint16_t v = pop16(gb); gb->A = (uint8_t)(v >> 8); gb->F = (uint8_t)(v & 0xF0); gb->PC = (uint16_t)(pc + 1); return 12; }
        case 0xC5: case 0xD5: case 0xE5:
            push16(gb, get_rr(gb, (op >> 4) & 3)); gb->PC = (uint16_t)(pc + 1); return 16;
        case 0xF5: push16(gb, (uint16_t)((gb->A << 8) | gb->F)); gb->PC = (uint16_t)(pc + 1); return 16;
        case 0xC2: case 0xCA: case 0xD2: case 0xDA:
            n16 = (uint16_t)(RD(pc + 1) | (RD(pc + 2) << 8));
            if (cond(gb, (op >> 3) & 3)) { gb->PC = n16; return 16; }
            gb->PC = (uint16_t)(pc + 3); return 12;
        case 0xC3: n16 = (uint16_t)(RD(pc + 1) | (RD(pc + 2) << 8)); gb->PC = n16; return 16;
        case 0xE9: gb->PC = gb->HL; return 4;
        case 0xC4: case 0xCC: case 0xD4: case 0xDC:
            n16 = (uint16_t)(RD(pc + 1) | (RD(pc + 2) << 8));
            if (cond(gb, (op >> 3) & 3)) { push16(gb, (uint16_t)(pc + 3)); gb->PC = n16; return 24; }
            gb->PC = (uint16_t)(pc + 3); return 12;
        case 0xCD:
            n16 = (uint16_t)(RD(pc + 1) | (RD(pc + 2) << 8));
            push16(gb, (uint16_t)(pc + 3)); gb->PC = n16; return 24;
        case 0xC7: case 0xCF: case 0xD7: case 0xDF: case 0xE7: case 0xEF: case 0xF7: case 0xFF:
            push16(gb, (uint16_t)(pc + 1)); gb->PC = (uint16_t)(op & 0x38); return 16;
        case 0xC6: case 0xCE: case 0xD6: case 0xDE: case 0xE6: case 0xEE: case 0xF6: case 0xFE:
            n8 = RD(pc + 1); alu(gb, (op >> 3) & 7, n8); gb->PC = (uint16_t)(pc + 2); return 8;
        case 0xE0: n8 = RD(pc + 1); WR(0xFF00 + n8, gb->A); gb->PC = (uint16_t)(pc + 2); return 12;
        case 0xF0: n8 = RD(pc + 1); gb->A = RD(0xFF00 + n8); gb->PC = (uint16_t)(pc + 2); return 12;
        case 0xE2: WR(0xFF00 + gb->C, gb->A); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0xF2: gb->A = RD(0xFF00 + gb->C); gb->PC = (uint16_t)(pc + 1); return 8;
        case 0xEA: n16 = (uint16_t)(RD(pc + 1) | (RD(pc + 2) << 8)); WR(n16, gb->A); gb->PC = (uint16_t)(pc + 3); return 16;
        case 0xFA: n16 = (uint16_t)(RD(pc + 1) | (RD(pc + 2) << 8)); gb->A = RD(n16); gb->PC = (uint16_t)(pc + 3); return 16;
        case 0xE8: case 0xF8: {
            n8 = RD(pc + 1);
            uint32_t sp = gb->SP;
            uint16_t r = (uint16_t)(sp + (int8_t)n8);
            gb->F = (uint8_t)(((((sp & 0xF) + (n8 & 0xF)) > 0xF) ? FH : 0) | ((((sp & 0xFF) + n8) > 0xFF) ? FC : 0));
            if (op == 0xE8) { gb->SP = r; gb->PC = (uint16_t)(pc + 2); return 16; }
            gb->HL = r; gb->PC = (uint16_t)(pc + 2); return 12;
        }
        case 0xF9: gb->SP = gb->HL; gb->PC = (uint16_t)(pc + 1); return 8;
        case 0xF3: gb->ime = 0; gb->PC = (uint16_t)(pc + 1); return 4;
        case 0xFB: gb->ime = 1; gb->PC = (uint16_t)(pc + 1); return 4;
    }
}

/* cpu.check_interrupts */
static int cpu_check_interrupts(gb_t* gb) {
    if (gb->queued) return 0;
    uint8_t pend = (uint8_t)(gb->IF & gb->IE & 0x1F);
    if (pend) {
        if (gb->halted) gb->PC = (uint16_t)(gb->PC + 1); /* escape HALT on return */
        if (gb->ime) {
            uint8_t flag;
            uint16_t vec;
            if (pend & INTR_VBLANK) { flag = INTR_VBLANK; vec = 0x40; }
            else if (pend & INTR_LCDC) { flag = INTR_LCDC; vec = 0x48; }
            else if (pend & INTR_TIMER) { flag = INTR_TIMER; vec = 0x50; }
            else if (pend & INTR_SERIAL) { flag = INTR_SERIAL; vec = 0x58; }
            else { flag = INTR_HIGHTOLOW; vec = 0x60; }
            gb->IF ^= flag;
            WR((uint16_t)(gb->SP - 1), gb->PC >> 8);
            WR((uint16_t)(gb->SP - 2), gb->PC & 0xFF);
            gb->SP = (uint16_t)(gb->SP - 2);
            gb->PC = vec;
            gb->ime = 0;
        }
        gb->queued = 1;
        return 1;
    }
    return 0;
}

/* cpu.tick */
static uint32_t cpu_tick(gb_t* gb) {
    if (gb->crashed) return 4;
    if (cpu_check_interrupts(gb)) {
        gb->halted = 0;
        return 0;
    }
    if (gb->halted && gb->queued) {
        gb->halted = 0;
        gb->PC = (uint16_t)(gb->PC + 1);
    } else if (gb->halted) {
        return 4;
    }
    uint32_t cyc = cpu_execute(gb);
    gb->queued = 0;
    return cyc;
}

/* ------------------------------------------------------------------ motherboard ------------- */
/* Frame watchdog (extension; PyBoy would spin forever): a program that keeps re-disabling the
 * LCD faster than once per frame resets lcd.clock and never reaches a frame boundary.  After
 * PK_FRAME_BUDGET units (cycles + 1 per tick) the frame is ended.  The HIP kernel does the same. */
#define PK_FRAME_BUDGET (16u * FRAME_CYCLES)

void gb_tick(gb_t* gb) {
    uint32_t budget = 0;
    do {
        uint64_t cycles = cpu_tick(gb);
        if (gb->halted) {
            /* HALT fast-forward: max(0, min(lcd, timer)) cycles */
            int64_t a = lcd_cycles_to_interrupt(gb), b = timer_cycles_to_interrupt(gb);
            int64_t m = a < b ? a : b;
            cycles = m < 0 ? 0 : (uint64_t)m;
        }
        if (timer_tick(gb, (uint32_t)cycles)) gb->IF |= INTR_TIMER;
        gb->IF |= lcd_tick(gb, (uint32_t)cycles);
        budget += (uint32_t)cycles + 1u;
        gb->iter_count++;
        gb->cyc_total += cycles;
        if (gb->halted) gb->cyc_halted += cycles;
        if (!(gb->LCDC & 0x80)) gb->cyc_lcdoff += cycles;
        if (budget > PK_FRAME_BUDGET) gb->frame_done = 1;
    } while (!gb->frame_done);
    gb->frame_done = 0;
    gb->frame_count++;
}

void gb_set_rendering(gb_t* gb, int on) { gb->render = on ? 1 : 0; }

int gb_action_button(int action) {
    static const int map[8] = {GB_BTN_DOWN, GB_BTN_LEFT, GB_BTN_RIGHT, GB_BTN_UP,
                               GB_BTN_A, GB_BTN_B, GB_BTN_START, GB_BTN_SELECT};
    if (action < 0 || action > 7) return -1;
    return map[action];
}

/* pyboy_binding.run_action_on_emulator (pyboy_binding.py:71-91) */
void gb_run_action(gb_t* gb, int action, int frame_skip, int release_frame) {
    int btn = gb_action_button(action);
    if (btn >= 0) gb_button(gb, btn, 1);
    gb_set_rendering(gb, 0);
    for (int i = 0; i < frame_skip; i++) {
        if (i == release_frame && btn >= 0) gb_button(gb, btn, 0);
        if (i == frame_skip - 1) gb_set_rendering(gb, 1);
        gb_tick(gb);
    }
}

/* ------------------------------------------------------------------ state ------------------- */
static inline uint64_t rd64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}
static inline void wr64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; i++) { p[i] = (uint8_t)v; v >>= 8; }
}

void gb_power_on(gb_t* gb) {
    const uint8_t* rom = gb->rom;
    uint32_t banks = gb->rom_banks;
    uint8_t mbc = gb->mbc;
    memset(gb, 0, sizeof(*gb));
    gb->rom = rom; gb->rom_banks = banks; gb->mbc = mbc;
    gb->rombank = 1;
    gb->A = 0x01; gb->F = 0xB0; gb->B = 0x00; gb->C = 0x13; gb->D = 0x00; gb->E = 0xD8;
    gb->HL = 0x014D; gb->SP = 0xFFFE; gb->PC = 0x0100;
    gb->LCDC = 0x91; gb->BGP = 0xFC; gb->OBP0 = 0xFF; gb->OBP1 = 0xFF;
    gb->STAT = 0x82; gb->LY = 0; gb->clock = 0; gb->clock_target = 80; gb->next_stat_mode = 3;
    gb->io[0] = 0xCF;
    gb->directional = 0x0F; gb->standard = 0x0F;
    gb->ly_window = -1;
    gb->DIV = 0xAB;
}

int gb_load_state(gb_t* gb, const uint8_t* s, uint32_t len) {
    if (len != GB_STATE_V9_SIZE || s[0] != 9) return -1;
    const uint8_t* rom = gb->rom;
    uint32_t banks = gb->rom_banks;
    uint8_t mbc = gb->mbc;
    memset(gb, 0, sizeof(*gb));
    gb->rom = rom; gb->rom_banks = banks; gb->mbc = mbc;
    memcpy(gb->hdr, s + 1, 4);
    gb->A = s[5]; gb->F = s[6]; gb->B = s[7]; gb->C = s[8]; gb->D = s[9]; gb->E = s[10];
    gb->HL = (uint16_t)(s[11] | (s[12] << 8));
    gb->SP = (uint16_t)(s[13] | (s[14] << 8));
    gb->PC = (uint16_t)(s[15] | (s[16] << 8));
    gb->ime = s[17]; gb->halted = s[18]; gb->stopped = s[19]; gb->IE = s[20]; gb->queued = s[21]; gb->IF = s[22];
    memcpy(gb->vram, s + 23, 8192);
    memcpy(gb->oam, s + 8215, 160);
    const uint8_t* r = s + 8375;
    gb->LCDC = r[0]; gb->BGP = r[1]; gb->OBP0 = r[2]; gb->OBP1 = r[3]; gb->STAT = r[4]; gb->LY = r[5];
    gb->LYC = r[6]; gb->SCY = r[7]; gb->SCX = r[8]; gb->WY = r[9]; gb->WX = r[10];
    gb->lcd_cgb = s[8386]; gb->lcd_ds = s[8387];
    gb->clock = rd64(s + 8388); gb->clock_target = rd64(s + 8396); gb->next_stat_mode = s[8404];
    memcpy(gb->scan_params, s + 8405, 720);
    const uint8_t* px = s + 9125;
    for (int i = 0; i < GB_ROWS * GB_COLS; i++) {
        uint8_t g = px[i * 4 + 1];
        ((uint8_t*)gb->screen)[i] = g == 0xFF ? 0 : g == 0x99 ? 1 : g == 0x55 ? 2 : 3;
    }
    memcpy(gb->wram, s + 101285, 8192);
    memcpy(gb->fea0, s + 109477, 96);
    memcpy(gb->io, s + 109573, 76);
    memcpy(gb->hram, s + 109649, 127);
    memcpy(gb->ff4c, s + 109776, 52);
    const uint8_t* t = s + 109828;
    gb->DIV = t[0]; gb->TIMA = t[1];
    gb->DIV_counter = (uint32_t)(t[2] | (t[3] << 8));
    gb->TIMA_counter = (uint32_t)(t[4] | (t[5] << 8));
    gb->TMA = t[6]; gb->TAC = t[7];
    const uint8_t* c = s + 109836;
    gb->rombank = c[0]; gb->rambank = c[1]; gb->ram_enabled = c[2]; gb->memorymodel = c[3];
    memcpy(gb->sram, s + 109842, 4 * 8192);
    gb->directional = 0x0F; gb->standard = 0x0F;
    gb->ly_window = -1;
    return 0;
}

static const uint8_t SHADE_RGB[4] = {0xFF, 0x99, 0x55, 0x00};

int gb_save_state(const gb_t* gb, uint8_t* s, uint32_t len) {
    if (len < GB_STATE_V9_SIZE) return -1;
    memset(s, 0, GB_STATE_V9_SIZE);
    s[0] = 9;
    memcpy(s + 1, gb->hdr, 4);
    s[5] = gb->A; s[6] = gb->F; s[7] = gb->B; s[8] = gb->C; s[9] = gb->D; s[10] = gb->E;
    s[11] = (uint8_t)gb->HL; s[12] = (uint8_t)(gb->HL >> 8);
    s[13] = (uint8_t)gb->SP; s[14] = (uint8_t)(gb->SP >> 8);
    s[15] = (uint8_t)gb->PC; s[16] = (uint8_t)(gb->PC >> 8);
    s[17] = gb->ime; s[18] = gb->halted; s[19] = gb->stopped; s[20] = gb->IE; s[21] = gb->queued; s[22] = gb->IF;
    memcpy(s + 23, gb->vram, 8192);
    memcpy(s + 8215, gb->oam, 160);
    uint8_t* r = s + 8375;
    r[0] = gb->LCDC; r[1] = gb->BGP; r[2] = gb->OBP0; r[3] = gb->OBP1; r[4] = gb->STAT; r[5] = gb->LY;
    r[6] = gb->LYC; r[7] = gb->SCY; r[8] = gb->SCX; r[9] = gb->WY; r[10] = gb->WX;
    s[8386] = gb->lcd_cgb; s[8387] = gb->lcd_ds;
    wr64(s + 8388, gb->clock); wr64(s + 8396, gb->clock_target); s[8404] = gb->next_stat_mode;
    memcpy(s + 8405, gb->scan_params, 720);
    uint8_t* px = s + 9125;
    for (int i = 0; i < GB_ROWS * GB_COLS; i++) {
        uint8_t sh = ((const uint8_t*)gb->screen)[i];
        px[i * 4 + 0] = sh == 0 ? 1 : 0;
        px[i * 4 + 1] = px[i * 4 + 2] = px[i * 4 + 3] = SHADE_RGB[sh];
    }
    memcpy(s + 101285, gb->wram, 8192);
    memcpy(s + 109477, gb->fea0, 96);
    memcpy(s + 109573, gb->io, 76);
    memcpy(s + 109649, gb->hram, 127);
    memcpy(s + 109776, gb->ff4c, 52);
    uint8_t* t = s + 109828;
    t[0] = (uint8_t)gb->DIV; t[1] = (uint8_t)gb->TIMA;
    t[2] = (uint8_t)gb->DIV_counter; t[3] = (uint8_t)(gb->DIV_counter >> 8);
    t[4] = (uint8_t)gb->TIMA_counter; t[5] = (uint8_t)(gb->TIMA_counter >> 8);
    t[6] = (uint8_t)gb->TMA; t[7] = (uint8_t)gb->TAC;
    uint8_t* c = s + 109836;
    c[0] = gb->rombank; c[1] = gb->rambank; c[2] = gb->ram_enabled; c[3] = gb->memorymodel;
    memcpy(s + 109842, gb->sram, 4 * 8192);
    return 0;
}

const uint8_t* gb_screen_shades(const gb_t* gb) { return (const uint8_t*)gb->screen; }
const uint8_t* gb_wram(const gb_t* gb) { return gb->wram; }
uint64_t gb_instr_count(const gb_t* gb) { return gb->instr_count; }
uint64_t gb_frame_count(const gb_t* gb) { return gb->frame_count; }
uint64_t gb_iter_count(const gb_t* gb) { return gb->iter_count; }
int gb_crashed(const gb_t* gb) { return gb->crashed; }

int gb_render_from_state(const uint8_t* state, uint32_t len, uint8_t* out) {
    /* needs only the state prefix: header, CPU, VRAM, OAM, LCD regs, per-line params */
    if (len < 9125 || state[0] != 9) return -1;
    gb_t* gb = (gb_t*)calloc(1, sizeof(gb_t));
    if (!gb) return -2;
    memcpy(gb->vram, state + 23, 8192);
    memcpy(gb->oam, state + 8215, 160);
    const uint8_t* r = state + 8375;
    gb->LCDC = r[0]; gb->BGP = r[1]; gb->OBP0 = r[2]; gb->OBP1 = r[3];
    gb->ly_window = -1;
    /* render each line with the latched per-line params (SCX,SCY,WX,WY) */
    for (int y = 0; y < GB_ROWS; y++) {
        gb->SCX = state[8405 + y * 5 + 0];
        gb->SCY = state[8405 + y * 5 + 1];
        gb->WX = state[8405 + y * 5 + 2];
        gb->WY = state[8405 + y * 5 + 3];
        render_scanline(gb, y);
    }
    memcpy(out, gb->screen, GB_ROWS * GB_COLS);
    free(gb);
    return 0;
}

int gb_batch_run(const uint8_t* rom, uint32_t rom_len, const uint8_t* state, uint32_t state_len,
                 uint32_t n, uint32_t steps, const uint8_t* actions, int render_last,
                 uint8_t* states_out, uint8_t* screens_out) {
    gb_t* tmpl = gb_new(rom, rom_len);
    if (!tmpl) return -1;
    if (state && gb_load_state(tmpl, state, state_len)) { gb_free(tmpl); return -2; }
    for (uint32_t e = 0; e < n; e++) {
        gb_t* gb = gb_clone(tmpl);
        for (uint32_t s = 0; s < steps; s++) {
            gb_run_action(gb, actions[(size_t)s * n + e], 24, 8);
        }
        (void)render_last;
        if (states_out) gb_save_state(gb, states_out + (size_t)e * GB_STATE_V9_SIZE, GB_STATE_V9_SIZE);
        if (screens_out) memcpy(screens_out + (size_t)e * GB_ROWS * GB_COLS, gb->screen, GB_ROWS * GB_COLS);
        gb_free(gb);
    }
    gb_free(tmpl);
    return 0;
}

/* The benchmark action stream: action (0-7) of env e at env-step t, the top 3 bits of a splitmix64
   finalizer over (seed, e, t).  (A plain xor of the three products, used before, gave each env a
   structured action sequence that never walked through a door in 16,896 env-steps; numpy random
   actions warp in ~0.1 % of them, as the GPU bench's Philox actions do.) */
static inline int bench_action(uint32_t seed, uint32_t e, uint32_t t) {
    uint64_t z = (((uint64_t)seed << 42) ^ ((uint64_t)e << 21) ^ (uint64_t)t) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (int)(z >> 61);
}

/* CPU baseline ("port"): n envs, `warmup` untimed env-steps, then `steps` timed env-steps with
 * uniform random actions 0..7 from a counter-based hash of (seed, env, t).  Single thread.
 * Returns elapsed seconds of the timed part; *instr_out = emulated instructions in it. */
double gb_bench(const uint8_t* rom, uint32_t rom_len, const uint8_t* state, uint32_t state_len,
                uint32_t n, uint32_t warmup, uint32_t steps, uint32_t seed, uint64_t* instr_out) {
    gb_t* tmpl = gb_new(rom, rom_len);
    if (!tmpl) return -1.0;
    if (state && gb_load_state(tmpl, state, state_len)) { gb_free(tmpl); return -2.0; }
    gb_t** envs = (gb_t**)calloc(n, sizeof(gb_t*));
    for (uint32_t e = 0; e < n; e++) envs[e] = gb_clone(tmpl);
    #define ACT(e, t) bench_action(seed, (e), (t))
    for (uint32_t t = 0; t < warmup; t++)
        for (uint32_t e = 0; e < n; e++) gb_run_action(envs[e], ACT(e, t), 24, 8);
    uint64_t i0 = 0;
    for (uint32_t e = 0; e < n; e++) i0 += envs[e]->instr_count;
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (uint32_t t = warmup; t < warmup + steps; t++)
        for (uint32_t e = 0; e < n; e++) gb_run_action(envs[e], ACT(e, t), 24, 8);
    clock_gettime(CLOCK_MONOTONIC, &b);
    uint64_t i1 = 0;
    for (uint32_t e = 0; e < n; e++) { i1 += envs[e]->instr_count; gb_free(envs[e]); }
    #undef ACT
    free(envs);
    gb_free(tmpl);
    if (instr_out) *instr_out = i1 - i0;
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

/* Workload intensity of the bench's action stream (the same actions as gb_bench): out[0] emulated
 * instructions, [1] ticks, [2] cycles, [3] cycles spent halted (HALT fast-forward), [4] cycles with
 * the LCD off, [5] frames — summed over n envs x steps env-steps after warmup. */

int gb_intensity(const uint8_t* rom, uint32_t rom_len, const uint8_t* state, uint32_t state_len,
                 uint32_t n, uint32_t warmup, uint32_t steps, uint32_t seed, uint64_t* out) {
    gb_t* tmpl = gb_new(rom, rom_len);
    if (!tmpl) return -1;
    if (state && gb_load_state(tmpl, state, state_len)) { gb_free(tmpl); return -2; }
    for (int k = 0; k < 6; k++) out[k] = 0;
    #define ACT(e, t) bench_action(seed, (e), (t))
    for (uint32_t e = 0; e < n; e++) {
        gb_t* g = gb_clone(tmpl);
        for (uint32_t t = 0; t < warmup; t++) gb_run_action(g, ACT(e, t), 24, 8);
        const uint64_t i0 = g->instr_count, k0 = g->iter_count, c0 = g->cyc_total, h0 = g->cyc_halted,
                       l0 = g->cyc_lcdoff, f0 = g->frame_count;
        for (uint32_t t = warmup; t < warmup + steps; t++) gb_run_action(g, ACT(e, t), 24, 8);
        out[0] += g->instr_count - i0; out[1] += g->iter_count - k0; out[2] += g->cyc_total - c0;
        out[3] += g->cyc_halted - h0; out[4] += g->cyc_lcdoff - l0; out[5] += g->frame_count - f0;
        gb_free(g);
    }
    #undef ACT
    gb_free(tmpl);
    return 0;
}
