// pk_capi.cpp — the C ABI (include/pokegym_amd.h) over the HIP kernels in pk_kernels.hip.
//
// Owns the per-GPU device state: lane-interleaved RAM images, SoA lane registers, per-line
// render latches, the persistent grey screen, the ROM and the decode table, plus a parsed copy
// of the template savestate used by pk_reset.  Savestate import/export restates the PyBoy v9
// layout pinned on the reference's 264 savestates (oracle/gbcore.c load/save).
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/pokegym_amd.h"
#include "pk_ucode.h"
#include "pk_layout.h"
#include "pk_reward.h"

hipError_t pk_launch_step(const PkStepArgs& a, hipStream_t s);
hipError_t pk_launch_step_small(const PkStepArgs& a, hipStream_t s);   // pk_step.hip built with PK_K1_SMALL
hipError_t pk_launch_render(const PkStepArgs& a, hipStream_t s);
hipError_t pk_launch_reset(const PkResetArgs& a, hipStream_t s);
hipError_t pk_launch_list(const uint8_t* mask, uint32_t env0, uint32_t env1, uint32_t* cnt, uint32_t* ids, hipStream_t s);
hipError_t pk_launch_render_latched(const PkStepArgs& a, hipStream_t s);
hipError_t pk_launch_gather_env(const uint8_t* mem, uint32_t env, uint32_t sh, uint8_t* out, hipStream_t s);
hipError_t pk_launch_gather_range(const uint8_t* mem, uint32_t env0, uint32_t count, uint32_t sh, uint8_t* out, hipStream_t s);
hipError_t pk_launch_scatter_env(uint8_t* mem, uint32_t env, uint32_t sh, const uint8_t* in, hipStream_t s);
hipError_t pk_launch_done(const uint32_t* time_reg, uint32_t n, uint32_t max_steps, uint8_t* term,
                          uint8_t* trunc, double* rew, hipStream_t s);
hipError_t pk_launch_reward(const PkRewardArgs& a, hipStream_t s);
hipError_t pk_launch_rreset_pre(const PkRewardArgs& a, hipStream_t s);
hipError_t pk_launch_rreset_post(const PkRewardArgs& a, hipStream_t s);
hipError_t pk_launch_obs(const PkRewardArgs& a, hipStream_t s);
hipError_t pk_launch_seen_rehash(const uint32_t* old_tab, uint32_t old_lg, uint32_t* new_tab, uint32_t new_lg,
                                 const uint32_t* rs, uint32_t n, uint32_t np, hipStream_t s);
hipError_t pk_launch_ram_copy(uint8_t* mem, uint8_t* dense, uint32_t n, uint32_t sh, uint32_t phys0, uint32_t len,
                              uint32_t to_dense, hipStream_t s);

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) return fail(-EIO, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// v9 savestate offsets
constexpr size_t S_VER = 0, S_HDR = 1, S_CPU = 5, S_VRAM = 23, S_OAM = 8215, S_LCDREG = 8375,
                 S_LCDX = 8386, S_CLOCK = 8388, S_TARGET = 8396, S_NEXTMODE = 8404,
                 S_SCAN = 8405, S_SCREEN = 9125, S_WRAM = 101285, S_FEA0 = 109477,
                 S_IO = 109573, S_HRAM = 109649, S_FF4C = 109776, S_TIMER = 109828,
                 S_MBC = 109836, S_SRAM = 109842, S_SIZE = 142610;

struct Template {
    uint32_t regs[PK_NREGS];
    std::vector<uint8_t> mem;       // PK_PHYS
    uint32_t lat[3 * PK_ROWS];
    std::vector<uint8_t> screen;    // 144*160 grey
    uint8_t hdr[4];
    uint8_t lcdx[2];
};

uint64_t rd64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}
void wr64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; i++) { p[i] = (uint8_t)v; v >>= 8; }
}

int parse_v9(const uint8_t* s, size_t len, Template& t) {
    if (len != S_SIZE || s[S_VER] != 9) return fail(-EINVAL, "not a PyBoy v9 savestate (len %zu)", len);
    uint64_t clock = rd64(s + S_CLOCK), target = rd64(s + S_TARGET);
    if (clock > 0xFFFFFFFFull || target > 0xFFFFFFFFull) return fail(-EINVAL, "LCD clock out of range");
    memset(t.regs, 0, sizeof t.regs);
    const uint8_t* c = s + S_CPU;  // A F B C D E HL SP PC ime halted stopped IE queued IF
    t.regs[PK_R_W0] = c[3] | (c[2] << 8) | (c[5] << 16) | ((uint32_t)c[4] << 24);
    t.regs[PK_R_W1] = c[6] | (c[7] << 8) | (c[0] << 16) | ((uint32_t)c[1] << 24);
    t.regs[PK_R_SP] = c[8] | (c[9] << 8);
    t.regs[PK_R_PC] = c[10] | (c[11] << 8);
    t.regs[PK_R_CPU] = (c[12] ? 1u : 0u) | (c[13] ? 2u : 0u) | (c[16] ? 4u : 0u) | (c[14] ? 16u : 0u) |
                       ((uint32_t)c[15] << 8) | ((uint32_t)c[17] << 16);
    t.regs[PK_R_CLOCK] = (uint32_t)clock;
    t.regs[PK_R_TARGET] = (uint32_t)target;
    const uint8_t* r = s + S_LCDREG;  // LCDC BGP OBP0 OBP1 STAT LY LYC SCY SCX WY WX
    t.regs[PK_R_LCD0] = r[0] | (r[4] << 8) | (r[5] << 16) | ((uint32_t)r[6] << 24);
    t.regs[PK_R_LCD1] = r[7] | (r[8] << 8) | (r[9] << 16) | ((uint32_t)r[10] << 24);
    t.regs[PK_R_LCD2] = r[1] | (r[2] << 8) | (r[3] << 16) | ((uint32_t)s[S_NEXTMODE] << 24);
    const uint8_t* tm = s + S_TIMER;  // DIV TIMA DIVc(le16) TIMAc(le16) TMA TAC
    t.regs[PK_R_TIM0] = tm[0] | (tm[1] << 8) | (tm[6] << 16) | ((uint32_t)tm[7] << 24);
    t.regs[PK_R_TIM1] = (tm[2] | (tm[3] << 8)) | ((uint32_t)(tm[4] | (tm[5] << 8)) << 16);
    const uint8_t* mb = s + S_MBC;
    t.regs[PK_R_MBC] = mb[0] | (mb[1] << 8) | (mb[2] << 16) | ((uint32_t)mb[3] << 24);
    t.regs[PK_R_MISC] = 0x0Fu | (0x0Fu << 8);  // no button held, ly_window = -1
    t.mem.assign(PK_PHYS, 0);
    memcpy(&t.mem[PK_P_VRAM], s + S_VRAM, 8192);
    memcpy(&t.mem[PK_P_WRAM], s + S_WRAM, 8192);
    memcpy(&t.mem[PK_P_OAM], s + S_OAM, 160);
    memcpy(&t.mem[PK_P_OAM + 0xA0], s + S_FEA0, 96);
    memcpy(&t.mem[PK_P_IO], s + S_IO, 76);
    memcpy(&t.mem[PK_P_IO + 0x4C], s + S_FF4C, 52);
    memcpy(&t.mem[PK_P_HRAM], s + S_HRAM, 127);
    memcpy(&t.mem[PK_P_SRAM], s + S_SRAM, 4 * 8192);
    t.screen.resize(PK_SCREEN);
    for (size_t i = 0; i < PK_SCREEN; i++) t.screen[i] = s[S_SCREEN + i * 4 + 1];
    for (uint32_t y = 0; y < PK_ROWS; y++) {
        const uint8_t* p = s + S_SCAN + y * 5;  // SCX SCY WX WY tiledata_select
        uint32_t lcdc = (r[0] & ~0x10u) | ((p[4] & 1u) << 4);
        t.lat[y] = lcdc | (p[0] << 8) | (p[1] << 16) | ((uint32_t)p[2] << 24);
        t.lat[PK_ROWS + y] = p[3] | (r[1] << 8) | (r[2] << 16) | ((uint32_t)r[3] << 24);
        t.lat[2 * PK_ROWS + y] = 0;
    }
    memcpy(t.hdr, s + S_HDR, 4);
    t.lcdx[0] = s[S_LCDX];
    t.lcdx[1] = s[S_LCDX + 1];
    return 0;
}

void power_on(Template& t) {
    // our own post-boot DMG state (PyBoy would execute its bundled boot ROM instead);
    // identical to oracle/gbcore.c gb_power_on
    memset(t.regs, 0, sizeof t.regs);
    t.regs[PK_R_W0] = 0x13 | (0x00 << 8) | (0xD8 << 16) | (0x00u << 24);
    t.regs[PK_R_W1] = 0x4D | (0x01 << 8) | (0x01 << 16) | (0xB0u << 24);
    t.regs[PK_R_SP] = 0xFFFE;
    t.regs[PK_R_PC] = 0x0100;
    t.regs[PK_R_CPU] = 0;
    t.regs[PK_R_CLOCK] = 0;
    t.regs[PK_R_TARGET] = 80;
    t.regs[PK_R_LCD0] = 0x91 | (0x82 << 8);
    t.regs[PK_R_LCD1] = 0;
    t.regs[PK_R_LCD2] = 0xFC | (0xFF << 8) | (0xFF << 16) | (3u << 24);
    t.regs[PK_R_TIM0] = 0xAB;
    t.regs[PK_R_TIM1] = 0;
    t.regs[PK_R_MBC] = 1;
    t.regs[PK_R_MISC] = 0x0Fu | (0x0Fu << 8);
    t.mem.assign(PK_PHYS, 0);
    t.mem[PK_P_IO] = 0xCF;
    t.screen.assign(PK_SCREEN, 0xFF);  // shade 0
    for (uint32_t y = 0; y < PK_ROWS; y++) {
        t.lat[y] = 0;
        t.lat[PK_ROWS + y] = 0;
        t.lat[2 * PK_ROWS + y] = 0;
    }
    memset(t.hdr, 0, 4);
    t.lcdx[0] = t.lcdx[1] = 0;
}

uint8_t grey_to_flag(uint8_t g) { return g == 0xFF ? 1 : 0; }

void export_v9(const Template& tp, const uint32_t* regs, const uint8_t* mem, const uint32_t* lat,
               const uint8_t* screen, uint8_t* s) {
    memset(s, 0, S_SIZE);
    s[S_VER] = 9;
    memcpy(s + S_HDR, tp.hdr, 4);
    uint32_t w0 = regs[PK_R_W0], w1 = regs[PK_R_W1];
    uint8_t* c = s + S_CPU;
    c[0] = (w1 >> 16) & 0xFF; c[1] = (w1 >> 24) & 0xFF;  // A F
    c[2] = (w0 >> 8) & 0xFF; c[3] = w0 & 0xFF;            // B C
    c[4] = (w0 >> 24) & 0xFF; c[5] = (w0 >> 16) & 0xFF;   // D E
    c[6] = w1 & 0xFF; c[7] = (w1 >> 8) & 0xFF;            // HL
    c[8] = regs[PK_R_SP] & 0xFF; c[9] = (regs[PK_R_SP] >> 8) & 0xFF;
    c[10] = regs[PK_R_PC] & 0xFF; c[11] = (regs[PK_R_PC] >> 8) & 0xFF;
    uint32_t cpu = regs[PK_R_CPU];
    c[12] = cpu & 1; c[13] = (cpu >> 1) & 1; c[14] = (cpu >> 4) & 1;
    c[15] = (cpu >> 8) & 0xFF; c[16] = (cpu >> 2) & 1; c[17] = (cpu >> 16) & 0xFF;
    memcpy(s + S_VRAM, mem + PK_P_VRAM, 8192);
    memcpy(s + S_OAM, mem + PK_P_OAM, 160);
    uint32_t l0 = regs[PK_R_LCD0], l1 = regs[PK_R_LCD1], l2 = regs[PK_R_LCD2];
    uint8_t* r = s + S_LCDREG;
    r[0] = l0 & 0xFF; r[1] = l2 & 0xFF; r[2] = (l2 >> 8) & 0xFF; r[3] = (l2 >> 16) & 0xFF;
    r[4] = (l0 >> 8) & 0xFF; r[5] = (l0 >> 16) & 0xFF; r[6] = (l0 >> 24) & 0xFF;
    r[7] = l1 & 0xFF; r[8] = (l1 >> 8) & 0xFF; r[9] = (l1 >> 16) & 0xFF; r[10] = (l1 >> 24) & 0xFF;
    s[S_LCDX] = tp.lcdx[0];
    s[S_LCDX + 1] = tp.lcdx[1];
    wr64(s + S_CLOCK, regs[PK_R_CLOCK]);
    wr64(s + S_TARGET, regs[PK_R_TARGET]);
    s[S_NEXTMODE] = (l2 >> 24) & 0xFF;
    for (uint32_t y = 0; y < PK_ROWS; y++) {
        uint32_t a = lat[y], b = lat[PK_ROWS + y];
        uint8_t* p = s + S_SCAN + y * 5;
        p[0] = (a >> 8) & 0xFF; p[1] = (a >> 16) & 0xFF; p[2] = (a >> 24) & 0xFF; p[3] = b & 0xFF;
        p[4] = (a >> 4) & 1;
    }
    for (size_t i = 0; i < PK_SCREEN; i++) {
        uint8_t g = screen[i];
        s[S_SCREEN + i * 4 + 0] = grey_to_flag(g);
        s[S_SCREEN + i * 4 + 1] = s[S_SCREEN + i * 4 + 2] = s[S_SCREEN + i * 4 + 3] = g;
    }
    memcpy(s + S_WRAM, mem + PK_P_WRAM, 8192);
    memcpy(s + S_FEA0, mem + PK_P_OAM + 0xA0, 96);
    memcpy(s + S_IO, mem + PK_P_IO, 76);
    memcpy(s + S_HRAM, mem + PK_P_HRAM, 127);   // 0xFF80-0xFFFE: never phys 0x41FF (PK_P_UNUSED, K1's dummy store)
    memcpy(s + S_FF4C, mem + PK_P_IO + 0x4C, 52);
    uint32_t t0 = regs[PK_R_TIM0], t1 = regs[PK_R_TIM1];
    uint8_t* tm = s + S_TIMER;
    tm[0] = t0 & 0xFF; tm[1] = (t0 >> 8) & 0xFF;
    tm[2] = t1 & 0xFF; tm[3] = (t1 >> 8) & 0xFF; tm[4] = (t1 >> 16) & 0xFF; tm[5] = (t1 >> 24) & 0xFF;
    tm[6] = (t0 >> 16) & 0xFF; tm[7] = (t0 >> 24) & 0xFF;
    uint32_t mbc = regs[PK_R_MBC];
    uint8_t* m = s + S_MBC;
    m[0] = mbc & 0xFF; m[1] = (mbc >> 8) & 0xFF; m[2] = (mbc >> 16) & 0xFF; m[3] = (mbc >> 24) & 0xFF;
    memcpy(s + S_SRAM, mem + PK_P_SRAM, 4 * 8192);
}

}  // namespace

struct pk_handle {
    int device = 0;
    uint32_t n = 0, npad = 0, ngroups = 0;
    uint32_t wave_lanes = 0;   // envs per wave in K1: 0 = by launch size (k1_wave_lanes), else PK_WAVE_LANES
    uint32_t simds = 1024;     // SIMDs of the device (4 per CU)
    uint32_t k1_block = 0;     // K1 workgroup size override (PK_K1_BLOCK), 0 = by geometry
    uint32_t ilv_sh = 6;       // RAM image interleave 1 << ilv_sh (pk_layout.h pk_img_off): K1's envs per wave
    int k1_prio = -1;          // K1 wave-priority variant override (PK_K1_PRIO 0/1), -1 = by shape
    uint32_t frames = 24, release = 8, flags = 0, max_steps = 20480;
    uint32_t mbc = 3, bank_mask = 0;
    uint8_t* mem = nullptr;
    uint32_t* regs = nullptr;
    uint32_t* lat = nullptr;
    uint8_t* screen = nullptr;
    uint8_t* rom = nullptr;
    uint32_t* ucode = nullptr;  // microcode table (pk_ucode.h)
    uint8_t* t_mem = nullptr;
    uint32_t* t_regs = nullptr;
    uint32_t* t_lat = nullptr;
    uint8_t* t_screen = nullptr;
    uint8_t* scratch = nullptr;  // PK_PHYS staging for one env
    int8_t* bank_slot = nullptr;  // [128] LDS slot per ROM bank (-1 = global)
    uint8_t* slot_bank = nullptr; // [PK_LDS_SLOTS]
    uint32_t nslots = 1;
    // the small-LDS K1 (pk_layout.h): its own slot tables (PK_SMALL_LDS_SLOTS banks)
    int8_t* bank_slot_s = nullptr;
    uint8_t* slot_bank_s = nullptr;
    uint32_t nslots_s = 1;
    int k1_small = -1;         // PK_K1_SMALL: -1 = for concurrent sub-batch ranges (<= 32 envs per wave), 0 never, 1 always
    size_t lat_stride = 0;
    Template tmpl;
    // reward stack (PK_F_REWARD), see pk_reward.h
    uint32_t* rs = nullptr;
    double* rsd = nullptr;
    uint32_t* seen = nullptr;
    uint32_t* mask = nullptr;
    uint32_t* cutc = nullptr;
    uint8_t* obs = nullptr;
    uint8_t* reload = nullptr;
    // reset lists (pk_list_kernel): [0] reload count, [1] obs count, then npad reload ids, npad obs ids
    uint32_t* lists = nullptr;
    unsigned long long* dbg = nullptr;  // K1 phase-cycle counters of a -DPK_STAMP build
    double* info = nullptr;       // [PK_INFO_NFIELDS][npad]
    uint8_t* info_flag = nullptr; // [npad]
    int32_t* heat = nullptr;      // [npad][444 * 436] (PK_F_HEATMAP)
    uint32_t* info_bits = nullptr; // [PK_INFO_BITS_WORDS][npad]
    uint32_t cap_log2 = 0;
    double reward_scale = 4.0;
    // profiling: 4 events per profiled step (start, after K1, after K2, after K4+K3)
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
};

static int prof_event(pk_handle* h, hipStream_t s) {
    if (h->ev_used == h->ev_pool.size()) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        h->ev_pool.push_back(e);
    }
    HIPCHK(hipEventRecord(h->ev_pool[h->ev_used++], s));
    return 0;
}

extern "C" {

static int template_reset(pk_handle* h, const uint8_t* mask, uint32_t env0, uint32_t env1, void* stream);

const char* pk_last_error(void) { return g_err.c_str(); }
int pk_abi_version(void) { return PK_ABI_VERSION; }
uint8_t* pk_screen_ptr(pk_handle* h) { return h ? h->screen : nullptr; }
uint8_t* pk_obs_ptr(pk_handle* h) { return h ? h->obs : nullptr; }
const uint32_t* pk_error_ptr(pk_handle* h) { return (h && h->rs) ? h->rs + (size_t)RS_ERR * h->npad : nullptr; }
const double* pk_info_ptr(pk_handle* h) { return h ? h->info : nullptr; }
const uint8_t* pk_info_flag_ptr(pk_handle* h) { return h ? h->info_flag : nullptr; }
int32_t* pk_heatmap_ptr(pk_handle* h) { return h ? h->heat : nullptr; }
const uint32_t* pk_info_bits_ptr(pk_handle* h) { return h ? h->info_bits : nullptr; }
uint32_t pk_num_envs(const pk_handle* h) { return h ? h->n : 0; }
uint32_t pk_info_stride(const pk_handle* h) { return h ? h->npad : 0; }

void pk_destroy(pk_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    for (hipEvent_t e : h->ev_pool) (void)hipEventDestroy(e);
    void* ptrs[] = {h->mem, h->regs, h->lat, h->screen, h->rom, h->ucode, h->bank_slot, h->slot_bank, h->t_mem, h->t_regs,
                    h->t_lat, h->t_screen, h->scratch, h->rs, h->rsd, h->seen, h->mask, h->cutc, h->obs, h->reload,
                    h->lists, h->dbg, h->info, h->info_flag, h->heat, h->info_bits, h->bank_slot_s, h->slot_bank_s};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete h;
}

static uint32_t k1_wave_lanes(const struct pk_handle* h, uint32_t count);

int pk_create(const pk_config* cfg, pk_handle** out) {
    if (!cfg || !out) return fail(-EINVAL, "null argument");
    *out = nullptr;
    if (cfg->n_envs == 0) return fail(-EINVAL, "n_envs must be > 0");
    if (!cfg->rom || cfg->rom_len < 0x8000 || (cfg->rom_len & 0x3FFF))
        return fail(-EINVAL, "ROM must be a multiple of 16 KiB and >= 32 KiB");
    uint32_t banks = (uint32_t)(cfg->rom_len / 0x4000);
    if (banks & (banks - 1)) return fail(-EINVAL, "ROM bank count must be a power of two");
    uint8_t type = cfg->rom[0x147];
    uint32_t mbc;
    if (type == 0x00) mbc = 0;
    else if (type >= 0x0F && type <= 0x13) mbc = 3;
    else return fail(-ENOTSUP, "cartridge type 0x%02x not supported (ROM-only and MBC3 are)", type);
    // frame_skip 0 = no emulation (reward-stack replay tests drive RAM through pk_set_ram)
    if (cfg->frame_skip > 1024) return fail(-EINVAL, "bad frame_skip");

    pk_handle* h = new pk_handle();
    h->device = cfg->device;
    h->n = cfg->n_envs;
    h->npad = (cfg->n_envs + PK_LANES - 1) / PK_LANES * PK_LANES;
    h->ngroups = h->npad / PK_LANES;
    {
        // K1 wave shape: chosen per launch from the launch's env count (k1_wave_lanes);
        // PK_WAVE_LANES (a power of two <= 64) fixes it.
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cfg->device) != hipSuccess || ncu <= 0) ncu = 256;
        h->simds = 4u * (uint32_t)ncu;
        h->wave_lanes = 0;
        if (const char* wl = getenv("PK_WAVE_LANES")) {
            int v = atoi(wl);
            if (v < 1 || v > 64 || (v & (v - 1))) { delete h; return fail(-EINVAL, "PK_WAVE_LANES must be a power of two <= 64"); }
            h->wave_lanes = (uint32_t)v;
        }
        // K1 workgroup size override (parity tests run the benchmarked 512-thread shape at small n):
        // a multiple of 64 whose envs fit the 512-env HRAM mirror of a workgroup
        if (const char* bl = getenv("PK_K1_BLOCK")) {
            int v = atoi(bl);
            if (v < 64 || v > 512 || (v % 64) || (uint32_t)(v / 64) * (h->wave_lanes ? h->wave_lanes : 32u) > 512u) {
                delete h;
                return fail(-EINVAL, "PK_K1_BLOCK must be a multiple of 64 in [64, 512] with (block/64)*wave_lanes <= 512");
            }
            h->k1_block = (uint32_t)v;
        }
        if (const char* pr = getenv("PK_K1_PRIO")) h->k1_prio = atoi(pr) ? 1 : 0;
        if (const char* sm = getenv("PK_K1_SMALL")) h->k1_small = atoi(sm) ? 1 : 0;
        // image interleave = K1's envs per wave for this handle (no 64-byte line shared by two
        // waves; a wave's lanes share one sub-block base).  PK_ILV overrides it with any power of
        // two <= 64: narrower than the wave puts one wave's envs in several sub-blocks (K1 reaches
        // them through its per-lane offset), wider shares a sub-block between waves
        uint32_t ilv = k1_wave_lanes(h, h->n);
        if (const char* iv = getenv("PK_ILV")) {
            int v = atoi(iv);
            if (v < 1 || v > 64 || (v & (v - 1))) {
                delete h;
                return fail(-EINVAL, "PK_ILV must be a power of two <= 64");
            }
            ilv = (uint32_t)v;
        }
        h->ilv_sh = (uint32_t)__builtin_ctz(ilv);
    }
    h->frames = cfg->frame_skip;
    h->release = cfg->release_frame;
    h->flags = cfg->flags;
    h->max_steps = cfg->max_episode_steps ? cfg->max_episode_steps : 20480;
    h->reward_scale = cfg->reward_scale != 0.0 ? cfg->reward_scale : 4.0;
    // seen-coordinate set: one entry per step at most, load factor <= 3/4
    h->cap_log2 = 10;
    while ((1ull << h->cap_log2) * 3 < ((uint64_t)h->max_steps + 2) * 4) h->cap_log2++;
    h->mbc = mbc;
    h->bank_mask = banks - 1;
    h->lat_stride = (size_t)h->ngroups * PK_ROWS * PK_LANES;
    int rc;
    if (cfg->state) {
        if ((rc = parse_v9(cfg->state, cfg->state_len, h->tmpl))) { delete h; return rc; }
    } else {
        power_on(h->tmpl);
    }
#define ALLOC(ptr, bytes)                                                                  \
    do {                                                                                   \
        hipError_t e_ = hipMalloc((void**)&(ptr), (bytes));                                \
        if (e_ != hipSuccess) {                                                            \
            pk_destroy(h);                                                                 \
            return fail(-ENOMEM, "hipMalloc(%zu): %s", (size_t)(bytes), hipGetErrorString(e_)); \
        }                                                                                  \
    } while (0)
    if (hipSetDevice(h->device) != hipSuccess) { delete h; return fail(-ENODEV, "hipSetDevice(%d) failed", cfg->device); }
    ALLOC(h->mem, (size_t)h->ngroups * PK_GROUP_STRIDE);
    ALLOC(h->regs, (size_t)PK_NREGS * h->npad * 4);
    ALLOC(h->lat, 3 * h->lat_stride * 4);
    ALLOC(h->screen, (size_t)h->npad * PK_SCREEN);
    ALLOC(h->rom, cfg->rom_len + 16);
    ALLOC(h->ucode, PK_UC_WORDS * 4);
    ALLOC(h->bank_slot, 128);
    ALLOC(h->slot_bank, PK_LDS_SLOTS);
    ALLOC(h->bank_slot_s, 128);
    ALLOC(h->slot_bank_s, PK_SMALL_LDS_SLOTS);
    ALLOC(h->t_mem, PK_PHYS);
    ALLOC(h->t_regs, PK_NREGS * 4);
    ALLOC(h->t_lat, 3 * PK_ROWS * 4);
    ALLOC(h->t_screen, PK_SCREEN);
    ALLOC(h->scratch, PK_PHYS + PK_NREGS * 4 + 3 * PK_ROWS * 4 + PK_SCREEN);
    ALLOC(h->lists, (2 * (size_t)h->ngroups + 2 * (size_t)h->npad) * 4);
#if defined(PK_STAMP) || defined(PK_WAVETIME)
    ALLOC(h->dbg, PK_DBG_WORDS * 8);
    (void)hipMemset(h->dbg, 0, PK_DBG_WORDS * 8);
#endif
    if (h->flags & PK_F_REWARD) {
        ALLOC(h->rs, (size_t)RS_NFIELDS * h->npad * 4);
        ALLOC(h->rsd, (size_t)RSD_NFIELDS * h->npad * 8);
        ALLOC(h->seen, (size_t)h->npad * (1ull << h->cap_log2) * 4);
        ALLOC(h->mask, (size_t)h->npad * PK_MASK_WORDS * 4);
        ALLOC(h->cutc, (size_t)h->npad * PK_CUTC_CAP * 4);
        ALLOC(h->obs, (size_t)h->npad * PK_OBS_BYTES);
        ALLOC(h->reload, h->npad);
        ALLOC(h->info, (size_t)PK_INFO_NFIELDS * h->npad * 8);
        ALLOC(h->info_flag, h->npad);
        ALLOC(h->info_bits, (size_t)PK_INFO_BITS_WORDS * h->npad * 4);
        if (h->flags & PK_F_HEATMAP) ALLOC(h->heat, (size_t)h->npad * PK_HEAT_ROWS * PK_HEAT_COLS * 4);
    }
#undef ALLOC
    std::vector<uint32_t> uc(PK_UC_WORDS);
    pk_build_ucode(uc.data());
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipMemset(h->rom + cfg->rom_len, 0xFF, 16);
    if (e == hipSuccess) e = hipMemcpy(h->rom, cfg->rom, cfg->rom_len, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->ucode, uc.data(), uc.size() * 4, hipMemcpyHostToDevice);
    {
        // ROM banks staged in LDS by the step kernel: bank 0, then the switchable banks that hold
        // code or data, in bank order (a bank of one repeated byte — an unused bank of the
        // cartridge — only after those), so a small slot budget is not spent on an empty bank.
        // PK_STAGE_BANKS=b1,b2,... puts those banks first (experiments); PK_LDS_SLOTS=1..6 caps the count.
        const uint32_t nb = banks < 128u ? banks : 128u;   // MBC3: 7-bit bank number
        std::vector<uint32_t> order;
        std::vector<bool> used(nb, false);
        used[0] = true;
        order.push_back(0);
        if (const char* ev = getenv("PK_STAGE_BANKS")) {
            for (const char* q = ev; *q;) {
                char* end = nullptr;
                const unsigned long b = strtoul(q, &end, 10);
                if (end == q) break;
                if (b < nb && !used[b]) { used[b] = true; order.push_back((uint32_t)b); }
                q = *end ? end + 1 : end;
            }
        }
        for (int pass = 0; pass < 2; pass++)
            for (uint32_t b = 1; b < nb; b++) {
                if (used[b]) continue;
                const uint8_t* bp = cfg->rom + (size_t)b * 0x4000u;
                bool blank = true;
                for (uint32_t i = 1; i < 0x4000u && blank; i++) blank = bp[i] == bp[0];
                if (blank == (pass == 1)) { used[b] = true; order.push_back(b); }
            }
        uint32_t want = PK_LDS_SLOTS;
        if (const char* ev = getenv("PK_LDS_SLOTS")) want = (uint32_t)atoi(ev);
        if (want < 1) want = 1;
        if (want > PK_LDS_SLOTS) want = PK_LDS_SLOTS;
        if (want > nb) want = nb;
        int8_t bs[128];
        uint8_t sb[PK_LDS_SLOTS] = {0};
        memset(bs, -1, sizeof bs);
        for (uint32_t k = 0; k < want; k++) { sb[k] = (uint8_t)order[k]; bs[order[k]] = (int8_t)k; }
        h->nslots = want;
        if (e == hipSuccess) e = hipMemcpy(h->bank_slot, bs, sizeof bs, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(h->slot_bank, sb, sizeof sb, hipMemcpyHostToDevice);
        // the small-LDS kernel stages the first PK_SMALL_LDS_SLOTS of the same banks
        h->nslots_s = want < PK_SMALL_LDS_SLOTS ? want : PK_SMALL_LDS_SLOTS;
        for (uint32_t k = h->nslots_s; k < want; k++) bs[order[k]] = -1;
        if (e == hipSuccess) e = hipMemcpy(h->bank_slot_s, bs, sizeof bs, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(h->slot_bank_s, sb, PK_SMALL_LDS_SLOTS, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipMemcpy(h->t_mem, h->tmpl.mem.data(), PK_PHYS, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->t_regs, h->tmpl.regs, sizeof h->tmpl.regs, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->t_lat, h->tmpl.lat, sizeof h->tmpl.lat, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->t_screen, h->tmpl.screen.data(), PK_SCREEN, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(h->regs, 0, (size_t)PK_NREGS * h->npad * 4);
    if (e == hipSuccess) e = hipMemset(h->lat, 0, 3 * h->lat_stride * 4);
    if (h->flags & PK_F_REWARD) {
        // nothing has been reset yet (reset_count 0); update_heat_map's last_map = -1 (:462)
        if (e == hipSuccess) e = hipMemset(h->rs, 0, (size_t)RS_NFIELDS * h->npad * 4);
        if (e == hipSuccess) e = hipMemset(h->rs + (size_t)RS_HEAT_LAST * h->npad, 0xFF, (size_t)h->npad * 4);
        if (e == hipSuccess) e = hipMemset(h->rs + (size_t)RS_MASK_MAP * h->npad, 0xFF, (size_t)h->npad * 4);
        if (e == hipSuccess) e = hipMemset(h->rsd, 0, (size_t)RSD_NFIELDS * h->npad * 8);
        if (e == hipSuccess) e = hipMemset(h->seen, 0, (size_t)h->npad * (1ull << h->cap_log2) * 4);
        if (e == hipSuccess) e = hipMemset(h->mask, 0, (size_t)h->npad * PK_MASK_WORDS * 4);
        if (e == hipSuccess) e = hipMemset(h->obs, 0, (size_t)h->npad * PK_OBS_BYTES);
        if (e == hipSuccess) e = hipMemset(h->info, 0, (size_t)PK_INFO_NFIELDS * h->npad * 8);
        if (e == hipSuccess) e = hipMemset(h->info_flag, 0, h->npad);
        if (e == hipSuccess) e = hipMemset(h->info_bits, 0, (size_t)PK_INFO_BITS_WORDS * h->npad * 4);
        if (e == hipSuccess && h->heat) e = hipMemset(h->heat, 0, (size_t)h->npad * PK_HEAT_ROWS * PK_HEAT_COLS * 4);
    }
    if (e != hipSuccess) {
        pk_destroy(h);
        return fail(-EIO, "device upload failed: %s", hipGetErrorString(e));
    }
    if ((rc = template_reset(h, nullptr, 0, h->n, nullptr))) { pk_destroy(h); return rc; }
    if (hipDeviceSynchronize() != hipSuccess) { pk_destroy(h); return fail(-EIO, "initial reset failed"); }
    *out = h;
    return 0;
}

static PkRewardArgs reward_args(pk_handle* h, uint32_t env0, uint32_t env1) {
    PkRewardArgs r;
    memset(&r, 0, sizeof r);
    r.mem = h->mem; r.regs = h->regs; r.rs = h->rs; r.rsd = h->rsd; r.seen = h->seen; r.mask = h->mask;
    r.cutc = h->cutc; r.reload = h->reload; r.screen = h->screen; r.obs = h->obs;
    r.info = h->info; r.info_flag = h->info_flag; r.heat = h->heat; r.info_bits = h->info_bits;
    r.reward_scale = h->reward_scale; r.n = h->n; r.npad = h->npad; r.cap_log2 = h->cap_log2;
    r.max_steps = h->max_steps; r.reload_always = (h->flags & PK_F_RELOAD_ON_RESET) ? 1 : 0;
    r.env0 = env0; r.env1 = env1; r.ilv_sh = h->ilv_sh;
    return r;
}

// reset lists of an env range (env0 % 64 == 0): counters [2 * (env0 / 64)] (reload) and [+1] (obs),
// ids from env0 in the reload and obs id arrays — disjoint ranges (sub-batches on their own
// streams) never share a counter or an id slot
static uint32_t* list_cnt(pk_handle* h, uint32_t env0, int which) { return h->lists + 2u * (env0 / PK_LANES) + which; }
static uint32_t* list_ids(pk_handle* h, uint32_t env0, int which) {
    return h->lists + 2u * h->ngroups + (size_t)which * h->npad + env0;
}

// reload the template state (regs, RAM image, latches, screen) into the masked envs of [env0, env1):
// the envs are listed on the device first, so the reset costs in proportion to the envs it touches
static int template_reset(pk_handle* h, const uint8_t* mask, uint32_t env0, uint32_t env1, void* stream) {
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(list_cnt(h, env0, 0), 0, 4, s));
    HIPCHK(pk_launch_list(mask, env0, env1, list_cnt(h, env0, 0), list_ids(h, env0, 0), s));
    PkResetArgs a;
    a.mem = h->mem; a.regs = h->regs; a.lat = h->lat; a.screen = h->screen;
    a.tmpl_mem = h->t_mem; a.tmpl_regs = h->t_regs; a.tmpl_lat = h->t_lat; a.tmpl_screen = h->t_screen;
    a.cnt = list_cnt(h, env0, 0); a.ids = list_ids(h, env0, 0); a.n = h->n; a.npad = h->npad;
    a.lat_stride = (uint32_t)h->lat_stride; a.env0 = env0; a.env1 = env1; a.ilv_sh = h->ilv_sh;
    HIPCHK(pk_launch_reset(a, s));
    return 0;
}

static int check_range(pk_handle* h, uint32_t env0, uint32_t count) {
    if (!h) return fail(-EINVAL, "null handle");
    if (count == 0 || env0 % PK_LANES || (uint64_t)env0 + count > h->n)
        return fail(-EINVAL, "env range [%u, +%u): the start must be a multiple of 64 and the end <= n = %u", env0, count, h->n);
    return 0;
}

int pk_reset_range(pk_handle* h, uint32_t env0, uint32_t count, const uint8_t* mask, void* stream) {
    int rc;
    if ((rc = check_range(h, env0, count))) return rc;
    const uint32_t env1 = env0 + count;
    if (!(h->flags & PK_F_REWARD)) return template_reset(h, mask, env0, env1, stream);
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    PkRewardArgs r = reward_args(h, env0, env1);
    r.env_mask = mask;
    HIPCHK(pk_launch_rreset_pre(r, s));
    if ((rc = template_reset(h, h->reload, env0, env1, stream))) return rc;
    HIPCHK(pk_launch_rreset_post(r, s));
    // the observation of the reset envs only (list of the masked envs)
    HIPCHK(hipMemsetAsync(list_cnt(h, env0, 1), 0, 4, s));
    HIPCHK(pk_launch_list(mask, env0, env1, list_cnt(h, env0, 1), list_ids(h, env0, 1), s));
    r.ocnt = list_cnt(h, env0, 1);
    r.oids = list_ids(h, env0, 1);
    HIPCHK(pk_launch_obs(r, s));
    return 0;
}

int pk_reset(pk_handle* h, const uint8_t* mask, void* stream) {
    if (!h) return fail(-EINVAL, "null handle");
    return pk_reset_range(h, 0, h->n, mask, stream);
}

int pk_get_ram(pk_handle* h, uint16_t addr, uint32_t len, uint8_t* dense, void* stream) {
    if (!h || !dense) return fail(-EINVAL, "null argument");
    bool wram = addr >= 0xC000 && (uint32_t)addr + len <= 0xFE00, hram = addr >= 0xFF80 && (uint32_t)addr + len <= 0xFFFF;
    if (!len || !(wram || hram)) return fail(-EINVAL, "pk_get_ram: [0x%04x, +%u) is not inside WRAM/echo or HRAM", addr, len);
    if (wram && (addr & 0x1FFF) + len > 0x2000) return fail(-EINVAL, "pk_get_ram: range wraps the echo mirror");
    HIPCHK(hipSetDevice(h->device));
    uint32_t phys0 = wram ? PK_P_WRAM + (addr & 0x1FFFu) : PK_P_HRAM + (addr - 0xFF80u);
    HIPCHK(pk_launch_ram_copy(h->mem, dense, h->n, h->ilv_sh, phys0, len, 1, (hipStream_t)stream));
    return 0;
}

int pk_set_ram(pk_handle* h, uint16_t addr, uint32_t len, const uint8_t* dense, void* stream) {
    if (!h || !dense) return fail(-EINVAL, "null argument");
    bool wram = addr >= 0xC000 && (uint32_t)addr + len <= 0xFE00, hram = addr >= 0xFF80 && (uint32_t)addr + len <= 0xFFFF;
    if (!len || !(wram || hram)) return fail(-EINVAL, "pk_set_ram: [0x%04x, +%u) is not inside WRAM/echo or HRAM", addr, len);
    if (wram && (addr & 0x1FFF) + len > 0x2000) return fail(-EINVAL, "pk_set_ram: range wraps the echo mirror");
    HIPCHK(hipSetDevice(h->device));
    uint32_t phys0 = wram ? PK_P_WRAM + (addr & 0x1FFFu) : PK_P_HRAM + (addr - 0xFF80u);
    HIPCHK(pk_launch_ram_copy(h->mem, const_cast<uint8_t*>(dense), h->n, h->ilv_sh, phys0, len, 0, (hipStream_t)stream));
    return 0;
}

// K1 envs per wave for a launch of `count` envs (measured, profiles/r02_sweep_*, r02_ab/ab_prio.txt):
// the widest wave that still gives two waves per SIMD, whose priority variant hides one wave's
// fetch -> operand-read chain behind the other's datapath — 64 from 131,072 envs, 32 from 65,536
// (two 32-lane waves per SIMD beat one 64-lane wave by ~10 %), 16 for (16,384, 32,768] (configs[3]'s
// per-GPU shard: two 16-lane waves with priority +5 % over one 32-lane wave; without priority they
// were 4 % slower).  Smaller launches are latency-bound and keep one 32-lane wave per SIMD (more,
// narrower waves do not help: 4,096 envs at 4 per wave on every CU measured 2.4x slower); between
// the thresholds the narrower shape would need a second round of workgroups.  PK_WAVE_LANES fixes it.
static uint32_t k1_wave_lanes(const pk_handle* h, uint32_t count) {
    if (h->wave_lanes) return h->wave_lanes;
    const uint32_t npad = (count + PK_LANES - 1u) & ~(PK_LANES - 1u);
    if (npad / 64u >= 2u * h->simds) return 64u;
    if (npad / 32u >= 2u * h->simds) return 32u;
    if (npad / 16u > h->simds && npad / 16u <= 2u * h->simds) return 16u;
    return 32u;
}

// K1 wave shape and workgroup size of a launch.  A sub-batch range is shaped as if every env of the
// handle were resident at once: VecEnv steps its sub-batches concurrently on their own streams, and
// K1 runs one workgroup per CU (LDS), so concurrent ranges share the GPU only when each is laid
// out for its part of the CUs — e.g. the two 65,536-env halves of a 131,072-env handle run as 64-env
// waves in 512-thread workgroups, 128 CUs each, two waves per SIMD overall (shaped alone, each
// took every CU and the second range waited: 485k vs 688k env-steps/s).
// The wide (512-thread) shape puts two waves on each SIMD; those launches take K1's wave-priority
// variant (measured +5 % at 65,536 envs; with one wave per SIMD it only costs its two instructions).
static void k1_shape(const pk_handle* h, bool small, uint32_t& lanes, uint32_t& block, uint32_t& prio) {
    lanes = k1_wave_lanes(h, h->n);
    const uint32_t wg_envs = small ? PK_SMALL_WG_ENVS : PK_WG_ENVS;
    const uint32_t max_threads = small ? PK_SMALL_MAX_THREADS : PK_K1_MAX_THREADS;
    if (h->k1_block) {
        // PK_K1_BLOCK with the lanes picked for this handle: a workgroup holds at most wg_envs envs
        // (its HRAM code mirror), so a block too large for the wave width is narrowed
        block = h->k1_block < max_threads ? h->k1_block : max_threads;
        if ((block / PK_LANES) * lanes > wg_envs) block = wg_envs / lanes * PK_LANES;
    } else {
        const uint32_t waves = ((h->n + PK_LANES - 1u) / PK_LANES) * (PK_LANES / lanes);
        const uint32_t wide = wg_envs * PK_LANES / lanes < max_threads ? wg_envs * PK_LANES / lanes : max_threads;
        block = waves <= h->simds ? 256u : wide;
    }
    // wave priority pays with two waves of one workgroup per SIMD (measured +5 %); with the small
    // kernel the SIMD's second wave belongs to the other sub-batch, and priority measured -4 %
    // (profiles/r04b/summary.txt)
    prio = h->k1_prio >= 0 ? (uint32_t)h->k1_prio : (block > 256u && !small ? 1u : 0u);
}

// K1 variant of a launch: the small-LDS kernel for a range smaller than the handle (a VecEnv
// sub-batch, stepped concurrently with the others on its own stream) while waves carry <= 32 envs
// (its HRAM mirror holds 128 envs per 256-thread workgroup); measured +3 % on configs[3]'s 32,768-env
// shard in 2 sub-batches, -3..-7 % for whole-handle launches, which gain nothing from a second
// workgroup per CU but lose the staged banks (profiles/r04b, r04c)
static bool k1_small(const pk_handle* h, uint32_t env0, uint32_t env1) {
    if (h->k1_small >= 0) return h->k1_small != 0 && k1_wave_lanes(h, h->n) <= 32u;
    return (env1 - env0) < h->n && k1_wave_lanes(h, h->n) <= 32u;
}

static PkStepArgs step_args(pk_handle* h, const uint8_t* actions, uint32_t env0, uint32_t env1) {
    PkStepArgs a;
    memset(&a, 0, sizeof a);
    a.mem = h->mem; a.rom = h->rom; a.romw = reinterpret_cast<const uint32_t*>(h->rom); a.regs = h->regs; a.ucode = h->ucode; a.actions = actions;
    a.lat = h->lat; a.screen = h->screen; a.n = h->n; a.npad = h->npad;
    a.rom_bank_mask = h->bank_mask; a.mbc = h->mbc; a.frames = h->frames;
    a.release_frame = h->release; a.render_last = (h->flags & PK_F_RENDER) ? 1 : 0;
    a.lat_stride = (uint32_t)h->lat_stride;
    const bool small = k1_small(h, env0, env1);
    a.small = small ? 1u : 0u;
    a.nslots = small ? h->nslots_s : h->nslots;
    a.bank_slot = small ? h->bank_slot_s : h->bank_slot;
    a.slot_bank = small ? h->slot_bank_s : h->slot_bank;
    a.all_staged = a.nslots >= h->bank_mask + 1u ? 1u : 0u;   // pk_step.hip ALL: no unstaged-bank paths
    k1_shape(h, small, a.wave_lanes, a.block, a.prio);
    a.simds = h->simds;
    a.dbg = h->dbg;
    a.env0 = env0; a.env1 = env1;
    a.ilv_sh = h->ilv_sh;
    return a;
}

int pk_render_latched(pk_handle* h, void* stream) {
    if (!h) return fail(-EINVAL, "null handle");
    HIPCHK(hipSetDevice(h->device));
    PkStepArgs a = step_args(h, nullptr, 0, h->n);
    HIPCHK(pk_launch_render_latched(a, (hipStream_t)stream));
    return 0;
}

int pk_step_range(pk_handle* h, uint32_t env0, uint32_t count, const uint8_t* actions, double* rew, uint8_t* term,
                  uint8_t* trunc, void* stream) {
    int rc;
    if ((rc = check_range(h, env0, count))) return rc;
    if (!actions) return fail(-EINVAL, "actions_dev is required");
    HIPCHK(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    const uint32_t env1 = env0 + count;
    PkStepArgs a = step_args(h, actions, env0, env1);
    if (h->prof && (rc = prof_event(h, s))) return rc;
    HIPCHK(a.small ? pk_launch_step_small(a, s) : pk_launch_step(a, s));
    if (h->prof && (rc = prof_event(h, s))) return rc;
    if (a.render_last) HIPCHK(pk_launch_render(a, s));
    if (h->prof && (rc = prof_event(h, s))) return rc;
    if (h->flags & PK_F_REWARD) {
        PkRewardArgs r = reward_args(h, env0, env1);
        r.actions = actions; r.rew = rew; r.term = term; r.trunc = trunc;
        HIPCHK(pk_launch_reward(r, s));
        HIPCHK(pk_launch_obs(r, s));
    } else if (rew || term || trunc) {
        HIPCHK(pk_launch_done(h->regs + (size_t)PK_R_TIME * h->npad + env0, count, h->max_steps, term ? term + env0 : nullptr,
                              trunc ? trunc + env0 : nullptr, rew ? rew + env0 : nullptr, s));
    }
    if (h->prof && (rc = prof_event(h, s))) return rc;
    return 0;
}

int pk_step(pk_handle* h, const uint8_t* actions, uint8_t* screen_out, double* rew, uint8_t* term,
            uint8_t* trunc, void* stream) {
    if (!h) return fail(-EINVAL, "null handle");
    int rc = pk_step_range(h, 0, h->n, actions, rew, term, trunc, stream);
    if (rc) return rc;
    if (screen_out)
        HIPCHK(hipMemcpyAsync(screen_out, h->screen, (size_t)h->n * PK_SCREEN, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}

// gather one env's full state to host: mem (PK_PHYS), regs, latches, screen
static int fetch_env(pk_handle* h, uint32_t env, std::vector<uint8_t>& mem, uint32_t* regs,
                     uint32_t* lat, std::vector<uint8_t>& screen) {
    if (env >= h->n) return fail(-EINVAL, "env %u out of range (n=%u)", env, h->n);
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(pk_launch_gather_env(h->mem, env, h->ilv_sh, h->scratch, nullptr));
    mem.resize(PK_PHYS);
    HIPCHK(hipMemcpy(mem.data(), h->scratch, PK_PHYS, hipMemcpyDeviceToHost));
    for (uint32_t f = 0; f < PK_NREGS; f++)
        HIPCHK(hipMemcpy(&regs[f], h->regs + (size_t)f * h->npad + env, 4, hipMemcpyDeviceToHost));
    uint32_t gid = env / PK_LANES, lane = env % PK_LANES;
    for (uint32_t k = 0; k < 3; k++) {
        std::vector<uint32_t> tmp((size_t)PK_ROWS * PK_LANES);
        HIPCHK(hipMemcpy(tmp.data(), h->lat + k * h->lat_stride + (size_t)gid * PK_ROWS * PK_LANES,
                         tmp.size() * 4, hipMemcpyDeviceToHost));
        for (uint32_t y = 0; y < PK_ROWS; y++) lat[k * PK_ROWS + y] = tmp[(size_t)y * PK_LANES + lane];
    }
    screen.resize(PK_SCREEN);
    HIPCHK(hipMemcpy(screen.data(), h->screen + (size_t)env * PK_SCREEN, PK_SCREEN, hipMemcpyDeviceToHost));
    return 0;
}

int pk_snapshot(pk_handle* h, uint32_t env, uint8_t* out, uint64_t len) {
    if (!h || !out) return fail(-EINVAL, "null argument");
    if (len < S_SIZE) return fail(-EINVAL, "buffer too small for a v9 state");
    std::vector<uint8_t> mem, screen;
    uint32_t regs[PK_NREGS], lat[3 * PK_ROWS];
    int rc = fetch_env(h, env, mem, regs, lat, screen);
    if (rc) return rc;
    export_v9(h->tmpl, regs, mem.data(), lat, screen.data(), out);
    return 0;
}

int pk_snapshot_range(pk_handle* h, uint32_t env0, uint32_t count, uint8_t* out, uint64_t len) {
    if (!h || !out) return fail(-EINVAL, "null argument");
    if (count == 0) return 0;
    if ((uint64_t)env0 + count > h->n) return fail(-EINVAL, "envs [%u, %u) out of range (n=%u)", env0, env0 + count, h->n);
    if (len < (uint64_t)count * S_SIZE) return fail(-EINVAL, "buffer too small for %u v9 states", count);
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    const uint32_t chunk = count < 1024u ? count : 1024u;
    uint8_t* dmem = nullptr;
    HIPCHK(hipMalloc((void**)&dmem, (size_t)chunk * PK_PHYS));
    std::vector<uint8_t> mem((size_t)chunk * PK_PHYS), screen((size_t)chunk * PK_SCREEN);
    std::vector<uint32_t> regs((size_t)PK_NREGS * chunk), latg;
    int rc = 0;
    for (uint32_t c0 = 0; c0 < count && !rc; c0 += chunk) {
        const uint32_t e0 = env0 + c0, m = (count - c0) < chunk ? (count - c0) : chunk;
        hipError_t e = pk_launch_gather_range(h->mem, e0, m, h->ilv_sh, dmem, nullptr);
        if (e == hipSuccess) e = hipMemcpy(mem.data(), dmem, (size_t)m * PK_PHYS, hipMemcpyDeviceToHost);
        for (uint32_t f = 0; f < PK_NREGS && e == hipSuccess; f++)
            e = hipMemcpy(&regs[(size_t)f * chunk], h->regs + (size_t)f * h->npad + e0, (size_t)m * 4, hipMemcpyDeviceToHost);
        if (e == hipSuccess)
            e = hipMemcpy(screen.data(), h->screen + (size_t)e0 * PK_SCREEN, (size_t)m * PK_SCREEN, hipMemcpyDeviceToHost);
        // latches of the groups covering [e0, e0 + m)
        const uint32_t g0 = e0 / PK_LANES, g1 = (e0 + m - 1) / PK_LANES + 1, rows = (g1 - g0) * PK_ROWS * PK_LANES;
        latg.resize((size_t)3 * rows);
        for (uint32_t k = 0; k < 3 && e == hipSuccess; k++)
            e = hipMemcpy(&latg[(size_t)k * rows], h->lat + k * h->lat_stride + (size_t)g0 * PK_ROWS * PK_LANES,
                          (size_t)rows * 4, hipMemcpyDeviceToHost);
        if (e != hipSuccess) { rc = fail(-EIO, "pk_snapshot_range: %s", hipGetErrorString(e)); break; }
        for (uint32_t i = 0; i < m; i++) {
            const uint32_t env = e0 + i, gi = env / PK_LANES - g0, lane = env % PK_LANES;
            uint32_t r[PK_NREGS], lat[3 * PK_ROWS];
            for (uint32_t f = 0; f < PK_NREGS; f++) r[f] = regs[(size_t)f * chunk + i];
            for (uint32_t k = 0; k < 3; k++)
                for (uint32_t y = 0; y < PK_ROWS; y++)
                    lat[k * PK_ROWS + y] = latg[(size_t)k * rows + ((size_t)gi * PK_ROWS + y) * PK_LANES + lane];
            export_v9(h->tmpl, r, &mem[(size_t)i * PK_PHYS], lat, &screen[(size_t)i * PK_SCREEN], out + (size_t)(c0 + i) * S_SIZE);
        }
    }
    (void)hipFree(dmem);
    return rc;
}

int pk_load_env(pk_handle* h, uint32_t env, const uint8_t* in, uint64_t len) {
    if (!h || !in) return fail(-EINVAL, "null argument");
    if (env >= h->n) return fail(-EINVAL, "env %u out of range", env);
    Template t;
    int rc = parse_v9(in, len, t);
    if (rc) return rc;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(h->scratch, t.mem.data(), PK_PHYS, hipMemcpyHostToDevice));
    HIPCHK(pk_launch_scatter_env(h->mem, env, h->ilv_sh, h->scratch, nullptr));
    HIPCHK(hipDeviceSynchronize());
    // machine state only: the env's step counter (PK_R_TIME, pokegym `self.time`) and the per-step
    // bookkeeping slots survive a load, as in load_pyboy_state (pyboy_binding.py:59-62), which
    // leaves self.time alone; only reset() zeroes it
    for (uint32_t f = 0; f <= PK_R_MISC; f++)
        HIPCHK(hipMemcpy(h->regs + (size_t)f * h->npad + env, &t.regs[f], 4, hipMemcpyHostToDevice));
    uint32_t gid = env / PK_LANES, lane = env % PK_LANES;
    for (uint32_t k = 0; k < 3; k++)
        for (uint32_t y = 0; y < PK_ROWS; y++)
            HIPCHK(hipMemcpy(h->lat + k * h->lat_stride + ((size_t)gid * PK_ROWS + y) * PK_LANES + lane,
                             &t.lat[k * PK_ROWS + y], 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->screen + (size_t)env * PK_SCREEN, t.screen.data(), PK_SCREEN, hipMemcpyHostToDevice));
    return 0;
}

// guest-address view of one env's memory (PyBoy get_memory_value semantics for RAM regions and
// the special IO registers)
static int guest_phys(uint32_t addr, const uint32_t* regs, uint32_t mbc, uint32_t* phys, int* special) {
    *special = -1;
    if (addr < 0x8000) return -1;
    if (addr < 0xA000) { *phys = PK_P_VRAM + addr - 0x8000; return 0; }
    if (addr < 0xC000) {
        uint32_t m = regs[PK_R_MBC];
        if (mbc == 0 || !((m >> 16) & 0xFF)) return -2;
        *phys = PK_P_SRAM + (((m >> 8) & 3) * 0x2000) + (addr - 0xA000);
        return 0;
    }
    if (addr < 0xFE00) { *phys = PK_P_WRAM + (addr & 0x1FFF); return 0; }
    if (addr < 0xFF00) { *phys = PK_P_OAM + (addr - 0xFE00); return 0; }
    if (addr >= 0xFF80) {
        if (addr == 0xFFFF) { *special = (int)addr; return 1; }
        *phys = PK_P_HRAM + addr - 0xFF80;
        return 0;
    }
    if ((addr >= 0xFF04 && addr <= 0xFF07) || addr == 0xFF0F || (addr >= 0xFF10 && addr <= 0xFF4B)) {
        *special = (int)addr;
        return 1;
    }
    *phys = PK_P_IO + (addr - 0xFF00);
    return 0;
}

static uint8_t special_read(uint32_t a, const uint32_t* R) {
    auto b = [](uint32_t v, int sh) { return (uint8_t)((v >> sh) & 0xFF); };
    switch (a) {
        case 0xFF04: return b(R[PK_R_TIM0], 0);
        case 0xFF05: return b(R[PK_R_TIM0], 8);
        case 0xFF06: return b(R[PK_R_TIM0], 16);
        case 0xFF07: return b(R[PK_R_TIM0], 24);
        case 0xFF0F: return b(R[PK_R_CPU], 16);
        case 0xFF40: return b(R[PK_R_LCD0], 0);
        case 0xFF41: return b(R[PK_R_LCD0], 8);
        case 0xFF42: return b(R[PK_R_LCD1], 0);
        case 0xFF43: return b(R[PK_R_LCD1], 8);
        case 0xFF44: return b(R[PK_R_LCD0], 16);
        case 0xFF45: return b(R[PK_R_LCD0], 24);
        case 0xFF47: return b(R[PK_R_LCD2], 0);
        case 0xFF48: return b(R[PK_R_LCD2], 8);
        case 0xFF49: return b(R[PK_R_LCD2], 16);
        case 0xFF4A: return b(R[PK_R_LCD1], 16);
        case 0xFF4B: return b(R[PK_R_LCD1], 24);
        case 0xFFFF: return b(R[PK_R_CPU], 8);
        default: return 0;
    }
}

int pk_peek(pk_handle* h, uint32_t env, uint16_t addr, uint32_t len, uint8_t* out) {
    if (!h || !out) return fail(-EINVAL, "null argument");
    if ((uint32_t)addr + len > 0x10000u) return fail(-EINVAL, "range past 0xFFFF");
    std::vector<uint8_t> mem, screen;
    uint32_t regs[PK_NREGS], lat[3 * PK_ROWS];
    int rc = fetch_env(h, env, mem, regs, lat, screen);
    if (rc) return rc;
    std::vector<uint8_t> rom;
    for (uint32_t i = 0; i < len; i++) {
        uint32_t a = (uint32_t)addr + i, phys;
        int special;
        int k = guest_phys(a, regs, h->mbc, &phys, &special);
        if (k == 0) out[i] = mem[phys];
        else if (k == 1) out[i] = special_read(a, regs);
        else if (k == -2) out[i] = 0xFF;
        else {
            // ROM read
            uint32_t off = a < 0x4000 ? a : ((regs[PK_R_MBC] & 0xFF) & h->bank_mask) * 0x4000u + (a - 0x4000u);
            HIPCHK(hipMemcpy(&out[i], h->rom + off, 1, hipMemcpyDeviceToHost));
        }
    }
    return 0;
}

int pk_poke(pk_handle* h, uint32_t env, uint16_t addr, uint32_t len, const uint8_t* in) {
    if (!h || !in) return fail(-EINVAL, "null argument");
    if (env >= h->n) return fail(-EINVAL, "env %u out of range", env);
    if ((uint32_t)addr + len > 0x10000u) return fail(-EINVAL, "range past 0xFFFF");
    std::vector<uint8_t> mem, screen;
    uint32_t regs[PK_NREGS], lat[3 * PK_ROWS];
    int rc = fetch_env(h, env, mem, regs, lat, screen);
    if (rc) return rc;
    for (uint32_t i = 0; i < len; i++) {
        uint32_t a = (uint32_t)addr + i, phys;
        int special;
        if (guest_phys(a, regs, h->mbc, &phys, &special) != 0)
            return fail(-ENOTSUP, "pk_poke supports RAM regions only (addr 0x%04x)", a);
        HIPCHK(hipMemcpy(h->mem + pk_img_off(env, phys, h->ilv_sh), &in[i], 1,
                         hipMemcpyHostToDevice));
    }
    return 0;
}

int pk_profile_enable(pk_handle* h, int on) {
    if (!h) return fail(-EINVAL, "null handle");
    h->prof = on != 0;
    return 0;
}

int pk_profile_read(pk_handle* h, double* emu_ms, double* render_ms, double* reward_ms, uint64_t* steps) {
    if (!h || !emu_ms || !render_ms || !reward_ms || !steps) return fail(-EINVAL, "null argument");
    HIPCHK(hipSetDevice(h->device));
    double a = 0, b = 0, c = 0;
    size_t n = h->ev_used / 4;
    if (n) HIPCHK(hipEventSynchronize(h->ev_pool[h->ev_used - 1]));
    for (size_t i = 0; i < n; i++) {
        float t1 = 0, t2 = 0, t3 = 0;
        HIPCHK(hipEventElapsedTime(&t1, h->ev_pool[4 * i], h->ev_pool[4 * i + 1]));
        HIPCHK(hipEventElapsedTime(&t2, h->ev_pool[4 * i + 1], h->ev_pool[4 * i + 2]));
        HIPCHK(hipEventElapsedTime(&t3, h->ev_pool[4 * i + 2], h->ev_pool[4 * i + 3]));
        a += t1;
        b += t2;
        c += t3;
    }
    *emu_ms = a;
    *render_ms = b;
    *reward_ms = c;
    *steps = n;
    h->ev_used = 0;
    return 0;
}

// Environment.reset(max_episode_steps, reward_scale) (environment.py:1233, :1258-1259): the episode
// length and reward scale of the following steps.  When the new episode length needs a larger
// seen-coordinate set, every env's current-episode entries are re-inserted into the larger table
// (pk_seen_rehash_kernel), so envs that are not reset keep their seen coordinates.
int pk_set_episode_params(pk_handle* h, uint32_t max_episode_steps, double reward_scale) {
    if (!h) return fail(-EINVAL, "null handle");
    if (max_episode_steps == 0) return fail(-EINVAL, "max_episode_steps must be > 0");
    HIPCHK(hipSetDevice(h->device));
    if (h->flags & PK_F_REWARD) {
        uint32_t need = 10;
        while ((1ull << need) * 3 < ((uint64_t)max_episode_steps + 2) * 4) need++;
        if (need > h->cap_log2) {
            HIPCHK(hipDeviceSynchronize());
            uint32_t* seen = nullptr;
            const size_t bytes = (size_t)h->npad * (1ull << need) * 4;
            if (hipMalloc((void**)&seen, bytes) != hipSuccess) return fail(-ENOMEM, "hipMalloc(%zu) for the seen set", bytes);
            if (hipMemset(seen, 0, bytes) != hipSuccess) { (void)hipFree(seen); return fail(-EIO, "hipMemset failed"); }
            hipError_t e = pk_launch_seen_rehash(h->seen, h->cap_log2, seen, need, h->rs, h->n, h->npad, nullptr);
            if (e == hipSuccess) e = hipDeviceSynchronize();
            if (e != hipSuccess) { (void)hipFree(seen); return fail(-EIO, "seen-set rehash: %s", hipGetErrorString(e)); }
            (void)hipFree(h->seen);
            h->seen = seen;
            h->cap_log2 = need;
        }
    }
    h->max_steps = max_episode_steps;
    h->reward_scale = reward_scale;
    return 0;
}

// diagnostic: the K1 phase-cycle counters of a -DPK_STAMP build (zeros otherwise), then reset
int pk_debug_counters(pk_handle* h, uint64_t* out, uint32_t n) {
    if (!h || !out) return fail(-EINVAL, "null argument");
    memset(out, 0, (size_t)n * 8);
    if (!h->dbg) return 0;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(out, h->dbg, (size_t)(n < PK_DBG_WORDS ? n : PK_DBG_WORDS) * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemset(h->dbg, 0, PK_DBG_WORDS * 8));
    return 0;
}

int pk_last_instr_count(pk_handle* h, uint64_t* out) {
    if (!h || !out) return fail(-EINVAL, "null argument");
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());
    std::vector<uint32_t> v(h->n);
    HIPCHK(hipMemcpy(v.data(), h->regs + (size_t)PK_R_ICOUNT * h->npad, (size_t)h->n * 4, hipMemcpyDeviceToHost));
    uint64_t s = 0;
    for (uint32_t x : v) s += x;
    *out = s;
    return 0;
}

int pk_launch_shape(pk_handle* h, uint32_t env0, uint32_t count, uint32_t* out5) {
    int rc;
    if (!out5) return fail(-EINVAL, "null argument");
    if ((rc = check_range(h, env0, count))) return rc;
    const PkStepArgs a = step_args(h, nullptr, env0, env0 + count);
    out5[0] = a.small;
    out5[1] = a.wave_lanes;
    out5[2] = a.block;
    out5[3] = a.prio;
    out5[4] = a.all_staged;
    return 0;
}

}  // extern "C"
