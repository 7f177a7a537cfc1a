// pk_reward.h — device layout of the reward stack (K4), reset (K5r) and obs compose (K3).
//
// Per-env reward state restating the Python attributes pokegym keeps per Environment
// (environment.py:102-197, :437-522, :1256-1331).  SoA u32 fields rs[field * npad + env], three
// f64 fields rsd[field * npad + env], and three per-env side tables:
//   seen  u32[npad][cap]    open-addressing set of (r, c, map) = self.seen_coords (:1345);
//                           slot = r | c<<8 | map<<16 | gen<<24 (gen = episode tag 1..255, a slot
//                           with another gen is empty, so a reset never clears the table)
//   mask  u32[npad][2048]   256x256-bit visited mask of the CURRENT map = screen_memory[map]
//                           (:157-160, :256-263); rebuilt from `seen` when the map changes
//   cutc  u32[npad][64]     self.cut_coords in insertion order (:1519-1525)
#pragma once
#include <stdint.h>

enum {
    RS_FLAGS = 0,     // RSF_* bits
    RS_ERR,           // first error (PK_ERR_*), sticky until reset
    RS_USED_CUT,      // self.used_cut
    RS_SEEN_N,        // len(self.seen_coords)
    RS_GEN,           // seen-set episode tag 1..255
    RS_MAX_LEVEL,     // self.max_level_sum
    RS_MAX_OPP,       // self.max_opponent_level (info only)
    RS_MAX_EVENTS,    // self.max_events
    RS_LAST_PARTY,    // self.last_party_size
    RS_DEATHS,        // self.death_count (info only)
    RS_LAST_MAP1,     // self.last_10_map_ids[0][0]
    RS_HEAT_LAST,     // update_heat_map's self.last_map (-1 = none); survives resets
    RS_CUTSTATE0,     // self.cut_state: 3 x 6 bytes, oldest first, in words CUTSTATE0..4
    RS_CUTSTATE1,
    RS_CUTSTATE2,
    RS_CUTSTATE3,
    RS_CUTSTATE4,
    RS_CUTSTATE_N,    // entries in cut_state (0..3)
    RS_CUT_TILES,     // 8 words: 256-bit set of self.cut_tiles keys
    RS_CUT_TILES_END = RS_CUT_TILES + 8,
    RS_CUTC_N = RS_CUT_TILES_END,  // entries in cutc
    RS_MOVES,         // 6 words: self.moves_obtained bitmap (165 entries)
    RS_MOVES_END = RS_MOVES + 6,
    RS_MASK_MAP = RS_MOVES_END,    // map whose visited mask is in `mask` (0xFFFFFFFF = none)
    RS_RESET_POS,     // r | c<<8 | map<<16 | 1<<24 of the reset-time render() (:1334)
    RS_RESET_COUNT,   // self.reset_count
    RS_NFIELDS
};

enum { RSD_LAST_REWARD = 0, RSD_TOTAL_HEALING, RSD_LAST_HP, RSD_COORD /* np.sum(counts_map), survives resets */,
       RSD_NFIELDS };

// RS_FLAGS bits
#define RSF_HAS_LAST 1u       // self.last_reward is not None
#define RSF_IS_DEAD 2u        // self.is_dead (survives resets)
#define RSF_CUT 4u            // self.cut
#define RSF_MENU0 8u          // seen_start_menu, pokemon, stats, bag, cancel_bag: bits 3..7
#define RSF_BAG0 0x100u       // has_{lemonade,silph_scope,lift_key,pokedoll,bicycle}_in_bag_reward: bits 8..12 (survive resets)
#define RSF_STUCK_INIT 0x2000u  // self.stuck_cnt exists (survives resets)
#define RSF_KEEP (RSF_IS_DEAD | (0x1Fu * RSF_BAG0) | RSF_STUCK_INIT)

// error codes (the reference raises; include/pokegym_amd.h PK_ERR_*)
#define PKE_MAP_KEY 1u
#define PKE_STUCK_ATTR 2u
#define PKE_MOVE_INDEX 3u
#define PKE_CUT_COORDS 4u
#define PKE_HEATMAP_INDEX 5u
#define PKE_BUS_INDEX 6u
#define PKE_CAPACITY 7u       // device table full (no reference equivalent)
#define PKE_EMPTY_PARTY 8u    // ValueError: max(party_levels) of an empty party in the info dict (:1672)

// info telemetry record (environment.py:1621-1704; field order = pokegym_amd/info.py FIELDS)
#define PK_INFO_NSTATS 58u
#define PK_INFO_NREWARD 21u
#ifndef PK_INFO_NFIELDS
#define PK_INFO_NFIELDS 79u   // == include/pokegym_amd.h
#endif
static_assert(PK_INFO_NFIELDS == PK_INFO_NSTATS + PK_INFO_NREWARD, "info record layout");

#define PK_CUTC_CAP 64u
#define PK_INFO_BITS_WORDS 5u  // 130 event-monitor bits (ram_map_leanke monitor_*_events), MONITORS order
#define PK_HEAT_ROWS 444u     // counts_map = np.zeros((444, 436)) (environment.py:448)
#define PK_HEAT_COLS 436u
#define PK_MASK_WORDS 2048u   // 256 rows x 8 words
#define PK_OBS_H 72u
#define PK_OBS_W 80u
#define PK_OBS_BYTES (PK_OBS_H * PK_OBS_W * 4u)

struct PkRewardArgs {
    uint8_t* mem;             // lane-interleaved RAM images (pk_layout.h)
    uint32_t* regs;           // K1 lane registers (TIME, special IO regs)
    uint32_t* rs;             // [RS_NFIELDS][npad]
    double* rsd;              // [RSD_NFIELDS][npad]
    uint32_t* seen;           // [npad][cap]
    uint32_t* mask;           // [npad][PK_MASK_WORDS]
    uint32_t* cutc;           // [npad][PK_CUTC_CAP]
    const uint8_t* actions;   // [n]
    const uint8_t* env_mask;  // reset: envs to reset (null = all)
    uint8_t* reload;          // reset: [n] out = template reload wanted
    const uint8_t* screen;    // [npad][144][160] grey
    uint8_t* obs;             // [n][72][80][4]
    const uint32_t* ocnt;     // obs for listed envs only (reset): count (device memory) and ids,
    const uint32_t* oids;     // or null = all n envs
    double* rew;              // [n] or null
    uint8_t* term;            // [n] or null
    uint8_t* trunc;           // [n] or null
    double* info;             // [PK_INFO_NFIELDS][npad] info record, written where info_flag = 1
    uint8_t* info_flag;       // [n] 1 = this step built the reference's info dict (done or time % 10000 == 0)
    uint32_t* info_bits;      // [PK_INFO_BITS_WORDS][npad] monitor bits of the info record's step
    int32_t* heat;            // [npad][PK_HEAT_ROWS * PK_HEAT_COLS] counts_map, or null (PK_F_HEATMAP off)
    double reward_scale;
    uint32_t n, npad;
    uint32_t cap_log2;        // seen table capacity = 1 << cap_log2
    uint32_t max_steps;
    uint32_t reload_always;   // PK_F_RELOAD_ON_RESET
    uint32_t env0, env1;      // env range of this launch (sub-batches); arrays stay full-size [n]
    uint32_t ilv_sh;          // image interleave (pk_layout.h pk_img_off)
};
