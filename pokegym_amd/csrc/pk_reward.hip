// pk_reward.hip — MI355X kernels for the per-step reward stack, reset and observation.
//
//   K4 pk_reward_kernel      one lane per env, after K1/K2: pokegym Environment.step after
//                            run_action_on_emulator (environment.py:1338-1612): the ram_map /
//                            ram_map_leanke / red_ram_api peeks, their WRAM writes, the episode
//                            bookkeeping and the order-sensitive float64 reward, plus the visited
//                            mask update of render() (:256-263).
//   K5r pk_rreset_*_kernel   Environment.reset (environment.py:1233-1334) around the template
//                            reload of pk_kernels.hip (reload only on the first reset, :1241).
//   K3 pk_obs_kernel         render(): screen[::2, ::2] (3 grey channels) + the 72x80 window of
//                            the visited mask (get_fixed_window, :233-254) -> u8 (72, 80, 4).
//
// Parity: bit-exact against oracle/reward.py, itself pinned on the reference's own outputs
// (tests/golden/reward_replay.npz).  Reads go to the same lane-interleaved RAM images K1 runs
// on (64 lanes of a group read the same guest address -> one coalesced 64-byte access).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pk_layout.h"
#include "pk_reward.h"
#include "pk_reward_tables.h"

typedef uint32_t u32;
typedef uint8_t u8;

// every float64 expression below is evaluated as written (Python evaluates `a * b + c` as two
// rounded operations): no FMA contraction in this file.
#pragma clang fp contract(off)

namespace {

struct RMem {
    u8* g;          // the env's image sub-block (pk_layout.h)
    u32 lane, sh;   // lane within it, interleave shift
    const u32* regs;
    u32 np, env;
    u32 err;
};

__device__ __forceinline__ void rmem_at(RMem& M, u8* mem, u32 e, u32 sh) {
    M.lane = e & (PK_LANES - 1u) & ((1u << sh) - 1u);
    M.g = mem + pk_img_off(e, 0u, sh) - M.lane;
    M.sh = sh;
}

__device__ __forceinline__ u32 bfe8(u32 v, u32 sh) { return (v >> sh) & 0xFFu; }

// PyBoy get_memory_value for the regions the reward stack can reach (WRAM, echo, FE00-FFFF)
__device__ u32 rd(RMem& M, u32 a) {
    if (a > 0xFFFFu) {
        if (!M.err) M.err = PKE_BUS_INDEX;
        return 0;
    }
    if (a >= 0xFE00u) {
        const u32 r = M.env;
        if ((a >= 0xFF04u && a <= 0xFF07u) || a == 0xFF0Fu || (a >= 0xFF10u && a <= 0xFF4Bu) || a == 0xFFFFu) {
            const u32 tim0 = M.regs[PK_R_TIM0 * M.np + r], cpu = M.regs[PK_R_CPU * M.np + r];
            const u32 l0 = M.regs[PK_R_LCD0 * M.np + r], l1 = M.regs[PK_R_LCD1 * M.np + r], l2 = M.regs[PK_R_LCD2 * M.np + r];
            switch (a) {
                case 0xFF04: return bfe8(tim0, 0);
                case 0xFF05: return bfe8(tim0, 8);
                case 0xFF06: return bfe8(tim0, 16);
                case 0xFF07: return bfe8(tim0, 24);
                case 0xFF0F: return bfe8(cpu, 16);
                case 0xFF40: return bfe8(l0, 0);
                case 0xFF41: return bfe8(l0, 8);
                case 0xFF42: return bfe8(l1, 0);
                case 0xFF43: return bfe8(l1, 8);
                case 0xFF44: return bfe8(l0, 16);
                case 0xFF45: return bfe8(l0, 24);
                case 0xFF47: return bfe8(l2, 0);
                case 0xFF48: return bfe8(l2, 8);
                case 0xFF49: return bfe8(l2, 16);
                case 0xFF4A: return bfe8(l1, 16);
                case 0xFF4B: return bfe8(l1, 24);
                case 0xFFFF: return bfe8(cpu, 8);
                default: return 0;
            }
        }
        return M.g[((size_t)(a - 0xBE00u) << M.sh) + M.lane];
    }
    if (a < 0xC000u) return 0;  // not reachable from the reward stack
    return M.g[((size_t)(PK_P_WRAM + (a & 0x1FFFu)) << M.sh) + M.lane];
}

// PyBoy set_memory_value for WRAM (the only region the reward stack writes)
__device__ __forceinline__ void wr(RMem& M, u32 a, u32 v) {
    M.g[((size_t)(PK_P_WRAM + (a & 0x1FFFu)) << M.sh) + M.lane] = (u8)v;
}

__device__ __forceinline__ u32 rbit(RMem& M, u32 a, u32 b) { return (rd(M, a) >> b) & 1u; }

// red_ram_api.py:667-675 Menus._get_menu_item_state
__device__ u32 menu_item_state(RMem& M, u32 cur) {
    if (cur == pk_menu_item_keys[0] || cur == pk_menu_item_keys[1] || cur == pk_menu_item_keys[2]) {
        if (rd(M, 0xC48F) == 0x7Eu) return PK_MV_ITEM_QUANTITY;
        const u32 k = rd(M, 0xCC26) + rd(M, 0xCC36) + 1u;
        for (u32 i = 0; i < PK_NITEM_LOC; i++)
            if (pk_item_loc[i][0] == k) return pk_item_loc[i][1];
        return PK_MV_ITEM_RANGE_ERROR;
    }
    return PK_SV_UNKNOWN;
}

// red_ram_api.py:203-225 Battle.get_battle_state (+ :149-201)
__device__ u32 battle_state(RMem& M) {
    u32 bt = rd(M, 0xD057);
    if (bt == 255u) bt = 4u;
    const u32 pre = rd(M, 0xD059);
    if (!(bt || pre)) return PK_GS_UNKNOWN;
    const u32 cur = rd(M, 0xCC30) | (rd(M, 0xCC31) << 8);
    u32 state = PK_MV_UNKNOWN;
    for (u32 i = 0; i < PK_NMENU_LOC; i++)
        if ((pk_menu_loc[i] & 0xFFFFu) == cur) state = pk_menu_loc[i] >> 16;
    u32 gs = state;
    if (gs == PK_MV_PC_LOGOFF) gs = PK_MV_MENU_YES;
    else if (gs == PK_MV_SELECT_STATS) gs = PK_MV_BATTLE_SWITCH;
    else if (gs == PK_MV_SELECT_SWITCH) gs = PK_MV_BATTLE_STATS;
    u32 ov = 0xFFFFFFFFu;
    if (gs == PK_MV_MENU_YES || gs == PK_MV_MENU_NO) {
        const u32 tdp = rd(M, 0xCC3A);
        if (tdp == 0xF0u) ov = gs == PK_MV_MENU_YES ? PK_MV_NAME_YES : PK_MV_NAME_NO;
        else if (tdp == 0xEDu) ov = gs == PK_MV_MENU_YES ? PK_MV_SWITCH_YES : PK_MV_SWITCH_NO;
    }
    if (ov == 0xFFFFFFFFu)
        ov = (gs == PK_MV_MENU_YES || gs == PK_MV_MENU_NO || gs == PK_MV_BATTLE_SWITCH || gs == PK_MV_BATTLE_STATS) ? gs : PK_GS_UNKNOWN;
    if (ov != PK_GS_UNKNOWN) return ov;
    if (cur == 0u || !bt) return PK_GS_BATTLE_ANIMATION;
    if ((rd(M, 0xD125) == 1u && rd(M, 0xD730) != 0x40u) || rd(M, 0xCC52) == 0u) return PK_GS_BATTLE_TEXT;
    if (state != PK_MV_UNKNOWN) {
        if (menu_item_state(M, cur) != PK_SV_UNKNOWN) {
            const u32 k = rd(M, 0xCC26) + rd(M, 0xCC36) + 1u;
            state = PK_MV_ITEM_RANGE_ERROR;
            for (u32 i = 0; i < PK_NITEM_LOC; i++)
                if (pk_item_loc[i][0] == k) state = pk_item_loc[i][1];
        }
        return state;
    }
    return PK_GS_UNKNOWN;
}

__device__ __forceinline__ u32 seen_hash(u32 key, u32 lg) { return (key * 2654435761u) >> (32u - lg); }

// insert (r, c, map) into this env's seen set; returns 1 if new, 0 if present, 2 if full
__device__ u32 seen_insert(u32* tab, u32 lg, u32 gen, u32 key, u32 count) {
    const u32 cap = 1u << lg, msk = cap - 1u;
    const u32 tagged = key | (gen << 24);
    u32 h = seen_hash(key, lg);
    for (u32 probe = 0; probe < cap; probe++, h = (h + 1u) & msk) {
        const u32 v = tab[h];
        if ((v >> 24) != gen) {
            if (count + 2u >= cap) return 2u;
            tab[h] = tagged;
            return 1u;
        }
        if (v == tagged) return 0u;
    }
    return 2u;
}

__device__ __forceinline__ void mask_set(u32* mk, u32 r, u32 c) {
    if (r <= 254u && c <= 254u) mk[r * 8u + (c >> 5)] |= 1u << (c & 31u);
}

// screen_memory[map] for the current map == {reset-time position} U {seen (r, c, map)}
__device__ void mask_rebuild(u32* mk, const u32* tab, u32 lg, u32 gen, u32 map, u32 reset_pos) {
    for (u32 i = 0; i < PK_MASK_WORDS; i++) mk[i] = 0;
    const u32 cap = 1u << lg;
    for (u32 i = 0; i < cap; i++) {
        const u32 v = tab[i];
        if ((v >> 24) == gen && ((v >> 16) & 0xFFu) == map) mask_set(mk, v & 0xFFu, (v >> 8) & 0xFFu);
    }
    if ((reset_pos >> 24) && ((reset_pos >> 16) & 0xFFu) == map) mask_set(mk, reset_pos & 0xFFu, (reset_pos >> 8) & 0xFFu);
}

// environment.py:1027-1039 update_last_10_map_ids: only the victory-road writes are observable
__device__ void update_last_map(RMem& M, u32& last1) {
    const u32 cur = rd(M, 0xD35E) + 1u;
    if (cur == last1) return;
    last1 = cur;
    const u32 m = cur - 1u;
    if (m == 0x6Cu || m == 0xC2u || m == 0xC6u || m == 0x22u) {
        wr(M, 0xD7EE, rd(M, 0xD7EE) | 0x01u);
        wr(M, 0xD7EE, rd(M, 0xD7EE) | 0x80u);
        wr(M, 0xD813, rd(M, 0xD813) | 0x01u);
        wr(M, 0xD813, rd(M, 0xD813) | 0x40u);
        wr(M, 0xD869, rd(M, 0xD869) | 0x80u);
    }
}

// environment.py:733-753 update_seen_map_dict: KeyError / uninitialised stuck_cnt paths
__device__ u32 seen_map_check(RMem& M, u32 last1, u32& flags) {
    const u32 m = last1 - 1u;
    if (m > 255u || !pk_map_dims[m][2]) return PKE_MAP_KEY;
    const u32 x = rd(M, 0xD362), y = rd(M, 0xD361);
    if (y >= (u32)pk_map_dims[m][0] || x >= (u32)pk_map_dims[m][1])
        return (flags & RSF_STUCK_INIT) ? 0u : PKE_STUCK_ATTR;
    flags |= RSF_STUCK_INIT;
    return 0u;
}

__device__ __forceinline__ void local_to_global(u32 r, u32 c, u32 m, int& gr, int& gc) {
    gr = (int)r;
    gc = (int)c;
    if (pk_map_coord[m][2]) {
        gr += pk_map_coord[m][1];
        gc += pk_map_coord[m][0];
    }
}

__device__ __forceinline__ bool seq_eq(u32 b0, u32 b1, u32 b2, u32 b3, u32 b4, u32 b5, const int* row, bool skip0) {
    return (skip0 || (int)b0 == row[0]) && (int)b1 == row[1] && (int)b2 == row[2] && (int)b3 == row[3] &&
           (int)b4 == row[4] && (int)b5 == row[5];
}

__device__ __forceinline__ u32 cs_byte(const u32* w, u32 i) { return (w[i >> 2] >> ((i & 3u) * 8u)) & 0xFFu; }

}  // namespace

// environment.py:48-50
__device__ __constant__ int k_cut_seq[2][2][6] = {{{0x3D, 1, 1, 0, 4, 1}, {0x3D, 1, 1, 0, 1, 1}},
                                                  {{0x50, 1, 1, 0, 4, 1}, {0x50, 1, 1, 0, 1, 1}}};
__device__ __constant__ int k_cut_grass[3][6] = {{0x52, 255, 1, 0, 1, 1}, {0x52, 255, 1, 0, 1, 1}, {0x52, 1, 1, 0, 1, 1}};
__device__ __constant__ int k_cut_fail[3][6] = {{-1, 255, 0, 0, 4, 1}, {-1, 255, 0, 0, 1, 1}, {-1, 255, 0, 0, 1, 1}};
__device__ __constant__ u32 k_party_species[6] = {0xD16B, 0xD197, 0xD1C3, 0xD1EF, 0xD21B, 0xD247};
__device__ __constant__ u32 k_party_level[6] = {0xD18C, 0xD1B8, 0xD1E4, 0xD210, 0xD23C, 0xD268};
__device__ __constant__ u32 k_hp[6] = {0xD16C, 0xD198, 0xD1C4, 0xD1F0, 0xD21C, 0xD248};
__device__ __constant__ u32 k_max_hp[6] = {0xD18D, 0xD1B9, 0xD1E5, 0xD211, 0xD23D, 0xD269};
__device__ __constant__ u32 k_opp_level[6] = {0xD8C5, 0xD8F1, 0xD91D, 0xD949, 0xD975, 0xD9A1};

// ---------------------------------------------------------------------------------------------
// K4: one env-step of the reward stack
__global__ void __launch_bounds__(256) pk_reward_kernel(PkRewardArgs A) {
    const u32 e = A.env0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= A.env1) return;
    const u32 np = A.npad;
    u32* rs = A.rs;
    double* rsd = A.rsd;
    RMem M;
    rmem_at(M, A.mem, e, A.ilv_sh);
    M.regs = A.regs;
    M.np = np;
    M.env = e;
    M.err = 0;
    const u32 time = A.regs[PK_R_TIME * np + e];   // K1 already did self.time += 1 (:1338)
    const bool done = time >= A.max_steps;          // :1613
    if (A.term) A.term[e] = done ? 1 : 0;
    if (A.trunc) A.trunc[e] = done ? 1 : 0;
    if (A.info_flag) A.info_flag[e] = 0;
    if (rs[RS_ERR * np + e]) {                      // the reference env raised: frozen
        if (A.rew) A.rew[e] = 0.0;
        return;
    }
    u32 flags = rs[RS_FLAGS * np + e];
    u32* tab = A.seen + (size_t)e * (1u << A.cap_log2);
    const u32 gen = rs[RS_GEN * np + e];

    // exploration (:1344-1345): position() clamps map_n to 247 (ram_map.py:1522-1538)
    const u32 r = rd(M, 0xD361), c = rd(M, 0xD362), map = min(rd(M, 0xD35E), 247u);
    u32 seen_n = rs[RS_SEEN_N * np + e];
    {
        const u32 k = seen_insert(tab, A.cap_log2, gen, r | (c << 8) | (map << 16), seen_n);
        if (k == 2u) M.err = PKE_CAPACITY;
        seen_n += k & 1u;
    }
    // process_game_states (:1348; red_ram_api.py:59-73, :571-602)
    if (rd(M, 0xCFC4) == 0u && battle_state(M) == PK_GS_UNKNOWN && rd(M, 0xCD38) == 0u) {
        wr(M, 0xCC30, 0);
        wr(M, 0xCC31, 0);
        for (u32 i = 0; i < 10u; i++) wr(M, 0xCF7C + i, 0);
    }
    // get_bag_item_ids names (:1349; red_ram_api.py:404-422): all 20 slots
    u32 has = 0;
    for (u32 i = 0; i < 20u; i++) {
        const u32 v = rd(M, 0xD31E + 2u * i);
        for (u32 t = 0; t < 5u; t++) has |= ((pk_bag_name_bits[t][v >> 5] >> (v & 31u)) & 1u) << t;
    }
    u32 last1 = rs[RS_LAST_MAP1 * np + e];
    update_last_map(M, last1);                      // :1352
    {
        const u32 ek = seen_map_check(M, last1, flags);  // :1354
        if (ek && !M.err) M.err = ek;
    }
    flags |= has * RSF_BAG0;                        // :1358-1372 (never reset)
    const u32 used_cut = rs[RS_USED_CUT * np + e];
    const double exploration = (used_cut < 1u ? 0.02 : 0.1) * (double)seen_n;   // :1375
    {   // update_heat_map (:1377, :648-679): a map change writes counts_map[(gr, gc)] unguarded
        int gr, gc;
        local_to_global(r, c, map, gr, gc);
        const int last = (int)rs[RS_HEAT_LAST * np + e];
        const bool same = last == (int)map || last == -1;
        if (!same && (gr >= 444 || gc >= 436) && !M.err) M.err = PKE_HEATMAP_INDEX;
        // the map itself (PK_F_HEATMAP): +1 on the same map (an out-of-range cell is skipped, the
        // reference swallows that IndexError, :669-673), -1 at the entry cell of a new map (:676)
        if (A.heat && !M.err && gr < 444 && gc < 436) {
            int32_t* cell = A.heat + (size_t)e * (PK_HEAT_ROWS * PK_HEAT_COLS) + (u32)gr * PK_HEAT_COLS + (u32)gc;
            const int old = *cell, nv = same ? old + 1 : -1;
            *cell = nv;
            rsd[RSD_COORD * np + e] = rsd[RSD_COORD * np + e] + (double)(nv - old);
        }
        rs[RS_HEAT_LAST * np + e] = map;
    }
    // level (:1386-1391)
    const u32 party_size = rd(M, 0xD163);
    u32 lsum = 0;
    for (u32 k = 0; k < 6u; k++) lsum += rd(M, k_party_level[k]);   // zero levels add nothing
    u32 max_level = max(rs[RS_MAX_LEVEL * np + e], lsum);
    const double level_reward = max_level < 50u ? (double)max_level : 50.0 + (double)(max_level - 50u) / 4.0;
    // healing / death (:1394-1408; ram_map.py:1567-1575)
    u32 hps = 0, mhs = 0;
    for (u32 k = 0; k < 6u; k++) {
        hps += 256u * rd(M, k_hp[k]) + rd(M, k_hp[k] + 1u);
        mhs += 256u * rd(M, k_max_hp[k]) + rd(M, k_max_hp[k] + 1u);
    }
    const double hp = mhs == 0u ? 1.0 : (double)hps / (double)mhs;
    const double last_hp = rsd[RSD_LAST_HP * np + e];
    double total_healing = rsd[RSD_TOTAL_HEALING * np + e];
    const double hp_delta = hp - last_hp;
    if (hp_delta > 0.2 && party_size == rs[RS_LAST_PARTY * np + e] && !(flags & RSF_IS_DEAD)) total_healing = total_healing + hp_delta;
    u32 deaths = rs[RS_DEATHS * np + e];
    if (hp <= 0.0 && last_hp > 0.0) {
        deaths += 1u;
        flags |= RSF_IS_DEAD;
    } else if (hp > 0.01) {
        flags &= ~RSF_IS_DEAD;
    }
    // badges, bill, HMs, cut (:1411-1426)
    const u32 badges_reward = 10u * (u32)__builtin_popcount(rd(M, 0xD356));
    const u32 bill_reward = 5u * rbit(M, 0xD7F2, 3);
    u32 hm_count = 0;
    {
        u32 seenhm = 0;
        for (u32 i = 0; i < 10u; i++) {   // ram_map.get_items_in_bag: first 10 slots, stop at 0/FF
            const u32 v = rd(M, 0xD31E + 2u * i);
            if (v == 0u || v == 0xFFu) break;
            if (v >= 0xC4u && v <= 0xC8u) seenhm |= 1u << (v - 0xC4u);
        }
        hm_count = (u32)__builtin_popcount(seenhm);
    }
    const u32 hm_reward = hm_count * 10u;
    const u32 cut_rew = (flags & RSF_CUT) ? 8u : 0u;
    // trees (:1429-1431, :277-312) in global coordinates, literal (x, y) order quirk
    double tree = 0.0;
    {
        int gr, gc;
        local_to_global(r, c, map, gr, gc);
        for (u32 i = 0; i < PK_NTREES; i++) {
            if ((u32)pk_trees[i][0] != map) continue;
            const int dx = gr - pk_trees[i][1], dy = gc - pk_trees[i][2];
            const int d = (dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy);
            if (d <= 5) tree = tree + 1.0 / (double)(d > 1 ? d : 1);
        }
    }
    {   // opponent level (:1438-1439, info only)
        u32 mo = 0;
        for (u32 k = 0; k < 6u; k++) mo = max(mo, rd(M, k_opp_level[k]));
        rs[RS_MAX_OPP * np + e] = max(rs[RS_MAX_OPP * np + e], mo);
    }
    // events (:1443-1445; ram_map.py:1592-1601)
    u32 ev = 0;
    for (u32 a = 0xD747; a < 0xD886; a++) ev += (u32)__builtin_popcount(rd(M, a));
    const int events = max((int)ev - 13 - (int)rbit(M, 0xD754, 0), 0);
    const u32 max_events = max(rs[RS_MAX_EVENTS * np + e], (u32)events);
    // dojo (:1448; ram_map_leanke.py:793-814)
    int dojo = 0;
    {
        const u32 v = rd(M, 0xD7B1);
        for (u32 b = 0; b < 8u; b++) dojo += ((v >> b) & 1u) ? pk_dojo_w[b] : 0;
    }
    // nine monitor dicts through calculate_event_rewards (:1457-1491, :1201-1219)
    int mon[PK_NMON];
    u32 mbits[PK_INFO_BITS_WORDS] = {0, 0, 0, 0, 0};   // the monitor bits, for the info dicts
    for (u32 k = 0; k < PK_NMON; k++) {
        int total = 0, cur = 10;
        for (u32 i = pk_mon_start[k]; i < pk_mon_start[k + 1]; i++) {
            const u32 en = pk_mon_ent[i];
            const int w = (int)((en >> 20) & 0xFFu) - 128;
            const u32 b = rbit(M, en & 0xFFFFu, (en >> 16) & 0xFu);
            mbits[i >> 5] |= b << (i & 31u);
            const int pts = w * (int)b;
            if (pts > 0) {
                total += cur * pts;
                cur += 2;
            }
        }
        mon[k] = total;
    }
    // cut state machine (:1496-1538)
    u32* cutc = A.cutc + (size_t)e * PK_CUTC_CAP;
    u32 cutc_n = rs[RS_CUTC_N * np + e];
    if (rd(M, 0xD057) == 0u && (flags & RSF_CUT)) {
        const u32 d = rd(M, 0xC109);
        const int x = (int)rd(M, 0xD362), y = (int)rd(M, 0xD361);
        const u32 mid = rd(M, 0xD35E);
        const bool known = d == 0u || d == 4u || d == 8u || d == 0xCu;
        const int cx = d == 8u ? x - 1 : d == 0xCu ? x + 1 : x;
        const int cy = d == 0u ? y + 1 : d == 4u ? y - 1 : y;
        // append to the 3-deep deque (bytes 0..17, oldest first)
        u32 w[5];
        for (u32 i = 0; i < 5u; i++) w[i] = rs[(RS_CUTSTATE0 + i) * np + e];
        u32 ncs = rs[RS_CUTSTATE_N * np + e];
        u32 b[18];
        for (u32 i = 0; i < 18u; i++) b[i] = cs_byte(w, i);
        if (ncs == 3u) {
            for (u32 i = 0; i < 12u; i++) b[i] = b[i + 6u];
            ncs = 2u;
        }
        const u32 addrs[6] = {0xCFC6, 0xCFCB, 0xCD6A, 0xD367, 0xD125, 0xCD3D};
        for (u32 i = 0; i < 6u; i++) b[ncs * 6u + i] = rd(M, addrs[i]);
        ncs += 1u;
        for (u32 i = 0; i < 5u; i++) w[i] = 0;
        for (u32 i = 0; i < 18u; i++) w[i >> 2] |= b[i] << ((i & 3u) * 8u);
        for (u32 i = 0; i < 5u; i++) rs[(RS_CUTSTATE0 + i) * np + e] = w[i];
        rs[RS_CUTSTATE_N * np + e] = ncs;
        int hit = 0;  // 1 = 10, 2 = 0.001
        if (ncs == 3u) {
            for (u32 s = 0; s < 2u; s++)
                if (seq_eq(b[6], b[7], b[8], b[9], b[10], b[11], k_cut_seq[s][0], false) &&
                    seq_eq(b[12], b[13], b[14], b[15], b[16], b[17], k_cut_seq[s][1], false)) hit = 1;
            if (!hit) {
                bool g = true, f = true;
                for (u32 j = 0; j < 3u; j++) {
                    g = g && seq_eq(b[6 * j], b[6 * j + 1], b[6 * j + 2], b[6 * j + 3], b[6 * j + 4], b[6 * j + 5], k_cut_grass[j], false);
                    f = f && seq_eq(b[6 * j], b[6 * j + 1], b[6 * j + 2], b[6 * j + 3], b[6 * j + 4], b[6 * j + 5], k_cut_fail[j], true);
                }
                if (g || f) hit = 2;
            }
        }
        if (hit) {
            if (!known) {
                if (!M.err) M.err = PKE_CUT_COORDS;
            } else {
                const u32 key = (u32)(cx + 1) | ((u32)(cy + 1) << 10) | (mid << 20) | (1u << 30);
                u32 i = 0;
                while (i < cutc_n && (cutc[i] & 0x7FFFFFFFu) != key) i++;
                if (i == cutc_n) {
                    if (cutc_n == PK_CUTC_CAP) {
                        if (!M.err) M.err = PKE_CAPACITY;
                        i = PK_CUTC_CAP - 1u;
                    } else {
                        cutc_n += 1u;
                    }
                }
                cutc[i] = key | (hit == 1 ? 0x80000000u : 0u);
                const u32 tile = b[12];
                rs[(RS_CUT_TILES + (tile >> 5)) * np + e] |= 1u << (tile & 31u);
            }
        }
        if (rbit(M, 0xD803, 0)) {
            const u32 d057 = rd(M, 0xD057), cf13 = rd(M, 0xCF13), cf94 = rd(M, 0xCF94);
            const u32 a = A.actions ? A.actions[e] : 8u;
            if (d057 == 0u && cf13 == 0u && rd(M, 0xFF8C) == 6u && cf94 == 0u) flags |= RSF_MENU0 << 0;
            if (d057 == 0u && cf13 == 0u && rd(M, 0xFF8C) == 6u && cf94 == 2u) flags |= RSF_MENU0 << 1;
            if (d057 == 0u && cf13 == 0u) flags |= RSF_MENU0 << 2;
            if (d057 == 0u && cf13 == 0u && cf94 == 3u) flags |= RSF_MENU0 << 3;
            // WindowEvent.PRESS_BUTTON_A (PyBoy 1.x id 5) compared with the action id (:691)
            if (a == 5u && d057 == 0u && cf13 == 0u && cf94 == 3u && rd(M, 0xD31D) == rd(M, 0xCC36) + rd(M, 0xCC26))
                flags |= RSF_MENU0 << 4;
        }
    }
    rs[RS_CUTC_N * np + e] = cutc_n;
    // update_pokedex (:552-558)
    u32 seen_cnt = 0, caught_cnt = 0;
    for (u32 i = 0; i < 19u; i++) {
        seen_cnt += (u32)__builtin_popcount(rd(M, 0xD30A + i));
        caught_cnt += (u32)__builtin_popcount(rd(M, 0xD2F7 + i));
    }
    // update_moves_obtained (:560-580)
    u32 mv[6];
    for (u32 i = 0; i < 6u; i++) mv[i] = rs[(RS_MOVES + i) * np + e];
    for (u32 k = 0; k < 6u; k++) {
        if (rd(M, k_party_species[k]) == 0u) continue;
        for (u32 j = 0; j < 4u; j++) {
            const u32 m = rd(M, k_party_species[k] + j + 8u);
            if (m == 0u) continue;
            if (m >= 0xA5u) { if (!M.err) M.err = PKE_MOVE_INDEX; continue; }
            mv[m >> 5] |= 1u << (m & 31u);
            if (m == 15u) flags |= RSF_CUT;
        }
    }
    {
        const u32 nbox = rd(M, 0xDA80);
        for (u32 i = 0; i < nbox && !M.err; i++) {
            const u32 off = i * 200u + 0xDA96u;
            if (rd(M, off) == 0u) continue;
            for (u32 j = 0; j < 4u && !M.err; j++) {
                const u32 m = rd(M, off + j + 8u);
                if (m == 0u) continue;
                if (m >= 0xA5u) { M.err = PKE_MOVE_INDEX; break; }
                mv[m >> 5] |= 1u << (m & 31u);
            }
        }
    }
    for (u32 i = 0; i < 6u; i++) rs[(RS_MOVES + i) * np + e] = mv[i];
    u32 moves_cnt = 0;
    for (u32 i = 0; i < 6u; i++) moves_cnt += (u32)__builtin_popcount(mv[i]);
    // bill_capt (ram_map.py:1889-1898)
    const u32 bill_capt = 5u * (rbit(M, 0xD7F1, 0) + rbit(M, 0xD7F2, 3) + rbit(M, 0xD7F2, 4) + rbit(M, 0xD7F2, 5) +
                                rbit(M, 0xD7F2, 6) + rbit(M, 0xD7F2, 7) + rbit(M, 0xD803, 0) + rbit(M, 0xD803, 1));
    // used cut (:1547-1552)
    u32 used_cut2 = used_cut;
    if (!M.err && rd(M, 0xCD4D) == 61u) {
        wr(M, 0xCD4D, 0);
        used_cut2 += 1u;
    }
    // reward assembly (:1555-1600), Python's left-to-right float64 evaluation
    const double scale = A.reward_scale;
    const double start_menu = (double)((flags >> 3) & 1u) * 0.01;
    const double pokemon_menu = (double)((flags >> 4) & 1u) * 0.1;
    const double stats_menu = (double)((flags >> 5) & 1u) * 0.1;
    const double bag_menu = (double)((flags >> 6) & 1u) * 0.1;
    double cut_coords = 0.0;
    for (u32 i = 0; i < cutc_n; i++) cut_coords = cut_coords + ((cutc[i] >> 31) ? 10.0 : 0.001);
    u32 ntiles = 0;
    for (u32 i = 0; i < 8u; i++) ntiles += (u32)__builtin_popcount(rs[(RS_CUT_TILES + i) * np + e]);
    const double that_guy = ((start_menu + pokemon_menu) + stats_menu) + bag_menu;
    double s = (double)max_events + (double)bill_capt;
    s = s + scale * (double)seen_cnt;
    s = s + scale * (double)caught_cnt;
    s = s + scale * (double)moves_cnt;
    s = s + (double)bill_reward;
    s = s + (double)hm_reward;
    s = s + level_reward;
    s = s + 0.0;  // death_reward
    s = s + (double)badges_reward;
    s = s + total_healing;
    s = s + exploration;
    s = s + (double)cut_rew;
    s = s + that_guy / 2.0;
    s = s + cut_coords * 1.0;
    s = s + (double)ntiles * 1.0;
    s = s + tree * 0.6;
    s = s + (double)(dojo * 5);
    for (u32 t = 0; t < 5u; t++) s = s + (((flags >> (8u + t)) & 1u) ? 20.0 : 0.0);
    int evsum = 0;
    for (u32 k = 0; k < PK_NMON; k++) evsum += mon[k];
    s = s + (double)evsum;
    s = s + (double)(mon[4] + mon[5] + mon[6] + mon[7] + mon[8]);
    double reward = scale * s;
    if (!(flags & RSF_HAS_LAST)) {                   // :1604-1610
        rsd[RSD_LAST_REWARD * np + e] = 0.0;
        reward = 0.0;
        flags |= RSF_HAS_LAST;
    } else {
        const double nxt = reward;
        reward = reward - rsd[RSD_LAST_REWARD * np + e];
        rsd[RSD_LAST_REWARD * np + e] = nxt;
    }
    // render(): visited mask of the current map (:256-263)
    u32* mk = A.mask + (size_t)e * PK_MASK_WORDS;
    if (rs[RS_MASK_MAP * np + e] != map) {
        mask_rebuild(mk, tab, A.cap_log2, gen, map, rs[RS_RESET_POS * np + e]);
        rs[RS_MASK_MAP * np + e] = map;
    }
    mask_set(mk, r, c);

    // info telemetry (:1621-1704): built on done or every 10000th step; rare, so its extra peeks
    // stay off the common path.  Every numeric scalar of info["stats"] / info["reward"].
    if (!M.err && (done || time % 10000u == 0u)) {
        u32 lv[6], hi = 0;
        for (u32 k = 0; k < 6u; k++) { lv[k] = rd(M, k_party_level[k]); hi = max(hi, lv[k]); }
        // highest_pokemon_level = max(nonzero levels): for an empty party the reference raises
        // ValueError (max([]), :1672) after every state update of the step — PK_ERR_EMPTY_PARTY
        if (hi == 0u) M.err = PKE_EMPTY_PARTY;
        if (A.info && !M.err) {
            const u32 nb = badges_reward / 10u;
            const u32 d7b1 = rd(M, 0xD7B1);
            auto bcd = [](u32 v) { return 10u * ((v >> 4) & 0xFu) + (v & 0xFu); };
            const u32 money = 10000u * bcd(rd(M, 0xD347)) + 100u * bcd(rd(M, 0xD348)) + bcd(rd(M, 0xD349));
            double* o = A.info + e;
            u32 f = 0;
            auto put = [&](double v) { o[(size_t)(f++) * np] = v; };
            put((double)time); put((double)c); put((double)r); put((double)map); put((double)party_size);
            for (u32 k = 0; k < 6u; k++) put((double)lv[k]);
            put((double)lsum);                      // levels_sum (raw levels)
            put((double)deaths); put((double)deaths);  // deaths, deaths_per_episode (both reset, :1269, :1297)
            put((double)nb); put(0.0);              // badges, self.badge_count (never updated)
            for (u32 k = 1; k <= 6u; k++) put(nb >= k ? 1.0 : 0.0);
            put(0.0);                               // events = len(past_events_string) = 0 after reset (:1301)
            put((double)rs[RS_MAX_OPP * np + e]);
            put((double)rbit(M, 0xD7F1, 0));
            for (u32 b = 3; b <= 7u; b++) put((double)rbit(M, 0xD7F2, b));
            put((double)rbit(M, 0xD803, 0)); put((double)rbit(M, 0xD803, 1));
            put((double)party_size); put((double)hi); put((double)lsum); put((double)events); put((double)money);
            put(0.0);                               // seen_npcs_count
            put((double)seen_cnt); put((double)caught_cnt); put((double)moves_cnt);
            put(0.0);                               // hidden_obj_count
            put((double)(bill_reward / 5u)); put((double)hm_count); put((flags & RSF_CUT) ? 1.0 : 0.0);
            put((double)bill_capt / 5.0); put(cut_coords * 1.0); put((double)ntiles * 1.0);
            put(bag_menu); put(stats_menu); put(pokemon_menu); put(start_menu);
            put((double)used_cut2); put(0.0);       // used_cut, state_loaded_instead_of_resetting_in_game
            put((double)(d7b1 & 1u)); put((double)(3u * ((d7b1 >> 6) & 1u))); put((double)(3u * ((d7b1 >> 7) & 1u)));
            put(A.heat ? rsd[RSD_COORD * np + e] : __builtin_nan(""));   // coord = np.sum(counts_map)
            // info["reward"]
            put(reward); put((double)max_events); put(level_reward);
            put(0.006 * (double)rs[RS_MAX_OPP * np + e]); put(0.0);
            put((double)badges_reward); put((double)bill_reward); put((double)hm_reward);
            put(total_healing); put(exploration);
            put(scale * (double)seen_cnt); put(scale * (double)caught_cnt); put(scale * (double)moves_cnt);
            put((double)cut_rew); put(tree); put((double)dojo);
            for (u32 t = 0; t < 5u; t++) put(((flags >> (8u + t)) & 1u) ? 20.0 : 0.0);
            if (A.info_bits)
                for (u32 j = 0; j < PK_INFO_BITS_WORDS; j++) A.info_bits[(size_t)j * np + e] = mbits[j];
            if (A.info_flag) A.info_flag[e] = 1;
        }
    }

    rs[RS_FLAGS * np + e] = flags;
    rs[RS_SEEN_N * np + e] = seen_n;
    rs[RS_LAST_MAP1 * np + e] = last1;
    rs[RS_USED_CUT * np + e] = used_cut2;
    rs[RS_MAX_LEVEL * np + e] = max_level;
    rs[RS_MAX_EVENTS * np + e] = max_events;
    rs[RS_LAST_PARTY * np + e] = party_size;
    rs[RS_DEATHS * np + e] = deaths;
    rsd[RSD_TOTAL_HEALING * np + e] = total_healing;
    rsd[RSD_LAST_HP * np + e] = hp;
    rs[RS_ERR * np + e] = M.err;
    if (A.rew) A.rew[e] = M.err ? 0.0 : reward;
}

// ---------------------------------------------------------------------------------------------
// K5r (before the template reload): get_base_event_flags' D778 write (:1137-1138) and the
// reload decision (reload only on the first reset, :1241-1242, unless PK_F_RELOAD_ON_RESET)
__global__ void __launch_bounds__(256) pk_rreset_pre_kernel(PkRewardArgs A) {
    const u32 e = A.env0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= A.env1) return;
    const bool sel = !A.env_mask || A.env_mask[e];
    u8 rl = 0;
    if (sel) {
        RMem M;
        rmem_at(M, A.mem, e, A.ilv_sh);
        M.regs = A.regs;
        M.np = A.npad;
        M.env = e;
        M.err = 0;
        wr(M, 0xD778, rd(M, 0xD778) | 0x10u);
        rl = (A.reload_always || A.rs[RS_RESET_COUNT * A.npad + e] == 0u) ? 1 : 0;
    }
    A.reload[e] = rl;
}

// K5r (after the reload): the per-episode attributes of reset() and its three update_* calls
__global__ void __launch_bounds__(256) pk_rreset_post_kernel(PkRewardArgs A) {
    const u32 e = A.env0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= A.env1) return;
    if (A.env_mask && !A.env_mask[e]) return;
    const u32 np = A.npad;
    u32* rs = A.rs;
    RMem M;
    rmem_at(M, A.mem, e, A.ilv_sh);
    M.regs = A.regs;
    M.np = np;
    M.env = e;
    M.err = 0;
    u32 flags = rs[RS_FLAGS * np + e] & RSF_KEEP;
    const u32 keep_heat = rs[RS_HEAT_LAST * np + e];
    const u32 keep_count = rs[RS_RESET_COUNT * np + e];
    u32 gen = rs[RS_GEN * np + e];
    for (u32 f = 0; f < RS_NFIELDS; f++) rs[f * np + e] = 0;
    // a new episode tag for the seen set; clear the table when the tag wraps
    gen = gen % 255u + 1u;
    if (gen == 1u) {
        u32* tab = A.seen + (size_t)e * (1u << A.cap_log2);
        for (u32 i = 0; i < (1u << A.cap_log2); i++) tab[i] = 0;
    }
    rs[RS_GEN * np + e] = gen;
    rs[RS_HEAT_LAST * np + e] = keep_heat;
    rs[RS_RESET_COUNT * np + e] = keep_count + 1u;
    rs[RS_LAST_PARTY * np + e] = 1u;                 // self.last_party_size = 1
    A.rsd[RSD_LAST_REWARD * np + e] = 0.0;
    A.rsd[RSD_TOTAL_HEALING * np + e] = 0.0;
    A.rsd[RSD_LAST_HP * np + e] = 1.0;               // self.last_hp = 1.0
    A.regs[PK_R_TIME * np + e] = 0;                  // self.time = 0
    u32 last1 = 0;                                   // last_10_map_ids = zeros
    update_last_map(M, last1);
    rs[RS_LAST_MAP1 * np + e] = last1;
    const u32 ek = seen_map_check(M, last1, flags);
    rs[RS_ERR * np + e] = ek ? ek : M.err;
    // render() of reset: the reset position enters screen_memory (:1251-1254, :1334)
    const u32 r = rd(M, 0xD361), c = rd(M, 0xD362), map = min(rd(M, 0xD35E), 247u);
    rs[RS_RESET_POS * np + e] = r | (c << 8) | (map << 16) | (1u << 24);
    u32* mk = A.mask + (size_t)e * PK_MASK_WORDS;
    for (u32 i = 0; i < PK_MASK_WORDS; i++) mk[i] = 0;
    mask_set(mk, r, c);
    rs[RS_MASK_MAP * np + e] = map;
    rs[RS_FLAGS * np + e] = flags;
}

// ---------------------------------------------------------------------------------------------
// K3: obs (72, 80, 4) = screen[::2, ::2] x 3 channels + mask window centred on (r, c).
// One thread = 4 consecutive pixels (one 16-byte store); grid-stride over (env, row, quad).
// With a list (A.ocnt/A.oids: the envs a reset touched) only those envs are rebuilt.
__global__ void __launch_bounds__(256) pk_obs_kernel(PkRewardArgs A) {
    const u32 cnt = A.ocnt ? *A.ocnt : A.env1 - A.env0;
    const size_t total = (size_t)cnt * PK_OBS_H * (PK_OBS_W / 4u);
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        const u32 q = (u32)(t % (PK_OBS_W / 4u));
        const u32 y = (u32)((t / (PK_OBS_W / 4u)) % PK_OBS_H);
        const u32 k = (u32)(t / ((size_t)PK_OBS_H * (PK_OBS_W / 4u)));
        const u32 e = A.oids ? A.oids[k] : A.env0 + k;
        const int r = A.mem[pk_img_off(e, PK_P_WRAM + 0x1361u, A.ilv_sh)];
        const int c = A.mem[pk_img_off(e, PK_P_WRAM + 0x1362u, A.ilv_sh)];
        const u8* srow = A.screen + (size_t)e * PK_SCREEN + (size_t)(2u * y) * PK_COLS + 8u * q;
        const uint2 sp = *reinterpret_cast<const uint2*>(srow);
        const u32* mk = A.mask + (size_t)e * PK_MASK_WORDS;
        const int mr = r - 36 + (int)y;
        u32 out[4];
        for (u32 k = 0; k < 4u; k++) {
            const u32 grey = k < 2u ? ((sp.x >> (16u * k)) & 0xFFu) : ((sp.y >> (16u * (k - 2u))) & 0xFFu);
            const int mc = c - 40 + (int)(4u * q + k);
            u32 m = 0;
            if (mr >= 0 && mr <= 254 && mc >= 0 && mc <= 254) m = (mk[mr * 8 + (mc >> 5)] >> (mc & 31)) & 1u;
            out[k] = grey | (grey << 8) | (grey << 16) | ((m ? 0xFFu : 0u) << 24);
        }
        uint4 v;
        v.x = out[0]; v.y = out[1]; v.z = out[2]; v.w = out[3];
        *reinterpret_cast<uint4*>(A.obs + (size_t)e * PK_OBS_BYTES + (size_t)y * PK_OBS_W * 4u + 16u * q) = v;
    }
}

// bulk RAM gather/scatter for all envs: dense[e * len + i] <-> guest [addr, addr + len)
__global__ void __launch_bounds__(256) pk_ram_copy_kernel(uint8_t* mem, uint8_t* dense, u32 n, u32 sh, u32 phys0, u32 len,
                                                          u32 to_dense) {
    const size_t total = (size_t)((n + PK_LANES - 1) / PK_LANES) * PK_LANES * len;
    for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
        // lane fastest: consecutive threads touch consecutive interleaved bytes
        const u32 lane = (u32)(t % PK_LANES);
        const size_t rest = t / PK_LANES;
        const u32 i = (u32)(rest % len);
        const u32 gid = (u32)(rest / len);
        const u32 e = gid * PK_LANES + lane;
        if (e >= n) continue;
        uint8_t* p = mem + pk_img_off(e, phys0 + i, sh);
        if (to_dense) dense[(size_t)e * len + i] = *p;
        else *p = dense[(size_t)e * len + i];
    }
}

// seen set grown by pk_set_episode_params: every env's entries of its current episode (tag ==
// rs[RS_GEN]) re-inserted into the larger table (the new table is zeroed: older tags are dropped)
__global__ void pk_seen_rehash_kernel(const u32* old_tab, u32 old_lg, u32* new_tab, u32 new_lg, const u32* rs, u32 n, u32 np) {
    const u32 e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const u32 gen = rs[RS_GEN * np + e];
    const u32* src = old_tab + (size_t)e * (1u << old_lg);
    u32* dst = new_tab + (size_t)e * (1u << new_lg);
    u32 count = 0;
    for (u32 i = 0; i < (1u << old_lg); i++) {
        const u32 v = src[i];
        if (gen != 0u && (v >> 24) == gen) count += seen_insert(dst, new_lg, gen, v & 0xFFFFFFu, count) & 1u;
    }
}

// ---------------------------------------------------------------------------------------------
hipError_t pk_launch_seen_rehash(const u32* old_tab, u32 old_lg, u32* new_tab, u32 new_lg, const u32* rs, u32 n, u32 np,
                                 hipStream_t s) {
    hipLaunchKernelGGL(pk_seen_rehash_kernel, dim3((n + 255) / 256), dim3(256), 0, s, old_tab, old_lg, new_tab, new_lg, rs, n, np);
    return hipGetLastError();
}

hipError_t pk_launch_reward(const PkRewardArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pk_reward_kernel, dim3((a.env1 - a.env0 + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t pk_launch_rreset_pre(const PkRewardArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pk_rreset_pre_kernel, dim3((a.env1 - a.env0 + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t pk_launch_rreset_post(const PkRewardArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(pk_rreset_post_kernel, dim3((a.env1 - a.env0 + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t pk_launch_obs(const PkRewardArgs& a, hipStream_t s) {
    const size_t total = (size_t)(a.env1 - a.env0) * PK_OBS_H * (PK_OBS_W / 4u);
    const u32 grid = (u32)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
    hipLaunchKernelGGL(pk_obs_kernel, dim3(grid), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t pk_launch_ram_copy(uint8_t* mem, uint8_t* dense, u32 n, u32 sh, u32 phys0, u32 len, u32 to_dense, hipStream_t s) {
    const u32 ngroups = (n + PK_LANES - 1) / PK_LANES;
    const size_t total = (size_t)ngroups * PK_LANES * len;
    const u32 grid = (u32)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
    hipLaunchKernelGGL(pk_ram_copy_kernel, dim3(grid), dim3(256), 0, s, mem, dense, n, sh, phys0, len, to_dense);
    return hipGetLastError();
}
