/*
 * pokegym_amd.h — C ABI of the MI355X-native batched Pokémon Red env.step.
 *
 * Plain C: pointers and sizes only, no torch/HIP types.  `stream` arguments are hipStream_t
 * values passed as void* (NULL = the default stream).  Device buffers passed in are owned by the
 * caller (e.g. PyTorch-ROCm tensors' data_ptr()); buffers returned by pk_*_ptr() are owned by
 * the handle and live until pk_destroy.  Calls are stream-ordered and asynchronous unless noted.
 * One handle per GPU; a handle is not thread-safe.  Every function returns 0 on success or a
 * negative errno-style code; pk_last_error() describes the last failure of the calling thread.
 *
 * Each entry point replaces one piece of the reference's per-env Python/PyBoy path
 * (/root/reference/pokegym, file:line):
 *   pk_create        make_env + open_state_file        pyboy_binding.py:42-64, environment.py:121-122
 *   pk_reset         load_pyboy_state / Env.reset      pyboy_binding.py:66-69, environment.py:1233-1242
 *   pk_step          run_action_on_emulator + the      pyboy_binding.py:71-91,
 *                    per-step screen obs               environment.py:1336-1337, :268
 *   pk_peek          PyBoy get_memory_value (WRAM)     ram_map.py:1768-1770 (mem_val)
 *   pk_poke          PyBoy set_memory_value (WRAM)     ram_map.py:1772-1774 (write_mem)
 *   pk_snapshot      PyBoy save_state (v9 format)      environment.py:208-214
 *   pk_load_env      PyBoy load_state for one env      pyboy_binding.py:66-69
 *   pk_destroy       Env.close                         environment.py:412-413
 *   pk_obs_ptr       Env.render (72,80,4) observation  environment.py:256-274, :233-254
 *   pk_error_ptr     exceptions the reference raises   environment.py:739,744,568/580,1519,676
 *   pk_get_ram       per-env RAM views (RAM-only obs)  ram_map.py:1768-1770 (batched)
 *   pk_set_ram       per-env RAM writes                ram_map.py:1772-1774 (batched)
 * With PK_F_REWARD, pk_step also runs the reward stack of Environment.step
 * (environment.py:1338-1612) and pk_reset follows Environment.reset (:1233-1334).
 */
#ifndef POKEGYM_AMD_H
#define POKEGYM_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PK_ABI_VERSION 6
#define PK_STATE_V9_BYTES 142610u
#define PK_SCREEN_ROWS 144u
#define PK_SCREEN_COLS 160u

/* flags */
#define PK_F_RENDER 1u          /* rasterise the last frame of every step into the screen obs */
#define PK_F_REWARD 2u          /* reward stack + (72,80,4) obs + reference reset semantics */
#define PK_F_RELOAD_ON_RESET 4u /* reload the template state on EVERY reset (the reference
                                   reloads only on an env's first reset, environment.py:1241) */
#define PK_F_HEATMAP 8u         /* keep each env's 444x436 counts_map (environment.py:448, :648-679):
                                   int32, 774,336 B per env, persists across resets (PK_F_REWARD) */

/* per-env error codes (pk_error_ptr): where the reference's step/reset raises, the env stops
 * (reward 0, state frozen) and reports which exception the reference would have raised */
#define PK_ERR_NONE 0
#define PK_ERR_MAP_KEY 1        /* KeyError, MAP_ID_REF lookup (environment.py:739) */
#define PK_ERR_STUCK_ATTR 2     /* AttributeError, stuck_cnt read before assignment (:744) */
#define PK_ERR_MOVE_INDEX 3     /* IndexError, moves_obtained[move >= 0xA5] (:568, :580) */
#define PK_ERR_CUT_COORDS 4     /* UnboundLocalError, cut coords for an unknown facing (:1519) */
#define PK_ERR_HEATMAP_INDEX 5  /* IndexError, counts_map outside 444x436 (:676) */
#define PK_ERR_BUS_INDEX 6      /* IndexError, memory read past 0xFFFF (box scan, :574-578) */
#define PK_ERR_CAPACITY 7       /* device table full (no reference equivalent) */
#define PK_ERR_EMPTY_PARTY 8    /* ValueError, info["stats"]["highest_pokemon_level"] = max([]) (:1672) */

/* info telemetry record: the numeric scalars of info["stats"] (57) and info["reward"] (21),
 * environment.py:1621-1704, field order pokegym_amd/info.py FIELDS ("coord" is NaN without
 * PK_F_HEATMAP) */
#define PK_INFO_NFIELDS 79

typedef struct pk_config {
    uint32_t n_envs;             /* envs on this GPU */
    int32_t device;              /* HIP device ordinal */
    const uint8_t* rom;          /* host bytes of the cartridge ROM (MBC3 or ROM-only) */
    uint64_t rom_len;
    const uint8_t* state;        /* host bytes of a PyBoy v9 savestate, or NULL = power-on */
    uint64_t state_len;
    uint32_t frame_skip;         /* frames per env-step; pokegym uses 24 (pyboy_binding.py:72) */
    uint32_t release_frame;      /* button released before this frame; pokegym: 8 (:80) */
    uint32_t flags;              /* PK_F_* */
    uint32_t max_episode_steps;  /* truncation horizon; pokegym default 20480 (environment.py:1233) */
    double reward_scale;         /* reset(reward_scale=4.0) (environment.py:1233); 0 = 4.0 */
} pk_config;

typedef struct pk_handle pk_handle;

int pk_create(const pk_config* cfg, pk_handle** out);
void pk_destroy(pk_handle* h);
const char* pk_last_error(void);
int pk_abi_version(void);

/* Reset envs whose env_mask_dev[e] != 0 (device u8[n]; NULL = all).  Without PK_F_REWARD:
 * reload the template state and zero the step counter.  With PK_F_REWARD: Environment.reset —
 * D778 |= 0x10, template reload on the env's first reset only (or always with
 * PK_F_RELOAD_ON_RESET), fresh episode bookkeeping, and the reset observation in pk_obs_ptr(). */
int pk_reset(pk_handle* h, const uint8_t* env_mask_dev, void* stream);

/* One env-step for all envs.
 *   actions_dev : device u8[n], values 0..7 = Down Left Right Up A B Start Select
 *                 (pyboy_binding.py:40 ACTIONS); 8 = press nothing (extension).
 *   screen_dev  : optional device u8[n][144][160] copy of the grey screen (0xFF/0x99/0x55/0x00);
 *                 the handle's own persistent buffer is pk_screen_ptr().  NULL = no copy.
 *   rew_dev     : optional device f64[n]; the step reward (PK_F_REWARD; 0 otherwise).
 *   term_dev / trunc_dev : optional device u8[n]; time >= max_episode_steps
 *                 (environment.py:1612-1613: terminated = truncated = done). */
int pk_step(pk_handle* h, const uint8_t* actions_dev, uint8_t* screen_dev, double* rew_dev,
            uint8_t* term_dev, uint8_t* trunc_dev, void* stream);

/* Sub-batch forms (PufferLib batch_size < num_envs, README.md:116-118: 72 envs stepped 24 at a
 * time): the same step / reset restricted to envs [env0, env0 + count).  env0 is a multiple of
 * 64 (a 64-env image group); the end may be anywhere up to n.  All arrays stay full-size (device
 * u8/f64[n]); only the range's elements are read or written, so disjoint ranges may run
 * concurrently on different streams (each range has its own reset lists).  A range that ends
 * inside a group leaves the rest of that group untouched; a caller that steps those envs
 * concurrently in another range cannot (no range starts inside a group), so sub-batches of any
 * size are laid out one per group-aligned slot (pokegym_amd VecEnv pads 24-env sub-batches to 64). */
int pk_step_range(pk_handle* h, uint32_t env0, uint32_t count, const uint8_t* actions_dev, double* rew_dev,
                  uint8_t* term_dev, uint8_t* trunc_dev, void* stream);
int pk_reset_range(pk_handle* h, uint32_t env0, uint32_t count, const uint8_t* env_mask_dev, void* stream);

/* Environment.reset(max_episode_steps, reward_scale) (environment.py:1233, :1258-1259): set the
 * episode length and reward scale for the following steps (all envs of the handle).  Synchronous
 * when the seen-coordinate set must grow for a longer episode (it restarts empty then); call it
 * before the reset it belongs to. */
int pk_set_episode_params(pk_handle* h, uint32_t max_episode_steps, double reward_scale);

/* Rasterise every env's 144 latched scanlines (the per-line SCX/SCY/WX/WY/tile-data latches that
 * pk_create / pk_load_env restore from a v9 savestate, or that the last rendered frame latched)
 * into the screen with K2, the HIP renderer of pk_step — PyBoy's renderer.scanline over a loaded
 * state (the reference's 264 savestate frames pin it). Stream-ordered. */
int pk_render_latched(pk_handle* h, void* stream);

/* device pointer to the persistent u8[n][144][160] grey screen */
uint8_t* pk_screen_ptr(pk_handle* h);
/* device pointer to the u8[n][72][80][4] observation (PK_F_REWARD), updated by pk_step/pk_reset */
uint8_t* pk_obs_ptr(pk_handle* h);
/* device pointer to u32[n] PK_ERR_* codes (PK_F_REWARD), sticky until the env's next reset */
const uint32_t* pk_error_ptr(pk_handle* h);
/* device pointers to the info telemetry of the last pk_step (PK_F_REWARD).  info_flag u8[n] = 1
 * where the reference's step built its info dict (done or time % 10000 == 0, environment.py:1621);
 * for those envs info f64[PK_INFO_NFIELDS][npad] (field-major, env stride = npad, the padded
 * env count: pk_info_stride) holds the record.  Replaces the info dict of Environment.step. */
const double* pk_info_ptr(pk_handle* h);
const uint8_t* pk_info_flag_ptr(pk_handle* h);
uint32_t pk_info_stride(const pk_handle* h);
/* device pointer to u32 [5][stride] event-monitor bits of the info step (ram_map_leanke.py
 * monitor_*_events, 130 bits in reward_tables.MONITORS order): the detailed_rewards_* and
 * *_events_aggregate dicts of the reference's info (environment.py:1706-1808) */
const uint32_t* pk_info_bits_ptr(pk_handle* h);
/* device pointer to the int32 [n][444][436] counts_map of every env (PK_F_HEATMAP), null without it */
int32_t* pk_heatmap_ptr(pk_handle* h);

/* Stream-ordered bulk RAM access for all envs: dense_dev[e * len + i] <-> guest address
 * addr + i of env e.  RAM regions only (0xC000-0xFDFF incl. echo, 0xFF80-0xFFFE). */
int pk_get_ram(pk_handle* h, uint16_t addr, uint32_t len, uint8_t* dense_dev, void* stream);
int pk_set_ram(pk_handle* h, uint16_t addr, uint32_t len, const uint8_t* dense_dev, void* stream);
uint32_t pk_num_envs(const pk_handle* h);

/* Synchronous host-side accessors (parity tests, reward host mirrors, debugging). */
int pk_peek(pk_handle* h, uint32_t env, uint16_t addr, uint32_t len, uint8_t* host_out);
int pk_poke(pk_handle* h, uint32_t env, uint16_t addr, uint32_t len, const uint8_t* host_in);
int pk_snapshot(pk_handle* h, uint32_t env, uint8_t* host_v9, uint64_t len);
int pk_load_env(pk_handle* h, uint32_t env, const uint8_t* host_v9, uint64_t len);
/* v9 savestates of envs [env0, env0 + count) into host_v9 (count * PK_STATE_V9_BYTES bytes,
 * env-major): the bulk form of pk_snapshot for whole-batch parity checks (synchronous) */
int pk_snapshot_range(pk_handle* h, uint32_t env0, uint32_t count, uint8_t* host_v9, uint64_t len);

/* Emulated instructions executed by the last pk_step, summed over envs (synchronous). */
int pk_last_instr_count(pk_handle* h, uint64_t* out);

/* The K1 launch shape pk_step_range(h, env0, count, ...) takes (host-side, no GPU work):
 * out[0] = 1 for the small-LDS kernel, out[1] = envs per wave, out[2] = threads per workgroup,
 * out[3] = 1 for the wave-priority variant, out[4] = 1 for the every-bank-staged (ALL) instance.
 * Lets parity tests assert that they run the benchmarked launch. */
int pk_launch_shape(pk_handle* h, uint32_t env0, uint32_t count, uint32_t* out5);

/* Kernel timing with HIP events recorded on the step's stream around K1 (emulate), K2 (render)
 * and K4+K3 (reward + obs) of every pk_step while enabled.  pk_profile_read synchronises,
 * returns the summed milliseconds and the number of profiled steps since the last read, and
 * resets the sums. */
int pk_profile_enable(pk_handle* h, int on);
int pk_profile_read(pk_handle* h, double* emulate_ms, double* render_ms, double* reward_ms, uint64_t* steps);

#ifdef __cplusplus
}
#endif
#endif
