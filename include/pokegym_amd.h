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
 */
#ifndef POKEGYM_AMD_H
#define POKEGYM_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PK_ABI_VERSION 1
#define PK_STATE_V9_BYTES 142610u
#define PK_SCREEN_ROWS 144u
#define PK_SCREEN_COLS 160u

/* flags */
#define PK_F_RENDER 1u /* rasterise the last frame of every step into the screen obs */

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
} pk_config;

typedef struct pk_handle pk_handle;

int pk_create(const pk_config* cfg, pk_handle** out);
void pk_destroy(pk_handle* h);
const char* pk_last_error(void);
int pk_abi_version(void);

/* Reset envs whose env_mask_dev[e] != 0 (device u8[n]; NULL = all) to the template state and
 * zero their step counters. */
int pk_reset(pk_handle* h, const uint8_t* env_mask_dev, void* stream);

/* One env-step for all envs.
 *   actions_dev : device u8[n], values 0..7 = Down Left Right Up A B Start Select
 *                 (pyboy_binding.py:40 ACTIONS); 8 = press nothing (extension).
 *   screen_dev  : optional device u8[n][144][160] copy of the grey screen (0xFF/0x99/0x55/0x00);
 *                 the handle's own persistent buffer is pk_screen_ptr().  NULL = no copy.
 *   rew_dev     : optional device f64[n]; reward (0 until the reward stack is enabled).
 *   term_dev / trunc_dev : optional device u8[n]; time >= max_episode_steps
 *                 (environment.py:1612-1613: terminated = truncated = done). */
int pk_step(pk_handle* h, const uint8_t* actions_dev, uint8_t* screen_dev, double* rew_dev,
            uint8_t* term_dev, uint8_t* trunc_dev, void* stream);

/* device pointer to the persistent u8[n][144][160] grey screen */
uint8_t* pk_screen_ptr(pk_handle* h);
uint32_t pk_num_envs(const pk_handle* h);

/* Synchronous host-side accessors (parity tests, reward host mirrors, debugging). */
int pk_peek(pk_handle* h, uint32_t env, uint16_t addr, uint32_t len, uint8_t* host_out);
int pk_poke(pk_handle* h, uint32_t env, uint16_t addr, uint32_t len, const uint8_t* host_in);
int pk_snapshot(pk_handle* h, uint32_t env, uint8_t* host_v9, uint64_t len);
int pk_load_env(pk_handle* h, uint32_t env, const uint8_t* host_v9, uint64_t len);

/* Emulated instructions executed by the last pk_step, summed over envs (synchronous). */
int pk_last_instr_count(pk_handle* h, uint64_t* out);

/* Kernel timing with HIP events recorded on the step's stream around K1 (emulate) and K2
 * (render) of every pk_step while enabled.  pk_profile_read synchronises, returns the summed
 * milliseconds and the number of profiled steps since the last read, and resets the sums. */
int pk_profile_enable(pk_handle* h, int on);
int pk_profile_read(pk_handle* h, double* emulate_ms, double* render_ms, uint64_t* steps);

#ifdef __cplusplus
}
#endif
#endif
