/*
 * gbcore — CPU ORACLE (test infrastructure only; never linked into the product path).
 *
 * A plain-C restatement of the DMG emulator semantics that pokegym's hot path gets from
 * PyBoy 1.x (`setup.py:12` pins `pyboy<2.0.0`; PyBoy is a third-party Cython dependency
 * that is NOT vendored in /root/reference and NOT installed here).  What it restates:
 *   - PyBoy 1.x `Motherboard.tick()` frame loop with HALT fast-forward,
 *   - the SM83 CPU (`cpu.py` tick/interrupts + generated `opcodes.py` semantics),
 *   - the memory bus (`mb.getitem/setitem`), ROM-only and MBC3 (`cartridge` package),
 *   - LCD mode/LY/STAT timing (`lcd.py`), DIV/TIMA timer (`timer.py`),
 *   - joypad (`interaction.py`), instantaneous OAM DMA, sound regs not emulated,
 *   - the DMG scanline renderer (`renderer` in `lcd.py`),
 *   - savestate format v9 (layout pinned empirically on the 264 reference savestates,
 *     SURVEY.md §5).
 * and the pokegym call site that drives it: `pokegym/pyboy_binding.py:71-91`
 * (`run_action_on_emulator`: press, 24 ticks, release before tick 8, render only tick 24).
 *
 * PARITY STATUS:
 *   - savestate layout + PPU: pinned — the renderer reproduces all 264 frames embedded in the
 *     reference's savestates bit-exactly (tests/test_oracle_ppu.py).
 *   - CPU/timing trajectories vs PyBoy: UNPINNED — PyBoy and pokemon_red.gb are absent, the
 *     reference holds no recorded trajectory.  The HIP kernel is pinned to THIS restatement.
 */
#ifndef GBCORE_H
#define GBCORE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GB_STATE_V9_SIZE 142610u
#define GB_ROWS 144
#define GB_COLS 160

typedef struct gb gb_t;

/* joypad buttons (mirror the pyboy.utils.WindowEvent press/release pairs, pyboy_binding.py:7-38) */
enum {
    GB_BTN_RIGHT = 0, GB_BTN_LEFT = 1, GB_BTN_UP = 2, GB_BTN_DOWN = 3,
    GB_BTN_A = 4, GB_BTN_B = 5, GB_BTN_SELECT = 6, GB_BTN_START = 7
};

gb_t* gb_new(const uint8_t* rom, uint32_t rom_len);
void gb_free(gb_t* gb);
gb_t* gb_clone(const gb_t* gb);
/* post-boot DMG state (our own init; PyBoy would run its bundled boot ROM instead) */
void gb_power_on(gb_t* gb);
int gb_load_state(gb_t* gb, const uint8_t* buf, uint32_t len);
int gb_save_state(const gb_t* gb, uint8_t* buf, uint32_t len);

/* press (pressed=1) / release (pressed=0) a button: PyBoy send_input -> Interaction.key_event */
void gb_button(gb_t* gb, int button, int pressed);
void gb_set_rendering(gb_t* gb, int on);
/* one PyBoy frame (Motherboard.tick) */
void gb_tick(gb_t* gb);
/* pyboy_binding.run_action_on_emulator: action id per ACTIONS (pyboy_binding.py:40) */
void gb_run_action(gb_t* gb, int action, int frame_skip, int release_frame);
/* action -> button: 0 Down 1 Left 2 Right 3 Up 4 A 5 B 6 Start 7 Select; 8 = no press (extension) */
int gb_action_button(int action);

uint8_t gb_read(gb_t* gb, uint16_t addr);           /* PyBoy get_memory_value */
void gb_write(gb_t* gb, uint16_t addr, uint8_t v);  /* PyBoy set_memory_value */

const uint8_t* gb_screen_shades(const gb_t* gb);     /* 144*160 shade ids 0..3 */
const uint8_t* gb_wram(const gb_t* gb);              /* 8192 */
uint64_t gb_instr_count(const gb_t* gb);
uint64_t gb_frame_count(const gb_t* gb);
int gb_crashed(const gb_t* gb);                      /* illegal opcode hit */

/* Render the screen from a savestate's VRAM/OAM/LCD regs/per-line params (golden PPU check).
 * out: 144*160 shade ids. Returns 0 on success. */
int gb_render_from_state(const uint8_t* state, uint32_t len, uint8_t* out);

/* n independent envs, each run `steps` env-steps with action actions[s*n+e]; used as the CPU
 * baseline ("port") and by the parity tests. states_in: n*v9 buffers (or one shared if
 * shared_state). */
int gb_batch_run(const uint8_t* rom, uint32_t rom_len, const uint8_t* state, uint32_t state_len,
                 uint32_t n, uint32_t steps, const uint8_t* actions, int render_last,
                 uint8_t* states_out /* n*v9 or NULL */, uint8_t* screens_out /* n*144*160 or NULL */);

/* CPU baseline timing (single thread); returns seconds of the timed part. */
int gb_intensity(const uint8_t* rom, uint32_t rom_len, const uint8_t* state, uint32_t state_len,
                 uint32_t n, uint32_t warmup, uint32_t steps, uint32_t seed, uint64_t* out);
double gb_bench(const uint8_t* rom, uint32_t rom_len, const uint8_t* state, uint32_t state_len,
                uint32_t n, uint32_t warmup, uint32_t steps, uint32_t seed, uint64_t* instr_out);

#ifdef __cplusplus
}
#endif
#endif
