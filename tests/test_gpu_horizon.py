"""Long-horizon parity: the HIP emulator vs the oracle over 10,000 scripted env-steps.

BASELINE.json's north_star asks for bit-exact WRAM over 10k scripted steps, and the reference's
only benchmark is 10,000 x step(0) (/root/reference/test.py:16-29).  Timing bugs (DIV-mixing RNG,
folded LCD events, HALT skip-ahead, fused instruction pairs) grow with the horizon, so this
compares the WHOLE machine state (v9 savestate digest: WRAM, VRAM, OAM, HRAM, IO, CPU/LCD/timer/
MBC registers, clocks, the rendered screen) every 100 env-steps along 64 trajectories of 10,000
steps each from power-on: trajectory 0 presses Down every step (test.py's a_t = 0), trajectory 1
the [0,3,1,2] cycle of configs[1], trajectories 2..63 seeded random presses 0..8 (8 = no button).

The 10,000 steps of a trajectory are split into 20 segments of 500 that run side by side in one
1,280-env launch: segment k starts from the oracle's own v9 state at step 500k (pk_load_env) —
so the device is checked over every step of the 10k horizon, each segment a continuous run of
500 device steps, while the wall time is that of 500 steps.  Segment 0 starts from power-on on
both sides; the whole state is compared every 100 steps.  The run is repeated for each K1 launch
shape the benchmark launches (SHAPES): the small-LDS kernel pk_step_kernel_small at 32 and 16 envs
per wave (what the VecEnv sub-batches of configs[2] and configs[3]/[4] run) and the 512-thread
workgroups with the wave-priority kernel, pk_step_kernel<true>, at 32 envs per wave (whole-handle
launches), and the auto-picked shape of a 1,280-env handle, which is configs[1]'s 4,096-env launch
(256-thread workgroups, one 32-env wave per SIMD).  Both K1 instances are covered: the 512-thread shape stages all four pkbench banks (the
ALL instance), the small kernel's two slots do not (bank 3 runs from the global ROM), and
test_horizon_64_bank_rom runs the 6-slot kernel's unstaged-bank instance.  PK_HORIZON_EXTENDED=1
adds the shape no benchmark launches any more (512-thread workgroups of 16-env waves) — not part
of the driver's suite.

PK_HORIZON_EXTENDED=1 also runs test_horizon_10k_continuous_small_l32: the 64 trajectories as one
continuous 10,000-step run in the headline's kernel shape, compared every 500 steps.

test_horizon_65536_envs runs configs[2]'s own launch (65,536 envs) continuously for 240 steps and
compares one env of every workgroup with the oracle."""
import os

import numpy as np
import pytest

from oracle import oracle
from tests import oracle_pool as OP

pytestmark = pytest.mark.gpu

TOTAL, SEGS, EVERY, NTRAJ = 10000, 20, 100, 64
SEG = TOTAL // SEGS
PARTS = SEG // EVERY
# K1 launch shapes: (PK_WAVE_LANES, PK_K1_BLOCK, PK_K1_SMALL); None = what the handle picks.
# small_*: the small-LDS kernel the VecEnv sub-batches of configs[2]..[4] run (round 4), forced on
# the whole 1,280-env launch in its 256-thread workgroups
# "auto" at 1,280 envs is configs[1]'s launch (4,096-env handles: 256-thread workgroups, one 32-env
# wave per SIMD, no priority).
SHAPES = {"small_l32": ("32", "256", "1"), "small_l16": ("16", "256", "1"), "wg512_l32": ("32", "512", None),
          "auto": (None, None, None)}
if os.environ.get("PK_HORIZON_EXTENDED") == "1":
    SHAPES.update({"wg512_l16": ("16", "512", None)})
SHAPE_VARS = ("PK_WAVE_LANES", "PK_K1_BLOCK", "PK_K1_SMALL")


def horizon_actions(total=TOTAL, ntraj=NTRAJ) -> np.ndarray:
    a = np.random.default_rng(10000).integers(0, 9, (total, ntraj), dtype=np.uint8)
    a[:, 0] = 0
    a[:, 1] = np.array([0, 3, 1, 2], np.uint8)[np.arange(total) % 4]
    return a


def _with_shape(shape, fn):
    """Call fn() with the K1 shape environment of `shape` (read by pk_create)."""
    old = {k: os.environ.get(k) for k in SHAPE_VARS}
    try:
        for k, v in zip(SHAPE_VARS, SHAPES[shape]):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def oracle_horizon():
    from pokegym_amd.testrom.game import game_rom
    rom = game_rom()
    actions = horizon_actions()
    with OP.pool() as ex:
        dig, keep = OP.trajectories(ex, rom, None, actions, every=EVERY, keep_every=SEG, chunk=4)
    return rom, actions, dig, keep


@pytest.fixture(scope="module", params=list(SHAPES))
def horizon(request, oracle_horizon):
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    rom, actions, dig, keep = oracle_horizon
    emu = _with_shape(request.param, lambda: BatchedEmulator(rom, SEGS * NTRAJ, render=True))
    for k in range(1, SEGS):
        for j in range(NTRAJ):
            emu.load_env(k * NTRAJ + j, keep[(k, j)])
    # device action table: env k*64+j at local step t plays actions[k*SEG + t, j]
    table = np.concatenate([actions[k * SEG:(k + 1) * SEG] for k in range(SEGS)], axis=1)
    st = {"emu": emu, "acts": torch.from_numpy(np.ascontiguousarray(table)).to(emu.device), "dig": dig, "t": 0,
          "ok": True, "shape": request.param}
    yield st
    emu.close()


@pytest.mark.parametrize("part", range(PARTS))
def test_horizon_10k_segments(horizon, part):
    import torch
    st = horizon
    if not st["ok"] or st["t"] != part * EVERY:
        pytest.skip("an earlier part of the horizon failed")
    emu, acts = st["emu"], st["acts"]
    st["ok"] = False
    for t in range(part * EVERY, (part + 1) * EVERY):
        emu.step(acts[t])
    torch.cuda.synchronize()
    st["t"] = (part + 1) * EVERY
    got = oracle.state_digests(emu.snapshot_range(0, emu.n)).reshape(SEGS, NTRAJ)
    bad = []
    for k in range(SEGS):
        step = k * SEG + (part + 1) * EVERY               # global env-step of this checkpoint
        want = st["dig"][step // EVERY - 1]
        for j in np.nonzero(got[k] != want)[0]:
            bad.append((int(step), int(j)))
    assert not bad, f"[{st['shape']}] {len(bad)} (step, trajectory) checkpoints differ: {bad[:8]}"
    st["ok"] = True


@pytest.mark.skipif(os.environ.get("PK_HORIZON_EXTENDED") != "1",
                    reason="~5 min of GPU time: PK_HORIZON_EXTENDED=1 (one recorded run per kernel, profiles/)")
def test_horizon_10k_continuous_small_l32(oracle_horizon):
    """The 64 trajectories as ONE continuous 10,000-step device run (no oracle state ever loaded) in
    the headline's kernel shape — the small-LDS K1 with 32-env waves in 256-thread workgroups, as
    the VecEnv sub-batches of configs[2] run — the whole v9 state compared with the oracle every 500
    steps.  (K1 recomputes every lane-cached value — the pending-interrupt bit, the tick limit, the
    prefetch, the HRAM code mirror, the ROM-bank slot — from the stored state at the entry of every
    launch, i.e. every env-step, so the segmented form above sees the same kernel entries; this run
    also rules out drift in anything carried across launches.)"""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    rom, actions, dig, _ = oracle_horizon
    emu = _with_shape("small_l32", lambda: BatchedEmulator(rom, NTRAJ, render=True))
    assert emu.launch_shape()["small"] and emu.launch_shape()["wave_lanes"] == 32
    acts = torch.from_numpy(np.ascontiguousarray(actions)).to(emu.device)
    bad = []
    for t in range(TOTAL):
        emu.step(acts[t])
        if (t + 1) % 500 == 0:
            torch.cuda.synchronize()
            got = oracle.state_digests(emu.snapshot_range(0, NTRAJ))
            bad += [(t + 1, int(j)) for j in np.nonzero(got != dig[(t + 1) // EVERY - 1])[0]]
            print(f"continuous small_l32: step {t + 1}, {len(bad)} differing checkpoints so far", flush=True)
            if bad:
                break
    emu.close()
    assert not bad, f"{len(bad)} (step, trajectory) checkpoints differ: {bad[:8]}"


def test_horizon_65536_envs():
    """configs[2]'s benchmarked launch (65,536 envs: 512-thread workgroups, 32-env waves, the
    wave-priority kernel) stepped continuously for 240 random-action steps; one env of every
    workgroup (a different lane position in each) is compared with the oracle every 80 steps."""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    rom, n, steps, every = game_rom(), 65536, 240, 80
    per_wg = 256                                     # 8 waves x 32 envs per 512-thread workgroup
    sample = np.array([g * per_wg + (g * 37) % per_wg for g in range(n // per_wg)])
    actions = np.random.default_rng(240).integers(0, 8, (steps, n), dtype=np.uint8)
    with OP.pool() as ex:
        futs = [(e0, ex.submit(OP._trajectory, rom, None, np.ascontiguousarray(actions[:, sample[e0:e0 + 8]]),
                               every, steps)) for e0 in range(0, len(sample), 8)]
        emu = BatchedEmulator(rom, n, render=True)
        acts = torch.from_numpy(actions).to(emu.device)
        got = np.zeros((steps // every, len(sample)), np.uint64)
        for t in range(steps):
            emu.step(acts[t])
            if (t + 1) % every == 0:
                torch.cuda.synchronize()
                st = np.stack([emu.snapshot_range(int(e), 1)[0] for e in sample])
                got[(t + 1) // every - 1] = oracle.state_digests(st)
        emu.close()
        want = np.zeros_like(got)
        for e0, f in futs:
            d, _ = f.result()
            want[:, e0:e0 + d.shape[1]] = d
    bad = [(int((k + 1) * every), int(sample[j])) for k, j in zip(*np.nonzero(got != want))]
    assert not bad, f"{len(bad)} (step, env) checkpoints differ: {bad[:8]}"


def test_horizon_64_bank_rom():
    """The 1 MiB pkbench layout (overworld engine in 60 unstaged switchable banks: global-ROM fetch
    and reads, Bankswitch every frame) over 2,000 scripted steps: 64 trajectories in 16 segments of
    125 steps run side by side, whole v9 state compared with the oracle at every segment end."""
    import torch
    from pokegym_amd.emulator import BatchedEmulator
    from pokegym_amd.testrom.game import game_rom
    rom = game_rom(64)
    total, segs, ntraj = 2000, 16, 64
    seg = total // segs
    actions = horizon_actions(total, ntraj)
    with OP.pool() as ex:
        dig, keep = OP.trajectories(ex, rom, None, actions, every=seg, keep_every=seg, chunk=4)
    emu = BatchedEmulator(rom, segs * ntraj, render=True)
    for k in range(1, segs):
        for j in range(ntraj):
            emu.load_env(k * ntraj + j, keep[(k, j)])
    table = np.concatenate([actions[k * seg:(k + 1) * seg] for k in range(segs)], axis=1)
    acts = torch.from_numpy(np.ascontiguousarray(table)).to(emu.device)
    for t in range(seg):
        emu.step(acts[t])
    torch.cuda.synchronize()
    got = oracle.state_digests(emu.snapshot_range(0, emu.n)).reshape(segs, ntraj)
    emu.close()
    bad = [(k, int(j)) for k in range(segs) for j in np.nonzero(got[k] != dig[k])[0]]
    assert not bad, f"{len(bad)} (segment, trajectory) states differ: {bad[:8]}"
