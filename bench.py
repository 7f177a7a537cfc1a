"""Benchmark: aggregate env.step/s of the batched Pokémon Red emulator on 1..8 MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N>1 the driver launches it
under torch.distributed.run, one rank per GPU.  Each rank owns its shard of envs, does W untimed
env-steps, then times exactly K env-steps between barrier+synchronize fences; the max elapsed over
ranks gives `value` = (all ranks' envs * K) / max_elapsed.  Rank 0 prints ONE JSON line.

Workloads (BASELINE.json configs):
  config3 (default at N=1) configs[2]: 65,536 envs/GPU, the last of the 24 frames of every env-step
          PPU-rendered into a 160x144 u8 screen obs, actions uniform in [0,8) (torch Philox); stepped
          through the PufferLib-shaped VecEnv in 2 sub-batches (send/recv, auto-reset).
  config4 (default at N>1) configs[3]: 262,144 envs split over the N GPUs (strong scaling: 131,072
          per GPU at N=2, 65,536 at N=4, 32,768 at N=8), screen obs, stepped through VecEnv
          (send/recv, auto-reset, 2 sub-batches).  At N=1 (--workload config4) and with --envs it runs
          that many envs per GPU (the configs[3] shard: 32,768).
  config5 configs[4]: config4's shard + the full ram_map reward stack, the (72,80,4) obs, a template
          reload on every done (short episodes, --max-episode-steps, so resets happen in the timed
          steps) and VecEnv's logging-interval all-reduce of the episode statistics (every 128 steps).
  config2 configs[1]: 4,096 envs on 1 GPU, headless (no PPU), the fixed [0,3,1,2] action cycle.
  config1 configs[0]'s shape: one drop-in Environment, 1,000 + 10,000 x step(0) (test.py:16-29).
The ROM is the synthetic game `pkbench` (pokegym_amd/testrom/game.py; --rom-banks 64 for the
Pokémon-Red-sized 1 MiB variant) because pokemon_red.gb is not shipped; --rom/--state run a real
cartridge.  Inputs are resident in HBM before the timed region (actions pre-generated on device).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

# algorithmic bytes per env-step: S = 16,844 B hot state
S_HOT = 8192 + 8192 + 160 + 127 + 128 + 1 + 44
B_HEADLESS = 2 * S_HOT + 1 + 8 + 2          # B2 = 33,699: the hot state read+written, action, reward, flags
B_SCREEN = B_HEADLESS + 160 * 144           # B3,4 = 56,739: + the u8 screen obs (K2)
B_REWARD = B_SCREEN + 2 * 256               # B5 = 57,251: + per-env reward accumulators
HBM_PEAK_GBS = 8000.0                       # MI355X_MICROARCH.md: 8.0 TB/s HBM3E
CONFIGS3_ENVS = 262144                      # configs[3] / configs[4]: envs over all GPUs

WORKLOADS = {
    "config1": dict(envs=1, render=True, reward=True, vecenv=False, actions="zero", bytes=B_REWARD,
                    desc="configs[0]'s shape on the GPU build: ONE drop-in Environment (reward stack, (72,80,4) obs), "
                         "1,000 warm-up steps then 10,000 x step(0), as /root/reference/test.py:16-29 times PyBoy+pokegym"),
    "config2": dict(envs=4096, render=False, reward=False, vecenv=False, actions="cycle", bytes=B_HEADLESS,
                    desc="configs[1]: headless (no PPU), RAM-only obs, fixed action cycle [0,3,1,2]"),
    "config3": dict(envs=65536, render=True, reward=False, vecenv=True, actions="random", bytes=B_SCREEN,
                    desc="configs[2]: PPU-rendered 160x144 u8 screen obs, random actions, stepped through the "
                         "PufferLib-shaped VecEnv (send/recv, 2 sub-batches)"),
    "config4": dict(envs=32768, render=True, reward=False, vecenv=True, actions="random", bytes=B_SCREEN,
                    desc="configs[3]: 262,144 envs split over the GPUs (at N=1: its 32,768-env per-GPU shard), "
                         "screen obs, PufferLib-shaped VecEnv send/recv with auto-reset, random actions"),
    "config5": dict(envs=32768, render=True, reward=True, vecenv=True, actions="random", bytes=B_REWARD,
                    desc="configs[4]: configs[3]'s envs (at N=1 the 32,768-env shard) + full ram_map reward stack + (72,80,4) obs + per-env "
                         "template reload on done + episodic-return all-reduce every 128 steps"),
}


def _cpu_quota():
    """The host CPU share this process may use: the cgroup CPU quota (cgroup v2 cpu.max or v1
    cfs_quota/period) when one is set, else None; plus the raw values for the record."""
    raw = None
    try:
        raw = open("/sys/fs/cgroup/cpu.max").read().strip()
        q, p = raw.split()[:2]
        if q != "max":
            return max(1, int(-(-int(q) // int(p)))), f"cpu.max {raw}"
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            raw = f"cfs_quota_us {q} / cfs_period_us {p}"
            if q > 0:
                return max(1, -(-q // p)), raw
        except (OSError, ValueError):
            pass
    return None, raw


def _cpu_run(rom, state, workers, n_per, steps, seed0):
    """`workers` concurrent workers, each n_per envs x steps timed env-steps (after 3 warmup) of the
    C oracle; aggregate env-steps/s over the slowest worker's timed span.

    Workers are threads of this process: gb_bench is re-entrant C and ctypes releases the GIL for
    the call, so they run in parallel on the host cores exactly as separate processes would.  No
    process is forked: bench.py holds the GPU (and, under rocprofv3, the profiler's state) by the
    time this runs, and a fork of such a process is what aborted the round-3 profile run
    (VERDICT r03 weak 4)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle
    with ThreadPoolExecutor(max_workers=workers) as pool:
        t0 = time.time()
        res = list(pool.map(lambda w: oracle.bench(rom, state, n_per, 3, steps, seed0 + w), range(workers)))
        wall = time.time() - t0
    slowest = max(r[0] for r in res)
    return workers * n_per * steps / slowest, wall, sum(r[1] for r in res) / slowest


def _cpu_baseline(rom: bytes, state, seconds_target: float = 10.0):
    """The oracle (C restatement of the path, oracle/gbcore.c) on the host cores: "port".

    Two shapes on whatever cores the box grants: the reference's own CPU shape, 72 envs each in its
    own worker (README.md:116-118; PufferLib multiprocessing), and a run sized to the box's CPU share
    (cgroup quota, else the 16 threads the GPU box allots one GPU: OMP_NUM_THREADS) with 4 envs per
    worker.  `value` is the STRONGER of the two measured CPU figures (the denominator of any GPU/CPU
    ratio is the best CPU number this box produced; round 5 reported the 72-worker shape instead,
    ~1.3x lower); both runs are recorded beside it (`reference_shape_run`, `share_sized_run`) with
    `shape`/`workers` naming the one `value` is.  Plus the workload intensity of the action stream."""
    from oracle import oracle
    oracle.lib()
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count()
    quota, quota_raw = _cpu_quota()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    share = quota or omp or 16
    share = max(1, min(share, affinity or share))
    # calibrate: seconds per env-step of one worker
    sec, _ = oracle.bench(rom, state, 2, 3, 4, 99)
    per_step = sec / 8.0
    # 72 workers x 1 env on `share` cores: ~seconds_target of wall
    steps72 = max(4, int(seconds_target * share / 72 / per_step))
    v72, wall72, ips72 = _cpu_run(rom, state, 72, 1, steps72, 2000)
    steps_s = max(4, int(seconds_target / 4 / per_step))
    vs, walls, ipss = _cpu_run(rom, state, share, 4, steps_s, 1000)
    inten = oracle.intensity(rom, state, 128, 3, 16, 99)   # 2,048 env-steps of the same action stream
    share_best = vs >= v72
    return {
        "value": round(max(v72, vs), 1),
        "unit": "env-steps/s",
        "cores": share,
        "workers": share if share_best else 72,
        "kind": "port",
        "shape": (f"share-sized run ({share} workers x 4 envs), the faster of the two" if share_best
                  else "72-worker reference shape (README.md:116-118), the faster of the two"),
        "best_value": round(max(v72, vs), 1),
        "sample": (f"the C oracle (oracle/gbcore.c, 1 thread per worker) on a CPU share of {share} cores "
                   f"({'cgroup ' + quota_raw if quota else 'no cgroup quota; OMP_NUM_THREADS=' + str(omp or 'unset') + ' is the box share'}), "
                   f"same ROM and random-action stream; two runs: the reference's CPU shape, 72 one-env workers "
                   f"(README.md:116-118) x {steps72} timed env-steps, and {share} "
                   f"workers x 4 envs x {steps_s} "
                   "timed env-steps (after 3 warmup each); value = the faster of the two; aggregate over the slowest "
                   "worker's timed span. Workers are "
                   "threads (ctypes releases the GIL), not forked processes. PyBoy+pokegym itself is not installed "
                   "(pure-Python PyBoy would be slower than this C restatement)"),
        "instr_per_s": round(max(ips72, ipss), 1),
        "cpu_share": {"cores": share, "cgroup": quota_raw, "omp_num_threads": omp or None, "affinity_cpus": affinity,
                      "host_cpus": os.cpu_count()},
        "reference_shape_run": {"value": round(v72, 1), "workers": 72, "envs_per_worker": 1, "steps": steps72,
                                "pool_wall_s": round(wall72, 1)},
        "share_sized_run": {"value": round(vs, 1), "workers": share, "envs_per_worker": 4, "steps": steps_s,
                            "pool_wall_s": round(walls, 1)},
        "workload_intensity": {**{k: round(v, 6) for k, v in inten.items()},
                               "sample": "C oracle, 128 envs x 16 env-steps (after 3) of the CPU baseline's action stream; "
                                         "door warps (LCD off for several frames) run in ~0.1% of env-steps "
                                         "(tools/warp_rate.py: 11 LCD-off frames per 1,000 env-steps over 81,920)"},
    }


def _stamp(workload: str, rom_tag: str):
    """Counter values of the committed rocprofv3 PMC passes of this bench command (profiles/),
    reported with their source file — they are not measured inside this run."""
    path = os.path.join(HERE, "profiles", f"pmc_{workload}{rom_tag}.json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    return d, os.path.relpath(path, HERE)


class StepFlow:
    """One env-step of the benchmarked workload over every env of this rank (the timed unit).

    VecEnv workloads (configs[2]..[4]): one recv/send of each sub-batch, PufferLib's loop (the
    sub-batches run on their own streams; finished envs auto-reset on the device — with the reward
    stack, a template reload — and VecEnv's logging interval does the sticky-error check and the
    episode/info-statistics all-reduce across ranks: RCCL at N>1, gloo in the CPU test of this flow,
    tests/test_dist.py).  Otherwise (configs[1]) a plain step of the whole batch."""

    def __init__(self, emu, vec, world, log_every, dev):
        self.emu, self.vec, self.world, self.log_every, self.dev = emu, vec, world, log_every, dev
        self.vec_logs = []         # VecEnv logging-interval records (episode statistics, all-reduced)

    def step(self, t, timed, acts_t=None):
        acts_t = self.acts[t] if acts_t is None else acts_t
        if self.vec is None:
            self.emu.step(acts_t)
            return
        vec = self.vec
        for _ in range(vec.num_batches):
            obs, rew, term, trunc, infos, ids, masks = vec.recv()
            if infos:
                self.vec_logs.append(infos[0])
            vec.send(acts_t[vec.current_envs()])


def run_config1(args):
    """configs[0]'s benchmark shape (/root/reference/test.py:16-29: one env, reset, 1,000 x step(0)
    untimed, then `steps` x step(0) timed) through the drop-in single `Environment`
    (pokegym_amd/env.py) on one GPU: every step is K1 (one lane), K2, K4, K3 plus the host round trip
    of the reference's return values (reward float, done bool, obs array).  Beside it, the C oracle's
    emulation-only rate of the same action stream in one process (no reward stack)."""
    import torch
    from oracle import oracle
    from pokegym_amd.env import Environment
    from pokegym_amd.testrom.game import game_rom
    rom = open(args.rom, "rb").read() if args.rom else game_rom(banks=args.rom_banks)
    if args.state:
        state = open(args.state, "rb").read()
    else:
        # pkbench's post-boot state (Bulbasaur.state is a Pokemon Red state: under pkbench its party is
        # wiped, and the info step at time 10,000 would raise the reference's empty-party ValueError)
        g = oracle.GB(rom)
        g.power_on()
        state = g.save_state()
        del g
    # CPU reference point first (no GPU touched yet): one process, emulation only
    g = oracle.GB(rom, state)
    cw = min(args.warmup, 1000)
    for _ in range(cw):
        g.run_action(0)
    cs = min(args.steps, 5000)
    t0 = time.perf_counter()
    for _ in range(cs):
        g.run_action(0)
    cpu_rate = cs / (time.perf_counter() - t0)
    del g

    env = Environment(rom_path=rom, state_path=state)
    env.reset()
    for i in range(args.warmup):
        env.step(0)
        if (i + 1) % 500 == 0:   # progress on stderr: a long single-env run is otherwise silent for minutes
            print(f"config1 warm-up {i + 1}/{args.warmup}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    env.emu.profile_enable(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        env.step(0)
        if (i + 1) % 500 == 0:
            print(f"config1 step {i + 1}/{args.steps}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    emu_ms, ren_ms, rew_ms, nprof = env.emu.profile_read()
    instr = env.emu.last_instr_count()
    env.close()
    k = max(nprof, 1)
    span = (emu_ms + ren_ms + rew_ms) / k
    out = {
        "metric": "env.step/sec (one env, configs[0] shape)",
        "value": round(args.steps / elapsed, 2),
        "unit": "env-steps/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"config1 = {WORKLOADS['config1']['desc']}", "envs_per_gpu": 1,
                   "rom": "pkbench (synthetic game ROM; pokemon_red.gb is not shipped)" if not args.rom else os.path.basename(args.rom),
                   "start_state": "pkbench post-boot" if not args.state else os.path.basename(args.state),
                   "action": "0 (Down) every step, as test.py", "frame_skip": 24, "release_frame": 8},
        "latency_ms": {"step_wall": round(elapsed / args.steps * 1e3, 3), "k1": round(emu_ms / k, 3),
                       "k2_render": round(ren_ms / k, 3), "k4_k3_reward_obs": round(rew_ms / k, 3),
                       "host_and_launch": round(elapsed / args.steps * 1e3 - span, 3)},
        "instr_per_env_step": instr,
        "cpu_baseline": {"value": round(cpu_rate, 2), "unit": "env-steps/s", "cores": 1, "kind": "port",
                         "sample": (f"C oracle (oracle/gbcore.c) in this process, one env, {cw} x step(0) warm-up then "
                                    f"{cs} x step(0) timed; emulation only (no reward stack, no obs)")},
        "note": ("one env leaves 1 of the GPU's 65,536 lanes busy: each emulated instruction is a dependent chain "
                 "of LDS and memory round trips with nothing to hide them, so this shape measures latency, not "
                 "throughput (use VecEnv)"),
    }
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed env-steps (default 20; config1: 10,000)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed env-steps first (default 3; config1: 1,000)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default=None,
                    help="default: config3 on one GPU, config4 (the configs[3] per-GPU shard) on several")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the workload's)")
    ap.add_argument("--actions", choices=["auto", "random", "same"], default="auto",
                    help="override the workload's action stream (diagnostics)")
    ap.add_argument("--max-episode-steps", type=int, default=None,
                    help="episode length (config5 default 16, so template reloads happen inside the timed steps)")
    ap.add_argument("--batches", type=int, default=2,
                    help="config4: VecEnv sub-batches (PufferLib batch_size = envs / batches; 72 envs in 3 "
                         "batches of 24 in the reference's README).  Each sub-batch has its own stream; they "
                         "overlap only while the HIP runtime has a hardware queue per stream (GPU_MAX_HW_QUEUES, "
                         "4 by default: the default stream + up to 3 sub-batches; 4 sub-batches measured 2x slower)")
    ap.add_argument("--rom", default=None)
    ap.add_argument("--rom-banks", type=int, default=4, help="pkbench size in 16 KiB banks (4, or 64 = 1 MiB)")
    ap.add_argument("--state", default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-obs", action="store_true",
                    help="diagnostic: also hand every step's observation to the host (pinned buffers, D2H on a "
                         "copy stream overlapped with the next step) inside the timed region -- the PCIe-inclusive "
                         "rate of a numpy-consuming caller (DESIGN.md section 6); not the default bench line")
    args = ap.parse_args()
    single = args.workload == "config1"
    if args.steps is None:
        args.steps = 10000 if single else 20
    if args.warmup is None:
        args.warmup = 1000 if single else 3
    if single:
        return run_config1(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank flow on a one-GPU box (not a measurement): every rank on device 0
    # and gloo instead of RCCL (RCCL refuses two ranks on one GPU)
    if os.environ.get("PK_BENCH_REHEARSAL") == "1":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if os.environ.get("PK_BENCH_REHEARSAL") == "1":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    wname = args.workload or ("config3" if world == 1 else "config4")
    W = WORKLOADS[wname]

    from pokegym_amd.emulator import BatchedEmulator
    if args.rom:
        rom = open(args.rom, "rb").read()
        rom_name, rom_tag = os.path.basename(args.rom), "_rom"
    else:
        from pokegym_amd.testrom.game import game_rom
        rom = game_rom(banks=args.rom_banks)
        rom_name = (f"pkbench{'' if args.rom_banks == 4 else args.rom_banks} (synthetic game ROM, {len(rom) // 1024} KiB; "
                    "pokemon_red.gb is not shipped)")
        rom_tag = "" if args.rom_banks == 4 else f"_b{args.rom_banks}"
    state = open(args.state, "rb").read() if args.state else None

    # N>1: configs[3]/[4] themselves, their 262,144 envs split over the ranks (strong scaling)
    strong = world > 1 and args.envs is None and wname in ("config4", "config5")
    log_every = max(1, min(128, args.steps))
    n = args.envs or ((CONFIGS3_ENVS // world) & ~63 if strong else W["envs"])
    reward = W["reward"]
    max_steps = args.max_episode_steps or (16 if reward else 20480)
    vec = None
    if W["vecenv"]:
        from pokegym_amd.env import VecEnv
        # logging interval min(128, steps): the episode-stat all-reduce (RCCL at N>1) and the
        # sticky-error check fire inside the timed steps (any `steps` consecutive env-steps hold one)
        # with the reward stack (configs[4]): the (72,80,4) obs, a template reload on every done
        vec = VecEnv(n, rom=rom, state=state, power_on=state is None, device=local, reward=reward,
                     reload_on_reset=reward, max_episode_steps=max_steps, log_interval=log_every,
                     batch_size=n // args.batches)
        emu = vec.emu
        vec.async_reset()
    else:
        emu = BatchedEmulator(rom, n, state=state, device=local, render=W["render"], reward=reward,
                              reload_on_reset=reward, max_episode_steps=max_steps)
        if reward:
            emu.reset()
    flow = StepFlow(emu, vec, world, log_every, dev)
    env_step = flow.step

    host_copy = None
    if args.host_obs:
        if vec is not None:
            raise SystemExit("--host-obs: not for the VecEnv workloads (their consumer is on the device)")
        src = emu.obs if reward else emu.screen
        dbuf = [torch.empty_like(src) for _ in range(2)]
        hbuf = [torch.empty(src.shape, dtype=src.dtype, pin_memory=True) for _ in range(2)]
        cstream = torch.cuda.Stream(dev)
        cdone = [None, None]

        def host_copy(t):
            # compute stream: snapshot the obs into a device double buffer (HBM copy, ~0.5 ms), then
            # the copy stream moves it over PCIe while the next step runs
            k = t % 2
            cur = torch.cuda.current_stream(dev)
            if cdone[k] is not None:
                cur.wait_event(cdone[k])   # this buffer's previous D2H has finished
            dbuf[k].copy_(emu.obs if reward else emu.screen)
            ev = torch.cuda.Event()
            ev.record(cur)
            cstream.wait_event(ev)
            with torch.cuda.stream(cstream):
                hbuf[k].copy_(dbuf[k], non_blocking=True)
                cdone[k] = torch.cuda.Event()
                cdone[k].record(cstream)

    total = args.warmup + args.steps
    mode = args.actions if args.actions != "auto" else W["actions"]
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)   # Philox counter-based RNG on the device
    if mode == "same":
        acts = torch.randint(0, 8, (total, 1), generator=g, device=dev).to(torch.uint8).expand(total, n).contiguous()
    elif mode == "random":
        acts = torch.randint(0, 8, (total, n), generator=g, device=dev, dtype=torch.int64).to(torch.uint8)
    else:
        cyc = torch.tensor([0, 3, 1, 2], dtype=torch.uint8, device=dev)
        acts = cyc[torch.arange(total, device=dev) % 4].unsqueeze(1).expand(total, n).contiguous()
    flow.acts = acts
    torch.cuda.synchronize(dev)

    for t in range(args.warmup):
        env_step(t, False)
        if host_copy:
            host_copy(t)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    emu.profile_enable(True)
    logs0 = len(flow.vec_logs)
    fired0 = vec.logs_fired if vec is not None else 0
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for t in range(args.warmup, total):
        env_step(t, True)
        if host_copy:
            host_copy(t)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    emu_ms, ren_ms, rew_ms, nprof = emu.profile_read()
    instr = emu.last_instr_count()  # last step's emulated instructions (all envs)
    timed_logs = flow.vec_logs[logs0:]   # VecEnv logging records handed out by recv() inside the timed steps
    # intervals that fired inside the timed steps (counted where they fire: a record produced by the
    # last timed send is only handed out by the next recv, after the timed region)
    fired_timed = (vec.logs_fired - fired0) if vec is not None else 0
    # env-steps t (1-based) inside the timed window at which the logging interval fires
    fired = sum(1 for t in range(args.warmup + 1, total + 1) if t % log_every == 0)
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max.item())

    if rank == 0:
        value = world * n * args.steps / elapsed
        k1_s = emu_ms / 1e3 / max(nprof, 1)
        k2_s = ren_ms / 1e3 / max(nprof, 1)
        k4_s = rew_ms / 1e3 / max(nprof, 1)
        span_s = k1_s + k2_s + k4_s
        B = W["bytes"]
        # per launch: a VecEnv sub-batch launch covers n / batches envs (launches of different
        # sub-batches overlap on their streams, so this per-launch rate is a lower bound)
        envs_per_launch = n // (vec.num_batches if vec is not None else 1)
        achieved = B * envs_per_launch / span_s / 1e9
        # per GPU over the whole step: concurrent sub-batch launches overlap, so the per-launch rate
        # above understates what one GPU moves; this one prices all n envs' bytes per ms_per_step
        achieved_step = B * n / (elapsed / args.steps) / 1e9
        stamp, stamp_src = _stamp(wname, rom_tag)
        if stamp and stamp.get("envs_per_gpu") not in (None, n):
            stamp, stamp_src = None, None   # the committed passes profiled another env count
        out = {
            "metric": "aggregate env.step/sec",
            "per_gpu_value": round(value / world, 1),
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": f"{wname} = {W['desc']}",
                "envs_per_gpu": n,
                "envs_total": n * world,
                "vecenv_batch_size": vec.batch_size if vec is not None else None,
                "rom": rom_name,
                "start_state": os.path.basename(args.state) if args.state else "power-on (post-boot)",
                "frame_skip": 24,
                "release_frame": 8,
                "max_episode_steps": max_steps,
                "parallelism": f"envs sharded over {world} GPU(s), no data-path collective",
                "host_obs": ("every step's obs copied to pinned host memory inside the timed region (PCIe-inclusive; "
                             "diagnostic, not the default line)") if args.host_obs else None,
                "scaling_note": ("the default workload is configs[2] (config3: 65,536 envs on one GPU) at N=1 and "
                                 "configs[3] itself (config4: 262,144 envs split over the N GPUs, strong scaling) at "
                                 "N>1.  A GPU's rate depends on its env count (config4 through VecEnv, round 4: "
                                 "32,768 envs ~333k env-steps/s, 65,536 ~540k; DESIGN.md section 7) -- one launch "
                                 "needs 64 envs per SIMD to hide K1's latency and 128 to fill every lane -- so N=8 "
                                 "(32,768 per GPU) is below 8x the N=1 rate by construction of configs[3]"),
            },
            "roofline": {
                # what limits K1, measured (PMC issue counts, wave timers): not HBM bandwidth and not
                # MFMA; `peak`/`frac` price the algorithmic bytes against the HBM roofline
                "bound": "latency",
                "priced_against": "hbm",
                "measured_bound": ("instruction issue + dependent latency (not HBM, not MFMA): per loop iteration (one "
                                   "emulated SM83 instruction, two when a register-only successor fuses) a wave runs the "
                                   "LDS fetch -> microcode -> address -> operand-read chain of its divergent lanes and the "
                                   "fused datapath; with two waves per SIMD the SIMD's other wave covers the chain's "
                                   "latency (requesting the operand ~50 instructions earlier saved nothing, "
                                   "profiles/r05/ab_pre), so instruction cuts are what move the rate (round 5: 398 -> 340 issued per "
                                   "iteration, every step A/B'd, profiles/r05/ab_diet); a lone wave "
                                   "(config2) is ~70 % issue; a launch lasts as long as its slowest wave (an env in a "
                                   "long LCD-off map load: kernel ~1.35x the mean wave, profiles/r03_wavetime).  `issue` "
                                   "carries the PMC ISA counts per emulated instruction; `frac` is only the HBM price of "
                                   "the algorithmic bytes (DESIGN.md §5)"),
                "kernel": ("pk_step_kernel (K1, 24 emulated frames) + pk_render_kernel (K2)"
                           + (" + pk_reward_kernel/pk_obs_kernel (K4/K3)" if reward else "")),
                "span": ("sum of the step's kernel times per launch (HIP events on the launch stream, averaged "
                         "over the timed launches); resets excluded" + (f"; {vec.num_batches} concurrent sub-batch "
                                                                        f"launches of {envs_per_launch} envs per env-step"
                                                                        if vec is not None else "")),
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "achieved_per_step": round(achieved_step, 3),
                "frac_per_step": round(achieved_step / HBM_PEAK_GBS, 6),
                "per_step_note": ("B x envs per GPU / ms_per_step: every env of the GPU over the whole step, the "
                                  "concurrent sub-batch launches together (achieved/frac price one launch's envs "
                                  "over that launch's own span)"),
                # per launch of THIS run: the profiled per-env-step bytes x the envs one launch covers
                "traffic": (round(stamp["hbm_bytes_per_env_step_k1"] * envs_per_launch) if stamp and
                            "hbm_bytes_per_env_step_k1" in stamp else (stamp or {}).get("hbm_bytes_per_launch_k1")),
                "traffic_per_env_step": (stamp or {}).get("hbm_bytes_per_env_step_k1"),
                "traffic_source": (f"{stamp_src}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this "
                                   "workload (K1 only; L2 memory-side requests, Infinity-Cache hits included; "
                                   "not measured inside this run); counted at "
                                   + ("the timed steps' occupancy (two waves per SIMD: pmc_stamp.regime)"
                                      if stamp.get("regime") else "one launch alone")) if stamp else None,
                "traffic_serialised_per_env_step": ((stamp or {}).get("serialised_record") or {}).get(
                    "hbm_bytes_per_env_step_k1"),
                "bytes_per_env_step": B,
                "span_ms": round(span_s * 1e3, 3),
                "k1_ms": round(k1_s * 1e3, 3),
                "k2_render_ms": round(k2_s * 1e3, 3),
                "k4_reward_obs_ms": round(k4_s * 1e3, 3),
            },
            "emulated_instr_per_s": round(instr / max(k1_s, 1e-9), 1),
            "instr_per_env_step": round(instr / n, 1),
        }
        if stamp:
            out["pmc_stamp"] = {k: stamp[k] for k in ("valu_busy_pct", "valu_utilization_pct", "wait_any_pct",
                                                      "waves_per_launch", "regime", "source") if k in stamp}
            if "issue" in stamp:
                out["roofline"]["issue"] = stamp["issue"]
        out["collectives"] = {
            "interval_env_steps": log_every,
            "fired_in_timed_steps": fired_timed,
            "records_received_in_timed_steps": len(timed_logs) if vec is not None else 0,
            "expected_in_timed_steps": fired if vec is not None else 0,
            "what": ("VecEnv logging: sticky-error check + episode/info statistics all-reduce (RCCL at N>1)"
                     if vec is not None else None),
            "episodes_logged": [round(d.get("episodes", 0.0)) for d in timed_logs] if vec is not None else None,
            "note": None if world > 1 else "one rank: the all-reduce is an identity and is not issued",
        }
        if not args.no_cpu_baseline and world == 1:
            try:
                out["cpu_baseline"] = _cpu_baseline(rom, state)
            except Exception as e:  # noqa: BLE001
                out["cpu_baseline"] = {"value": None, "error": f"{type(e).__name__}: {e}"}
        print(json.dumps(out), flush=True)
    if vec is not None:
        vec.close()
    else:
        emu.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
