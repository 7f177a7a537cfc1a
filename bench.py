"""Benchmark: aggregate env.step/s of the batched Pokémon Red emulator on 1..8 MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N>1 the driver launches it
under torch.distributed.run, one rank per GPU.  Each rank owns `--envs` emulators (weak scaling),
does W untimed env-steps, then times exactly K env-steps between barrier+synchronize fences; the
max elapsed over ranks gives `value` = (N * envs * K) / max_elapsed.  Rank 0 prints ONE JSON line.

Workload (BASELINE.json configs[2], per GPU): 65,536 envs, the last of the 24 frames of every
env-step PPU-rendered into a 160x144 u8 screen obs, actions uniform in [0,8) from a counter-based
(Philox) RNG.  The ROM is the synthetic game `pkbench` (pokegym_amd/testrom/game.py) because
pokemon_red.gb is not shipped; pass `--rom path --state path` to run a real cartridge.
Inputs are resident in HBM before the timed region (actions pre-generated on device).
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
B_HEADLESS = 2 * S_HOT + 1 + 8 + 2          # 33,699: K1 reads+writes the hot state, action, reward, flags
B_SCREEN = B_HEADLESS + 160 * 144           # 56,739: + the u8 screen obs (K2)
B_REWARD = B_SCREEN + 2 * 256               # 57,251: + per-env reward accumulators (config 5)
HBM_PEAK_GBS = 8000.0                       # MI355X_MICROARCH.md: 8.0 TB/s HBM3E


def _cpu_baseline(rom: bytes, state, seconds_target: float = 12.0):
    """The oracle (C restatement of the path, oracle/gbcore.c) on the host cores: "port"."""
    import multiprocessing as mp
    from oracle import oracle
    oracle.lib()
    workers = int(os.environ.get("PK_CPU_BASELINE_PROCS", "16"))
    # calibrate: one short single-thread run sizes the per-worker sample to ~seconds_target/2
    sec, _ = oracle.bench(rom, state, 2, 3, 4, 99)
    per_step = sec / 8.0
    steps = max(4, int(seconds_target / 2.0 / per_step / 4))
    n_per = 4
    ctx = mp.get_context("fork")
    with ctx.Pool(workers) as pool:
        t0 = time.time()
        res = pool.starmap(oracle.bench, [(rom, state, n_per, 3, steps, 1000 + w) for w in range(workers)])
        wall = time.time() - t0
    total_steps = workers * n_per * steps
    slowest = max(r[0] for r in res)
    return {
        "value": round(total_steps / slowest, 1),
        "unit": "env-steps/s",
        "cores": workers,
        "kind": "port",
        "sample": (f"{workers} processes x {n_per} envs x {steps} timed env-steps (after 3 warmup) of the same "
                   f"ROM/workload on the C oracle (oracle/gbcore.c, 1 thread/process); aggregate over the slowest "
                   f"process's timed span; pool wall {wall:.1f}s; PyBoy+pokegym itself is not installed"),
        "instr_per_s": round(sum(r[1] for r in res) / slowest, 1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--workload", choices=["config3", "config2", "config5"], default="config3",
                    help="config3: rendered screen obs + random actions; config2: headless, fixed action cycle; "
                         "config5: config3 + reward stack + (72,80,4) obs + per-env reset on done + stats all-reduce")
    ap.add_argument("--actions", choices=["auto", "random", "same"], default="auto",
                    help="override the workload's action stream (diagnostics)")
    ap.add_argument("--rom", default=None)
    ap.add_argument("--state", default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from pokegym_amd.emulator import BatchedEmulator
    if args.rom:
        rom = open(args.rom, "rb").read()
        rom_name = os.path.basename(args.rom)
    else:
        from pokegym_amd.testrom.game import game_rom
        rom = game_rom()
        rom_name = "pkbench (synthetic game ROM; pokemon_red.gb is not shipped)"
    state = open(args.state, "rb").read() if args.state else None

    render = args.workload in ("config3", "config5")
    reward = args.workload == "config5"
    n = args.envs
    emu = BatchedEmulator(rom, n, state=state, device=local, render=render, reward=reward,
                          reload_on_reset=reward)
    if reward:
        emu.reset()
    ep_ret = torch.zeros(n, dtype=torch.float64, device=dev)
    stats = torch.zeros(2, dtype=torch.float64, device=dev)  # [sum of episodic returns, episodes]

    def env_step(t):
        obs, rew, term, trunc = emu.step(acts[t])
        if reward:
            # per-env reload of the template state on done, episodic-return bookkeeping, and the
            # RCCL all-reduce of the episode statistics every 128 steps (configs[4])
            d = term.to(torch.float64)
            ep_ret.add_(rew)
            stats[0] += (ep_ret * d).sum()
            stats[1] += d.sum()
            ep_ret.mul_(1.0 - d)
            emu.reset(term)
            if world > 1 and t % 128 == 127:
                dist.all_reduce(stats)
    total = args.warmup + args.steps
    if args.actions == "same":
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + rank)
        acts = torch.randint(0, 8, (total, 1), generator=g, device=dev).to(torch.uint8).expand(total, n).contiguous()
    elif args.workload in ("config3", "config5") or args.actions == "random":
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + rank)   # Philox counter-based RNG on the device
        acts = torch.randint(0, 8, (total, n), generator=g, device=dev, dtype=torch.int64).to(torch.uint8)
    else:
        cyc = torch.tensor([0, 3, 1, 2], dtype=torch.uint8, device=dev)
        acts = cyc[torch.arange(total, device=dev) % 4].unsqueeze(1).expand(total, n).contiguous()
    torch.cuda.synchronize(dev)

    for t in range(args.warmup):
        env_step(t)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    emu.profile_enable(True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    instr = 0
    for t in range(args.warmup, total):
        env_step(t)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    emu_ms, ren_ms, rew_ms, nprof = emu.profile_read()
    instr = emu.last_instr_count()  # last step's emulated instructions (all envs)
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max.item())

    if rank == 0:
        value = world * n * args.steps / elapsed
        k1_s = emu_ms / 1e3 / max(nprof, 1)
        k2_s = ren_ms / 1e3 / max(nprof, 1)
        k4_s = rew_ms / 1e3 / max(nprof, 1)
        achieved = B_HEADLESS * n / k1_s / 1e9
        traffic = None
        prof_path = os.path.join(HERE, "profiles", f"pmc_{args.workload}.json")
        if os.path.exists(prof_path) and not args.rom:
            try:
                traffic = json.load(open(prof_path)).get("hbm_bytes_per_launch_k1")
            except Exception:  # noqa: BLE001
                traffic = None
        out = {
            "metric": "aggregate env.step/sec",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": {"config3": "configs[2]: 65536 envs/GPU, PPU-rendered 160x144 u8 screen obs, random actions",
                             "config2": "configs[1]: headless (no PPU), RAM-only obs, fixed action cycle [0,3,1,2]",
                             "config5": "configs[4]: configs[2] + full ram_map reward stack + (72,80,4) obs + "
                                        "per-env template reload on done + episodic-return all-reduce every 128 steps",
                             }[args.workload],
                "envs_per_gpu": n,
                "rom": rom_name,
                "start_state": os.path.basename(args.state) if args.state else "power-on (post-boot)",
                "frame_skip": 24,
                "release_frame": 8,
                "parallelism": f"envs sharded over {world} GPU(s), no data-path collective",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "pk_step_kernel (K1: 24 emulated frames)",
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic,
                "bytes_per_env_step": B_HEADLESS,
                "k1_ms": round(k1_s * 1e3, 3),
                "k2_render_ms": round(k2_s * 1e3, 3),
                "k4_reward_obs_ms": round(k4_s * 1e3, 3),
            },
            "emulated_instr_per_s": round(instr / max(k1_s, 1e-9), 1),
            "instr_per_env_step": round(instr / n, 1),
        }
        if not args.no_cpu_baseline and world == 1:
            try:
                out["cpu_baseline"] = _cpu_baseline(rom, state)
            except Exception as e:  # noqa: BLE001
                out["cpu_baseline"] = {"value": None, "error": f"{type(e).__name__}: {e}"}
        print(json.dumps(out), flush=True)
    emu.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
