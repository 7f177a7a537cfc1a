"""Timing probe (GPU): ms per env-step and K1 ms for (envs, action mode, render) settings.

usage: python tools/probe_lat.py N:MODE:RENDER ...   MODE = random | cycle | down | same
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pokegym_amd.emulator import BatchedEmulator  # noqa: E402
from pokegym_amd.testrom.game import game_rom  # noqa: E402


def run(rom, n, mode, render, steps=6, warm=3):
    emu = BatchedEmulator(rom, n, render=render)
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    tot = warm + steps
    if mode == "random":
        acts = torch.randint(0, 8, (tot, n), generator=g, device="cuda").to(torch.uint8)
    elif mode == "cycle":
        cyc = torch.tensor([0, 3, 1, 2], dtype=torch.uint8, device="cuda")
        acts = cyc[torch.arange(tot, device="cuda") % 4].unsqueeze(1).expand(tot, n).contiguous()
    elif mode == "down":
        acts = torch.zeros((tot, n), dtype=torch.uint8, device="cuda")
    else:
        acts = torch.randint(0, 8, (tot, 1), generator=g, device="cuda").to(torch.uint8).expand(tot, n).contiguous()
    for t in range(warm):
        emu.step(acts[t])
    torch.cuda.synchronize()
    emu.profile_enable(True)
    t0 = time.perf_counter()
    for t in range(warm, tot):
        emu.step(acts[t])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    k1, k2, k4, ns = emu.profile_read()
    ic = emu.last_instr_count()
    emu.close()
    return dt * 1e3, k1 / ns, ic / n


rom = game_rom()
for a in sys.argv[1:]:
    n, mode, render = a.split(":")
    ms, k1, ipe = run(rom, int(n), mode, render == "1")
    print(json.dumps({"n": int(n), "mode": mode, "render": render == "1", "ms_step": round(ms, 2),
                      "k1_ms": round(k1, 2), "env_steps_per_s": round(int(n) / ms * 1e3),
                      "instr_per_env_step": round(ipe)}), flush=True)
