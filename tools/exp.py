"""Ad-hoc timing sweep (GPU): ms per env-step for several (envs, actions, render) settings."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pokegym_amd.emulator import BatchedEmulator
from pokegym_amd.testrom.game import game_rom
from pokegym_amd.testrom.fuzz import fuzz_rom

def run(rom, n, mode, render, steps=4, warm=3):
    emu = BatchedEmulator(rom, n, render=render)
    g = torch.Generator(device="cuda"); g.manual_seed(0)
    tot = warm + steps
    if mode == "random":
        acts = torch.randint(0, 8, (tot, n), generator=g, device="cuda").to(torch.uint8)
    elif mode == "same":
        acts = torch.randint(0, 8, (tot, 1), generator=g, device="cuda").to(torch.uint8).expand(tot, n).contiguous()
    else:
        acts = torch.full((tot, n), 8, dtype=torch.uint8, device="cuda")
    for t in range(warm): emu.step(acts[t])
    torch.cuda.synchronize()
    emu.profile_enable(True)
    t0 = time.perf_counter()
    for t in range(warm, tot): emu.step(acts[t])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    k1, k2, ns = emu.profile_read()
    ic = emu.last_instr_count()
    emu.close()
    return dt * 1e3, k1 / ns, ic / n

rom = game_rom()
specs = [(a.split(":")[0], int(a.split(":")[1]), a.split(":")[2], a.split(":")[3] == "1") for a in sys.argv[1:]]
for romname, n, mode, render in specs:
    r = rom if romname == "game" else fuzz_rom(int(romname[4:]))
    ms, k1, ipe = run(r, n, mode, render)
    print(json.dumps({"rom": romname, "n": n, "mode": mode, "render": render, "ms_step": round(ms, 2), "k1_ms": round(k1, 2),
                      "instr_per_env_step": round(ipe), "ns_per_lane_instr": round(k1 * 1e6 / ipe, 1)}), flush=True)
