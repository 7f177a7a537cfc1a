"""Quick GPU check: small kernel-vs-oracle parity + a timing probe (run via gpurun)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle  # noqa: E402
from pokegym_amd.emulator import BatchedEmulator  # noqa: E402
from pokegym_amd.testrom.fuzz import fuzz_rom  # noqa: E402

try:
    import pyboy  # noqa: F401
    print("pyboy importable on this box:", pyboy.__file__)
except Exception as e:  # noqa: BLE001
    print("pyboy not importable:", type(e).__name__)
print("nproc", os.cpu_count(), "gpu", torch.cuda.get_device_name(0), flush=True)

for seed in (0, 1):
    rom = fuzz_rom(seed)
    n, steps = 128, 3
    rng = np.random.default_rng(seed)
    acts = rng.integers(0, 9, size=(steps, n), dtype=np.uint8)
    emu = BatchedEmulator(rom, n)
    for s in range(steps):
        emu.step(torch.from_numpy(acts[s]).to(emu.device))
    torch.cuda.synchronize()
    gpu = [emu.snapshot(e) for e in range(n)]
    ref, _ = oracle.batch_run(rom, None, acts, want_screens=False)
    bad = [e for e in range(n) if gpu[e] != ref[e].tobytes()]
    print(f"seed {seed}: mismatching envs {len(bad)}/{n}", flush=True)
    if bad:
        a = np.frombuffer(gpu[bad[0]], np.uint8)
        b = ref[bad[0]]
        idx = np.nonzero(a != b)[0]
        print("  first diffs at", idx[:20].tolist(), "gpu", a[idx[:8]].tolist(), "ref", b[idx[:8]].tolist())
    emu.close()

rom = fuzz_rom(0)
for n, mode in ((4096, "random"), (65536, "random"), (65536, "same"), (131072, "random")):
    emu = BatchedEmulator(rom, n)
    if mode == "random":
        acts = torch.randint(0, 8, (n,), dtype=torch.uint8, device="cuda")
    else:
        acts = torch.zeros(n, dtype=torch.uint8, device="cuda")
    emu.step(acts)
    torch.cuda.synchronize()
    t = time.time()
    k = 3
    for _ in range(k):
        emu.step(acts)
    torch.cuda.synchronize()
    dt = (time.time() - t) / k
    ic = emu.last_instr_count()
    print(f"n={n} {mode}: {dt*1e3:.1f} ms/step  {n/dt:,.0f} env-steps/s  {ic/dt/1e9:.2f} G emulated instr/s  {ic/n:.0f} instr/env-step", flush=True)
    emu.close()
