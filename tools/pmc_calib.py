"""Known-byte-count kernels for calibrating rocprofv3 FETCH_SIZE / WRITE_SIZE units on gfx950:
a 1 GiB device-to-device copy (reads 1 GiB, writes 1 GiB; well past the 256 MiB Infinity Cache)."""
import torch

n = 1 << 30
a = torch.empty(n, dtype=torch.uint8, device="cuda").fill_(1)
b = torch.empty(n, dtype=torch.uint8, device="cuda")
torch.cuda.synchronize()
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
print("copied", n)
