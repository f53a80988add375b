# torch copy (y = x) bandwidth vs buffer size on one MI355X: does a plain streaming kernel lose efficiency at a few
# GiB per launch the way the product's kernels do?  Prints GB/s moved (read + write) and the fraction of 8 TB/s.
import torch
torch.cuda.set_device(0)
for gib in (0.5, 1, 2, 4, 8, 16, 28):
    n = int(gib * 2 ** 30)
    x = torch.empty(n, dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    x.fill_(1)
    for _ in range(3):
        y.copy_(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(3, int(16 / gib))
    e0.record()
    for _ in range(reps):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / reps
    print(f"{gib:5.1f} GiB: {t * 1e3:8.3f} ms per copy, {2 * n / t / 1e9:7.1f} GB/s = {2 * n / t / 8e12:.3f} of 8 TB/s",
          flush=True)
    del x, y
    torch.cuda.empty_cache()
