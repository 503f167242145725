"""PCIe duplex probe: pinned H2D alone, D2H alone, then both at once on two streams (GB/s).
Tells whether the host pipeline's H2D and D2H copies can overlap."""
import time
import torch

n = 2 << 30
h_in = torch.empty(n, dtype=torch.uint8).pin_memory()
h_out = torch.empty(n, dtype=torch.uint8).pin_memory()
d_a = torch.empty(n, dtype=torch.uint8, device="cuda")
d_b = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def run(h2d, d2h, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_in, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_out.copy_(d_b, non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return n / best / 1e9


print(f"H2D alone {run(True, False):.1f} GB/s, D2H alone {run(False, True):.1f} GB/s, "
      f"both at once {run(True, True):.1f} GB/s each way", flush=True)
