"""HBM ceilings on this MI355X for the writer's shape: a device-to-device copy
of 2 GB (torch copy_), a 4 GB read (sum), a 2 GB fill; reported as bytes
moved / kernel time."""
import json
import torch

def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps

n = 2 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda")
y = torch.empty(n, dtype=torch.uint8, device="cuda")
x.random_(0, 255)
r = {}
t = timed(lambda: y.copy_(x))
r["copy_2GB"] = {"ms": t, "TB/s (read+write)": 2 * n / t / 1e9}
xi = x.view(torch.int64)
t = timed(lambda: xi.sum())
r["read_2GB_sum_i64"] = {"ms": t, "TB/s": n / t / 1e9}
t = timed(lambda: y.fill_(7))
r["fill_2GB"] = {"ms": t, "TB/s": n / t / 1e9}
print(json.dumps(r))
