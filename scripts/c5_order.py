"""c5-agg-sum after another workload in the same process: which earlier
workload leaves the host slower (usage: c5_order.py W [W ...]; c5-agg-sum runs
after them, and once first for comparison when W is 'none')."""
import gc
import sys
import time

sys.argv = [sys.argv[0], "--no-cpu-baseline", "--no-e2e", "--steps", "10", "--warmup", "2"] + \
    [a for a in sys.argv[1:] if a.startswith("--")] + ["--"] + [a for a in sys.argv[1:] if not a.startswith("--")]
sep = sys.argv.index("--")
pre = sys.argv[sep + 1:]
del sys.argv[sep:]
import bench  # noqa: E402

a = bench.parse()
ctx = bench.Ctx(a)
for w in pre:
    if w != "none":
        r = bench.run_workload(ctx, w, 0, {})
        print(w, round(r["ms_per_step"], 3), flush=True)
    gc.collect()
    import threading
    print("python threads", threading.active_count(), flush=True)
r = bench.run_workload(ctx, "c5-agg-sum", 0, {})
print("c5-agg-sum", round(r["ms_per_step"], 3), r["kernel_ms_max_over_partitions"], flush=True)
