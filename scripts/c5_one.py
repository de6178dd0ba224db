"""One C5 partition alone: aggregate-sum over 1 M decimal records (the c5-agg-sum
slice of partition 0), per-phase times from the chain's timings."""
import json
import sys
import time

from fluvio_amd import synth
from fluvio_amd.smartengine import (ResidentSlice, SmartEngine, SmartModuleChainBuilder, SmartModuleConfig, builtin,
                                    process_slices)

mod = sys.argv[1] if len(sys.argv) > 1 else "aggregate-sum"
eng = SmartEngine(0)
sl = synth.make_slice_array(3, 1_000_000, seed=synth.SEEDS[3])
b = SmartModuleChainBuilder.default()
b.add_smart_module(SmartModuleConfig.builder().build(), builtin(mod))
ch = b.initialize(eng)
rs = ResidentSlice(eng, sl)
res = []
for i in range(6):
    t0 = time.perf_counter()
    process_slices([ch], [rs])
    dt = (time.perf_counter() - t0) * 1e3
    t = ch.last_timings()
    res.append({"wall_ms": round(dt, 3), **{k: round(v, 3) for k, v in t.items() if k.endswith("_ms")}})
print(json.dumps({"module": mod, "batches": t.get("n_batches"), "runs": res[1:]}))
