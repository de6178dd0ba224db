"""Lean-path diagnostic on one MI355X: eval time and deferred batches per chain
over the C2 synthetic slice (median of 7 process_slice calls)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluvio_amd import synth  # noqa: E402
from fluvio_amd.smartengine import (ResidentSlice, SmartEngine, SmartModuleChainBuilder,  # noqa: E402
                                    SmartModuleConfig, builtin)

nrec = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
chains = {
    "substr": [("filter_init", {"key": "timeout"})],
    "json": [("filter_json", {})],
    "c3": [("filter_init", {"key": "timeout"}), ("map_json_project", {"field": "message"}), ("map", {})],
}
eng = SmartEngine(0)
sl = synth.make_slice_array(2, nrec)
rs = ResidentSlice(eng, sl)
for name, mods in chains.items():
    if only and name not in only:
        continue
    b = SmartModuleChainBuilder.default()
    for m, p in mods:
        b.add_smart_module(SmartModuleConfig.builder().params(p).build(), builtin(m))
    ch = b.initialize(eng)
    ev = []
    for _ in range(8):
        ch.process_slice(rs, download=False)
        ev.append(ch.last_timings()["eval_ms"])
    t = ch.last_timings()
    print(f"{name:8s} eval {statistics.median(ev[1:]):.3f} ms path {t['eval_path']} deferred {t['deferred']} / "
          f"{t['n_batches']} in {t['in_bytes'] / 1e9:.3f} GB", flush=True)
