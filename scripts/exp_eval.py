"""Ad-hoc eval-time comparison on one MI355X: several chains over the same
resident slice, eval_ms / total_ms from fsg_chain_last_timings (median of 7)."""
import statistics
import sys

sys.path.insert(0, ".")
from fluvio_amd import synth  # noqa: E402
from fluvio_amd.smartengine import (ResidentSlice, SmartEngine, SmartModuleChainBuilder,  # noqa: E402
                                    SmartModuleConfig, builtin)

kind, nrec = int(sys.argv[1]), int(sys.argv[2])
chains = {
    "json": [("filter_json", {})],
    "c3": [("filter_init", {"key": "timeout"}), ("map_json_project", {"field": "message"}), ("map", {})],
} if kind == 2 else {
    "regex_ssn": [("regex-filter", {"regex": r"\d{3}-\d{2}-\d{4}"})],
    "regex_lit": [("regex-filter", {"regex": "zqzq"})],
    "regex_cls": [("regex-filter", {"regex": r"[0-9]-[0-9]"})],
    "substr_dash": [("filter_init", {"key": "-"})],
    "substr_long": [("filter_init", {"key": "zqzqzq"})],
    "map": [("map", {})],
}
eng = SmartEngine(0)
sl = synth.make_slice_array(kind, nrec)
rs = ResidentSlice(eng, sl)
for name, mods in chains.items():
    b = SmartModuleChainBuilder.default()
    for m, p in mods:
        b.add_smart_module(SmartModuleConfig.builder().params(p).build(), builtin(m))
    ch = b.initialize(eng)
    ev, tot = [], []
    for _ in range(8):
        ch.process_slice(rs, download=False)
        t = ch.last_timings()
        ev.append(t["eval_ms"])
        tot.append(t["total_ms"])
    t = ch.last_timings()
    print(f"{name:12s} eval {statistics.median(ev[1:]):.3f} ms total {statistics.median(tot[1:]):.3f} ms "
          f"path {t['eval_path']} deferred {t['deferred']} / {t['n_batches']} in {t['in_bytes'] / 1e9:.3f} GB "
          f"out {t['out_bytes'] / 1e9:.3f} GB", flush=True)
