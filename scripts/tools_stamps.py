"""Diagnostic: per-phase cycle shares of k_eval (stamped build, FSG_LIB=libfsg_stamps.so)."""
import ctypes, os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["FSG_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fluvio_amd", "_lib", "libfsg_stamps.so")
from fluvio_amd import _ffi, synth
from fluvio_amd.smartengine import *
kind = int(sys.argv[1]) if len(sys.argv) > 1 else 2
mod = sys.argv[2] if len(sys.argv) > 2 else "filter_init"
params = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {"key": "timeout"}
n = int(sys.argv[4]) if len(sys.argv) > 4 else 1_000_000
e = SmartEngine(0)
b = SmartModuleChainBuilder.default(); b.set_store_memory_limit(1 << 36)
b.add_smart_module(SmartModuleConfig.builder().params(params).build(), builtin(mod))
ch = b.initialize(e)
rs = ResidentSlice(e, synth.make_slice_array(kind, n))
L = _ffi.lib(); L.fsg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
ch.process_slice(rs, download=False)
L.fsg_debug_stamps(buf, 1)
ch.process_slice(rs, download=False)
L.fsg_debug_stamps(buf, 0)
lean = os.environ.get("LEAN_STAMPS") == "1"
names = ["pre/loop", "load_window", "walk", "eval(rest)", "emit", "tail", "", "", "windows", "exact_walks", "ev.clear", "ev.scan", "ev.perrec"]
if lean:
    names = ["load", "chase", "parse", "scan", "gap+check", "emit", "", "", "", "", "", "", ""]
tot = sum(buf[i] for i in range(6)) + (0 if lean else sum(buf[i] for i in (10, 11, 12)))
print("kind", kind, mod, "timings", ch.last_timings())
for i in range(13):
    if names[i]:
        print(f"{names[i]:12s} {buf[i]:16d} {100.0*buf[i]/tot if i not in (8, 9) else 0:6.1f}%")
print("cycles per wave", tot / rs.n_batches, "batches", rs.n_batches)
