"""Diagnostic: run one chain over a resident synthetic slice with a chosen
library build (FSG_LIB) and print the kernel timings (for rocprofv3 counter
attribution between experiment builds)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluvio_amd import synth
from fluvio_amd.smartengine import *
kind = int(sys.argv[1]); mod = sys.argv[2]; params = json.loads(sys.argv[3]); n = int(sys.argv[4])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 3
e = SmartEngine(0)
b = SmartModuleChainBuilder.default(); b.set_store_memory_limit(1 << 36)
b.add_smart_module(SmartModuleConfig.builder().params(params).build(), builtin(mod))
ch = b.initialize(e)
rs = ResidentSlice(e, synth.make_slice_array(kind, n))
for _ in range(reps):
    ch.process_slice(rs, download=False)
print(os.environ.get("FSG_LIB", "libfsg.so"), ch.last_timings())
