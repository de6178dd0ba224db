"""Decompression-at-ingest throughput on the GPU (not a pytest test: run as
`python tests/perf_decompress.py` on the GPU box).  C2 records re-stored with
each codec (oracle/fsg_codec.c encoders, Python gzip, libzstd level 3), then ingested
(fsg_slice_upload: framing, CRC check of the stored bytes, decompression
sizing + writing passes, re-framing) and processed once for parity."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fluvio_amd import synth  # noqa: E402
from fluvio_amd.smartengine import (ResidentSlice, SmartEngine, SmartModuleChainBuilder,  # noqa: E402
                                    SmartModuleConfig, builtin)
from oracle import oracle as O  # noqa: E402
from tests.compressed_slices import recompress  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    sl = synth.make_slice(2, n)
    engine = SmartEngine(0)
    out = {"records": n, "uncompressed_bytes": len(sl)}
    for name, codec, flags in (("gzip", 1, 0), ("snappy", 2, 0), ("lz4", 3, 0), ("zstd", 4, 0x100 | 3)):
        csl = recompress(sl, [codec], flags)
        ResidentSlice(engine, csl)  # warm
        t0 = time.perf_counter()
        rs = ResidentSlice(engine, csl)
        dt = time.perf_counter() - t0
        b = SmartModuleChainBuilder.default()
        b.add_smart_module(SmartModuleConfig.builder().param("key", "timeout").build(), builtin("filter_init"))
        g = b.initialize(engine).process_batch(csl)
        ref = O.OracleChain([("filter_init", {"key": "timeout"}, None)]).process_batch(csl)
        out[name] = {"compressed_bytes": len(csl), "ingest_s": dt,
                     "decompressed_gbps": rs.bytes / dt / 1e9, "records": rs.n_records,
                     "bit_exact": g.raw == ref["bytes"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
