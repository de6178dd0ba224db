"""bench.py — SmartModule filter chain on MI355X (BASELINE.json metric).

One step = one SPU process_batch (fluvio-spu/src/smartengine/batch.rs:41-142)
over an HBM-resident fetch slice of stored batches: decode, chain evaluation,
compaction + offset fix-up, output batch re-encode and CRC32C — the whole path,
output left in HBM.  Default workload = BASELINE.json configs[1] (C2):
substring filter (filter_init, key="timeout") over ~1 KB JSON log records
(synthetic, seed 0xF101, ~16 KB batches, one partition per GPU).

Multi-GPU: one process per GPU (torch.distributed.run); topic partitions are
sharded p -> rank, each rank filters its own partition slice, no data-path
collective ("weak" scaling).  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # name: (synth kind, chain modules, records per GPU, description)
    "c2-substring": (2, [("filter_init", {"key": "timeout"}, None)], 4_000_000,
                     "substring filter (filter_init key=timeout) on 1 KB JSON records"),
    "c1-regex": (1, [("regex-filter", {"regex": r"\d{3}-\d{2}-\d{4}"}, None)], 8_000_000,
                 "regex-filter \\d{3}-\\d{2}-\\d{4} on 256 B records"),
    "c3-filter-map": (2, [("filter_init", {"key": "timeout"}, None), ("map", {}, None)], 4_000_000,
                      "filter -> map (uppercase) chain with compaction, re-encode, CRC32C"),
    "c2-json": (2, [("filter_json", {}, None)], 4_000_000,
                "JSON-field filter (filter_json: serde_json StructuredLog, keep level > debug) on 1 KB JSON records"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2-substring", choices=sorted(WORKLOADS))
    ap.add_argument("--records", type=int, default=0, help="records per GPU (0 = workload default)")
    ap.add_argument("--cpu-sample", type=int, default=1_500_000, help="records in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    kind, modules, nrec_default, desc = WORKLOADS[a.workload]
    nrec = a.records or nrec_default

    # the engine (libfsg, HIP) is loaded before torch; torch is only the
    # multi-process control plane (gloo barrier / max-reduce of timings)
    from fluvio_amd import synth
    from fluvio_amd.smartengine import (ResidentSlice, SmartEngine, SmartModuleChainBuilder,
                                        SmartModuleChainMetrics, SmartModuleConfig, builtin)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    engine = SmartEngine(local)
    b = SmartModuleChainBuilder.default()
    b.set_store_memory_limit(64 << 30)
    for name, params, acc in modules:
        b.add_smart_module(SmartModuleConfig.builder().params(params).build(), builtin(name))
    chain = b.initialize(engine)

    # partition slice of this rank (p -> rank), ingested into HBM once
    t0 = time.time()
    sl_bytes = synth.make_slice_array(kind, nrec, seed=synth.SEEDS[kind] + rank, base_offset=0)
    gen_s = time.time() - t0
    t0 = time.time()
    rs = ResidentSlice(engine, sl_bytes)
    ingest_s = time.time() - t0

    def barrier():
        if dist is not None:
            dist.barrier()

    metrics = SmartModuleChainMetrics()
    for _ in range(a.warmup):
        chain.process_slice(rs, metrics=metrics, download=False)
    barrier()
    acc = {"eval_ms": 0.0, "plan_ms": 0.0, "write_ms": 0.0, "crc_ms": 0.0, "total_ms": 0.0}
    t0 = time.perf_counter()
    for _ in range(a.steps):
        chain.process_slice(rs, metrics=metrics, download=False)  # synchronizes its stream at the end
        t = chain.last_timings()
        for k in acc:
            acc[k] += t[k]
    barrier()
    elapsed = time.perf_counter() - t0
    t = chain.last_timings()
    if dist is not None:
        import torch
        v = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        elapsed = float(v.item())

    steps = a.steps
    ms_per_step = elapsed / steps * 1e3
    in_bytes = t["in_bytes"]
    out_bytes = t["out_bytes"]
    recs = rs.n_records
    value = recs * world * steps / elapsed
    per = {k: acc[k] / steps for k in acc}
    # algorithmic bytes per launch: k_eval reads the slice once; k_write reads the
    # survivors' payloads (~ the output size) and writes the output batch once
    kernels = {"k_eval": (per["eval_ms"], in_bytes), "k_write": (per["write_ms"], 2 * out_bytes),
               "k_crc": (per["crc_ms"], out_bytes)}
    dom = max(kernels, key=lambda k: kernels[k][0])
    dom_ms, dom_bytes = kernels[dom]
    peak = 8000.0  # GB/s, MI355X HBM3E (MI355X_MICROARCH.md)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    pipe_gbps = (in_bytes + out_bytes) / (per["total_ms"] * 1e-3) / 1e9

    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tpath):  # PMC HBM bytes per launch of the same command (scripts/traffic_from_pmc.py)
        db = json.load(open(tpath)).get(a.workload)
        if db:
            # the eval timing brackets k_eval_lean plus the deferred exact k_eval<N>
            # (and crc brackets k_crc16 + k_crc_final): sum every launch in the bracket
            hits = [v["total"] for kname, v in db["kernels"].items()
                    if kname.split("<")[0].startswith("fsg::" + dom)]
            if hits:
                traffic, traffic_src = sum(hits), db["source"]

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        from oracle.oracle import OracleChain
        # the sample is a batch-aligned prefix of this rank's own slice
        pos, n_s = 0, 0
        while pos < len(sl_bytes) and n_s < a.cpu_sample:
            hdr = sl_bytes[pos:pos + 61].tobytes()
            blen = int.from_bytes(hdr[8:12], "big")
            n_s += int.from_bytes(hdr[57:61], "big")
            pos += 12 + blen
        sample = sl_bytes[:pos].tobytes()
        oc = OracleChain(modules)
        t1 = time.perf_counter()
        r = oc.process_batch(sample)
        cpu_s = time.perf_counter() - t1
        assert r["status"] == 0
        cpu = {"value": n_s / cpu_s, "unit": "records/s", "cores": 1, "kind": "port",
               "sample": f"{n_s} records of the same workload (one process_batch over "
                         f"{len(sample)} B) through the scalar C oracle on 1 host core; wasmtime "
                         f"itself is not available here (no Rust)",
               "seconds": cpu_s}

    if rank == 0:
        line = {
            "metric": "records/sec + achieved HBM GB/s for SmartModule filter chain, 1/2/4/8 MI355X",
            "value": value,
            "unit": "records/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (fluvio_amd/tools/synth.c), HBM-resident batches",
            "config": {"workload": a.workload, "description": desc, "records_per_gpu": recs,
                       "batches_per_gpu": rs.n_batches, "slice_bytes_per_gpu": in_bytes,
                       "output_bytes_per_gpu": out_bytes, "chain": [m[0] for m in modules],
                       "parallelism": f"partitions sharded over {world} GPU(s)"},
            "gbps_pipeline": pipe_gbps,
            "gbps_input": in_bytes * world * steps / elapsed / 1e9,
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": peak, "unit": "GB/s",
                         "frac": achieved / peak, "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": dom_ms},
            "kernel_ms": per,
            "cpu_baseline": cpu,
            "setup_s": {"generate": gen_s, "ingest_h2d": ingest_s},
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
