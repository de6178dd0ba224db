"""bench.py — SmartModule record-transform path on MI355X (BASELINE.json metric).

One step = one SPU process_batch (fluvio-spu/src/smartengine/batch.rs:41-142)
over an HBM-resident fetch slice of stored batches: decode, chain evaluation,
compaction + offset fix-up, output batch re-encode and CRC32C — the whole path,
output left in HBM.  The headline line is BASELINE.json configs[1] (C2):
substring filter (filter_init key="timeout") over ~1 KB JSON log records
(synthetic, seed 0xF101, ~16 KB batches, one partition per GPU).

The same JSON line carries `workloads`, each timed in the same run with the
same contract (warmup, barrier + sync, max over ranks):
  c1-regex       regex-filter \\d{3}-\\d{2}-\\d{4} over 256 B records   (configs[0] shape)
  c2-json        filter_json (serde_json StructuredLog, level > debug)  (configs[1])
  c3-filter-map  filter -> projection -> uppercase, re-encode + CRC32C  (configs[2])
  c4-array-map   array_map_json_array, 1-16 elements per record         (configs[3])
  c5-keyed-agg   aggregate-json (per-key u32 sums) over 64 partitions, keys
                 routed by SipHash; each step every rank's keyed state is
                 merged topic-wide (all_gather over RCCL)               (configs[4])
  c5-agg-sum     aggregate-sum over 64 partitions, the 64-slot partition
                 state vector all-reduced over RCCL each step

Multi-GPU: one process per GPU (torch.distributed.run).  c1..c4: every rank
filters its own partition (p -> rank, no data-path collective, "weak").
c5: the 64 partitions are sharded p -> rank p mod N ("strong"), the state is
merged over RCCL each step.  Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import gc
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# name: (synth kind, chain modules, records per GPU, description)
WORKLOADS = {
    "c2-substring": (2, [("filter_init", {"key": "timeout"}, None)], 4_000_000,
                     "substring filter (filter_init key=timeout) on 1 KB JSON records"),
    "c1-regex": (1, [("regex-filter", {"regex": r"\d{3}-\d{2}-\d{4}"}, None)], 8_000_000,
                 "regex-filter \\d{3}-\\d{2}-\\d{4} on 256 B records"),
    "c2-json": (2, [("filter_json", {}, None)], 4_000_000,
                "JSON-field filter (filter_json: serde_json StructuredLog, keep level > debug) on 1 KB JSON records"),
    "c3-filter-map": (2, [("filter_init", {"key": "timeout"}, None), ("map_json_project", {"field": "message"}, None),
                          ("map", {}, None)], 4_000_000,
                      "filter -> map (field projection of `message` + ASCII uppercase) with compaction, re-encode, "
                      "CRC32C"),
    "c4-array-map": (5, [("array_map_json_array", {}, None)], 4_000_000,
                     "array_map_json_array exploding JSON arrays of 1-16 ints / short strings"),
    "f4-dedup": (3, [("filter_hashset", {}, None)], 4_000_000,
                 "filter_hashset dedup (BoundedHashSet, unbounded) over decimal i32 records in [-1000, 1000]; "
                 "steady state: the state persists across steps, so after the first step every value is a "
                 "duplicate (the decisions, table build and compaction still run over every record)"),
}
C5 = {"partitions": 64, "records_per_partition": 1_000_000,
      "modules": [("aggregate-sum", {}, None)],
      "description": "aggregate-sum over 64 partitions (decimal i32 records), per-partition accumulators in HBM, "
                     "RCCL all-reduce of the partition state vector each step"}
C5K = {"partitions": 64, "records_per_partition": 50_000, "keys": 1024,
       "modules": [("aggregate-json", {}, None)],
       "description": "aggregate-json over 64 partitions: records {\"repo-NNNN\": n} keyed by the repo name "
                      "(1024 keys routed by SipHash, ~16 per partition), per-key u32 sums, every record's output = "
                      "the pretty-printed map; each step the ranks' keyed states are merged topic-wide "
                      "through the C ABI (fsg_keyed_*: exact keys, RCCL all-gather of the key lists, union "
                      "dictionary, dense u32 all-reduce)"}
EXTRA = ["c1-regex", "c2-json", "c3-filter-map", "c4-array-map", "c5-keyed-agg", "c5-agg-sum", "f4-dedup",
         "f3-one-record"]
C5_ALL = ("c5-keyed-agg", "c5-agg-sum")
PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2-substring", choices=sorted(WORKLOADS) + list(C5_ALL) + ["f3-one-record"])
    ap.add_argument("--records", type=int, default=0, help="records per GPU of the headline workload (0 = default)")
    ap.add_argument("--only", action="store_true", help="time the headline workload only (no `workloads`)")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="records per CPU-baseline process")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--detail", default=os.path.join(ROOT, "bench_detail.json"),
                    help="the full result (phases, prose, fetch, e2e) is written here; stdout gets the compact line")
    ap.add_argument("--dry-run", action="store_true",
                    help="rank plumbing only (launch, rendezvous, barrier, max over ranks, the JSON line): no GPU work, "
                         "for the CPU tests of --gpus N")
    return ap.parse_args()


def launch_ranks(a):
    """--gpus N without a torch.distributed launcher around us: start one process
    per GPU under torch.distributed.run (127.0.0.1 rendezvous) as a CHILD of this
    GPU-free process and exit with its code.  Returns None when this process is
    already a rank (or N == 1).  A launcher's WORLD_SIZE that disagrees with
    --gpus is an error: the line would report the wrong n_gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        explicit = any(x == "--gpus" or x.startswith("--gpus=") for x in sys.argv[1:])
        if explicit and int(ws) != a.gpus:
            sys.stderr.write(f"bench.py: WORLD_SIZE={ws} but --gpus {a.gpus}\n")
            return 2
        return None
    if a.gpus <= 1:
        return None
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


KERNEL_SOURCES = ("fsg_kernels.hip", "fsg_lean.hip", "fsg_array.hip", "fsg_device.h", "fsg_dev_util.h", "fsg_codec_dev.h", "fsg_json_dev.h",
                  "fsg_json_dfa.h", "fsg_launch.h")


def lib_tag():
    """Content hash of the device-code sources: PMC traffic is quoted only for the
    kernels it was measured on (host-runtime edits do not change device traffic)."""
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(ROOT, "fluvio_amd", "csrc", f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(workload, kernel, n_records, n_batches):
    """Per-launch HBM bytes of the dominant kernel bracket from profiles/traffic.json
    (scripts/traffic_from_pmc.py), only when measured on this build and shape."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None, None
    db = json.load(open(path)).get(workload)
    if not db or db.get("lib") != lib_tag() or db.get("n_records") != n_records or db.get("n_batches") != n_batches:
        return None, None
    # the eval bracket covers k_chase + k_eval_lean, the flat path's k_flat_scan + k_flat_decide,
    # k_arr_frame + k_arr_lean, and the deferred exact k_eval<N>; crc: k_crc16 + k_crc_final;
    # write: k_write(_lean) + k_write_canon
    pre = ("fsg::" + kernel,) + (("fsg::k_arr_frame", "fsg::k_arr_lean", "fsg::k_flat_", "fsg::k_chase") if kernel == "k_eval" else ())
    hits = [v["total"] for k, v in db["kernels"].items() if k.split("<")[0].startswith(pre)]
    return (sum(hits), db["source"]) if hits else (None, None)


class Ctx:
    def __init__(self, a):
        self.a = a
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self._nccl = None
        if self.world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, v):
        if self.dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def broadcast_bytes(self, b, n):
        if self.dist is None:
            return b
        import torch
        t = torch.tensor(list(b) if self.rank == 0 else [0] * n, dtype=torch.uint8)
        self.dist.broadcast(t, 0)
        return bytes(t.tolist())


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_proc(args):
    """One CPU-baseline process = one partition: its own synthetic slice through
    the scalar C oracle (process_batch), timed inside the process."""
    kind, modules, nrec, seed = args
    from fluvio_amd import synth
    from oracle.oracle import OracleChain
    if kind == "keyed":
        p = seed % C5K["partitions"]
        sl = synth.make_keyed_slices(C5K["partitions"], nrec, C5K["keys"], owned=[p])[p]
    else:
        sl = synth.make_slice(kind, nrec, seed=seed)
    oc = OracleChain(modules)
    t0 = time.perf_counter()
    r = oc.process_batch(sl)
    dt = time.perf_counter() - t0
    assert r["status"] == 0
    return nrec, dt


def cpu_baseline(kind, modules, per_proc):
    """Oracle CPU baseline, one process per partition on the host cores this box
    grants (os.cpu_count() shows the whole machine; the GPU box's share is 16)."""
    import multiprocessing as mp
    cores = max(1, min(16, os.cpu_count() or 1, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 16))
    jobs = [(kind, modules, per_proc, 0xC0DE + p) for p in range(cores)]
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(cores) as pool:
        res = pool.map(_cpu_proc, jobs)
    wall = time.perf_counter() - t0
    n = sum(r[0] for r in res)
    busy = max(r[1] for r in res)  # slowest process's process_batch time (generation excluded)
    return {"value": n / busy, "unit": "records/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "sample": f"{cores} processes x {per_proc} records (one partition each, synthetic, same generator) "
                      f"through the scalar C oracle process_batch; value = all records / slowest process's time; "
                      f"wasmtime itself is not available here (no Rust toolchain)",
            "seconds": busy, "wall_s": wall}


def roofline(per, t, workload, n_records, n_batches, records_out, step_ms):
    """The dominant phase of the step and its HBM roofline, plus the whole step.
    Phases (HIP events on the chain's stream) and their algorithmic bytes per
    launch: eval reads the slice once (k_chase + k_eval_lean /
    k_arr_lean + deferred k_eval); plan reads a 64-B descriptor per surviving
    record and ~300 B of scan rows per batch (k_mins, k_size, k_scan_*, k_plan);
    text is the aggregate text / order phase (output bytes); write reads the
    survivors' payloads and writes the output once (array_map: k_arr_write reads
    the input and writes the output); crc reads the output once."""
    ib, ob = t["in_bytes"], t["out_bytes"]
    c4 = workload == "c4-array-map"
    phases = {"k_eval": (per["eval_ms"], ib),
              "k_plan": (per["plan_ms"], 64 * records_out + 300 * n_batches),
              "k_text": (per.get("text_ms", 0.0), ob),
              "k_write": (per["write_ms"], ib + ob if c4 else 2 * ob),
              "k_crc": (per["crc_ms"], ob)}
    dom = max(phases, key=lambda k: phases[k][0])
    dom_ms, dom_bytes = phases[dom]
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    traffic, src = pmc_traffic(workload, dom, n_records, n_batches)
    step_gbps = (ib + ob) / (step_ms * 1e-3) / 1e9 if step_ms > 0 else 0.0
    return {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / PEAK_GBPS, "traffic": traffic, "traffic_source": src,
            "algorithmic_bytes_per_launch": dom_bytes, "avg_launch_ms": dom_ms,
            "phases_ms": {k: v[0] for k, v in phases.items()},
            "step": {"bytes": ib + ob, "ms": step_ms, "achieved": step_gbps, "frac": step_gbps / PEAK_GBPS,
                     "note": "whole step: input + output bytes / ms_per_step (every kernel of the step)"}}


def roofline_step(bytes_per_step, step_ms, kernel, kernel_ms, note):
    """C5: the partitions' chains run concurrently, so per-chain kernel times
    summed over chains are no launch duration.  Priced on the step: the bytes
    every owned partition moves per step / ms_per_step; `kernel` names the
    dominant launch and its own duration (HIP events around it)."""
    achieved = bytes_per_step / (step_ms * 1e-3) / 1e9 if step_ms > 0 else 0.0
    return {"bound": "hbm", "kernel": kernel, "achieved": achieved, "peak": PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / PEAK_GBPS, "traffic": None, "traffic_source": None,
            "algorithmic_bytes_per_launch": bytes_per_step, "avg_launch_ms": step_ms,
            "priced_on": "step", "dominant_kernel_ms": kernel_ms, "note": note}


PHASES = ("eval_ms", "plan_ms", "text_ms", "write_ms", "crc_ms", "total_ms")
PHASE_KERNEL = {"eval_ms": "k_eval", "plan_ms": "k_plan", "text_ms": "k_text", "write_ms": "k_write",
                "crc_ms": "k_crc", "total_ms": "step"}

_SLICES = {}


def get_slice(kind, nrec, rank):
    from fluvio_amd import synth
    key = (kind, nrec, rank)
    if key not in _SLICES:
        t0 = time.time()
        _SLICES[key] = (synth.make_slice_array(kind, nrec, seed=synth.SEEDS[kind] + rank, base_offset=0),
                        time.time() - t0)
    return _SLICES[key]


def cpu_one_record():
    """f3's CPU baseline: the scalar oracle's process() of the same one-record
    SmartModuleInput (one host core, called through ctypes), p50 over 20000 calls."""
    from fluvio_amd import protocol as P
    from oracle.oracle import OracleChain
    raw = P.encode_records([P.Record.new(b'{"level":"warn","message":"request timeout"}')])
    oc = OracleChain([("filter_init", {"key": "timeout"}, None)])
    for _ in range(200):
        oc.process(raw, 0, -1)
    n = 20000
    lat = []
    for _ in range(n):
        t1 = time.perf_counter()
        r = oc.process(raw, 0, -1)
        lat.append(time.perf_counter() - t1)
    assert r["status"] == 0 and r["n_records"] == 1
    lat.sort()
    return {"value": lat[n // 2] * 1e6, "unit": "us", "cores": 1, "kind": "port", "p99_us": lat[n * 99 // 100] * 1e6,
            "sample": f"{n} calls of the scalar C oracle's process() on the same one-record input, p50 (includes "
                      f"the ctypes call and result marshalling, ~a few us); wasmtime itself is not available here"}


def cpu_baselines_first(ctx, names):
    """CPU baselines run before this process touches the GPU (the pool's
    processes are started from a GPU-free parent), rank 0 at N=1 only."""
    a = ctx.a
    if ctx.rank != 0 or ctx.world != 1 or a.no_cpu_baseline:
        return {}
    out = {}
    for w in names:
        if w == "f3-one-record":
            out[w] = cpu_one_record()
            continue
        if w == "c5-agg-sum":
            out[w] = cpu_baseline(3, C5["modules"], min(a.cpu_sample, C5["records_per_partition"]))
        elif w == "c5-keyed-agg":
            out[w] = cpu_baseline("keyed", C5K["modules"], min(a.cpu_sample, C5K["records_per_partition"]))
        else:
            kind, modules, nrec, _ = WORKLOADS[w]
            out[w] = cpu_baseline(kind, modules, min(a.cpu_sample, nrec))
    return out


def run_filter(ctx, name, nrec, cpu):
    """One workload: chain over this rank's resident partition slice."""
    from fluvio_amd.smartengine import (ResidentSlice, SmartEngine, SmartModuleChainBuilder,
                                        SmartModuleChainMetrics, SmartModuleConfig, builtin)
    a = ctx.a
    kind, modules, nrec_default, desc = WORKLOADS[name]
    nrec = nrec or nrec_default
    engine = SmartEngine(ctx.local)
    b = SmartModuleChainBuilder.default()
    b.set_store_memory_limit(64 << 30)
    for mname, params, acc in modules:
        b.add_smart_module(SmartModuleConfig.builder().params(params).build(), builtin(mname))
    chain = b.initialize(engine)
    sl_bytes, gen_s = get_slice(kind, nrec, ctx.rank)
    t0 = time.time()
    rs = ResidentSlice(engine, sl_bytes)
    ingest_s = time.time() - t0
    # CRC32C verify on ingest (north_star): every stored batch's CRC checked on
    # the GPU against its header (report only, as the reference never checks)
    rs.verify_crc()
    vbad, _vfirst, vms = min((rs.verify_crc() for _ in range(3)), key=lambda r: r[2])
    metrics = SmartModuleChainMetrics()
    for _ in range(a.warmup):
        chain.process_slice(rs, metrics=metrics, download=False)
    ctx.barrier()
    acc = {"eval_ms": 0.0, "plan_ms": 0.0, "text_ms": 0.0, "write_ms": 0.0, "crc_ms": 0.0, "total_ms": 0.0}
    ro0 = metrics.records_out()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        chain.process_slice(rs, metrics=metrics, download=False)  # synchronizes its stream at the end
        t = chain.last_timings()
        for k in acc:
            acc[k] += t[k]
    ctx.barrier()
    elapsed = ctx.max_over_ranks(time.perf_counter() - t0)
    t = chain.last_timings()
    per = {k: acc[k] / a.steps for k in acc}
    rec_out = (metrics.records_out() - ro0) // a.steps
    recs = rs.n_records
    res = {"metric": "records/s", "value": recs * ctx.world * a.steps / elapsed, "unit": "records/s",
           "ms_per_step": elapsed / a.steps * 1e3, "scaling": "weak", "dtype": "u8",
           "config": {"workload": name, "description": desc, "records_per_gpu": recs,
                      "batches_per_gpu": rs.n_batches, "slice_bytes_per_gpu": t["in_bytes"],
                      "output_bytes_per_gpu": t["out_bytes"], "chain": [m[0] for m in modules]},
           "gbps_input": t["in_bytes"] * ctx.world * a.steps / elapsed / 1e9,
           "gbps_pipeline": (t["in_bytes"] + t["out_bytes"]) / (per["total_ms"] * 1e-3) / 1e9,
           "records_out_per_gpu": rec_out,
           "roofline": roofline(per, t, name, recs, rs.n_batches, rec_out, elapsed / a.steps * 1e3),
           "kernel_ms": per, "setup_s": {"generate": gen_s, "ingest_h2d": ingest_s},
           "crc_verify": {"ms": vms, "gbps": t["in_bytes"] / (vms * 1e-3) / 1e9 if vms > 0 else None,
                          "mismatches": vbad,
                          "note": "k_verify_crc: CRC32C of every stored batch vs its header, on ingest, outside "
                                  "the timed step (the reference never verifies)"}}
    if rs.device_framed:
        # fetch-shaped step: a fresh slice in HBM each step (as read from the
        # log), so the per-fetch work is inside the timed region: device batch
        # framing, CRC32C verify of every stored batch, then the same process
        # (the verify runs on the slice's own stream beside process_batch:
        # both only read the stored bytes; its result is collected per step)
        fbad = 0
        for _ in range(2):
            rs.reframe()
            rs.verify_crc_start()
            chain.process_slice(rs, metrics=metrics, download=False)
            fbad += rs.verify_crc()[0]
        ctx.barrier()
        fsteps = max(3, a.steps // 2)
        t0 = time.perf_counter()
        for _ in range(fsteps):
            rs.reframe()
            rs.verify_crc_start()
            chain.process_slice(rs, metrics=metrics, download=False)
            fbad += rs.verify_crc()[0]
        ctx.barrier()
        fe = ctx.max_over_ranks(time.perf_counter() - t0) / fsteps
        res["fetch"] = {"value": recs * ctx.world / fe, "unit": "records/s", "ms_per_step": fe * 1e3,
                        "steps": fsteps, "crc_mismatches": fbad,
                        "includes": "per step on the HBM-resident slice: device batch framing (k_frame_*), "
                                    "CRC32C verify of every stored batch (k_verify_crc, on its own stream "
                                    "beside process_batch), process_batch (eval, plan, write, CRC of the "
                                    "output); the step ends when both are done"}
    if not a.no_e2e:
        # end to end at the C ABI (what the SPU's FFI sees): host slice -> H2D
        # ingest + device framing -> the same process_batch -> D2H of the output
        # batch into a library-owned host buffer (fsg_chain_process_batch)
        from fluvio_amd import _ffi
        lib = _ffi.lib()
        src = np.ascontiguousarray(sl_bytes, dtype=np.uint8)
        sp = ctypes.cast(ctypes.c_void_p(src.ctypes.data), ctypes.c_char_p)

        def abi_call():
            o = ctypes.POINTER(_ffi.fsg_batch_output)()
            rc = lib.fsg_chain_process_batch(chain._h, sp, src.nbytes, (1 << 64) - 1, None, ctypes.byref(o))
            if rc:
                raise RuntimeError(_ffi.last_error())
            n = o.contents.batch_len
            lib.fsg_batch_output_free(o)
            return n

        abi_call()
        ctx.barrier()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            n_out = abi_call()
        ctx.barrier()
        e2e = ctx.max_over_ranks(time.perf_counter() - t0) / reps
        # the Python binding on top: bytes in, bytes out (one more host copy each way)
        raw = sl_bytes.tobytes()
        t0 = time.perf_counter()
        out = chain.process_batch(raw)
        py_s = time.perf_counter() - t0
        assert len(out.raw) == n_out
        chunks = chain.last_timings()["chunks"]
        res["e2e"] = {"value": recs * ctx.world / e2e, "unit": "records/s", "ms_per_step": e2e * 1e3,
                      "gbps_h2d_plus_d2h": (src.nbytes + n_out) / e2e / 1e9,
                      "includes": "fsg_chain_process_batch: H2D of the slice (pageable host memory), device "
                                  "batch framing, the GPU process_batch, D2H of the output batch into host "
                                  "memory; pipelined over `chunks` slice chunks (upload of one piece, processing "
                                  "of chunk k, download of chunk k-1 overlap; 0 = serial)",
                      "chunks": chunks, "output_bytes": n_out, "python_binding_ms": py_s * 1e3}
        del raw, out, src
    res["cpu_baseline"] = cpu.get(name)
    del rs, chain
    return res


def run_c5(ctx, cpu):
    """C5: topic of 64 partitions, aggregate-sum per partition, partitions sharded
    p -> rank p mod N; per-partition accumulators stay in HBM and are merged with
    one RCCL all-reduce of the 64-slot state vector per step."""
    from fluvio_amd import partitions as PT
    from fluvio_amd import synth
    from fluvio_amd.smartengine import (PartitionState, ResidentSlice, SmartEngine, SmartModuleChainBuilder,
                                        SmartModuleConfig, builtin, comm_unique_id, process_slices)
    a = ctx.a
    P, nrec = C5["partitions"], C5["records_per_partition"]
    engine = SmartEngine(ctx.local)
    uid = comm_unique_id() if ctx.rank == 0 else bytes(128)
    engine.comm_init(ctx.broadcast_bytes(uid, 128), ctx.world, ctx.rank)
    owned = PT.owned_partitions(P, ctx.world, ctx.rank)
    t0 = time.time()
    slices, vsum = {}, {}
    for p in owned:
        slices[p] = synth.make_slice_array(3, nrec, seed=synth.SEEDS[3] + p)
        vsum[p] = synth.last_int_sum()  # the generator's ground truth (no GPU, no oracle)
    gen_s = time.time() - t0
    chains, rsl = {}, {}
    for p in owned:
        b = SmartModuleChainBuilder.default()
        for mname, params, acc in C5["modules"]:
            b.add_smart_module(SmartModuleConfig.builder().params(params).build(), builtin(mname))
        chains[p] = b.initialize(engine)
        rsl[p] = ResidentSlice(engine, slices[p])
    state = PartitionState(engine, P)
    kms = {k: 0.0 for k in PHASES}
    kmax = {k: 0.0 for k in PHASES}
    out_bytes = [0]
    clist, slist = [chains[p] for p in owned], [rsl[p] for p in owned]

    def step():
        process_slices(clist, slist)  # every owned partition's chain in one call, concurrently
        smax = {k: 0.0 for k in PHASES}
        for p in owned:
            state.collect(p, chains[p])
            t = chains[p].last_timings()
            for k in kms:
                kms[k] += t[k]
                smax[k] = max(smax[k], t[k])
            out_bytes[0] += t["out_bytes"]
        for k in kmax:
            kmax[k] += smax[k]
        state.allreduce()  # RCCL sum over xGMI: the topic-wide per-partition table on every rank

    for _ in range(a.warmup):
        step()
    ctx.barrier()
    for k in kms:
        kms[k] = kmax[k] = 0.0
    out_bytes[0] = 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    ctx.barrier()
    elapsed = ctx.max_over_ranks(time.perf_counter() - t0)
    total_recs = sum(rsl[p].n_records for p in owned)
    in_bytes = sum(chains[p].last_timings()["in_bytes"] for p in owned)
    vec = state.read()
    # every partition's accumulator after warmup + steps calls over its slice:
    # (calls x the generator's sum) wrapping i32, checked on the owned slots
    calls = a.warmup + a.steps
    bad = sum(1 for p in owned if vec[p] != PT.wrap_i32(calls * vsum[p]))
    if ctx.dist is not None:
        import torch
        tt = torch.tensor([total_recs, bad], dtype=torch.float64)
        ctx.dist.all_reduce(tt)
        total_recs, bad = int(tt[0].item()), int(tt[1].item())
    assert bad == 0, f"c5-agg-sum: {bad} partition accumulators differ from the generator's sums"
    per = {k: v / a.steps for k, v in kms.items()}
    pmax = {k: v / a.steps for k, v in kmax.items()}
    res = {"metric": "records/s", "value": total_recs * a.steps / elapsed, "unit": "records/s",
           "ms_per_step": elapsed / a.steps * 1e3, "scaling": "strong", "dtype": "i32",
           "config": {"workload": "c5-agg-sum", "description": C5["description"], "partitions": P,
                      "records_per_partition": nrec, "partitions_per_gpu": len(owned),
                      "slice_bytes_this_gpu": in_bytes,
                      "host_call": "fsg_chain_group_process_slices (one call, every owned chain)",
                      "parallelism": f"partitions sharded p -> rank p mod {ctx.world}"},
           "kernel_ms_sum_over_partitions": per,
           "kernel_ms_max_over_partitions": pmax,
           "gbps_input_per_gpu": in_bytes * a.steps / elapsed / 1e9,
           "state_checksum": sum(vec) & 0xFFFFFFFF,
           "state_check": f"ok: all {P} partition accumulators == (warmup + steps) x the generator's sum of the "
                          f"partition's integers (wrapping i32), merged by RCCL all-reduce",
           "setup_s": {"generate": gen_s}}
    # step-level roofline: every owned slice read once, every output batch written
    # once, 4 B of state per partition; the dominant phase by its longest chain
    # (text_ms holds no kernel of aggregate-sum: the plan read-back and the header)
    dom = max(pmax, key=lambda k: pmax[k] if k not in ("total_ms", "text_ms") else -1.0)
    res["roofline"] = roofline_step(in_bytes + out_bytes[0] / a.steps + 4 * len(owned), res["ms_per_step"],
                                    PHASE_KERNEL[dom], pmax[dom],
                                    "c5-agg-sum: input + output bytes of all owned partitions per step / ms_per_step; "
                                    "the partitions' chains run concurrently (one group call)")
    res["cpu_baseline"] = cpu.get("c5-agg-sum")
    return res


def run_c5k(ctx, cpu):
    """C5 keyed: 64 partitions of {"repo-NNNN": n} records (key = repo name,
    SipHash-routed), aggregate-json per partition (every output record = the
    partition's whole map, keys in the guest HashMap's order), partitions
    sharded p -> rank p mod N.  Per step: every owned partition's slice through
    its chain (one group call: the order walks of all chains in one launch,
    k_aggj_order_group), then the topic-wide per-key totals through the C ABI
    (fsg_keyed_collect per chain: exact key bytes into the rank's table;
    fsg_keyed_allreduce: RCCL all-gather of the key lists, the union
    dictionary, one dense u32 all-reduce)."""
    import torch
    from fluvio_amd import partitions as PT
    from fluvio_amd import synth
    from fluvio_amd.smartengine import (KeyedState, ResidentSlice, SmartEngine, SmartModuleChainBuilder,
                                        SmartModuleConfig, builtin, comm_unique_id, process_slices)
    a = ctx.a
    P, nrec = C5K["partitions"], C5K["records_per_partition"]
    engine = SmartEngine(ctx.local)
    uid = comm_unique_id() if ctx.rank == 0 else bytes(128)
    engine.comm_init(ctx.broadcast_bytes(uid, 128), ctx.world, ctx.rank)
    owned = PT.owned_partitions(P, ctx.world, ctx.rank)
    t0 = time.time()
    ksum = {}
    raw = synth.make_keyed_slices(P, nrec, C5K["keys"], owned=owned, key_sums=ksum)
    gen_s = time.time() - t0
    chains, rsl = {}, {}
    for p in owned:
        b = SmartModuleChainBuilder.default()
        b.set_store_memory_limit(64 << 30)
        for mname, params, acc in C5K["modules"]:
            b.add_smart_module(SmartModuleConfig.builder().params(params).build(), builtin(mname))
        chains[p] = b.initialize(engine)
        rsl[p] = ResidentSlice(engine, raw[p])
    del raw
    keyed = KeyedState(engine)
    kms = {k: 0.0 for k in PHASES + ("order_ms",)}
    kmax = {k: 0.0 for k in PHASES + ("order_ms",)}
    out_bytes = [0]
    clist, slist = [chains[p] for p in owned], [rsl[p] for p in owned]

    def step():
        # every owned partition's chain in one call (fsg_chain_group_process_slices:
        # the chains run concurrently, their aggregate-json order walks as one launch)
        process_slices(clist, slist)
        smax = {k: 0.0 for k in kmax}
        for c in clist:
            t = c.last_timings()
            for k in kms:
                kms[k] += t[k]
                smax[k] = max(smax[k], t[k])
            out_bytes[0] += t["out_bytes"]
        for k in kmax:
            kmax[k] += smax[k]
        # the topic-wide totals: every owned partition's map (exact keys, in HBM)
        # into the rank's table, then the union dictionary + dense u32 all-reduce over RCCL
        keyed.reset()
        for p in owned:
            keyed.collect(chains[p])
        keyed.allreduce()

    for _ in range(a.warmup):
        step()
    ctx.barrier()
    for k in kms:
        kms[k] = kmax[k] = 0.0
    out_bytes[0] = 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    ctx.barrier()
    elapsed = ctx.max_over_ranks(time.perf_counter() - t0)
    total_recs = sum(rsl[p].n_records for p in owned)
    in_bytes = sum(chains[p].last_timings()["in_bytes"] for p in owned)
    merged = keyed.read()
    # the keys this rank's partitions own (SipHash routing: each key in one
    # partition): topic total == (warmup + steps) x the generator's sum, u32 wrapping
    calls = a.warmup + a.steps
    bad = sum(1 for k, v in ksum.items() if merged.get(k) != (calls * v) & 0xFFFFFFFF)
    nkeys_owned = len(ksum)
    if ctx.dist is not None:
        tt = torch.tensor([total_recs, bad, nkeys_owned], dtype=torch.float64)
        ctx.dist.all_reduce(tt)
        total_recs, bad, nkeys_owned = int(tt[0].item()), int(tt[1].item()), int(tt[2].item())
    assert bad == 0 and len(merged) == nkeys_owned, \
        f"c5-keyed-agg: {bad} keyed totals differ from the generator's sums ({len(merged)} vs {nkeys_owned} keys)"
    per = {k: v / a.steps for k, v in kms.items()}
    pmax = {k: v / a.steps for k, v in kmax.items()}
    res = {"metric": "records/s", "value": total_recs * a.steps / elapsed, "unit": "records/s",
           "ms_per_step": elapsed / a.steps * 1e3, "scaling": "strong", "dtype": "u32",
           "config": {"workload": "c5-keyed-agg", "description": C5K["description"], "partitions": P,
                      "records_per_partition": nrec, "keys": C5K["keys"], "partitions_per_gpu": len(owned),
                      "slice_bytes_this_gpu": in_bytes, "output_bytes_this_gpu_per_step": out_bytes[0] / a.steps,
                      "host_call": "fsg_chain_group_process_slices (one call, every owned chain)",
                      "chain": [m[0] for m in C5K["modules"]],
                      "parallelism": f"partitions sharded p -> rank p mod {ctx.world}"},
           "kernel_ms_sum_over_partitions": per,
           "kernel_ms_max_over_partitions": pmax,
           "gbps_input_per_gpu": in_bytes * a.steps / elapsed / 1e9,
           "gbps_output_per_gpu": out_bytes[0] / elapsed / 1e9,
           "merged_keys": len(merged), "state_checksum": sum(merged.values()) & 0xFFFFFFFF,
           "state_check": f"ok: all {len(merged)} topic keys == (warmup + steps) x the generator's per-key sums "
                          f"(u32 wrapping), merged through fsg_keyed_* (exact keys, RCCL)",
           "setup_s": {"generate": gen_s}}
    # step-level roofline; the dominant launch is the one order walk of all the
    # rank's chains (k_aggj_order_group), timed with HIP events around it
    res["roofline"] = roofline_step(in_bytes + out_bytes[0] / a.steps, res["ms_per_step"], "k_aggj_order_group",
                                    pmax["order_ms"],
                                    "c5-keyed-agg: input + output bytes of all owned partitions per step / "
                                    "ms_per_step; the serial per-partition order walk (one workgroup per chain, "
                                    "all chains in one launch) is latency-bound, not HBM-bound")
    res["cpu_baseline"] = cpu.get("c5-keyed-agg")
    del rsl, chains
    return res


def run_one_record(ctx, cpu):
    """f3: the producer's one-record path (crates/fluvio/src/producer/mod.rs:430-473
    -> SmartModuleChainInstance::process of one SmartModuleInput): latency of one
    fsg_chain_process call (upload, the kernel chain, download) per record."""
    from fluvio_amd import protocol as P
    from fluvio_amd.smartengine import (SmartEngine, SmartModuleChainBuilder, SmartModuleConfig,
                                        SmartModuleInput, builtin)
    engine = SmartEngine(ctx.local)
    b = SmartModuleChainBuilder.default()
    b.add_smart_module(SmartModuleConfig.builder().param("key", "timeout").build(), builtin("filter_init"))
    chain = b.initialize(engine)
    inp = SmartModuleInput.try_from_records([P.Record.new(b'{"level":"warn","message":"request timeout"}')])
    for _ in range(20):
        chain.process(inp)
    n = 2000
    lat = []
    t0 = time.perf_counter()
    for _ in range(n):
        t1 = time.perf_counter()
        out = chain.process(inp)
        lat.append(time.perf_counter() - t1)
    mean = (time.perf_counter() - t0) / n
    assert len(out.successes) == 1
    lat.sort()
    dt = lat[n // 2]  # p50: one slow call on a shared host does not move it
    return {"metric": "latency per one-record process() call (p50)", "value": dt * 1e6, "unit": "us",
            "higher_is_better": False, "calls": n, "mean_us": mean * 1e6, "p99_us": lat[n * 99 // 100] * 1e6,
            "records_per_s": 1.0 / mean, "ms_per_step": dt * 1e3,
            "scaling": "weak", "dtype": "u8",
            "config": {"workload": "f3-one-record", "chain": ["filter_init"],
                       "description": "fsg_chain_process of a one-record SmartModuleInput (H2D upload, eval, "
                                      "plan with one host sync, write, CRC, D2H of the output)"}, "cpu_baseline": cpu.get("f3-one-record")}


def run_workload(ctx, w, nrec, cpu):
    if w == "f3-one-record":
        return run_one_record(ctx, cpu)
    if w == "c5-keyed-agg":
        return run_c5k(ctx, cpu)
    if w == "c5-agg-sum":
        return run_c5(ctx, cpu)
    return run_filter(ctx, w, nrec, cpu)


def dry_run(ctx):
    """--dry-run: the multi-rank plumbing of the real line without any GPU work
    (each rank's "step" is a short sleep): barrier, timed steps, max over ranks,
    rank 0 prints the line.  The CPU tests run it under --gpus 2."""
    a = ctx.a
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        time.sleep(0.001 * (1 + ctx.rank))
    ctx.barrier()
    elapsed = ctx.max_over_ranks(time.perf_counter() - t0)
    if ctx.rank == 0:
        full = {"metric": "records/sec + achieved HBM GB/s for SmartModule filter chain, 1/2/4/8 MI355X",
                "value": None, "unit": "records/s", "n_gpus": ctx.world, "steps": a.steps,
                "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "none (dry run)",
                "config": {"workload": a.workload, "parallelism": f"partitions sharded over {ctx.world} GPU(s)"}}
        j = json.loads(compact_line(full))
        j.update(dry_run=True, ranks=ctx.world)
        print(json.dumps(j, allow_nan=False, separators=(",", ":")), flush=True)
    if ctx.dist is not None:
        ctx.dist.destroy_process_group()


LINE_MAX = 8192  # the driver parses one stdout line; everything else goes to the detail file


def _finite(v):
    """JSON-safe: NaN / Infinity become null (json.dumps would print bare NaN)."""
    if isinstance(v, float):
        return v if v == v and v not in (float("inf"), float("-inf")) else None
    if isinstance(v, dict):
        return {k: _finite(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_finite(x) for x in v]
    return v


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _rnd(v, nd=4):
    """Significant-digit rounding for the compact line (values stay exact in the detail file)."""
    if isinstance(v, float) and v == v and v not in (float("inf"), float("-inf")) and v != 0.0:
        from math import floor, log10
        return round(v, max(0, nd - 1 - int(floor(log10(abs(v))))))
    if isinstance(v, dict):
        return {k: _rnd(x, nd) for k, x in v.items()}
    return v


def compact_line(full):
    """The ONE line the driver parses (< LINE_MAX bytes, no NaN / Infinity): the
    headline keys, its roofline and cpu_baseline, and per workload a summary
    {value, unit, ms_per_step, roofline {kernel, frac, achieved}, cpu_baseline
    {value, cores}}.  Phases, prose, fetch and e2e details live in the detail file."""
    head = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    out = _pick(full, head)
    cfg = full.get("config") or {}
    out["config"] = _pick(cfg, ("workload", "records_per_gpu", "batches_per_gpu", "slice_bytes_per_gpu",
                                "output_bytes_per_gpu", "chain", "partitions", "records_per_partition",
                                "parallelism"))
    rf = full.get("roofline")
    if rf:
        r = _pick(rf, ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic",
                       "algorithmic_bytes_per_launch", "avg_launch_ms", "priced_on"))
        if isinstance(rf.get("step"), dict):
            r["step_frac"] = rf["step"].get("frac")
        out["roofline"] = r
    cb = full.get("cpu_baseline")
    out["cpu_baseline"] = None if not cb else dict(
        _pick(cb, ("value", "unit", "cores", "kind", "cpu_model")),
        sample=f"{cb.get('cores')} partitions x bounded sample through the scalar C oracle (port); see detail file"
        if cb.get("unit") != "us" else "20000 one-record calls of the scalar C oracle, p50")
    for k in ("fetch", "e2e"):
        if isinstance(full.get(k), dict):
            out[k] = _pick(full[k], ("value", "unit", "ms_per_step"))
    wl = {}
    for name, w in (full.get("workloads") or {}).items():
        s = _pick(w, ("value", "unit", "ms_per_step", "higher_is_better", "scaling", "dtype"))
        if isinstance(w.get("roofline"), dict):
            s["roofline"] = _pick(w["roofline"], ("kernel", "frac", "achieved", "traffic", "priced_on"))
            if isinstance(w["roofline"].get("step"), dict):
                s["roofline"]["step_frac"] = w["roofline"]["step"].get("frac")
        if isinstance(w.get("cpu_baseline"), dict):
            s["cpu_baseline"] = _pick(w["cpu_baseline"], ("value", "unit", "cores", "kind"))
        wl[name] = s
    if wl:
        out["workloads"] = wl
    out["detail"] = "bench_detail.json"
    out = _finite(_rnd(out))
    line = json.dumps(out, allow_nan=False, separators=(",", ":"))
    if len(line) >= LINE_MAX:  # drop per-workload extras before anything the contract names
        for s in out.get("workloads", {}).values():
            for k in ("higher_is_better", "scaling", "dtype"):
                s.pop(k, None)
        out.pop("fetch", None)
        out.pop("e2e", None)
        line = json.dumps(out, allow_nan=False, separators=(",", ":"))
    assert len(line) < LINE_MAX, len(line)
    return line


def main():
    a = parse()
    rc = launch_ranks(a)
    if rc is not None:
        sys.exit(rc)
    ctx = Ctx(a)
    if a.dry_run:
        dry_run(ctx)
        return
    assert ctx.world == a.gpus or (a.gpus == 1 and not any(x.startswith("--gpus") for x in sys.argv[1:])), \
        f"--gpus {a.gpus} but {ctx.world} rank(s)"
    head = a.workload
    extra = [] if a.only else [w for w in EXTRA if w != head]
    cpu = cpu_baselines_first(ctx, [head] + extra)
    line = dict(run_workload(ctx, head, a.records, cpu))
    workloads = {}
    for w in extra:
        # the previous workload's engines, slices and streams go before the next
        # one is timed (their buffers and streams otherwise stay until exit)
        gc.collect()
        workloads[w] = run_workload(ctx, w, 0, cpu)
    if ctx.rank == 0:
        out = {
            "metric": "records/sec + achieved HBM GB/s for SmartModule filter chain, 1/2/4/8 MI355X",
            "value": line["value"],
            "unit": line.get("unit", "records/s"),
            "n_gpus": ctx.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": line["ms_per_step"],
            "higher_is_better": line.get("higher_is_better", True),
            "scaling": line["scaling"],
            "vs_baseline": None,
            "dtype": line["dtype"],
            "data": "synthetic (fluvio_amd/tools/synth.c), HBM-resident batches",
            "config": dict(line["config"], parallelism=f"partitions sharded over {ctx.world} GPU(s)"),
        }
        for k, v in line.items():
            if k not in out and k not in ("metric",):
                out[k] = v
        if workloads:
            out["workloads"] = workloads
        if head == "f3-one-record":  # a latency line, not the headline metric
            out["metric"] = line["metric"]
        with open(a.detail, "w") as fh:
            json.dump(_finite(out), fh, indent=1, allow_nan=False)
        print(compact_line(out), flush=True)
    if ctx.dist is not None:
        ctx.dist.destroy_process_group()


if __name__ == "__main__":
    main()
