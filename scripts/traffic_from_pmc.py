"""Per-launch HBM traffic of each kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE), corrected as MI355X_MICROARCH.md prescribes:
FETCH_SIZE is in KiB and reports half of the bytes of a wide coalesced read on
gfx950 (x2); WRITE_SIZE is in KiB and exact for 16-B/lane streaming stores.

usage: python scripts/traffic_from_pmc.py <pmc dir> <workload> <bench json line file> [<round tag>]
  <pmc dir> holds fetch_<workload>/ and write_<workload>/ (scripts/gpu_prof.sh)
Updates profiles/traffic.json[workload] = {kernel: {read, write, total}} plus
the shape (records, batches) and the kernel-source tag (bench.lib_tag) it was measured on;
bench.py quotes it as roofline.traffic only for that same build and shape.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                vals[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    d, wl, bj = sys.argv[1], sys.argv[2], sys.argv[3]
    tag = sys.argv[4] if len(sys.argv) > 4 else os.path.basename(d.rstrip("/"))
    fetch = per_kernel(os.path.join(d, "fetch_" + wl), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "write_" + wl), "WRITE_SIZE")
    line = json.loads(open(bj).read().strip().splitlines()[-1])
    sys.path.insert(0, ROOT)
    import bench
    out = {}
    for k in sorted(set(fetch) | set(write)):
        if "rocclr" in k:
            continue
        rd = fetch.get(k, 0.0) * 1024 * 2
        wr = write.get(k, 0.0) * 1024
        out[k] = {"read": rd, "write": wr, "total": rd + wr}
    path = os.path.join(ROOT, "profiles", "traffic.json")
    db = json.load(open(path)) if os.path.exists(path) else {}
    db[wl] = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, {tag} (FETCH_SIZE x2 gfx950 correction)",
              "kernels": out, "lib": bench.lib_tag(), "n_records": line["config"]["records_per_gpu"],
              "n_batches": line["config"]["batches_per_gpu"]}
    json.dump(db, open(path, "w"), indent=1, sort_keys=True)
    for k, v in out.items():
        print(f"{k:32s} read {v['read']/1e9:8.3f} GB  write {v['write']/1e9:8.3f} GB")


if __name__ == "__main__":
    main()
