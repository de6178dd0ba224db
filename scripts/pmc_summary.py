"""Summarise rocprofv3 counter CSVs: per kernel, mean counter value per dispatch and per wave."""
import collections, csv, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:34]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f)
    for k, d in agg.items():
        if "rocclr" in k:
            continue
        m = {c: sum(v) / len(v) for c, v in d.items()}
        w = m.get("SQ_WAVES", 0) or 1
        extra = {c.replace("SQ_", ""): round(v / w, 1) for c, v in m.items() if c.startswith("SQ_INSTS")}
        print(f"  {k:36s} " + " ".join(f"{c}={v:.4g}" for c, v in m.items()) + (f"  per-wave {extra}" if "SQ_WAVES" in m else ""))
for f in sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)):
    print(f)
    for r in csv.DictReader(open(f)):
        if "rocclr" not in r["Name"]:
            print(f"  {r['Name'].replace('(anonymous namespace)::', '').split('(')[0][:34]:36s} calls={r['Calls']} avg_us={float(r['AverageNs'])/1000:.1f}")
