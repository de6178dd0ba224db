"""bench.py's stdout line is what the driver parses: one JSON line under 8 KB with
no NaN / Infinity, the headline keys, `roofline` and `cpu_baseline`, and a
per-workload summary.  Checked on the full round-5 result (profiles/
r05f_bench_full.json, the 27 KB line the driver could not parse), on a result
with NaN / inf values, and through `bench.py --dry-run`."""
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _strict(line):
    def bad(c):
        raise AssertionError(f"non-finite constant {c} in the line")
    return json.loads(line, parse_constant=bad)


def test_full_round5_result_compacts():
    b = _bench()
    full = json.load(open(os.path.join(ROOT, "profiles", "r05f_bench_full.json")))
    assert len(json.dumps(full)) > 20000  # the shape that broke the driver's parser
    line = b.compact_line(full)
    assert len(line) < 8192 and "\n" not in line
    j = _strict(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config"):
        assert k in j, k
    assert j["value"] == full["value"] or abs(j["value"] / full["value"] - 1) < 1e-3
    r = j["roofline"]
    for k in ("kernel", "achieved", "peak", "frac", "traffic", "algorithmic_bytes_per_launch", "avg_launch_ms"):
        assert k in r, k
    assert abs(r["frac"] - full["roofline"]["frac"]) < 1e-3
    c = j["cpu_baseline"]
    for k in ("value", "cores", "kind", "cpu_model", "sample"):
        assert k in c, k
    assert set(j["workloads"]) == set(full["workloads"])
    for name, w in j["workloads"].items():
        assert "value" in w and "ms_per_step" in w, name
        if name != "f3-one-record":  # a latency line: no bytes to price
            assert "frac" in w["roofline"] and "kernel" in w["roofline"], name
        assert "value" in w["cpu_baseline"], name


def test_non_finite_values_become_null():
    b = _bench()
    full = {"metric": "m", "value": float("nan"), "unit": "records/s", "n_gpus": 1, "steps": 1, "warmup": 0,
            "ms_per_step": float("inf"), "dtype": "u8", "config": {"workload": "w"},
            "roofline": {"kernel": "k", "achieved": float("-inf"), "frac": 0.5, "peak": 8000.0},
            "cpu_baseline": {"value": float("nan"), "cores": 1, "kind": "port", "unit": "records/s"},
            "workloads": {"x": {"value": 1.0, "ms_per_step": float("nan"), "roofline": {"kernel": "k", "frac": 0.1},
                                "cpu_baseline": None}}}
    j = _strict(b.compact_line(full))
    assert j["value"] is None and j["ms_per_step"] is None and j["roofline"]["achieved"] is None
    assert j["workloads"]["x"]["ms_per_step"] is None


def test_dry_run_line_parses():
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "2"],
                       capture_output=True, text=True, timeout=120, env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and len(lines[0]) < 8192
    j = _strict(lines[0])
    assert j["n_gpus"] == 1 and j["dry_run"] is True
