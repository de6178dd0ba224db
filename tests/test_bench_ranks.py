"""bench.py's multi-GPU contract on the CPU (no GPU work): `--gpus N` without a
launcher starts N ranks under torch.distributed.run, the line reports
n_gpus == N, and a launcher whose WORLD_SIZE disagrees with --gpus is refused.
The GPU path is the same code past the rank plumbing (`--dry-run` stops there)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                          "MASTER_PORT")}
    e.update(kw)
    return e


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_2_launches_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    j = _line(r.stdout)
    assert j["n_gpus"] == 2 and j["ranks"] == 2
    # max over ranks: rank 1 sleeps 2 ms a step, rank 0 1 ms
    assert j["ms_per_step"] >= 2.0


def test_gpus_1_default():
    r = subprocess.run([sys.executable, BENCH, "--dry-run", "--steps", "2"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert _line(r.stdout)["n_gpus"] == 1


def test_world_size_mismatch_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run", "--steps", "1"], capture_output=True,
                       text=True, timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr
