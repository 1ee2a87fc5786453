"""CPU: bench.py's JSON contract on the one configuration that runs without a
GPU (--config c1 --no-gpu: BASELINE configs[0], the CPU path; the oracle at
one thread and all cores, cpu.cpp's own build beside it when present)."""
import json
import os
import subprocess
import sys

from conftest import REPO

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def test_bench_c1_json_line():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--config", "c1", "--no-gpu"],
                         capture_output=True, text=True, timeout=300, cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, "bench prints ONE JSON line"
    d = json.loads(lines[0])
    for k in CONTRACT:
        assert k in d, k
    assert d["unit"] == "GCUPS" and d["higher_is_better"] is True and d["data"] == "synthetic"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["config"] == "c1" and "workload" in d["config"]
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1
    assert 0 < cb["one_thread"] <= cb["value"] * 1.2
