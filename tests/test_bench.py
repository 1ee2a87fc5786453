"""CPU: bench.py's JSON contract on the one configuration that runs without a
GPU (--config c1 --no-gpu: BASELINE configs[0], the CPU path; the oracle at
one thread and all cores, cpu.cpp's own build beside it when present)."""
import json
import os
import subprocess
import sys

import numpy as np

from conftest import REPO

CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")


def test_bench_refuses_world_size_mismatch():
    """--gpus N under a torchrun environment of another size exits non-zero
    (before importing torch or touching a GPU) instead of measuring one rank."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"],
                         capture_output=True, text=True, timeout=120, cwd=REPO, env=env)
    assert out.returncode != 0
    assert "WORLD_SIZE 1" in out.stderr and out.stdout.strip() == ""


def test_bench_check_world():
    sys.path.insert(0, REPO)
    import bench
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == 4
    assert bench.check_world(1, {}) == 1
    for gpus, env in ((8, {}), (2, {"WORLD_SIZE": "8"})):
        try:
            bench.check_world(gpus, env)
        except SystemExit:
            continue
        raise AssertionError("no refusal for --gpus %d, env %s" % (gpus, env))


def test_bench_launches_its_own_ranks(monkeypatch):
    """Without WORLD_SIZE, --gpus N starts ONE torch.distributed.run child with
    N ranks on 127.0.0.1 and relays exactly one JSON line and its exit code."""
    sys.path.insert(0, REPO)
    import bench
    seen = {}

    class FakeProc:
        def __init__(self, cmd, **kw):
            seen["cmd"] = cmd
            self.stdout = iter(['[rank1] chatter\n', '{"metric": "m", "value": 1.0, "n_gpus": 2}\n'])

        def wait(self):
            return 0

    monkeypatch.setattr(bench.subprocess, "Popen", FakeProc)
    rc = bench.launch_ranks(2, ["--gpus", "2", "--backend", "gloo"])
    assert rc == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "2"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "2", "--backend", "gloo"]


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


def test_bench_sustained_object():
    """The `sustained` object of the bench line (back-to-back steps after the
    timed region, outside value): its keys and arithmetic."""
    sys.path.insert(0, REPO)
    import bench
    d = bench.sustained_summary(5.0, 4000, 9.6e9, 4000 * 1.2, 4000, 1)
    for k in ("seconds", "steps", "n_gpus", "value", "unit", "ms_per_step", "kernel_ms_per_scan", "note"):
        assert k in d, k
    assert d["unit"] == "GCUPS" and d["steps"] == 4000
    assert abs(d["value"] - 9.6e9 * 4000 / 5.0 / 1e9) < 0.01
    assert abs(d["ms_per_step"] - 1.25) < 1e-9 and abs(d["kernel_ms_per_scan"] - 1.2) < 1e-9


def test_bench_rendezvous_retry(monkeypatch):
    """A rendezvous port taken between picking and binding:
    the launch is retried once on a new port."""
    sys.path.insert(0, REPO)
    import bench
    calls = []

    class FakeProc:
        def __init__(self, cmd, **kw):
            calls.append(cmd[cmd.index("--master-port") + 1])
            first = len(calls) == 1
            self.stdout = iter(["RuntimeError: Address already in use\n"] if first else
                               ['{"metric": "m", "value": 1.0, "n_gpus": 2}\n'])
            self.rc = 1 if first else 0

        def wait(self):
            return self.rc

    monkeypatch.setattr(bench.subprocess, "Popen", FakeProc)
    assert bench.launch_ranks(2, ["--gpus", "2"]) == 0
    assert len(calls) == 2


def test_bench_valu_roofline_algorithmic():
    """valu_roofline: the algorithmic floor (5 packed ops per cell pair
    affine, 3 linear, 4.25 cycles each, 1,024 SIMDs) beside the kernel's own
    instruction mix (issue_efficiency)."""
    sys.path.insert(0, REPO)
    import bench
    assert abs(bench.algorithmic_peak_gcups(True, 2.4) - 14803.0) < 1.0
    assert abs(bench.algorithmic_peak_gcups(False, 2.4) - 24672.0) < 1.0
    kern = "sw_inter_x2s<32,8,affine,fp16>"
    v = bench.valu_roofline(kern, 7.68e10, 6.93, 11000.0, True, 2.2)
    assert v["bound"] == "valu-issue" and v["unit"] == "GCUPS"
    alg = v["algorithmic"]
    assert alg["floor_packed_ops_per_cell_pair"] == 5 and alg["clock_ghz"] == 2.4
    assert abs(v["achieved"] - 7.68e10 / 6.93e-3 / 1e9) < 0.1
    assert abs(alg["frac"] - v["achieved"] / alg["peak"]) < 1e-3 and v["frac"] == alg["frac"]
    assert abs(alg["peak_under_load"] - bench.algorithmic_peak_gcups(True, 2.2)) < 0.1
    assert alg["frac_under_load"] > alg["frac"]
    ie = v["issue_efficiency"]
    assert ie["peak"] < alg["peak"] and ie["frac"] > alg["frac"]  # the kernel's own mix: more ops than the floor
    lin = bench.valu_roofline("no-such-kernel", 1e10, 1.0, 0.0, False)
    assert lin["algorithmic"]["floor_packed_ops_per_cell_pair"] == 3 and "issue_efficiency" not in lin
    assert lin["algorithmic"]["peak_under_load"] is None


def test_bench_reference_scoring_parity(sw, oracle):
    """The reference-scoring leg's parity: bench.verify
    under BLOSUM50 / linear 2 re-scores the whole (small) share with the
    oracle and passes for the oracle's own scores, fails for one changed
    score; reference_scoring_summary carries the result."""
    sys.path.insert(0, REPO)
    import bench
    res, offs = sw.synth.database(400, shard=0)
    n = len(offs) - 1
    q = sw.encode(bench.read_query("P02232"))
    scoring = (sw.capi.builtin_matrix(0), 2, 2)
    gs = np.stack([oracle.scan(q, res, offs, mat=scoring[0], gap_open=2, gap_extend=2, nthreads=4)])
    gids = np.arange(n, dtype=np.int32)
    K = 10
    top = np.stack([bench._pad_keys(sw.dist.local_topk(gs[0], gids, K), K)])
    sampler = bench.host_sampler(res, offs)
    sampler.full = (res, offs)
    r, ok = bench.verify(sw, sw.dist, 1, 0, [q], sampler, n, gids, gs, top, top, K, scoring, 4, 30.0, "gloo")
    assert ok and r["whole_database"] and r["scores_equal_oracle"] and r["merged_topk_equal"]
    kt = {"scans": 4, "wave_ms": 4.0, "coop_ms": 0.0, "intra_ms": 0.4, "total_ms": 4.4}
    d = bench.reference_scoring_summary(0.5, 1e9, 100, kt, ("k", "i"), 1.5, r, ok)
    assert d["parity"]["scores_equal_oracle"] and d["parity_ok"] is True and d["cold_first_scan_ms"] == 1.5
    assert abs(d["value"] - 1e9 * 100 / 0.5 / 1e9) < 1e-6 and "BLOSUM50" in d["scoring"]
    bad = gs.copy()
    bad[0, n // 2] += 1
    r2, ok2 = bench.verify(sw, sw.dist, 1, 0, [q], sampler, n, gids, bad, top, top, K, scoring, 4, 30.0, "gloo")
    assert not ok2 and not r2["scores_equal_oracle"]


def test_bench_rehearse_exchange_needs_a_share():
    """--rehearse-exchange rehearses the N-rank exchange beside a share's
    scans: without --shard-of it exits non-zero before touching a GPU."""
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--rehearse-exchange"],
                         capture_output=True, text=True, timeout=120, cwd=REPO)
    assert out.returncode != 0 and "--rehearse-exchange needs --shard-of" in out.stderr
    assert out.stdout.strip() == ""
