"""CPU: scripts/share_summary.py, the arithmetic behind the per-rank share
claims: the slowest rank over C2 on the same box and the N-GPU
projection SCALE's own formula gives (all ranks' cells / the slowest rank's
step)."""
import json
import os
import subprocess
import sys

from conftest import REPO


def _line(value, ms, ref_value, ref_ms, subjects=100, residues=1000):
    return json.dumps({"value": value, "ms_per_step": ms, "parity_sample_ok": True,
                       "config": {"subjects_rank0": subjects, "residues_rank0": residues},
                       "reference_scoring": {"value": ref_value, "ms_per_step": ref_ms, "parity_ok": True}})


def test_share_summary(tmp_path):
    d = tmp_path
    (d / "c2_first.json").write_text("noise\n" + _line(1000.0, 8.0, 1500.0, 5.0) + "\n")
    (d / "c2_last.json").write_text(_line(1010.0, 7.9, 1490.0, 5.1) + "\n")
    # two ranks of N = 2: cells per step = value x ms (GCUPS x ms = 1e6 cells)
    (d / "s2_r0.json").write_text(_line(900.0, 4.0, 1400.0, 2.5) + "\n")
    (d / "s2_r1.json").write_text(_line(950.0, 3.9, 1380.0, 2.6) + "\n")
    out = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "share_summary.py"), str(d)],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    s = json.loads(out.stdout)
    assert s["c2_mean"] == {"affine": 1005.0, "reference": 1495.0}
    two = s["shares"]["2"]
    assert two["complete"] and two["ranks"]["0"]["affine"] == 900.0
    aff = two["affine"]
    assert aff["slowest_rank"] == 0 and aff["min"] == 900.0
    assert abs(aff["min_over_c2"] - round(900.0 / 1005.0, 4)) < 1e-9
    want = (900.0 * 4.0 + 950.0 * 3.9) / 4.0  # all cells / the slowest step
    assert abs(aff["projected_value"] - round(want, 1)) < 1e-6
    assert abs(aff["projected_speedup"] - round(round(want, 1) / 1005.0, 3)) < 1e-9
    ref = two["reference"]
    assert ref["slowest_rank"] == 1 and ref["min"] == 1380.0
    assert abs(ref["projected_value"] - round((1400.0 * 2.5 + 1380.0 * 2.6) / 2.6, 1)) < 1e-6
