"""The merged launch's work table (csrc/sw_plan.cpp lpt_plan) against the
kernel's decoding of it (sw_inter_x2.hip x2p_wg, sw_intra_x2.h's pipelined
pair ranges), on the CPU: tests/native/plan_check.cpp builds tables for C2's
1/8-share shape under both scorings and for edge mixes (more tri groups than
single-wave blocks, tail pairs beside tris, pipelined pairs at both ends, every
pair pipelined, no long subjects) and checks that every 64-subject block and
every long-subject pair is scanned by exactly one entry and that the table is
longest first."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ece1782-smith-waterman-cuda_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(shutil.which(HIPCC) is None, reason="hipcc not found")
def test_lpt_table_covers_every_block_and_pair_once(tmp_path):
    exe = str(tmp_path / "plan_check")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-std=c++17", "-Wall", "-I" + CSRC,
                    "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "native", "plan_check.cpp"),
                    os.path.join(CSRC, "sw_plan.cpp"), "-o", exe], check=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.rstrip().endswith("plan_check ok"), r.stdout + r.stderr
    # the 1/8 share's tri table: 275 tri workgroups with spare waves, 4 pipelined pairs
    assert "share8-affine-tri: 888 entries, npipe 4, pipe_tail 1561 of 1561 pairs, spares 275" in r.stdout
    # linear scans of quad databases pipeline their last 2 % of pairs (to 8)
    assert "share8-linear-tailpipe: 895 entries, npipe 4, pipe_tail 1529 of 1561 pairs" in r.stdout
