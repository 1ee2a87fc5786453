"""The in-tree build (csrc/Makefile, driven by __graft_entry__.build()):
every object that compiles a header's code is rebuilt when that header
changes.  Round 3 lost GPU time to a stale library: sw_intra_x2.h (the intra
kernel body, also compiled into the merged launch in sw_inter_x2.hip) was
missing from the dependencies, so header-only edits did not rebuild.
`make -n -W FILE` lists what a newer FILE would rebuild without touching
anything."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "ece1782-smith-waterman-cuda_amd", "csrc")

# header -> the objects whose translation units include it
INCLUDERS = {
    "sw_intra_x2.h": {"sw_intra_x2.o", "sw_inter_x2.o"},
    "sw_kernels.h": {"sw_kernels.o", "sw_inter_x2.o", "sw_intra_x2.o", "sw_align.o", "sw_synth.o",
                     "sw_profile.o", "sw_topk.o", "sw_capi.o", "sw_group.o"},
}


def would_rebuild(header):
    out = subprocess.run(["make", "-n", "-C", CSRC, "ARCH=gfx950", "-W", os.path.join(CSRC, header)],
                         check=True, capture_output=True, text=True).stdout
    return set(re.findall(r"-o \S*/(sw_\w+\.o) ", out))


@pytest.mark.skipif(shutil.which("make") is None, reason="no make")
@pytest.mark.parametrize("header", sorted(INCLUDERS))
def test_header_change_rebuilds_its_objects(header):
    assert INCLUDERS[header] <= would_rebuild(header)


def test_includers_table_matches_the_sources():
    # every csrc translation unit that includes a header is listed for it
    for header, objs in INCLUDERS.items():
        for src in os.listdir(CSRC):
            if not src.endswith((".hip", ".cpp")) or src in ("main.cpp", "swsolver.cpp", "sw_tests.cpp"):
                continue
            text = open(os.path.join(CSRC, src)).read()
            direct = '#include "%s"' % header in text
            via_ix2 = header == "sw_kernels.h" and '#include "sw_intra_x2.h"' in text
            if direct or via_ix2:
                assert src.rsplit(".", 1)[0] + ".o" in objs, (header, src)
