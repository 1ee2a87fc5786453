"""GPU: bench.py's exchange on hardware — the device top-K, RCCL's
all_gather_into_tensor (one rank: the collective and its stream ordering,
not the peers' transfers), the gathered rows and the device merge on the
exchange stream beside the scan (tests/gpu_child/exchange_child.py, in a
process of its own because it creates a process group)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_exchange_one_rank_rccl_allgather_and_merge():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    out = subprocess.run([sys.executable, os.path.join(HERE, "gpu_child", "exchange_child.py")],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0 and "exchange ok" in out.stdout, out.stdout[-2000:] + out.stderr[-4000:]
