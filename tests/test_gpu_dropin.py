"""GPU: the drop-in C++ path at scale and the multi-GPU group API.

* lib/main (main.cpp:19-74 contract) on a 100,000-record synthetic FASTA:
  every id:score equal to the oracle's, one GPU and the sharded path
  (--gpus 2 over one device listed twice, SW_DEVICES=0,0) byte-identical;
* sw_group_* through ctypes: a one-device group (one-rank RCCL
  communicator: the ncclAllGather path), a device listed twice (host
  exchange) and, on a multi-GPU box, every distinct device (RCCL over >= 2
  ranks): full scores == sw_scan's, top-K == the oracle's top-K."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, read_query

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(REPO, "scripts"))


@pytest.fixture(scope="module")
def fasta_100k(sw, tmp_path_factory):
    import dropin_scale
    res, offs = sw.synth.database(100_000, shard=4)
    path = str(tmp_path_factory.mktemp("dropin") / "synth100k.fasta")
    dropin_scale.write_fasta(path, res, offs)
    return path, res, offs


def test_main_100k_records_equal_oracle(sw, oracle, fasta_100k):
    import dropin_scale
    path, res, offs = fasta_100k
    q = read_query("P02232")
    q += "/" * (-len(q) % 8)  # SWSolver.cu:267-269
    want = oracle.scan(oracle.encode(q), res, offs, mat=oracle.matrix(), gap_open=2, gap_extend=2, nthreads=16)
    pairs, metrics, out = dropin_scale.run_main("P02232", path)
    assert len(pairs) == 100_000 and len(np.unique(pairs[:, 0])) == 100_000
    got = np.zeros(100_000, dtype=np.int64)
    got[pairs[:, 0]] = pairs[:, 1]
    assert np.array_equal(got, want)
    assert "Num subjects: 100000" in out
    for k in ("parse_s", "flatten_s", "upload_s", "scan_s"):
        assert metrics[k] >= 0
    assert metrics["gpus"] == 1
    env = dict(os.environ, SW_DEVICES="0,0")
    pairs2, m2, _ = dropin_scale.run_main("P02232", path, gpus=2, env=env)
    assert m2["gpus"] == 2
    assert np.array_equal(pairs2, pairs)


def _device_count():
    import torch
    return torch.cuda.device_count()


# one device, one device listed twice / three times (host exchange), and every
# distinct device of the box (2..8: ncclCommInitAll over >= 2 ranks, the
# ncclAllGather path across devices) when it has more than one
_DEVICE_SETS = [[0], [0, 0], [0, 0, 0]] + ([list(range(min(_device_count(), 8)))] if _device_count() >= 2 else [])


@pytest.mark.parametrize("devices", _DEVICE_SETS, ids=lambda d: "dev" + "_".join(map(str, d)))
def test_group_scan_and_topk(sw, oracle, handle, devices):
    res, offs = sw.synth.database(9000, shard=9)
    ids = np.random.default_rng(3).permutation(12000)[:9000].astype(np.int32)
    g = sw.Group(devices)
    distinct = len(set(devices)) == len(devices)
    info = g.info()
    # the communicators are created by the first top-K, not by the group
    assert info.startswith("rccl allgather (communicators" if distinct else "host")
    gdb = g.database(res, offs, ids=ids)
    shards = [gdb.shard(k) for k in range(len(devices))]
    assert sum(s[0] for s in shards) == 9000 and sum(s[1] for s in shards) == int(offs[-1])
    lens = offs[1:] - offs[:-1]
    assert max(s[1] for s in shards) - min(s[1] for s in shards) <= lens.max()
    q = sw.encode(read_query("P07327"))
    m = sw.capi.builtin_matrix(1)
    db = sw.Database(handle, res, offs, ids=ids)
    want_full = db.scan(q, m, 12, 1)
    assert np.array_equal(gdb.scan(q, m, 12, 1), want_full)
    want = oracle.scan(q, res, offs, mat=m, gap_open=12, gap_extend=1)
    assert np.array_equal(want_full[ids], want)
    for k in (1, 100, 4096):
        keys = gdb.topk(q, k, m, 12, 1)
        assert np.array_equal(keys, sw.dist.local_topk(want, ids, k)), k
    if distinct:
        n = len(devices)
        assert g.info() == "rccl allgather (%d rank%s)" % (n, "" if n == 1 else "s"), g.info()
    gdb.close()
    db.close()
    g.close()


def test_group_distinct_devices_cli(oracle, fasta_100k):
    """main --gpus 2 over two DISTINCT devices: on a box with two or more GPUs
    every id:score equals the oracle's (and the one-GPU output); on a one-GPU
    box it is refused cleanly (no device), never silently served by one GPU."""
    import dropin_scale
    path, res, offs = fasta_100k
    env = dict(os.environ)
    env.pop("SW_DEVICES", None)
    lib = os.path.join(REPO, "ece1782-smith-waterman-cuda_amd", "lib", "main")
    qf = os.path.join(REPO, "tests", "golden", "queries", "P02232.fasta")
    if _device_count() >= 2:
        q = read_query("P02232")
        q += "/" * (-len(q) % 8)  # SWSolver.cu:267-269
        want = oracle.scan(oracle.encode(q), res, offs, mat=oracle.matrix(), gap_open=2, gap_extend=2, nthreads=16)
        pairs, metrics, _ = dropin_scale.run_main("P02232", path, gpus=2, env=env)
        assert metrics["gpus"] == 2
        got = np.zeros(len(offs) - 1, dtype=np.int64)
        got[pairs[:, 0]] = pairs[:, 1]
        assert np.array_equal(got, want)
        return
    out = subprocess.run([lib, "--query", qf, "--db", path, "--gpus", "2"], capture_output=True, text=True,
                         env=env, timeout=300)
    assert out.returncode != 0 and "device" in out.stderr


def test_main_100k_headline_scoring_and_topk(sw, oracle, fasta_100k):
    """The headline scoring through the drop-in CLI at scale: main --matrix
    blosum62 --gap-open 12 --gap-extend 1 on 100,000 records equals the
    oracle on every record; --topk 100 prints the oracle's top-100 (score
    desc, id asc), one GPU and the sharded path (one device listed twice)."""
    import dropin_scale
    path, res, offs = fasta_100k
    m = sw.capi.builtin_matrix(1)
    q = oracle.encode(read_query("P07327"))  # not padded: a chosen scoring scans the query as written
    want = oracle.scan(q, res, offs, mat=m, gap_open=12, gap_extend=1, nthreads=16)
    flags = ["--matrix", "blosum62", "--gap-open", "12", "--gap-extend", "1"]
    pairs, _, _ = dropin_scale.run_main("P07327", path, extra=flags)
    got = np.zeros(100_000, dtype=np.int64)
    got[pairs[:, 0]] = pairs[:, 1]
    assert len(pairs) == 100_000 and np.array_equal(got, want)
    order = np.lexsort((np.arange(len(want)), -want.astype(np.int64)))[:100]
    top = np.stack([order, want[order]], axis=1)
    for gpus, env in ((1, None), (2, dict(os.environ, SW_DEVICES="0,0"))):
        tp, m2, _ = dropin_scale.run_main("P07327", path, gpus=gpus, env=env, extra=flags + ["--topk", "100"])
        assert m2["gpus"] == gpus and np.array_equal(tp, top), gpus


def test_scan_topk_ranks_result_ids(sw, oracle, handle):
    """sw_scan_topk: the device top-K over the database's result ids only
    (custom ids with gaps: unmapped score slots never appear), k beyond the
    database padded with INT64_MIN, ties by id ascending."""
    res, offs = sw.synth.database(3000, shard=17)
    ids = np.random.default_rng(5).permutation(9000)[:3000].astype(np.int32)
    db = sw.Database(handle, res, offs, ids=ids)
    q = sw.encode(read_query("P02232"))
    for mat, go, ge in ((None, 2, 2), (sw.capi.builtin_matrix(1), 12, 1)):
        m = mat if mat is not None else sw.capi.builtin_matrix(0)
        want = oracle.scan(q, res, offs, mat=m, gap_open=go, gap_extend=ge, nthreads=16)
        for k in (1, 64, 3000, 4096):
            keys = db.scan_topk(q, k, mat, go, ge)
            assert np.array_equal(keys, sw.dist.local_topk(want, ids, k) if k <= 3000 else
                                  np.concatenate([sw.dist.local_topk(want, ids, 3000),
                                                  np.full(k - 3000, np.iinfo(np.int64).min)])), k
    db.close()
