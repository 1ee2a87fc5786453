"""GPU: the scan's ranking.  sw_scan_rank_device scans
and ranks in one call; sw_topk_device ranks in ONE launch (sw_topk_fused:
chunks, then the last workgroup to arrive selects and sorts the survivors)
whenever k <= 1,024 and the survivors fit, else by chained stages.  Keys
must equal the oracle's top-K at every k, id form and scan form, and — at
C2's size, where the oracle is too slow — the CPU top-K of the device's own
scores, with the ranking on a second stream beside the next scan as bench.py
runs it (a survivor read before its workgroup published it would differ)."""
import numpy as np
import pytest

from conftest import read_query

pytestmark = pytest.mark.gpu

PAD = np.iinfo(np.int64).min
SCORINGS = [(1, 12, 1), (0, 2, 2)]  # BLOSUM62 11/1 affine (the headline), the reference's BLOSUM50 linear 2


def _padded(keys, k):
    return np.concatenate([keys, np.full(k - len(keys), PAD, dtype=np.int64)]) if len(keys) < k else keys


@pytest.fixture(scope="module")
def small_db(sw):
    return sw.synth.database(8000, shard=31)


@pytest.fixture
def merged(knobs):
    """The merged launch on the small database: its wave pairs from 64
    columns (C2's widths are far above the library's cut), the fp16-first
    chain kept (the adaptive routing never moves work out of the launch)."""
    knobs(lpt="1", pair_width="64", inter_i16_span="0", intra_i16_first="0")


def _rank(sw, db, q, k, m, go, ge, gids=None, id_base=0):
    import torch
    dev = torch.device("cuda", 0)
    scores = torch.full((db.n_out,), -7, dtype=torch.int32, device=dev)
    keys = torch.zeros(k, dtype=torch.int64, device=dev)
    g = torch.from_numpy(gids).to(dev) if gids is not None else None
    db.scan_rank_device(q, scores.data_ptr(), k, keys.data_ptr(), m, go, ge,
                        gids_dev_ptr=(g.data_ptr() if g is not None else None), id_base=id_base)
    torch.cuda.synchronize()
    return keys.cpu().numpy(), scores.cpu().numpy()


@pytest.mark.parametrize("scoring", SCORINGS)
def test_scan_rank_equals_oracle(sw, oracle, handle, merged, small_db, scoring):
    """The merged launch's scores ranked at k from 1 to 2,000 (one launch up
    to 1,024, chained stages past it), with ids offset and mapped."""
    mid, go, ge = scoring
    res, offs = small_db
    n = len(offs) - 1
    ids = np.arange(n, dtype=np.int32)
    m = sw.capi.builtin_matrix(mid)
    db = sw.Database(handle, res, offs)
    gids = np.random.default_rng(3).permutation(3 * n)[:n].astype(np.int32)
    for L, shard in ((375, 50), (120, 51)):
        q = sw.synth.query(L, shard=shard)
        want = oracle.scan(q, res, offs, mat=m, gap_open=go, gap_extend=ge, nthreads=16)
        for k in (1, 7, 100, 1024, 2000):
            keys, _ = _rank(sw, db, q, k, m, go, ge)
            assert "+lpt" in handle.last_kernel(), handle.last_kernel()
            assert np.array_equal(keys, sw.dist.local_topk(want, ids, k)), (L, k)
        keys, _ = _rank(sw, db, q, 64, m, go, ge, id_base=12345)
        assert np.array_equal(keys, sw.dist.local_topk(want, ids + 12345, 64))
        keys, _ = _rank(sw, db, q, 64, m, go, ge, gids=gids)
        assert np.array_equal(keys, sw.dist.local_topk(want, gids, 64))
    db.close()


def test_scan_rank_other_scan_forms(sw, oracle, handle, knobs, small_db):
    """Scans that do not run as the merged launch (sw_opts lpt 0; the int32
    forms) rank the same keys."""
    res, offs = small_db
    ids = np.arange(len(offs) - 1, dtype=np.int32)
    db = sw.Database(handle, res, offs)
    q = sw.encode(read_query("P02232"))
    m = sw.capi.builtin_matrix(1)
    want = oracle.scan(q, res, offs, mat=m, gap_open=12, gap_extend=1, nthreads=16)
    knobs(lpt=0)
    keys, _ = _rank(sw, db, q, 100, m, 12, 1)
    assert "+lpt" not in handle.last_kernel()
    assert np.array_equal(keys, sw.dist.local_topk(want, ids, 100))
    knobs(lpt=-1, int16_guard=0, inter_variant="32x8", intra_x2=0)
    keys, _ = _rank(sw, db, q, 100, m, 12, 1)
    assert np.array_equal(keys, sw.dist.local_topk(want, ids, 100))
    db.close()


def test_scan_rank_custom_result_ids_and_empty_query(sw, oracle, handle, merged):
    """A database with its own result ids (gaps between them): the ranking
    runs over the subjects' ids only (unmapped score slots hold garbage and
    never appear); k past the database pads with INT64_MIN; an empty query
    ranks all-zero scores by id."""
    res, offs = sw.synth.database(3000, shard=17)
    n = len(offs) - 1
    ids = np.random.default_rng(5).permutation(9000)[:n].astype(np.int32)
    db = sw.Database(handle, res, offs, ids=ids)
    q = sw.encode(read_query("P02232"))
    m = sw.capi.builtin_matrix(1)
    want = oracle.scan(q, res, offs, mat=m, gap_open=12, gap_extend=1, nthreads=16)
    for k in (1, 64, 1024):
        keys, _ = _rank(sw, db, q, k, m, 12, 1)
        assert np.array_equal(keys, sw.dist.local_topk(want, ids, k)), k
    keys, _ = _rank(sw, db, q, n + 50, m, 12, 1)  # k beyond the database: INT64_MIN after the n keys
    assert np.array_equal(keys, _padded(sw.dist.local_topk(want, ids, n), n + 50))
    keys, _ = _rank(sw, db, np.zeros(0, dtype=np.uint8), 10, m, 12, 1)
    assert np.array_equal(keys, sw.dist.local_topk(np.zeros(n, dtype=np.int32), ids, 10))
    db.close()


@pytest.mark.parametrize("n", [1, 4096, 4097, 8191, 65536, 65537, 524288, 570000, 2_000_000])
@pytest.mark.parametrize("k", [1, 100, 1024, 1025])
def test_topk_one_launch_sizes(sw, handle, n, k):
    """sw_topk_device around the one-launch plan's edges (one chunk; 4,096-
    and 8,192-key chunks; survivors up to 8,192; k past 1,024 chained),
    many equal scores (ties broken by id), twice on one workspace (the
    counter the last workgroup resets)."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(n + k)
    s = rng.integers(0, 60, n).astype(np.int32)
    d = torch.from_numpy(s).to(dev)
    for rep in range(2):
        out = torch.zeros(k, dtype=torch.int64, device=dev)
        handle.topk_device(d.data_ptr(), n, k, out.data_ptr(), id_base=rep)
        torch.cuda.synchronize()
        want = _padded(sw.dist.local_topk(s, np.arange(n, dtype=np.int32) + rep, k), k)
        assert np.array_equal(out.cpu().numpy(), want), (n, k, rep)


@pytest.mark.parametrize("scoring", SCORINGS)
def test_rank_beside_next_scan_c2_size(sw, handle, scoring):
    """C2's database (570,000 synthetic subjects, generated in HBM) scanned
    back to back with alternating queries into a ring of score buffers; each
    step's top-K runs on a second handle and stream beside the next scan, as
    bench.py's exchange does (70 chunks of 8,192 in one launch).  Every
    step's keys equal the CPU top-K of that step's own scores; the steps
    that repeat a query repeat its keys."""
    import torch
    mid, go, ge = scoring
    dev = torch.device("cuda", 0)
    db = sw.Database.synthetic(handle, 1782, 570000)
    n = db.n_out
    m = sw.capi.builtin_matrix(mid)
    stream = torch.cuda.Stream(dev)
    handle.set_stream(stream.cuda_stream)
    xstream = torch.cuda.Stream(dev, priority=-1)
    xh = sw.Handle(0, env_opts=False)
    xh.set_stream(xstream.cuda_stream)
    qs = [sw.encode(read_query("P07327")), sw.synth.query(250, shard=77)]
    K, NB, steps = 100, 3, 8
    bufs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(NB)]
    keys = [torch.zeros(K, dtype=torch.int64, device=dev) for _ in range(steps)]
    ranked = [torch.cuda.Event() for _ in range(NB)]
    try:
        for i in range(steps):
            b = i % NB
            if i >= NB:
                stream.wait_event(ranked[b])
            db.scan_device(qs[i % 2], bufs[b].data_ptr(), m, go, ge)
            handle.stream_wait_scan(xstream.cuda_stream)
            xh.topk_device(bufs[b].data_ptr(), n, K, keys[i].data_ptr())
            ranked[b].record(xstream)
        torch.cuda.synchronize()
        for i in range(steps - NB, steps):  # buffers not rewritten after their step
            s = bufs[i % NB].cpu().numpy()
            assert np.array_equal(keys[i].cpu().numpy(), sw.dist.local_topk(s, np.arange(n, dtype=np.int32), K)), i
        for i in range(steps - 2):
            assert np.array_equal(keys[i].cpu().numpy(), keys[i + 2].cpu().numpy()), i
    finally:
        torch.cuda.synchronize()
        handle.set_stream(None)
        xh.close()
        db.close()
