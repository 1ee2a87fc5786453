"""GPU: sw_scan_rank_device — a scan and the device top-K of its scores in one
call (the ranking no longer queues behind the next scan).
When the scan runs as the merged launch its last workgroups rank the scores
inside that launch (sw_rank.h rank_tail; sw_last_kernel ends "+rank"); other
scan forms, and rankings too large for the tail, rank by a top-K launch after
the scan.  Keys must equal the oracle's top-K of the same query at every k,
id form and kernel form, and — at C2's size, where the oracle is too slow —
the CPU top-K of the device's own scores (a ranking that read a score before
its workgroup published it would differ: every scan rewrites every score)."""
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


@pytest.fixture
def merged(knobs):
    """The merged launch on the small database: its wave pairs from 64
    columns (C2's widths are far above the library's cut), the fp16-first
    chain kept (the adaptive routing never moves work out of the launch)."""
    knobs(lpt="1", pair_width="64", inter_i16_span="0", intra_i16_first="0")


@pytest.mark.parametrize("scoring", SCORINGS)
def test_rank_in_merged_launch_equals_oracle(sw, oracle, handle, merged, small_db, scoring):
    mid, go, ge = scoring
    res, offs = small_db
    n = len(offs) - 1
    m = sw.capi.builtin_matrix(mid)
    db = sw.Database(handle, res, offs)
    gids = np.random.default_rng(3).permutation(3 * n)[:n].astype(np.int32)
    for L, shard in ((375, 50), (120, 51)):
        q = sw.synth.query(L, shard=shard)
        want = oracle.scan(q, res, offs, mat=m, gap_open=go, gap_extend=ge, nthreads=16)
        for k in (1, 7, 100, 1024):
            keys, _ = _rank(sw, db, q, k, m, go, ge)
            assert handle.last_kernel().endswith("+rank"), handle.last_kernel()
            assert np.array_equal(keys, sw.dist.local_topk(want, np.arange(n, dtype=np.int32), k)), (L, k)
        keys, _ = _rank(sw, db, q, 64, m, go, ge, id_base=12345)
        assert np.array_equal(keys, sw.dist.local_topk(want, np.arange(n, dtype=np.int32) + 12345, 64))
        keys, _ = _rank(sw, db, q, 64, m, go, ge, gids=gids)
        assert handle.last_kernel().endswith("+rank")
        assert np.array_equal(keys, sw.dist.local_topk(want, gids, 64))
    db.close()


def test_rank_fallback_forms_equal_oracle(sw, oracle, handle, merged, knobs, small_db):
    """k past the tail's limit (kRankMaxK 1,024), and scans that do not run
    as the merged launch (sw_opts lpt 0; an int32-only scoring), rank by a
    top-K launch after the scan: the same keys."""
    res, offs = small_db
    n = len(offs) - 1
    ids = np.arange(n, dtype=np.int32)
    db = sw.Database(handle, res, offs)
    q = sw.encode(read_query("P02232"))
    m = sw.capi.builtin_matrix(1)
    want = oracle.scan(q, res, offs, mat=m, gap_open=12, gap_extend=1, nthreads=16)
    keys, _ = _rank(sw, db, q, 2000, m, 12, 1)
    assert not handle.last_kernel().endswith("+rank")
    assert np.array_equal(keys, sw.dist.local_topk(want, ids, 2000))
    knobs(lpt=0)
    keys, _ = _rank(sw, db, q, 100, m, 12, 1)
    assert "+lpt" not in handle.last_kernel()
    assert np.array_equal(keys, sw.dist.local_topk(want, ids, 100))
    knobs(lpt=-1, int16_guard=0, inter_variant="32x8", intra_x2=0)
    keys, _ = _rank(sw, db, q, 100, m, 12, 1)
    assert np.array_equal(keys, sw.dist.local_topk(want, ids, 100))
    db.close()


def test_rank_custom_result_ids_and_empty_query(sw, oracle, handle, merged):
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
        assert handle.last_kernel().endswith("+rank"), handle.last_kernel()
        assert np.array_equal(keys, sw.dist.local_topk(want, ids, k)), k
    keys, _ = _rank(sw, db, q, n + 50, m, 12, 1)  # k beyond the database: INT64_MIN after the n keys
    assert np.array_equal(keys, _padded(sw.dist.local_topk(want, ids, n), n + 50))
    keys, _ = _rank(sw, db, np.zeros(0, dtype=np.uint8), 10, m, 12, 1)
    assert np.array_equal(keys, sw.dist.local_topk(np.zeros(n, dtype=np.int32), ids, 10))
    db.close()


@pytest.mark.parametrize("scoring", SCORINGS)
def test_rank_back_to_back_c2_size(sw, handle, scoring):
    """C2's database (570,000 synthetic subjects, generated in HBM) scanned
    back to back with alternating queries into two score buffers, ranked in
    each scan's launch: every step's keys equal the CPU top-K of that step's
    own scores (the affine scans rank in the launch's tail, the linear ones
    — C2's size takes two launches under linear gaps — after it; the tail
    reads every workgroup's scores through the
    device-scope release / acquire pairs; a stale read would show the other
    query's scores); the steps that repeat a query repeat its keys."""
    import torch
    mid, go, ge = scoring
    dev = torch.device("cuda", 0)
    db = sw.Database.synthetic(handle, 1782, 570000)
    n = db.n_out
    m = sw.capi.builtin_matrix(mid)
    qs = [sw.encode(read_query("P07327")), sw.synth.query(250, shard=77)]
    K = 100
    bufs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
    keys = [torch.zeros(K, dtype=torch.int64, device=dev) for _ in range(6)]
    for i in range(6):
        db.scan_rank_device(qs[i % 2], bufs[i % 2].data_ptr(), K, keys[i].data_ptr(), m, go, ge)
        if i >= 4:  # the last two steps: their buffers are not rewritten afterwards
            torch.cuda.synchronize()
            s = bufs[i % 2].cpu().numpy()
            assert np.array_equal(keys[i].cpu().numpy(), sw.dist.local_topk(s, np.arange(n, dtype=np.int32), K)), i
    assert handle.last_kernel().endswith("+rank") == (go != ge), handle.last_kernel()
    for i in range(4):  # same query, same keys
        assert np.array_equal(keys[i].cpu().numpy(), keys[i + 2].cpu().numpy()), i
    db.close()
