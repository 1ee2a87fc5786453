"""GPU: the merged launch's tail pairs (sw_scan_lpt, x2p_wg's tail range) and
its looped grid.
The narrowest blocks [blk_tail, nblocks) run by wave pairs after the
single-wave range, two blocks per workgroup (sw_opts tail_pairs n: the
narrowest n blocks; by default one round of pair workgroups on databases
whose single-wave workgroups fill the GPU more than twice).  Scores must
equal the oracle's at every pass count (pairs with an idle second wave at 1
pass are not formed), odd and even counts, under both gap models and with
the fp16 guard band flagging tail blocks into the launch's own drain."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCORINGS = [(1, 12, 1), (0, 2, 2)]  # BLOSUM62 11/1 affine (the headline), the reference's BLOSUM50 linear 2


@pytest.fixture(scope="module")
def small_db(sw):
    return sw.synth.database(8000, shard=31)


def _tail_knobs(knobs, n):
    knobs(lpt="1", pair_width="500", inter_i16_span="0", intra_i16_first="0", tail_pairs=str(n))


@pytest.mark.parametrize("scoring", SCORINGS)
@pytest.mark.parametrize("qlen", [120, 375, 440])
def test_tail_pairs_equal_oracle(sw, oracle, handle, knobs, small_db, scoring, qlen):
    """2, 6 and 7 passes; 1, 2, 33 and all but one of the single-wave
    blocks by tail pairs, then none: every scan equals the oracle."""
    mid, go, ge = scoring
    res, offs = small_db
    db = sw.Database(handle, res, offs, long_threshold=2048)
    q = sw.synth.query(qlen, shard=70 + qlen)
    m = sw.capi.builtin_matrix(mid)
    want = oracle.scan(q, res, offs, mat=m, gap_open=go, gap_extend=ge, nthreads=16)
    for n in (1, 2, 33, 10 ** 6):
        _tail_knobs(knobs, n)
        got = db.scan(q, m, go, ge)
        k = handle.last_kernel()
        assert "+lpt" in k and "+tail" in k, (n, k)
        assert np.array_equal(got, want), (n, k, np.nonzero(got != want)[0][:8])
    _tail_knobs(knobs, 0)
    assert np.array_equal(db.scan(q, m, go, ge), want)
    assert "+tail" not in handle.last_kernel()
    db.close()


@pytest.mark.parametrize("scoring", SCORINGS)
def test_tail_pairs_flag_into_the_drain(sw, oracle, handle, knobs, small_db, scoring):
    """Short subjects carry segments of the query under a matrix
    scaled to entries up to 100 (the library's limit), so their fp16 cells
    leave the guard band: the tail pairs
    flag their blocks and the launch's drain re-scores them in int16 (fp16
    holds no odd integer above 2,048, so scores past 3,700 equal to the
    oracle's were re-scored); scores equal the oracle's."""
    mid, go, ge = scoring
    res, offs = small_db
    res = res.copy()
    q = sw.synth.query(300, shard=91)
    lens = offs[1:] - offs[:-1]
    short = np.argsort(lens, kind="stable")[1000:1400]  # in the narrowest 60 blocks
    rng = np.random.default_rng(5)
    for i in short:
        L = int(lens[i])
        s0 = int(rng.integers(0, len(q) - L)) if L < len(q) else 0
        res[offs[i]:offs[i] + min(L, len(q))] = q[s0:s0 + min(L, len(q))]
    m0 = sw.capi.builtin_matrix(mid).astype(np.int32)
    f = 100 // int(np.abs(m0).max())
    m = (m0 * f).astype(np.int8)
    go, ge = go * f, ge * f
    db = sw.Database(handle, res, offs, long_threshold=2048)
    want = oracle.scan(q, res, offs, mat=m, gap_open=go, gap_extend=ge, nthreads=16)
    assert want[short].max() > 3700  # past the fp16 guard band at this scale
    _tail_knobs(knobs, 60)
    got = db.scan(q, m, go, ge)
    assert "+tail" in handle.last_kernel(), handle.last_kernel()
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
    db.close()


@pytest.mark.parametrize("scoring", SCORINGS)
@pytest.mark.parametrize("grid", [2, 7, 40])
def test_looped_grid_equals_oracle(sw, oracle, handle, knobs, small_db, scoring, grid):
    """The merged launch's looped form (one workgroup per resident slot, each
    taking its next table entry from a counter; the default for tables of 3+
    rounds, C2's) forced with 2, 7 and 40 workgroups on the small database:
    every entry is taken exactly once (tail pairs, quads, intra items and the
    drain's entries included) and the counter starts at zero on every scan —
    two scans in a row equal the oracle, then the one-workgroup-per-entry form."""
    mid, go, ge = scoring
    res, offs = small_db
    db = sw.Database(handle, res, offs, long_threshold=700)  # intra items too
    q = sw.synth.query(375, shard=81)
    m = sw.capi.builtin_matrix(mid)
    want = oracle.scan(q, res, offs, mat=m, gap_open=go, gap_extend=ge, nthreads=16)
    knobs(lpt="1", pair_width="500", quad_width="900", inter_i16_span="0", intra_i16_first="0",
          tail_pairs="30", lpt_persist=str(grid))
    for _ in range(2):
        got = db.scan(q, m, go, ge)
        assert "+tail" in handle.last_kernel() and "+lpt" in handle.last_kernel(), handle.last_kernel()
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
    knobs(lpt_persist="0")
    assert np.array_equal(db.scan(q, m, go, ge), want)
    db.close()


def test_looped_grid_drains(sw, oracle, handle, knobs, small_db):
    """The looped form with the fp16 guard band flagging blocks (the tail
    test's planted segments under a matrix scaled to 100): entries flagged
    by one workgroup are drained while others still take table entries."""
    res, offs = small_db
    res = res.copy()
    q = sw.synth.query(300, shard=91)
    lens = offs[1:] - offs[:-1]
    planted = np.argsort(lens, kind="stable")[::97][:60]  # spread over the blocks
    rng = np.random.default_rng(6)
    for i in planted:
        L = int(min(lens[i], len(q)))
        s0 = int(rng.integers(0, len(q) - L + 1))
        res[offs[i]:offs[i] + L] = q[s0:s0 + L]
    m0 = sw.capi.builtin_matrix(1).astype(np.int32)
    f = 100 // int(np.abs(m0).max())
    m = (m0 * f).astype(np.int8)
    db = sw.Database(handle, res, offs, long_threshold=700)
    want = oracle.scan(q, res, offs, mat=m, gap_open=12 * f, gap_extend=f, nthreads=16)
    assert want[planted].max() > 3700
    knobs(lpt="1", pair_width="500", inter_i16_span="0", intra_i16_first="0", tail_pairs="30", lpt_persist="5")
    for _ in range(2):
        got = db.scan(q, m, 12 * f, f)
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
    db.close()


@pytest.mark.parametrize("scoring", SCORINGS)
def test_c2_size_merged_equals_separate_launches(sw, oracle, handle, knobs, scoring):
    """C2's whole database (570,000 subjects) under both scorings: the
    default merged launch (tail pairs, the looped grid; 96-row passes under
    the linear scoring) equals the separate-launch form on every subject and
    the oracle on a sample of 3,000 (the oracle is too slow for all)."""
    mid, go, ge = scoring
    res, offs = sw.synth.database(570000, shard=0)
    db = sw.Database(handle, res, offs)
    q = sw.encode(__import__("conftest").read_query("P07327"))
    m = sw.capi.builtin_matrix(mid)
    knobs(lpt="-1")
    got = db.scan(q, m, go, ge)
    k = handle.last_kernel()
    assert "+tail" in k and "+lpt" in k, k
    knobs(lpt="0")
    sep = db.scan(q, m, go, ge)
    assert "+lpt" not in handle.last_kernel()
    assert np.array_equal(got, sep), np.nonzero(got != sep)[0][:8]
    pick = np.sort(np.random.default_rng(mid).choice(len(offs) - 1, 3000, replace=False))
    lens = offs[pick + 1] - offs[pick]
    sub = np.concatenate([res[offs[i]:offs[i + 1]] for i in pick])
    so = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    want = oracle.scan(q, sub, so, mat=m, gap_open=go, gap_extend=ge, nthreads=16)
    assert np.array_equal(got[pick], want)
    db.close()
