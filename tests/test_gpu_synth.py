"""Device-generated synthetic shards: the GPU
scores of sampled subjects equal the oracle's on the same subjects
regenerated on the CPU from (seed, global id) by synth.counter_residues."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def regenerate(sw, seed, gids):
    L, lut = sw.capi.synth_tables()
    lens = sw.synth.counter_lengths(seed, gids, L)
    seqs = [sw.synth.counter_residues(seed, int(g), int(n), lut) for g, n in zip(gids, lens)]
    offs = np.zeros(len(seqs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    return np.concatenate(seqs), offs


@pytest.mark.parametrize("seed,id_base,thr", [(1782, 0, None), (99, 6_250_000, 600)])
def test_synthetic_shard_scores_vs_oracle(sw, oracle, handle, seed, id_base, thr):
    n = 4000
    db = sw.Database.synthetic(handle, seed, n, id_base=id_base, long_threshold=thr)
    lens, ids = db.subjects()
    L, _ = sw.capi.synth_tables()
    assert np.array_equal(ids, np.arange(n))
    assert np.array_equal(lens, sw.synth.counter_lengths(seed, np.arange(id_base, id_base + n), L))
    q = sw.synth.query(375, shard=4)
    rng = np.random.default_rng(seed)
    sample = np.sort(rng.choice(n, 150, replace=False))
    # include the longest subjects (intra kernel when thr is set)
    sample = np.unique(np.concatenate([sample, np.argsort(lens)[-10:]]))
    r, o = regenerate(sw, seed, id_base + sample)
    for args in ((), (sw.capi.builtin_matrix(1), 12, 1)):
        got = db.scan(q, *args)
        mat = args[0] if args else None
        go, ge = (args[1], args[2]) if args else (2, 2)
        want = oracle.scan(q, r, o, mat=mat, gap_open=go, gap_extend=ge)
        assert np.array_equal(got[sample], want), np.nonzero(got[sample] != want)[0][:10]


def test_synthetic_align_and_save(sw, oracle, handle, tmp_path):
    seed, base, n = 5, 1000, 600
    db = sw.Database.synthetic(handle, seed, n, id_base=base)
    q = sw.synth.query(200, shard=8)
    scores = db.scan(q)
    ids, _ = sw.capi.topk(scores, 5)
    r, o = regenerate(sw, seed, base + ids)
    got = db.align(q, ids)
    for k, al in enumerate(got):
        assert al == oracle.align(q, r[o[k]:o[k + 1]])
    p = str(tmp_path / "syn.swdb")
    db.save(p)
    db2 = sw.Database.load(handle, p)
    assert np.array_equal(db2.scan(q), scores)


def test_c4_full_rank_shard(sw, oracle, handle):
    """one rank's WHOLE C4 shard at its bench size — the
    last of 8 id ranges of the 50,000,000-subject database (6,250,000
    subjects, ~2.25e9 residues generated in HBM) — scanned with the bench's
    query and scoring (P07327, BLOSUM62 affine 12/1).  The device top-100
    (sw_scan_topk) equals the CPU top-100 of the GPU's scores; every top-100
    hit and a random sample of 400 subjects, regenerated on the CPU from
    (seed, global id) by synth.counter_residues, score the same in the
    oracle."""
    seed, total, ranks = 1782, 50_000_000, 8
    per = -(-total // ranks)
    id_base = (ranks - 1) * per
    n = total - id_base
    assert n == 6_250_000
    db = sw.Database.synthetic(handle, seed, n, id_base=id_base)
    from conftest import read_query
    q = sw.encode(read_query("P07327"))
    m = sw.capi.builtin_matrix(1)
    scores = db.scan(q, m, 12, 1)
    assert scores.shape[0] >= n
    scores = scores[:n]
    keys = db.scan_topk(q, 100, m, 12, 1)
    ids, sc = sw.capi.decode_keys(keys)
    want_ids, want_sc = sw.capi.topk(scores, 100)
    assert np.array_equal(ids, want_ids) and np.array_equal(sc, want_sc)
    rng = np.random.default_rng(4)
    sample = np.unique(np.concatenate([rng.choice(n, 400, replace=False), ids]))
    r, o = regenerate(sw, seed, id_base + sample)
    want = oracle.scan(q, r, o, mat=m, gap_open=12, gap_extend=1, nthreads=16)
    assert np.array_equal(scores[sample], want), np.nonzero(scores[sample] != want)[0][:10]
    db.close()
