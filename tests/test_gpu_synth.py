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
