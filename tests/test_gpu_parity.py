"""GPU parity: the HIP path (through the C ABI) against the reference's golden
scores and against the CPU oracle, bit-exact (integer DP)."""
import numpy as np
import pytest

from conftest import GOLDEN, read_golden, read_query


def family(handle):
    """The last scan's kernel family: 'sw_inter_x2p<...>' (the same two-strips
    kernel with its widest blocks run by wave pairs) reads as sw_inter_x2s."""
    return handle.last_kernel().replace("sw_inter_x2p", "sw_inter_x2s")


pytestmark = pytest.mark.gpu

QUERIES = ["P02232", "P05013", "P14942", "P07327", "P01008", "P03435", "P42357", "P21177",
           "Q38941", "P27895", "P07756", "P04775", "P19096", "P28167", "P0C6B8", "P20930",
           "P08519", "Q7TMA5", "P33450", "Q9UKN1"]


def subset(oracle):
    recs = oracle.read_fasta_records(GOLDEN + "/subset111.fasta")
    seqs = [s for _, s in recs]
    res = np.concatenate([oracle.encode(s) for s in seqs])
    offs = np.zeros(len(seqs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(s) for s in seqs])
    return res, offs


@pytest.mark.parametrize("qname", ["P01008", "P02232"])
@pytest.mark.parametrize("long_threshold", [None, 300, 1])
def test_golden_subset111(sw, oracle, handle, qname, long_threshold):
    """Swissprot records 0..110 vs test/reference/<q>.txt lines 0..110."""
    res, offs = subset(oracle)
    db = sw.Database(handle, res, offs, long_threshold=long_threshold)
    got = db.scan(sw.encode(read_query(qname)))
    want = np.array(read_golden(qname + ".subset111.scores"), dtype=np.int32)
    assert np.array_equal(got, want), np.nonzero(got != want)


@pytest.mark.parametrize("qname", QUERIES)
def test_all_shipped_queries_vs_oracle(sw, oracle, handle, qname):
    """Every data/queries FASTA (144..5478 aa: no 1024 cap) on the subset."""
    res, offs = subset(oracle)
    db = sw.Database(handle, res, offs)
    q = sw.encode(read_query(qname))
    got = db.scan(q)
    want = oracle.scan(q, res, offs)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("n,qlen,thr", [(1000, 144, None), (777, 375, None), (300, 1100, None),
                                        (130, 33, 200), (257, 600, 500), (64, 2100, 64)])
def test_synthetic_vs_oracle(sw, oracle, handle, n, qlen, thr):
    r, o = sw.synth.database(n, shard=n)
    q = sw.synth.query(qlen, shard=qlen)
    db = sw.Database(handle, r, o, long_threshold=thr)
    got = db.scan(q)
    want = oracle.scan(q, r, o)
    assert np.array_equal(got, want), (np.nonzero(got != want)[0][:10], got[:5], want[:5])


@pytest.mark.parametrize("go,ge", [(10, 1), (11, 1), (5, 2), (3, 3)])
@pytest.mark.parametrize("mid", [0, 1])
def test_affine_vs_oracle(sw, oracle, handle, go, ge, mid):
    r, o = sw.synth.database(400, shard=7)
    q = sw.synth.query(250, shard=8)
    mat = oracle.matrix(mid)
    db = sw.Database(handle, r, o)
    got = db.scan(q, matrix=mat, gap_open=go, gap_extend=ge)
    want = oracle.scan(q, r, o, mat=mat, gap_open=go, gap_extend=ge)
    assert np.array_equal(got, want)
    db.set_long_threshold(100)
    got2 = db.scan(q, matrix=mat, gap_open=go, gap_extend=ge)
    assert np.array_equal(got2, want)


def test_edge_cases(sw, oracle, handle):
    """Empty and ragged subjects, an empty query, custom ids."""
    seqs = ["", "A", "W", "WW", "", "ACDEFGHIKLMNPQRSTVWY" * 7, "X*UO/", "M" * 17]
    res = np.concatenate([oracle.encode(s) for s in seqs if s] or [np.zeros(0, np.uint8)])
    offs = np.zeros(len(seqs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(s) for s in seqs])
    ids = np.array([5, 0, 3, 9, 1, 2, 4, 7], dtype=np.int32)
    db = sw.Database(handle, res, offs, ids=ids)
    q = sw.encode("MKWVTFISLLFLFSSAYSW")
    got = db.scan(q)
    want_k = oracle.scan(q, res, offs)
    want = np.zeros(10, dtype=np.int32)
    want[ids] = want_k
    assert np.array_equal(got, want)
    assert np.all(db.scan(np.zeros(0, np.uint8)) == 0)
    db.set_long_threshold(1)
    assert np.array_equal(db.scan(q), want)


def test_identity_matrix_vs_cpu_cpp_pairs(sw, oracle, handle):
    """cpu.cpp's own +3/-3 scheme: GPU pair scores = maxima cpu.cpp printed."""
    import json
    pairs = json.load(open(GOLDEN + "/cpu_pairs.json"))["pairs"]
    mat = sw.builtin_matrix(sw.MATRIX_IDENTITY3)
    for p in pairs:
        got = handle.score_pair(sw.encode(p["a"]), sw.encode(p["b"]), matrix=mat)
        assert got == p["max"], p


def test_batch_and_solver_api(sw, oracle, handle, tmp_path):
    res, offs = subset(oracle)
    db = sw.Database(handle, res, offs)
    qs = [sw.encode(read_query(n)) for n in ("P02232", "P01008", "P07327")]
    out = db.scan_batch(qs)
    for k, q in enumerate(qs):
        assert np.array_equal(out[k], oracle.scan(q, res, offs))
    # the reference's interface: (id, score) appended in descending padded length
    query = sw.FASTAQuery(GOLDEN + "/queries/P01008.fasta", True)
    fdb = sw.FASTADatabase(GOLDEN + "/subset111.fasta")
    result = []
    sw.smith_waterman_cuda(query, fdb, result)
    golden = read_golden("P01008.subset111.scores")
    assert len(result) == 111
    assert all(score == golden[i] for i, score in result)
    lens = [len(s) for i, s in sorted(fdb.records())]
    order = [lens[i] for i, _ in result]
    assert order == sorted(order, reverse=True)
    chars = sw.smith_waterman_cuda_char(query, fdb)
    assert [s for _, s in chars] == golden
    # the char path's own scoring ('*' / '/' padding = -5,
    # query unpadded) against the oracle over the same flattened records
    compat = sw.smith_waterman_cuda_char(query, fdb, compat=True)
    flat_res, flat_offs, _ = fdb.flat(sw.encode)
    want = oracle.scan(sw.encode(query.get_buffer()), flat_res, flat_offs,
                       mat=oracle.matrix(oracle.MATRIX_BLOSUM50_CHAR), gap_open=2, gap_extend=2)
    assert [s for _, s in compat] == [int(x) for x in want]


def test_char_compat_star_residues(sw, oracle, handle):
    """The compat table on sequences full of '*' (U, O, lowercase, '/' all
    encode to it): +1 per '*'/'*' cell, -5 against letters, vs the oracle."""
    rng = np.random.default_rng(4)
    alphabet = "ARNDCQEGHILKMFPSTWYVBJZX*UO/acg"
    seqs = ["".join(rng.choice(list(alphabet), size=int(rng.integers(1, 300)))) for _ in range(400)]
    res = np.concatenate([sw.encode(x) for x in seqs])
    offs = np.zeros(len(seqs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(x) for x in seqs])
    q = sw.encode("".join(rng.choice(list(alphabet), size=260)))
    m = sw.builtin_matrix(sw.MATRIX_BLOSUM50_CHAR)
    db = sw.Database(handle, res, offs, long_threshold=200)
    got = db.scan(q, m, 2, 2)
    want = oracle.scan(q, res, offs, mat=oracle.matrix(oracle.MATRIX_BLOSUM50_CHAR), gap_open=2, gap_extend=2)
    assert np.array_equal(got, want)


def test_long_query_self_hit_int32(sw, oracle, handle):
    """Q9UKN1 (5478 aa) against itself: > int16 range."""
    q = sw.encode(read_query("Q9UKN1"))
    offs = np.array([0, len(q)], dtype=np.int64)
    db = sw.Database(handle, q, offs)
    got = int(db.scan(q)[0])
    want = int(oracle.scan(q, q, offs)[0])
    assert got == want and got > 32767


@pytest.mark.parametrize("mid,go,ge,ww,reps", [(0, 2, 2, 15, 2100), (0, 2, 2, 15, 2190), (0, 2, 2, 15, 2300),
                                              (1, 12, 1, 11, 2870), (1, 12, 1, 11, 2990), (1, 12, 1, 11, 3100)])
@pytest.mark.parametrize("variant", ["", "f32x8"])
def test_int16_saturation_rescue(sw, oracle, handle, knobs, mid, go, ge, ww, reps, variant):
    """Scores at/above the 16-bit kernels' saturation guard are re-scored at
    int32 (block-level rescue), next to ordinary subjects in the same block;
    linear (BLOSUM50, W-W = 15) and affine (BLOSUM62, W-W = 11) scoring."""
    rng = np.random.default_rng(reps)
    q = sw.encode("W" * reps)
    seqs = [rng.integers(0, 20, size=rng.integers(50, 400)).astype(np.uint8) for _ in range(150)]
    seqs[37] = sw.encode("W" * reps)            # ww * reps: 31500 .. 34500
    seqs[90] = sw.encode("W" * (reps // 2) + "A" * 30 + "W" * (reps // 2))
    res = np.concatenate(seqs)
    offs = np.zeros(len(seqs) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(x) for x in seqs])
    db = sw.Database(handle, res, offs, long_threshold=4096)
    m = sw.capi.builtin_matrix(mid)
    got = db.scan(q, m, go, ge)
    want = oracle.scan(q, res, offs, mat=m, gap_open=go, gap_extend=ge)
    assert got[37] == ww * reps
    assert np.array_equal(got, want)
    assert family(handle).startswith("sw_inter_x2s")


@pytest.mark.parametrize("n,k", [(10, 4), (5000, 100), (100000, 100), (300000, 1000), (7, 20)])
def test_device_topk(sw, handle, n, k):
    """sw_topk_device and the multi-rank merge (sw_topk_keys_device):
    score descending, id ascending, against numpy."""
    import torch
    rng = np.random.default_rng(n + k)
    s = rng.integers(0, 60, size=n).astype(np.int32)   # many ties
    order = np.lexsort((np.arange(n), -s))[:k]
    m = min(n, k)
    d = torch.from_numpy(s).cuda()
    out = torch.empty(k, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    handle.topk_device(d.data_ptr(), n, k, out.data_ptr(), id_base=1000)
    torch.cuda.synchronize()
    ids, sc = sw.capi.decode_keys(out.cpu().numpy())
    assert ids[:m].tolist() == (order[:m] + 1000).tolist()
    assert sc[:m].tolist() == s[order[:m]].tolist()
    assert (ids[m:] == -1).all()
    # two "ranks": top-k of each half, all-gathered, merged == top-k of all
    h = n // 2
    parts = torch.empty(2 * k, dtype=torch.int64, device="cuda")
    handle.topk_device(d.data_ptr(), h, k, parts.data_ptr(), id_base=0)
    handle.topk_device(d[h:].data_ptr(), n - h, k, parts[k:].data_ptr(), id_base=h)
    merged = torch.empty(k, dtype=torch.int64, device="cuda")
    handle.topk_keys_device(parts.data_ptr(), 2 * k, k, merged.data_ptr())
    torch.cuda.synchronize()
    ids2, sc2 = sw.capi.decode_keys(merged.cpu().numpy())
    assert ids2[:m].tolist() == order[:m].tolist()
    assert sc2[:m].tolist() == s[order[:m]].tolist()


@pytest.mark.parametrize("n,k,dist", [(2_000_000, 4096, "ties"), (200_000, 300, "wide"), (50_000, 100, "equal"),
                                      (16_384, 100, "ties"), (16_385, 4096, "wide"), (1, 1, "ties"),
                                      (4_096, 100, "ties"), (4_097, 1024, "wide"), (570_000, 100, "ties"),
                                      (300_000, 1024, "ties"), (300_000, 1025, "equal")])
def test_device_topk_radix_select(sw, handle, n, k, dist):
    """The radix select's corners: scores over the whole int32 range
    ("wide"), one score for every subject ("equal": the order is the ids
    alone), many ties; chunk-size boundaries (4,096 keys per 256-thread
    workgroup for k <= 1,024, 16,384 per 1,024-thread workgroup above), the
    largest k, three stages (2M scores; C2's 570,000 at k = 100)."""
    import torch
    rng = np.random.default_rng(n ^ k)
    if dist == "wide":
        s = rng.integers(0, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
    elif dist == "equal":
        s = np.full(n, 7, dtype=np.int32)
    else:
        s = rng.integers(0, 90, size=n).astype(np.int32)
    m = min(n, k)
    order = np.lexsort((np.arange(n), -s))[:m]
    d = torch.from_numpy(s).cuda()
    out = torch.empty(k, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    handle.topk_device(d.data_ptr(), n, k, out.data_ptr(), id_base=5)
    torch.cuda.synchronize()
    ids, sc = sw.capi.decode_keys(out.cpu().numpy())
    assert ids[:m].tolist() == (order + 5).tolist()
    assert sc[:m].tolist() == s[order].tolist()
    assert (ids[m:] == -1).all()


# the shapes the library still builds: int32 (fall-back and rescue), the
# int16 two-strips kernel (rescue-chain stage 2), its fp16 form (default)
INTER_VARIANTS = ["32x8", "64x8", "y32x8", "f32x8", "f32x4"]


@pytest.mark.parametrize("variant", INTER_VARIANTS)
@pytest.mark.parametrize("coop", ["0", "128:0", "128:1"])
def test_inter_variants_vs_oracle(sw, oracle, handle, knobs, variant, coop):
    """Every inter-kernel shape with the cooperative wide-block kernel off /
    on (plain) / on (skewed), linear and affine."""
    width, _, skew = coop.partition(":")
    knobs(inter_variant=variant)
    knobs(coop_width=width)
    knobs(coop_skew=skew or "1")
    r, o = sw.synth.database(900, shard=11)
    db = sw.Database(handle, r, o, long_threshold=1500)
    for qlen, mid, go, ge in [(375, 0, 2, 2), (150, 1, 12, 1), (97, 1, 11, 2)]:
        q = sw.synth.query(qlen, shard=qlen + 1)
        m = sw.capi.builtin_matrix(mid)
        got = db.scan(q, m, go, ge)
        want = oracle.scan(q, r, o, mat=m, gap_open=go, gap_extend=ge)
        assert np.array_equal(got, want), (qlen, mid, go, ge, np.nonzero(got != want)[0][:10])


@pytest.mark.parametrize("guard", ["1", "0"])
@pytest.mark.parametrize("variant", ["", "y32x8"])
def test_long_query_int16_guard(sw, oracle, handle, knobs, variant, guard):
    """A query long enough that (qlen + 2) * (max S + gap open) >= 32767: the
    two-strips kernel runs guarded (sw_opts int16_guard auto / 1) or the
    int32 kernel runs (int16_guard 0).  Scores stay exact either way."""
    knobs(int16_guard=guard)
    if variant:
        knobs(inter_variant=variant)
    r, o = sw.synth.database(300, shard=5)
    q = sw.synth.query(2400, shard=9)
    # plant the query itself as a subject so one score is large
    r2 = np.concatenate([r, q])
    o2 = np.concatenate([o, [o[-1] + len(q)]])
    db = sw.Database(handle, r2, o2, long_threshold=3000)
    for mid, go, ge in [(1, 12, 1), (0, 2, 2)]:
        m = sw.capi.builtin_matrix(mid)
        got = db.scan(q, m, go, ge)
        want = oracle.scan(q, r2, o2, mat=m, gap_open=go, gap_extend=ge)
        assert np.array_equal(got, want), (mid, np.nonzero(got != want)[0][:10])
        assert got[-1] > 9000
        k = family(handle)
        if guard == "0":
            assert not k.startswith("sw_inter_x2"), k
        else:
            assert k.startswith("sw_inter_x2s"), k


def test_default_kernel_selection(sw, handle, knobs):
    """int16-safe scans run the packed two-strips-per-lane kernel; longer
    queries run it guarded; gaps too large for the guard band, or the guard
    switched off, run the int32 kernels."""
    r, o = sw.synth.database(200, shard=3)
    db = sw.Database(handle, r, o)
    q = sw.synth.query(375, shard=4)
    db.scan(q, sw.capi.builtin_matrix(1), 12, 1)
    assert family(handle) == "sw_inter_x2s<32,8,affine,fp16>"
    db.scan(q)
    assert family(handle) == "sw_inter_x2s<32,8,linear,fp16>"
    # beyond the static int16 bound but inside the guard band: guarded packed
    db.scan(q, sw.capi.builtin_matrix(0), 100, 1)
    assert family(handle) == "sw_inter_x2s<32,8,affine,fp16>"
    # max S + gap open >= 1000: int32
    db.scan(q, sw.capi.builtin_matrix(0), 1000, 1)
    assert handle.last_kernel() == "sw_inter<32,8,affine>"
    knobs(int16_guard="0")
    db.scan(q, sw.capi.builtin_matrix(0), 100, 100)
    assert handle.last_kernel() == "sw_inter<64,8,linear>"

def test_batch_all_shipped_queries_c3(sw, oracle, handle):
    """Config C3's shape at test size: the 20 shipped queries (144..5478 aa,
    int16-exact, guarded and int32 paths mixed) in one batch, host and
    device entry points, against the oracle query by query."""
    import torch
    r, o = sw.synth.database(700, shard=21)
    db = sw.Database(handle, r, o)
    qs = [sw.encode(read_query(n)) for n in QUERIES]
    m = sw.capi.builtin_matrix(1)
    out = db.scan_batch(qs, m, 12, 1)
    dev = torch.zeros((len(qs), db.n_out), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()  # the fill ran on torch's stream, the scans run on the handle's
    db.scan_batch_device(qs, dev.data_ptr(), m, 12, 1)
    torch.cuda.synchronize()  # device-wide: waits for the handle's streams too
    assert np.array_equal(dev.cpu().numpy(), out)
    for k, q in enumerate(qs):
        want = oracle.scan(q, r, o, mat=m, gap_open=12, gap_extend=1)
        assert np.array_equal(out[k], want), (QUERIES[k], np.nonzero(out[k] != want)[0][:10])


@pytest.mark.parametrize("scoring", [(0, 2, 2), (1, 12, 1)])
def test_batch_rescue_tails_overlap(sw, oracle, handle, scoring):
    """A rescue-heavy batch: long queries under the reference's cheap linear
    gaps (BLOSUM50 / 2) and BLOSUM62 11/1, planted near-copies scoring above
    the fp16 bound (~4,000) and above 32767 in both the inter and the intra
    part.  In a batch
    each query's rescue tail runs on the tail stream beside the next query's
    fp16 passes (parity lists, own boundary rows, profile slots reused after
    4 queries): every query equals the oracle and its single-query scan,
    twice (the second batch takes the adaptive int16 paths)."""
    mid, go, ge = scoring
    names = ["Q9UKN1", "P02232", "P20930", "P04775", "Q9UKN1", "P07327", "P33450"]
    qs = [sw.encode(read_query(n)) for n in names]
    r, o = sw.synth.database(1500, shard=31)
    big = qs[0]
    extra = [big, big[:1000], qs[2][:1500], qs[6][200:1100]]  # intra / inter near-copies
    r2 = np.concatenate([r] + extra)
    o2 = np.concatenate([o, o[-1] + np.cumsum([len(x) for x in extra])])
    db = sw.Database(handle, r2, o2, long_threshold=1200)
    m = sw.capi.builtin_matrix(mid)
    want = [oracle.scan(q, r2, o2, mat=m, gap_open=go, gap_extend=ge, nthreads=16) for q in qs]
    for _ in range(2):
        out = db.scan_batch(qs, m, go, ge)
        for k in range(len(qs)):
            assert np.array_equal(out[k], want[k]), (names[k], np.nonzero(out[k] != want[k])[0][:10])
    for k in (0, 3):
        assert np.array_equal(db.scan(qs[k], m, go, ge), want[k])
    # empty queries at the end and in the middle of a batch: the
    # batch still waits for every deferred rescue tail before it completes
    empty = np.zeros(0, dtype=np.uint8)
    for sel in ([0, 1, 2, None], [0, None, 3, None, None], [None, 6, 0]):
        batch = [qs[k] if k is not None else empty for k in sel]
        out = db.scan_batch(batch, m, go, ge)
        for j, k in enumerate(sel):
            if k is None:
                assert not out[j].any()
            else:
                assert np.array_equal(out[j], want[k]), (sel, names[k])
    if mid == 0:
        assert max(int(w.max()) for w in want) > 32767  # the int32 stage ran


def test_db_save_load_roundtrip(sw, oracle, handle, tmp_path):
    """sw_db_save / sw_db_load: identical scores[id], custom ids kept, bad
    files rejected."""
    r, o = sw.synth.database(500, shard=13)
    ids = np.random.default_rng(2).permutation(700)[:500].astype(np.int32)
    db = sw.Database(handle, r, o, ids=ids)
    p = str(tmp_path / "db.swdb")
    db.save(p)
    db2 = sw.Database.load(handle, p)
    assert db2.n == 500 and db2.n_out == int(ids.max()) + 1
    q = sw.synth.query(300, shard=3)
    for args in ((), (sw.capi.builtin_matrix(1), 12, 1)):
        assert np.array_equal(db.scan(q, *args), db2.scan(q, *args))
    with pytest.raises(sw.capi.SWError):
        sw.Database.load(handle, str(tmp_path / "missing.swdb"))
    open(str(tmp_path / "trunc.swdb"), "wb").write(open(p, "rb").read()[:100])
    with pytest.raises(sw.capi.SWError):
        sw.Database.load(handle, str(tmp_path / "trunc.swdb"))


@pytest.mark.parametrize("scoring", [(1, 12, 1), (0, 2, 2), (1, 14, 3), (0, 5, 5)])
@pytest.mark.parametrize("qlen,selfhit", [(375, True), (900, True), (2400, False)])
def test_fp16_guard_band(sw, oracle, handle, knobs, qlen, selfhit, scoring):
    """The fp16 kernels (biased cells: stored values sit up to 26 ge above
    the true ones, all of them offset by -2048 + 2 ge) are exact below
    4096 - 2 ge - 2 max S - 26 ge and flag their block otherwise: subjects
    scoring around and far above 2048 and 4096 (planted near-copies of the
    query: the 375-aa self-hits score 1,935-2,473, the 900-aa ones
    4,655-5,932) next to ordinary ones, affine (BLOSUM62 11/1 and 13/3) and
    linear (BLOSUM50, gap 2 and 5) against the oracle."""
    mid, go, ge = scoring
    knobs(inter_variant="f32x8")
    r, o = sw.synth.database(300, shard=qlen)
    q = sw.synth.query(qlen, shard=qlen + 5)
    extra = [q[: qlen // 2], q] if selfhit else [q[:400], q[:190]]
    r2 = np.concatenate([r] + extra)
    o2 = np.concatenate([o, o[-1] + np.cumsum([len(x) for x in extra])])
    db = sw.Database(handle, r2, o2, long_threshold=4000)
    m = sw.capi.builtin_matrix(mid)
    got = db.scan(q, m, go, ge)
    want = oracle.scan(q, r2, o2, mat=m, gap_open=go, gap_extend=ge)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert family(handle) == "sw_inter_x2s<32,8,%s,fp16>" % ("linear" if go == ge else "affine")
    assert want.max() > 1000


@pytest.mark.parametrize("variant", ["f32x8", "y32x8"])
@pytest.mark.parametrize("width", ["16", "300"])
@pytest.mark.parametrize("group", ["2", "4"])
def test_wave_pair_kernel(sw, oracle, handle, knobs, variant, width, group):
    """sw_inter_x2p (the widest blocks by wave pairs or quads; width 16 =
    every block): 1 to 15 passes (odd and even counts, fewer passes than
    waves), narrow blocks (the 6- / 12-tick period floor), a block count not
    a multiple of the groups per workgroup, linear and affine, and planted
    near-copies of the query whose blocks the fp16 kernel flags for the
    rescue chain — all against the oracle."""
    knobs(inter_variant=variant)
    knobs(pair_width=width)
    knobs(pair_group=group)
    r, o = sw.synth.database(1000, shard=17)
    q0 = sw.synth.query(900, shard=3)
    extra = [q0, q0[:450], q0[100:700]]
    r2 = np.concatenate([r] + extra)
    o2 = np.concatenate([o, o[-1] + np.cumsum([len(x) for x in extra])])
    db = sw.Database(handle, r2, o2, long_threshold=4000)
    for qlen, mid, go, ge in [(375, 1, 12, 1), (150, 1, 12, 1), (97, 1, 11, 2), (40, 1, 12, 1), (900, 1, 12, 1),
                              (375, 0, 2, 2), (260, 0, 2, 2)]:
        q = q0[:qlen]
        m = sw.capi.builtin_matrix(mid)
        got = db.scan(q, m, go, ge)
        want = oracle.scan(q, r2, o2, mat=m, gap_open=go, gap_extend=ge)
        assert np.array_equal(got, want), (qlen, mid, go, ge, np.nonzero(got != want)[0][:10])
        k = handle.last_kernel()
        pairs = db.stats()["pair_blocks"]
        assert k.startswith("sw_inter_x2p<32,8," if pairs else "sw_inter_x2s<32,8,"), k
        if qlen > 64:
            assert pairs > 0 and (width == "300" or pairs == db.stats()["n_blocks"]), pairs
        else:
            assert pairs == 0
        if qlen == 900:
            assert want.max() > 4096  # the fp16 guard band is crossed


@pytest.mark.parametrize("packed,ri", [("1", ""), ("1", "6"), ("1", "10"), ("1", "20"), ("0", "")])
def test_intra_two_subjects_per_wave(sw, oracle, handle, knobs, packed, ri):
    """sw_intra_x2 (two long subjects per wave, packed fp16; intra_x2 0:
    int32 sw_intra only): rows per lane 4..20 by the cost model (query lengths
    40..2100, one to several chunk passes) or forced to the 2-row-element
    shapes 6 and 10 and to the widest, 20 rows by 6-wave workgroups (this
    database has no inter blocks, so no merged launch can take the scan), an
    odd number of long subjects, pairs of unequal length,
    linear and affine scoring, and planted near-copies of the query whose fp16
    maxima cross the fp16 bound (~4,000: cells offset by -2048 + 2 ge;
    re-scored by sw_intra in list mode)."""
    knobs(intra_x2=packed)
    if ri:
        knobs(intra_x2_rows=ri)
    rng = np.random.default_rng(7)
    q0 = sw.synth.query(2100, shard=8)
    lens = rng.integers(70, 900, size=40)
    subs = [sw.synth.query(int(n), shard=100 + k) for k, n in enumerate(lens)]
    subs += [q0, q0[:1000], q0[300:1500]]   # 43 subjects: odd count
    r = np.concatenate(subs).astype(np.uint8)
    o = np.concatenate([[0], np.cumsum([len(x) for x in subs])]).astype(np.int64)
    db = sw.Database(handle, r, o, long_threshold=64)
    assert db.stats()["n_long"] == len(subs)
    for qlen, mid, go, ge in [(40, 1, 12, 1), (375, 1, 12, 1), (600, 1, 12, 1), (700, 1, 11, 2), (1100, 0, 2, 2),
                              (1500, 0, 2, 2), (2100, 1, 12, 1), (260, 0, 8, 8), (40, 0, 2, 2), (600, 1, 3, 3)]:
        q = q0[:qlen]
        m = sw.capi.builtin_matrix(mid)
        got = db.scan(q, m, go, ge)
        want = oracle.scan(q, r, o, mat=m, gap_open=go, gap_extend=ge)
        assert np.array_equal(got, want), (qlen, mid, go, ge, np.nonzero(got != want)[0][:10])
        if packed == "1" and ri:
            assert handle.last_intra_kernel().startswith("sw_intra_x2<%s" % ri), handle.last_intra_kernel()
        if qlen >= 1500:
            assert want.max() > 4096


@pytest.mark.parametrize("order", ["", "0", "1"])
def test_intra_rescue_chain_fp16_int16_int32(sw, oracle, handle, knobs, order):
    """The intra rescue chain end to end: sw_intra_x2 (fp16) flags subjects
    near its bound (4096 - 2 ge - 2 max S - 26 ge: cells offset by -2048 +
    2 ge) into list 1, its int16 form re-scores list 1 and flags those near
    32767 into list 2, and int32 sw_intra re-scores list 2.  Cheap linear
    gaps (the reference scoring, BLOSUM50, 2 per gap) make random 5k-aa pairs
    score 2,300-7,100 (13 of the 19 above the bound); a planted copy of the
    6,500-aa query scores above 32767;
    ordinary subjects sit next to both in the same pairs.  The chain's order
    (sw_opts intra_i16_first): adaptive (int16 first once a scan with the same
    scoring flagged over a third of the long subjects at a query no longer than
    this one), never, always."""
    if order:
        knobs(intra_i16_first=order)
    rng = np.random.default_rng(11)
    q = sw.synth.query(6500, shard=21)
    lens = rng.integers(1500, 5500, size=17)
    subs = [sw.synth.query(int(n), shard=300 + k) for k, n in enumerate(lens)]
    subs.insert(5, q.copy())
    subs.insert(9, q[:3000].copy())
    r = np.concatenate(subs).astype(np.uint8)
    o = np.concatenate([[0], np.cumsum([len(x) for x in subs])]).astype(np.int64)
    db = sw.Database(handle, r, o, long_threshold=64)
    m = sw.capi.builtin_matrix(0)
    for rnd, (go, ge) in enumerate([(2, 2), (12, 1), (2, 2), (12, 1)]):
        want = oracle.scan(q, r, o, mat=m, gap_open=go, gap_extend=ge)
        for qq in (q, q[:5000]):
            w = want if len(qq) == len(q) else oracle.scan(qq, r, o, mat=m, gap_open=go, gap_extend=ge)
            got = db.scan(qq, m, go, ge)
            assert np.array_equal(got, w), (order, go, ge, len(qq), np.nonzero(got != w)[0][:10])
            # adaptive: BLOSUM50 / 2 flags nearly all of them, so its second
            # round runs int16 first; 12 / 1 flags only the planted copies
            i16 = handle.last_intra_kernel().endswith(",int16>")
            assert i16 == (order == "1" or (order == "" and rnd == 2)), (order, rnd, len(qq))
            if len(qq) == 5000:
                assert (w >= 4010).sum() * 3 > len(subs) or ge == 1
        assert want.max() > 32767
        assert ((want > 4096) & (want < 32000)).sum() >= (2 if ge == 2 else 1)


def test_inter_widest_blocks_int16_first(sw, oracle, handle, knobs):
    """Long queries whose scores against the widest blocks leave the fp16
    range (true scores up to ~4,000; here BLOSUM50 + 3 with linear gap 2,
    under which random 2,600 x 1,650 pairs score 4,900-8,200, while short
    subjects stay below 1,800) put those blocks in the fp16 guard band; once
    a scan has flagged most of blocks [0, span), later scans with queries at
    least as long run those blocks in int16 by wave pairs beside the fp16
    launch (sw_opts inter_i16_span forces a span: one block, some, more than the
    pair blocks, all of them; and under affine scoring).  Every scan
    bit-exact against the oracle."""
    r1, o1 = sw.synth.fixed_length_database(1280, 1650, 200, shard=41)
    r2, o2 = sw.synth.fixed_length_database(3000, 250, 80, shard=42)
    r = np.concatenate([r1, r2])
    o = np.concatenate([o1, o2[1:] + o1[-1]])
    q = sw.synth.query(2600, shard=43)
    m = (np.asarray(sw.capi.builtin_matrix(0), dtype=np.int32) + 3).astype(np.int8)
    db = sw.Database(handle, r, o, long_threshold=4096)
    assert db.stats()["n_long"] == 0
    want = oracle.scan(q, r, o, mat=m, gap_open=2, gap_extend=2)
    got = db.scan(q, m, 2, 2)
    assert np.array_equal(got, want)
    assert "+int16" not in handle.last_kernel()       # nothing observed yet
    got = db.scan(q, m, 2, 2)
    assert np.array_equal(got, want)
    k = handle.last_kernel()
    assert "+int16[0," in k, k                         # the widest ~19 blocks
    assert 10 <= int(k.split("+int16[0,")[1].rstrip(")")) <= 30, k
    q2 = q[:2000]
    want2 = oracle.scan(q2, r, o, mat=m, gap_open=2, gap_extend=2)
    assert np.array_equal(db.scan(q2, m, 2, 2), want2)
    assert "+int16" not in handle.last_kernel()       # shorter than any observation
    nblocks = db.stats()["n_blocks"]
    knobs(pair_width="2000")       # few pair blocks: spans beyond them
    for span in (1, 7, 25, nblocks):
        knobs(inter_i16_span=str(span))
        got = db.scan(q, m, 2, 2)
        assert np.array_equal(got, want), (span, np.nonzero(got != want)[0][:10])
        assert handle.last_kernel().endswith("+int16[0,%d)" % span)
    knobs(inter_i16_span="5")
    m62 = sw.capi.builtin_matrix(1)
    want3 = oracle.scan(q2, r, o, mat=m62, gap_open=12, gap_extend=1)
    assert np.array_equal(db.scan(q2, m62, 12, 1), want3)
    assert handle.last_kernel().endswith("+int16[0,5)")


@pytest.mark.parametrize("case", range(int(__import__("os").environ.get("SW_RANDOM_CASES", "24"))))
def test_random_scoring_and_shapes(sw, oracle, handle, case):
    """Seeded random cases against the oracle: a random symmetric matrix
    (entries -9..13, positive diagonal), gap pairs with open >= extend and a
    few with open < extend, ragged databases with subjects of 1..4,000
    residues, queries of 1..1,600, and the long threshold at the default, 64
    or 500, so every kernel family and both rescue chains get random inputs.
    Each database is scanned twice (the second scan may take the adaptive
    int16 paths).  SW_RANDOM_CASES=n runs n cases and SW_RANDOM_QMAX the
    longest query (stress runs)."""
    rng = np.random.default_rng(1000 + case)
    m = rng.integers(-9, 14, size=(25, 25))
    m = np.triu(m) + np.triu(m, 1).T
    np.fill_diagonal(m, rng.integers(1, 14, size=25))
    m = m.astype(np.int8).reshape(-1)
    ge = int(rng.integers(1, 8))
    go = int(ge + rng.integers(0, 15)) if case % 6 else int(rng.integers(1, ge + 1))
    n = int(rng.integers(50, 400))
    lens = np.clip(rng.lognormal(np.log(300), 0.9, size=n), 1, 4000).astype(np.int64)
    subs = [rng.integers(0, 25, size=int(L)).astype(np.uint8) for L in lens]
    r = np.concatenate(subs)
    o = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    thr = [None, 64, 500][case % 3]
    qmax = int(__import__("os").environ.get("SW_RANDOM_QMAX", "1600"))
    q = rng.integers(0, 25, size=int(rng.integers(1, qmax))).astype(np.uint8)
    db = sw.Database(handle, r, o, long_threshold=thr)
    want = oracle.scan(q, r, o, mat=m, gap_open=go, gap_extend=ge)
    for _ in range(2):
        got = db.scan(q, m, go, ge)
        assert np.array_equal(got, want), (case, go, ge, len(q), handle.last_kernel(),
                                           handle.last_intra_kernel(), np.nonzero(got != want)[0][:10])


@pytest.mark.parametrize("quad_width, pipe", [("0", "0"), ("200", "0"), ("16", "0"), ("200", "2"), ("0", "100")])
@pytest.mark.parametrize("scoring", [(1, 12, 1), (0, 2, 2)])
def test_merged_lpt_launch(sw, oracle, handle, knobs, quad_width, pipe, scoring):
    """sw_scan_lpt (the inter blocks by quads / pairs / single waves and the
    long subjects' fp16 pass in one launch, longest work first): queries for
    the three intra shapes it supports (4, 6, 8 rows per lane), quads for
    none, the widest or every group block, the longest pairs in the
    pipelined form (a query chunk per wave) for none, 8 or every long
    subject, planted near-copies in both kernels' halves (rescued inside the
    merged launch), against the oracle and the two-launch form."""
    mid, go, ge = scoring
    knobs(lpt="1")
    knobs(lpt_pipe=pipe)
    knobs(quad_width=quad_width, tri_width="0")  # (3-wave groups: test_tri_groups)
    knobs(pair_width="64")
    r, o = sw.synth.database(2500, shard=23)
    q0 = sw.synth.query(500, shard=8)
    extra = [q0, q0[:300], np.concatenate([q0, q0])]  # a long near-copy goes to the intra half
    r2 = np.concatenate([r] + extra)
    o2 = np.concatenate([o, o[-1] + np.cumsum([len(x) for x in extra])])
    db = sw.Database(handle, r2, o2, long_threshold=700)
    m = sw.capi.builtin_matrix(mid)
    for qlen in (200, 375, 500):
        q = q0[:qlen]
        got = db.scan(q, m, go, ge)
        assert "+lpt" in handle.last_kernel(), handle.last_kernel()
        want = oracle.scan(q, r2, o2, mat=m, gap_open=go, gap_extend=ge)
        assert np.array_equal(got, want), (qlen, np.nonzero(got != want)[0][:10])
        knobs(lpt="0")
        assert np.array_equal(db.scan(q, m, go, ge), got)
        assert "+lpt" not in handle.last_kernel()
        knobs(lpt="1")


@pytest.mark.parametrize("tail", ["1", "37", "100000"])
@pytest.mark.parametrize("scoring", [(1, 12, 1), (0, 2, 2)])
def test_tail_pipelined_pairs(sw, oracle, handle, knobs, tail, scoring):
    """The merged launch's last long-subject pairs in the pipelined form too
    (sw_opts lpt_pipe_tail: one, some, every pair; with the longest pairs
    pipelined as well, and without): every pair is scored exactly once,
    planted copies rescued in the launch, against the oracle."""
    mid, go, ge = scoring
    knobs(lpt="1", lpt_pipe_tail=tail, pair_width="64", inter_i16_span="0", intra_i16_first="0")
    r, o = sw.synth.database(2500, shard=31)
    q0 = sw.synth.query(500, shard=10)
    extra = [np.concatenate([q0, q0]), q0[:300], np.concatenate([q0[:400], q0[:400]])]
    r2 = np.concatenate([r] + extra)
    o2 = np.concatenate([o, o[-1] + np.cumsum([len(x) for x in extra])])
    db = sw.Database(handle, r2, o2, long_threshold=700)
    m = sw.capi.builtin_matrix(mid)
    for pipe in ("0", "3"):
        knobs(lpt_pipe=pipe)
        for qlen in (200, 375, 500):
            q = q0[:qlen]
            want = oracle.scan(q, r2, o2, mat=m, gap_open=go, gap_extend=ge)
            for _ in range(2):
                got = db.scan(q, m, go, ge)
                assert "+lpt" in handle.last_kernel(), handle.last_kernel()
                assert np.array_equal(got, want), (pipe, qlen, np.nonzero(got != want)[0][:10])
    db.close()


@pytest.mark.parametrize("tri_width", ["16", "200", "450"])
@pytest.mark.parametrize("scoring", [(1, 12, 1), (0, 13, 3), (0, 2, 2)])
def test_tri_groups(sw, oracle, handle, knobs, tri_width, scoring):
    """The merged launch's 3-wave groups (sw_opts tri_width; affine gaps,
    queries of 3, 5 or 6 passes of 64 rows): every group block, the widest
    ones or a few as tris, each workgroup's fourth wave on a single-wave
    block (more tris than singles included: 2,500 subjects, pair width 64),
    planted near-copies rescued inside the launch, against the oracle and
    the two-launch form; other pass counts and linear gaps keep the quads."""
    mid, go, ge = scoring
    knobs(lpt="1", tri_width=tri_width, pair_width="64", inter_i16_span="0", intra_i16_first="0")
    r, o = sw.synth.database(2500, shard=29)
    q0 = sw.synth.query(500, shard=9)
    extra = [q0, q0[:300], np.concatenate([q0, q0])]
    r2 = np.concatenate([r] + extra)
    o2 = np.concatenate([o, o[-1] + np.cumsum([len(x) for x in extra])])
    db = sw.Database(handle, r2, o2, long_threshold=700)
    m = sw.capi.builtin_matrix(mid)
    for qlen in (150, 300, 375, 500):
        q = q0[:qlen]
        got = db.scan(q, m, go, ge)
        passes = -(-qlen // 64)
        tri = go != ge and -(-passes // 3) <= -(-passes // 4)
        assert ("+tri" in handle.last_kernel()) == tri, (qlen, handle.last_kernel())
        want = oracle.scan(q, r2, o2, mat=m, gap_open=go, gap_extend=ge)
        assert np.array_equal(got, want), (qlen, np.nonzero(got != want)[0][:10])
        assert np.array_equal(db.scan(q, m, go, ge), want)  # the cached table, twice
        knobs(lpt="0")
        assert np.array_equal(db.scan(q, m, go, ge), want)
        knobs(lpt="1")
    db.close()


@pytest.mark.parametrize("ri", ["4", "8"])
@pytest.mark.parametrize("scoring", [(0, 2, 2), (0, 12, 1)])
def test_merged_launch_drains_rescue_lists(sw, oracle, handle, knobs, ri, scoring):
    """The merged launch re-scores what its fp16 cells flag inside the same
    launch (sw_scan_lpt's drain, no rescue launches after it): planted hits
    of every stage — inter blocks above the fp16 bound (int16 re-score) and
    above 32767 (int16 flags again -> int32), long subjects likewise (int16
    pairs -> int32 subjects), in quad, pair and single-wave blocks — equal
    the oracle and the separate-launch form, twice (the lists' entries are
    reset by whoever takes them, so the second scan starts clean)."""
    mid, go, ge = scoring
    knobs(lpt="1")
    knobs(intra_x2_rows=ri)
    knobs(pair_width="64")
    # keep the fp16-first order on the second scan (the adaptive routing would
    # send this many flagged blocks / subjects to int16 first)
    knobs(inter_i16_span="0")
    knobs(intra_i16_first="0")
    W = sw.encode("W")[0]
    q = np.full(2300, W, dtype=np.uint8)  # W/W scores 15: 34,500 for a full copy
    r, o = sw.synth.database(2000, shard=41)
    rng = np.random.default_rng(41)

    def planted(n, at, k):
        s = sw.synth.query(n, shard=int(rng.integers(1 << 30)))
        s[at:at + k] = W
        return s
    extra = [np.full(2300, W, np.uint8),   # inter, > 32767: A -> B -> int32
             planted(600, 100, 400),       # inter, ~6,000: A -> int16
             planted(2000, 50, 300),       # inter, widest blocks (quads): A -> int16
             np.full(2600, W, np.uint8),   # long, > 32767: 1 -> 2 -> int32
             planted(3000, 900, 400),      # long, ~6,000: 1 -> int16
             planted(2700, 10, 2290)]      # long, ~34,000: 1 -> 2 -> int32
    r2 = np.concatenate([r] + extra)
    o2 = np.concatenate([o, o[-1] + np.cumsum([len(x) for x in extra])])
    db = sw.Database(handle, r2, o2, long_threshold=2500)
    m = sw.capi.builtin_matrix(mid)
    want = oracle.scan(q, r2, o2, mat=m, gap_open=go, gap_extend=ge, nthreads=16)
    assert int(want.max()) > 32767 and int((want > 4096).sum()) >= 6
    for _ in range(2):
        got = db.scan(q, m, go, ge)
        assert handle.last_kernel().endswith("+lpt+drain"), handle.last_kernel()
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    knobs(lpt="0")
    assert np.array_equal(db.scan(q, m, go, ge), want)
    db.close()


@pytest.mark.gpu
def test_drain_timeout_reports_sw_e_device(sw, oracle, handle, knobs):
    """a drain wait that gives up on a claimed rescue-list entry
    (sw_opts drain_spin 0 makes every wait give up at once) is not silent:
    the scan returns SW_E_DEVICE (-7) instead of unrescued scores, and the
    database's next scan, with the default bound, re-initialises the lists
    and equals the oracle again."""
    knobs(lpt="1", pair_width="64", inter_i16_span="0", intra_i16_first="0", intra_x2_rows="8")
    W = sw.encode("W")[0]
    q = np.full(1200, W, dtype=np.uint8)  # planted copies score above fp16's 2,048: they flag
    r, o = sw.synth.database(1500, shard=43)
    extra = [np.full(1200, W, np.uint8), np.full(2600, W, np.uint8)]  # an inter block and a long subject
    r2 = np.concatenate([r] + extra)
    o2 = np.concatenate([o, o[-1] + np.cumsum([len(x) for x in extra])])
    db = sw.Database(handle, r2, o2, long_threshold=2500)
    m = sw.capi.builtin_matrix(1)
    want = oracle.scan(q, r2, o2, mat=m, gap_open=12, gap_extend=1, nthreads=16)
    assert int(want.max()) > 4096
    knobs(drain_spin="0")
    with pytest.raises(sw.capi.SWError, match="error -7"):
        db.scan(q, m, 12, 1)
    assert handle.last_kernel().endswith("+lpt+drain"), handle.last_kernel()
    knobs(drain_spin="")
    for _ in range(2):
        assert np.array_equal(db.scan(q, m, 12, 1), want)
    db.close()


@pytest.mark.parametrize("scoring", [(0, 12, 1), (1, 12, 1)])
def test_drain_waits_for_previous_deferred_tail(sw, oracle, handle, knobs, scoring):
    """in a batch, a merged launch that drains its rescue
    lists re-scores on the deferred tails' boundary rows, so it must not
    overlap the rescue tail of a non-merged scan just before it.  A 2,300-aa
    query that flagged most long subjects and the widest blocks routes later
    queries at least as long int16-first (two launches, its rescue tail
    deferred to the tail stream in a batch); a 1,500-aa query with the same
    scoring still takes the merged launch and drains what it flags on the
    same rows.  Batches alternating the two equal the oracle, query by
    query."""
    mid, go, ge = scoring
    knobs(pair_width=64, intra_x2_rows=8)  # (the merged launch has the 4-, 6- and 8-row intra forms)
    W = sw.encode("W")[0]
    qa = np.full(2300, W, dtype=np.uint8)
    qb = np.full(1500, W, dtype=np.uint8)
    r, o = sw.synth.database(2000, shard=43)
    rng = np.random.default_rng(43)

    def planted(n, at, k):
        s = sw.synth.query(n, shard=int(rng.integers(1 << 30)))
        s[at:at + k] = W
        return s
    extra = [np.full(2300, W, np.uint8), planted(600, 100, 400), planted(2000, 50, 1800),
             planted(2400, 0, 2400), np.full(2600, W, np.uint8), planted(3000, 900, 2000),
             planted(2700, 10, 2290), planted(3200, 200, 2500), planted(2900, 5, 2800)]
    r2 = np.concatenate([r] + extra)
    o2 = np.concatenate([o, o[-1] + np.cumsum([len(x) for x in extra])])
    db = sw.Database(handle, r2, o2, long_threshold=2500)
    m = sw.capi.builtin_matrix(mid)
    want = {len(q): oracle.scan(q, r2, o2, mat=m, gap_open=go, gap_extend=ge, nthreads=16) for q in (qa, qb)}
    # the first scan of A is fp16-first (nothing observed yet) and teaches
    # the database its int16-first routing for queries of >= 2,300 aa
    assert np.array_equal(db.scan(qa, m, go, ge), want[2300])
    assert np.array_equal(db.scan(qa, m, go, ge), want[2300])
    assert "+lpt" not in handle.last_kernel(), handle.last_kernel()
    assert np.array_equal(db.scan(qb, m, go, ge), want[1500])
    assert handle.last_kernel().endswith("+lpt+drain"), handle.last_kernel()
    for order in ([qa, qb, qa, qb], [qb, qa, qb, qa, qb], [qa, qa, qb, qb, qa, qb]):
        out = db.scan_batch(order, m, go, ge)
        for k, q in enumerate(order):
            assert np.array_equal(out[k], want[len(q)]), (k, len(q), np.nonzero(out[k] != want[len(q)])[0][:10])
    db.close()


@pytest.mark.parametrize("scoring", [(1, 12, 1), (0, 2, 2), (1, 14, 3)])
@pytest.mark.parametrize("form", ["single", "merged"])
def test_single_wave_block_widths(sw, oracle, handle, knobs, scoring, form):
    """The single-wave fp16 pass (x2s_block, chained passes): block widths
    8 ... 136 (odd and even multiples of 8), queries of one pass (standalone
    kernel, no chaining), of two, and of up to six chained passes, planted
    near-copies that the guard flags for the rescue chain, both gap models;
    alone and inside the merged launch (the widest block by a wave pair, long
    subjects beside it), against the oracle.  (Round 5 ran a 16-column bias
    period with an LDS delay line through it: parity-green, 1.4 % fewer VALU
    instructions, 2.3 % slower: DESIGN.md §4.)"""
    mid, go, ge = scoring
    rng = np.random.default_rng(71)
    q0 = sw.synth.query(333, shard=71)
    subs = []
    for w in (8, 16, 24, 32, 40, 48, 56, 64, 72, 80, 96, 104, 120, 136):
        lens = rng.integers(max(1, w - 7), w + 1, size=64)
        subs += [sw.synth.query(int(n), shard=1000 * w + k) for k, n in enumerate(lens)]
    subs += [q0[:130].copy(), q0[100:200].copy(), np.concatenate([q0[:60], q0[:60]])]  # near-copies
    long_threshold = 100000
    if form == "merged":
        subs += [sw.synth.query(700, shard=72), sw.synth.query(650, shard=73), q0.copy()]  # long subjects
        long_threshold = 300
        knobs(lpt=1, pair_width=130)
    else:
        knobs(lpt=0, pair_width=100000)
    r = np.concatenate(subs)
    o = np.zeros(len(subs) + 1, dtype=np.int64)
    o[1:] = np.cumsum([len(x) for x in subs])
    db = sw.Database(handle, r, o, long_threshold=long_threshold)
    m = sw.capi.builtin_matrix(mid)
    for qlen in (40, 64, 65, 130, 200, 333):
        q = q0[:qlen]
        got = db.scan(q, m, go, ge)
        want = oracle.scan(q, r, o, mat=m, gap_open=go, gap_extend=ge)
        assert np.array_equal(got, want), (qlen, np.nonzero(got != want)[0][:10])
        if form == "merged" and qlen > 64:
            assert "+lpt" in handle.last_kernel(), handle.last_kernel()
    db.close()
