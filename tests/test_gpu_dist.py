"""GPU: strong-scaling search of ONE database over 2 ranks (gloo collectives,
both ranks on the one GPU of the test box) with the real HIP scan, against
the oracle's global top-K (north_star: bit-exact top-score
list).  Also bench.py's per-rank device top-K with an id map."""
import os

import numpy as np
import pytest

from test_dist import free_port

pytestmark = pytest.mark.gpu

QUERY = "P07327"
N_DB = 6000
K = 50


def _db(sw):
    return sw.synth.database(N_DB, shard=7)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import _swpkg
    from conftest import read_query
    sw = _swpkg.load()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    h = sw.Handle(0, env_opts=False)
    qc = sw.encode(read_query(QUERY))
    mat = sw.capi.builtin_matrix(1)
    r, o = _db(sw)

    def scan(res, offs):
        db = sw.Database(h, res, offs)
        try:
            return db.scan(qc, mat, 12, 1)
        finally:
            db.close()

    ids, scores = sw.dist.search(scan, r, o, K, rank, world)
    q.put((rank, ids.tolist(), scores.tolist()))
    h.close()
    dist.destroy_process_group()


def test_two_rank_search_equals_oracle_topk(sw, oracle):
    import torch.multiprocessing as mp
    from conftest import read_query
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r, o = _db(sw)
    want = oracle.scan(sw.encode(read_query(QUERY)), r, o, mat=sw.capi.builtin_matrix(1), gap_open=12,
                       gap_extend=1)
    want_ids, want_sc = sw.dist.decode_keys(sw.dist.local_topk(want, np.arange(N_DB), K))
    for rank, ids, scores in got:
        assert ids == want_ids.tolist() and scores == want_sc.tolist(), rank


def test_device_topk_with_id_map(sw, handle):
    """sw_topk_device_ids: keys carry the mapped (global) ids, ties by id."""
    import torch
    rng = np.random.default_rng(5)
    for n, k in ((1000, 10), (70000, 100), (40000, 4096)):
        scores = rng.integers(0, 50, size=n).astype(np.int32)  # many ties
        gids = np.sort(rng.choice(10 * n, size=n, replace=False)).astype(np.int32)
        rng.shuffle(gids)
        s = torch.from_numpy(scores).cuda()
        g = torch.from_numpy(gids).cuda()
        out = torch.empty(k, dtype=torch.int64, device="cuda")
        handle.set_stream(torch.cuda.current_stream().cuda_stream)
        handle.topk_device_ids(s.data_ptr(), n, g.data_ptr(), k, out.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), sw.dist.local_topk(scores, gids, k)), (n, k)
    handle.set_stream(None)
