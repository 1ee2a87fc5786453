"""CPU: multi-rank sharding and the top-K exchange over torch.distributed
(gloo, world_size 2 — the same code path runs over RCCL on the GPU box)."""
import os
import socket

import numpy as np
import pytest


def test_shard_balance(sw):
    r, o = sw.synth.database(5000, shard=3)
    lens = o[1:] - o[:-1]
    for w in (1, 2, 3, 8):
        parts = sw.dist.shard_indices(lens, w)
        allidx = np.sort(np.concatenate(parts))
        assert np.array_equal(allidx, np.arange(5000))
        loads = [lens[p].sum() for p in parts]
        assert max(loads) - min(loads) <= lens.max()


def test_keys_roundtrip(sw):
    s = np.array([3, 9, 9, 0], dtype=np.int32)
    g = np.array([10, 4, 2, 7])
    keys = sw.dist.local_topk(s, g, 3)
    ids, sc = sw.dist.decode_keys(keys)
    assert ids.tolist() == [2, 4, 10] and sc.tolist() == [9, 9, 3]


def fake_scan(res, offs):
    """Deterministic stand-in scorer (tests the exchange, not the DP)."""
    return np.array([int(res[offs[k]:offs[k + 1]].astype(np.int64).sum()) % 97
                     for k in range(len(offs) - 1)], dtype=np.int32)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import _swpkg
    sw = _swpkg.load()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, o = sw.synth.database(3000, shard=11)
    ids, scores = sw.dist.search(fake_scan, r, o, 50, rank, world)
    q.put((rank, ids.tolist(), scores.tolist()))
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_topk_exchange(sw, world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r, o = sw.synth.database(3000, shard=11)
    full = fake_scan(r, o)
    want_ids, want_sc = sw.dist.decode_keys(sw.dist.local_topk(full, np.arange(3000), 50))
    for rank, ids, scores in got:
        assert ids == want_ids.tolist() and scores == want_sc.tolist(), rank
