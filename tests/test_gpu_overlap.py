"""GPU: the bench's overlapped step (bench.py step()): the scan of step i on
one handle and stream, the device top-K of the step before on a second
handle and a high-priority stream, two score buffers ordered by events.
Every step scans a DIFFERENT query, so a top-K that read a buffer the next
scan was rewriting would rank the wrong query: each step's keys must equal
the oracle's top-K of its own query."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scoring", [(1, 12, 1), (0, 2, 2)])
def test_overlapped_scan_and_topk(sw, oracle, scoring):
    import torch
    mid, go, ge = scoring
    dev = torch.device("cuda", 0)
    res, offs = sw.synth.database(8000, shard=31)
    n = len(offs) - 1
    h = sw.Handle(0, env_opts=False)
    stream = torch.cuda.Stream(dev)
    h.set_stream(stream.cuda_stream)
    xstream = torch.cuda.Stream(dev, priority=-1)
    xh = sw.Handle(0, env_opts=False)
    xh.set_stream(xstream.cuda_stream)
    db = sw.Database(h, res, offs)
    m = sw.capi.builtin_matrix(mid)
    queries = [sw.synth.query(L, shard=40 + i) for i, L in enumerate((120, 375, 200, 640, 90, 300, 500, 64))]
    K = 50
    bufs = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in range(2)]
    tops = [torch.empty(K, dtype=torch.int64, device=dev) for _ in queries]
    scanned = [torch.cuda.Event(), torch.cuda.Event()]
    ranked = [torch.cuda.Event(), torch.cuda.Event()]
    for i, q in enumerate(queries):
        b = i % 2
        if i >= 2:
            stream.wait_event(ranked[b])  # step i-2's top-K has read this buffer
        db.scan_device(q, bufs[b].data_ptr(), m, go, ge)
        scanned[b].record(stream)
        xstream.wait_event(scanned[b])
        xh.topk_device(bufs[b].data_ptr(), n, K, tops[i].data_ptr())
        ranked[b].record(xstream)
    torch.cuda.synchronize()
    ids = np.arange(n, dtype=np.int32)
    for i, q in enumerate(queries):
        want = oracle.scan(q, res, offs, mat=m, gap_open=go, gap_extend=ge, nthreads=16)
        assert np.array_equal(tops[i].cpu().numpy(), sw.dist.local_topk(want, ids, K)), (i, len(q))
    db.close()
    xh.close()
    h.close()
