"""Child process of tests/test_gpu_exchange.py (its own process: it creates
a torch.distributed process group).  The exchange of bench.py's step on one
GPU: a scan on the main stream, the device top-K on a second handle and a
high-priority stream, a one-rank RCCL all_gather_into_tensor of the keys
(the collective bench.py runs at N > 1), the other N - 1 rows copied in and
the device merge of N x K keys, all on the exchange stream.  Prints
"exchange ok" when the keys equal the CPU top-K of the scores and the merge
of N identical lists equals each of its best K / N keys N times."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as tdist

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import _swpkg  # noqa: E402


def main():
    sw = _swpkg.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    tdist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1, device_id=dev)
    N, K = 8, 64
    res, offs = sw.synth.database(6000, shard=17)
    n = len(offs) - 1
    h = sw.Handle(0, env_opts=False)
    stream = torch.cuda.Stream(dev)
    h.set_stream(stream.cuda_stream)
    xstream = torch.cuda.Stream(dev, priority=-1)
    xh = sw.Handle(0, env_opts=False)
    xh.set_stream(xstream.cuda_stream)
    db = sw.Database(h, res, offs)
    m = sw.capi.builtin_matrix(1)
    scores = torch.zeros(n, dtype=torch.int32, device=dev)
    top = torch.empty((1, K), dtype=torch.int64, device=dev)
    gathered = torch.empty((N, 1, K), dtype=torch.int64, device=dev)
    final = torch.empty((1, K), dtype=torch.int64, device=dev)
    with torch.cuda.stream(stream):
        db.scan_device(sw.synth.query(375, shard=4), scores.data_ptr(), m, 12, 1)
    h.stream_wait_scan(xstream.cuda_stream)
    with torch.cuda.stream(xstream):
        xh.topk_device(scores.data_ptr(), n, K, top[0].data_ptr())
        tdist.all_gather_into_tensor(gathered[:1], top)
        gathered[1:].copy_(top.unsqueeze(0).expand(N - 1, 1, K))
        merged = gathered[:, 0, :].contiguous()
        xh.topk_keys_device(merged.data_ptr(), N * K, K, final[0].data_ptr())
    torch.cuda.synchronize()
    keys = top[0].cpu().numpy()
    ids, sc = sw.capi.decode_keys(keys)
    want_ids, want_sc = sw.capi.topk(scores.cpu().numpy(), K)
    assert np.array_equal(ids, want_ids) and np.array_equal(sc, want_sc), "device top-K != CPU top-K"
    assert np.array_equal(gathered[0, 0].cpu().numpy(), keys), "all-gather row 0 != the rank's keys"
    assert np.array_equal(final[0].cpu().numpy(), np.repeat(keys[:K // N], N)), "merge of N copies"
    db.close()
    xh.close()
    h.close()
    tdist.destroy_process_group()
    print("exchange ok", flush=True)


if __name__ == "__main__":
    main()
