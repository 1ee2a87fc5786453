"""Multi-GPU database search: residue-balanced shards + top-K exchange.

The reference is single-GPU (no NCCL/MPI, no cudaSetDevice).
Here the database shards embarrassingly (every subject is independent); the
only exchange is each rank's top-K (score, global id), gathered with one
all-gather (RCCL over xGMI on the GPU box, gloo in the CPU tests) and merged
identically on every rank.  K x 8 bytes per rank: latency-bound and tiny.

Ordering of hits: score descending, global id ascending (deterministic).
"""
import heapq

import numpy as np

ID_BITS = 31
ID_MASK = (1 << 32) - 1


def shard_indices(lengths, world):
    """Deal subjects to `world` ranks, longest first, each to the currently
    lightest rank (LPT), balancing residues (= DP cells for a fixed query).
    Returns one sorted index array per rank.  Deterministic."""
    lengths = np.asarray(lengths, dtype=np.int64)
    if world == 1:
        return [np.arange(len(lengths), dtype=np.int64)]
    order = np.argsort(-lengths, kind="stable")
    owner = np.empty(len(lengths), dtype=np.int64)
    # heap of (load, rank): the lightest rank, the lowest index among equals
    heap = [(0, r) for r in range(world)]
    for i, L in zip(order.tolist(), lengths[order].tolist()):
        load, r = heapq.heappop(heap)
        owner[i] = r
        heapq.heappush(heap, (load + L, r))
    return [np.nonzero(owner == r)[0] for r in range(world)]


def shard(residues, offsets, rank, world):
    """Rank `rank`'s share of ONE database (strong scaling): (global ids
    int32 [n_r], residues, offsets) of its LPT subjects, in id order."""
    idx = shard_indices(offsets[1:] - offsets[:-1], world)[rank]
    if world == 1:
        return idx.astype(np.int32), residues, offsets
    res, offs = subset(residues, offsets, idx)
    return idx.astype(np.int32), res, offs


def allgather_np(arr, group=None):
    """All-gather one equally shaped numpy array per rank -> [world, ...]
    (device tensors over nccl/RCCL, CPU tensors over gloo)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if dist.get_backend(group) == "nccl":
        t = t.to(torch.device("cuda", torch.cuda.current_device()))
        out = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=group)
        return out.cpu().numpy()
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return np.stack([o.numpy() for o in outs])


def subset(residues, offsets, idx):
    """Residues/offsets of the subjects `idx` (in that order)."""
    idx = np.asarray(idx, dtype=np.int64)
    lens = offsets[idx + 1] - offsets[idx]
    offs = np.zeros(len(idx) + 1, dtype=np.int64)
    offs[1:] = np.cumsum(lens)
    if len(idx) == 0:
        return np.zeros(0, dtype=np.uint8), offs
    res = np.concatenate([residues[offsets[i]:offsets[i + 1]] for i in idx])
    return res, offs


def encode_keys(scores, global_ids):
    """int64 keys that sort as (score desc, id asc) under a descending sort."""
    s = np.asarray(scores, dtype=np.int64)
    g = np.asarray(global_ids, dtype=np.int64)
    return (s << 32) | (((1 << ID_BITS) - 1) - g)


def decode_keys(keys):
    keys = np.asarray(keys, dtype=np.int64)
    return ((1 << ID_BITS) - 1) - (keys & ID_MASK), keys >> 32


def local_topk(scores, global_ids, k):
    keys = encode_keys(scores, global_ids)
    k = min(k, len(keys))
    if k == 0:
        return np.zeros(0, dtype=np.int64)
    part = np.argpartition(-keys, k - 1)[:k]
    return np.sort(keys[part])[::-1]


def merge_topk(key_lists, k):
    allk = np.concatenate([np.asarray(x, dtype=np.int64) for x in key_lists]) if key_lists else \
        np.zeros(0, dtype=np.int64)
    allk = allk[allk != np.iinfo(np.int64).min]  # padding from short shards
    return np.sort(allk)[::-1][:k]


def allgather_topk(keys, k, group=None):
    """All-gather every rank's top-k keys (padded to k) and merge.  Works with
    any torch.distributed backend (gloo on CPU tensors, nccl/RCCL on GPU)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    pad = np.full(k, np.iinfo(np.int64).min, dtype=np.int64)
    pad[:len(keys)] = keys[:k]
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    t = torch.from_numpy(pad).to(dev)
    if backend == "nccl":
        out = torch.empty(world * k, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, t, group=group)
        return merge_topk([out.cpu().numpy()], k)
    outs = [torch.empty(k, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return merge_topk([o.numpy() for o in outs], k)


def search(scan_fn, residues, offsets, k, rank, world, group=None):
    """Strong-scaling search of ONE database over `world` ranks.

    scan_fn(res, offs) -> int32 scores of that shard (on the GPU this is
    Database(...).scan).  Returns the merged global top-k as (ids, scores)."""
    lengths = offsets[1:] - offsets[:-1]
    idx = shard_indices(lengths, world)[rank]
    res, offs = subset(residues, offsets, idx)
    scores = scan_fn(res, offs) if len(idx) else np.zeros(0, dtype=np.int32)
    keys = local_topk(scores, idx, k)
    if world > 1:
        keys = allgather_topk(keys, k, group)
    return decode_keys(keys)
