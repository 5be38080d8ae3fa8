"""Multi-GPU sharded training under torch.distributed (one process per GPU).

torch.distributed (any backend; bench.py uses gloo) only carries set-up data
between the ranks: the P2P mailbox handles (default transport) or the RCCL
unique id.  The per-merge exchange runs inside libbpe_amd.so: one push kernel
over xGMI into the peers' IPC-mapped mailboxes (p2p.hip), or RCCL
collectives on the library's own communicator (include/bpe_gpu.h).
"""
import os

from . import api


def rccl_group(device):
    """ShardGroup holding this rank's shard over RCCL; shard index == rank"""
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    obj = [api.comm_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return api.ShardGroup(device, nranks=world, rank=rank, comm_id=obj[0])


def p2p_group(device, max_merges, strict=True):
    """ShardGroup holding this rank's shard over P2P mailboxes; shard index ==
    rank.  max_merges bounds the merges of any train call on it.  The ranks
    agree on success: with strict=False a failure on ANY rank (mailbox
    allocation, IPC export or mapping) returns None on every rank."""
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    g, err = None, None
    try:
        g = api.ShardGroup(device, nranks=world, rank=rank, p2p_max_merges=max_merges)
    except api.BpeError as e:
        err = str(e)
    handles = [None] * world
    dist.all_gather_object(handles, g.p2p_handle if g else None)
    if g and all(h is not None for h in handles):
        try:
            g.p2p_connect(handles)
        except api.BpeError as e:
            err = str(e)
    oks = [None] * world
    dist.all_gather_object(oks, err)
    errs = [e for e in oks if e is not None] + ([] if all(h is not None for h in handles) else ["a rank failed"])
    if errs:
        if g:
            g.close()
        if strict:
            raise api.BpeError("p2p group set-up failed: " + "; ".join(errs))
        return None
    return g


def group(device, max_merges, transport=None):
    """P2P group (default; RCCL if P2P cannot be set up on every rank) or RCCL
    group (transport="rccl" or BPE_XPORT=rccl).  Every rank must pick the same
    transport."""
    transport = transport or os.environ.get("BPE_XPORT", "p2p")
    if transport == "rccl":
        return rccl_group(device)
    if transport != "p2p":
        raise ValueError(f"unknown transport {transport!r}")
    g = p2p_group(device, max_merges, strict=False)
    return g if g is not None else rccl_group(device)


def shard_range(n_total, rank, world):
    """contiguous [lo, hi) slice of an n_total-byte corpus for `rank`"""
    step = n_total // world
    lo = rank * step
    return lo, (n_total if rank == world - 1 else lo + step)
