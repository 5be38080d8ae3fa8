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


def peer_problem(device, pcis):
    """why this rank cannot map the other ranks' mailboxes, or None.  pcis:
    every rank's device PCI bus id.  A peer device visible here must accept
    direct access (hipDeviceCanAccessPeer); one not visible here (another
    HIP_VISIBLE_DEVICES) is left to the IPC mapping itself."""
    local = {}
    for d in range(api.device_count()):
        try:
            local[api.device_pci(d).lower()] = d
        except api.BpeError:
            pass
    for r, pci in enumerate(pcis):
        peer = local.get(pci.lower())
        if peer is None or peer == device:
            continue
        if not api.peer_access(device, peer):
            return f"device {device} ({pcis[r]}) has no peer access to rank {r}'s device {peer}"
    return None


def p2p_group(device, max_merges, strict=True):
    """ShardGroup holding this rank's shard over P2P mailboxes; shard index ==
    rank.  max_merges bounds the merges of any train call on it.  The ranks
    agree on success: with strict=False a failure on ANY rank (no peer access
    between two ranks' devices, mailbox allocation, IPC export or mapping)
    returns None on every rank, and p2p_group.last_failure says why."""
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    g, err = None, None
    pcis = [None] * world
    try:  # (every rank reaches every all_gather_object below, whatever fails)
        mine = api.device_pci(device)
    except api.BpeError as e:
        mine, err = "", str(e)
    dist.all_gather_object(pcis, mine)
    try:
        if err is None:
            err = peer_problem(device, pcis)
        if err is None:
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
        p2p_group.last_failure = "; ".join(errs)
        if strict:
            raise api.BpeError("p2p group set-up failed: " + p2p_group.last_failure)
        return None
    p2p_group.last_failure = None
    return g


p2p_group.last_failure = None


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
    if g is not None:
        return g
    g = rccl_group(device)
    g.fallback_reason = "P2P set-up failed, RCCL instead: " + str(p2p_group.last_failure)
    return g


def first_job(g, device, job, make_rccl=None):
    """Run job(g) once on every rank; the ranks agree on the outcome.  A P2P
    group whose job failed on ANY rank (e.g. a bounded mailbox wait that timed
    out: the cross-device xGMI path is first exercised by a multi-GPU run) is
    closed on every rank and replaced by an RCCL group, whose fallback_reason
    says why.  job may return a digest of what every rank must agree on (the
    merges): digests that differ count as a failure too.  Returns (group, ok):
    ok False means the returned group is the new one and the caller loads its
    shard into it and runs the job again.  A failure on an RCCL group is
    raised (nothing to fall back to)."""
    import torch.distributed as dist
    err, dig, other = None, None, None
    try:
        dig = job(g)
    except api.BpeError as e:
        err = str(e)
    except Exception as e:  # (any failure: the other ranks must not block in the gather)
        err, other = f"{type(e).__name__}: {e}", e
    outs = [None] * dist.get_world_size()
    dist.all_gather_object(outs, (err, dig, other is not None))
    # not a transport failure somewhere: every rank raises (no fallback
    # group, whose set-up would wait for the failed rank)
    if other is not None:
        raise other
    fatal = [e for e, _, f in outs if f]
    if fatal:
        raise api.BpeError("sharded job failed on another rank: " + fatal[0])
    errs = [e for e, _, _ in outs if e]
    if not errs and len({d for _, d, _ in outs}) > 1:
        errs = ["the ranks' results differ"]
    if not errs:
        return g, True
    if g.transport() != "p2p":
        raise api.BpeError("sharded job failed: " + errs[0])
    g.close()
    g2 = (make_rccl or rccl_group)(device)
    g2.fallback_reason = "P2P job failed, RCCL instead: " + errs[0]
    return g2, False


def shard_range(n_total, rank, world):
    """contiguous [lo, hi) slice of an n_total-byte corpus for `rank`"""
    step = n_total // world
    lo = rank * step
    return lo, (n_total if rank == world - 1 else lo + step)
