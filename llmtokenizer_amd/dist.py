"""Multi-GPU sharded training under torch.distributed (one process per GPU).

torch.distributed (any backend; bench.py uses gloo) only carries the RCCL
unique id from rank 0 to the other ranks; the per-merge exchange runs inside
libbpe_amd.so on its own RCCL communicator over xGMI (include/bpe_gpu.h).
"""
from . import api


def rccl_group(device):
    """ShardGroup holding this rank's shard; shard index == rank"""
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    obj = [api.comm_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return api.ShardGroup(device, nranks=world, rank=rank, comm_id=obj[0])


def shard_range(n_total, rank, world):
    """contiguous [lo, hi) slice of an n_total-byte corpus for `rank`"""
    step = n_total // world
    lo = rank * step
    return lo, (n_total if rank == world - 1 else lo + step)
