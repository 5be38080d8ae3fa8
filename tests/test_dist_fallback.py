"""dist.first_job (bench.py's first N > 1 job): the ranks agree on a P2P
job's outcome, and a failure on ANY rank moves EVERY rank to an RCCL group.
CPU only: two gloo processes, stand-in group objects (no device)."""
import os
import socket

import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Group:
    def __init__(self, transport):
        self._t = transport
        self.closed = False
        self.jobs = 0

    def transport(self):
        return self._t

    def close(self):
        self.closed = True


def _worker(rank, world, port, fail_rank, transport, q, differ=False, kind="bpe"):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from llmtokenizer_amd import api, dist as bdist
        g = _Group(transport)

        def job(gg):
            gg.jobs += 1
            if rank == fail_rank:
                if kind == "runtime":
                    raise RuntimeError("not a transport failure (test)")
                raise api.BpeError("mailbox wait timed out (test)")
            return "md5-%d" % rank if differ else "md5"

        try:
            g2, ok = bdist.first_job(g, 0, job, make_rccl=lambda dev: _Group("rccl"))
            q.put((rank, ok, g2.transport(), g.closed, getattr(g2, "fallback_reason", None), None))
        except (api.BpeError, RuntimeError) as e:
            q.put((rank, None, None, g.closed, None, f"{type(e).__name__}: {e}"))
    finally:
        dist.destroy_process_group()


def _run(fail_rank, transport, world=2, differ=False, kind="bpe"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fail_rank, transport, q, differ, kind)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_first_job_success_keeps_the_p2p_group():
    for rank, ok, t, closed, why, err in _run(-1, "p2p"):
        assert ok and t == "p2p" and not closed and why is None and err is None


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_first_job_failure_on_one_rank_moves_every_rank_to_rccl(fail_rank):
    for rank, ok, t, closed, why, err in _run(fail_rank, "p2p"):
        assert ok is False and t == "rccl" and closed and err is None
        assert "mailbox wait timed out" in why


def test_first_job_failure_on_rccl_is_raised_on_every_rank():
    for rank, ok, t, closed, why, err in _run(1, "rccl"):
        assert ok is None and not closed and "sharded job failed" in err


def test_first_job_results_that_differ_move_every_rank_to_rccl():
    for rank, ok, t, closed, why, err in _run(-1, "p2p", differ=True):
        assert ok is False and t == "rccl" and closed and "results differ" in why


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_first_job_other_exception_is_raised_on_every_rank(fail_rank):
    """a failure that is not the transport's (no BpeError) is not retried on
    RCCL: every rank raises instead of one blocking in the fallback set-up"""
    for rank, ok, t, closed, why, err in _run(fail_rank, "p2p", kind="runtime"):
        assert ok is None and not closed
        if rank == fail_rank:
            assert err.startswith("RuntimeError: not a transport failure")
        else:
            assert err.startswith("BpeError: sharded job failed on another rank: RuntimeError")
