"""The CPU tests' world-N gloo launcher (tests/gloo_ranks.py): a group whose
init fails is started again on a fresh port; a failure inside the ranks'
work is reported, never retried."""
import socket

import pytest

import gloo_ranks


def _sum_ranks(rank, world):
    import torch
    import torch.distributed as dist
    t = torch.tensor([rank + 1])
    dist.all_reduce(t)
    return rank, world, int(t.item())


def _raise_on_rank1(rank, world):
    if rank == 1:
        raise ValueError("rank 1's work failed")
    return rank


@pytest.mark.timeout(180)
def test_retries_a_group_whose_init_failed(monkeypatch):
    # the first port handed out is held by another listener: rank 0 cannot
    # host the rendezvous store there, the group's init fails, the launcher
    # starts it again on the next port
    busy = socket.socket()
    busy.bind(("127.0.0.1", 0))
    busy.listen(8)
    ports = [busy.getsockname()[1]]
    real, handed = gloo_ranks.free_port, []

    def port():
        handed.append(ports.pop() if ports else real())
        return handed[-1]

    monkeypatch.setattr(gloo_ranks, "free_port", port)
    try:
        got = gloo_ranks.run(_sum_ranks, 2, timeout=60)
    finally:
        busy.close()
    assert got == [(0, 2, 3), (1, 2, 3)] and len(handed) == 2


@pytest.mark.timeout(180)
def test_a_failure_in_the_work_is_not_retried():
    with pytest.raises(AssertionError, match="exited with"):
        gloo_ranks.run(_raise_on_rank1, 2, timeout=60)
