"""Collective fingerprinting catches rank-divergent collective sequences (bug B7)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddp_amd.parallel import free_port


def _worker(rank, ws, port, diverge, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    from ddp_amd.utils.debug import CollectiveDivergence, CollectiveTracer

    with CollectiveTracer() as tr:
        t = torch.zeros(3)
        dist.broadcast(t, src=0)
        dist.all_reduce(t)
        if diverge:  # same bytes on the wire (gloo pairs them) but a different logical tensor
            dist.broadcast(torch.zeros(6) if rank == 0 else torch.zeros(2, 3), src=0)
        try:
            tr.verify()
            q.put((rank, "ok"))
        except CollectiveDivergence as e:
            q.put((rank, str(e)))
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("diverge", [False, True])
def test_collective_fingerprint(diverge):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(2, free_port(), diverge, q), nprocs=2, start_method="spawn")
    res = dict(q.get() for _ in range(2))
    if diverge:
        assert all("diverges" in v and "call #2" in v for v in res.values()), res
    else:
        assert res == {0: "ok", 1: "ok"}


def test_step_timer_cpu():
    from ddp_amd.utils.profiling import StepTimer, images_per_sec

    t = StepTimer()
    for _ in range(3):
        with t("work"):
            sum(range(1000))
    s = t.summary()
    assert s["work"]["n"] == 3 and s["work"]["total_ms"] >= 0
    assert images_per_sec(100, 0.5) == 200
