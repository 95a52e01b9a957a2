"""the start-up check's independent oracle, on the CPU (gloo, 2 ranks).

The fused engine's verify_chain compares its xGMI-reduced gradient with every rank's local
gradient gathered over the process group and summed in rank order on the host
(engine/fused_step.py gather_rank_sum / oracle_mismatches); the agreed verdicts pick the
chain (chain_decision).  Here the same functions run in two gloo processes: a correct
reduction passes on both ranks, and a one-ulp error in ONE rank's reduced bucket makes BOTH
ranks agree to leave the xGMI plane (RCCL; "fail" without an RCCL plane)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddp_amd.engine.fused_step import agree, chain_decision, gather_rank_sum, oracle_mismatches


def test_chain_decision_table():
    assert chain_decision(True, True, True, True) == "keep"
    assert chain_decision(False, True, True, True) == "conservative"
    assert chain_decision(True, True, False, True) == "rccl"
    assert chain_decision(False, True, False, True) == "rccl"   # the plane itself is not trusted
    assert chain_decision(True, False, True, True) == "rccl"
    assert chain_decision(True, True, False, False) == "fail"   # gloo control plane: nothing to fall to
    assert chain_decision(True, False, True, False) == "fail"


def test_oracle_mismatch_is_bitwise():
    a = torch.tensor([1.0, -0.0, 2.5, 3.0])
    b = a.clone()
    b[1] = 0.0  # +0 vs -0: equal as numbers, different bits
    assert oracle_mismatches(a, a.clone(), [(0, 4)]) == 0
    assert oracle_mismatches(b, a, [(0, 4)]) == 1
    c = a.clone()
    c[3] = torch.nextafter(c[3], torch.tensor(1e9))
    assert oracle_mismatches(c, a, [(0, 2)]) == 0   # outside the bucket ranges: not compared
    assert oracle_mismatches(c, a, [(0, 2), (3, 1)]) == 1


def _worker(rank, world, port, corrupt_rank, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        n = 10_000
        ranges = [(0, 9_000), (9_000, 1_000)]
        local = torch.randn(n, generator=torch.Generator().manual_seed(100 + rank)) * (1.0 / world)
        # what a correct direct all-reduce leaves in every rank's buffer: the rank-order sum
        allin = [torch.randn(n, generator=torch.Generator().manual_seed(100 + r)) * (1.0 / world)
                 for r in range(world)]
        reduced = allin[0].clone()
        for r in range(1, world):
            reduced = reduced + allin[r]
        if rank == corrupt_rank:
            reduced[ranges[0][0]] = torch.nextafter(reduced[ranges[0][0]], torch.tensor(float("inf")))
        want = gather_rank_sum(local, world)
        bad = oracle_mismatches(reduced, want, ranges)
        store = dist.distributed_c10d._get_default_store()
        ok_all = agree(store, "test/oracle", rank, world, bad == 0)
        action = chain_decision(True, True, ok_all, have_rccl=True)
        action_gloo = chain_decision(True, True, ok_all, have_rccl=False)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", bad, action, action_gloo))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e), None, None, None))


@pytest.mark.parametrize("corrupt_rank", [None, 1])
def test_oracle_two_ranks_gloo(corrupt_rank):
    from ddp_amd.parallel import free_port

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, corrupt_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
    assert all(r[1] == "ok" for r in res), res
    if corrupt_rank is None:
        assert [r[2] for r in res] == [0, 0]
        assert {r[3] for r in res} == {"keep"}
    else:
        # only the corrupted rank sees the mismatch, but EVERY rank acts on it
        assert [r[2] for r in res] == [0 if r != corrupt_rank else 1 for r in range(world)]
        assert {r[3] for r in res} == {"rccl"} and {r[4] for r in res} == {"fail"}
