"""the multi-GPU placement is chosen on the node it runs on.

bench.py times every bitwise-equivalent placement (dist_mode 3 pair launch, 0 serial, 1
fork) on throwaway engines before the timed run and every rank agrees on the fastest through
the c10d store (engine/fused_step.py choose_placement / agree_placement); the record carries
``config.placement`` with the per-mode times.  Here with faked timings."""
import threading

import torch.distributed as dist

from ddp_amd.engine.fused_step import agree_placement, choose_placement, placement_candidates


def test_candidates_per_plane():
    assert placement_candidates("xgmi") == (4, 3, 0, 1)
    assert placement_candidates("xgmi1") == (4, 3, 0, 1)
    assert placement_candidates("xgmi", "fp32") == (3, 0, 1)  # (the step head is bf16)
    assert placement_candidates("rccl") == (0, 1)
    assert placement_candidates("rccl:Ring/LL") == (0, 1)
    assert placement_candidates("none") == ()


def test_slowest_rank_decides():
    # rank 0 alone would pick 3, but rank 1 is slow on it: the step is as slow as its slowest rank
    best, worst = choose_placement([{3: 40.0, 0: 50.0, 1: 60.0}, {3: 70.0, 0: 52.0, 1: 61.0}])
    assert best == 0 and worst == {0: 52.0, 1: 61.0, 3: 70.0}


def test_failed_mode_never_wins_and_ties_are_deterministic():
    best, worst = choose_placement([{3: None, 0: 50.0}, {3: 10.0, 0: 50.0}])
    assert best == 0 and worst[3] is None
    assert choose_placement([{3: 45.0, 0: 45.0, 1: 45.0}])[0] == 0
    assert choose_placement([{3: None}])[0] is None


def test_agree_through_store_two_ranks():
    store = dist.HashStore()
    times = {0: {3: 45.8, 0: 66.7, 1: 77.0}, 1: {3: 46.1, 0: 60.0, 1: 75.0}}
    out = {}

    def rank(r):
        out[r] = agree_placement(store, "t/placement", r, 2, times[r])

    th = [threading.Thread(target=rank, args=(r,)) for r in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    assert out[0] == out[1]
    best, worst = out[0]
    assert best == 3 and worst == {0: 66.7, 1: 77.0, 3: 46.1}


def test_single_rank_needs_no_store():
    assert agree_placement(None, "k", 0, 1, {3: 1.0, 0: 2.0}) == (3, {0: 2.0, 3: 1.0})
