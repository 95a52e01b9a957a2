"""The xGMI cost-model bucket plan (parallel/bucket_model.py) pinned on CPU:
SimpleCNN's engine plan, ResNet-18's module plan at 2 / 4 / 8 ranks, the DP's optimality on
small cases against brute force, and the one-/two-shot crossover."""
import itertools

import pytest
import torch

from ddp_amd.models import SimpleCNN, resnet18
from ddp_amd.models.layers import flat_space
from ddp_amd.parallel.bucket_model import (XgmiCost, backward_times_us, engine_plan, module_plan,
                                           plan_buckets, ready_times_us)
from ddp_amd.parallel.ddp import bucket_plan


@pytest.mark.parametrize("world", [2, 4, 8])
def test_simplecnn_engine_plan_is_one_bucket_per_stage(world):
    """The fused engine finishes all fc gradients at once (stage 0) and all conv gradients
    at once (stage 1): splitting a stage only adds fixed costs, so the model picks exactly
    the reference DDP's rebuilt layout - [fl.*] then [net.2.*, net.0.*] - and the conv
    bucket's one-shot kernel."""
    fs = flat_space(SimpleCNN())
    buckets, finish = engine_plan(fs, world)
    assert buckets == [["fl.bias", "fl.weight"], ["net.2.bias", "net.2.weight", "net.0.bias", "net.0.weight"]]
    assert buckets == bucket_plan(fs)  # == torch's 1 MiB / 25 MiB rule here
    cost = XgmiCost(world)
    assert cost.allreduce(18816 * 4)[1] == "oneshot"
    assert cost.allreduce(501770 * 4)[1] == ("oneshot" if world == 2 else "twoshot")
    assert finish > 18.0  # the last (conv) all-reduce follows the conv backward


@pytest.mark.parametrize("world,nb", [(2, 2), (4, 2), (8, 2)])
def test_resnet18_module_plan(world, nb):
    """ResNet-18 (BASELINE config 5, B = 32, 224^2): the last-ready bucket is small (its
    all-reduce is the only one after the backward), the big bucket's all-reduce runs under
    the rest of the backward, and the plan beats torch's size rule under the same model."""
    m = resnet18()
    fs = flat_space(m)
    x = torch.randn(32, 3, 224, 224)
    buckets, finish = module_plan(fs, m, x, world)
    assert [n for b in buckets for n in b] == list(fs.names)
    assert len(buckets) == nb
    last = sum(fs.numels[n] * 4 for n in buckets[-1])
    assert last < 1 << 20, last  # < 1 MiB: a few us after the backward
    bwd = backward_times_us(m, x)
    ready = ready_times_us(fs.names, {n: n.rsplit(".", 1)[0] for n in fs.names}, bwd)
    assert ready[-1] < finish < ready[-1] + 15.0  # comm almost fully hidden
    cost, t, j = XgmiCost(world), 0.0, 0
    for b in bucket_plan(fs):  # torch's rule, same cost model
        j += len(b)
        t = max(ready[j - 1], t) + cost.allreduce(sum(fs.numels[n] * 4 for n in b))[0]
    assert finish < t


def test_dp_matches_brute_force():
    """Exhaustive check of the DP on random small instances (every contiguous split)."""
    g = torch.Generator().manual_seed(0)
    cost = XgmiCost(8)
    for _ in range(25):
        n = int(torch.randint(2, 8, (1,), generator=g))
        sizes = [int(v) for v in torch.randint(1_000, 4_000_000, (n,), generator=g)]
        ready = sorted(float(v) for v in torch.rand(n, generator=g) * 300)

        def finish(cuts):
            t, i = 0.0, 0
            for j in list(cuts) + [n]:
                t = max(ready[j - 1], t) + cost.allreduce(sum(sizes[i:j]))[0]
                i = j
            return t

        best = min(finish(c) for k in range(n) for c in itertools.combinations(range(1, n), k))
        bounds, f = plan_buckets(sizes, ready, cost)
        # the DP returns the fewest buckets within 0.5 % of the optimum
        assert best - 1e-6 <= f <= best * 1.005 + 1e-6
        assert abs(finish([b for _, b in bounds[:-1]]) - f) < 1e-6


def test_oneshot_crossover():
    for w in (4, 8):
        c = XgmiCost(w)
        lim = c.oneshot_max_elems()
        assert c.allreduce(lim * 4)[1] == "oneshot" and c.allreduce((lim + 64) * 4)[1] == "twoshot"
