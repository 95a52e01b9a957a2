"""Fixed per-run overhead of a short timed region (the driver's ``--steps 20 --warmup 5``).

For a few graph chunk sizes and the eager path it times, on the host, from a synchronized
device: ``pre_launch_us`` - run_steps' Python before the graph launch call, ``launch_us`` -
until run_steps returns (hipGraphLaunch submits the graph's nodes), ``wall_us`` - until
torch.cuda.synchronize() returns (what a short run pays on top of K * step time)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ddp_amd import native  # noqa: E402
from ddp_amd.data import DeviceMNIST, synthetic_mnist  # noqa: E402
from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine  # noqa: E402
from ddp_amd.models import SimpleCNN  # noqa: E402
from ddp_amd.ops import FusedSGD  # noqa: E402


def make(k, use_graph=True):
    torch.manual_seed(0)
    model = SimpleCNN().cuda()
    opt = FusedSGD(model, lr=0.01)
    imgs, labels = synthetic_mnist()
    data = DeviceMNIST(imgs, labels, torch.device("cuda", 0), "synthetic")
    eng = FusedSimpleCNNEngine(model, opt, data, 32, 1, 0, None,
                               EngineOptions(graph_steps=k, use_graph=use_graph))
    eng.refresh()
    if use_graph:
        eng.run_steps(0)
        eng._ensure_graph()
    eng.run_steps(5)
    eng.synchronize()
    return eng


class _Timed:
    """The engine's native handle with replay() timestamped on entry (host time spent in
    run_steps before the graph launch call)."""

    def __init__(self, inner):
        self._inner, self.t_replay = inner, None

    def replay(self):
        self.t_replay = time.perf_counter()
        return self._inner.replay()

    def __getattr__(self, name):
        return getattr(self._inner, name)


def probe(eng, nsteps, trials):
    rows = []
    first = None
    timed = _Timed(eng.eng)
    eng.eng = timed
    for t in range(trials):
        torch.cuda.synchronize()
        timed.t_replay = None
        t0 = time.perf_counter()
        eng.run_steps(nsteps)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rows.append({"pre_launch_us": ((timed.t_replay or t1) - t0) * 1e6, "launch_us": (t1 - t0) * 1e6,
                     "wall_us": (t2 - t0) * 1e6})
        if t == 0:
            first = {k: round(v, 1) for k, v in rows[0].items()}
    rows.sort(key=lambda r: r["wall_us"])
    med = rows[len(rows) // 2]
    out = {k: round(v, 1) for k, v in med.items()}
    out["first"] = first  # the driver's case: the first replay after capture + warm-up
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=15)
    args = ap.parse_args()
    native.require()
    out = {}
    for k, n in ((20, 20), (20, 1000), (5, 20)):
        eng = make(k)
        out[f"graph{k}_steps{n}"] = probe(eng, n, args.trials)
        print(json.dumps({f"graph{k}_steps{n}": out[f"graph{k}_steps{n}"]}), flush=True)
    eng = make(20, use_graph=False)
    out["eager_steps20"] = probe(eng, 20, args.trials)
    print(json.dumps({"eager_steps20": out["eager_steps20"]}), flush=True)
    # bare sync latency of an idle stream / an empty-kernel round trip
    t = []
    for _ in range(50):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e6)
    out["idle_sync_us"] = round(sorted(t)[25], 1)
    x = torch.zeros(1, device="cuda")
    t = []
    for _ in range(50):
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e6)
    out["one_kernel_roundtrip_us"] = round(sorted(t)[25], 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
