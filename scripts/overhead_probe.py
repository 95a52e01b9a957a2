"""Fixed per-run overhead of a short timed region (the driver's ``--steps 20 --warmup 5``).

For a few graph chunk sizes and the eager path it times, on the host, the launch call
alone, launch + stream sync, and the device span (events on the engine stream) of a
K-step run.  wall - device = host launch latency + sync wake-up (what a short run pays
on top of K * step time)."""
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


def probe(eng, nsteps, trials):
    rows = []
    first = None
    for t in range(trials):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(eng.stream)
        eng.run_steps(nsteps)
        t1 = time.perf_counter()
        e1.record(eng.stream)
        eng.synchronize()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rows.append({"launch_us": (t1 - t0) * 1e6, "wall_us": (t2 - t0) * 1e6,
                     "dev_us": e0.elapsed_time(e1) * 1e3, "resync_us": (t3 - t2) * 1e6})
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
    for k, n in ((20, 20), (20, 1000), (10, 20)):
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
