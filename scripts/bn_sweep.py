"""In-graph timing of the BatchNorm backward (bn_bwd = strip reduce + apply) on every
ResNet-18 BN shape at batch 32, across the reduce grid's pixels per block
(resnet_ops.hip bn_bwd_rows).  Each point is REPS back-to-back launches captured in one
hipGraph and replayed; JSON lines to stdout.

    python scripts/bn_sweep.py [--px 98,196,392,784] [--reps 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ddp_amd import native  # noqa: E402

BF = torch.bfloat16
# (pixels, channels) of the batch-32 ResNet-18 BN layers
SHAPES = [(32 * 112 * 112, 64), (32 * 56 * 56, 64), (32 * 28 * 28, 128), (32 * 14 * 14, 256),
          (32 * 7 * 7, 512)]


def graph_time(fn, reps, iters):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / (iters * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--px", default="98,196,392,784,1568")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C = native.require()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for P, Ch in SHAPES:
        dout = torch.randn(P, Ch, device=dev).to(BF)
        out = torch.randn(P, Ch, device=dev).to(BF)
        y = torch.randn(P, Ch, device=dev).to(BF)
        mean = torch.randn(Ch, device=dev) * 0.1
        invstd = torch.rand(Ch, device=dev) + 0.5
        gamma = torch.randn(Ch, device=dev)
        sums = torch.empty(2 * Ch, device=dev)
        dg, db = torch.empty(Ch, device=dev), torch.empty(Ch, device=dev)
        dy, dres = torch.empty_like(y), torch.empty_like(y)
        ref = None
        for t in (int(v) for v in a.px.split(",")):
            C.bn_bwd_set_px_per_block(t)
            ws = torch.empty(C.bn_bwd_rows(P, Ch), 2, Ch, device=dev)

            def fn():
                C.bn_bwd(dout, out, y, mean, invstd, gamma, float(P), ws, sums, dg, db, False, dy, dres)

            us = graph_time(fn, a.reps, a.iters)
            fn()
            torch.cuda.synchronize()
            got = torch.cat([sums, dy.float().flatten()[:4096]])
            if ref is None:
                ref = got.clone()
            err = float((got - ref).abs().max() / (ref.abs().max() + 1e-30))
            print(json.dumps({"P": P, "C": Ch, "px_per_block": t, "rows": C.bn_bwd_rows(P, Ch),
                              "us": round(us, 2), "rel_err_vs_first": err}), flush=True)
    C.bn_bwd_set_px_per_block(392)


if __name__ == "__main__":
    main()
