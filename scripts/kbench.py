"""Per-kernel microbenchmark of the SimpleCNN step kernels (B=32 shapes by default).

Each variant is launched REPS times back to back inside a captured CUDA/HIP graph
and replayed; the reported time is (replay wall time) / REPS, i.e. the in-graph
cost of one launch including its dependent-kernel boundary - the quantity that
adds up to the engine's step time.  ``noop`` gives the per-launch floor.

    python scripts/kbench.py [--batch 32] [--reps 50] [--iters 20] [--only conv3x3_fwd]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ddp_amd import native  # noqa: E402

BF = torch.bfloat16


def timed(fn, reps, iters, eager=False):
    if eager:  # plain launches (for counter collection); host-bound timing
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return float("nan")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # warm / lazy init outside capture
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
    return e0.elapsed_time(e1) * 1000.0 / (iters * reps)  # us per launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--eager", action="store_true", help="no graphs (rocprofv3 --pmc runs)")
    a = ap.parse_args()
    C = native.require()
    dev = "cuda"
    B, H, W, C1, C2, NO = a.batch, 28, 28, 32, 64, 10
    HW = H * W
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g)  # noqa: E731
    x_u8 = torch.randint(0, 256, (60000, HW), dtype=torch.uint8, device=dev)
    idx = torch.randperm(60000, device=dev, generator=g).to(torch.int32)
    ctr = torch.zeros(1, dtype=torch.int32, device=dev)
    labels = torch.randint(0, 10, (60000,), dtype=torch.int32, device=dev)
    w1, b1 = r(C1, 9) * 0.3, r(C1) * 0.1
    w2 = (r(C2, 9, C1) * 0.05).to(BF)
    w2t = torch.empty(C2 * 9 * C1, dtype=BF, device=dev)
    C.transpose_w(w2.float().contiguous().view(C2, 3, 3, C1), w2t)
    b2 = r(C2) * 0.1
    wfc = (r(NO, HW, C2) * 0.01).to(BF)
    a1 = torch.relu(r(B, H, W, C1)).to(BF)
    a2 = torch.empty(B, H, W, C2, dtype=BF, device=dev)
    part = torch.empty(2 * NO * C.conv3x3_dgrad_blocks(B, H, W, 1), device=dev)
    dl = r(B, NO) * 0.01
    dz2 = torch.empty(B, H, W, C2, dtype=BF, device=dev)
    dz1 = torch.empty(B, H, W, C1, dtype=BF, device=dev)
    dWfc = torch.empty(NO * HW * C2, device=dev)
    lossr = torch.empty(B, device=dev)
    losso = torch.empty(1, device=dev)
    dbias = torch.empty(NO, device=dev)
    bfc = r(NO)
    res = {}

    def run(name, fn):
        if a.only and a.only not in name:
            return
        try:
            res[name] = round(timed(fn, a.reps, a.iters, a.eager), 2)
        except Exception as e:  # report, keep going
            res[name] = f"error: {e}"
        print(f"{name:48s} {res[name]}", flush=True)

    run("noop 1 block", lambda: C.noop(1))
    run("noop 256 blocks", lambda: C.noop(256))
    run("noop 1024 blocks", lambda: C.noop(1024))
    run("conv1_fwd u8", lambda: C.conv1_fwd(x_u8, idx, ctr, B, 0, w1, b1, a1, B, H, W))
    for pxt in (1, 2):
        run(f"conv3x3_fwd pxt{pxt} relu", lambda: C.conv3x3_fwd(a1, w2, b2, a2, True, None, None, NO, pxt))
        run(f"conv3x3_fwd pxt{pxt} +fc", lambda: C.conv3x3_fwd(a1, w2, b2, a2, True, wfc, part, NO, pxt))
    C.conv3x3_fwd(a1, w2, b2, a2, True, wfc, part, NO, 2)
    run("xent_rows", lambda: C.xent_rows(part, HW, 128, bfc, labels, idx, dl, lossr, 1.0 / B))
    run("fc_bwd mask", lambda: C.fc_bwd(dl, a2.view(B, -1), wfc.view(NO, -1), dz2.view(B, -1), dWfc, 1.0,
                                         True, dbias, lossr, losso))
    for pxt in (1, 2):
        nblk = C.conv3x3_dgrad_blocks(B, H, W, pxt)
        w1slab = torch.empty(nblk * 320, device=dev)
        run(f"conv3x3_dgrad pxt{pxt} mask_x", lambda: C.conv3x3_dgrad(dz2, None, w2t, a1, dz1, pxt))
        run(f"conv3x3_dgrad pxt{pxt} fused_w1", lambda: C.conv3x3_dgrad_fused_w1(
            dz2, w2t, a1, dz1, x_u8, idx, ctr, B, 0, w1slab, pxt))
    for R in (2, 4, 7, 14):
        nb = C.conv3x3_wgrad_blocks(B, H, R)
        slab = torch.empty(nb * (C2 * 9 * C1 + C2), device=dev)
        run(f"conv3x3_wgrad R{R} ({nb} blk)", lambda: C.conv3x3_wgrad(dz2, None, a1, slab, R))
    nb = C.conv3x3_wgrad_blocks(B, H, 7)
    slab = torch.empty(nb * (C2 * 9 * C1 + C2), device=dev)
    w1slab = torch.empty(C.conv3x3_dgrad_blocks(B, H, W, 2) * 320, device=dev)
    gw = torch.empty(C2 * 9 * C1 + C2 + 320, device=dev)
    n_w2 = C2 * 9 * C1
    o1, o2 = n_w2 + C2, n_w2 + C2 + 288
    segs = [(slab, n_w2 + C2, 0, n_w2, nb, gw[:n_w2], 1.0), (slab, n_w2 + C2, n_w2, C2, nb, gw[n_w2:o1], 1.0),
            (w1slab, 320, 0, 288, w1slab.numel() // 320, gw[o1:o2], 1.0),
            (w1slab, 320, 288, 32, w1slab.numel() // 320, gw[o2:o2 + 32], 1.0)]
    run("grad_reduce (4 segs)", lambda: C.grad_reduce(segs))
    n = 520586
    p = r(n + 64)[:n]
    gr = r(n + 64)[:n] * 0.01
    sh = torch.empty(n, dtype=BF, device=dev)
    run("sgd plain", lambda: C.sgd(p, gr, None, 0.01, 0.0, 0.0, 0.0, False, False, False, True, []))
    run("sgd +bf16 shadow", lambda: C.sgd(p, gr, None, 0.01, 0.0, 0.0, 0.0, False, False, False, True,
                                          [(0, n, sh, 1, 0, 0, 0)]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"batch": B, "reps": a.reps, "us_per_launch": res}, f, indent=1)


if __name__ == "__main__":
    main()
