"""Time every ResNet-18 convolution (batch 32, 224x224) under each launch plan of
conv_gemm (pixel tile x channel tile x K splits) and print the auto plan's choice next
to the best, per layer and direction.  Used to tune conv_gemm_plan's heuristic.

    python scripts/resnet_conv_sweep.py [--batch 32] [--iters 20]
"""
import argparse
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

BF = torch.bfloat16


def layers(B):
    # (name, N, H, Cin, Cout, K, stride, pad)
    out = [("stem", B, 224, 4, 64, 7, 2, 3)]
    out += [("l1.3x3", B, 56, 64, 64, 3, 1, 1)]
    for i, (cin, cout, h) in enumerate(((64, 128, 56), (128, 256, 28), (256, 512, 14)), start=2):
        out += [(f"l{i}.3x3s2", B, h, cin, cout, 3, 2, 1), (f"l{i}.3x3", B, h // 2, cout, cout, 3, 1, 1),
                (f"l{i}.1x1s2", B, h, cin, cout, 1, 2, 0)]
    return out


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from ddp_amd import native

    C = native.require()
    dev = "cuda"
    plans = [(bp, bc, s) for bp, bc, s in itertools.product((64, 128), (64, 128), (1, 2, 4, 8))]
    rows = []
    for name, N, H, Cin, Cout, K, st, pd in layers(a.batch):
        OH = (H + 2 * pd - K) // st + 1
        x = torch.randn(N, H, H, Cin, device=dev).to(BF)
        w = (torch.randn(Cout, K, K, Cin, device=dev) * 0.05).to(BF)
        y = torch.empty(N, OH, OH, Cout, dtype=BF, device=dev)
        dy = torch.randn(N, OH, OH, Cout, device=dev).to(BF)
        dx = torch.empty_like(x)
        for kind in ("fwd", "dgrad"):
            if kind == "dgrad" and Cin == 4:
                continue
            res = {}
            C_rows = Cout if kind == "fwd" else Cin
            pars = (-1, 0) if (kind == "dgrad" and st == 2) else (-1,)
            for (bp, bc, s), par in itertools.product([(0, 0, 0)] + plans, pars):
                if bc and C_rows % bc:
                    continue
                if Cin == 4 and (bp, bc, s) != (0, 0, 0):
                    continue
                if bp == 0 and par != -1:
                    continue
                if kind == "fwd":
                    pbp, pbc, sp, nrows, _, used = C.conv_gemm_plan(x, y, K, K, st, pd, False, bp, bc, s)
                    stats = torch.empty(nrows, 2, Cout, device=dev)
                    part = torch.empty(sp * y.numel(), device=dev) if sp > 1 else None
                    fn = lambda: C.conv_gemm_fwd(x, w, None, y, K, K, st, pd, False, stats, part, bp, bc, s)  # noqa: E731
                else:
                    pbp, pbc, sp, _, used, _ = C.conv_gemm_plan(x, dy, K, K, st, pd, True, bp, bc, s, par)
                    part = torch.empty(sp * x.numel(), device=dev) if sp > 1 else None
                    fn = lambda: C.conv_gemm_dgrad(dy, w, None, dx, K, K, st, pd, part, bp, bc, s, par)  # noqa: E731
                tag = f"{pbp}x{pbc}/s{sp}" + ("/par" if kind == "dgrad" and used else "")
                key = "auto" if bp == 0 else tag
                if bp and key in res:
                    continue
                res[key] = (round(timeit(fn, a.iters), 2), tag)
            best = min(((v[0], v[1]) for k, v in res.items() if k != "auto"), default=res["auto"])
            flops = 2.0 * N * OH * OH * Cout * K * K * (3 if Cin == 4 else Cin)
            r = {"layer": name, "kind": kind, "auto_us": res["auto"][0], "auto_plan": res["auto"][1],
                 "best_us": best[0], "best_plan": best[1],
                 "auto_tflops": round(flops / res["auto"][0] / 1e6, 1),
                 "all": {k: v[0] for k, v in res.items()}}
            rows.append(r)
            print(json.dumps(r), flush=True)
        # weight gradient at the auto chunking of resnet_fn
        tiles = C.conv_gemm_wgrad_tiles(x, dy, K, K, st, pd)
        P = N * OH * OH
        res = {}
        auto_ppc = C.conv_gemm_wgrad_ppc(x, dy, K, K, st, pd)
        for target in ("auto", "auto/ks32", "auto/ks64", 128, 256, 512, 1024, 2048):
            ks = {"auto/ks32": 32, "auto/ks64": 64}.get(target, 0)
            if isinstance(target, str):
                ppc = auto_ppc
            else:
                ppc = -(-P // max(1, target // tiles))  # ceil(P / chunks), rounded up to 32
                ppc = max(32, -(-ppc // 32) * 32)
            ch = C.conv_gemm_wgrad_chunks(x, dy, K, K, st, pd, ppc)
            row = Cout * K * K * (3 if Cin == 4 else Cin)
            g = torch.zeros(row, device=dev)
            slab = torch.empty(ch, row, device=dev) if ch > 1 else None

            def fn():
                if ch == 1:
                    C.conv_gemm_wgrad(dy, x, g, K, K, st, pd, ppc, True, ks)
                else:
                    C.conv_gemm_wgrad(dy, x, slab, K, K, st, pd, ppc, False, ks)
                    C.grad_reduce([(slab, row, 0, row, ch, g, 1.0, True)])
            res[target] = (round(timeit(fn, a.iters), 2), ch)
        flops = 2.0 * N * OH * OH * Cout * K * K * (3 if Cin == 4 else Cin)
        best = min(res.items(), key=lambda kv: kv[1][0])
        r = {"layer": name, "kind": "wgrad", "tiles": tiles, "us_by_target_blocks": {str(k): v for k, v in res.items()},
             "best_tflops": round(flops / best[1][0] / 1e6, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
    tot = sum(r["auto_us"] for r in rows if "auto_us" in r)
    best = sum(r["best_us"] for r in rows if "best_us" in r)
    print(json.dumps({"sum_auto_us_fwd_dgrad": round(tot, 1), "sum_best_us_fwd_dgrad": round(best, 1)}))


if __name__ == "__main__":
    main()
