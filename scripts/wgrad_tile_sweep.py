"""Weight-gradient tile x pixel-chunking sweep on the batch-32 ResNet-18 layers.

For every layer and forced block tile (64/128 x 64/128; `auto` = conv_gemm.hip
wgrad_tile), the grid is chunked over pixels to about `target` blocks (`1` = one chunk).
Each point is timed as wgrad + the chunk reduction (grad_reduce) when chunked.  JSON
lines to stdout, one per layer:

    python scripts/wgrad_tile_sweep.py [--batch 32] [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from resnet_conv_sweep import layers, timeit  # noqa: E402

BF = torch.bfloat16
TILES = ["auto", (64, 64), (128, 64), (64, 128), (128, 128)]
TARGETS = ["auto", 1, 256, 512, 1024]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from ddp_amd import native

    C = native.require()
    dev = "cuda"
    for name, N, H, Cin, Cout, K, st, pd in layers(a.batch):
        if Cin == 4:
            continue
        OH = (H + 2 * pd - K) // st + 1
        x = torch.randn(N, H, H, Cin, device=dev).to(BF)
        dy = torch.randn(N, OH, OH, Cout, device=dev).to(BF)
        P = N * OH * OH
        row = Cout * K * K * Cin
        flops = 2.0 * P * row
        res = {}
        ref = None
        for tile in TILES:
            if tile != "auto" and (Cout % tile[0] or Cin % tile[1]):
                continue
            C.conv_gemm_wgrad_force_tile(*(tile if tile != "auto" else (0, 0)))
            tiles = C.conv_gemm_wgrad_tiles(x, dy, K, K, st, pd)
            for target in TARGETS:
                if target == "auto":
                    ppc = C.conv_gemm_wgrad_ppc(x, dy, K, K, st, pd)
                else:
                    chunks = max(1, target // tiles)
                    ppc = -(-P // chunks)          # ceil(P / chunks)
                    ppc = max(32, -(-ppc // 32) * 32)  # rounded up to 32
                ch = C.conv_gemm_wgrad_chunks(x, dy, K, K, st, pd, ppc)
                g = torch.zeros(row, device=dev)
                slab = torch.empty(ch, row, device=dev) if ch > 1 else None

                def fn():
                    if ch == 1:
                        C.conv_gemm_wgrad(dy, x, g, K, K, st, pd, ppc, False, 0)
                    else:
                        C.conv_gemm_wgrad(dy, x, slab, K, K, st, pd, ppc, False, 0)
                        C.grad_reduce([(slab, row, 0, row, ch, g, 1.0, False)])

                us = timeit(fn, a.iters)
                fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = g.clone()
                err = float((g - ref).abs().max() / (ref.abs().max() + 1e-30))
                tname = "auto" if tile == "auto" else f"{tile[0]}x{tile[1]}"
                res[f"{tname}/{target}"] = [round(us, 2), ch, tiles * ch, round(err, 7)]
        C.conv_gemm_wgrad_force_tile(0, 0)
        best = min(res.items(), key=lambda kv: kv[1][0])
        print(json.dumps({"layer": name, "auto_us": res["auto/auto"][0], "best": best[0], "best_us": best[1][0],
                          "best_tflops": round(flops / best[1][0] / 1e6, 1),
                          "all_us_chunks_blocks_err": res}), flush=True)


if __name__ == "__main__":
    main()
