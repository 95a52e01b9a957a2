"""Per-layer roofline of the ResNet-18 training step (BASELINE config 5).

Two phases:

    rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv -d OUT -- \
        python scripts/resnet_roofline.py run --out OUT/calls.json
    python scripts/resnet_roofline.py report OUT [--md profiles/r4_resnet/roofline.md]

``run`` trains a few EAGER module-path steps (B = 32, 224^2, our DDP at world 1) with every
native conv / BatchNorm / reduction call wrapped in a roctx range named after the call and
its layer shape ("conv3x3/s1 64->64 @56 | dgrad").  ``report`` maps every kernel of the
last step to its range (kernel correlation id -> the HIP launch call -> the innermost
marker range around it) and prints, per conv layer shape and pass (fwd / dgrad / wgrad -
each including its split-K / slab reduction kernels): launches, FLOP, the minimum HBM bytes
(inputs read once + output written once, bf16 activations / fp32 slabs), measured
microseconds, achieved TFLOP/s and TB/s, and the bound: the larger of FLOP / 2.5 PFLOP/s
(dense bf16 MFMA) and bytes / 8 TB/s, as a fraction of the measured time.  BatchNorm and the
rest are listed per kernel family.  Eager steps (one kernel per launch visible to the
tracer); the kernel durations are device time, as in the graph-replayed step.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_TFLOPS = 2500.0  # dense bf16 MFMA, MI355X
PEAK_TBPS = 8.0       # HBM3E

# native calls wrapped: name -> pass label
WRAP = {"conv_gemm_fwd": "fwd", "conv_gemm_dgrad": "dgrad", "conv_gemm_wgrad": "wgrad",
        "grad_reduce": "wgrad-reduce", "bn_finalize": "bn", "bn_apply": "bn", "bn_bwd": "bn-bwd",
        "maxpool_fwd": "pool", "maxpool_bwd": "pool", "avgpool_fwd": "pool", "avgpool_bwd": "pool",
        "sgemm": "head", "sgd": "sgd"}


def _roctx():
    """(push, pop) of the rocprofiler-sdk roctx API (what rocprofv3 --marker-trace records)."""
    import ctypes

    for lib in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"):
        for d in ("/opt/rocm/lib", ""):
            try:
                h = ctypes.CDLL(os.path.join(d, lib) if d else lib)
                h.roctxRangePushA.argtypes = [ctypes.c_char_p]
                return (lambda t: h.roctxRangePushA(t.encode())), (lambda: h.roctxRangePop())
            except OSError:
                continue
    import torch

    return torch.cuda.nvtx.range_push, torch.cuda.nvtx.range_pop


def run(a):
    import torch

    from ddp_amd import native
    from ddp_amd.models import resnet18
    from ddp_amd.ops import CrossEntropyLoss, FusedSGD
    from ddp_amd.ops.resnet_fn import to_nhwc4
    from ddp_amd.parallel import DistributedDataParallel, free_port, setup

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(free_port()))
    C = native.require()
    push, pop = _roctx()
    calls = []
    state = {"on": False, "layer": {}}

    def shape_of(args, name):
        # conv calls: (x, w, ..., KH, KW, stride, pad ...) or dgrad (dy, w, Xact, dx, KH, ...)
        try:
            if name == "conv_gemm_fwd":
                x, w, y, KH, KW, st = args[0], args[1], args[3 if name == "conv_gemm_fwd" else 2], args[4 if name == "conv_gemm_fwd" else 3], args[5 if name == "conv_gemm_fwd" else 4], args[6 if name == "conv_gemm_fwd" else 5]
                N, H, W_, Cin = x.shape
                return dict(N=N, H=H, W=W_, Cin=Cin, Cout=y.shape[3], OH=y.shape[1], OW=y.shape[2], KH=KH, KW=KW, s=st)
            if name == "conv_gemm_dgrad":
                dy, w, _, dx, KH, KW, st = args[:7]
                N, OH, OW, Cout = dy.shape
                return dict(N=N, H=dx.shape[1], W=dx.shape[2], Cin=dx.shape[3], Cout=Cout, OH=OH, OW=OW, KH=KH, KW=KW, s=st)
            if name == "conv_gemm_wgrad":
                dy, x, _, KH, KW, st = args[:6]
                N, OH, OW, Cout = dy.shape
                return dict(N=N, H=x.shape[1], W=x.shape[2], Cin=x.shape[3], Cout=Cout, OH=OH, OW=OW, KH=KH, KW=KW, s=st)
        except Exception:  # noqa: BLE001
            return None
        return None

    class Proxy:
        def __getattr__(self, name):
            fn = getattr(C, name)
            if name not in WRAP:
                return fn

            def wrapped(*args, **kw):
                if not state["on"]:
                    return fn(*args, **kw)
                sh = shape_of(args, name)
                if sh is not None:
                    stem = sh["Cin"] == 4
                    lab = (f"conv{sh['KH']}x{sh['KW']}/s{sh['s']} {3 if stem else sh['Cin']}->{sh['Cout']} "
                           f"@{sh['OH']}")
                    state["last_conv"] = (lab, sh)
                elif name == "grad_reduce" and "last_conv" in state:
                    lab, sh = state["last_conv"]
                else:
                    lab, sh = name, None
                tag = f"{lab} | {WRAP[name]}"
                calls.append({"tag": tag, "shape": sh, "call": name})
                push(tag)
                try:
                    return fn(*args, **kw)
                finally:
                    pop()
            return wrapped

    import ddp_amd.ops.resnet_fn as rf

    proxy = Proxy()
    rf._C = lambda: proxy  # every native call of the module path goes through the proxy
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    setup(0, 1, backend="nccl", verbose=False)
    torch.manual_seed(0)
    model = resnet18().to(dev)
    ddp = DistributedDataParallel(model)
    opt = FusedSGD(model, lr=0.01, momentum=0.9)
    lossf = CrossEntropyLoss()
    B, S = a.batch_size, a.image_size
    x = to_nhwc4(torch.randn(B, 3, S, S, device=dev))
    y = torch.randint(0, 1000, (B,), device=dev)
    for i in range(a.steps):
        state["on"] = i == a.steps - 1  # ranges on the last step only
        if state["on"]:
            torch.cuda.synchronize()
            push("STEP")
        opt.zero_grad()
        loss = lossf(ddp(x), y)
        loss.backward()
        opt.step()
        if state["on"]:
            pop()
    torch.cuda.synchronize()
    with open(a.out, "w") as f:
        json.dump(calls, f)
    print(f"loss {float(loss):.4f}, {len(calls)} wrapped calls in the traced step")


def _csv(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    rows = []
    for f in fs:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def flops_bytes(sh, pss):
    """(FLOP, minimum HBM bytes) of one conv pass."""
    P = sh["N"] * sh["OH"] * sh["OW"]
    cin = 3 if sh["Cin"] == 4 else sh["Cin"]  # the stem's input is padded to 4 channels
    K = sh["KH"] * sh["KW"] * cin
    fl = 2.0 * P * K * sh["Cout"]
    x = sh["N"] * sh["H"] * sh["W"] * sh["Cin"] * 2
    yb = P * sh["Cout"] * 2
    wb = sh["Cout"] * K * 2
    if pss == "fwd":
        by = x + wb + yb
    elif pss == "dgrad":
        by = yb + wb + x
    else:  # wgrad: dY + X in, fp32 gradient out
        by = yb + x + sh["Cout"] * K * 4
    return fl, by


def report(a):
    kern = _csv(a.trace, "*kernel_trace.csv")
    api = _csv(a.trace, "*hip_api_trace.csv")
    mark = _csv(a.trace, "*marker_api_trace.csv")
    calls = json.load(open(a.calls or os.path.join(a.trace, "calls.json")))
    shape = {c["tag"]: c["shape"] for c in calls if c["shape"]}
    launch_t = {}
    for r in api:
        launch_t[r["Correlation_Id"]] = int(r["Start_Timestamp"])
    ranges = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Message") or r.get("Function") or "")
              for r in mark]
    step = [r for r in ranges if r[2] == "STEP"]
    if not step:
        raise SystemExit("no STEP range in the marker trace")
    s0, s1 = step[-1][0], step[-1][1]
    inner = sorted([r for r in ranges if r[2] != "STEP" and s0 <= r[0] <= s1], key=lambda r: r[0])
    per = defaultdict(lambda: [0, 0.0, set()])  # tag -> [kernels, us, names]
    other = defaultdict(lambda: [0, 0.0])
    total = 0.0
    for k in kern:
        t = launch_t.get(k["Correlation_Id"])
        if t is None or not (s0 <= t <= s1):
            continue
        us = (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3
        total += us
        tag = None
        for r in inner:  # innermost range containing the launch
            if r[0] <= t <= r[1]:
                tag = r[2]
        name = k["Kernel_Name"].split("(")[0].replace("void ", "")
        if tag is None:
            other[name.split("<")[0]][0] += 1
            other[name.split("<")[0]][1] += us
        else:
            per[tag][0] += 1
            per[tag][1] += us
            per[tag][2].add(name.split("<")[0].replace("ddp_amd::", ""))
    # conv rows: merge the reduction kernels into their pass
    conv = defaultdict(lambda: [0, 0.0, 0.0, 0.0, set(), 0])  # (layer, pass) -> [kern, us, fl, by, names, calls]
    nonconv = defaultdict(lambda: [0, 0.0])
    for tag, (n, us, names) in per.items():
        lab, pss = tag.split(" | ")
        if lab.startswith("conv"):
            p = "wgrad" if pss == "wgrad-reduce" else pss
            c = conv[(lab, p)]
            c[0] += n
            c[1] += us
            c[4] |= names
        else:
            nonconv[pss][0] += n
            nonconv[pss][1] += us
    # FLOP / bytes per call (identical shapes share a row: count the calls)
    for cl in calls:
        if not cl["shape"]:
            continue
        lab, pss = cl["tag"].split(" | ")
        if pss not in ("fwd", "dgrad", "wgrad"):
            continue
        fl, by = flops_bytes(cl["shape"], pss)
        c = conv[(lab, pss)]
        c[2] += fl
        c[3] += by
        c[5] += 1
    lines = [f"# ResNet-18 per-layer roofline (B = {calls and next(c['shape']['N'] for c in calls if c['shape'])}, "
             "224^2, bf16, one eager step)", "",
             f"Step kernel time: {total:.1f} us (sum of kernel durations).  Bound = max(FLOP / {PEAK_TFLOPS:.0f} "
             f"TFLOP/s, bytes / {PEAK_TBPS:.0f} TB/s); 'of bound' = bound / measured.", "",
             "| layer (shape) | pass | calls | kernels | us | GFLOP | MB | TFLOP/s | TB/s | bound us | of bound | kernels |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    conv_us = 0.0
    for (lab, p), (n, us, fl, by, names, ncall) in sorted(conv.items(), key=lambda kv: (-kv[1][1])):
        bound = max(fl / (PEAK_TFLOPS * 1e6), by / (PEAK_TBPS * 1e6))
        conv_us += us
        lines.append(f"| {lab} | {p} | {ncall} | {n} | {us:.1f} | {fl / 1e9:.2f} | {by / 1e6:.2f} | "
                     f"{fl / us / 1e6 if us else 0:.0f} | {by / us / 1e6 if us else 0:.2f} | {bound:.1f} | "
                     f"{bound / us if us else 0:.0%} | {', '.join(sorted(names))[:80]} |")
    lines += ["", f"Conv passes: {conv_us:.1f} us ({100 * conv_us / total:.0f} % of the step).", "",
              "| other (by call) | kernels | us | % of step |", "|---|---|---|---|"]
    for k, (n, us) in sorted(nonconv.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| {k} | {n} | {us:.1f} | {100 * us / total:.1f} |")
    for k, (n, us) in sorted(other.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| (unwrapped) {k} | {n} | {us:.1f} | {100 * us / total:.1f} |")
    text = "\n".join(lines) + "\n"
    if a.md:
        os.makedirs(os.path.dirname(a.md), exist_ok=True)
        open(a.md, "w").write(text)
    print(text)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--out", required=True)
    r.add_argument("--steps", type=int, default=4)
    r.add_argument("--batch_size", type=int, default=32)
    r.add_argument("--image_size", type=int, default=224)
    p = sub.add_parser("report")
    p.add_argument("trace")
    p.add_argument("--calls", default=None)
    p.add_argument("--md", default=None)
    a = ap.parse_args()
    run(a) if a.cmd == "run" else report(a)


if __name__ == "__main__":
    main()
