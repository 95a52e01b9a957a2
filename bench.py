"""Headline benchmark: images/sec of MNIST SimpleCNN DDP training on N MI355X GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch_size 32]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N`` (N > 1) without a launcher environment SELF-LAUNCHES: the parent never
touches the GPU (no torch.cuda call, no native import); it starts
``torch.distributed.run`` with N fresh worker processes (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT) as a child process - the
reference's launcher derives N processes from world_size the same way
(``/root/reference/train_ddp.py:221-224``) - and, unless ``--no_scaling_ref``, first a
1-rank child run of the same config, so its ONE JSON line carries
``scaling_efficiency`` = value(N) / (N * value(1)).  Workers assert
``dist.get_world_size() == N`` and the native RCCL communicator's nranks == N and report
both (``ranks_seen``, ``rccl_nranks``), plus the data plane (``bucket_allreduce``) and
each bucket's isolated all-reduce time (``bucket_allreduce_us``).

Metric/config are BASELINE.json's: images/sec of the reference's SimpleCNN
(520,586 params) DDP training step at the reference's default per-rank batch
(32), weak scaling (per-GPU batch fixed), synthetic MNIST-shaped uint8 data and
random-init weights (no network for the real dataset), bf16 compute with fp32
master weights / gradients / optimizer.  A timed step is the complete training
step of the reference's loop: batch gather + forward + loss + backward + DDP
bucket all-reduce (N>1) + SGD update - executed by the native fused engine (2 HIP
kernels per step on one GPU; at N>1 3 kernels + one all-reduce per gradient bucket - the
direct xGMI kernel, RCCL as the fallback - replayed from a hipGraph).  After the bf16
headline the same process times the exact-fp32 engine (the reference's precision) the same
way and reports it as ``config.fp32_images_per_sec`` (``--no_fp32`` skips it).

W untimed warmup steps, then EXACTLY K timed steps bracketed by barrier +
``torch.cuda.synchronize()`` on both sides; the step time is the MAX over ranks;
rank 0 prints one JSON line.  ``vs_baseline`` divides by the reference's
best measured aggregate throughput at the same world size and per-rank batch 32
(BASELINE.md survey table: ws1 2,799, ws2 2,665, ws4 3,384 img/s on the 8-core
host - the reference publishes no numbers; ws8 at B=32 was not measured there,
so its best measured aggregate at any batch, 3,670 img/s, is used).
"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec MNIST SimpleCNN DDP at 1/2/4/8 MI355X; DDP scaling efficiency"
BASELINE_IMG_S = {1: 2799.0, 2: 2665.0, 4: 3384.0, 8: 3670.0}


def kernels_per_step(eng):
    """Kernels per step of the chain a FusedSimpleCNNEngine ran (level 3 only): 2 on one GPU
    and with the in-launch all-reduce, 3 with both buckets' all-reduces in one launch
    (dist_mode 3); otherwise fc_bwd and one all-reduce kernel per bucket come on top, and the
    separate grad_reduce kernel when the conv backward did not fuse the slab reduction (the
    exact-fp32 default)."""
    if not eng.eng.last_level3:
        return None
    nar = 0 if eng.eng.last_xar or eng.comm_kind == "none" else 1 if eng.eng.last_pair else len(eng.ranges)
    k = (2 if eng.eng.last_fc_role else 3) + nar + (0 if getattr(eng.eng, "last_fused_reduce", True) else 1)
    gs, heads = eng.eng.graph_steps, eng.eng.graph_heads
    if heads and gs:  # dist_mode 4 graph: every step head saves a launch (per-step average)
        k = round(k - heads / gs, 3)
    return k


def graph_chunk(k: int, cap: int = 100) -> int:
    for d in range(min(cap, k), 0, -1):
        if k % d == 0:
            return d
    return 1


LAUNCH_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child_json(cmd, env, timeout):
    """Run one launcher child; return (its last JSON stdout line or None, reason).

    The child (torch.distributed.run) leads its own process group: on a timeout it first
    gets SIGTERM so the elastic agent can stop its workers, then, after a grace period, the
    whole group is SIGKILLed - hung workers (spinning in an xGMI or in-launch wait) must not
    survive into the next fallback attempt on the same GPUs.  Returns only once
    every process of the group has exited."""
    import signal

    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=None, text=True,
                         start_new_session=True)
    try:
        out, _ = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        _kill_group(p, signal)
        out, _ = p.communicate()
        sys.stdout.write(out or "")
        return None, f"timed out after {timeout:.0f} s"
    _reap_group(p.pid, signal)  # workers the agent left behind (it exited abnormally)
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        sys.stdout.write(out)
        return None, f"rc={p.returncode}"
    return json.loads(lines[-1]), None


def _kill_group(p, signal, grace: float = 20.0):
    """SIGTERM the child's process group, wait up to ``grace`` s, then SIGKILL the group."""
    try:
        os.killpg(p.pid, signal.SIGTERM)
    except ProcessLookupError:
        return
    try:
        p.wait(timeout=grace)
    except subprocess.TimeoutExpired:
        pass
    _reap_group(p.pid, signal)


def _reap_group(pgid: int, signal, wait_s: float = 30.0):
    """SIGKILL whatever is left in process group ``pgid`` and wait until it is empty."""
    try:
        os.killpg(pgid, signal.SIGKILL)
    except (ProcessLookupError, PermissionError):
        return
    t0 = time.time()
    while time.time() - t0 < wait_s:
        try:
            os.killpg(pgid, 0)
        except ProcessLookupError:
            return
        time.sleep(0.1)


# What the parent retries with when an N-rank child fails or times out (VERDICT r3 #3b):
# the production chain first, then the conservative kernel chain (level 1, separate slab
# reduction), then the same over RCCL instead of the direct xGMI kernels.  Each attempt is
# a fresh child (fresh processes, fresh GPU contexts); the parent never touches the GPU.
FALLBACKS = (
    ("production", ()),
    ("conservative chain", ("--fuse_level", "1", "--fuse_reduce", "0")),
    ("conservative chain over RCCL", ("--fuse_level", "1", "--fuse_reduce", "0", "--comm", "rccl")),
)


def run_with_fallback(launch, timeout):
    """``launch(extra_args, timeout)`` -> (record | None, reason) for each FALLBACKS entry in
    turn until one succeeds; the record carries ``config.fallback`` (None when the first
    attempt succeeded) and ``config.failed_attempts``."""
    failed = []
    for name, extra in FALLBACKS:
        rec, why = launch(extra, timeout)
        if rec is not None:
            cfg = rec.setdefault("config", {})
            cfg["fallback"] = None if not failed else name
            cfg["failed_attempts"] = failed
            return rec
        print(f"[bench] {name} attempt failed ({why}); retrying in a fresh child", file=sys.stderr, flush=True)
        failed.append({"attempt": name, "reason": why})
    raise SystemExit(f"[bench] every attempt failed: {failed}")


def self_launch(args, argv):
    """``--gpus N`` without a launcher env: N fresh worker processes via torch.distributed.run
    (a child process - this parent never initialises the GPU and never execs)."""
    n = args.gpus
    here = os.path.abspath(__file__)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL / xGMI peer mappings)

    def run(nproc):
        def launch(extra, timeout):
            port = _free_port()
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", f"--master-port={port}",
                   here, *_with_gpus(argv, nproc), *extra]
            return _child_json(cmd, env, timeout)
        return run_with_fallback(launch, args.launch_timeout)

    if args.dry_launch:
        rec = run(n)
        print(json.dumps(rec), flush=True)
        return
    ref = None
    if not args.no_scaling_ref:
        ref = run(1)
    rec = run(n)
    rec.setdefault("config", {})["launcher"] = "self (torch.distributed.run child)"
    if ref is not None and ref.get("value"):
        rec["config"]["n1_value"] = ref["value"]
        rec["config"]["scaling_efficiency"] = round(rec["value"] / (n * ref["value"]), 4)
    print(json.dumps(rec), flush=True)


def _with_gpus(argv, n):
    """argv with --gpus forced to n (both "--gpus N" and "--gpus=N" spellings)."""
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a == "--gpus":
            skip = True
            continue
        if a.startswith("--gpus="):
            continue
        out.append(a)
    return ["--gpus", str(n), *out]


def dry_worker(args):
    """--dry_launch inside a worker: report what the launcher gave this rank, gathered on
    rank 0 over a gloo group (no GPU)."""
    rank, ws = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    # test hook of the parent's fallback: fail unless this child runs fallback #dry_fail
    level = 2 if args.comm == "rccl" else (1 if args.fuse_level == 1 else 0)
    if level < args.dry_fail:
        raise SystemExit(3)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    mine = {k: os.environ.get(k) for k in LAUNCH_ENV}
    allenv = [None] * ws
    dist.all_gather_object(allenv, mine)
    if rank == 0:
        print(json.dumps({"dry_launch": True, "n_gpus": args.gpus, "ranks_seen": dist.get_world_size(),
                          "children": allenv, "fuse_level": args.fuse_level, "comm": args.comm}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--batch_size", type=int, default=32, help="per-rank batch (reference default 32)")
    ap.add_argument("--graph_steps", type=int, default=None)
    ap.add_argument("--no_graph", action="store_true")
    ap.add_argument("--fuse_level", type=int, default=None,
                    choices=[0, 1, 3],
                    help="engine fusion level (0: 8 kernels/step, 1: 3 kernels/step, 3: dZ2 in the forward, "
                         "fc weight gradient inside the conv backward - 2 kernels/step); default = engine default (3)")
    ap.add_argument("--l3_fc_role", type=int, default=None, choices=[0, 1],
                    help="fuse level 3, one GPU: fc weight gradient inside the conv backward launch on "
                         "blocks after every conv block (1) or as its own kernel between forward and conv "
                         "backward (0)")
    ap.add_argument("--graph_head", type=int, default=None,
                    help="timed steps launched eagerly before the graph replays (default 0)")
    ap.add_argument("--sync_spin", type=int, default=0, choices=[0, 1],
                    help="1: hipDeviceScheduleSpin (synchronize polls instead of sleeping)")
    ap.add_argument("--fuse_reduce", type=int, default=None, choices=[0, 1, 2],
                    help="slab reduction in the conv backward: 1 = reducers within half the resident "
                         "capacity (default), 2 = the whole capacity when single-process, 0 = separate kernel")
    ap.add_argument("--pxt_fwd", type=int, default=None, help="conv fwd pixel tiles per wave (1|2)")
    ap.add_argument("--pxt_dgrad", type=int, default=None, help="conv dgrad pixel tiles per wave (1|2)")
    ap.add_argument("--wgrad_rows", type=int, default=None, help="conv wgrad image rows per block")
    ap.add_argument("--wgrad_split", type=int, default=None, choices=[1, 2],
                    help="fused conv backward: wgrad blocks per slab row (input-channel halves)")
    ap.add_argument("--store_a1", type=int, default=None, choices=[0, 1, 2],
                    help="fused engine: conv1 output for the backward recomputed (0) / stored for dgrad (1) / for both (2)")
    ap.add_argument("--comm", choices=["auto", "tune", "xgmi", "xgmi1", "xgmi2", "rccl"], default="auto",
                    help="bucket all-reduce at N>1: auto = direct xGMI kernels (one-shot for the small "
                         "bucket), RCCL if their self-test fails; tune = fastest of xgmi2 / xgmi1 / RCCL "
                         "timed on the node")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="control-plane process group (nccl = RCCL); gloo + --comm xgmi rehearses "
                         "N ranks on ONE GPU (RCCL refuses duplicate GPUs)")
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--bucket_cap_mb", type=float, default=25.0,
                    help="DDP bucket cap (torch rule: first bucket 1 MiB, then this cap)")
    ap.add_argument("--first_bucket_mb", type=float, default=1.0)
    ap.add_argument("--bucket_plan", choices=["model", "torch"], default="model",
                    help="gradient buckets: model = the xGMI cost model's plan (parallel/bucket_model.py), "
                         "torch = torch DDP's size rule with --bucket_cap_mb / --first_bucket_mb")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16",
                    help="compute precision: bf16 MFMA operands (default) or exact fp32 MFMA (the "
                         "reference's precision)")
    ap.add_argument("--model", choices=["simplecnn", "resnet18"], default="simplecnn",
                    help="simplecnn = the headline metric; resnet18 = BASELINE config 5 (synthetic 3x224x224)")
    ap.add_argument("--image_size", type=int, default=224, help="resnet18 input size")
    ap.add_argument("--wgrad_halo", type=int, default=1, choices=[0, 1, 2],
                    help="resnet18: tap-fused halo weight gradient for every eligible stride-1 3x3 "
                         "layer (1, 2) or the per-tap GEMM kernel only (0)")
    ap.add_argument("--wgrad_halo_target", type=int, default=256, help="resnet18: halo wgrad blocks per launch")
    ap.add_argument("--wgrad_halo_cit", type=int, default=0, choices=[0, 16, 32],
                    help="resnet18: input channels per halo wgrad block (0 = planner default)")
    ap.add_argument("--no_fp32", action="store_true",
                    help="skip the exact-fp32 (reference precision) run after the bf16 headline")
    ap.add_argument("--no_comm_calibration", action="store_true",
                    help="N>1: skip the post-run sweep that refits the xGMI all-reduce cost model")
    ap.add_argument("--force_allreduce", action="store_true",
                    help="N=1: run the multi-GPU step chain anyway (fc weight gradient kernel, bucket "
                         "all-reduces on the --comm plane at world size 1) - times the dist chain on one GPU")
    ap.add_argument("--plan_world", type=int, default=None,
                    help="bucket plan as for this many ranks (default: the world size; --force_allreduce: 8)")
    ap.add_argument("--dist_mode", type=int, default=None, choices=[0, 1, 2, 3, 4],
                    help="N>1, level 3: 3 = both bucket all-reduces in one launch behind the conv backward "
                         "(xGMI, default); 2 = inside the conv backward launch; 1 = fc weight gradient + fc "
                         "bucket all-reduce on a graph branch forked after the forward; 0 = the round-4 serial order")
    ap.add_argument("--xar_blocks", type=int, default=None,
                    help="dist_mode 2: most blocks per bucket channel (in-launch all-reduce role)")
    ap.add_argument("--no_breakdown", action="store_true",
                    help="N>1 / --force_allreduce: skip the comm-free local run that splits the step into "
                         "local compute and exposed communication (config.step_breakdown)")
    ap.add_argument("--no_placement", action="store_true",
                    help="N>1 / --force_allreduce: do not time the placements (dist_mode 3 / 0 / 1) "
                         "before the run; use --dist_mode or the engine default")
    ap.add_argument("--no_chain_check", action="store_true",
                    help="N>1: skip the start-up check that the production kernel chain gives the "
                         "conservative chain's bits across the ranks")
    ap.add_argument("--dry_launch", action="store_true",
                    help="self-launch test hook: workers report their launcher env and exit (no GPU)")
    ap.add_argument("--dry_fail", type=int, default=0,
                    help="test hook (--dry_launch): workers exit 3 unless launched as fallback >= this")
    ap.add_argument("--no_scaling_ref", action="store_true",
                    help="self-launch: skip the 1-rank reference run (scaling_efficiency null)")
    ap.add_argument("--launch_timeout", type=float, default=900.0, help="self-launch: per-child seconds")
    argv = sys.argv[1:]
    args = ap.parse_args(argv)
    launched = all(k in os.environ for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"))
    if not launched and args.gpus > 1:
        return self_launch(args, argv)
    if args.dry_launch:
        if launched:
            return dry_worker(args)
        print(json.dumps({"dry_launch": True, "n_gpus": 1, "ranks_seen": 1, "children": []}))
        return
    if args.model == "resnet18":
        return bench_resnet(args)

    from ddp_amd import native
    from ddp_amd.data import DeviceMNIST, synthetic_mnist
    from ddp_amd.engine import EngineOptions, FusedSimpleCNNEngine
    from ddp_amd.models import SimpleCNN, param_count
    from ddp_amd.models.layers import flat_space
    from ddp_amd.ops import FusedSGD
    from ddp_amd.parallel import native_comm, setup

    native.require()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if ws != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks")
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":  # rehearsal: several ranks may share the visible GPUs
        lrank %= max(1, torch.cuda.device_count())
    if args.sync_spin:  # before torch creates the device context
        rc = native.require().hip_set_device_flags(lrank, 1)  # hipDeviceScheduleSpin
        if rc != 0:
            print(f"[bench] hipSetDeviceFlags(spin) returned {rc}; keeping the default wait policy",
                  file=sys.stderr)
    torch.cuda.set_device(lrank)
    dev = torch.device("cuda", lrank)
    comm = None
    ranks_seen, rccl_nranks = 1, None
    force = bool(args.force_allreduce) and ws == 1
    if ws > 1 or force:
        setup(rank, ws, backend=args.backend, verbose=False)
        ranks_seen = dist.get_world_size()
        assert ranks_seen == ws == args.gpus, (ranks_seen, ws, args.gpus)
        if args.backend == "nccl":
            comm = native_comm()
            rccl_nranks = comm.world
            assert rccl_nranks == ws, f"native RCCL communicator has {rccl_nranks} ranks, expected {ws}"
        elif args.comm == "rccl":
            raise SystemExit("--backend gloo has no RCCL data plane: use --comm xgmi")

    imgs, labels = synthetic_mnist()
    data = DeviceMNIST(imgs, labels, dev, "synthetic")

    # at N > 1 fit the xGMI cost model on this node's real bucket kernels
    # BEFORE the engine is built (untimed, a few ms) and plan the buckets with it; on real
    # peers the fit is also stored (xgmi/<N>, with provenance) for later runs
    calib = None
    if ws > 1 and args.comm != "rccl" and not args.no_comm_calibration:
        from ddp_amd.parallel.comm_calibration import calibrate, save, topology

        calib = calibrate(rank, ws, dev)
        if calib is not None:
            calib["topology"] = topology(ws, rank=rank)
            if calib["topology"] == "xgmi" and rank == 0:
                try:
                    save({k: v for k, v in calib.items() if k != "topology"}, ws, "xgmi",
                         extra={"source": "bench.py pre-engine calibration"})
                except OSError as e:
                    print(f"[bench] could not store the xGMI fit ({e})", file=sys.stderr)

    def barrier():
        if ws > 1:
            if args.backend == "nccl":
                dist.barrier(device_ids=[lrank])
            else:
                dist.barrier()
        torch.cuda.synchronize()

    placement = {"source": "not applicable (one rank, no forced all-reduce)"}

    def max_over_ranks(dt):
        if ws > 1:
            t = torch.tensor([dt], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    def pick_placement(dtype):
        """time every bitwise-equivalent placement (dist_mode) of the multi-GPU
        chain on THIS node - a throwaway engine each, a few graph replays, untimed for the
        metric - and agree on the fastest through the store (the slowest rank's time counts).
        An explicit --dist_mode skips it."""
        from ddp_amd.engine.fused_step import PLACEMENT_NAMES, agree_placement, placement_candidates

        if args.dist_mode is not None:
            return {"source": "fixed (--dist_mode)", "chosen": args.dist_mode}
        # (an xGMI plane whose self-test fails runs RCCL: mode 3 then times as mode 0)
        cands = placement_candidates("rccl" if args.comm == "rccl" else "xgmi", dtype)
        if len(cands) < 2:
            return {"source": "single candidate", "chosen": cands[0] if cands else None}
        mine = {}
        for mode in cands:
            eng, *_ = build(dtype, False, mode)
            try:
                eng.refresh()
                if not args.no_graph:
                    eng.run_steps(0)
                    eng._ensure_graph()
                n = max(20, 2 * (args.graph_steps or graph_chunk(max(1, args.steps))))
                eng.run_steps(min(n, 20))
                eng.synchronize()
                barrier()
                t0 = time.perf_counter()
                eng.run_steps(n)
                barrier()
                dt = time.perf_counter() - t0
                eng.synchronize()
                mine[mode] = round(dt * 1e6 / n, 3)
            except RuntimeError as e:  # a placement that fails here simply does not compete
                print(f"[bench] rank {rank}: placement dist_mode {mode} failed ({e})", file=sys.stderr)
                mine[mode] = None
            del eng
        store = dist.distributed_c10d._get_default_store() if dist.is_initialized() else None
        best, worst = agree_placement(store, f"ddp_amd/bench/placement/{dtype}", rank, ws, mine)
        return {"source": "timed on this node (untimed for the metric)", "chosen": best,
                "chosen_name": PLACEMENT_NAMES.get(best), "placement_us": {str(k): v for k, v in worst.items()},
                "this_rank_us": {str(k): v for k, v in mine.items()}}

    def build(dtype, local, mode=None):
        """A fresh seeded model (rank-0 init broadcast) and its engine for ``dtype``;
        ``mode``: the dist_mode to build with (None: args / placement / engine default)."""
        torch.manual_seed(0)
        model = SimpleCNN(compute_dtype=torch.float32 if dtype == "fp32" else torch.bfloat16).to(dev)
        fs = flat_space(model)
        if ws > 1 and not local:
            if args.backend == "nccl":
                dist.broadcast(fs.params, src=0)  # DDP construction semantics (rank-0 init)
            else:
                t = fs.params.detach().cpu()
                dist.broadcast(t, src=0)
                fs.params.data.copy_(t)
        opt = FusedSGD(model, lr=args.lr)
        # --graph_head: the first steps launch eagerly while the host submits the graph
        # (measured neutral on the driver-shaped run: profiles/r3_spin/README.md)
        head = args.graph_head or 0
        head = 0 if args.no_graph else min(head, args.steps)
        k = args.graph_steps or graph_chunk(max(1, args.steps - head))
        args.graph_head_used = head
        eo = EngineOptions(graph_steps=k, use_graph=not args.no_graph, dtype=dtype,
                           bucket_cap_mb=args.bucket_cap_mb, first_bucket_mb=args.first_bucket_mb,
                           bucket_plan=args.bucket_plan)
        eo.comm = args.comm
        for f in ("fuse_level", "pxt_fwd", "pxt_dgrad", "wgrad_rows", "store_a1", "wgrad_split", "l3_fc_role",
                  "fuse_reduce", "dist_mode", "xar_blocks"):
            if getattr(args, f) is not None and not (dtype == "fp32" and f == "store_a1"):
                setattr(eo, f, getattr(args, f))
        if dtype == "fp32":
            eo.store_a1 = 0  # the exact-fp32 chains recompute conv1 (engine.cpp launch_step_f32)
            eo.fuse_level = max(int(eo.fuse_level), 1)  # (no level-0 fp32 chain: --fuse_level 0 times level 1)
        eo.force_allreduce = force and not local
        if not local:
            eo.plan_world = args.plan_world or (8 if force else None)
            eo.cost_fit = calib
            if mode is not None:
                eo.dist_mode = mode
            elif placement.get("chosen") is not None:
                eo.dist_mode = placement["chosen"]
        if local:
            eng = FusedSimpleCNNEngine(model, opt, data, args.batch_size, 1, 0, None, eo)
        else:
            eng = FusedSimpleCNNEngine(model, opt, data, args.batch_size, ws, rank, comm, eo)
        return eng, fs, model, k, eo

    def timed_run(dtype, local=False):
        """Build the engine for ``dtype`` (fresh seeded model, rank-0 init broadcast), warm up,
        time exactly ``args.steps`` steps between barrier + synchronize brackets; returns
        (seconds = MAX over ranks, engine, flat space, model, graph chunk).  ``local``: the
        same config as a comm-free one-rank engine on every rank at once (the step-breakdown
        reference: what the step costs without any collective).  At N > 1 (or forced) the
        placement is timed first (pick_placement)."""
        nonlocal placement
        if (ws > 1 or force) and not local and not args.no_placement:
            placement = pick_placement(dtype)
        eng, fs, model, k, eo = build(dtype, local)
        eng.refresh()
        if (ws > 1 or force) and not local and not args.no_chain_check:
            eng.verify_chain()  # untimed: production vs conservative chain, bitwise, all ranks
        if not args.no_graph:
            eng.run_steps(0)           # uploads epoch 0's indices
            eng._ensure_graph()        # capture outside the timed region
        if args.warmup:
            eng.run_steps(args.warmup)
        eng.synchronize()
        barrier()
        t0 = time.perf_counter()
        eng.run_steps(args.steps, head=args.graph_head_used)
        barrier()  # torch.cuda.synchronize() waits for the engine's streams too
        dt = time.perf_counter() - t0
        eng.synchronize()  # (idle by now) raises if an in-launch / cross-GPU wait timed out
        return max_over_ranks(dt), eng, fs, model, k, eo

    dt, eng, fs, model, k, eo = timed_run(args.dtype)
    placement_main = dict(placement, dist_mode_run=eo.dist_mode)
    ms = dt * 1000.0 / args.steps
    img_s = ws * args.batch_size * args.steps / dt
    bucket_us = eng.measure_bucket_allreduce() if (ws > 1 or force) else None  # after the timed region
    # what the multi-GPU step costs over the one-GPU step.  Every rank times the
    # same config as a comm-free local engine (the ws=1 chain: 2 kernels, fc role fused) right
    # after the headline, untimed for the metric; the difference is the exposed communication
    # (+ the dist chain's extra kernels), the rest is local compute.
    breakdown = None
    if (ws > 1 or force) and not args.no_breakdown:
        dtl, engl, _, _, _, _ = timed_run(args.dtype, local=True)
        loc_us = dtl * 1e6 / args.steps
        step_us = dt * 1e6 / args.steps
        breakdown = {"step_us": round(step_us, 2), "local_step_us": round(loc_us, 2),
                     "exposed_comm_us": round(step_us - loc_us, 2),
                     "dist_over_local": round(step_us / loc_us, 4),
                     "local_kernels_per_step": kernels_per_step(engl),
                     "bucket_allreduce_isolated_us": bucket_us}
        del engl
    from ddp_amd.parallel.bucket_model import describe

    plan = describe(eng.buckets, fs, eng.cost, ranges=eng.ranges) if (ws > 1 or force) else None
    finite = bool(torch.isfinite(fs.params).all().item())
    level3 = bool(eng.eng.last_level3)
    kps = kernels_per_step(eng)
    same = True
    if ws > 1:  # DDP invariant: every rank holds bit-identical parameters after the run
        pd = dev if args.backend == "nccl" else "cpu"
        mine = fs.params.detach().to(pd)
        ref = mine.clone()
        dist.broadcast(ref, src=0)
        diff = torch.tensor([0 if torch.equal(ref, mine) else 1], device=pd)
        dist.all_reduce(diff)
        same = int(diff.item()) == 0
    # the reference's own precision (fp32 nn.Conv2d / nn.Linear, /root/reference/model.py:8-16):
    # the exact-fp32 engine timed the same way, after the headline
    fp32 = None
    if args.dtype == "bf16" and not args.no_fp32:
        dt32, eng32, _, _, _, _ = timed_run("fp32")
        fp32 = {"images_per_sec": round(ws * args.batch_size * args.steps / dt32, 1),
                "ms_per_step": round(dt32 * 1000.0 / args.steps, 5),
                "level3": bool(eng32.eng.last_level3),
                "kernels_per_step": kernels_per_step(eng32)}
        del eng32
    if rank == 0:
        base = BASELINE_IMG_S.get(ws)
        print(json.dumps({
            "metric": METRIC,
            "value": round(img_s, 1),
            "unit": "images/sec",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / base, 2) if base else None,
            "dtype": eng.dtype,
            "data": "synthetic (MNIST-shaped uint8 60000x28x28, random-init weights)",
            "config": {"model": f"SimpleCNN ({param_count(model):,} params)",
                       "global_batch": ws * args.batch_size, "per_rank_batch": args.batch_size,
                       "seq_len": None, "image": "1x28x28", "parallelism": f"dp{ws}",
                       "engine": "fused hipGraph" if not args.no_graph else "fused eager",
                       "graph_steps": k, "graph_head": getattr(args, "graph_head_used", 0), "fuse_level": eo.fuse_level, "level3": level3,
                       "kernels_per_step": kps,
                       "tiling": {"pxt_fwd": eng.opts.pxt_fwd, "pxt_dgrad": eo.pxt_dgrad,
                                  "wgrad_rows": eng.wgrad_rows, "store_a1": eng.store_a1,
                                  "wgrad_split": eo.wgrad_split},
                       "params_finite": finite,
                       "bucket_allreduce": eng.comm_kind, "bucket_allreduce_us": bucket_us,
                       "buckets_elems": [n for _, n in eng.ranges],
                       "params_identical_across_ranks": same, "ranks_seen": ranks_seen,
                       "rccl_nranks": rccl_nranks, "backend": args.backend if ws > 1 else None,
                       "scaling_efficiency": None, "tuned_planes_us": eng.allreduce_us,
                       "bucket_plan": {"rule": args.bucket_plan, "buckets": plan,
                                       "cost_source": eng.cost.source if (ws > 1 or force) else None,
                                       "plan_world": eo.plan_world,
                                       "pred_last_allreduce_done_us": (round(eng.pred_comm_us, 2)
                                                                       if ws > 1 and eng.pred_comm_us else None)},
                       "chain_check": eng.chain_check, "downgrades": getattr(eng, "downgrades", []),
                       "force_allreduce": force, "step_breakdown": breakdown,
                       "inlaunch_allreduce": bool(eng.eng.last_xar),
                       "pair_allreduce": bool(eng.eng.last_pair),
                       "placement": placement_main,
                       "comm_calibration": calib,
                       "fp32_images_per_sec": fp32["images_per_sec"] if fp32 else None,
                       "fp32_level3": fp32["level3"] if fp32 else None,
                       "fp32_kernels_per_step": fp32["kernels_per_step"] if fp32 else None,
                       "fp32_ms_per_step": fp32["ms_per_step"] if fp32 else None},
        }), flush=True)
    if ws > 1 or force:
        barrier()
        dist.destroy_process_group()


def bench_resnet(args):
    """ResNet-18 DDP training step (module path: HIP conv/BN/pool kernels, our DDP with the
    native C++ reducer + RCCL), synthetic ImageNet-shaped data resident on the device."""
    from ddp_amd import native
    from ddp_amd.models import param_count, resnet18
    from ddp_amd.ops import CrossEntropyLoss, FusedSGD
    from ddp_amd.ops.resnet_fn import to_nhwc4
    from ddp_amd.parallel import DistributedDataParallel, setup

    native.require().conv_gemm_wgrad_set_halo(args.wgrad_halo, args.wgrad_halo_target, args.wgrad_halo_cit)
    if args.dtype != "bf16":
        raise SystemExit("--model resnet18 runs the bf16 MFMA kernels only")
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if ws != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but the launcher started WORLD_SIZE={ws} ranks")
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":  # rehearsal: several ranks share the visible GPUs
        lrank %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(lrank)
    dev = torch.device("cuda", lrank)
    setup(rank, ws, backend=args.backend, verbose=False)
    torch.manual_seed(0)
    model = resnet18().to(dev)
    S0 = args.image_size
    # gloo rehearsal: no buffer broadcast (a c10d gloo call is not graph-capturable)
    from ddp_amd.engine.trainer import module_comm

    plan = None
    if args.bucket_plan == "model" and ws > 1:
        from ddp_amd.models.layers import flat_space
        from ddp_amd.parallel.bucket_model import module_plan

        # cost-model plan from the CPU twin's layer shapes (same module tree, per-rank batch)
        cpu_twin = resnet18()
        plan, _ = module_plan(flat_space(cpu_twin), cpu_twin, torch.randn(args.batch_size, 3, S0, S0), ws)
    ddp = DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb,
                                  broadcast_buffers=args.backend == "nccl", comm=module_comm(args.comm),
                                  buckets=plan)
    opt = FusedSGD(model, lr=args.lr, momentum=0.9)
    lossf = CrossEntropyLoss()
    B, S = args.batch_size, args.image_size
    g = torch.Generator(device=dev).manual_seed(rank)
    pool = 4  # distinct resident batches cycled through
    xs = [to_nhwc4(torch.randn(B, 3, S, S, device=dev, generator=g)) for _ in range(pool)]
    ys = [torch.randint(0, 1000, (B,), device=dev, generator=g) for _ in range(pool)]

    def train_step(x, y):
        opt.zero_grad()
        loss = lossf(ddp(x), y)
        loss.backward()
        opt.step()
        return loss

    # whole-step hipGraph (engine/graph_step.py) at any world size: the DDP buffer
    # broadcast (native RCCL on the current stream) and the bucket all-reduces (native
    # reducer's comm stream, forked / joined by events) are captured with the step
    use_graph = not args.no_graph
    if use_graph:
        # its capture warm-up steps are part of the untimed warm-up
        from ddp_amd.engine import GraphedStep

        nwarm = max(1, min(3, args.warmup))
        graphed = GraphedStep(train_step, (xs[0], ys[0]), warmup=nwarm)

        def step(i):
            return graphed(xs[i % pool], ys[i % pool])
    else:
        def step(i):
            return train_step(xs[i % pool], ys[i % pool])

    for i in range(args.warmup):
        step(i)

    def barrier():
        if ws > 1:
            if args.backend == "nccl":
                dist.barrier(device_ids=[lrank])
            else:
                dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    barrier()
    dt = time.perf_counter() - t0
    if ws > 1:
        t = torch.tensor([dt], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    img_s = ws * B * args.steps / dt
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec ResNet-18 DDP (BASELINE config 5)", "value": round(img_s, 1),
            "unit": "images/sec", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt * 1000 / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": f"synthetic (3x{S}x{S} gaussian images, random labels, random-init weights)",
            "config": {"model": f"ResNet-18 ({param_count(model):,} params)", "global_batch": ws * B,
                       "per_rank_batch": B, "seq_len": None, "parallelism": f"dp{ws}",
                       "engine": "module path (HIP autograd + native reducer)"
                                 + (", whole step in one hipGraph" if use_graph else ", eager"),
                       "wgrad_halo": args.wgrad_halo, "wgrad_halo_target": args.wgrad_halo_target,
                       "bucket_allreduce": ddp.comm_kind if ws > 1 else "none",
                       "buckets": len(ddp.buckets), "ranks_seen": dist.get_world_size(),
                       "loss": round(float(loss.item()), 4)},
        }), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
