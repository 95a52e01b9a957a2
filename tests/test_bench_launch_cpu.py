"""bench.py's self-launch path: ``python bench.py --gpus N`` without a
launcher environment must start N fresh worker processes itself - through a
``torch.distributed.run`` CHILD process, never an exec from a process that touched the GPU -
and every worker must see a consistent RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set.
Reference: the launcher derives N processes from world_size (/root/reference/train_ddp.py:221-224).
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK",
                                                              "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], cwd=REPO, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout  # ONE JSON line for the whole run
    return json.loads(lines[0])


@pytest.mark.slow
@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_spawns_n_ranks(n):
    rec = _run(["--gpus", str(n), "--backend", "gloo", "--comm", "xgmi", "--dry_launch"])
    assert rec["dry_launch"] and rec["ranks_seen"] == n
    kids = rec["children"]
    assert len(kids) == n
    assert sorted(int(k["RANK"]) for k in kids) == list(range(n))
    assert sorted(int(k["LOCAL_RANK"]) for k in kids) == list(range(n))
    assert all(int(k["WORLD_SIZE"]) == n for k in kids)
    assert all(k["MASTER_ADDR"] == "127.0.0.1" for k in kids)
    assert len({k["MASTER_PORT"] for k in kids}) == 1


def test_with_gpus_rewrites_argv():
    sys.path.insert(0, REPO)
    import bench

    assert bench._with_gpus(["--gpus", "8", "--steps", "5"], 1) == ["--gpus", "1", "--steps", "5"]
    assert bench._with_gpus(["--gpus=4", "--warmup", "2"], 4) == ["--gpus", "4", "--warmup", "2"]
    assert bench._with_gpus(["--steps", "5"], 2) == ["--gpus", "2", "--steps", "5"]


def test_fallback_order_unit():
    """VERDICT r3 #3b: a failing N-rank child is retried in a fresh child with the
    conservative chain, then over RCCL; the record says which attempt produced it."""
    sys.path.insert(0, REPO)
    import bench

    seen = []

    def launch(extra, timeout):
        seen.append(tuple(extra))
        if "--comm" not in extra:
            return None, "rc=1"
        return {"value": 1.0, "config": {}}, None

    rec = bench.run_with_fallback(launch, 5.0)
    assert [("production"), ("conservative chain")] == [a["attempt"] for a in rec["config"]["failed_attempts"]]
    assert rec["config"]["fallback"] == "conservative chain over RCCL"
    assert seen[0] == () and seen[1] == ("--fuse_level", "1", "--fuse_reduce", "0")
    ok = bench.run_with_fallback(lambda e, t: ({"value": 2.0}, None), 5.0)
    assert ok["config"]["fallback"] is None and ok["config"]["failed_attempts"] == []
    with pytest.raises(SystemExit):
        bench.run_with_fallback(lambda e, t: (None, "timed out"), 5.0)


@pytest.mark.slow
def test_self_launch_falls_back_on_failing_child():
    """The real launcher path: the workers exit non-zero until the parent retries with the
    conservative chain (``--dry_fail 1``)."""
    rec = _run(["--gpus", "2", "--backend", "gloo", "--comm", "xgmi", "--dry_launch", "--dry_fail", "1"])
    assert rec["ranks_seen"] == 2
    assert rec["config"]["fallback"] == "conservative chain", rec
    assert rec["fuse_level"] == 1 and rec["comm"] == "xgmi"
    assert rec["config"]["failed_attempts"][0]["attempt"] == "production"


def test_child_timeout_kills_the_whole_group(tmp_path):
    """a launcher child that times out is torn down WITH its workers (its process
    group: SIGTERM, grace, SIGKILL) before the next fallback attempt starts - a hung worker
    must not keep the GPUs busy.  The child here spawns a grandchild that ignores SIGTERM and
    would outlive a plain subprocess.run timeout; both must be gone when _child_json returns."""
    import importlib.util
    import time

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    pidfile = tmp_path / "grandchild.pid"
    script = (
        "import os, signal, subprocess, sys, time\n"
        "g = subprocess.Popen([sys.executable, '-c', 'import signal, time; "
        "signal.signal(signal.SIGTERM, signal.SIG_IGN); time.sleep(600)'])\n"
        f"open({str(pidfile)!r}, 'w').write(str(g.pid))\n"
        "time.sleep(600)\n")
    t0 = time.time()
    rec, why = bench._child_json([sys.executable, "-c", script], dict(os.environ), timeout=3)
    assert rec is None and "timed out" in why
    assert time.time() - t0 < 60
    gpid = int(pidfile.read_text())
    for _ in range(50):
        try:
            os.kill(gpid, 0)
        except ProcessLookupError:
            break
        time.sleep(0.1)
    else:
        raise AssertionError("the grandchild survived the timeout")


def test_kernels_per_step_record():
    """config.kernels_per_step / fp32_kernels_per_step of the chain that ran: 2 on one GPU,
    2 with the in-launch all-reduce, 3 with both buckets in one launch (dist_mode 3), fc_bwd +
    one kernel per bucket otherwise; None off level 3."""
    import types

    sys.path.insert(0, REPO)
    import bench

    def eng(l3=True, fc_role=True, xar=False, pair=False, comm="xgmi1", nb=2, steps=0, heads=0, fred=True):
        e = types.SimpleNamespace(last_level3=l3, last_fc_role=fc_role, last_xar=xar, last_pair=pair,
                                  graph_steps=steps, graph_heads=heads, last_fused_reduce=fred)
        return types.SimpleNamespace(eng=e, comm_kind=comm, ranges=[(0, 1)] * nb)

    assert bench.kernels_per_step(eng(comm="none")) == 2
    assert bench.kernels_per_step(eng(xar=True)) == 2
    assert bench.kernels_per_step(eng(pair=True)) == 3
    assert bench.kernels_per_step(eng(fc_role=False, nb=2)) == 5
    assert bench.kernels_per_step(eng(l3=False)) is None
    # the exact-fp32 default: the slab reduction in its own grad_reduce kernel
    assert bench.kernels_per_step(eng(comm="none", fred=False)) == 3
    # dist_mode 4: a graph of 5 steps with 4 step heads (the first step's forward stands alone)
    assert bench.kernels_per_step(eng(pair=True, steps=5, heads=4)) == 2.2
    assert bench.kernels_per_step(eng(pair=True, steps=100, heads=99)) == 2.01
