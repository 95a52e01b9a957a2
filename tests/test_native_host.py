"""Host-only native code under AddressSanitizer / UBSan.

The reducer's bucket bookkeeping (csrc/runtime/bucket_state.h) has no device
code, so it is compiled for the host with -fsanitize=address,undefined and run
here (GPU sanitizers are not available on the MI355X pool).  The bound planner
is also cross-checked against the Python bucket plan used by DDP.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_bucket_state_asan_ubsan(tmp_path):
    exe = tmp_path / "test_bucket_state"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-I", os.path.join(ROOT, "csrc"),
           os.path.join(ROOT, "tests", "native", "test_bucket_state.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    if "does not come first" in r.stderr:
        pytest.skip("another preloaded runtime precedes ASan in this environment")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_native_planner_matches_python_bucket_plan():
    import torch  # noqa: F401

    from ddp_amd import native
    from ddp_amd.models import SimpleCNN, resnet18
    from ddp_amd.models.layers import flat_space
    from ddp_amd.parallel.ddp import bucket_plan

    native.build_if_needed()
    C = native.require()
    for model, caps in ((SimpleCNN(), [(1.0, 25.0), (0.01, 0.05)]), (resnet18(), [(1.0, 25.0), (1.0, 5.0)])):
        fs = flat_space(model)
        nbytes = [fs.numels[n] * 4 for n in fs.names]
        for first, cap in caps:
            want = bucket_plan(fs, cap, first)
            got = C.plan_buckets(nbytes, int(first * 1024 * 1024), int(cap * 1024 * 1024))
            assert [[fs.names[i] for i in b] for b in got] == want
