#!/bin/bash
# Fast iteration loop: engine + kernel GPU tests, stamp timeline, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -rfE > gpurun_out/quick_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/quick_pytest.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -u scripts/stamps.py > gpurun_out/stamps.log 2>&1 && cat gpurun_out/stamps.log | grep -v amdgpu.ids && \
timeout -k 10 200 python bench.py > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err && cat gpurun_out/bench_quick.json
timeout -k 10 120 python -u scripts/stamps.py --graph > gpurun_out/stamps_graph.log 2>&1 && cat gpurun_out/stamps_graph.log | grep -v amdgpu.ids
