#!/bin/bash
# SimpleCNN kernel / engine GPU tests, then scripts/gpu_r3_cnn.sh (bench, rocprof, stamps)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3cnn}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_fp32_gpu.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $out/pytest.log | head -20; exit $rc; }
bash scripts/gpu_r3_cnn.sh ${1:-r3cnn}
