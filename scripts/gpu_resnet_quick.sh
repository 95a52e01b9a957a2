#!/bin/bash
# ResNet quick iteration: kernel tests + graphed bench + eager kernel trace (10 steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_resnet.log 2>&1 && \
timeout -k 10 300 python bench.py --model resnet18 --steps 50 --warmup 10 > gpurun_out/resnet_graph.json 2> gpurun_out/resnet.err && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/prof_resnet" -o rn -- python "$R/bench.py" --model resnet18 --steps 10 --warmup 5 --no_graph > "$R/gpurun_out/prof_resnet.log" 2>&1)
rc=$?; echo "chain rc=$rc"; tail -1 gpurun_out/pytest_resnet.log; grep -h '^{' gpurun_out/resnet_graph.json; exit $rc
