#!/bin/bash
# One GPU session: tests, smoke, 1-GPU bench, rocprofv3 kernel stats.  Each GPU step has
# its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rfE > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err && \
timeout -k 10 300 python bench.py --no_graph --steps 300 --warmup 30 > gpurun_out/bench1_nograph.json 2>> gpurun_out/bench1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 200 --warmup 20 > gpurun_out/prof.log 2>&1
echo "chain rc=$?"
