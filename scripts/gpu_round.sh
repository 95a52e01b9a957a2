#!/bin/bash
# Full GPU session: all GPU tests, smoke, 1-GPU headline bench (both fusion levels),
# rocprofv3 kernel statistics of the headline bench, stamp timeline.  Each GPU step has
# its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rfE > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest failed rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_f1.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python bench.py --fuse_level 0 > gpurun_out/bench_f0.json 2>> gpurun_out/bench.err && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- python "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/prof.log" 2>&1) && \
timeout -k 10 120 python -u scripts/stamps.py --graph > gpurun_out/stamps_graph.log 2>&1
rc=$?; echo "chain rc=$rc"; cat gpurun_out/bench_f*.json; exit $rc
