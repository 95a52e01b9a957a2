#!/bin/bash
# One GPU session: tests, smoke, 1-GPU bench, rocprofv3 kernel stats.  Each GPU step has
# its own time limit and the chain stops at the first failure (or a crashed test run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rfE > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then echo "pytest crashed/timed out (rc=$rc): stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --fuse_level 0 > gpurun_out/bench1_f0.json 2> gpurun_out/bench1.err && \
timeout -k 10 300 python bench.py --fuse_level 1 > gpurun_out/bench1_f1.json 2>> gpurun_out/bench1.err && \
timeout -k 10 300 python bench.py --no_graph --steps 300 --warmup 30 > gpurun_out/bench1_nograph.json 2>> gpurun_out/bench1.err && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o bench -- python "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --fuse_level 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1) && \
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 3 > gpurun_out/bench_resnet.json 2>> gpurun_out/bench1.err
echo "chain rc=$?"
