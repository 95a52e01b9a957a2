#!/bin/bash
# Kernel-level GPU tests + per-kernel in-graph microbenchmarks + headline bench (both fusion levels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kb
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -q -rfE -x > gpurun_out/kb/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/kb/pytest.log
if [ $rc -ne 0 ]; then echo "pytest failed rc=$rc"; exit $rc; fi
timeout -k 10 300 python scripts/kbench.py --json gpurun_out/kb/kbench.json > gpurun_out/kb/kbench.log 2>&1 || exit $?
for fl in 0 1; do
  timeout -k 10 120 python bench.py --steps 500 --warmup 50 --fuse_level $fl --pxt_fwd 1 >> gpurun_out/kb/bench.jsonl 2>> gpurun_out/kb/bench.err || exit $?
done
echo kbench done
