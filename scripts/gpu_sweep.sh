#!/bin/bash
# Engine tests + tiling/fusion sweep of the headline bench + per-kernel profiles of both fusion levels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -q -rfE -x > gpurun_out/sweep/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/sweep/pytest.log
if [ $rc -ne 0 ]; then echo "pytest failed rc=$rc"; exit $rc; fi
for fl in 0 1; do for pf in 1 2; do for pd in 1 2; do
  timeout -k 10 120 python bench.py --steps 500 --warmup 50 --fuse_level $fl --pxt_fwd $pf --pxt_dgrad $pd >> gpurun_out/sweep/bench.jsonl 2>> gpurun_out/sweep/bench.err || exit $?
done; done; done
for R in 2 4 7; do
  timeout -k 10 120 python bench.py --steps 500 --warmup 50 --fuse_level 0 --wgrad_rows $R >> gpurun_out/sweep/bench.jsonl 2>> gpurun_out/sweep/bench.err || exit $?
done
for fl in 0 1; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/sweep/prof_f$fl" -o bench -- python "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --fuse_level $fl > "$GRAFT_REPO_ROOT/gpurun_out/sweep/prof_f$fl.log" 2>&1) || exit $?
done
echo sweep done
