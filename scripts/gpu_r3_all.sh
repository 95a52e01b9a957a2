#!/bin/bash
# Every GPU test (one process, per-test timeout), then smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3all}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rfE > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/pytest_gpu.log; tail -3 $out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?; tail -1 $out/smoke.log; exit $rc
