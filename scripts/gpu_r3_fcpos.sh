#!/bin/bash
# level-3 fc role placement: bitwise test of l3_fc_role 3 vs 1, then alternating benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3fcpos}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "level3 or fc_role" -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -gt 1 ] && exit $rc
for r in 1 2 3; do
  for m in 1 3; do
    timeout -k 10 120 python bench.py --no_fp32 --no_scaling_ref --l3_fc_role $m > $out/f${m}_$r.json 2>> $out/err.log || exit $?
    echo "l3_fc_role=$m run $r: $(grep -o '"value": [0-9.]*' $out/f${m}_$r.json)"
  done
done
timeout -k 10 120 python -u scripts/stamps.py --graph > $out/stamps_default.log 2>&1; tail -6 $out/stamps_default.log | cut -c1-200
