#!/bin/bash
# engine tests + (store_a1, wgrad_rows) sweep of the headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep2
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sweep2/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/sweep2/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
for sa in 0 1 2; do for R in 4 5 7; do
  timeout -k 10 120 python bench.py --steps 500 --warmup 50 --store_a1 $sa --wgrad_rows $R >> gpurun_out/sweep2/bench.jsonl 2>> gpurun_out/sweep2/bench.err || exit $?
done; done
python - <<'PY'
import json
for l in open("gpurun_out/sweep2/bench.jsonl"):
    d = json.loads(l); c = d["config"]["tiling"]
    print(c["store_a1"], c["wgrad_rows"], d["ms_per_step"] * 1000, d["value"])
PY
