#!/bin/bash
# In-call A/B: driver-shaped run with the graph launched first (head 0) vs 2 eager head steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3head}
mkdir -p $out
for r in 1 2 3 4; do
  for h in 0 2 4; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no_fp32 --no_scaling_ref --graph_head $h > $out/h${h}_$r.json 2>> $out/err.log || exit $?
    echo "head=$h run $r: $(grep -o '"value": [0-9.]*' $out/h${h}_$r.json)"
  done
done
