#!/bin/bash
# Level-3 tiling sweep (alternating configs in one call): pxt_fwd, pxt_dgrad, wgrad_rows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3sweep}
mkdir -p $out
cfgs=("--pxt_fwd 2" "--pxt_fwd 1" "--wgrad_rows 4" "--pxt_dgrad 1" "--wgrad_rows 14")
for r in 1 2; do
  for i in "${!cfgs[@]}"; do
    timeout -k 10 120 python bench.py --steps 1000 --warmup 100 --no_fp32 --no_scaling_ref ${cfgs[$i]} > $out/c${i}_$r.json 2>> $out/err.log
    rc=$?
    echo "${cfgs[$i]} run $r (rc $rc): $(grep -o '"value": [0-9.]*' $out/c${i}_$r.json) $(grep -o '"level3": [a-z]*' $out/c${i}_$r.json)"
    [ $rc -gt 1 ] && exit $rc
  done
done
exit 0
