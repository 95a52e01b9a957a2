#!/bin/bash
# A/B: reducer waves at raised issue priority (DDP_AMD_RED_PRIO 0 / 2 / 3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3rprio}
mkdir -p $out
for r in 1 2 3; do
  for m in 0 2 3; do
    DDP_AMD_RED_PRIO=$m timeout -k 10 120 python bench.py --no_fp32 --no_scaling_ref > $out/r${m}_$r.json 2>> $out/err.log || exit $?
    echo "red_prio=$m run $r: $(grep -o '"value": [0-9.]*' $out/r${m}_$r.json)"
  done
done
