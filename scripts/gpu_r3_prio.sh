#!/bin/bash
# A/B: fc-role waves at raised issue priority (DDP_AMD_FC_PRIO=1) vs default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3prio}
mkdir -p $out
for r in 1 2 3; do
  for m in 1 0; do
    DDP_AMD_FC_PRIO=$m timeout -k 10 120 python bench.py --no_fp32 --no_scaling_ref > $out/p${m}_$r.json 2>> $out/err.log || exit $?
    echo "fc_prio=$m run $r: $(grep -o '"value": [0-9.]*' $out/p${m}_$r.json)"
  done
done
