#!/bin/bash
# In-call A/B of the host wait policy (hipDeviceScheduleSpin) on the driver-shaped run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3spin}
mkdir -p $out
for r in 1 2 3 4; do
  for m in 0 1; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no_fp32 --no_scaling_ref --sync_spin $m > $out/s${m}_$r.json 2>> $out/err.log || exit $?
    echo "spin=$m run $r: $(grep -o '"value": [0-9.]*' $out/s${m}_$r.json)"
  done
done
for m in 0 1; do
  timeout -k 10 200 python bench.py --no_fp32 --no_scaling_ref --sync_spin $m > $out/l${m}.json 2>> $out/err.log || exit $?
  echo "spin=$m 1000 steps: $(grep -o '"value": [0-9.]*' $out/l${m}.json)"
done
