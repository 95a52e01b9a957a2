#!/bin/bash
# A/B of the forced multi-GPU chain (dist_mode 4) across builds in one gpurun call:
#   bash scripts/ab_regress.sh <out> <rounds> <tag=so-path|tree:dir|cur>...
# "cur" = this tree; "so-path" = a variant _C.so (DDP_AMD_NATIVE_SO); "tree:dir" = another
# exported tree with its own build (its bench.py).  Prints value / step_us per run.
set -o pipefail
out=gpurun_out/$1; n=$2; shift 2
mkdir -p "$out"
A="--no_fp32 --force_allreduce --dist_mode 4 --no_placement"
for r in $(seq 1 "$n"); do
  for v in "$@"; do
    tag=${v%%=*}; what=${v#*=}
    f=$out/${tag}_$r.json
    if [[ $what == cur ]]; then
      timeout -k 10 200 python bench.py $A > "$f" 2>> "$out/err.log" || exit $?
    elif [[ $what == tree:* ]]; then
      (cd "${what#tree:}" && timeout -k 10 200 python bench.py $A) > "$f" 2>> "$out/err.log" || exit $?
    else
      DDP_AMD_NATIVE_SO=$what timeout -k 10 200 python bench.py $A > "$f" 2>> "$out/err.log" || exit $?
    fi
    echo "$tag $r: $(grep -o '"value": [0-9.]*' "$f") $(grep -o '"step_us": [0-9.]*' "$f")"
  done
done
