#!/bin/bash
# ResNet-18: kernel tests, A/B of the stem BN+ReLU deferred into the maxpool (env), default-path
# rocprofv3 kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3rn4}
mkdir -p $out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $out/pytest.log | head -20; exit $rc; }
for r in 1 2 3; do
  for m in 1 0; do
    DDP_AMD_DEFER_BN=$m timeout -k 10 200 python bench.py --model resnet18 --steps 50 --warmup 10 --no_scaling_ref > $out/b_m${m}_$r.json 2>> $out/bench.err || exit $?
    echo "defer_bn=$m run $r: $(grep -o '"value": [0-9.]*' $out/b_m${m}_$r.json)"
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$out/prof" -o rn -- python "$R/bench.py" --model resnet18 --steps 10 --warmup 5 --no_scaling_ref > "$R/$out/prof.log" 2>&1)
rc=$?; echo "prof rc=$rc"; exit $rc
