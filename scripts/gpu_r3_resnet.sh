#!/bin/bash
# Round 3 ResNet-18: kernel tests, A/B benches of the BatchNorm fusions (tail finalise in
# the conv launch, one-launch BN backward), rocprofv3 kernel trace of the graphed step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3rn}
mkdir -p $out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $out/pytest.log | head -20; exit $rc; }
for v in "1 1" "0 0" "1 0" "0 1" "1 1" "0 0"; do
  set -- $v
  DDP_AMD_BN_TAIL=$1 DDP_AMD_BN_BWD_FUSED=$2 timeout -k 10 200 python bench.py --model resnet18 --steps 50 --warmup 10 --no_scaling_ref > $out/b_t$1_f$2.json 2>> $out/bench.err || exit $?
  echo "tail=$1 fused=$2: $(grep -o '"value": [0-9.]*' $out/b_t$1_f$2.json)"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$out/prof" -o rn -- python "$R/bench.py" --model resnet18 --steps 10 --warmup 5 --no_scaling_ref > "$R/$out/prof.log" 2>&1)
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
(cd /tmp && DDP_AMD_BN_TAIL=0 DDP_AMD_BN_BWD_FUSED=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$out/prof0" -o rn -- python "$R/bench.py" --model resnet18 --steps 10 --warmup 5 --no_scaling_ref > "$R/$out/prof0.log" 2>&1)
rc=$?; echo "prof0 rc=$rc"; exit $rc
