#!/bin/bash
# exact-fp32 step: fused-reduction tests, then an in-call A/B of the reducer budget
# (fuse_reduce 1 = half capacity -> separate grad_reduce at B=32; 2 = whole capacity -> fused)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3fp32}
mkdir -p $out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -k "fused_reduce or channel_split or fp32" tests/test_fp32_gpu.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $out/pytest.log | head -20; exit $rc; }
for r in 1 2; do
  for m in 1 2; do
    timeout -k 10 200 python bench.py --dtype fp32 --fuse_reduce $m --no_scaling_ref > $out/f$m_$r.json 2>> $out/bench.err || exit $?
    echo "fuse_reduce=$m run $r: $(grep -o '"value": [0-9.]*' $out/f$m_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $out/f$m_$r.json)"
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof" -o fp32 -- python "$R/bench.py" --dtype fp32 --steps 200 --warmup 20 --no_scaling_ref > "$R/$out/prof.log" 2>&1) && \
timeout -k 10 120 python -u scripts/stamps.py --graph --dtype fp32 > $out/stamps_fp32.log 2>&1
rc=$?; echo "rc=$rc"; exit $rc
