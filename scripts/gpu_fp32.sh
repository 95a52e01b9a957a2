# fp32 engine: fused-reduction bitwise tests + fp32 GPU tests + bench (fused reduce on / A-B)
set -o pipefail
out=gpurun_out/${1:-fp32}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_fp32_gpu.py -x -v --timeout 120 --timeout-method thread -k "fused_reduce or fp32 or engine" > $out/pytest_fp32.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --dtype fp32 > $out/b_fp32_$r.json 2>> $out/err.log || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python -u bench.py --dtype fp32 --steps 200 --warmup 20 > $out/prof.log 2>&1
echo exit=$?
