# fp32 path check: fp32 kernel/engine tests, the full GPU suite, bf16 + fp32 benches,
# rocprof kernel stats of the fp32 bench.
set -o pipefail
out=gpurun_out/${1:-r2b}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_fp32_gpu.py -x -v --timeout 120 --timeout-method thread > $out/pytest_fp32.log 2>&1
rc=$?; tail -3 $out/pytest_fp32.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
tail -3 $out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u bench.py > $out/bench_bf16.json 2> $out/bench.err && \
timeout -k 10 180 python -u bench.py --dtype fp32 > $out/bench_fp32.json 2>> $out/bench.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_fp32 -o run -- python -u bench.py --dtype fp32 --steps 200 --warmup 20 > $out/prof.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_bf16 -o run -- python -u bench.py --steps 200 --warmup 20 >> $out/prof.log 2>&1
echo exit=$?
cat $out/bench_bf16.json $out/bench_fp32.json
