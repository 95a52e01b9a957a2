# quick perf check: engine tests, both benches, stamp timeline, kernel stats
set -o pipefail
out=gpurun_out/${1:-q}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 && \
timeout -k 10 180 python -u bench.py > $out/bench_bf16.json 2> $out/bench.err && \
timeout -k 10 180 python -u bench.py --dtype fp32 > $out/bench_fp32.json 2>> $out/bench.err && \
timeout -k 10 120 python -u scripts/stamps.py --graph > $out/stamps_graph.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_bf16 -o run -- python -u bench.py --steps 200 --warmup 20 > $out/prof.log 2>&1
rc=$?
tail -2 $out/pytest.log; cat $out/bench_bf16.json $out/bench_fp32.json | cut -c1-220; cat $out/stamps_graph.txt
python - <<PY
import csv
r=list(csv.DictReader(open('$out/prof_bf16/run_kernel_stats.csv')))
for x in r[:5]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1000,2))
PY
exit $rc
