# ResNet hot-path leaks: head on sgemm, residual join fused; tests + graphed bench + per-kernel profile
set -o pipefail
out=gpurun_out/${1:-r2e}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_resnet_gpu.py -x -v --timeout 240 --timeout-method thread > $out/pytest_resnet.log 2>&1
rc=$?; grep -E "passed|failed|Error" $out/pytest_resnet.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --model resnet18 --steps 100 --warmup 10 > $out/bench_resnet.json 2> $out/bench.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python -u bench.py --model resnet18 --steps 20 --warmup 5 > $out/prof.log 2>&1
rc=$?
cat $out/bench_resnet.json
python - <<PY
import csv
r=list(csv.DictReader(open('$out/prof/run_kernel_stats.csv')))
for x in r: 
    n=x['Name']
    if 'Cijk' in n or 'Functor_add' in n or 'sgemm' in n or 'elementwise' in n: print(n[:90], x['Calls'], round(float(x['AverageNs'])/1000,2))
PY
exit $rc
