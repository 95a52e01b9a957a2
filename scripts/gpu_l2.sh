# fuse level 2 check: engine tests (level 2 vs 1 bitwise, NaN-poisoned sweep), benches of
# both levels, stamps + kernel stats of level 2
set -o pipefail
out=gpurun_out/${1:-l2}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log; [ $rc -ne 0 ] && exit $rc
for lv in 1 2 1 2; do timeout -k 10 120 python -u bench.py --fuse_level $lv >> $out/bench.jsonl 2>> $out/bench.err || exit $?; done
timeout -k 10 120 python -u scripts/stamps.py --graph --fuse_level 2 > $out/stamps.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python -u bench.py --steps 200 --warmup 20 --fuse_level 2 > $out/prof.log 2>&1
rc=$?
python -c "
import json
for l in open('$out/bench.jsonl'):
    d=json.loads(l); print(d['config']['fuse_level'], d['value'], d['ms_per_step'])
"
cat $out/stamps.txt | grep -v amdgpu.ids
python - <<PY
import csv
r=list(csv.DictReader(open('$out/prof/run_kernel_stats.csv')))
for x in r[:5]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1000,2))
PY
exit $rc
