set -o pipefail
out=gpurun_out/${1:-hwp}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad or train or step" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for h in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p$h -o run -- python -u bench.py --model resnet18 --steps 30 --warmup 5 --wgrad_halo $h > $out/p$h.log 2>&1 || exit $?
done
python - <<PY
import csv, collections
for h in (1, 0):
    r = list(csv.DictReader(open('$out/p%d/run_kernel_stats.csv' % h)))
    print('halo', h)
    for x in r:
        n = x['Name']
        if 'wgrad' in n or 'grad_reduce' in n or 'slab' in n:
            print('  %-70s %5s %8.2f %9.1f' % (n[:70], x['Calls'], float(x['AverageNs'])/1000, float(x['TotalDurationNs'])/1000/35))
PY
