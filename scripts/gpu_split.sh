# wgrad channel split: bitwise tests, then bench / stamps for split 1 vs 2 over wgrad rows
set -o pipefail
out=gpurun_out/${1:-split}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "channel_split or fused_reduce" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for cfg in "1 7" "2 7" "2 14" "2 4" "1 7" "2 7"; do
  set -- $cfg
  timeout -k 10 120 python -u bench.py --wgrad_split $1 --wgrad_rows $2 > $out/b_$1_$2.json 2>> $out/bench.err || exit $?
  python -c "import json; d=json.load(open('$out/b_$1_$2.json')); print('split $1 rows $2', d['value'], d['ms_per_step'])"
done
timeout -k 10 120 python -u bench.py --wgrad_split 2 --batch_size 64 > $out/b64.json 2>> $out/bench.err && python -c "import json; d=json.load(open('$out/b64.json')); print('B64 split2', d['value'], d['ms_per_step'])"
timeout -k 10 120 python -u scripts/stamps.py --graph --wgrad_split 2 > $out/stamps2.txt 2>&1 || exit $?
grep -v amdgpu.ids $out/stamps2.txt
