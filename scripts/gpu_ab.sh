# A/B: engine bitwise tests + alternating benches of the default config and given variants
# usage: gpu_ab.sh OUT "label1:args1" "label2:args2" ...
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for rep in 1 2; do
  for v in "$@"; do
    lab=${v%%:*}; args=${v#*:}
    timeout -k 10 120 python -u bench.py $args > $out/b_${lab}_$rep.json 2>> $out/bench.err || exit $?
    python -c "import json; d=json.load(open('$out/b_${lab}_$rep.json')); print('$lab', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 120 python -u scripts/stamps.py --graph > $out/stamps.txt 2>&1 || exit $?
grep -v amdgpu.ids $out/stamps.txt
