# alternating bench sweep of SimpleCNN engine tilings (one box, so runs are comparable)
set -o pipefail
out=gpurun_out/${1:-ts}; shift
mkdir -p $out
for rep in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    timeout -k 10 120 python -u bench.py $v > $out/b_${i}_$rep.json 2>> $out/err.log || exit $?
    python -c "import json; d=json.load(open('$out/b_${i}_$rep.json')); print('[$v]', d['value'], d['ms_per_step'])"
  done
done
