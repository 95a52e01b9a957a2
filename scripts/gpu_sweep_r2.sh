# headline-config sweep: wgrad rows / dgrad tiling / stored a1, plus B=64 (README example)
set -o pipefail
out=gpurun_out/${1:-sw}
mkdir -p $out
: > $out/sweep.jsonl
for args in "" "--wgrad_rows 14" "--wgrad_rows 4" "--pxt_dgrad 1" "--store_a1 1" "--store_a1 2" "--batch_size 64" "--batch_size 64 --wgrad_rows 7" "--dtype fp32" "--dtype fp32 --batch_size 64" "--dtype fp32 --wgrad_rows 4" "--dtype fp32 --pxt_dgrad 1"; do
  timeout -k 10 120 python -u bench.py --steps 1000 --warmup 100 $args > $out/one.json 2>> $out/sweep.err || exit $?
  python -c "
import json,sys; d=json.load(open('$out/one.json')); c=d['config']
print(json.dumps({'args': '$args', 'img_s': d['value'], 'us_step': round(d['ms_per_step']*1000,2), 'dtype': d['dtype'], 'B': c['per_rank_batch'], 'tiling': c['tiling']}))" >> $out/sweep.jsonl
done
cat $out/sweep.jsonl
