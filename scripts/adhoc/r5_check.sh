set -o pipefail
out=gpurun_out/r5_check; mkdir -p $out
scripts/gpu.sh tests r5_check/t "level3 or bench_ or b64 or B64" &&
timeout -k 10 200 python bench.py --batch_size 64 --no_fp32 > $out/b64.json 2>> $out/err.log &&
python -c "import json;r=json.loads(open('$out/b64.json').read().strip().splitlines()[-1]);print(r['value'],r['config']['level3'],r['config']['kernels_per_step'])"
