# In-call A/B of two builds of the extension (box-to-box variance is a few %):
# gpu_abso.sh OUT A_SO "bench args" [reps]  - alternates DDP_AMD_NATIVE_SO=A_SO and the
# in-tree _C.so, REPS rounds each, prints value / ms per run.
set -o pipefail
out=gpurun_out/$1; a=$2; args=$3; reps=${4:-3}
mkdir -p $out
for r in $(seq $reps); do
  DDP_AMD_NATIVE_SO=$a timeout -k 10 120 python -u bench.py $args > $out/a_$r.json 2>> $out/err.log || exit $?
  timeout -k 10 120 python -u bench.py $args > $out/b_$r.json 2>> $out/err.log || exit $?
  python -c "import json; j=lambda f: json.loads([l for l in open(f) if l.startswith('{')][-1]); a=j('$out/a_$r.json'); b=j('$out/b_$r.json'); print('A', a['value'], a['ms_per_step'], ' B', b['value'], b['ms_per_step'])"
done
