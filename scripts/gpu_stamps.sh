# In-kernel phase stamps of the fused step for a few engine configs (diagnostic).
set -o pipefail
out=gpurun_out/${1:-stamps}
mkdir -p $out
for lvl in ${2:-1 3}; do
  timeout -k 10 120 python -u scripts/stamps.py --fuse_level $lvl --graph > $out/stamps_l${lvl}_graph.txt 2>&1 || exit $?
done
