set -o pipefail
scripts/gpu.sh tests r5_benchchk/t "bench_" && timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r5_benchchk/b.json 2>/dev/null && cat gpurun_out/r5_benchchk/b.json
