# reducer: deep (w1) slab chunk loads pipelined - bitwise tests, A/B vs the previous build (bf16 + fp32), stamps
out=gpurun_out/${1:-r4_p}; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_fp32_gpu.py \
  -k "level3 or fuse_level or bitwise or reduce" > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
bash scripts/gpu.sh ab ${1:-r4_p} so=abso/_C_prev.so AB=1 3 || exit 1
for e in so=abso/_C_prev.so AB=1 so=abso/_C_prev.so AB=1; do
  if [[ $e == so=* ]]; then envs="DDP_AMD_NATIVE_SO=${e#so=}"; else envs="$e"; fi
  env $envs timeout -k 10 200 python bench.py --dtype fp32 --no_fp32 > $out/f32.json 2>>$out/err.log || exit 1
  echo "fp32 $e: $(grep -o '"value": [0-9.]*' $out/f32.json)"
done
timeout -k 10 200 python scripts/stamps.py --graph > $out/stamps_b32.txt 2>&1 && grep grad_reduce $out/stamps_b32.txt
timeout -k 10 200 python scripts/stamps.py --graph --dtype fp32 > $out/stamps_fp32.txt 2>&1 && grep -E "grad_reduce|wgrad" $out/stamps_fp32.txt
