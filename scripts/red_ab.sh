# reducer offsets precomputed before the wait: bitwise tests, A/B vs the previous build, stamps
out=gpurun_out/${1:-r4_n}; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_fp32_gpu.py \
  -k "level3 or fuse_level or bitwise" > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
bash scripts/gpu.sh ab ${1:-r4_n} so=abso/_C_prev.so AB=1 3 || exit 1
timeout -k 10 200 python scripts/stamps.py --graph > $out/stamps_b32.txt 2>&1 && grep grad_reduce $out/stamps_b32.txt
