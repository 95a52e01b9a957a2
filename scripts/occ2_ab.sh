# level-3 forward at two blocks per CU (DDP_AMD_FWD_OCC2) - correctness at B = 64, then A/B
out=gpurun_out/${1:-r4_j}; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py \
  -k "level3 or fuse_level" > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for r in 1 2; do for o in 0 1; do
  DDP_AMD_FWD_OCC2=$o timeout -k 10 200 python bench.py --batch_size 64 --no_fp32 > $out/b64_o${o}_$r.json 2>>$out/err.log || exit 1
  DDP_AMD_FWD_OCC2=$o timeout -k 10 200 python bench.py --batch_size 64 --no_fp32 --steps 20 --warmup 5 > $out/b64d_o${o}_$r.json 2>>$out/err.log || exit 1
  echo "B64 occ2=$o run $r: 1000 $(grep -o '"value": [0-9.]*' $out/b64_o${o}_$r.json) | driver $(grep -o '"value": [0-9.]*' $out/b64d_o${o}_$r.json)"
done; done
for o in 0 1; do DDP_AMD_FWD_OCC2=$o timeout -k 10 200 python scripts/stamps.py --batch_size 64 --graph > $out/stamps_o$o.txt 2>>$out/err.log || exit 1; done
head -30 $out/stamps_o1.txt
