# fc role with two 128-column chunks per wave (DDP_AMD_FC_CPW=2): bitwise tests, A/B at B = 32 / 64
out=gpurun_out/${1:-r4_o}; mkdir -p $out
DDP_AMD_FC_CPW=2 timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py \
  tests/test_fp32_gpu.py -k "level3 or fuse_level or bitwise" > $out/pytest.log 2>&1 || { tail -20 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
bash scripts/gpu.sh ab ${1:-r4_o} DDP_AMD_FC_CPW=1 DDP_AMD_FC_CPW=2 3 || exit 1
for c in 1 2; do DDP_AMD_FC_CPW=$c timeout -k 10 200 python bench.py --no_fp32 --batch_size 64 > $out/b64_c$c.json 2>>$out/err.log || exit 1
  echo "B64 cpw $c: $(grep -o '"value": [0-9.]*' $out/b64_c$c.json)"; done
DDP_AMD_FC_CPW=2 timeout -k 10 200 python scripts/stamps.py --graph > $out/stamps_b32_c2.txt 2>&1 && grep -E "fc_bwd|grad_reduce|wgrad|dgrad " $out/stamps_b32_c2.txt
