# Level-3 check: engine GPU tests (bitwise vs level 1), bench A/B of level 1 / level 3 (fc
# role: persistent blocks after the conv blocks = 1, after the dgrad blocks = 2, own kernel =
# 0), alternating, then stamps + rocprofv3 kernel stats.
set -o pipefail
out=gpurun_out/${1:-l3}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -k "level3 or rccl or xgmi_world1 or graph_replay or one_step" > $out/pytest_engine.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --fuse_level 1 --no_fp32 > $out/b_l1_$r.json 2>> $out/err.log || exit $?
  timeout -k 10 120 python -u bench.py --l3_fc_role 1 --no_fp32 > $out/b_l3p1_$r.json 2>> $out/err.log || exit $?
  timeout -k 10 120 python -u bench.py --l3_fc_role 2 --no_fp32 > $out/b_l3p2_$r.json 2>> $out/err.log || exit $?
  timeout -k 10 120 python -u bench.py --l3_fc_role 0 --no_fp32 > $out/b_l3s_$r.json 2>> $out/err.log || exit $?
done
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $out/b_l3_driver.json 2>> $out/err.log || exit $?
timeout -k 10 120 python -u scripts/stamps.py --graph > $out/stamps_l3.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- python -u bench.py --steps 200 --warmup 20 --no_fp32 > $out/prof.log 2>&1
echo exit=$?
