set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -rfE > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then echo "pytest crashed rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --fuse_level 0 > gpurun_out/bench_f0.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python bench.py --fuse_level 1 > gpurun_out/bench_f1.json 2>> gpurun_out/bench.err && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o bench -- python "$GRAFT_REPO_ROOT/bench.py" --steps 200 --warmup 20 --fuse_level 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1)
rc=$?; echo "chain rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; cat gpurun_out/bench_f*.json; exit $rc
