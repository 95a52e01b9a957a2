#!/bin/bash
# End-of-round check: every GPU test, smoke, the default bench (bf16 headline + fp32), the
# driver-shaped 20-step bench, ResNet-18, rocprofv3 kernel stats of the headline step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3final}
mkdir -p $out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rfE > $out/pytest_gpu.log 2>&1
rc=$?; tail -2 $out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_driver.json 2>> $out/bench.err && \
timeout -k 10 300 python bench.py --model resnet18 --steps 50 --warmup 10 > $out/bench_resnet.json 2>> $out/bench.err && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof" -o bench -- python "$R/bench.py" --steps 200 --warmup 20 --no_fp32 > "$R/$out/prof.log" 2>&1)
rc=$?; echo "chain rc=$rc"; tail -1 $out/smoke.log; for f in $out/bench*.json; do echo "$f: $(grep -o '"value": [0-9.]*' $f) $(grep -o '"fp32_images_per_sec": [0-9.]*' $f)"; done; exit $rc
