#!/bin/bash
# SimpleCNN headline: smoke, default bench (bf16 headline + fp32), driver-shaped 20-step bench,
# rocprofv3 kernel stats, in-kernel phase stamps of the graphed step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r3cnn}
mkdir -p $out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_fp32 > $out/bench_driver.json 2>> $out/bench.err && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof" -o bench -- python "$R/bench.py" --steps 200 --warmup 20 --no_fp32 > "$R/$out/prof.log" 2>&1) && \
timeout -k 10 120 python -u scripts/stamps.py --graph > $out/stamps_graph.log 2>&1
rc=$?; echo "chain rc=$rc"; cat $out/bench*.json | cut -c1-400; exit $rc
