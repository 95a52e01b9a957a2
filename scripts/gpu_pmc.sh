#!/bin/bash
# Tests + in-graph kernel bench + PMC counters of the eager kernel bench + headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -q -rfE -x > gpurun_out/pmc/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pmc/pytest.log
if [ $rc -ne 0 ]; then echo "pytest failed rc=$rc"; exit $rc; fi
timeout -k 10 300 python scripts/kbench.py --json gpurun_out/pmc/kbench.json > gpurun_out/pmc/kbench.log 2>&1 || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pmc/kt" -o kb -- python "$R/scripts/kbench.py" --eager --reps 20 > "$R/gpurun_out/pmc/kt.log" 2>&1) || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/pmc1" -o kb -- python "$R/scripts/kbench.py" --eager --reps 3 > "$R/gpurun_out/pmc/pmc1.log" 2>&1) || exit $?
for fl in 0 1; do
  timeout -k 10 120 python bench.py --steps 500 --warmup 50 --fuse_level $fl --pxt_fwd 1 >> gpurun_out/pmc/bench.jsonl 2>> gpurun_out/pmc/bench.err || exit $?
done
echo pmc done
