#!/bin/bash
# Hardware counters of the round-3 SimpleCNN step (level 3, eager launches so every dispatch
# is attributed): one rocprofv3 --pmc pass per counter group, no tracing domains.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
A="--no_graph --steps 20 --warmup 5 --no_fp32 --no_scaling_ref"
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d "$R/gpurun_out/pmc3/s1" -o s -- python "$R/bench.py" $A > "$R/gpurun_out/pmc3/s1.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc3/s2" -o s -- python "$R/bench.py" $A > "$R/gpurun_out/pmc3/s2.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc3/s3" -o s -- python "$R/bench.py" $A > "$R/gpurun_out/pmc3/s3.log" 2>&1
rc=$?; echo "pmc rc=$rc"; cd "$R" && python scripts/pmc_summary.py gpurun_out/pmc3/s1/s_counter_collection.csv gpurun_out/pmc3/s2/s_counter_collection.csv gpurun_out/pmc3/s3/s_counter_collection.csv > gpurun_out/pmc3/simplecnn.md 2>&1; cat gpurun_out/pmc3/simplecnn.md; exit $rc
