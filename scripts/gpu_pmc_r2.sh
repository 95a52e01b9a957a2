#!/bin/bash
# Hardware counters of the 3-kernel SimpleCNN step (rocprofv3 --pmc, one pass per
# counter group, no tracing domains; eager run so counters are per dispatch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
OUT=${1:-pmc2}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d "$R/gpurun_out/$OUT/s1" -o s -- python "$R/bench.py" --no_graph --steps 20 --warmup 5 > "$R/gpurun_out/$OUT/s1.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/$OUT/s2" -o s -- python "$R/bench.py" --no_graph --steps 20 --warmup 5 > "$R/gpurun_out/$OUT/s2.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/$OUT/s3" -o s -- python "$R/bench.py" --no_graph --steps 20 --warmup 5 > "$R/gpurun_out/$OUT/s3.log" 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
