#!/bin/bash
# Hardware counters (rocprofv3 --pmc, one pass per counter group, no tracing domains)
# over eager runs of the SimpleCNN headline step and the ResNet-18 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$(pwd)"
mkdir -p gpurun_out/pmc_r
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d "$R/gpurun_out/pmc_r/s1" -o s -- python "$R/bench.py" --no_graph --steps 20 --warmup 5 > "$R/gpurun_out/pmc_r/s1.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_r/s2" -o s -- python "$R/bench.py" --no_graph --steps 20 --warmup 5 > "$R/gpurun_out/pmc_r/s2.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_r/s3" -o s -- python "$R/bench.py" --no_graph --steps 20 --warmup 5 > "$R/gpurun_out/pmc_r/s3.log" 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc $P1 --output-format csv -d "$R/gpurun_out/pmc_r/r1" -o r -- python "$R/bench.py" --model resnet18 --no_graph --steps 3 --warmup 2 > "$R/gpurun_out/pmc_r/r1.log" 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_r/r2" -o r -- python "$R/bench.py" --model resnet18 --no_graph --steps 3 --warmup 2 > "$R/gpurun_out/pmc_r/r2.log" 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
