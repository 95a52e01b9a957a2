#!/bin/bash
# One parameterised GPU driver (run through gpurun from the repo root):
#
#   scripts/gpu.sh <task> <out> [extra args...]      results land in gpurun_out/<out>/
#
# tasks (each GPU step runs under its own timeout; the first failure ends the call):
#   tests [pytest -k expr]     pytest -m gpu (one process), log in pytest_gpu.log
#   smoke                      __graft_entry__.smoke()
#   bench [bench args]         driver-shaped bench (--steps 20 --warmup 5), then 1000 steps
#   trace [bench args]         rocprofv3 kernel trace of the driver-shaped run + per-step table
#   stats [bench args]         rocprofv3 --kernel-trace --stats of a 200-step run
#   ab <envA> <envB> [n] [bench args]   alternate two env settings (e.g. DDP_AMD_GRAPH_UPLOAD=0
#                              vs DDP_AMD_GRAPH_UPLOAD=1) over n rounds of driver-shaped +
#                              1000-step runs; "so=<path>" as an env selects another _C.so
#   resnet [bench args]        ResNet-18 bench (graph) + rocprofv3 stats
#   pmc <counters> [bench args]  one PMC pass (<= 8 SQ counters) over a 200-step run
#   roofline                   ResNet-18 per-layer roofline (scripts/resnet_roofline.py) -> roofline.md
#   rehearse [n...]            N-rank rehearsal of the xGMI data plane on ONE GPU (gloo control
#                              plane, bench.py --backend gloo --comm xgmi; default n = 4 8)
#   calibrate [n]              fit the xGMI cost model on n same-GPU ranks (scripts/comm_calibrate.py)
#   sweep <run>...             bench variants, each run "tag|ENV=v ENV2=w|bench args" (env and args
#                              may be empty): 1000-step + driver-shaped json per tag, one line each
#   stamps [stamps.py args]    in-kernel phase timeline (scripts/stamps.py --graph) -> stamps.txt
#   all                        tests + smoke + bench + stats + resnet (round-end evidence)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
task=$1; out=gpurun_out/${2:?out dir}; shift 2
mkdir -p "$out"
T() { timeout -k 10 "$@"; }
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"

run_tests() { T 1100 $PYT -m gpu tests ${1:+-k "$1"} > "$out/pytest_gpu.log" 2>&1; rc=$?; tail -3 "$out/pytest_gpu.log"; return $rc; }
run_smoke() { T 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 && cat "$out/smoke.log"; }
run_bench() {
  T 300 python bench.py --steps 20 --warmup 5 "$@" > "$out/bench_driver.json" 2>> "$out/err.log" &&
    echo "driver-shaped: $(cat "$out/bench_driver.json")" &&
    T 300 python bench.py "$@" > "$out/bench.json" 2>> "$out/err.log" &&
    echo "1000 steps: $(cat "$out/bench.json")"
}
run_trace() {
  T 300 rocprofv3 --kernel-trace --output-format csv -d "$out/trace" -- python bench.py --steps 20 --warmup 5 \
      --no_fp32 "$@" > "$out/trace_bench.json" 2>> "$out/err.log" &&
    python scripts/step_trace.py "$out/trace" 20 > "$out/step_trace.md" && cat "$out/step_trace.md"
}
run_stats() {
  T 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -- python bench.py --steps 200 \
      --warmup 20 "$@" > "$out/stats_bench.json" 2>> "$out/err.log" &&
    f=$(find "$out/prof" -name '*kernel_stats.csv' | head -1) && cp "$f" "$out/kernel_stats.csv" &&
    head -12 "$out/kernel_stats.csv"
}
run_ab() {
  A=$1; Bv=$2; n=${3:-3}; shift 3
  for r in $(seq 1 "$n"); do
    for e in "$A" "$Bv"; do
      tag=$(echo "$e" | tr -c 'A-Za-z0-9_=.\n' '_')
      if [[ $e == so=* ]]; then envs="DDP_AMD_NATIVE_SO=${e#so=}"; else envs="$e"; fi
      env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no_fp32 "$@" > "$out/d_${tag}_$r.json" 2>> "$out/err.log" || return $?
      env $envs timeout -k 10 300 python bench.py --no_fp32 "$@" > "$out/l_${tag}_$r.json" 2>> "$out/err.log" || return $?
      echo "$e run $r: driver $(grep -o '"value": [0-9.]*' "$out/d_${tag}_$r.json") | 1000 $(grep -o '"value": [0-9.]*' "$out/l_${tag}_$r.json")"
    done
  done
}
run_resnet() {
  T 400 python bench.py --model resnet18 --steps 50 --warmup 10 "$@" > "$out/bench_resnet.json" 2>> "$out/err.log" &&
    cat "$out/bench_resnet.json" &&
    T 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_resnet" -- python bench.py --model resnet18 \
      --steps 20 --warmup 5 "$@" > /dev/null 2>> "$out/err.log" &&
    f=$(find "$out/prof_resnet" -name '*kernel_stats.csv' | head -1) && cp "$f" "$out/resnet_kernel_stats.csv"
}
run_pmc() {
  c=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out/pmc" -- python bench.py --steps 200 \
      --warmup 20 --no_fp32 "$@" > /dev/null 2>> "$out/err.log"
}

run_roofline() {
  T 400 rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv -d "$out/rf" -- python \
      scripts/resnet_roofline.py run --out "$out/calls.json" > "$out/roofline_run.log" 2>&1 &&
    python scripts/resnet_roofline.py report "$out/rf" --calls "$out/calls.json" --md "$out/roofline.md" > /dev/null &&
    head -40 "$out/roofline.md"
}

run_rehearse() {
  export DDP_AMD_XGMI_GRID_CAP=${DDP_AMD_XGMI_GRID_CAP:-16} DDP_AMD_XGMI_TIMEOUT_S=${DDP_AMD_XGMI_TIMEOUT_S:-20}
  for n in ${@:-4 8}; do
    T 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --backend gloo --comm xgmi --steps 200 --warmup 20 \
      --no_comm_calibration > "$out/bench_n$n.log" 2>&1 || { echo "n=$n failed"; return 1; }
    tail -1 "$out/bench_n$n.log"
  done
}
run_calibrate() {
  T 300 python scripts/comm_calibrate.py --ranks ${1:-2} --out "$out/xgmi_calibration.json" > "$out/calibrate.log" 2>&1 &&
    cat "$out/calibrate.log"
}
run_sweep() {
  for spec in "$@"; do
    IFS='|' read -r tag envs args <<< "$spec"
    env $envs timeout -k 10 200 python bench.py $args > "$out/l_$tag.json" 2>> "$out/err.log" || return $?
    env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 $args > "$out/d_$tag.json" 2>> "$out/err.log" || return $?
    echo "$tag: 1000 $(grep -o '"value": [0-9.]*' "$out/l_$tag.json") | driver $(grep -o '"value": [0-9.]*' "$out/d_$tag.json")"
  done
}
run_stamps() { T 200 python scripts/stamps.py --graph "$@" > "$out/stamps.txt" 2>&1 && grep -v amdgpu.ids "$out/stamps.txt"; }

case $task in
  tests) run_tests "$@" ;;
  smoke) run_smoke ;;
  bench) run_bench "$@" ;;
  trace) run_trace "$@" ;;
  stats) run_stats "$@" ;;
  ab) run_ab "$@" ;;
  resnet) run_resnet "$@" ;;
  pmc) run_pmc "$@" ;;
  roofline) run_roofline ;;
  rehearse) run_rehearse "$@" ;;
  calibrate) run_calibrate "$@" ;;
  sweep) run_sweep "$@" ;;
  stamps) run_stamps "$@" ;;
  all) run_tests && run_smoke && run_bench && run_stats && run_resnet ;;
  *) echo "unknown task $task"; exit 2 ;;
esac
