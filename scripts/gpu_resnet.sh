#!/bin/bash
# ResNet-18 (BASELINE config 5) session: kernel/equivalence tests, our bench (graphed and
# eager), stock PyTorch-ROCm on the same config, the conv launch-plan sweep, and
# rocprofv3 kernel traces of ours and of stock PyTorch.  Each GPU step has its own limit;
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$(pwd)"
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_resnet.log 2>&1 && \
timeout -k 10 300 python bench.py --model resnet18 --steps 50 --warmup 10 > gpurun_out/resnet_graph.json 2> gpurun_out/resnet.err && \
timeout -k 10 300 python bench.py --model resnet18 --steps 50 --warmup 10 --no_graph > gpurun_out/resnet_eager.json 2>> gpurun_out/resnet.err && \
timeout -k 10 300 python scripts/resnet_torch_ref.py --steps 50 --warmup 10 > gpurun_out/resnet_torch.json 2>> gpurun_out/resnet.err && \
timeout -k 10 300 python -u scripts/resnet_conv_sweep.py > gpurun_out/conv_sweep.jsonl 2>&1 && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_resnet" -o rn -- python "$R/bench.py" --model resnet18 --steps 10 --warmup 5 --no_graph > "$R/gpurun_out/prof_resnet.log" 2>&1) && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_resnet_torch" -o rt -- python "$R/scripts/resnet_torch_ref.py" --steps 10 --warmup 30 > "$R/gpurun_out/prof_resnet_torch.log" 2>&1)
rc=$?; echo "chain rc=$rc"; tail -1 gpurun_out/pytest_resnet.log; grep -h '^{' gpurun_out/resnet_*.json; exit $rc
