#!/bin/bash
# ResNet kernel iteration: kernel tests, conv + wgrad sweeps, graphed bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_resnet.log 2>&1 && \
timeout -k 10 300 python -u scripts/resnet_conv_sweep.py > gpurun_out/conv_sweep.jsonl 2> gpurun_out/conv_sweep.err && \
timeout -k 10 240 python -u scripts/wgrad_tile_sweep.py > gpurun_out/wgrad_tiles.jsonl 2> gpurun_out/wgrad_tiles.err && \
timeout -k 10 300 python bench.py --model resnet18 --steps 50 --warmup 10 > gpurun_out/resnet_graph.json 2> gpurun_out/resnet.err
rc=$?; echo "chain rc=$rc"; tail -1 gpurun_out/pytest_resnet.log; tail -1 gpurun_out/conv_sweep.jsonl; grep -h '^{' gpurun_out/resnet_graph.json; exit $rc
