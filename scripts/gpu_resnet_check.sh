# ResNet-18 kernel tests, a 200-step graphed bench and a rocprofv3 kernel-stats pass
set -o pipefail
out=gpurun_out/${1:-rc}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 && \
timeout -k 10 180 python -u bench.py --model resnet18 --steps 200 --warmup 10 > $out/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python -u bench.py --model resnet18 --steps 20 --warmup 3 > $out/prof.log 2>&1
echo exit=$?
