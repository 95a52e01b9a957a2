# Multi-rank GPU trainer rehearsal (2 ranks on one GPU, gloo control plane + xGMI data plane)
# and the engine / xGMI GPU tests.
set -o pipefail
out=gpurun_out/${1:-mr}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_cli_multirank_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > $out/pytest_mr.log 2>&1
echo exit=$?
