set -o pipefail
mkdir -p gpurun_out/ws2
for px in 0 1568 6272; do
DDP_AMD_WGRAD_STREAM_PX=$px timeout -k 10 180 python -u bench.py --model resnet18 --steps 200 --warmup 10 > gpurun_out/ws2/bench_px$px.log 2>&1 || exit 1
done
DDP_AMD_WGRAD_STREAM_PX=0 timeout -k 10 180 python -u bench.py --model resnet18 --steps 200 --warmup 10 > gpurun_out/ws2/bench_px0b.log 2>&1
echo exit=$?
