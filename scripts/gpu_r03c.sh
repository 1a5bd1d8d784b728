# latency path on the GPU: parity against goldens and the batch path, then per-arrival latency
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03c
timeout -k 10 300 python -u -m pytest tests/test_gpu_lat.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03c/pytest_lat.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out gpurun_out/r03c/latency_lat.json > gpurun_out/r03c/latency_lat.log 2>&1 || exit 12
timeout -k 10 300 python -u tools/latency_bench.py --reps 5 --lat-max 0 --out gpurun_out/r03c/latency_batch.json > gpurun_out/r03c/latency_batch.log 2>&1 || exit 13
echo done
