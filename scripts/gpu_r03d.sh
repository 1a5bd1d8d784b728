# full GPU suite on the current tree (latency path + lane-form recover), then per-arrival latency
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03d/pytest_gpu.log 2>&1 || exit 11
timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out gpurun_out/r03d/latency_lat.json > gpurun_out/r03d/latency_lat.log 2>&1 || exit 12
echo done
