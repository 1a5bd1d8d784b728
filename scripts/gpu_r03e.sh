# four-wave team verify: lat parity first (short limit), then the full GPU suite and latency numbers
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03e
timeout -k 10 180 python -u -m pytest tests/test_gpu_lat.py -x -v --timeout 60 --timeout-method thread > gpurun_out/r03e/pytest_lat.log 2>&1 || exit 11
timeout -k 10 120 python -u tools/latency_bench.py --reps 10 --out gpurun_out/r03e/latency_lat.json > gpurun_out/r03e/latency_lat.log 2>&1 || exit 12
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03e/pytest_gpu.log 2>&1 || exit 13
echo done
