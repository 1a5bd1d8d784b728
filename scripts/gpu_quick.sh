# quick GPU iteration: parity tests, fp microbench, one 1M bench (each step time-limited)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-quick}
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit 12
if [ -x tools/fpbench ]; then timeout -k 10 120 tools/fpbench > gpurun_out/${TAG}_fpbench.txt 2>&1 || exit 13; fi
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --cpu-per-worker 0 > gpurun_out/${TAG}_bench.log 2>&1 || exit 14
echo done
