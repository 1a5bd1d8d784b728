# latency of the per-arrival callers (tools/latency_bench.py) + GPU tests
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-lat}
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit 12
timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out gpurun_out/${TAG}_latency.json > gpurun_out/${TAG}_latency.log 2>&1 || exit 13

if [ -f variants/base.so ]; then
  DRAND_AMD_LIB=$PWD/variants/base.so timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out gpurun_out/${TAG}_latency_base.json > gpurun_out/${TAG}_latency_base.log 2>&1 || exit 14
fi
echo done
