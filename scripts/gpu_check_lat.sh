# GPU tests, 1M bench, variants A/B, then the per-arrival latency bench (tools/latency_bench.py)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-chk}
bash scripts/gpu_check.sh $TAG || exit $?
timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out gpurun_out/${TAG}_latency.json > gpurun_out/${TAG}_latency.log 2>&1 || exit 16
if [ -f variants/base.so ]; then
  DRAND_AMD_LIB=$PWD/variants/base.so timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out gpurun_out/${TAG}_latency_base.json > gpurun_out/${TAG}_latency_base.log 2>&1 || exit 17
fi
echo done
