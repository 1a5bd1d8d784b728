# parity tests + A/B variant benches (+ microbenchmarks when built)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-vt}
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit 12
if [ -x tools/madbench ]; then timeout -k 10 120 tools/madbench > gpurun_out/${TAG}_madbench.txt 2>&1 || exit 13; fi
bash scripts/gpu_variants.sh $TAG
