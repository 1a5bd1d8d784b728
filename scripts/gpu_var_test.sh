# parity tests + A/B variant benches
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-vt}
timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit 12
bash scripts/gpu_variants.sh $TAG
