# A/B of variants/*.so at 1M (bench) plus the GPU scale tests on each variant (they run the >64Ki paths)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-abs}
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 > gpurun_out/${TAG}_bench_1m.json 2> gpurun_out/${TAG}_bench_1m.err || exit 13
for so in variants/*.so; do
  [ -f "$so" ] || continue
  v=$(basename $so .so)
  DRAND_AMD_LIB=$PWD/$so timeout -k 10 200 python -u bench.py --n 1000000 --steps 5 --warmup 1 --cpu-per-worker 0 > gpurun_out/${TAG}_var_$v.json 2> gpurun_out/${TAG}_var_$v.err || exit 14
  DRAND_AMD_LIB=$PWD/$so timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_var_${v}_scale.log 2>&1 || exit 15
done
echo done
