# persistent-grid lines pass (BLS_LINES_PERSIST=1: a grid of the resident slots walks the work items):
# GPU suite, same-box A/B against the one-workgroup-per-item grid (variants/np)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 12
for v in main np main np; do
  lib=$PWD/drand_amd/libblsverify.so; [ $v = main ] || lib=$PWD/variants/libblsverify_$v.so
  DRAND_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 >> $O/bench_$v.json 2>> $O/bench_$v.err || exit 13
done
echo done
