# AMDGPU machine-scheduler strategies for the hash, decompression, Miller and final-exp units
# (variants/ilp: max-ilp, iter: iterative-ilp, mclause: max-memory-clause) vs the default (main):
# same-box A/B, then the GPU suite on each variant
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03sched
mkdir -p $O
for v in main ilp iter mclause main ilp iter mclause; do
  lib=$PWD/drand_amd/libblsverify.so; [ $v = main ] || lib=$PWD/variants/libblsverify_$v.so
  DRAND_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 >> $O/bench_$v.json 2>> $O/bench_$v.err || exit 13
done
for v in ilp iter mclause; do
  DRAND_AMD_LIB=$PWD/variants/libblsverify_$v.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu_$v.log 2>&1 || exit 12
done
echo done
