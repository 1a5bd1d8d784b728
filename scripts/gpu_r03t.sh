# lines pass with T parked in LDS (BLS_LINES_T_LDS=1, scratch 0): GPU suite, same-box A/B against
# T in registers (variants/tr) and against T in LDS plus the folded line operands (variants/fold)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 12
for v in main tr fold main tr fold; do
  lib=$PWD/drand_amd/libblsverify.so; [ $v = main ] || lib=$PWD/variants/libblsverify_$v.so
  DRAND_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 >> $O/bench_$v.json 2>> $O/bench_$v.err || exit 13
done
echo done
