# call-free Miller line steps at 2 waves/SIMD: full GPU suite, then same-box A/B against the called
# steps (variants/linesold), serial-stage kernel stats and the lines kernel's HBM traffic
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 12
for v in main linesold main; do
  lib=$PWD/drand_amd/libblsverify.so; [ $v = main ] || lib=$PWD/variants/libblsverify_$v.so
  DRAND_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 >> $O/bench_$v.json 2>> $O/bench_$v.err || exit 13
done
BLSV_SERIAL_STAGES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --cpu-per-worker 0 > $O/bench_serial_prof.json 2> $O/prof.log || exit 16
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > $O/pmc_fetch.log 2>&1 || exit 17
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > $O/pmc_write.log 2>&1 || exit 18
echo done
