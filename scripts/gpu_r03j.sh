# final-exponentiation squaring chains A/B: split Granger-Scott (default build), Granger-Scott on three
# lanes (variants/libblsverify_gs.so), Karabina (variants/libblsverify_kara.so); parity of each first
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03j
mkdir -p $O
for v in main gs kara; do
  lib=$PWD/drand_amd/libblsverify.so; [ $v = main ] || lib=$PWD/variants/libblsverify_$v.so
  DRAND_AMD_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -v -k "final_exp or pairing or chained_golden" --timeout 120 --timeout-method thread > $O/pytest_fexp_$v.log 2>&1 || exit 11
done
for v in main gs kara main; do
  lib=$PWD/drand_amd/libblsverify.so; [ $v = main ] || lib=$PWD/variants/libblsverify_$v.so
  DRAND_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 >> $O/bench_$v.json 2>> $O/bench_$v.err || exit 13
done
BLSV_SERIAL_STAGES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --cpu-per-worker 0 > $O/bench_serial_prof.json 2> $O/prof.log || exit 16
echo done
