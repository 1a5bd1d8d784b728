# hash phase A and the G2 decompression at 3 waves/SIMD (168 VGPRs: the square-root window table
# without scratch) vs 4 (variants/w3 vs main): same-box A/B, GPU suite on main
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03x
mkdir -p $O
for v in main w3 main w3; do
  lib=$PWD/drand_amd/libblsverify.so; [ $v = main ] || lib=$PWD/variants/libblsverify_$v.so
  DRAND_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 >> $O/bench_$v.json 2>> $O/bench_$v.err || exit 13
done
echo done
