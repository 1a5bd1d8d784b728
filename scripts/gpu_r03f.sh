# latency contract through the plain-C harness, the latency-vs-batch crossover sweep, the configs[3]
# full-size shard test and configs[2]/[4] (with the CPU timing of the threshold round)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03f
nproc > gpurun_out/r03f/nproc.txt
timeout -k 10 120 tools/cabi_smoke > gpurun_out/r03f/cabi_smoke.txt 2>&1 || exit 11
timeout -k 10 400 python -u tools/latency_bench.py --reps 5 --sweep 64,256,512,768,1024,1536,2048,3072,4096 --out gpurun_out/r03f/latency_sweep.json > gpurun_out/r03f/latency_sweep.log 2>&1 || exit 12
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -k configs3 -x -v --timeout 240 --timeout-method thread > gpurun_out/r03f/pytest_cfg3.log 2>&1 || exit 13
timeout -k 10 400 python -u tools/config_bench.py --reps 5 --partials-n 0 --store-n 0 > gpurun_out/r03f/config_bench.json 2> gpurun_out/r03f/config_bench.err || exit 14
# Miller-lines variants (scripts/build_variant.sh): per-kernel times of a short bench each
for v in base lines1 linesinl; do
  lib=drand_amd/libblsverify.so; [ $v = base ] || lib=variants/libblsverify_$v.so
  DRAND_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03f/prof_$v -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-per-worker 0 > gpurun_out/r03f/bench_$v.json 2> gpurun_out/r03f/bench_$v.err || exit 15
done
echo done
