# r02 first GPU pass: C-ABI harness (no torch), smoke (no torch), GPU tests, default bench, configs[3] slice
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 tools/cabi_smoke tests/golden/cabi_vectors.txt > gpurun_out/r02_cabi_smoke.txt 2>&1 || exit 11
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || exit 12
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/r02_pytest_gpu.log 2>&1 || exit 13
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r02_bench_1m.json 2> gpurun_out/r02_bench_1m.err || exit 14
timeout -k 10 600 python -u bench.py --total-rounds 100000000 --slice 7/8 --steps 2 --warmup 1 > gpurun_out/r02_bench_cfg3_slice7of8.json 2> gpurun_out/r02_bench_cfg3.err || exit 15
echo done
