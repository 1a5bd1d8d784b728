set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 tools/intrate > gpurun_out/intrate.txt 2>&1 || exit 11
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 12
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 13
timeout -k 10 300 python -u bench.py --n 65536 --steps 2 --warmup 1 --cpu-per-worker 1 > gpurun_out/bench_small.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_small -o run -- python -u bench.py --n 65536 --steps 2 --warmup 1 --cpu-per-worker 0 > gpurun_out/rocprof_small.log 2>&1 || exit 15
echo done
