set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --cpu-per-worker 1 > gpurun_out/bench_1m.log 2>&1 || exit 14
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_1m -o run -- python -u bench.py --steps 2 --warmup 1 --cpu-per-worker 0 > gpurun_out/rocprof_1m.log 2>&1 || exit 15
echo done
