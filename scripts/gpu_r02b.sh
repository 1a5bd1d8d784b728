# r02 baseline of the current tree: GPU tests, 1M bench, rocprofv3 kernel stats, PMC FETCH/WRITE passes
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02b}
timeout -k 10 120 tools/issuebench > gpurun_out/${TAG}_issuebench.txt 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit 12
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/${TAG}_bench_1m.json 2> gpurun_out/${TAG}_bench_1m.err || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 -u bench.py --steps 2 --warmup 1 --cpu-per-worker 0 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.log || exit 14
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || exit 15
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > gpurun_out/${TAG}_pmc_write.log 2>&1 || exit 16
echo done
