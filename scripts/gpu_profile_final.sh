# Round-end profile of the current tree: 1M bench, rocprofv3 kernel stats, two PMC passes (HBM bytes).
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o run -- python3 -u bench.py --steps 2 --warmup 1 --cpu-per-worker 0 > gpurun_out/prof_final_bench.json 2> gpurun_out/prof_final.log || exit 15
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > gpurun_out/pmc_fetch.log 2>&1 || exit 16
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > gpurun_out/pmc_write.log 2>&1 || exit 17
echo done
