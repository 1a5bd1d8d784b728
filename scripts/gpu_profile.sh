# Profile of the current tree: smoke (no torch) + C-ABI harness, 1M bench, rocprofv3 kernel stats and
# PMC FETCH_SIZE / WRITE_SIZE passes (262k beacons, 3 verify launches each), latency bench.
# The profiled runs set BLSV_SERIAL_STAGES=1 (decompression after hashing on one stream) so that
# per-kernel durations are not inflated by the hash/decompression overlap of the production path.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-prof}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 11
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > gpurun_out/${TAG}_bench_1m.json 2> gpurun_out/${TAG}_bench_1m.err || exit 12
export BLSV_SERIAL_STAGES=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 -u bench.py --steps 2 --warmup 1 --cpu-per-worker 0 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.log || exit 13
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || exit 14
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > gpurun_out/${TAG}_pmc_write.log 2>&1 || exit 15
unset BLSV_SERIAL_STAGES
timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out gpurun_out/${TAG}_latency.json > gpurun_out/${TAG}_latency.log 2>&1 || exit 16
echo done
