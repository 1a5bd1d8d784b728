# one GPU iteration: parity tests, smoke, 1M bench, kernel trace, PMC passes (each its own run)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-iter}
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit 12
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 13
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python -u bench.py --n 262144 --steps 2 --warmup 1 --cpu-per-worker 0 > gpurun_out/${TAG}_trace.log 2>&1 || exit 15
if [ -n "$PMC" ]; then
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_pmc$i -o run -- python -u bench.py --n 65536 --steps 1 --warmup 0 --cpu-per-worker 0 > gpurun_out/${TAG}_pmc$i.log 2>&1 || exit $((20+i))
  done
fi
echo done
