# Profile set of the current tree: GPU suite, smoke (no torch), default bench (with cpu_baseline),
# rocprofv3 kernel stats (serial stages), PMC HBM traffic (FETCH/WRITE passes), per-kernel SQ/GRBM
# counters (two passes), latency contract (cabi_smoke, latency_bench)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 12
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 13
BLSV_SERIAL_STAGES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --cpu-per-worker 0 > $O/bench_serial_prof.json 2> $O/prof.log || exit 14
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > $O/pmc_fetch.log 2>&1 || exit 15
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > $O/pmc_write.log 2>&1 || exit 16
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
PB="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 240 rocprofv3 --pmc $PA --output-format csv -d $O/pmc_a -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > $O/pmc_a.log 2>&1 || exit 17
timeout -s KILL 240 rocprofv3 --pmc $PB --output-format csv -d $O/pmc_b -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > $O/pmc_b.log 2>&1 || exit 18
python3 tools/pmc_sq.py $O/pmc_sq.json $O/pmc_a/run_counter_collection.csv $O/pmc_b/run_counter_collection.csv > /dev/null || exit 19
timeout -k 10 120 tools/cabi_smoke > $O/cabi_smoke.txt 2>&1 || exit 20
timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out $O/latency.json > $O/latency.log 2>&1 || exit 21
echo done
