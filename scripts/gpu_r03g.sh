# r03 re-entry baseline of the committed tree: GPU tests, smoke (no torch), default bench, rocprofv3
# kernel stats of a short bench with serial stages (clean per-kernel times)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 12
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 13
BLSV_SERIAL_STAGES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --cpu-per-worker 0 > $O/bench_serial_prof.json 2> $O/prof.log || exit 14
echo done
