# latency-engine field microbenchmark (tools/wvbench): chain correctness + per-product latency;
# tools/latbench: dependent-issue latencies of the chained instructions
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03b
timeout -k 10 60 ./tools/latbench > gpurun_out/r03b/latbench.json 2>&1 || exit 10
timeout -k 10 120 ./tools/wvbench 2000 > gpurun_out/r03b/wvbench.json 2> gpurun_out/r03b/wvbench.err || exit 11
python3 tools/wvbench_check.py gpurun_out/r03b/wvbench.json gpurun_out/r03b/wvbench_summary.json || exit 12
echo done
