# Round-end check of the rebuilt tree (same sources as r03u): smoke (no torch), default bench with
# cpu_baseline, plain-C ABI harness (latency contract)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 13
timeout -k 10 120 tools/cabi_smoke > $O/cabi_smoke.txt 2>&1 || exit 20
echo done
