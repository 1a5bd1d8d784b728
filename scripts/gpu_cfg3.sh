# configs[3] shard slice (12.5M rounds = shard 7/8 of one 100M-round history) + configs[2]/[4] legs
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-cfg}
timeout -k 10 600 python -u bench.py --total-rounds 100000000 --slice 7/8 --steps 2 --warmup 1 > gpurun_out/${TAG}_cfg3_slice7of8.json 2> gpurun_out/${TAG}_cfg3.err || exit 11
timeout -k 10 600 python -u tools/config_bench.py > gpurun_out/${TAG}_config_bench.json 2> gpurun_out/${TAG}_config_bench.log || exit 12
echo done
