# A/B runs of library variants (variants/*.so via DRAND_AMD_LIB), one short bench each
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-var}
N=${N:-262144}
for so in variants/*.so; do
  v=$(basename $so .so)
  DRAND_AMD_LIB=$PWD/$so timeout -k 10 200 python -u bench.py --n $N --steps 3 --warmup 1 --cpu-per-worker 0 > gpurun_out/${TAG}_$v.log 2>&1 || exit 14
  echo "$v $(grep '^{' gpurun_out/${TAG}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stages_ms_per_launch'])")"
done
