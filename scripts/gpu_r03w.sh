# Miller sub-chunks as a two-stream pipeline (f pass of sub-chunk j on the side stream beside the lines
# of j + 1 into a second staging buffer): GPU suite, same-box A/B against BLSV_MILLER_PIPE=0
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 12
for v in pipe serial pipe serial; do
  p=1; [ $v = pipe ] || p=0
  BLSV_MILLER_PIPE=$p timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 >> $O/bench_$v.json 2>> $O/bench_$v.err || exit 13
done
echo done
