# Karabina (compressed) cyclotomic squaring in the final exponentiation: parity first, then the GPU
# suite, the 1M bench of the new tree, the Granger-Scott variant (variants/libblsverify_gs.so) on the
# same box, and rocprofv3 kernel stats of the new tree with serial stages.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "final_exp or pairing or chained_golden" --timeout 120 --timeout-method thread > $O/pytest_fexp.log 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 12
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 > $O/bench_1m.json 2> $O/bench_1m.err || exit 13
DRAND_AMD_LIB=$PWD/variants/libblsverify_gs.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 > $O/bench_1m_gs.json 2> $O/bench_1m_gs.err || exit 14
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-per-worker 0 > $O/bench_1m_b.json 2> $O/bench_1m_b.err || exit 15
BLSV_SERIAL_STAGES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --cpu-per-worker 0 > $O/bench_serial_prof.json 2> $O/prof.log || exit 16
echo done
