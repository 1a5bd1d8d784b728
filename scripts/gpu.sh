# One parameterised GPU-box runner (replaces the per-round scripts/gpu_r0*.sh).
#
#   gpurun -- bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Output goes to gpurun_out/TAG/. Steps run in order; the first failing step ends the call (no GPU
# step runs after a failure, a time limit or a fault). Steps:
#   tests            pytest -m gpu (the whole GPU suite)
#   tests:EXPR       pytest -m gpu -k EXPR
#   smoke            __graft_entry__.smoke() (no torch in the process) + the plain-C ABI harness
#   bench            default bench.py (configs[1], cpu_baseline)
#   fuzz10, fuzz:N   tests/test_gpu_fuzz.py with DRAND_AMD_FUZZ_SCALE=10 / N (that many times the random cases)
#   bench2           bench.py --gpus 2 --dist-backend gloo, weak and strong (two ranks on one GPU)
#   prof             rocprofv3 --kernel-trace --stats of bench.py with BLSV_SERIAL_STAGES=1
#   pmc              PMC passes: FETCH_SIZE, WRITE_SIZE, two SQ/GRBM sets (tools/pmc_sq.py)
#   cabi             tools/cabi_smoke (latency contract from plain C)
#   pmccal           FETCH_SIZE / WRITE_SIZE of tools/pmccal (known bytes in the engine's SoA patterns)
#   wvbench          tools/wvbench (per-operation latency of the latency engine's primitives)
#   fpbench          tools/fpbench (Fp multiply throughput: radix-2^28 interleaved vs 13 x 30-bit SOS)
#   intrate          tools/intrate (peak v_mad_u64_u32 rate) and its SQ/GRBM counters (clock of the peak)
#   lat              tools/latency_bench.py (lone verify, fused round)
#   latsweep         the same with the latency-vs-batch sweep (64 .. 2048 items: co-resident teams)
#   cfg              tools/config_bench.py (configs[2], configs[4], partials, drand.db)
#   variant:NAME     GPU suite + bench on variants/libblsverify_NAME.so (scripts/build_variant.sh,
#                    loaded through DRAND_AMD_LIB)
#   vbench:NAME      bench only on that variant (same-box A/B against a plain `bench` step)
#   ab:N1,N2,..      base and each variant interleaved, two passes (bench_<name>_<pass>.json)
#   vlat:NAME        tools/latency_bench.py on that variant (same-box A/B against a plain `lat` step)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 2
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
PYT="python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread"
B262="python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0"
rc=0
for step in "$@"; do
  echo "[gpu.sh] $step $(date +%T)"
  case "$step" in
    tests) timeout -k 10 900 $PYT > "$O/pytest_gpu.log" 2>&1 || rc=12 ;;
    tests:*) timeout -k 10 900 $PYT -k "${step#tests:}" > "$O/pytest_gpu_k.log" 2>&1 || rc=12 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || rc=11 ;;
    bench) timeout -k 10 400 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || rc=13 ;;
    fuzz10|fuzz:*)
      F=10; [ "$step" != fuzz10 ] && F=${step#fuzz:}
      DRAND_AMD_FUZZ_SCALE=$F timeout -k 10 1100 python -u -m pytest tests/test_gpu_fuzz.py -x -v -m gpu -s \
        --timeout 1000 --timeout-method thread > "$O/pytest_gpu_fuzz_x$F.log" 2>&1 || rc=16 ;;
    bench2)
      timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --n 262144 --steps 2 --warmup 1 \
        --cpu-per-worker 0 > "$O/bench2_weak.json" 2> "$O/bench2_weak.err" &&
      timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --total-rounds 524291 --steps 2 \
        --warmup 1 --cpu-per-worker 0 > "$O/bench2_strong.json" 2> "$O/bench2_strong.err" || rc=14 ;;
    prof)
      BLSV_SERIAL_STAGES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" \
        -o run -- python3 -u bench.py --steps 3 --warmup 1 --cpu-per-worker 0 > "$O/bench_serial_prof.json" \
        2> "$O/prof.log" || rc=15 ;;
    pmc)
      PA="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
      PB="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
      timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- $B262 \
        > "$O/pmc_fetch.log" 2>&1 &&
      timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- $B262 \
        > "$O/pmc_write.log" 2>&1 &&
      timeout -s KILL 240 rocprofv3 --pmc $PA --output-format csv -d "$O/pmc_a" -o run -- $B262 > "$O/pmc_a.log" 2>&1 &&
      timeout -s KILL 240 rocprofv3 --pmc $PB --output-format csv -d "$O/pmc_b" -o run -- $B262 > "$O/pmc_b.log" 2>&1 &&
      python3 tools/pmc_sq.py "$O/pmc_sq.json" "$O/pmc_a/run_counter_collection.csv" \
        "$O/pmc_b/run_counter_collection.csv" > /dev/null &&
      python3 tools/pmc_traffic.py "$O/pmc_fetch/run_counter_collection.csv" \
        "$O/pmc_write/run_counter_collection.csv" 786432 "$O/pmc_traffic.json" > /dev/null || rc=16 ;;
    intrate)
      make -s -C tools intrate > /dev/null &&
      timeout -k 10 120 tools/intrate > "$O/intrate.txt" 2>&1 &&
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
        --output-format csv -d "$O/pmc_intrate" -o run -- tools/intrate > "$O/pmc_intrate.log" 2>&1 &&
      python3 tools/pmc_sq.py "$O/pmc_intrate.json" "$O/pmc_intrate/run_counter_collection.csv" > /dev/null || rc=23 ;;
    pmccal)
      timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmccal_fetch" -o run -- tools/pmccal \
        > "$O/pmccal_fetch.log" 2>&1 &&
      timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmccal_write" -o run -- tools/pmccal \
        > "$O/pmccal_write.log" 2>&1 || rc=24 ;;
    fpbench) timeout -k 10 180 tools/fpbench > "$O/fpbench.json" 2>&1 || rc=28 ;;
    cabi) timeout -k 10 120 tools/cabi_smoke > "$O/cabi_smoke.txt" 2>&1 || rc=20 ;;
    wvbench) timeout -k 10 120 tools/wvbench > "$O/wvbench.json" 2>&1 || rc=25 ;;
    lat) timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out "$O/latency.json" > "$O/latency.log" 2>&1 || rc=21 ;;
    latsweep)
      timeout -k 10 400 python -u tools/latency_bench.py --reps 5 --sweep 64,256,512,1024,2048 \
        --out "$O/latency_sweep.json" > "$O/latency_sweep.log" 2>&1 || rc=24 ;;
    cfg) timeout -k 10 600 python -u tools/config_bench.py > "$O/config_bench.json" 2> "$O/config_bench.log" || rc=22 ;;
    variant:*)
      V=${step#variant:}
      L=variants/libblsverify_$V.so
      if [ ! -f "$L" ]; then echo "no $L"; rc=30; else
        DRAND_AMD_LIB=$L timeout -k 10 900 $PYT > "$O/pytest_gpu_$V.log" 2>&1 &&
        DRAND_AMD_LIB=$L timeout -k 10 400 python -u bench.py --cpu-per-worker 0 > "$O/bench_$V.json" \
          2> "$O/bench_$V.err" || rc=31
      fi ;;
    vlat:*)
      V=${step#vlat:}
      L=variants/libblsverify_$V.so
      if [ ! -f "$L" ]; then echo "no $L"; rc=30; else
        DRAND_AMD_LIB=$L timeout -k 10 300 python -u tools/latency_bench.py --reps 10 --out "$O/latency_$V.json" \
          > "$O/latency_$V.log" 2>&1 || rc=32
      fi ;;
    ab:*)
      # interleaved same-box A/B: base and each variant, two passes (bench_<name>_<pass>.json)
      IFS=, read -ra VS <<< "${step#ab:}"
      for pass in 1 2; do
        timeout -k 10 400 python -u bench.py --cpu-per-worker 0 > "$O/bench_base_$pass.json" 2> "$O/bench_base_$pass.err" || { rc=33; break; }
        for V in "${VS[@]}"; do
          L=variants/libblsverify_$V.so
          [ -f "$L" ] || { echo "no $L"; rc=30; break 2; }
          DRAND_AMD_LIB=$L timeout -k 10 400 python -u bench.py --cpu-per-worker 0 > "$O/bench_${V}_$pass.json" \
            2> "$O/bench_${V}_$pass.err" || { rc=33; break 2; }
        done
      done ;;
    vbench:*)
      V=${step#vbench:}
      L=variants/libblsverify_$V.so
      if [ ! -f "$L" ]; then echo "no $L"; rc=30; else
        DRAND_AMD_LIB=$L timeout -k 10 400 python -u bench.py --cpu-per-worker 0 > "$O/bench_$V.json" \
          2> "$O/bench_$V.err" || rc=31
      fi ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || { echo "[gpu.sh] step $step failed rc=$rc"; exit $rc; }
done
echo "[gpu.sh] done $(date +%T)"
