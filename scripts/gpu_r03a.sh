# r03 first call: box facts (CPU share for cpu_baseline), DPP/permlane semantics probe for the latency
# engine, and per-kernel SQ/GRBM counters of the current tree (occupancy, VALU busy).
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03a
O=gpurun_out/r03a
{
  echo "nproc: $(nproc)"
  python3 -c 'import os; print("affinity:", len(os.sched_getaffinity(0)), "cpu_count:", os.cpu_count())'
  grep -m1 "model name" /proc/cpuinfo
  grep -c ^processor /proc/cpuinfo
  echo "OMP_NUM_THREADS=$OMP_NUM_THREADS MAX_JOBS=$MAX_JOBS"
  cat /sys/fs/cgroup/cpu.max 2>/dev/null
  free -g | head -2
} > $O/box.txt 2>&1
timeout -k 10 60 ./tools/dpp_probe > $O/dpp_probe.txt 2>&1 || exit 11
timeout -s KILL 60 rocprofv3 -L > $O/counters_all.txt 2>&1 || true
grep -oE "\b(SQ|GRBM)_[A-Z0-9_]+" $O/counters_all.txt | sort -u > $O/counters.txt || true
pick() {  # keep only counters the box lists
  local out=""
  for c in "$@"; do grep -qx "$c" $O/counters.txt && out="$out $c"; done
  echo $out
}
PA=$(pick SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE)
PB=$(pick SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT)
echo "pass A: $PA" > $O/passes.txt
echo "pass B: $PB" >> $O/passes.txt
timeout -s KILL 240 rocprofv3 --pmc $PA --output-format csv -d $O/pmc_a -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > $O/pmc_a.log 2>&1 || exit 12
timeout -s KILL 240 rocprofv3 --pmc $PB --output-format csv -d $O/pmc_b -o run -- python3 -u bench.py --n 262144 --steps 1 --warmup 0 --cpu-per-worker 0 > $O/pmc_b.log 2>&1 || exit 13
python3 tools/pmc_sq.py $O/pmc_sq.json $O/pmc_a/run_counter_collection.csv $O/pmc_b/run_counter_collection.csv > /dev/null || exit 14
echo done
