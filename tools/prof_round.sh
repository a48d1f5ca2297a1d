#!/bin/bash
# One profiling session for the committed build (run through gpurun):
#   1. rocprofv3 --kernel-trace --stats of the driver's bench command, and
#      tools/prof_check.py tying the dominant kernel's dispatches to the line;
#   2. rocprofv3 --pmc passes, one counter group each (FETCH_SIZE, WRITE_SIZE,
#      SQ_INSTS_VALU + GRBM_GUI_ACTIVE) on the one-lane bench (BH_KEYS_FIRST=0:
#      one build launch per pass, as the resident passes run), summarised by
#      tools/pmc_summary.py into gpurun_out/pmc_summary.json and, stamped with
#      the kernel-source hash, gpurun_out/traffic.json;
#   3. the driver's bench command once more, plain (the line the counters join).
# Every GPU step has its own time limit; a fault / abort / timeout stops here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
stop() { echo "STOP after $1 (exit $2)"; exit "$2"; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_bench.json 2> gpurun_out/prof.log
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || stop prof $rc
python3 tools/prof_check.py gpurun_out/prof/run_kernel_trace.csv gpurun_out/prof_bench.json \
  gpurun_out/prof_check.json; cat gpurun_out/prof_check.json | head -30
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $grp | tr ' ' '_' | cut -c1-40)
  BH_LANES=1 BH_KEYS_FIRST=0 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv \
    -d gpurun_out/pmc_$tag -o pmc -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 \
    --hbm-resident 0 --side-configs 0 > gpurun_out/pmc_$tag.log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || stop "pmc $grp" $rc
done
python3 tools/pmc_summary.py gpurun_out gpurun_out/pmc_summary.json --traffic \
  --workload=config2:n1048576 --source=profiles/${PROF_TAG:-r06} \
  --traffic-out=gpurun_out/traffic.json > gpurun_out/pmc_summary.txt 2>&1 || echo "pmc_summary failed"
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json \
  2> gpurun_out/bench.err; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || stop bench $rc
echo DONE
