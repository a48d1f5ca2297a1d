#!/bin/bash
# Kernel timelines of the latency configs (3: one block, 4: one BDLS round),
# cold and warm calls, from rocprofv3 --kernel-trace; tools/lat_trace.py
# splits them per call. Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6lat}
mkdir -p $O
for c in ${CONFIGS:-4 3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c$c -o run \
    -- python3 bench.py --config $c --steps ${LAT_STEPS:-20} --warmup 3 > $O/c$c.json 2> $O/c$c.err
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "STOP c$c ($rc)"; exit $rc; }
  python3 tools/lat_trace.py $O/c$c/run_kernel_trace.csv ${LAT_CALLS:-45} > $O/c${c}_trace.json || echo "trace failed"
  head -c 600 $O/c$c.json; echo
done
echo DONE
