#!/bin/bash
# HIP API + kernel + memory-copy trace of the latency configs (no counters),
# to attribute the host-side gaps of a warm call. One GPU step per config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6api}
mkdir -p $O
for c in ${CONFIGS:-4 3}; do
  timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv \
    -d $O/c$c -o run -- python3 bench.py --config $c --steps ${LAT_STEPS:-8} --warmup 2 \
    > $O/c$c.json 2> $O/c$c.err
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "STOP c$c ($rc)"; exit $rc; }
  ls $O/c$c
done
echo DONE
