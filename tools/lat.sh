#!/bin/bash
# Latency benches (configs 3 and 4); each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in 3 4; do
  timeout -k 10 300 python bench.py --config $c --steps ${LAT_STEPS:-50} --warmup 3 > gpurun_out/lat$c.json 2> gpurun_out/lat$c.err
  rc=$?; cat gpurun_out/lat$c.json; tail -3 gpurun_out/lat$c.err
  case $rc in 0|3) ;; *) echo "STOP after lat$c (exit $rc)"; exit $rc ;; esac
done
