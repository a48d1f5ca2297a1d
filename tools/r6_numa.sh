#!/bin/bash
# Round 6: host NUMA placement of the staged BatchVerify / host path. Prints the
# GPU's NUMA node, then runs the default bench line (no side configs) with the
# whole process confined to each socket's CPUs (taskset, before any GPU call). Each run has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-numa}
mkdir -p $O
for d in /sys/class/drm/card*/device; do
  [ -f $d/numa_node ] && echo "$d numa_node=$(cat $d/numa_node) vendor=$(cat $d/vendor 2>/dev/null)"
done > $O/gpu_numa.txt 2>&1
cat $O/gpu_numa.txt
for node in 0 1; do
  cpus=$(cat /sys/devices/system/node/node$node/cpulist)
  for m in 0; do
    BH_PACK_SPREAD=$m timeout -k 10 300 taskset -c $cpus python bench.py --steps 20 --warmup 5 \
      --cpu-baseline 0 --side-configs 0 > $O/bench_n${node}_m$m.json 2> $O/bench_n${node}_m$m.err
    rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "STOP n$node m$m ($rc)"; tail -3 $O/bench_n${node}_m$m.err; exit $rc; }
    python3 -c "
import json; d=json.loads(open('$O/bench_n${node}_m$m.json').read().strip().splitlines()[-1]); e=d['host_path_e2e']; h=d['host_path']
print('node $node spread $m value', round(d['value']/1e6,1), 'host', round(h['value']/1e6,1), h['pcie_frac'], h.get('h2d_gbps_pinned'), 'e2e', round(e['value']/1e6,1), e['pcie_frac'], e['per_batch_ms'], 'submit', e['submit_ms_per_batch'], 'wait', e['wait_ms_per_batch'])"
  done
done
echo DONE
