#!/bin/bash
# Round 6: the packer's workers on the GPU's NUMA node (BH_PACK_NUMA, default
# on) against the inherited placement (0), unpinned process, two passes each;
# then the staged BatchVerify GPU tests. Each step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-numa2}
mkdir -p $O
for pass in 1 2; do
  for m in 1 0; do
    BH_PACK_NUMA=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 \
      --side-configs 0 > $O/bench_numa${m}_p$pass.json 2> $O/bench_numa${m}_p$pass.err
    rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "STOP numa$m ($rc)"; tail -3 $O/bench_numa${m}_p$pass.err; exit $rc; }
    python3 -c "
import json; d=json.loads(open('$O/bench_numa${m}_p$pass.json').read().strip().splitlines()[-1]); e=d['host_path_e2e']; h=d['host_path']
print('numa $m pass $pass value', round(d['value']/1e6,1), 'host', round(h['value']/1e6,1), h['pcie_frac'], 'e2e', round(e['value']/1e6,1), e['pcie_frac'], e['per_batch_ms'], 'submit', e['submit_ms_per_batch'], 'wait', e['wait_ms_per_batch'])"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_staged.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_staged.log 2>&1
rc=$?; tail -2 $O/pytest_staged.log; exit $rc
