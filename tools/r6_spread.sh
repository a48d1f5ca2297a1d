#!/bin/bash
# Round 6: packer worker placement A/B (BH_PACK_SPREAD: pack.h as of commit
# 62712ff; the switch was measured and removed) on one GPU box.
# (1) tools/pack_bench.py (the packer alone, CPU) at 8 and 15 threads for each
# mode; (2) the default bench line's host_path_e2e for each mode, two passes.
# Every step has its own limit; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-spread}
mkdir -p $O
(nproc; cat /sys/fs/cgroup/cpu.max; lscpu | grep -E "Model name|NUMA|L3") > $O/host.txt 2>&1
for m in 0 1 2; do
  BH_PACK_SPREAD=$m timeout -k 10 300 python -u tools/pack_bench.py 8 15 > $O/pack_m$m.jsonl 2> $O/pack_m$m.err
  rc=$?; echo "pack mode $m rc=$rc"; cat $O/pack_m$m.jsonl; [ $rc -eq 0 ] || exit $rc
done
for pass in 1 2; do
  for m in 0 1 2; do
    BH_PACK_SPREAD=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline 0 \
      --side-configs 0 > $O/bench_m${m}_p$pass.json 2> $O/bench_m${m}_p$pass.err
    rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "STOP bench m$m ($rc)"; exit $rc; }
    python3 -c "
import json; d=json.loads(open('$O/bench_m${m}_p$pass.json').read().strip().splitlines()[-1]); e=d['host_path_e2e']
print('mode $m pass $pass value', round(d['value']/1e6,1), 'e2e', round(e['value']/1e6,1), e['pcie_frac'], 'pack', e['per_batch_ms'], e['pack'].get('pass_b_ms'))"
  done
done
echo DONE
