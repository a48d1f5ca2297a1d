#!/bin/bash
# single-verify A/B: BH_SMALL_COPY_STREAM x BH_D2H_COPY
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sv
for v in "cs1_k:BH_SMALL_COPY_STREAM=1" "cs0_k:BH_SMALL_COPY_STREAM=0" "cs0_c:BH_SMALL_COPY_STREAM=0 BH_D2H_COPY=1"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/sv/$name.json 2> gpurun_out/sv/$name.err || { echo "STOP $name"; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/sv/$name.json').read().strip().splitlines()[-1]);sv=d['side_configs']['single_verify']
print('$name', {k:(v['p50_us'],v['p99_us'],round(v['verifies_per_s'])) for k,v in sv.items() if isinstance(v,dict) and 'p50_us' in v})"
done
