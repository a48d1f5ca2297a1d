#!/bin/bash
# A/B sweep of run-time knobs (lanes, build stagger) and library variants on the
# default config-2 bench line: one JSON per case under gpurun_out/sweep/.
# SWEEP="name:ENV=1+ENV2=2[:lib] ..."  (lib: an exp/ variant, default the main .so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
for pass in $(seq ${PASSES:-1}); do
  for c in ${SWEEP}; do
    name=${c%%:*}; rest=${c#*:}; envs=${rest%%:*}; lib=""; [ "$rest" != "$envs" ] && lib=${rest#*:}
    e=$(echo "$envs" | tr '+' ' ')
    [ -n "$lib" ] && e="$e BDLS_HIP_LIB=$PWD/exp/libbdlship_$lib.so"
    env $e timeout -k 10 300 python bench.py --steps ${STEPS_N:-20} --warmup 5 --cpu-baseline 0 --side-configs 0 > gpurun_out/sweep/${name}_p$pass.json 2> gpurun_out/sweep/${name}_p$pass.err; rc=$?
    echo "$name p$pass rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/sweep/${name}_p$pass.json'));h=d.get('host_path') or {};print(round(d['value']/1e6,1), d['parity'], 'host', round(h.get('value',0)/1e6,1), h.get('pcie_frac'))" 2>/dev/null)"
    case $rc in 0|3) ;; *) echo "STOP"; exit $rc ;; esac
  done
done
echo DONE
