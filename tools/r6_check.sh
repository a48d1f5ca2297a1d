#!/bin/bash
# Round-6 check of a build: -m gpu, smoke, the driver's default bench line, and
# one PMC pass (SQ_INSTS_VALU + SQ_ACTIVE_INST_VALU + GRBM_GUI_ACTIVE) over the
# one-lane bench, summarised per kernel by tools/pmc_summary.py.
# OUT=<dir under gpurun_out> names the run. Every GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6c}
mkdir -p $O
stop() { echo "STOP after $1 (exit $2)"; exit "$2"; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || stop tests $rc
  timeout -k 10 300 python -u __graft_entry__.py > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log
  [ $rc -eq 0 ] || stop smoke $rc
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 3 ] || stop bench $rc
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'parity', d['parity'], 'kernels', d.get('kernel_ms_per_step'))
print('host_path', d['host_path']['value'], 'e2e', d.get('host_path_e2e', {}).get('value'))
sv=d.get('side_configs',{}).get('single_verify',{})
print('sv', {k:(v.get('p50_us'),v.get('p99_us')) for k,v in sv.items() if isinstance(v,dict) and 'p99_us' in v})
sc=d.get('side_configs',{})
print('c3', sc.get('config3',{}).get('warm'), sc.get('config3',{}).get('cold'))
print('c4', sc.get('config4',{}).get('warm'), sc.get('config4',{}).get('cold'))
print('c5', sc.get('config5_rank',{}).get('hbm_resident_verifies_per_s'))
"
if [ "${PMC:-1}" = 1 ]; then
  grp="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
  tag=$(echo $grp | tr ' ' '_' | cut -c1-40)
  BH_LANES=1 BH_KEYS_FIRST=0 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv \
    -d $O/pmc_$tag -o pmc -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 \
    --hbm-resident 0 --side-configs 0 > $O/pmc_$tag.log 2>&1; rc=$?
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || stop pmc $rc
  python3 tools/pmc_summary.py $O $O/pmc_summary.json > $O/pmc_summary.txt 2>&1 || echo "pmc_summary failed"
  tail -20 $O/pmc_summary.txt
fi
echo DONE
