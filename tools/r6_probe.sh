#!/bin/bash
# Round-6 probes (one gpurun call): the single-Verify tail at 64 / 256 callers
# alone and right after a 256-thread CPU burst (the order bench.py runs them
# in), with csp_load's own CPU time; the packer's pass times at 1 / 8 / 15
# threads with and without key de-duplication (CPU only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6
cat /sys/fs/cgroup/cpu.max > gpurun_out/r6/cpu_max.txt 2>&1
cat /sys/fs/cgroup/cpu.stat > gpurun_out/r6/cpu_stat0.txt 2>&1
timeout -k 10 300 python -u tools/sv_tail.py 64 256 > gpurun_out/r6/sv_alone.json 2> gpurun_out/r6/sv_alone.err || { echo "STOP sv_alone"; exit 1; }
cat gpurun_out/r6/sv_alone.json
timeout -k 10 300 python -u -c "
import sys; sys.path.insert(0, '.')
import bench
print(bench.config1_measure(1, gpu=False))
" > gpurun_out/r6/burn.log 2>&1 || { echo "STOP burn"; exit 1; }
timeout -k 10 300 python -u tools/sv_tail.py 64 256 > gpurun_out/r6/sv_after.json 2> gpurun_out/r6/sv_after.err || { echo "STOP sv_after"; exit 1; }
cat gpurun_out/r6/sv_after.json
timeout -k 10 300 python -u tools/pack_bench.py 1 8 15 > gpurun_out/r6/pack.json 2> gpurun_out/r6/pack.err || { echo "STOP pack"; exit 1; }
cat gpurun_out/r6/pack.json
cat /sys/fs/cgroup/cpu.stat > gpurun_out/r6/cpu_stat1.txt 2>&1
echo DONE
