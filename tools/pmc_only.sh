set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $grp | tr ' ' '_' | cut -c1-40)
  BH_LANES=1 BH_KEYS_FIRST=0 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv \
    -d gpurun_out/pmc_$tag -o pmc -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 \
    --hbm-resident 0 --side-configs 0 > gpurun_out/pmc_$tag.log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "STOP pmc $grp $rc"; exit $rc; }
done
python3 tools/pmc_summary.py gpurun_out gpurun_out/pmc_summary.json --traffic \
  --workload=config2:n1048576 --source=profiles/r06/${PROF_TAG:-pmc} \
  --traffic-out=gpurun_out/traffic.json > gpurun_out/pmc_summary.txt 2>&1 || echo "pmc_summary failed"
echo DONE
