#!/bin/bash
# Round 6 on one GPU box: (1) the driver's N = 4 launch rehearsed with every
# rank on device 0 (torch.distributed.run, HIP_VISIBLE_DEVICES=0: the launcher,
# rank plumbing, barrier, max-over-ranks time and parity AND end to end; the
# value is one GPU's rate shared by four ranks); (2) config 5's whole 64M batch
# on one GPU with this round's kernels; (3) one PMC pass (VALU instructions /
# busy, GPU cycles) over a 1M-record unique-key config-5 pass, for the ladder
# kernel's issue utilisation. Each GPU step has its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-r6reh}
mkdir -p $O
HIP_VISIBLE_DEVICES=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 10 --warmup 3 \
  --side-configs 0 --cpu-baseline 0 > $O/rehearse4.json 2> $O/rehearse4.err
rc=$?; head -c 700 $O/rehearse4.json; echo; [ $rc -eq 0 ] || { echo "STOP rehearse4 ($rc)"; tail -5 $O/rehearse4.err; exit $rc; }
timeout -k 10 900 python -u bench.py --config 5 --gpus 1 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
rc=$?; head -c 900 $O/bench_c5.json; echo; [ $rc -eq 0 ] || { echo "STOP c5 ($rc)"; tail -5 $O/bench_c5.err; exit $rc; }
export TMPDIR=/tmp
grp="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
BH_LANES=1 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pmc_c5 -o pmc \
  -- python3 bench.py --config 5 --n-total 1048576 --steps 1 --warmup 0 --cpu-baseline 0 \
  --side-configs 0 > $O/pmc_c5.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { echo "STOP pmc_c5 ($rc)"; exit $rc; }
python3 tools/pmc_summary.py $O/pmc_c5 $O/pmc_c5_summary.json > $O/pmc_c5_summary.txt 2>&1 || echo "summary failed"
grep -E "ktab_ladder" $O/pmc_c5_summary.txt | cut -c1-400
echo DONE
