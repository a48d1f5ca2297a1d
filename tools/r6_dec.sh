#!/bin/bash
# Config 3's host half on the box: bh_fabric_block_preverify in decode-only
# mode (no device work) at 1 / 2 / 4 / 8 decode threads, with the library's
# BH_FAB_TIMING phase lines. CPU only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-r6dec}
mkdir -p $O
for t in 1 2 4 8; do
  BH_FAB_TIMING=1 BH_DECODE_THREADS=$t timeout -k 10 120 python3 tools/dec_probe.py > $O/dec_t$t.txt 2> $O/dec_t$t.err || { echo "STOP dec $t"; exit 1; }
  cat $O/dec_t$t.txt; tail -1 $O/dec_t$t.err
done
echo DONE
