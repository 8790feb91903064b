#!/bin/bash
# Microbenchmarks behind DESIGN.md §5: VALU issue costs (valu_rates) and the FETCH_SIZE calibration
# for the kernel's 32-B-per-lane loads (fetch_calib, one PMC pass per mode).  On the box:
#   bash tools/ubench_round.sh <tag>   -> gpurun_out/ubench_<tag>/
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ubench_$TAG
mkdir -p $OUT
timeout -k 10 120 $R/tools/ubench/valu_rates > $OUT/valu_rates.txt 2>&1 || { echo "valu_rates failed rc=$?"; exit 1; }
export TMPDIR=/tmp
cd /tmp
for m in 0 1; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch$m -o pmc -- $R/tools/ubench/fetch_calib $m > $OUT/fetch$m.log 2>&1 || { echo "fetch pass $m failed rc=$?"; exit 1; }
done
echo ubench_done
