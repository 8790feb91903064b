#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel-trace stats of the default bench workload, then
# the HBM-traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs; never combined with
# tracing domains).  Usage (from the repo root, on the box): bash tools/profile_round.sh <tag> [workload]
# Outputs under gpurun_out/prof_<tag>/; tools/traffic_summary.py turns them into profiles/.
set -u
TAG=$1
WL=${2:-uhd4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
  python3 $R/bench.py --workload $WL --no-cpu-baseline --e2e-frames 0 --extra none --encode none --steps 10 --warmup 3 > $OUT/trace_bench.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o pmc -- \
    python3 $R/bench.py --workload $WL --no-cpu-baseline --e2e-frames 0 --extra none --encode none --steps 2 --warmup 1 > $OUT/pmc_$c.log 2>&1 || { echo "pmc $c failed rc=$?"; exit 1; }
done
echo profile_done
