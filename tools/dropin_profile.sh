#!/bin/bash
# Per-call latency of the drop-in entry point (tools/dropin_latency.py), then the same calls under
# rocprofv3 kernel + memory-copy tracing for the H2D / kernel / D2H split (no counters).
#   bash tools/dropin_profile.sh <tag>   -> gpurun_out/dropin_<tag>/
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/dropin_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 200 python3 tools/dropin_latency.py 20 > $OUT/latency.json 2> $OUT/latency.err || { echo "latency failed rc=$?"; exit 1; }
cat $OUT/latency.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/tools/dropin_latency.py 20 > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
echo dropin_done
