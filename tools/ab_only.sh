#!/bin/bash
# In-process A/B only (no tests): the shipped library against ab/*.so builds on the given workloads.
#   bash tools/ab_only.sh <tag> "<workloads>" <lib.so> ...
set -u
TAG=$1; WLS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for wl in $WLS; do
  timeout -k 10 300 python -u tools/ab_inproc.py --workload $wl --rounds 4 --steps 6 webp-decoder_amd/lib/libvp8g.so "$@" > gpurun_out/ab_${TAG}_$wl.log 2>&1
  rc=$?; echo "== $wl"; grep '^{' gpurun_out/ab_${TAG}_$wl.log
  [ $rc -eq 0 ] || { echo "ab rc=$rc"; tail -5 gpurun_out/ab_${TAG}_$wl.log; exit $rc; }
done
echo ab_done
