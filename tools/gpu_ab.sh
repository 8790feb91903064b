#!/bin/bash
# One GPU call for a kernel change: the GPU test suite, then an in-process A/B of builds on the uhd4
# and fhd4 batches (tools/ab_inproc.py).  Stops at the first failing step (never retries a GPU step).
#   bash tools/gpu_ab.sh <tag> <lib.so> [<lib.so> ...]      (tag "-": skip the tests)
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
if [ "$TAG" != "-" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/t_$TAG.log 2>&1
  rc=$?; tail -4 gpurun_out/t_$TAG.log
  [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
fi
for wl in uhd4 fhd4; do
  timeout -k 10 300 python -u tools/ab_inproc.py --workload $wl --rounds 4 --steps 6 "$@" > gpurun_out/ab_${TAG}_$wl.log 2>&1
  rc=$?; echo "== $wl"; grep '^{' gpurun_out/ab_${TAG}_$wl.log
  [ $rc -eq 0 ] || { echo "ab rc=$rc"; tail -5 gpurun_out/ab_${TAG}_$wl.log; exit $rc; }
done
