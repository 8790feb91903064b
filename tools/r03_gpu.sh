#!/bin/bash
# Round-3 kernel-experiment call: GPU tests with the chain kernel forced on (VP8G_CHAIN=-1), an
# in-process A/B (tools/ab_inproc.py) of the shipped library against ab/*.so builds on uhd4 / fhd4 /
# synth, then the microbenchmarks (tools/ubench/valu_rates2, lf_packed).  Stops at the first failure.
#   bash tools/r03_gpu.sh <tag> <ab libs...>      (tag "-": skip the tests)
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
if [ "$TAG" != "-" ]; then
  VP8G_CHAIN=-1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/t_$TAG.log 2>&1
  rc=$?; tail -4 gpurun_out/t_$TAG.log
  [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
fi
for wl in uhd4 fhd4 synth; do
  timeout -k 10 300 python -u tools/ab_inproc.py --workload $wl --rounds 4 --steps 6 webp-decoder_amd/lib/libvp8g.so "$@" > gpurun_out/ab_${TAG}_$wl.log 2>&1
  rc=$?; echo "== $wl"; grep '^{' gpurun_out/ab_${TAG}_$wl.log
  [ $rc -eq 0 ] || { echo "ab rc=$rc"; tail -5 gpurun_out/ab_${TAG}_$wl.log; exit $rc; }
done
timeout -k 10 200 tools/ubench/valu_rates2 > gpurun_out/valu_rates2_$TAG.txt 2>&1 || { echo "valu_rates2 rc=$?"; exit 1; }
timeout -k 10 120 tools/ubench/lf_packed > gpurun_out/lf_packed_$TAG.txt 2>&1; echo "lf_packed rc=$?"; cat gpurun_out/lf_packed_$TAG.txt
echo r03_done
