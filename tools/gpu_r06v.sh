#!/bin/bash
# Round 6 call v: the final build's product timing beside its tail and skeleton ablations (diag
# abl32: the first 64 of a CU's 68 units; abl15: no loop filter / B_PRED / pixel stores / dependency
# wait; abl47: both) and the other single-phase ablations, on one box, uhd4 and synth.  Timing only.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/diag_r06v
mkdir -p $O
QUIET="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
D=webp-decoder_amd/lib/diag
for wl in uhd4 synth; do
  for v in webp-decoder_amd/lib/libvp8g.so $D/libvp8g_abl1.so $D/libvp8g_abl2.so $D/libvp8g_abl4.so $D/libvp8g_abl8.so $D/libvp8g_abl32.so $D/libvp8g_abl15.so $D/libvp8g_abl47.so; do
    n=$(basename $v .so)
    VP8G_LIB=$R/$v timeout -k 10 200 python3 bench.py $QUIET --workload $wl --steps 10 --warmup 2 > $O/${n}_$wl.json 2> $O/${n}_$wl.err || { echo "$n $wl failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$wl.json')); print('$wl $n', d['ms_per_step'])"
  done
done
echo diag_done
