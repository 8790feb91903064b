#!/bin/bash
# Round 6 call i: the tail's price (diag abl32: only the first 64 of a CU's 68 units; abl47: that and the
# four phase ablations of abl15) and the stamps of the B_PRED register hand-off (VP8G_BP_REG=3) beside
# the default stamps build, on uhd4 and synth.  Timing only: ablated outputs are wrong by construction.
# Libraries: make diag webp-decoder_amd/lib/diag/libvp8g_abl47.so;
#            bash tools/build_ab.sh stamps_bpr3 "-DVP8G_STAMPS -DVP8G_BP_REG=3".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/diag_r06i
mkdir -p $O
QUIET="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
D=webp-decoder_amd/lib/diag
for wl in uhd4 synth; do
  for v in $D/libvp8g_stamps.so webp-decoder_amd/lib/ab/stamps_bpr3.so $D/libvp8g_abl32.so $D/libvp8g_abl15.so $D/libvp8g_abl47.so webp-decoder_amd/lib/libvp8g.so; do
    n=$(basename $v .so)
    VP8G_LIB=$R/$v timeout -k 10 200 python3 bench.py $QUIET --workload $wl --steps 10 --warmup 2 > $O/${n}_$wl.json 2> $O/${n}_$wl.err || { echo "$n $wl failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$wl.json')); print('$wl $n', d['ms_per_step'], d.get('stamps', ''))"
  done
done
echo diag_done
