#!/bin/bash
# Round 6 call k: phase-priority re-sweep on the round-6 build (the table was tuned on round 5's):
# p1 residual 1 (VP8G_PRIO_TABLE=1,2,2,3,3,1,2,2), p2 loop-filter arithmetic 0 (VP8G_PRIO_LF=1,0),
# p3 B_PRED 2 (0,2,2,3,2,1,2,2), p4 flush 1 (0,2,2,3,3,1,1,2), p5 loop-filter gather 2 (VP8G_PRIO_LF=2,1).
# Libraries: bash tools/build_ab.sh p1 "-DVP8G_PRIO_TABLE=1,2,2,3,3,1,2,2" p2 "-DVP8G_PRIO_LF=1,0" ... (as above).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06k 0 uhd4,synth webp-decoder_amd/lib/libvp8g.so $L/p1.so $L/p2.so $L/p3.so $L/p4.so $L/p5.so || exit 1
# stamps of the build with the pixel stores dropped by the range check (st_abl4: -DVP8G_STAMPS -DVP8G_ABLATE=4):
# does the top-of-step prefetch wait go with the stores' memory side?
O=gpurun_out/diag_r06k
mkdir -p $O
QUIET="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
for wl in uhd4 synth; do
  for v in webp-decoder_amd/lib/diag/libvp8g_stamps.so $L/st_abl4.so; do
    n=$(basename $v .so)
    VP8G_LIB=$R/$v timeout -k 10 200 python3 bench.py $QUIET --workload $wl --steps 10 --warmup 2 > $O/${n}_$wl.json 2> $O/${n}_$wl.err || { echo "$n $wl failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${n}_$wl.json')); print('$wl $n', d['ms_per_step'], d.get('stamps', ''))"
  done
done
echo diag_done
