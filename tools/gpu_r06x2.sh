#!/bin/bash
# Round 6 call x2: the dependency poll's s_sleep length (VP8G_WAIT_SLEEP, default 1): 2, 3, 6, 12.
# Libraries: bash tools/build_ab.sh ws2 "-DVP8G_WAIT_SLEEP=2" ws3 "-DVP8G_WAIT_SLEEP=3" ws6 "-DVP8G_WAIT_SLEEP=6" ws12 "-DVP8G_WAIT_SLEEP=12".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06x2 0 synth,uhd4,fhd4 webp-decoder_amd/lib/libvp8g.so $L/ws2.so $L/ws3.so $L/ws6.so $L/ws12.so || exit 1
