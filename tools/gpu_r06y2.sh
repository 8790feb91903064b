#!/bin/bash
# Round 6 call y2: the dependency-poll sleep sweep (gpu_r06x2.sh), then quarter 3's context stores issued
# before the pixel stores with the publish waiting only for them (cf, -DVP8G_CTX_FIRST=1), and that with
# the prefetch + publish right after the dequantisation (cfpe, + -DVP8G_PREF_EARLY=1).
# Libraries: bash tools/build_ab.sh cf "-DVP8G_CTX_FIRST=1" cfpe "-DVP8G_CTX_FIRST=1 -DVP8G_PREF_EARLY=1".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_r06x2.sh || exit 1
bash tools/gpu_round.sh ab r06y2 0 synth,uhd4,fhd4 webp-decoder_amd/lib/libvp8g.so $L/cf.so $L/cfpe.so || exit 1
