#!/bin/bash
# Round 6 call bp2: B_PRED's register hand-off (VP8G_BP_REG, §3.2) for the three/four-B_PRED path only
# (bp2, bit 1), the compact path keeping its LDS round trips -- r06h measured both paths and the compact
# path alone, not this one -- against the build default (off).
# Library: bash tools/build_ab.sh bp2 "-DVP8G_BP_REG=2".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06bp2 0 synth,uhd4,fhd4 webp-decoder_amd/lib/libvp8g.so $L/bp2.so || exit 1
