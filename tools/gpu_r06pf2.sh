#!/bin/bash
# Round 6 call pf2: the coefficient prefetch two steps ahead (pf2, -DVP8G_PREF2=1: a second 17-VGPR
# set rotated each step, no spills in the step loop) against the build default (one step ahead).
# Library: bash tools/build_ab.sh pf2 "-DVP8G_PREF2=1".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06pf2 0 uhd4,synth,fhd4 webp-decoder_amd/lib/libvp8g.so $L/pf2.so || exit 1
