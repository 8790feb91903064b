#!/bin/bash
# Round 6 call w: the next step's prefetch (and the progress publish after it) issued right after the
# dequantisation (pfe, -DVP8G_PREF_EARLY=1), and the dependency poll's s_sleep (ws0 / ws3, default 1),
# against the build default.
# Libraries: bash tools/build_ab.sh pfe "-DVP8G_PREF_EARLY=1" ws0 "-DVP8G_WAIT_SLEEP=0" ws3 "-DVP8G_WAIT_SLEEP=3".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06w 0 synth,uhd4,fhd4 webp-decoder_amd/lib/libvp8g.so $L/pfe.so $L/ws0.so $L/ws3.so || exit 1
