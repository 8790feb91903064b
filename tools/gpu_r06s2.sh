#!/bin/bash
# Round 6 call s2: the progress word read ahead of the side info and the wait + context load after it
# (ce2, -DVP8G_CTX_EARLY=2), and role 1's luma store skipped when no lane has a piece (y1s,
# -DVP8G_Y1_SKIP=1), against the build default.
# Libraries: bash tools/build_ab.sh ce2 "-DVP8G_CTX_EARLY=2" y1s "-DVP8G_Y1_SKIP=1".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06s2 0 synth,uhd4,fhd4 webp-decoder_amd/lib/libvp8g.so $L/ce2.so $L/y1s.so || exit 1
