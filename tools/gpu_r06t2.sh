#!/bin/bash
# Round 6 call t2: GPU tests with the read-ahead progress poll as the build default (VP8G_CTX_EARLY=2),
# then an A/B against VP8G_CTX_EARLY=1 (ce1) on a second box.
# Library: bash tools/build_ab.sh ce1 "-DVP8G_CTX_EARLY=1".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06t2 1 synth,uhd4,fhd4 $L/ce1.so webp-decoder_amd/lib/libvp8g.so || exit 1
