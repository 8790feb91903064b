#!/bin/bash
# Round 6 call p: GPU tests with the early context load as the build default (VP8G_CTX_EARLY=1), then
# an A/B against the one-step-ahead load (ctx0) on a second box.
# Library: bash tools/build_ab.sh ctx0 "-DVP8G_CTX_EARLY=0".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06p 1 synth,uhd4,fhd4 $L/ctx0.so webp-decoder_amd/lib/libvp8g.so || exit 1
