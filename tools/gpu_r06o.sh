#!/bin/bash
# Round 6 call o: the row above's context loaded at the top of its own step after a wait for progress
# >= t + 8 (ctxe, -DVP8G_CTX_EARLY=1) against the build default (loaded one step ahead, progress >= t + 9).
# Library: bash tools/build_ab.sh ctxe "-DVP8G_CTX_EARLY=1".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06o 0 synth,uhd4,fhd4 webp-decoder_amd/lib/libvp8g.so $L/ctxe.so || exit 1
