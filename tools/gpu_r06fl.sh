#!/bin/bash
# Round 6 call fl: timing probe -- the loop filter run after the flush instead of before it (diag abl64:
# the same instruction stream, output wrong by construction), against the product build: what
# overlapping the stores with the filter's arithmetic would be worth.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_round.sh ab r06fl 0 uhd4,synth,fhd4 webp-decoder_amd/lib/libvp8g.so webp-decoder_amd/lib/diag/libvp8g_abl64.so || exit 1
