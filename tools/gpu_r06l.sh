#!/bin/bash
# Round 6 call l: progress published part of a step earlier (VP8G_PUB_AT=1: after the next step's
# prefetch issue, vmcnt(5); =2: before the loop filter, vmcnt(6)) against the end-of-step publish.
# Libraries: bash tools/build_ab.sh pub1 "-DVP8G_PUB_AT=1" pub2 "-DVP8G_PUB_AT=2".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06l 0 uhd4,synth,fhd4 webp-decoder_amd/lib/libvp8g.so $L/pub1.so $L/pub2.so || exit 1
