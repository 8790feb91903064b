#!/bin/bash
# Round 6 call m: GPU tests on the early-publish default (VP8G_PUB_AT=1), then an A/B against the
# end-of-step publish (pub0) and the before-loop-filter publish (pub2).
# Libraries: bash tools/build_ab.sh pub0 "-DVP8G_PUB_AT=0" pub2 "-DVP8G_PUB_AT=2".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06m 1 synth,uhd4,fhd4 $L/pub0.so webp-decoder_amd/lib/libvp8g.so $L/pub2.so || exit 1
