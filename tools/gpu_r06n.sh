#!/bin/bash
# Round 6 call n: the publish point and the 24-bit multiplies: pub0 (end-of-step publish), pub1only
# (after the prefetch issue, before the multiply fix), pub1m (after the prefetch issue, with it), and
# the build default (before the loop filter, with it).
# Libraries: pub0 = build_ab "-DVP8G_PUB_AT=0" (previous source), pub1only = build_ab "-DVP8G_PUB_AT=1"
# at e09e22b, pub1m = build_ab "-DVP8G_PUB_AT=1".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06n 0 synth,uhd4,fhd4 $L/pub0.so $L/pub1only.so $L/pub1m.so webp-decoder_amd/lib/libvp8g.so || exit 1
