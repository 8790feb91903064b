#!/bin/bash
# Round 6 call cl: the chain layouts re-checked on the round-6 quad kernel: nsil = no mirror split,
# two-frame interleave wherever it fits; nspl = no mirror split; il0 = no interleave; spl1 = the mirror
# split wherever it fits; against the build default (host picks: uhd4 mirror split, synth / fhd4
# interleave).
# Libraries: bash tools/build_ab.sh nsil "-DVP8G_SPLITCHAIN_DEFAULT=0 -DVP8G_CHAIN_IL_DEFAULT=1"
#   nspl "-DVP8G_SPLITCHAIN_DEFAULT=0" il0 "-DVP8G_CHAIN_IL_DEFAULT=0" spl1 "-DVP8G_SPLITCHAIN_DEFAULT=1".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06cl 0 uhd4,synth,fhd4 webp-decoder_amd/lib/libvp8g.so $L/nsil.so $L/nspl.so $L/il0.so $L/spl1.so || exit 1
