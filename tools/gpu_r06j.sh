#!/bin/bash
# Round 6 call j: memory-policy A/B of the quad kernel: non-temporal coefficient loads (qnt,
# -DVP8G_QLOAD_NT=1) and the paired pixel stores' cache policy sc1 + nt (aux18) / sc0 + sc1 (aux17)
# against the default (sc1 stores, default-policy loads).
# Libraries: bash tools/build_ab.sh qnt "-DVP8G_QLOAD_NT=1" aux18 "-DVP8G_QPAIR_AUX=18" aux17 "-DVP8G_QPAIR_AUX=17".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06j 0 uhd4,synth,fhd4 webp-decoder_amd/lib/libvp8g.so $L/qnt.so $L/aux18.so $L/aux17.so || exit 1
