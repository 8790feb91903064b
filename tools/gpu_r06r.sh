#!/bin/bash
# Round 6 call r: the whole round in one process -- the round-5 final build (r5final: webp-decoder_amd/csrc,
# include and host of commit 2472ed3 built with tools/build_ab.sh's flags, linked to this tree's
# libvp8host.so, unchanged since) against the round-6 build, on every bench workload.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06r 0 uhd4,synth,fhd4,uhd4_yuv $L/r5final.so webp-decoder_amd/lib/libvp8g.so || exit 1
