#!/bin/bash
# Round 6 call h: B_PRED register hand-off A/B (VP8G_BP_REG): old LDS wavefront (bpr0), compact path
# only (bpr1), both paths (the build default), both with the permlane16_swap halves read the other way
# round (bpr3x; a semantics check: its digests must fail if the default's pass).
# Libraries: bash tools/build_ab.sh bpr0 "-DVP8G_BP_REG=0" bpr1 "-DVP8G_BP_REG=1" bpr3x "-DVP8G_BP_SWAPX=1".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06h 0 synth,uhd4,fhd4 $L/bpr0.so webp-decoder_amd/lib/libvp8g.so $L/bpr1.so $L/bpr3x.so || exit 1
