#!/bin/bash
# Round 6 call r2: the whole-round A/B (gpu_r06r.sh) repeated on another box with 10 interleaved rounds,
# against the final round-6 build.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
AB_ROUNDS=10 bash tools/gpu_round.sh ab r06r2 0 uhd4,synth,fhd4 $L/r5final.so webp-decoder_amd/lib/libvp8g.so || exit 1
