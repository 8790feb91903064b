#!/bin/bash
# Round 6 call b: GPU tests on the default build, A/B of the loop-filter mask / B_PRED shift variants,
# then the synth profile and stamps (tools/gpu_r06_prof.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06b 1 uhd4,synth,fhd4 $L/v_base.so $L/v_bps.so $L/v_lfm.so $L/v_both.so || exit 1
bash tools/gpu_r06_prof.sh r06s || exit 1
