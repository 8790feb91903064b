#!/bin/bash
# Round 6 call q: the compiler's scheduler on the round-6 build: iterative-ilp / -minreg / -maxocc
# strategies, schedule-metric bias 50, no memory-op clustering, no unclustered high-RP reschedule.
# Libraries: bash tools/build_ab.sh sIilp "-mllvm -amdgpu-sched-strategy=iterative-ilp" sImr "... =iterative-minreg"
#   sImo "... =iterative-maxocc" sB50 "-mllvm -amdgpu-schedule-metric-bias=50" sNC "-mllvm -misched-cluster=0"
#   sDU "-mllvm -amdgpu-disable-unclustered-high-rp-reschedule".
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06q 0 uhd4,synth webp-decoder_amd/lib/libvp8g.so $L/sIilp.so $L/sImr.so $L/sImo.so $L/sB50.so $L/sNC.so $L/sDU.so || exit 1
