#!/bin/bash
# Round 6 call sch: three more compiler scheduler settings on the final build (r06q tried the iterative
# strategies, metric bias, clustering): trk = -mllvm -amdgpu-use-amdgpu-trackers=1 (the GCN register
# pressure trackers), mxilp = -mllvm -amdgpu-sched-strategy=max-ilp, mmc = -amdgpu-sched-strategy=
# max-memory-clause, against the build default.
# Libraries: bash tools/build_ab.sh trk "-mllvm -amdgpu-use-amdgpu-trackers=1" \
#   mxilp "-mllvm -amdgpu-sched-strategy=max-ilp" mmc "-mllvm -amdgpu-sched-strategy=max-memory-clause"
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
L=webp-decoder_amd/lib/ab
bash tools/gpu_round.sh ab r06sch 0 uhd4,synth webp-decoder_amd/lib/libvp8g.so $L/trk.so $L/mxilp.so $L/mmc.so || exit 1
