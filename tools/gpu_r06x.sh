#!/bin/bash
# Round 6 evidence call: GPU tests, default bench line, kernel-trace stats, HBM traffic and PMC of the
# committed build (uhd4), then the same profile for the synth workload.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r06x}
bash tools/gpu_round.sh evidence $TAG || exit 1
bash tools/gpu_round.sh profile ${TAG}s synth || exit 1
echo r06x_done
