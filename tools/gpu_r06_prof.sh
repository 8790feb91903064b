#!/bin/bash
# Round 6: synth profile (trace stats, HBM traffic, SQ / LDS PMC groups) and per-phase stamps of the
# shipped build on synth and uhd4 (tools/gpu_round.sh profile + the stamps build).  One GPU call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r06s}
bash tools/gpu_round.sh profile "$TAG" synth || exit 1
O=gpurun_out/diag_$TAG
mkdir -p $O
QUIET="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
for wl in synth uhd4; do
  VP8G_LIB=$R/webp-decoder_amd/lib/diag/libvp8g_stamps.so timeout -k 10 200 python3 bench.py $QUIET --workload $wl --steps 10 --warmup 2 > $O/stamps_$wl.json 2> $O/stamps_$wl.err || { echo "stamps $wl failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$O/stamps_$wl.json')); print('$wl', d['ms_per_step'], d.get('stamps'))"
done
timeout -k 10 200 python3 tools/wave_tail.py webp-decoder_amd/lib/diag/libvp8g_stamps.so --workload synth > $O/wave_tail_synth.txt 2>&1 || { echo "wave_tail failed"; exit 1; }
grep -v amdgpu.ids $O/wave_tail_synth.txt | head -3
echo r06prof_done
