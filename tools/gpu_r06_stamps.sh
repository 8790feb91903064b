#!/bin/bash
# Per-phase stamps, phase ablations and wave ends of the current build on uhd4 and synth (diagnostic
# builds from `make diag`; timing only, ablated outputs are wrong).  One GPU call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r06t}
O=gpurun_out/diag_$TAG
mkdir -p $O
QUIET="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
for wl in uhd4 synth; do
  for v in stamps abl1 abl2 abl4 abl8 abl15; do
    VP8G_LIB=$R/webp-decoder_amd/lib/diag/libvp8g_$v.so timeout -k 10 200 python3 bench.py $QUIET --workload $wl --steps 8 --warmup 2 > $O/${v}_$wl.json 2> $O/${v}_$wl.err || { echo "$v $wl failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_$wl.json')); print('$wl $v', d['ms_per_step'], d.get('stamps', ''))"
  done
  timeout -k 10 200 python3 tools/wave_tail.py webp-decoder_amd/lib/diag/libvp8g_stamps.so --workload $wl > $O/wave_tail_$wl.txt 2>&1 || { echo "wave_tail failed"; exit 1; }
  grep "mean duration" $O/wave_tail_$wl.txt
done
echo stamps_done
