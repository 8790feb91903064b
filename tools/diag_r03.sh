#!/bin/bash
# Round-3 phase diagnostics of the shipped schedule (chain mode): per-phase stamps and phase
# ablations (diagnostic builds from `make diag`, timing only), per-block durations (wave_tail.py).
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/diag_$TAG
mkdir -p $OUT
cd $R
ARGS="--extra none --e2e-frames 0 --encode none --no-cpu-baseline --steps 10 --warmup 2"
for v in stamps abl1 abl2 abl4 abl8 abl15; do
  VP8G_LIB=$R/webp-decoder_amd/lib/diag/libvp8g_$v.so timeout -k 10 200 python3 bench.py $ARGS > $OUT/$v.json 2> $OUT/$v.err || { echo "variant $v failed rc=$?"; exit 1; }
  echo "$v $(python3 -c "import json,sys; d=json.load(open('$OUT/$v.json')); print(d['ms_per_step'], d.get('stamps',''))")"
done
for wl in uhd4 fhd4; do
  timeout -k 10 200 python3 tools/wave_tail.py webp-decoder_amd/lib/diag/libvp8g_stamps.so --workload $wl > $OUT/wave_tail_$wl.txt 2>&1 || { echo "wave_tail failed rc=$?"; exit 1; }
  cat $OUT/wave_tail_$wl.txt
done
echo diag_done
