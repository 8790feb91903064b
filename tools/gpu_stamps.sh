#!/bin/bash
# Stamps build of the current source on the bench workload(s) (diagnostics): bash tools/gpu_stamps.sh <tag> [workloads]
set -u
TAG=$1; WLS=${2:-uhd4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/stamps_$TAG
for W in ${WLS//,/ }; do
  VP8G_LIB=$R/webp-decoder_amd/lib/diag/libvp8g_stamps.so timeout -k 10 200 python3 bench.py --workload $W --e2e-frames 0 --extra none --encode none --no-cpu-baseline --steps 10 --warmup 2 \
    > gpurun_out/stamps_$TAG/$W.json 2> gpurun_out/stamps_$TAG/$W.err || { echo "stamps $W failed"; exit 1; }
  echo "$W $(python3 -c "import json; d=json.load(open('gpurun_out/stamps_$TAG/$W.json')); print(d['ms_per_step'], d.get('stamps', ''))")"
done
