#!/bin/bash
# One GPU call of frame_kernel diagnostics on the uhd4 bench batch: the SQ / LDS / HBM PMC passes
# (tools/pmc_pass.sh), then the per-phase stamp build and the phase ablations (timing only; their
# parity reads MISMATCH by construction).  Usage on the box: bash tools/diag_round.sh <tag>
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/diag_$TAG
mkdir -p $R/$OUT
ARGS="--extra none --e2e-frames 0 --encode none --no-cpu-baseline --steps 6 --warmup 2"
bash $R/tools/pmc_pass.sh $OUT $ARGS || exit 1
cd $R
for v in stamps abl1 abl2 abl4 abl8 abl15; do
  VP8G_LIB=$R/webp-decoder_amd/lib/diag/libvp8g_$v.so timeout -k 10 200 python3 bench.py $ARGS --steps 10 > $OUT/$v.json 2> $OUT/$v.err || { echo "variant $v failed rc=$?"; exit 1; }
done
echo diag_done
