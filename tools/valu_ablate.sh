#!/bin/bash
# Dynamic instruction counts per phase: SQ_INSTS_* of the bench kernel for the product build and
# each ablation variant (make diag).  Usage: bash tools/valu_ablate.sh <outdir>
set -u
OUT=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
export TMPDIR=/tmp
cd /tmp
for v in base abl1 abl2 abl4 abl8; do
  if [ $v = base ]; then export VP8G_LIB=$R/webp-decoder_amd/lib/libvp8g.so; else export VP8G_LIB=$R/webp-decoder_amd/lib/diag/libvp8g_$v.so; fi
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $R/$OUT/$v -o pmc -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/$OUT/$v.log 2>&1 || { echo "pass $v failed rc=$?"; exit 1; }
done
echo done
