#!/bin/bash
# Dynamic instruction mix of the bench kernel for several libvp8g builds (one SQ counter group per
# rocprofv3 run, the bench workload's frame_kernel dispatches; diagnostics).  Usage (on the GPU box,
# from the repo root): bash tools/pmc_mix.sh <outdir> lib1.so lib2.so ...
set -u
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
export TMPDIR=/tmp
cd /tmp
i=0
for L in "$@"; do
  i=$((i+1))
  VP8G_LIB=$R/$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --output-format csv -d $R/$OUT/mix$i -o pmc -- python3 $R/bench.py --no-cpu-baseline --e2e-frames 0 --extra none --encode none --steps 2 --warmup 1 \
    > $R/$OUT/mix$i.log 2>&1 || { echo "pmc mix $L failed rc=$?"; exit 1; }
  echo "$i $L" >> $R/$OUT/libs.txt
done
echo pmc_mix_done
