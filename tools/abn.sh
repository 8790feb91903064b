#!/bin/bash
# Interleaved timing of N builds of libvp8g on one box: bash tools/abn.sh rounds lib1 lib2 ...
N=$1; shift
for i in $(seq $N); do
  for L in "$@"; do
    VP8G_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab.log 2>&1 || exit 1
    echo "$(basename $L) $(grep -o 'kernel_ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
