#!/bin/bash
# A/B timing of two builds of libvp8g on the same box, interleaved: bash tools/ab.sh libA libB [rounds]
A=$1; B=$2; N=${3:-3}
for i in $(seq $N); do
  for L in $A $B; do
    VP8G_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab.log 2>&1 || exit 1
    echo "$(basename $L) $(grep -o 'kernel_ms_per_step": [0-9.]*' gpurun_out/ab.log)"
  done
done
