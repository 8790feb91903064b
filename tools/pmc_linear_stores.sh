#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the linearised-store diagnostic build (where the extra HBM reads come from)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc16
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  VP8G_LIB=$R/webp-decoder_amd/lib/diag/libvp8g_abl16.so timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o pmc -- python3 $R/bench.py --no-cpu-baseline --e2e-frames 0 --extra none --encode none --steps 2 --warmup 1 > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
echo done16
