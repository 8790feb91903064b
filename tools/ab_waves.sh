set -e
for i in 1 2; do
for cfg in base.so:0 gctx8.so:0 gctx10.so:10; do
  L=${cfg%%:*}; W=${cfg##*:}
  if [ $W = 0 ]; then unset VP8G_WAVES; else export VP8G_WAVES=$W; fi
  VP8G_LIB=webp-decoder_amd/lib/ab/$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab.log 2>&1
  echo "$L $W $(grep -o 'kernel_ms_per_step": [0-9.]*' gpurun_out/ab.log) $(grep -o '"parity": "[^"]*"' gpurun_out/ab.log)"
done; done
