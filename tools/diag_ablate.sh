for v in abl1 abl2 abl4 abl8 abl15; do
  echo "== $v" >> gpurun_out/abl.log
  VP8G_LIB=webp-decoder_amd/lib/diag/libvp8g_$v.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/abl.log 2>&1
done
