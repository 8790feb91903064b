export TMPDIR=/tmp
for v in "" stamps abl1 abl2 abl4 abl8 abl15; do
  if [ -z "$v" ]; then L=webp-decoder_amd/lib/libvp8g.so; else L=webp-decoder_amd/lib/diag/libvp8g_$v.so; fi
  echo "== $v" >> gpurun_out/diag.log
  VP8G_LIB=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/diag.log 2>&1 || { echo "FAIL $v rc=$?" >> gpurun_out/diag.log; break; }
done
VP8G_LIB=webp-decoder_amd/lib/libvp8g.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --unfiltered >> gpurun_out/diag.log 2>&1
for w in 8 4; do echo "== waves $w" >> gpurun_out/diag.log; timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --waves $w >> gpurun_out/diag.log 2>&1; done
echo "== frames 256" >> gpurun_out/diag.log; timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --frames 256 >> gpurun_out/diag.log 2>&1
