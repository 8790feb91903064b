# frames / waves scan for the bench kernel
for fr in 32 128 256 512; do
  echo "== frames $fr" >> gpurun_out/scan.log
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --frames $fr >> gpurun_out/scan.log 2>&1
done
for w in 1 2 4 8 16; do
  echo "== frames 256 waves $w" >> gpurun_out/scan.log
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --frames 256 --waves $w >> gpurun_out/scan.log 2>&1
done
