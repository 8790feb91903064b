set -e
B="python -u bench.py --workload uhd4_yuv --extra none --no-cpu-baseline --e2e-frames 0 --e2e-device-frames 0 --encode none --steps 10 --warmup 3"
for i in 1 2; do
for s in auto 0 1; do
  if [ $s = auto ]; then timeout -k 10 120 $B > gpurun_out/yuvab_${s}_$i.json; else VP8G_SPLITCHAIN=$s timeout -k 10 120 $B > gpurun_out/yuvab_${s}_$i.json; fi
  echo $s $i $(python3 -c "import json;d=json.loads(open('gpurun_out/yuvab_${s}_$i.json').read().strip().splitlines()[-1]);print(d['kernel_ms_per_step'],d['parity'])")
done; done
