VP8G_LIB=webp-decoder_amd/lib/diag/libvp8g_stamps.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/d2.log 2>&1
bash tools/pmc_pass.sh gpurun_out/pmc_v2 --frames 512 --steps 2 --warmup 1
