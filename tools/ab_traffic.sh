bash tools/ab.sh webp-decoder_amd/lib/ab/libvp8g_A.so webp-decoder_amd/lib/ab/libvp8g_B.so 2 || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for v in A B; do
  VP8G_LIB=$R/webp-decoder_amd/lib/ab/libvp8g_$v.so timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/abw_$v -o pmc -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/abw_$v.log 2>&1 || exit 1
  VP8G_LIB=$R/webp-decoder_amd/lib/ab/libvp8g_$v.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/abf_$v -o pmc -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/abf_$v.log 2>&1 || exit 1
done
echo done
