set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/diag_r05c
Q="--e2e-frames 0 --extra none --encode none --no-cpu-baseline"
for v in stamps abl1 abl2 abl15; do
  VP8G_LIB=$R/webp-decoder_amd/lib/diag/libvp8g_$v.so timeout -k 10 200 python3 bench.py $Q --steps 10 --warmup 2 > gpurun_out/diag_r05c/$v.json 2> gpurun_out/diag_r05c/$v.err || { echo "variant $v failed"; exit 1; }
  echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/diag_r05c/$v.json')); print(d['ms_per_step'], d.get('stamps', ''))")"
done
bash tools/pmc_mix.sh gpurun_out/pmc_r05c webp-decoder_amd/lib/libvp8g.so webp-decoder_amd/lib/diag/libvp8g_abl1.so webp-decoder_amd/lib/diag/libvp8g_abl2.so webp-decoder_amd/lib/diag/libvp8g_abl4.so webp-decoder_amd/lib/diag/libvp8g_abl15.so
