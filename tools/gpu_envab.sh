#!/bin/bash
# one library under several environment settings (env switches are read once per process, so each
# setting is its own ab_inproc process on the same box): uhd4 kernel medians
set -o pipefail
mkdir -p gpurun_out/envab
for cfg in "X=0" "VP8G_SPLITCHAIN=0" "VP8G_SPLITCHAIN=0 VP8G_CHAIN_IL=1" "X=1"; do
	env $cfg timeout -k 10 300 python3 -u tools/ab_inproc.py --workload uhd4 --rounds 3 --steps 6 webp-decoder_amd/lib/libvp8g.so \
		> gpurun_out/envab/out.json 2> gpurun_out/envab/err.txt || { tail -5 gpurun_out/envab/err.txt; exit 1; }
	echo "$cfg $(cat gpurun_out/envab/out.json)"
done
