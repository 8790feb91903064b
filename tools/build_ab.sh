#!/bin/bash
# Build A/B variants of libvp8g.so into webp-decoder_amd/lib/ab/<name>.so, in parallel (<= 4 at a time).
# Usage: tools/build_ab.sh name1 "-DFLAG=1 -DX=2" name2 "-DFLAG=3" ...
cd "$(dirname "$0")/.."
L=webp-decoder_amd/lib
SRC="webp-decoder_amd/csrc/vp8g_kernels.hip webp-decoder_amd/csrc/vp8g_shim.hip webp-decoder_amd/csrc/vp8g_rgb.hip webp-decoder_amd/csrc/vp8g_pipeline.hip webp-decoder_amd/csrc/vp8g_m05.hip webp-decoder_amd/csrc/vp8g_digest.hip"
mkdir -p $L/ab
n=0
while [ $# -ge 2 ]; do
	name=$1 flags=$2; shift 2
	hipcc -std=c++17 -O3 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -fvisibility=hidden -I include -munsafe-fp-atomics $flags \
		-shared -Wl,-Bsymbolic -o $L/ab/$name.so $SRC -L$L -lvp8host -Wl,-rpath,'$ORIGIN/..' -lpthread 2>&1 | grep -E "error" &
	n=$((n+1)); [ $((n % 4)) -eq 0 ] && wait
done
wait
ls -la $L/ab | grep -v r03
