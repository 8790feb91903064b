#!/bin/bash
# Build a libvp8g variant with extra compile flags into webp-decoder_amd/lib/ab/<name>.so (A/B experiments):
#   bash tools/build_variant.sh <name> -DVP8G_PRIO_TABLE=0,2,2,3,3,1,3,2 ...
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p webp-decoder_amd/lib/ab
HIP_SRC="webp-decoder_amd/csrc/vp8g_kernels.hip webp-decoder_amd/csrc/vp8g_shim.hip webp-decoder_amd/csrc/vp8g_rgb.hip webp-decoder_amd/csrc/vp8g_pipeline.hip webp-decoder_amd/csrc/vp8g_m05.hip webp-decoder_amd/csrc/vp8g_digest.hip"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -munsafe-fp-atomics -Iinclude -Iwebp-decoder_amd/csrc "$@" -shared -Wl,-Bsymbolic \
  -o webp-decoder_amd/lib/ab/$NAME.so $HIP_SRC -Lwebp-decoder_amd/lib -lvp8host -Wl,-rpath,'$ORIGIN/..' -lpthread
