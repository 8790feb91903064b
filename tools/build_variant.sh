#!/bin/bash
# Build a diagnostic variant of libvp8g.so with extra -D flags: tools/build_variant.sh out.so -DFOO=...
# (links webp-decoder_amd/lib/libvp8host.so: build that first with `make lib`)
OUT=$1; shift
/opt/rocm/bin/hipcc -std=c++17 -O3 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -fvisibility=hidden \
  -I include -munsafe-fp-atomics "$@" -shared -Wl,-Bsymbolic -o "$OUT" \
  webp-decoder_amd/csrc/vp8g_kernels.hip webp-decoder_amd/csrc/vp8g_shim.hip webp-decoder_amd/csrc/vp8g_rgb.hip \
  webp-decoder_amd/csrc/vp8g_pipeline.hip -Lwebp-decoder_amd/lib -lvp8host \
  -Wl,-rpath,'$ORIGIN:$ORIGIN/..:$ORIGIN/../..' -lpthread
