# Top-level build (GNU make; no cmake/ninja needed).
#
#   make            libvp8host.so (C11 front end), libvp8g.so (HIP gfx950 kernels + C-ABI shim),
#                   bin/decoder (the CLI), oracle/liboracle.so (+ oracle/_ref when the reference exists)
#   make lib        just the product libraries + CLI
#
# Everything is built in-tree so the .so files travel to the GPU box with the snapshot.

PKG := webp-decoder_amd
LIB := $(PKG)/lib
BIN := $(PKG)/bin
HIPCC ?= /opt/rocm/bin/hipcc
CC ?= gcc
OFFLOAD_ARCH ?= gfx950

HOST_SRC := $(PKG)/host/webp_riff.c $(PKG)/host/vp8_parse.c $(PKG)/host/vp8_synth.c
HOST_HDR := $(PKG)/host/vp8_front.h $(PKG)/host/vp8_bool.h $(PKG)/host/vp8_tables.inc include/vp8g.h
HIP_SRC := $(PKG)/csrc/vp8g_kernels.hip $(PKG)/csrc/vp8g_shim.hip $(PKG)/csrc/vp8g_rgb.hip $(PKG)/csrc/vp8g_pipeline.hip $(PKG)/csrc/vp8g_m05.hip \
	$(PKG)/csrc/vp8g_digest.hip
HIP_HDR := $(PKG)/csrc/vp8g_device.h include/vp8g.h $(PKG)/host/vp8_front.h $(PKG)/csrc/vp8g_quad.inc
# libvp8g links the host front end (the end-to-end batch path runs m05 on worker threads)
HIP_LINK := -L$(LIB) -lvp8host -Wl,-rpath,'$$ORIGIN' -lpthread

CFLAGS := -std=c11 -O3 -march=x86-64-v3 -Wall -Wextra -Wpedantic -fPIC -D_POSIX_C_SOURCE=200809L
HIPFLAGS := -std=c++17 -O3 --offload-arch=$(OFFLOAD_ARCH) -fPIC -Wall -Wno-unused-function \
	-fvisibility=hidden -I include -munsafe-fp-atomics

all: lib oracle $(LIB)/diag/libvp8g_stall.so

# (oracle/ re-links the reference CLI against libvp8g.so: build the library first)
oracle: lib

lib: $(LIB)/libvp8host.so $(LIB)/libvp8g.so $(BIN)/decoder

$(LIB) $(BIN):
	mkdir -p $@

$(LIB)/libvp8host.so: $(HOST_SRC) $(HOST_HDR) | $(LIB)
	$(CC) $(CFLAGS) -shared -Wl,-Bsymbolic -o $@ $(HOST_SRC)

$(LIB)/libvp8g.so: $(HIP_SRC) $(HIP_HDR) $(LIB)/libvp8host.so | $(LIB)
	$(HIPCC) $(HIPFLAGS) -shared -Wl,-Bsymbolic -o $@ $(HIP_SRC) $(HIP_LINK)

$(BIN)/decoder: $(PKG)/host/decoder_main.c $(LIB)/libvp8host.so $(LIB)/libvp8g.so | $(BIN)
	$(CC) $(CFLAGS) -o $@ $(PKG)/host/decoder_main.c -L$(LIB) -lvp8host -lvp8g -Wl,-rpath,'$$ORIGIN/../lib'

oracle:
	$(MAKE) -C oracle

# Diagnostic variants of libvp8g (never loaded by the product path; select with VP8G_LIB=...):
# per-phase shader-clock stamps, and phase ablations (timing only, wrong output).
DIAG := $(LIB)/diag
DIAG_VARIANTS := stamps abl1 abl2 abl4 abl8 abl15 abl16 abl32 abl47 pairs
diag: $(foreach v,$(DIAG_VARIANTS),$(DIAG)/libvp8g_$(v).so) $(DIAG)/libvp8g_stall.so
$(DIAG):
	mkdir -p $@
$(DIAG)/libvp8g_stamps.so: $(HIP_SRC) $(HIP_HDR) | $(DIAG)
	$(HIPCC) $(HIPFLAGS) -DVP8G_STAMPS -shared -Wl,-Bsymbolic -o $@ $(HIP_SRC) -L$(LIB) -lvp8host -Wl,-rpath,'$$ORIGIN/..' -lpthread
# test build: wave 1 of every frame never publishes its progress and a wait gives up after 20 ms
# (tests/test_gpu_batch.py: a stalled producer must end the launch promptly with EIO)
$(DIAG)/libvp8g_stall.so: $(HIP_SRC) $(HIP_HDR) | $(DIAG)
	$(HIPCC) $(HIPFLAGS) -DVP8G_WAIT_TICKS=2000000ull -DVP8G_TEST_STALL_WAVE=1 -shared -Wl,-Bsymbolic -o $@ $(HIP_SRC) -L$(LIB) -lvp8host -Wl,-rpath,'$$ORIGIN/..' -lpthread
# A/B build: the chain with two MB rows per wave (frame_kernel) instead of the quad kernel
$(DIAG)/libvp8g_pairs.so: $(HIP_SRC) $(HIP_HDR) | $(DIAG)
	$(HIPCC) $(HIPFLAGS) -DVP8G_QUAD_DEFAULT=0 -shared -Wl,-Bsymbolic -o $@ $(HIP_SRC) -L$(LIB) -lvp8host -Wl,-rpath,'$$ORIGIN/..' -lpthread
$(DIAG)/libvp8g_abl%.so: $(HIP_SRC) $(HIP_HDR) | $(DIAG)
	$(HIPCC) $(HIPFLAGS) -DVP8G_ABLATE=$* -shared -Wl,-Bsymbolic -o $@ $(HIP_SRC) -L$(LIB) -lvp8host -Wl,-rpath,'$$ORIGIN/..' -lpthread

clean:
	rm -rf $(LIB) $(BIN)
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean diag
