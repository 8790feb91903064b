// Micro-benchmark: calibrate rocprofv3's FETCH_SIZE against a known byte count for the two load
// shapes the decode kernel uses (diagnostics only):
//   mode 0  16 B per lane, lanes contiguous (the guide's calibrated case: FETCH_SIZE = bytes / 2)
//   mode 1  32 B per lane as two 16-B loads (+0, +16), lanes 32 B apart -- frame_kernel's
//           coefficient prefetch (one 4x4 block of int16 per lane, Y blocks of an MB contiguous)
// Each launch reads a 2 GiB buffer (>> L2 and the 256 MB Infinity Cache) exactly once.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/fetch_calib.hip -o tools/ubench/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -- tools/ubench/fetch_calib <mode>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void read16(const u32x4* __restrict__ p, size_t n16, unsigned* out) {
	u32x4 acc = {0, 0, 0, 0};
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) acc ^= p[i];
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[0] = 1;  // keep the loads
}

__global__ void read32(const u32x4* __restrict__ p, size_t n32, unsigned* out) {
	u32x4 acc = {0, 0, 0, 0};
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n32; i += (size_t)gridDim.x * blockDim.x) {
		acc ^= p[2 * i];
		acc ^= p[2 * i + 1];
	}
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9E3779B9u) out[0] = 1;
}

int main(int argc, char** argv) {
	const int mode = argc > 1 ? atoi(argv[1]) : 0;
	const size_t bytes = (size_t)2 << 30;
	u32x4* p;
	unsigned* o;
	if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
	hipMemset(p, 1, bytes);
	hipDeviceSynchronize();
	for (int rep = 0; rep < 3; rep++) {
		if (mode == 0) hipLaunchKernelGGL(read16, dim3(4096), dim3(256), 0, 0, p, bytes / 16, o);
		else hipLaunchKernelGGL(read32, dim3(4096), dim3(256), 0, 0, p, bytes / 32, o);
	}
	hipDeviceSynchronize();
	printf("mode %d: %zu bytes read per launch (3 launches)\n", mode, bytes);
	return 0;
}
