// Micro-benchmark (diagnostics): can two 10-wave workgroups with 96 VGPRs and 81 040 B of
// LDS each share a CU (5 waves per SIMD)?  Records per wave HW_ID, XCC_ID and start/end s_memrealtime;
// every wave spins ~2 ms.  argv[1]: LDS bytes per workgroup (default 81 040).  Prints: block wave simd cu sh se xcc t_start t_end.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/wave_map10.hip -o tools/ubench/wave_map10
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(640, 5) void probe(unsigned long long* out) {
	extern __shared__ unsigned char lds[];
	const unsigned w = threadIdx.x >> 6;
	unsigned hw, xcc;
	asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
	asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
	asm volatile("v_mov_b32 v95, 0" ::: "v95");  // the kernel allocates 96 VGPRs, like frame_kernel<10>
	lds[threadIdx.x] = (unsigned char)hw;
	const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
	while (__builtin_amdgcn_s_memrealtime() - t0 < 200000ull) __builtin_amdgcn_s_sleep(8);
	const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
	if ((threadIdx.x & 63) == 0) {
		unsigned long long* o = out + 4 * (blockIdx.x * 10 + w);
		o[0] = hw;
		o[1] = xcc + lds[(threadIdx.x + 64) % 640] * 0u;
		o[2] = t0;
		o[3] = t1;
	}
}

#include <stdlib.h>
int main(int argc, char** argv) {
	const int nb = 512, lds = argc > 1 ? atoi(argv[1]) : 81040;  // LDS bytes per workgroup
	unsigned long long* d;
	if (hipMalloc(&d, nb * 10 * 32) != hipSuccess) return 1;
	if (hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return 3;
	hipLaunchKernelGGL(probe, dim3(nb), dim3(640), lds, 0, d);
	if (hipDeviceSynchronize() != hipSuccess) return 2;
	static unsigned long long h[512 * 10 * 4];
	if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 4;
	for (int b = 0; b < nb; b++)
		for (int w = 0; w < 10; w++) {
			const unsigned long long* o = h + 4 * (b * 10 + w);
			const unsigned hw = (unsigned)o[0];
			printf("%d %d %u %u %u %u %llu %llu %llu\n", b, w, (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7, o[1] & 15, o[2], o[3]);
		}
	return 0;
}
