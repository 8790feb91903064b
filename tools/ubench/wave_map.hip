// Micro-benchmark (diagnostics): where the waves of frame_kernel-shaped workgroups
// land.  512 workgroups x 8 waves with 73 104 B of LDS each (two per CU, as frame_kernel at 4K);
// every wave records HW_ID (gfx9 layout: wave slot [3:0], SIMD [5:4], CU [11:8], SH [12], SE
// [15:13]) and XCC_ID, then spins ~2 ms so all workgroups are resident together.  Prints one line
// per wave: block wave simd cu sh se xcc.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/wave_map.hip -o tools/ubench/wave_map
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(512) void probe(unsigned* out) {
	extern __shared__ unsigned char lds[];
	const unsigned w = threadIdx.x >> 6;
	unsigned hw, xcc;
	asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
	asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
	lds[threadIdx.x] = (unsigned char)hw;
	const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
	while (__builtin_amdgcn_s_memrealtime() - t0 < 200000ull) __builtin_amdgcn_s_sleep(8);  // 2 ms at 100 MHz
	if ((threadIdx.x & 63) == 0) {
		out[2 * (blockIdx.x * 8 + w)] = hw;
		out[2 * (blockIdx.x * 8 + w) + 1] = xcc + lds[(threadIdx.x + 64) & 511] * 0u;
	}
}

int main() {
	const int nb = 512;
	unsigned* d;
	if (hipMalloc(&d, nb * 8 * 8) != hipSuccess) return 1;
	hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 73104);
	hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 73104, 0, d);
	if (hipDeviceSynchronize() != hipSuccess) return 2;
	unsigned h[nb * 16];
	hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
	for (int b = 0; b < nb; b++)
		for (int w = 0; w < 8; w++) {
			const unsigned hw = h[2 * (b * 8 + w)], x = h[2 * (b * 8 + w) + 1];
			printf("%d %d %u %u %u %u %u\n", b, w, (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7, x & 15);
		}
	return 0;
}
