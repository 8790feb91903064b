// Micro-benchmark: dependent-issue latency of vector instructions on gfx950.  One wave runs K
// independent chains of one instruction (K = 1, 2, 4, 8) interleaved round-robin, at 1 and 4 waves
// per SIMD; prints s_memtime ticks per wave-instruction per SIMD.  K = 1 at one wave per SIMD is the
// dependent latency; the K at which the rate stops improving is the ILP a single wave needs to keep
// its issue slot busy -- which decides whether interleaving independent work (the next step's iDCT)
// into frame_kernel's dependent chains (loop-filter edges, B_PRED steps) can pay.  Diagnostics only.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITER 256

template <int OP>
__device__ __forceinline__ void op1(uint32_t& a, uint32_t k) {
	if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(k));
	if constexpr (OP == 1) asm volatile("v_med3_i32 %0, %0, %1, %0" : "+v"(a) : "v"(k));
	if constexpr (OP == 2) asm volatile("v_sad_u16 %0, %0, %1, %0" : "+v"(a) : "v"(k));
	if constexpr (OP == 3) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(k));
}

template <int OP, int K>
__global__ void bench(unsigned long long* out, uint32_t seed) {
	uint32_t a[8];
#pragma unroll
	for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x * (2 * i + 1);
	const uint32_t k = seed ^ 0x5555;
	__syncthreads();
	const uint64_t t0 = __builtin_amdgcn_s_memtime();
	for (int it = 0; it < N_ITER; it++) {
#pragma unroll
		for (int r = 0; r < 8; r++) {
#pragma unroll
			for (int c = 0; c < K; c++) op1<OP>(a[c], k);
		}
	}
	const uint64_t t1 = __builtin_amdgcn_s_memtime();
	__syncthreads();
	if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)(t1 - t0));
	uint32_t x = 0;
#pragma unroll
	for (int i = 0; i < 8; i++) x ^= a[i];
	if (x == 0x12345678u) out[2] = 1;
}

template <int OP, int K>
void run(const char* name, unsigned long long* d) {
	for (int waves_per_simd : {1, 4}) {
		hipMemset(d, 0, 24);
		hipLaunchKernelGGL((bench<OP, K>), dim3(256 * waves_per_simd), dim3(256), 0, 0, d, 7u);
		hipDeviceSynchronize();
		unsigned long long h[3];
		hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
		const double waves = 256.0 * 4 * waves_per_simd;
		const double per_wave = (double)h[0] / waves;
		const double instr = 8.0 * K * N_ITER;
		printf("%-14s chains %d waves/SIMD %d: %.2f ticks per instr per wave, %.2f per wave-instr per SIMD\n", name, K,
		       waves_per_simd, per_wave / instr, per_wave / instr / waves_per_simd);
	}
}

template <int OP>
void all(const char* name, unsigned long long* d) {
	run<OP, 1>(name, d);
	run<OP, 2>(name, d);
	run<OP, 4>(name, d);
	run<OP, 8>(name, d);
}

int main() {
	unsigned long long* d;
	(void)hipMalloc(&d, 24);
	all<0>("v_add_u32", d);
	all<1>("v_med3_i32", d);
	all<2>("v_sad_u16", d);
	all<3>("v_pk_add_u16", d);
	(void)hipFree(d);
	return 0;
}
