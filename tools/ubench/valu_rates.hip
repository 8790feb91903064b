// Micro-benchmark: issue cost of the vector instructions the decode kernel leans on, on gfx950.
// Each kernel runs a long unrolled chain of 8 independent streams of one instruction; waves per
// SIMD vary via the block size.  Prints cycles per wave-instruction per SIMD (s_memtime deltas
// aggregated over the CU).  Diagnostics only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define N_ITER 256
#define OPS8(ins)                                                                                  \
	asm volatile(ins " %0, %0, %8\n" ins " %1, %1, %8\n" ins " %2, %2, %8\n" ins " %3, %3, %8\n" ins \
	             " %4, %4, %8\n" ins " %5, %5, %8\n" ins " %6, %6, %8\n" ins " %7, %7, %8\n"              \
	             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)        \
	             : "v"(k))
#define OPS8_3(ins)                                                                                       \
	asm volatile(ins " %0, %0, %8, %0\n" ins " %1, %1, %8, %1\n" ins " %2, %2, %8, %2\n" ins " %3, %3, %8, %3\n" \
	             ins " %4, %4, %8, %4\n" ins " %5, %5, %8, %5\n" ins " %6, %6, %8, %6\n" ins " %7, %7, %8, %7\n"  \
	             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)               \
	             : "v"(k))

template <int OP>
__global__ void bench(unsigned long long* out, uint32_t seed) {
	uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15;
	const uint32_t k = seed ^ 0x5555;
	__syncthreads();
	const uint64_t t0 = __builtin_amdgcn_s_memtime();
	for (int i = 0; i < N_ITER; i++) {
		if constexpr (OP == 0) OPS8("v_add_u32");
		if constexpr (OP == 1) OPS8("v_pk_add_u16");
		if constexpr (OP == 2) OPS8_3("v_sad_u16");
		if constexpr (OP == 3) OPS8_3("v_med3_i32");
		if constexpr (OP == 4) OPS8_3("v_perm_b32");
		if constexpr (OP == 5) OPS8_3("v_dot4_u32_u8");
		if constexpr (OP == 6) OPS8_3("v_mad_u32_u24");
		if constexpr (OP == 7) OPS8("v_mul_lo_u32");
		if constexpr (OP == 8) OPS8("v_pk_max_i16");
		if constexpr (OP == 9) OPS8_3("v_bfe_u32");
		if constexpr (OP == 10) OPS8_3("v_add3_u32");
		if constexpr (OP == 11) OPS8("v_lshlrev_b32");
	}
	const uint64_t t1 = __builtin_amdgcn_s_memtime();
	__syncthreads();
	if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)(t1 - t0));
	if (threadIdx.x == 0) atomicAdd(out + 1, 1ull);
	if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345678u) out[2] = 1;  // keep results live
}

template <int OP>
void run(const char* name, unsigned long long* d) {
	for (int waves_per_simd : {1, 2, 4, 8}) {
		// 4-wave blocks (one wave per SIMD), waves_per_simd blocks per CU
		hipMemset(d, 0, 24);
		hipLaunchKernelGGL(bench<OP>, dim3(256 * waves_per_simd), dim3(256), 0, 0, d, 7u);
		hipDeviceSynchronize();
		unsigned long long h[3];
		hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
		const double waves = 256.0 * 4 * waves_per_simd;
		const double cyc_per_wave = (double)h[0] / waves;  // average wave duration (s_memtime ticks)
		const double instr = 8.0 * N_ITER;
		// SIMD time per wave-instruction = wave duration / (instr per wave * waves sharing the SIMD)
		printf("%-16s waves/SIMD %d: %.2f ticks per instr per wave, %.2f ticks per wave-instr per SIMD\n", name,
		       waves_per_simd, cyc_per_wave / instr, cyc_per_wave / instr / waves_per_simd);
	}
}

int main() {
	unsigned long long* d;
	hipMalloc(&d, 24);
	run<0>("v_add_u32", d);
	run<1>("v_pk_add_u16", d);
	run<2>("v_sad_u16", d);
	run<3>("v_med3_i32", d);
	run<4>("v_perm_b32", d);
	run<5>("v_dot4_u32_u8", d);
	run<6>("v_mad_u32_u24", d);
	run<7>("v_mul_lo_u32", d);
	run<8>("v_pk_max_i16", d);
	run<9>("v_bfe_u32", d);
	run<10>("v_add3_u32", d);
	run<11>("v_lshlrev_b32", d);
	return 0;
}
