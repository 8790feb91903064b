// Micro-benchmark: does a wave64 vector instruction cost less when only some of its lanes are
// active on gfx950 (e.g. a whole 32-lane half masked off by EXEC)?  frame_kernel runs phases in
// which one 32-lane half idles (a B_PRED MB beside a whole-block one, luma-only loop-filter edges),
// so the answer decides whether lane-role layouts should keep active lanes in one half.
// Same harness as valu_rates.hip: 8 independent streams of one instruction, s_memtime ticks per
// wave-instruction per SIMD at 1 / 4 waves per SIMD, for several EXEC masks.  Diagnostics only.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

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

// MASK: 0 all lanes, 1 lanes 0..31, 2 lanes 32..63, 3 lanes 0..15, 4 lane 0, 5 even lanes, 6 lanes 0..15 + 32..47
template <int OP, int MASK>
__global__ void bench(unsigned long long* out, uint32_t seed) {
	const int lane = (int)(threadIdx.x & 63);
	uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15;
	const uint32_t k = seed ^ 0x5555;
	bool on = true;
	if (MASK == 1) on = lane < 32;
	if (MASK == 2) on = lane >= 32;
	if (MASK == 3) on = lane < 16;
	if (MASK == 4) on = lane == 0;
	if (MASK == 5) on = (lane & 1) == 0;
	if (MASK == 6) on = (lane & 31) < 16;
	__syncthreads();
	const uint64_t t0 = __builtin_amdgcn_s_memtime();
	if (on) {
		for (int i = 0; i < N_ITER; i++) {
			if constexpr (OP == 0) OPS8("v_add_u32");
			if constexpr (OP == 1) OPS8_3("v_med3_i32");
			if constexpr (OP == 2) OPS8_3("v_perm_b32");
		}
	}
	const uint64_t t1 = __builtin_amdgcn_s_memtime();
	__syncthreads();
	if (lane == 0) atomicAdd(out, (unsigned long long)(t1 - t0));
	if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345678u) out[2] = 1;  // keep results live
}

template <int OP, int MASK>
void run(const char* name, const char* mask, unsigned long long* d) {
	for (int waves_per_simd : {1, 4}) {
		hipMemset(d, 0, 24);
		hipLaunchKernelGGL((bench<OP, MASK>), dim3(256 * waves_per_simd), dim3(256), 0, 0, d, 7u);
		hipDeviceSynchronize();
		unsigned long long h[3];
		hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
		const double waves = 256.0 * 4 * waves_per_simd;
		const double cyc_per_wave = (double)h[0] / waves;
		const double instr = 8.0 * N_ITER;
		printf("%-12s exec %-14s waves/SIMD %d: %.2f ticks per wave-instr per SIMD\n", name, mask, waves_per_simd,
		       cyc_per_wave / instr / waves_per_simd);
	}
}

template <int OP>
void all(const char* name, unsigned long long* d) {
	run<OP, 0>(name, "all 64", d);
	run<OP, 1>(name, "0..31", d);
	run<OP, 2>(name, "32..63", d);
	run<OP, 3>(name, "0..15", d);
	run<OP, 6>(name, "0..15,32..47", d);
	run<OP, 5>(name, "even", d);
	run<OP, 4>(name, "lane 0", d);
}

int main() {
	unsigned long long* d;
	hipMalloc(&d, 24);
	all<0>("v_add_u32", d);
	all<1>("v_med3_i32", d);
	all<2>("v_perm_b32", d);
	hipFree(d);
	return 0;
}
