#!/usr/bin/env python3
"""Generate tools/ubench/valu_rates2.hip: issue cost per wave-instruction of a wider set of vector
instructions on gfx950 (round 3) -- integer VOP2/VOP3 forms, FP32 and packed-FP32 forms, SDWA byte
selects, DPP -- measured like valu_rates.hip (8 independent streams per wave, 1/2/4/8 waves per
SIMD; s_memtime ticks per wave-instruction per SIMD).  Diagnostics only.
  python tools/ubench/gen_valu_rates2.py && hipcc --offload-arch=gfx950 -O3 -o tools/ubench/valu_rates2 tools/ubench/valu_rates2.hip
"""
import pathlib

# (name, one stream's asm with {r} = the stream register and {k} = the constant operand)
OPS = [
    ("v_add_u32", "v_add_u32 {r}, {r}, {k}"),
    ("v_sub_u32", "v_sub_u32 {r}, {r}, {k}"),
    ("v_and_b32", "v_and_b32 {r}, {r}, {k}"),
    ("v_xor_b32", "v_xor_b32 {r}, {r}, {k}"),
    ("v_max_i32", "v_max_i32 {r}, {r}, {k}"),
    ("v_min_u32", "v_min_u32 {r}, {r}, {k}"),
    ("v_lshrrev_b32", "v_lshrrev_b32 {r}, {k}, {r}"),
    ("v_mul_u32_u24", "v_mul_u32_u24 {r}, {r}, {k}"),
    ("v_add_u16", "v_add_u16 {r}, {r}, {k}"),
    ("v_cndmask_b32_vcc", "v_cndmask_b32 {r}, {r}, {k}, vcc"),
    ("v_mov_b32", "v_mov_b32 {r}, {k}"),
    ("v_add_u32_e64", "v_add_u32_e64 {r}, {r}, {k}"),
    ("v_add_u32_sdwa_b1", "v_add_u32_sdwa {r}, {r}, {k} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"),
    ("v_sub_u16_sdwa_wb", "v_sub_u16_sdwa {r}, {r}, {k} dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2 src1_sel:BYTE_0"),
    ("v_add_u32_dpp", "v_add_u32_dpp {r}, {r}, {k} row_shr:1 row_mask:0xf bank_mask:0xf"),
    ("v_add3_u32", "v_add3_u32 {r}, {r}, {k}, {r}"),
    ("v_med3_i32", "v_med3_i32 {r}, {r}, {k}, {r}"),
    ("v_max3_u32", "v_max3_u32 {r}, {r}, {k}, {r}"),
    ("v_sad_u16", "v_sad_u16 {r}, {r}, {k}, {r}"),
    ("v_sad_u8", "v_sad_u8 {r}, {r}, {k}, {r}"),
    ("v_perm_b32", "v_perm_b32 {r}, {r}, {k}, {r}"),
    ("v_bfi_b32", "v_bfi_b32 {r}, {r}, {k}, {r}"),
    ("v_lshl_or_b32", "v_lshl_or_b32 {r}, {r}, 8, {k}"),
    ("v_mad_u32_u24", "v_mad_u32_u24 {r}, {r}, {k}, {r}"),
    ("v_pk_add_u16", "v_pk_add_u16 {r}, {r}, {k}"),
    ("v_pk_sub_u16_clamp", "v_pk_sub_u16 {r}, {r}, {k} clamp"),
    ("v_pk_max_i16", "v_pk_max_i16 {r}, {r}, {k}"),
    ("v_pk_mad_i16", "v_pk_mad_i16 {r}, {r}, {k}, {r}"),
    ("v_add_f32", "v_add_f32 {r}, {r}, {k}"),
    ("v_mul_f32", "v_mul_f32 {r}, {r}, {k}"),
    ("v_max_f32", "v_max_f32 {r}, {r}, {k}"),
    ("v_fmac_f32", "v_fmac_f32 {r}, {r}, {k}"),
    ("v_fma_f32", "v_fma_f32 {r}, {r}, {k}, {r}"),
    ("v_med3_f32", "v_med3_f32 {r}, {r}, {k}, {r}"),
    ("v_cvt_f32_ubyte1", "v_cvt_f32_ubyte1 {r}, {r}"),
    ("v_pk_add_f32", "v_pk_add_f32 {p}, {p}, {q}"),
    ("v_pk_fma_f32", "v_pk_fma_f32 {p}, {p}, {q}, {p}"),
    ("v_pk_add_f16", "v_pk_add_f16 {r}, {r}, {k}"),
    ("v_pk_max_f16", "v_pk_max_f16 {r}, {r}, {k}"),
    ("v_dot2_u32_u16", "v_dot2_u32_u16 {r}, {r}, {k}, {r}"),
    # second pass (r03b): masks, carries, SGPR operands, shifts
    ("v_cndmask_e64_sgpr", "v_cndmask_b32_e64 {r}, {r}, {k}, s[20:21]"),
    ("v_cndmask_e64_const", "v_cndmask_b32_e64 {r}, 0, {r}, s[20:21]"),
    ("v_add_u32_sgpr", "v_add_u32 {r}, s22, {r}"),
    ("v_add_co_u32", "v_add_co_u32 {r}, vcc, {r}, {k}"),
    ("v_cmp_gt_u32_e64", "v_cmp_gt_u32_e64 s[24:25], {r}, {k}\\nv_add_u32 {r}, {r}, {k}"),
    ("v_add_u32_pair", "v_add_u32 {r}, {r}, {k}\\nv_add_u32 {r}, {r}, {k}"),
    ("v_ashrrev_i32", "v_ashrrev_i32 {r}, 3, {r}"),
    ("v_lshlrev_b32", "v_lshlrev_b32 {r}, 1, {r}"),
    ("v_or_b32", "v_or_b32 {r}, {r}, {k}"),
    ("v_not_b32", "v_not_b32 {r}, {r}"),
    ("v_bfe_u32", "v_bfe_u32 {r}, {r}, 8, 8"),
    ("v_lshl_add_u32", "v_lshl_add_u32 {r}, {r}, 1, {k}"),
    ("v_add_lshl_u32", "v_add_lshl_u32 {r}, {r}, {k}, 1"),
    ("v_mad_i32_i24", "v_mad_i32_i24 {r}, {r}, 3, {k}"),
    ("v_mul_lo_u16", "v_mul_lo_u16 {r}, {r}, {k}"),
    ("v_pk_mul_lo_u16", "v_pk_mul_lo_u16 {r}, {r}, {k}"),
    ("v_mul_hi_i32_i24", "v_mul_hi_i32_i24 {r}, {r}, {k}"),
    ("v_max_u16", "v_max_u16 {r}, {r}, {k}"),
    ("v_sub_u32_clamp", "v_sub_u32_e64 {r}, {r}, {k} clamp"),
    ("v_cvt_pk_u8_f32", "v_cvt_pk_u8_f32 {r}, {r}, 1, {r}"),
    ("v_readfirstlane", "v_readfirstlane_b32 s26, {r}\\nv_add_u32 {r}, {r}, {k}"),
    ("v_alignbit_b32", "v_alignbit_b32 {r}, {r}, {k}, 8"),
    ("v_lerp_u8", "v_lerp_u8 {r}, {r}, {k}, {r}"),
    ("v_cvt_f32_i32", "v_cvt_f32_i32 {r}, {r}"),
    ("v_floor_f32", "v_floor_f32 {r}, {r}"),
    ("v_min3_i32", "v_min3_i32 {r}, {r}, {k}, {r}"),
    # third pass (r03g): saturating packs, 16-bit forms, bitop3, lane swaps
    ("v_sat_pk_u8_i16", "v_sat_pk_u8_i16 {r}, {r}"),
    ("v_med3_i16", "v_med3_i16 {r}, {r}, {k}, {r}"),
    ("v_max_i16", "v_max_i16 {r}, {r}, {k}"),
    ("v_sub_i16_clamp", "v_sub_i16 {r}, {r}, {k} clamp"),
    ("v_add_u16_clamp", "v_add_u16 {r}, {r}, {k} clamp"),
    ("v_pk_add_i16_clamp", "v_pk_add_i16 {r}, {r}, {k} clamp"),
    ("v_bitop3_b32", "v_bitop3_b32 {r}, {r}, {k}, {r} bitop3:0xca"),
    ("v_permlane32_swap", "v_permlane32_swap_b32 {r}, {k}"),
    ("v_lshlrev_b16", "v_lshlrev_b16 {r}, 1, {r}"),
    ("v_mul_lo_u32", "v_mul_lo_u32 {r}, {r}, {k}"),
    ("v_cmp_vcc_cndmask", "v_cmp_gt_u32 vcc, {r}, {k}\\nv_cndmask_b32 {r}, {r}, {k}, vcc"),
    ("v_cmp_vcc_add", "v_cmp_gt_u32 vcc, {r}, {k}\\nv_add_u32 {r}, {r}, {k}"),
]

head = r'''// GENERATED by tools/ubench/gen_valu_rates2.py -- see there.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define N_ITER 256
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
'''
kern = r'''
__global__ void bench_{i}(unsigned long long* out, uint32_t seed) {{
	uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 9, a5 = a0 * 11, a6 = a0 * 13, a7 = a0 * 15;
	uint32_t b0 = a0 ^ 1, b1 = a1 ^ 1, b2 = a2 ^ 1, b3 = a3 ^ 1, b4 = a4 ^ 1, b5 = a5 ^ 1, b6 = a6 ^ 1, b7 = a7 ^ 1;
	const uint32_t k = seed ^ 0x5555;
	u32x2 kk = u32x2{{k, k + 1}};
	u32x2 p0 = u32x2{{a0, b0}}, p1 = u32x2{{a1, b1}}, p2 = u32x2{{a2, b2}}, p3 = u32x2{{a3, b3}};
	asm volatile("v_cmp_gt_u32 vcc, %0, %1\ns_mov_b64 s[20:21], vcc\ns_mov_b32 s22, 7" ::"v"(a0), "v"(k) : "vcc", "s20", "s21", "s22");
	__syncthreads();
	const uint64_t t0 = __builtin_amdgcn_s_memtime();
	for (int i = 0; i < N_ITER; i++) {{
{body}
	}}
	const uint64_t t1 = __builtin_amdgcn_s_memtime();
	__syncthreads();
	if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)(t1 - t0));
	if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ p0.x ^ p1.y ^ p2.x ^ p3.y) == 0x12345678u) out[2] = 1;
}}
'''
out = [head]
for i, (name, pat) in enumerate(OPS):
    if "{p}" in pat:
        lines = [pat.format(p="%%%d" % j, q="%4") for j in range(4)]
        lines = lines + lines  # 8 per iteration
        body = '\t\tasm volatile("%s" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(kk) : "vcc");' % "\\n".join(lines)
    else:
        lines = [pat.format(r="%%%d" % j, k="%8") for j in range(8)]
        body = ('\t\tasm volatile("%s" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) '
                ': "v"(k) : "vcc", "s20", "s21", "s22", "s24", "s25", "s26");' % "\\n".join(lines))
    out.append(kern.format(i=i, body=body))
out.append(r'''
typedef void (*Kern)(unsigned long long*, uint32_t);
int main() {
	unsigned long long* d;
	hipMalloc(&d, 24);
''')
for i, (name, pat) in enumerate(OPS):
    out.append('\t{ const Kern f = bench_%d; const char* name = "%s";\n' % (i, name))
    out.append(r'''		printf("%-22s", name);
		for (int w : {1, 2, 4, 8}) {
			hipMemset(d, 0, 24);
			hipLaunchKernelGGL(f, dim3(256 * w), dim3(256), 0, 0, d, 7u);
			hipDeviceSynchronize();
			unsigned long long h[3];
			hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
			const double per_wave = (double)h[0] / (256.0 * 4 * w) / (8.0 * N_ITER);
			printf(" %d:%.2f", w, per_wave / w);
		}
		printf("\n");
	}
''')
out.append("\treturn 0;\n}\n")
pathlib.Path(__file__).with_name("valu_rates2.hip").write_text("".join(out))
