// Does gfx950 honour unaligned dword LDS and global accesses (SH_MEM_CONFIG alignment mode)?
// Each lane writes a marker dword at LDS byte offset 5 + 7 * lane and reads it back, and loads
// one dword from global memory at byte offset 1 + 3 * lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(const unsigned char* g, unsigned* out) {
	__shared__ unsigned char lds[1024];
	const int t = threadIdx.x;
	for (int i = t; i < 1024; i += 64) lds[i] = 0;
	__syncthreads();
	typedef __attribute__((address_space(3))) unsigned lu32;
	typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
	typedef __attribute__((address_space(3))) u32x2 lu64;
	lu32* p = (lu32*)(lds + 5 + 7 * t);
	if (t < 32) {
		unsigned v = 0xA0B0C0D0u + t;
		asm volatile("ds_write_b32 %0, %1" ::"v"(p), "v"(v) : "memory");
	}
	if (t == 40) {  // an 8-byte store at an odd address
		u32x2 v = {0x11223344u, 0x55667788u};
		asm volatile("ds_write_b64 %0, %1" ::"v"((lu64*)(lds + 801)), "v"(v) : "memory");
	}
	__syncthreads();
	unsigned r = 0;
	if (t < 32) asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(p) : "memory");
	out[t] = r;
	if (t == 40) {
		u32x2 v;
		asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((lu64*)(lds + 801)) : "memory");
		out[192] = v.x, out[193] = v.y, out[194] = lds[801] | lds[802] << 8 | lds[803] << 16 | (unsigned)lds[804] << 24;
	}
	out[64 + t] = *(const volatile unsigned*)(g + 1 + 3 * t);
	out[128 + t] = lds[5 + 7 * (t & 31) + (t >> 5)];
}
int main() {
	unsigned char h[256];
	for (int i = 0; i < 256; i++) h[i] = (unsigned char)i;
	unsigned char* g; unsigned* o; unsigned ho[200];
	hipMalloc(&g, 256); hipMalloc(&o, 200 * 4);
	hipMemcpy(g, h, 256, hipMemcpyHostToDevice);
	hipLaunchKernelGGL(k, 1, 64, 0, 0, g, o);
	hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
	int bad_lds = 0, bad_g = 0;
	for (int t = 0; t < 32; t++) bad_lds += ho[t] != 0xA0B0C0D0u + t;
	for (int t = 0; t < 64; t++) { unsigned e = h[1+3*t] | h[2+3*t] << 8 | h[3+3*t] << 16 | (unsigned)h[4+3*t] << 24; bad_g += ho[64+t] != e; }
	printf("lds unaligned dword mismatches %d (lane0 %08x byte0 %02x byte1 %02x), global unaligned load mismatches %d (lane0 %08x)\n", bad_lds, ho[0], ho[128], ho[160], bad_g, ho[64]);
	printf("ds b64 at odd address: %08x %08x (bytes 801..804 = %08x; expect 11223344 55667788 11223344)\n", ho[192], ho[193], ho[194]);
	return 0;
}
