// xxh_latency.hip -- dependent-chain latency of the XXH32 round's three
// VALU steps on gfx950 (is ~55 cycles per stripe the
// instruction latencies?).  One wave per kernel; each chain is N dependent
// steps timed with clock64(); printed as cycles per step.
//   hipcc --offload-arch=gfx950 -O3 -o xxh_latency tools/xxh_latency.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u;
constexpr int N = 4096;

template <int OP>
__global__ void k_chain(uint32_t seed, uint32_t* out, unsigned long long* cyc)
{
	uint32_t acc = seed + threadIdx.x, w = seed * 3u + threadIdx.x;
	const unsigned long long r0 = wall_clock64();
	const unsigned long long t0 = clock64();
#pragma unroll 16
	for (int i = 0; i < N; ++i) {
		if (OP == 0)  // the full round: acc = rotl(acc + w * P2, 13) * P1
			acc = __builtin_amdgcn_alignbit(acc + w * P2, acc + w * P2, 19) * P1;
		else if (OP == 1)  // v_add_u32 chain
			acc = acc + w;
		else if (OP == 2)  // v_alignbit_b32 chain (the rotate)
			acc = __builtin_amdgcn_alignbit(acc, acc, 19);
		else  // v_mul_lo_u32 chain
			acc = acc * P1;
		asm volatile("" : "+v"(acc));
	}
	const unsigned long long t1 = clock64();
	const unsigned long long r1 = wall_clock64();
	out[threadIdx.x] = acc;
	if (threadIdx.x == 0) {
		cyc[0] = t1 - t0;
		cyc[1] = r1 - r0;
	}
}

// Issue cost: eight independent chains per lane (enough to cover latency),
// so cycles per step / 8 is one wave64 instruction's issue time.
template <int OP>
__global__ void k_ilp(uint32_t seed, uint32_t* out, unsigned long long* cyc)
{
	uint32_t a[8];
#pragma unroll
	for (int j = 0; j < 8; ++j)
		a[j] = seed + threadIdx.x + 77u * j;
	const uint32_t w = seed * 3u + threadIdx.x;
	const unsigned long long r0 = wall_clock64();
#pragma unroll 4
	for (int i = 0; i < N; ++i) {
#pragma unroll
		for (int j = 0; j < 8; ++j) {
			if (OP == 1)
				a[j] = a[j] + w;
			else if (OP == 2)
				a[j] = __builtin_amdgcn_alignbit(a[j], a[j], 19);
			else
				a[j] = a[j] * P1;
		}
#pragma unroll
		for (int j = 0; j < 8; ++j)
			asm volatile("" : "+v"(a[j]));
	}
	const unsigned long long r1 = wall_clock64();
	uint32_t x = 0;
#pragma unroll
	for (int j = 0; j < 8; ++j)
		x ^= a[j];
	out[threadIdx.x] = x;
	if (threadIdx.x == 0)
		cyc[1] = r1 - r0;
}

int main()
{
	uint32_t* d_out;
	unsigned long long* d_c;
	if (hipMalloc(&d_out, 256) != hipSuccess || hipMalloc(&d_c, 16) != hipSuccess)
		return 1;
	int wall_khz = 0, clk_khz = 0;
	(void)hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0);
	(void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
	printf("wall clock %d kHz, peak shader clock %d kHz\n", wall_khz, clk_khz);
	const char* names[4] = { "round (add+mul, alignbit, mul)", "v_add_u32", "v_alignbit_b32", "v_mul_lo_u32" };
	for (int rep = 0; rep < 2; ++rep) {
		for (int op = 0; op < 4; ++op) {
			switch (op) {
			case 0: hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, 7u, d_out, d_c); break;
			case 1: hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, 7u, d_out, d_c); break;
			case 2: hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, 7u, d_out, d_c); break;
			default: hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(64), 0, 0, 7u, d_out, d_c); break;
			}
			unsigned long long c[2] = { 0, 0 };
			if (hipMemcpy(c, d_c, 16, hipMemcpyDeviceToHost) != hipSuccess)
				return 1;
			if (rep)
				printf("%-32s %.2f clock64 ticks per step, %.2f ns per step (%.1f cycles at the peak clock)\n",
				       names[op], double(c[0]) / N, 1e6 * double(c[1]) / wall_khz / N,
				       1e6 * double(c[1]) / wall_khz / N * clk_khz * 1e-6);
		}
	}
	for (int rep = 0; rep < 2; ++rep) {
		for (int op = 1; op < 4; ++op) {
			switch (op) {
			case 1: hipLaunchKernelGGL(k_ilp<1>, dim3(1), dim3(64), 0, 0, 7u, d_out, d_c); break;
			case 2: hipLaunchKernelGGL(k_ilp<2>, dim3(1), dim3(64), 0, 0, 7u, d_out, d_c); break;
			default: hipLaunchKernelGGL(k_ilp<3>, dim3(1), dim3(64), 0, 0, 7u, d_out, d_c); break;
			}
			unsigned long long c[2] = { 0, 0 };
			if (hipMemcpy(c, d_c, 16, hipMemcpyDeviceToHost) != hipSuccess)
				return 1;
			if (rep)
				printf("issue %-26s %.2f cycles per wave64 instruction (8 independent chains)\n", names[op],
				       1e6 * double(c[1]) / wall_khz / N / 8 * clk_khz * 1e-6);
		}
	}
	return 0;
}
