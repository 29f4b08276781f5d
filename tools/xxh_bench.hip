// Micro-benchmark of the serial XXH32 round chain on gfx950 (diagnostic).
// hipcc --offload-arch=gfx950 -O3 tools/xxh_bench.hip -o tools/_build/xxh_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u;
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// A: 4 accumulators in lanes 0-3 (vector), data pre-multiplied
__global__ void kA(const uint32_t* __restrict__ d, uint64_t nwords, uint32_t* out)
{
	const uint32_t lane = threadIdx.x & 63;
	uint32_t acc = lane;
	for (uint64_t w = 0; w < nwords; w += 64 * 16) {
		uint32_t v[16];
#pragma unroll
		for (int r = 0; r < 16; ++r) v[r] = d[w + r * 64 + lane] * P2;
#pragma unroll
		for (int r = 0; r < 16; ++r) {
#pragma unroll
			for (int k = 0; k < 16; ++k) {
				const uint32_t x = __shfl(v[r], 4 * k + (lane & 3));
				acc = rotl(acc + x, 13) * P1;
			}
		}
	}
	out[threadIdx.x] = acc;
}

// B: scalar chains (4 accumulators in SGPRs), data via scalar loads
__global__ void kB(const uint32_t* __restrict__ d, uint64_t nwords, uint32_t* out)
{
	uint32_t a0 = 1, a1 = 2, a2 = 3, a3 = 4;
	for (uint64_t w = 0; w < nwords; w += 16) {
		const uint32_t* q = d + w;
		uint32_t x[16];
#pragma unroll
		for (int k = 0; k < 16; ++k) x[k] = __builtin_nontemporal_load(q + k);
#pragma unroll
		for (int k = 0; k < 16; k += 4) {
			a0 = rotl(a0 + x[k] * P2, 13) * P1;
			a1 = rotl(a1 + x[k + 1] * P2, 13) * P1;
			a2 = rotl(a2 + x[k + 2] * P2, 13) * P1;
			a3 = rotl(a3 + x[k + 3] * P2, 13) * P1;
		}
	}
	if (threadIdx.x == 0) out[0] = a0 ^ a1 ^ a2 ^ a3;
}

// C: like A but the multiply by P1 from 24-bit multiplies
__device__ __forceinline__ uint32_t mulP1(uint32_t r)
{
	constexpr uint32_t pl = P1 & 0xffffffu, ph = P1 >> 24;
	const uint32_t t0 = __umul24(r, pl);
	const uint32_t t1 = __umul24(r, ph) + __umul24(r >> 24, pl);
	return t0 + (t1 << 24);
}
__global__ void kC(const uint32_t* __restrict__ d, uint64_t nwords, uint32_t* out)
{
	const uint32_t lane = threadIdx.x & 63;
	uint32_t acc = lane;
	for (uint64_t w = 0; w < nwords; w += 64 * 16) {
		uint32_t v[16];
#pragma unroll
		for (int r = 0; r < 16; ++r) v[r] = d[w + r * 64 + lane] * P2;
#pragma unroll
		for (int r = 0; r < 16; ++r) {
#pragma unroll
			for (int k = 0; k < 16; ++k) {
				const uint32_t x = __shfl(v[r], 4 * k + (lane & 3));
				acc = mulP1(rotl(acc + x, 13));
			}
		}
	}
	out[threadIdx.x] = acc;
}

int main()
{
	const uint64_t bytes = 256ull << 20;
	uint32_t *d, *out;
	hipMalloc(&d, bytes);
	hipMalloc(&out, 4096);
	hipMemset(d, 1, bytes);
	const char* names[] = {"A vector lanes0-3 mul_lo", "B scalar 4 chains", "C vector mul24"};
	for (int m = 0; m < 3; ++m) {
		for (int rep = 0; rep < 2; ++rep) {
			hipEvent_t e0, e1;
			hipEventCreate(&e0);
			hipEventCreate(&e1);
			hipEventRecord(e0);
			if (m == 0) hipLaunchKernelGGL(kA, dim3(1), dim3(64), 0, 0, d, bytes / 4, out);
			if (m == 1) hipLaunchKernelGGL(kB, dim3(1), dim3(64), 0, 0, d, bytes / 4, out);
			if (m == 2) hipLaunchKernelGGL(kC, dim3(1), dim3(64), 0, 0, d, bytes / 4, out);
			hipEventRecord(e1);
			hipEventSynchronize(e1);
			float ms;
			hipEventElapsedTime(&ms, e0, e1);
			if (rep) printf("%-28s %8.2f ms  %6.2f GB/s\n", names[m], ms, bytes / ms / 1e6);
		}
	}
	return 0;
}
