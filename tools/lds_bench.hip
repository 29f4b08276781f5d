// Micro-benchmark of LDS access shapes on gfx950 (diagnostic tool).
// hipcc --offload-arch=gfx950 -O3 tools/lds_bench.hip -o tools/_build/lds_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512) void k(uint32_t* out, uint32_t seed, int iters, unsigned long long* cyc)
{
	__shared__ __attribute__((aligned(16))) uint8_t buf[65536 + 64];
	for (int i = threadIdx.x; i < 65536 / 4; i += 512)
		reinterpret_cast<uint32_t*>(buf)[i] = i * 2654435761u;
	__syncthreads();
	uint32_t x = seed ^ (threadIdx.x * 7919u);
	uint32_t acc = 0;
	const uint64_t t0 = __builtin_amdgcn_s_memtime();
	for (int it = 0; it < iters; ++it) {
		x = x * 1664525u + 1013904223u;
		uint32_t a = (x >> 8) & 65535u;
		a = (a + acc) & 65535u;  // dependent chain
		if (MODE == 0) {  // ds_read_u8
			acc += buf[a];
		} else if (MODE == 1) {  // aligned b128
			u32x4 v = *reinterpret_cast<const u32x4*>(buf + (a & ~15u));
			acc += v.x ^ v.w;
		} else if (MODE == 2) {  // unaligned b128 via memcpy
			u32x4 v;
			__builtin_memcpy(&v, buf + a, 16);
			acc += v.x ^ v.w;
		} else if (MODE == 3) {  // two aligned b64 + alignbyte
			const uint32_t al = a & ~7u;
			uint64_t w0, w1, w2;
			__builtin_memcpy(&w0, buf + al, 8);
			w1 = *reinterpret_cast<const uint64_t*>(buf + al + 8);
			w2 = *reinterpret_cast<const uint64_t*>(buf + al + 16);
			const uint32_t sh = (a & 7u) * 8;
			const uint64_t lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
			const uint64_t hi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
			acc += uint32_t(lo) ^ uint32_t(hi >> 32);
		} else if (MODE == 4) {  // unaligned b128 store then aligned read
			u32x4 v = {x, x + 1, x + 2, x + 3};
			__builtin_memcpy(buf + a, &v, 16);
			acc += buf[a + 3];
		} else if (MODE == 6) {  // two aligned b128 + funnel shift
			const uint32_t al = a & ~15u;
			const u32x4 v0 = *reinterpret_cast<const u32x4*>(buf + al);
			const u32x4 v1 = *reinterpret_cast<const u32x4*>(buf + al + 16);
			const uint32_t r = a & 15u;
			uint32_t d[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
			const uint32_t q = r >> 2, sh = (r & 3u) * 8;
			uint32_t o[4];
#pragma unroll
			for (int j = 0; j < 4; ++j) {
				uint32_t lo = d[j], hi = d[j + 1];
#pragma unroll
				for (int k = 1; k < 4; ++k) {
					lo = (q == uint32_t(k)) ? d[j + k] : lo;
					hi = (q == uint32_t(k)) ? d[j + k + 1] : hi;
				}
				o[j] = __builtin_amdgcn_alignbyte(hi, lo, sh);
			}
			acc += o[0] ^ o[3];
		} else if (MODE == 7) {  // 16 independent u8 reads
			uint32_t t = 0;
#pragma unroll
			for (int j = 0; j < 16; ++j)
				t += uint32_t(buf[a + j]) << (j & 3);
			acc += t;
		} else if (MODE == 8) {  // 16-byte store as aligned pieces
			uint64_t lo = x, hi = x + 7;
			uint32_t d = a;
			int n = 16;
			uint8_t* p = buf;
			if (d & 1) { p[d] = uint8_t(lo); lo = (lo >> 8) | (hi << 56); hi >>= 8; d += 1; n -= 1; }
			if ((d & 2) && n >= 2) { *reinterpret_cast<uint16_t*>(p + d) = uint16_t(lo); lo = (lo >> 16) | (hi << 48); hi >>= 16; d += 2; n -= 2; }
			if ((d & 4) && n >= 4) { *reinterpret_cast<uint32_t*>(p + d) = uint32_t(lo); lo = (lo >> 32) | (hi << 32); hi >>= 32; d += 4; n -= 4; }
			if ((d & 8) && n >= 8) { *reinterpret_cast<uint64_t*>(p + d) = lo; lo = hi; hi = 0; d += 8; n -= 8; }
			if (n >= 8) { *reinterpret_cast<uint64_t*>(p + d) = lo; lo = hi; d += 8; n -= 8; }
			if (n >= 4) { *reinterpret_cast<uint32_t*>(p + d) = uint32_t(lo); lo >>= 32; d += 4; n -= 4; }
			if (n >= 2) { *reinterpret_cast<uint16_t*>(p + d) = uint16_t(lo); lo >>= 16; d += 2; n -= 2; }
			if (n >= 1) { p[d] = uint8_t(lo); }
			acc += buf[a + 3];
		} else if (MODE == 9) {  // 16 x ds_write_b8
#pragma unroll
			for (int j = 0; j < 16; ++j)
				buf[a + j] = uint8_t(x >> j);
			acc += buf[a + 3];
		} else if (MODE == 10) {  // 16-byte store as 4 ds_write_b32 at any alignment
			const uint32_t la = uint32_t(reinterpret_cast<uintptr_t>(buf + a));
			asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %0, %2 offset:4\n\tds_write_b32 %0, %3 offset:8\n\tds_write_b32 %0, %4 offset:12"
			             ::"v"(la), "v"(x), "v"(x + 1), "v"(x + 2), "v"(x + 3) : "memory");
			acc += buf[a + 3];
		} else if (MODE == 5) {  // aligned b128 store
			u32x4 v = {x, x + 1, x + 2, x + 3};
			*reinterpret_cast<u32x4*>(buf + (a & ~15u)) = v;
			acc += buf[(a & ~15u) + 3];
		}
	}
	const uint64_t t1 = __builtin_amdgcn_s_memtime();
	out[blockIdx.x * 512 + threadIdx.x] = acc;
	if (threadIdx.x == 0)
		atomicAdd(cyc, (unsigned long long)(t1 - t0));
}

int main()
{
	uint32_t* out;
	unsigned long long* cyc;
	hipMalloc(&out, 256 * 2 * 512 * 4);
	hipMalloc(&cyc, 8);
	const char* names[] = {"u8", "b128 aligned", "b128 unaligned (memcpy)", "2x b64 + shift", "st b128 unaligned + u8", "st b128 aligned + u8", "2x b128 aligned + funnel", "16x u8 reads", "st 16B aligned pieces + u8", "st 16x b8 + u8", "st 4x b32 any-align + u8"};
	const int iters = 4096;
	for (int m = 0; m < 11; ++m) {
		for (int rep = 0; rep < 2; ++rep) {
			hipMemset(cyc, 0, 8);
			hipEvent_t e0, e1;
			hipEventCreate(&e0);
			hipEventCreate(&e1);
			hipEventRecord(e0);
			switch (m) {
			case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 3: hipLaunchKernelGGL(k<3>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 4: hipLaunchKernelGGL(k<4>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 5: hipLaunchKernelGGL(k<5>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 6: hipLaunchKernelGGL(k<6>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 7: hipLaunchKernelGGL(k<7>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 8: hipLaunchKernelGGL(k<8>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 9: hipLaunchKernelGGL(k<9>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			case 10: hipLaunchKernelGGL(k<10>, dim3(256), dim3(512), 0, 0, out, 1u, iters, cyc); break;
			}
			hipEventRecord(e1);
			hipEventSynchronize(e1);
			float ms;
			hipEventElapsedTime(&ms, e0, e1);
			unsigned long long c;
			hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
			if (rep)
				printf("%-28s %8.3f ms  %8.1f cyc/iter (per wave, dependent chain, 8 waves/CU)\n", names[m], ms,
				       double(c) / 256 / iters);
		}
	}
	return 0;
}
