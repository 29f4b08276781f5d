// lz4ada_dev.h -- device helpers shared by the gfx950 kernels
// (lz4ada_kernels.hip: per-wave decoder, XXH32, exact serial path;
// lz4ada_wg.hip: workgroup-per-block decoder).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lz4ada {

// Device code addresses HBM through address_space(1) pointers so that every
// access is a global_* instruction (a generic pointer becomes flat_*, which
// also ticks lgkmcnt and forces extra waits).
#define GLOBAL __attribute__((address_space(1)))
typedef const GLOBAL uint8_t cg8;
typedef GLOBAL uint8_t g8;
typedef const GLOBAL uint32_t cg32;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ __forceinline__ const GLOBAL T* gptr(const T* p)
{
	return (const GLOBAL T*)(p);
}
template <class T>
__device__ __forceinline__ GLOBAL T* gptr(T* p)
{
	return (GLOBAL T*)(p);
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r)
{
	return (x << r) | (x >> (32 - r));
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Unaligned little-endian dword from global memory.  Reads only the aligned
// dwords that contain wanted bytes, so it never touches a page the data
// does not.
__device__ __forceinline__ uint32_t ld32u_cached(cg8* p)
{
	uintptr_t a = reinterpret_cast<uintptr_t>(p);
	cg32* q = reinterpret_cast<cg32*>(a & ~uintptr_t(3));
	uint32_t sh = uint32_t(a & 3u);
	uint32_t lo = q[0];
	if (sh == 0)
		return lo;
	uint32_t hi = q[1];
	return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Inclusive prefix sum over the wave with DPP (row_shr within 16-lane rows,
// then row_bcast:15 / row_bcast:31 across rows) -- VALU latency, no LDS.
__device__ __forceinline__ int32_t wave_incl_scan(int32_t v)
{
	v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
	v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
	v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
	v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
	v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false); // row_bcast:15
	v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false); // row_bcast:31
	return v;
}

// Inclusive prefix maximum over the wave (values >= 0), DPP as wave_incl_scan.
__device__ __forceinline__ int32_t wave_incl_max(int32_t v)
{
	v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));   // row_shr:1
	v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));   // row_shr:2
	v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));   // row_shr:4
	v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));   // row_shr:8
	v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
	v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
	return v;
}

__device__ __forceinline__ void wave_lds_fence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ void lds_store_n(uint8_t* dst, u32x4 v, int32_t n)
{
	if (n >= 16) {
		__builtin_memcpy(dst, &v, 16);
		return;
	}
	uint64_t lo = uint64_t(v.x) | (uint64_t(v.y) << 32);
	uint64_t hi = uint64_t(v.z) | (uint64_t(v.w) << 32);
	if (n & 8) {
		__builtin_memcpy(dst, &lo, 8);
		dst += 8;
		lo = hi;
	}
	if (n & 4) {
		const uint32_t x = uint32_t(lo);
		__builtin_memcpy(dst, &x, 4);
		dst += 4;
		lo >>= 32;
	}
	if (n & 2) {
		const uint16_t x = uint16_t(lo);
		__builtin_memcpy(dst, &x, 2);
		dst += 2;
		lo >>= 16;
	}
	if (n & 1)
		*dst = uint8_t(lo);
}

// 16 bytes at byte address a of an LDS array of `size` bytes (a multiple
// of 16, wrapping): two aligned ds_read_b128 and a funnel shift -- an
// unaligned ds_read_b128 is split into byte accesses (tools/lds_bench.hip:
// 512 vs 214 cycles per dependent access at 8 waves/CU).
__device__ __forceinline__ u32x4 ld16u(const uint8_t* base, uint32_t a, uint32_t size)
{
	const uint32_t al = a & ~15u;
	uint32_t al1 = al + 16;
	al1 = (al1 >= size) ? al1 - size : al1;
	const u32x4 v0 = *reinterpret_cast<const u32x4*>(base + al);
	const u32x4 v1 = *reinterpret_cast<const u32x4*>(base + al1);
	const uint32_t r = a & 15u;
	const uint32_t q = r >> 2, sh = r & 3u;  // v_alignbyte shifts by bytes
	const uint32_t d[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
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
	u32x4 v;
	v.x = o[0];
	v.y = o[1];
	v.z = o[2];
	v.w = o[3];
	return v;
}

// Period-off (< 16) match pattern: from the off source bytes (s0 = bytes
// 0..7, s1 = bytes 8..15 of the source window) build the phase-0 pattern
// pv; storing it every *stp bytes (*width bytes per store, the last store
// clipped) writes the whole match -- overlapping stores write equal bytes.
__device__ __forceinline__ void make_pattern(uint64_t s0, uint64_t s1, int32_t off, u32x4& pv,
                                             int32_t& width, int32_t& stp)
{
	if (off <= 8) {
		uint64_t x = off == 8 ? s0 : (s0 & ((uint64_t(1) << (8 * off)) - 1));
		for (int32_t w = off; w < 8; w <<= 1)
			x |= x << (8 * w);
		pv.x = uint32_t(x);
		pv.y = uint32_t(x >> 32);
		pv.z = pv.x;
		pv.w = pv.y;
		width = 8;
		stp = off * (8 / off);
	} else {
		// bytes 0..off-1 = source, off..15 = source bytes 0..15-off
		const int32_t r = off - 8;
		const uint64_t hi = (s1 & ((uint64_t(1) << (8 * r)) - 1)) | (s0 << (8 * r));
		pv.x = uint32_t(s0);
		pv.y = uint32_t(s0 >> 32);
		pv.z = uint32_t(hi);
		pv.w = uint32_t(hi >> 32);
		width = 16;
		stp = off;
	}
}

}  // namespace lz4ada
