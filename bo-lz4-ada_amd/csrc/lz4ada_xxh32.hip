// lz4ada_xxh32.hip -- gfx950 XXH32 kernels of the MI355X LZ4Ada decompressor.
//
// Replaces Check_Checksum / Update_Checksum / XXHash32 (lib/lz4ada.adb
// :698-714, :923-1026):
//  * k_xxh32_rows -- per-block XXH32 (block checksums, output hashes), four
//    blocks per wave, the chain walking a 16-lane row's quads by DPP.
//  * k_xxh32_update -- streaming XXH32 of one buffer with the four
//    accumulator lanes mapped onto lanes 0-3 of a wavefront; all 64 lanes
//    load and pre-multiply 256 B per step, ds_bpermute feeds the chain.
// Its own file so it can take its own machine-scheduler strategy
// (csrc/Makefile).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4ada_internal.h"
#include "lz4ada_dev.h"

namespace lz4ada {

// ------------------------------------------------------------------ XXH32




constexpr int XR = 16;  // dwords per lane per step (4 KiB per wave)

// Load step w0's raw dwords: word w of the stream starts at byte 4w, `sh`
// bytes into aligned dword q[w].  With sh != 0 a word straddles q[w] and
// q[w+1], both holding wanted bytes (no overread).  The alignbyte happens
// at use, so the loads stay in flight.
template <bool MIS, bool GUARD>
__device__ __forceinline__ void xxh_load(uint32_t (&lo)[XR], uint32_t (&hi)[XR], cg32* q,
                                         uint64_t w0, uint64_t nwords)
{
	const uint32_t lane = lane_id();
#pragma unroll
	for (int r = 0; r < XR; ++r) {
		const uint64_t w = w0 + uint64_t(r) * 64 + lane;
		const uint64_t wl = (!GUARD || w < nwords) ? w : 0;
		lo[r] = __builtin_nontemporal_load(q + wl);
		if (MIS)
			hi[r] = __builtin_nontemporal_load(q + wl + 1);
	}
}

// 16 chain steps over the stripes held in one register of the step.
__device__ __forceinline__ uint32_t xxh_chain16(uint32_t acc, uint32_t word, int64_t limit)
{
	const uint32_t lane = lane_id();
	const uint32_t prod = word * P2;
	uint32_t xs[16];
#pragma unroll
	for (int k = 0; k < 16; ++k)
		xs[k] = __shfl(prod, 4 * k + int(lane & 3u));
	if (limit >= 16) {
#pragma unroll
		for (int k = 0; k < 16; ++k)
			acc = rotl32(acc + xs[k], 13) * P1;
	} else {
#pragma unroll
		for (int k = 0; k < 16; ++k)
			if (k < limit)
				acc = rotl32(acc + xs[k], 13) * P1;
	}
	return acc;
}

template <bool MIS>
__device__ uint32_t xxh32_stripes_impl(uint32_t acc, cg32* q, uint32_t sh, uint64_t nstripes)
{
	const uint64_t nwords = nstripes * 4;
	constexpr uint64_t STEP = 64 * XR;
	const uint64_t full = nwords / STEP * STEP;  // words covered by whole steps
	uint32_t clo[XR], chi[XR], nlo[XR], nhi[XR];
	if (full)
		xxh_load<MIS, false>(clo, chi, q, 0, nwords);
	for (uint64_t w0 = 0; w0 < full; w0 += STEP) {
		// issue the next step's loads first; they land while the chain runs
		if (w0 + STEP < full)
			xxh_load<MIS, false>(nlo, nhi, q, w0 + STEP, nwords);
#pragma unroll
		for (int r = 0; r < XR; ++r) {
			const uint32_t word = MIS ? __builtin_amdgcn_alignbyte(chi[r], clo[r], sh) : clo[r];
			acc = xxh_chain16(acc, word, 16);
		}
#pragma unroll
		for (int r = 0; r < XR; ++r) {
			clo[r] = nlo[r];
			if (MIS)
				chi[r] = nhi[r];
		}
	}
	if (full < nwords) {  // ragged last step
		xxh_load<MIS, true>(clo, chi, q, full, nwords);
		const int64_t left = int64_t((nwords - full) / 4);
#pragma unroll
		for (int r = 0; r < XR; ++r) {
			const uint32_t word = MIS ? __builtin_amdgcn_alignbyte(chi[r], clo[r], sh) : clo[r];
			acc = xxh_chain16(acc, word, left - 16 * r);
		}
	}
	return acc;
}

// Advance the four XXH32 accumulators over `nstripes` 16-byte stripes at p
// (Process, lz4ada.adb:979-991).  Whole-wave call; lane l carries
// accumulator (l & 3).  The chain is serial: all 64 lanes load 4 KiB per
// step one step ahead of it, and ds_bpermute hands stripe k's four
// pre-multiplied words to lanes 0-3.
__device__ uint32_t wave_xxh32_stripes(uint32_t acc, cg8* p, uint64_t nstripes)
{
	const uintptr_t a = reinterpret_cast<uintptr_t>(p);
	cg32* q = reinterpret_cast<cg32*>(a & ~uintptr_t(3));
	const uint32_t sh = uint32_t(a & 3u);
	return sh ? xxh32_stripes_impl<true>(acc, q, sh, nstripes)
	          : xxh32_stripes_impl<false>(acc, q, 0, nstripes);
}

// XXHash32.Final (lz4ada.adb:993-1017) from the 4 lanes + tail buffer.
__device__ uint32_t xxh32_final_dev(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3,
                                    const uint8_t* buf, int32_t bufsize, uint64_t total)
{
	uint32_t ret = uint32_t(total & 0xffffffffu);
	if (total >= 16)
		ret += rotl32(v0, 1) + rotl32(v1, 7) + rotl32(v2, 12) + rotl32(v3, 18);
	else
		ret += v2 + P5;
	int d = 0;
	while (d + 3 < bufsize) {
		uint32_t w = uint32_t(buf[d]) | (uint32_t(buf[d + 1]) << 8) |
		             (uint32_t(buf[d + 2]) << 16) | (uint32_t(buf[d + 3]) << 24);
		ret = rotl32(ret + w * P3, 17) * P4;
		d += 4;
	}
	while (d < bufsize) {
		ret = rotl32(ret + uint32_t(buf[d]) * P5, 11) * P1;
		d += 1;
	}
	ret = (ret ^ (ret >> 15)) * P2;
	ret = (ret ^ (ret >> 13)) * P3;
	return ret ^ (ret >> 16);
}

// ------------------------------------------------- XXH32, four blocks a wave
// The stripe chain is serial (acc = rotl(acc + w P2, 13) P1: three dependent
// VALU ops), so one block per wave leaves 60 of 64 lanes idle.
// k_xxh32_rows gives each 16-lane row its own block.  Lane 4m + a of a row
// loads word a of stripe 4t + m (register t: 16 consecutive words), so the
// row's four quads hold four consecutive stripes.  The chain walks the
// quads: sub-step k updates acc := rotl(ror4(acc) + x, 13) P1 in every lane,
// ror4 (DPP row_ror:4) handing quad k the accumulators quad k - 1 produced
// one sub-step earlier; only quad k's result is the chain's, the other quads
// compute values nobody reads.  No shuffles, no LDS: three VALU per stripe
// for four blocks.  Loads run XW registers ahead of the chain.  (Inline-asm
// loads with hand-counted waits were tried and dropped: the compiler may
// copy an asm load's destination before the data lands -- it faulted.)
constexpr int XG = 4;    // blocks per wave (16-lane rows)
#ifndef LZ4ADA_XW
#define LZ4ADA_XW 48
#endif
constexpr int XW = LZ4ADA_XW;  // registers in flight (vmcnt holds 63)

struct XRow {
	cg32* q;       // aligned-down start (a valid address even for an empty row)
	uint32_t sh;   // start misalignment, bytes
	int32_t nw;    // words in whole stripes
	int32_t dlast; // last whole-stripe word when sh == 0: its pair starts one word early
};

__device__ __forceinline__ int32_t xrow_w(const XRow& R, int32_t t)
{
	return min(16 * t + int32_t(lane_id() & 15u), max(R.nw - 1, 0));
}

// Register t's pair for this lane, clamped to the row's data: aligned dwords
// q[w], q[w + 1] -- for an aligned start's last word (q[w + 1] could pass the
// data's last page) q[w - 1], q[w].
__device__ __forceinline__ uint64_t xrow_load(const XRow& R, int32_t t)
{
	const int32_t w = xrow_w(R, t);
	uint64_t v;
	__builtin_memcpy(&v, R.q + (w - (w == R.dlast ? 1 : 0)), 8);
	return v;
}

__device__ __forceinline__ uint32_t xrow_word(const XRow& R, int32_t t, uint64_t v)
{
	const uint32_t lo = uint32_t(v), hi = uint32_t(v >> 32);
	return xrow_w(R, t) == R.dlast ? hi : __builtin_amdgcn_alignbyte(hi, lo, R.sh);
}

// Four sub-steps over register t's stripes (lim: how many of them are the
// row's; GUARD false: all four).
template <bool GUARD>
__device__ __forceinline__ uint32_t xrow_chain(uint32_t acc, uint32_t word, int32_t lim)
{
	const uint32_t x = word * P2;
#pragma unroll
	for (int k = 0; k < 4; ++k) {
		const uint32_t prev = uint32_t(__builtin_amdgcn_update_dpp(0, int(acc), 0x124, 0xf, 0xf, false));
		const uint32_t nacc = rotl32(prev + x, 13) * P1;  // row_ror:4 above
		acc = (!GUARD || k < lim) ? nacc : acc;
	}
	return acc;
}

// One round: consume registers t0 .. t0 + XW - 1, load t0 + XW .. t0 + 2 XW - 1.
__device__ __forceinline__ uint32_t xrow_round(const XRow& R, uint64_t (&buf)[XW], uint32_t acc,
                                               int32_t t0, int32_t tfull, int32_t tall)
{
#pragma unroll
	for (int r = 0; r < XW; ++r) {
		const int32_t t = t0 + r;
		const uint32_t word = xrow_word(R, t, buf[r]);
		// the slot's old pair dies before its next load is issued, so both
		// share registers: hoisted above the use, the load made the allocator
		// rotate all XW slots at the loop's back edge (XW copies behind a
		// vmcnt(0))
		__builtin_amdgcn_sched_barrier(0);
		buf[r] = xrow_load(R, t + XW);
		if (t < tfull)
			acc = xrow_chain<false>(acc, word, 4);
		else if (t < tall)
			acc = xrow_chain<true>(acc, word, (R.nw - 16 * t) >> 2);
	}
	return acc;
}

// XXH32 (seed 0, XXHash32.Hash: lz4ada.adb:979-1017) of row j's bytes
// [p, p + n); returned in the row's lane 0.  p may be null when n == 0
// (fallback: any valid device address).
__device__ __forceinline__ uint32_t xxh32_rows(cg8* p, uint64_t n, cg32* fallback)
{
	const uint32_t lane = lane_id();
	const uint64_t ns = n / 16;
	XRow R;
	if (ns == 0) {
		R.q = fallback;
		R.sh = 0;
		R.nw = 0;
	} else {
		const uintptr_t a = reinterpret_cast<uintptr_t>(p);
		R.q = reinterpret_cast<cg32*>(a & ~uintptr_t(3));
		R.sh = uint32_t(a & 3u);
		R.nw = int32_t(ns * 4);
	}
	R.dlast = (R.sh == 0 && R.nw > 0) ? R.nw - 1 : -1;
	int32_t tall = (R.nw + 15) >> 4, tfull = R.nw >> 4;
#pragma unroll
	for (int s = 16; s <= 32; s <<= 1) {
		tall = max(tall, __shfl_xor(tall, s));
		tfull = min(tfull, __shfl_xor(tfull, s));
	}
	tall = __builtin_amdgcn_readfirstlane(tall);  // wave-uniform: scalar loop bounds
	tfull = __builtin_amdgcn_readfirstlane(tfull);
	const uint32_t init[4] = { P1 + P2, P2, 0u, 0u - P1 };
	uint32_t acc = init[lane & 3u];  // every quad: sub-step 0 reads quad 3
	// settle the descriptor loads first: left pending into the chain loop,
	// the wait pass merges them into the loop head as a vmcnt(0) -- every
	// round, for the XW loads in flight too
	__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
	// the prologue in slot order (scheduled freely, it came out reversed,
	// and the loop head then waited vmcnt(0) for slot 0)
	uint64_t buf[XW];
#pragma unroll
	for (int r = 0; r < XW; ++r) {
		buf[r] = xrow_load(R, r);
		__builtin_amdgcn_sched_barrier(0);
	}
	for (int32_t t0 = 0; t0 < tall; t0 += XW)
		acc = xrow_round(R, buf, acc, t0, tfull, tall);
	// the chain's last sub-step ran in quad (ns - 1) mod 4
	const int src = int(lane & 48u) | int(((uint32_t(ns) + 3u) & 3u) << 2);
	const uint32_t v0 = __shfl(acc, src), v1 = __shfl(acc, src + 1), v2 = __shfl(acc, src + 2),
	               v3 = __shfl(acc, src + 3);
	uint32_t h = uint32_t(n);
	if ((lane & 15u) == 0) {
		h += n >= 16 ? rotl32(v0, 1) + rotl32(v1, 7) + rotl32(v2, 12) + rotl32(v3, 18) : P5;
		cg8* t = p + ns * 16;
		const int32_t tl = int32_t(n - ns * 16);
		int32_t d = 0;
		for (; d + 4 <= tl; d += 4) {
			const uint32_t w = uint32_t(t[d]) | (uint32_t(t[d + 1]) << 8) |
			                   (uint32_t(t[d + 2]) << 16) | (uint32_t(t[d + 3]) << 24);
			h = rotl32(h + w * P3, 17) * P4;
		}
		for (; d < tl; ++d)
			h = rotl32(h + uint32_t(t[d]) * P5, 11) * P1;
		h = (h ^ (h >> 15)) * P2;
		h = (h ^ (h >> 13)) * P3;
		h ^= h >> 16;
	}
	return h;
}

// out == nullptr: block checksums of the compressed data (blocks with
// B.Checksum; st[b].cksum).  Else: XXH32 of each block's decoded output
// (st[b].out_len bytes at out + out_off) into hash[b].
__global__ __launch_bounds__(64) void k_xxh32_rows(const uint8_t* __restrict__ frame,
                                                   const uint8_t* __restrict__ out,
                                                   const lz4ada_block_desc* __restrict__ desc,
                                                   uint32_t nblocks,
                                                   lz4ada_block_status* __restrict__ st,
                                                   uint32_t* __restrict__ hash)
{
	const uint32_t lane = lane_id();
	const uint32_t b = blockIdx.x * XG + (lane >> 4);
	cg8* p = nullptr;
	uint64_t n = 0;
	bool want = false;
	if (b < nblocks) {
		const lz4ada_block_desc d = desc[b];
		if (out) {
			p = gptr(out) + d.out_off;
			n = st[b].out_len;
			want = true;
		} else if (d.flags & LZ4ADA_BLOCK_HAS_CKSUM) {
			p = gptr(frame) + d.in_off;
			n = d.in_len;
			want = true;
		}
	}
	const uint32_t h = xxh32_rows(p, n, reinterpret_cast<cg32*>(gptr(desc)));
	if (want && (lane & 15u) == 0) {
		if (out)
			hash[b] = h;
		else
			st[b].cksum = h;
	}
}

// Streaming XXHash32.Update (lz4ada.adb:942-977) on a device-resident state.
__global__ __launch_bounds__(64) void k_xxh32_update(lz4ada_xxh32_state* __restrict__ s,
                                                      const uint8_t* __restrict__ data,
                                                      uint64_t len)
{
	const uint32_t lane = lane_id();
	uint32_t acc = s->state[lane & 3u];
	uint8_t buf[16];
	int32_t bs = s->buffer_size;
	for (int i = 0; i < 16; ++i)
		buf[i] = s->buffer[i];
	uint64_t total = s->total_length + len;
	uint64_t pos = 0;
	cg8* dg = gptr(data);
	// Refill a partially filled stripe byte by byte (Update1, :965-977).
	if (bs > 0) {
		while (bs < 16 && pos < len)
			buf[bs++] = dg[pos++];
		if (bs == 16) {
			uint32_t w = uint32_t(buf[4 * (lane & 3u)]) |
			             (uint32_t(buf[4 * (lane & 3u) + 1]) << 8) |
			             (uint32_t(buf[4 * (lane & 3u) + 2]) << 16) |
			             (uint32_t(buf[4 * (lane & 3u) + 3]) << 24);
			acc = rotl32(acc + w * P2, 13) * P1;
			bs = 0;
		}
	}
	if (bs == 0) {
		const uint64_t ns = (len - pos) / 16;
		acc = wave_xxh32_stripes(acc, dg + pos, ns);
		pos += ns * 16;
		while (pos < len)
			buf[bs++] = dg[pos++];
	}
	uint32_t v0 = __shfl(acc, 0), v1 = __shfl(acc, 1), v2 = __shfl(acc, 2), v3 = __shfl(acc, 3);
	uint32_t h = xxh32_final_dev(v0, v1, v2, v3, buf, bs, total);
	if (lane == 0) {
		s->state[0] = v0;
		s->state[1] = v1;
		s->state[2] = v2;
		s->state[3] = v3;
		for (int i = 0; i < 16; ++i)
			s->buffer[i] = buf[i];
		s->buffer_size = bs;
		s->total_length = total;
		s->hash = h;
	}
}

hipError_t launch_block_checksums(const uint8_t* d_frame, const lz4ada_block_desc* d_desc,
                                  uint32_t nblocks, lz4ada_block_status* d_status,
                                  hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(k_xxh32_rows, dim3((nblocks + XG - 1) / XG), dim3(64), 0, stream, d_frame,
	                   (const uint8_t*)nullptr, d_desc, nblocks, d_status, (uint32_t*)nullptr);
	return hipGetLastError();
}

hipError_t launch_output_checksums(const uint8_t* d_out, const lz4ada_block_desc* d_desc,
                                   uint32_t nblocks, const lz4ada_block_status* d_status,
                                   uint32_t* d_hash, hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(k_xxh32_rows, dim3((nblocks + XG - 1) / XG), dim3(64), 0, stream,
	                   (const uint8_t*)nullptr, d_out, d_desc, nblocks,
	                   const_cast<lz4ada_block_status*>(d_status), d_hash);
	return hipGetLastError();
}

hipError_t launch_xxh32_update(lz4ada_xxh32_state* d_state, const uint8_t* d_data, uint64_t len,
                               hipStream_t stream)
{
	hipLaunchKernelGGL(k_xxh32_update, dim3(1), dim3(64), 0, stream, d_state, d_data, len);
	return hipGetLastError();
}

}  // namespace lz4ada
