// lz4ada_sparse.hip -- bulk decoder for literal-heavy ("sparse") blocks.
//
// Same reference path as the index decoder (lib/lz4ada.adb:716-904:
// Decompress_Full_Block / Decompress_Sequence / Write_Output /
// Output_With_History), for the blocks its pass 1 declines because their
// sequences are too far apart for speculative walks to merge (long literal
// runs: incompressible text, mostly-stored content in compressed blocks).
// Such a block holds few sequences (~9k per 4 MiB at 470 B each) and is a
// copy job, so one wave per block:
//
//  * parse: the sequence chain walked wave-uniformly (scalar registers) over
//    a 16 KiB LDS ring the compressed stream is staged through in 4 KiB
//    coalesced chunks, one chunk prefetched in registers; sequence j of a
//    batch of 64 lands in lane j's registers;
//  * literals: groups of 8 runs, each copied by the whole wave (16 B per
//    lane, 2 KiB per run in one step), all loads of a group issued before
//    its stores: HBM -> HBM, no LDS;
//  * matches: lane j runs match j of the batch once no earlier match of the
//    batch writes a byte it reads (a dependency mask from two binary
//    searches over the batch's monotone match positions); the source is
//    read from the output already written (L1-bypassing loads after the
//    wave's stores have completed); a match reads only its first `off`
//    source bytes -- byte i is source byte i mod off -- so no piece reads
//    its own match.
//
// Anything unusual -- malformed data, a reference before the block start
// (D2), a slot overflow, or a chain denser than sparse data (one sequence
// per < 48 input bytes: the scalar parse would be slower than k_decode_pc)
// -- leaves the block DS_RETRY; k_decode_pc then redoes it and produces the
// exact statuses, so this kernel never changes a result, only the speed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4ada_internal.h"
#include "lz4ada_dev.h"

namespace lz4ada {
namespace sparse {

constexpr int STG = 2048;         // staged chunk (two LDS-DMA instructions)
constexpr int NSLOT = 8;          // ring slots
constexpr int RING = NSLOT * STG; // LDS ring of compressed bytes (16 KiB)
constexpr int DEPTH = 6;          // chunks in flight ahead of the parse
constexpr int NSEQ = 64;          // sequences per batch (one per lane)
constexpr int OWN = 2048;         // literal pieces (16 B) dealt per batch at most
constexpr int BIG = 4096;         // longer literal runs: copied by the whole wave
constexpr int LONGM = 512;        // longer matches: copied by the whole wave
constexpr int U = 8;              // pieces per lane in flight (8 KiB per wave)
constexpr int DENSE_BYTES = 48;   // fewer input bytes per sequence: decline

struct alignas(16) SpLds {
	uint8_t ring[RING];       // filled by LDS-DMA, STG-byte slots
	uint8_t own[OWN];         // piece t's sequence: marks at run starts, prefix max
	u32x4 rec[NSEQ];          // sequence j: src - 16 s_j, dst - 16 s_j, L + 16 s_j
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// 16 bytes from global memory at a, never reading at or past lim.
__device__ __forceinline__ u32x4 gload16(uintptr_t a, uintptr_t lim)
{
	u32x4 v;
	if (a + 16 <= lim) {
		__builtin_memcpy(&v, reinterpret_cast<cg8*>(a), 16);
	} else {
		uint8_t t[16];
		for (int i = 0; i < 16; ++i)
			t[i] = (a + i < lim) ? *reinterpret_cast<cg8*>(a + i) : 0;
		__builtin_memcpy(&v, t, 16);
	}
	return v;
}

// 16 bytes of the output already written (an earlier store of this wave,
// completed): nontemporal loads bypass the CU's L1, which may hold the line
// from before the store.  Never reads at or past olim (bytes there are 0:
// the callers use only bytes before the match, which lie below it).
__device__ __forceinline__ u32x4 oload16(const GLOBAL uint8_t* p, uintptr_t olim)
{
	const uintptr_t a = reinterpret_cast<uintptr_t>(p);
	const GLOBAL uint32_t* al = reinterpret_cast<const GLOBAL uint32_t*>(a & ~uintptr_t(3));
	const uint32_t sh = uint32_t(a & 3u);
	u32x4 v;
	if ((a & ~uintptr_t(3)) + 20 <= olim) {
		const uint32_t d0 = __builtin_nontemporal_load(al), d1 = __builtin_nontemporal_load(al + 1),
		               d2 = __builtin_nontemporal_load(al + 2), d3 = __builtin_nontemporal_load(al + 3),
		               d4 = sh ? __builtin_nontemporal_load(al + 4) : 0u;
		v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
		v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
		v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
		v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
		return v;
	}
	uint8_t t[16];
	for (int i = 0; i < 16; ++i)
		t[i] = (a + i < olim) ? __builtin_nontemporal_load(reinterpret_cast<const GLOBAL uint8_t*>(a + i))
		                      : uint8_t(0);
	__builtin_memcpy(&v, t, 16);
	return v;
}

// Exact-length store of n (0..16) bytes.
__device__ __forceinline__ void gstore_n(g8* dst, u32x4 v, int32_t n)
{
	if (n >= 16) {
		__builtin_memcpy(dst, &v, 16);
		return;
	}
	uint64_t lo = uint64_t(v.x) | (uint64_t(v.y) << 32);
	const uint64_t hi = uint64_t(v.z) | (uint64_t(v.w) << 32);
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

typedef unsigned __int128 u128;
__device__ __forceinline__ u128 to128(u32x4 v)
{
	return u128(v.x) | (u128(v.y) << 32) | (u128(v.z) << 64) | (u128(v.w) << 96);
}
__device__ __forceinline__ u32x4 from128(u128 x)
{
	u32x4 v;
	v.x = uint32_t(x);
	v.y = uint32_t(x >> 32);
	v.z = uint32_t(x >> 64);
	v.w = uint32_t(x >> 96);
	return v;
}

// Bytes [16k, 16k + 16) of a match of offset `off` whose source window
// [mdst - off, mdst) starts at src: byte i is source byte i mod off
// (Output_With_History's repeating copy, lz4ada.adb:892-903).  ph = 16k mod
// off; for off < 16, (plo, phi) = the source bytes repeated over 32 bytes.
__device__ __forceinline__ u32x4 match_piece(const GLOBAL uint8_t* src, int32_t off, int32_t ph,
                                             u128 plo, u128 phi, uintptr_t olim)
{
	if (off < 16) {
		if (ph == 0)
			return from128(plo);
		return from128((plo >> (8 * ph)) | (phi << (128 - 8 * ph)));
	}
	const u32x4 a = oload16(src + ph, olim);
	const int32_t na = off - ph;  // bytes of a before the window wraps
	if (na >= 16)
		return a;
	const u128 b = to128(oload16(src, olim));
	const u128 am = to128(a) & ((u128(1) << (8 * na)) - 1);
	return from128(am | (b << (8 * na)));
}

// Period pattern of a match with off < 16: 32 bytes of source byte i mod off,
// by doubling the off exact bytes (no private arrays: registers only).
__device__ __forceinline__ void make_pat(const GLOBAL uint8_t* src, int32_t off, uintptr_t olim,
                                         u128& lo, u128& hi)
{
	lo = to128(oload16(src, olim)) & ((u128(1) << (8 * off)) - 1);
	hi = 0;
	for (int32_t w = off; w < 32; w <<= 1) {
		const int32_t s = 8 * w;  // 8..248 bits
		u128 nlo, nhi;
		if (s < 128) {
			nlo = lo << s;
			nhi = (hi << s) | (lo >> (128 - s));
		} else {
			nlo = 0;
			nhi = s == 128 ? lo : (lo << (s - 128));
		}
		lo |= nlo;
		hi |= nhi;
	}
}

// One match of the batch (lane-local): ml bytes at ob + mdst from offset off.
__device__ __forceinline__ void run_match(g8* ob, int32_t mdst, int32_t off, int32_t ml,
                                          uintptr_t olim)
{
	const GLOBAL uint8_t* src = ob + (mdst - off);
	u128 plo = 0, phi = 0;
	if (off < 16)
		make_pat(src, off, olim, plo, phi);
	const int32_t d16 = off < 16 ? 16 % off : (off == 16 ? 0 : 16);
	int32_t ph = 0;
	for (int32_t i = 0; i < ml; i += 16) {
		gstore_n(ob + mdst + i, match_piece(src, off, ph, plo, phi, olim), min(16, ml - i));
		ph += d16;
		if (ph >= off)
			ph -= off;
	}
}

// One long match by the whole wave (uniform arguments): piece i of 16 bytes
// per lane, 1 KiB per instruction, U in flight.
__device__ __forceinline__ void run_match_wave(g8* ob, int32_t mdst, int32_t off, int32_t ml,
                                               uintptr_t olim)
{
	const GLOBAL uint8_t* src = ob + (mdst - off);
	u128 plo = 0, phi = 0;
	if (off < 16)
		make_pat(src, off, olim, plo, phi);
	const int32_t lane = int32_t(lane_id());
	for (int32_t c = 0; c < ml; c += 1024 * U) {
		u32x4 v[U];
#pragma unroll
		for (int u = 0; u < U; ++u) {
			const int32_t i = c + 1024 * u + 16 * lane;
			if (i < ml)
				v[u] = match_piece(src, off, int32_t(uint32_t(i) % uint32_t(off)), plo, phi, olim);
		}
#pragma unroll
		for (int u = 0; u < U; ++u) {
			const int32_t i = c + 1024 * u + 16 * lane;
			if (i < ml)
				gstore_n(ob + mdst + i, v[u], min(16, ml - i));
		}
	}
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_decode_sparse(const uint8_t* __restrict__ frame,
                                                      uint64_t frame_len,
                                                      const lz4ada_block_desc* __restrict__ desc,
                                                      uint32_t nblocks, uint8_t* __restrict__ out,
                                                      lz4ada_block_status* __restrict__ status)
{
	__shared__ SpLds S;
	const uint32_t b = blockIdx.x;
	if (b >= nblocks || status[b].code != DS_SPARSE)
		return;
	const int32_t lane = int32_t(lane_id());
	const lz4ada_block_desc d = desc[b];
	cg8* in = gptr(frame) + d.in_off;
	g8* ob = gptr(out) + d.out_off;
	const int32_t n = int32_t(d.in_len);
	const int32_t cap = int32_t(d.out_cap);
	const uintptr_t lim = reinterpret_cast<uintptr_t>(frame) + frame_len;
	const uintptr_t olim = reinterpret_cast<uintptr_t>(ob) + uintptr_t(cap);
	const int32_t mis = int32_t(reinterpret_cast<uintptr_t>(in) & 15u);
	const uintptr_t abase = reinterpret_cast<uintptr_t>(in) - uintptr_t(mis);

	// ---- staging: chunk c = aligned bytes [c STG, (c + 1) STG) from abase
	// goes to ring slot c % NSLOT by LDS-DMA (global_load_lds_dwordx4, 1 KiB
	// per instruction, no registers), DEPTH chunks ahead of the parse.  The
	// parse issues no other memory instruction, and every batch ends with
	// all memory settled, so "chunk c has landed" is vmcnt <= 2 (DEPTH - 1)
	// once chunks up to c + DEPTH - 1 are issued (in-order counter; extra
	// outstanding work only makes the wait longer, never short).
	const uint32_t ring_lds =
	    uint32_t(uintptr_t((__attribute__((address_space(3))) uint8_t*)(&S.ring[0])));
	int32_t issued = 0;  // chunks [0, issued) issued
	int32_t landed = 0;  // chunks [0, landed) known to be in LDS
	const int32_t nchunks = (n + mis + STG - 1) / STG;
	auto issue = [&](int32_t c) {
		// past the payload the chunk reads whatever follows in the frame,
		// clamped to the frame (its bytes are never used)
		uintptr_t g = abase + uintptr_t(c) * STG + 16u * uint32_t(lane);
#pragma unroll
		for (int r = 0; r < STG / 1024; ++r) {
			uintptr_t a = g + 1024u * r;
			if (a + 16 > lim)
				a = (lim - 16) & ~uintptr_t(15);
			const uint32_t l = uni(ring_lds + uint32_t(c % NSLOT) * STG + 1024u * r);
			uint32_t m0save;
			asm volatile(
			    "s_mov_b32 %0, m0\n\t"
			    "s_mov_b32 m0, %1\n\t"
			    "global_load_lds_dwordx4 %2, off\n\t"
			    "s_mov_b32 m0, %0"
			    : "=&s"(m0save)
			    : "s"(l), "v"(reinterpret_cast<const GLOBAL uint8_t*>(a))
			    : "memory");
		}
	};
	const int32_t maxc = nchunks;  // one chunk past the payload: 8-byte reads at its end
	for (; issued < DEPTH && issued <= maxc; ++issued)
		issue(issued);
	// 8 bytes at block-relative pos (reads only move forward).  pos is
	// wave-uniform but kept in VGPRs: the parse below runs on the VALU (four
	// per CU) -- on the scalar unit, which the CU's eight waves share, it
	// was SALU-bound at ~120 scalar instructions per sequence.
	int32_t shi = 0;  // = landed * STG: bytes below it (from abase) are in LDS
	// make block-relative bytes [.., pend) readable (pend wave-uniform)
	auto ensure = [&](int32_t pend) {
		pend = int32_t(uni(uint32_t(pend)));  // wave-uniform: scalar control and DMA operands
		const int32_t need = (pend + mis - 1) / STG;  // last chunk needed
		if (need >= issued) {
			// a long literal run jumped past the chunks in flight: settle them
			// and restart the stream two chunks before the one needed
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			issued = landed = max(need - 1, 0);
			for (int k = 0; k < DEPTH && issued <= maxc; ++k)
				issue(issued++);
		}
		while (landed <= need) {
			// chunk `landed` is the oldest in flight
			if (issued - landed >= DEPTH)
				asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (DEPTH - 1)) : "memory");
			else
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			++landed;
			if (issued <= maxc)
				issue(issued++);  // its slot's chunk (issued - NSLOT) is long read
		}
		shi = landed * STG;
	};
	// 8 bytes at block-relative pos, already readable.  pos is wave-uniform,
	// and so is the parse on it (scalar unit).
	auto lds8 = [&](int32_t pos, uint32_t& lo, uint32_t& hi) {
		const uint32_t a = uni(uint32_t(pos + mis));
		const uint32_t r0 = a & ~3u;
		const uint32_t* w = reinterpret_cast<const uint32_t*>(S.ring);
		const uint32_t w0 = w[(r0 & (RING - 1)) >> 2], w1 = w[((r0 + 4) & (RING - 1)) >> 2],
		               w2 = w[((r0 + 8) & (RING - 1)) >> 2];
		const uint32_t sh = a & 3u;
		lo = uni(__builtin_amdgcn_alignbyte(w1, w0, sh));
		hi = uni(__builtin_amdgcn_alignbyte(w2, w1, sh));
	};
	auto rd8 = [&](int32_t pos, uint32_t& lo, uint32_t& hi) {
		pos = int32_t(uni(uint32_t(pos)));
		if (pos + mis + 8 > shi)
			ensure(pos + 8);
		lds8(pos, lo, hi);
	};
	// A length extension (15 + 255... , lz4ada.adb:724-735) from byte x on,
	// the general way (runs of 255 over any length): adds to len, returns
	// the position after its last byte, -1 when it runs past the block end.
	auto ext_slow = [&](int32_t x, int32_t& len) -> int32_t {
		for (;;) {
			if (x >= n || len > cap)
				return -1;
			uint32_t lo, hi;
			rd8(x, lo, hi);
			const uint64_t w = uint64_t(lo) | (uint64_t(hi) << 32);
			const uint64_t f = ~w;
			if (f == 0) {
				len += 255 * 8;
				x += 8;
				continue;
			}
			const int32_t k = int32_t(__builtin_ctzll(f)) >> 3;
			if (x + k >= n)
				return -1;
			len += 255 * k + int32_t((w >> (8 * k)) & 0xffu);
			return x + k + 1;
		}
	};

	bool bad = false;
	int32_t p = 0;     // input position of the next sequence
	int32_t o = 0;     // output position
	int32_t nseq = 0;  // sequences so far
	bool done = n == 0;
	uint32_t t0 = 0, t1 = 0;  // the bytes at p (tv of them valid): the next
	int32_t tv = 0;           // token, from the previous offset read
	while (!done && !bad) {
		// ---- parse up to NSEQ sequences (Decompress_Sequence, :737-777);
		// sequence j of the batch lands in lane j
		int32_t r_lit = 0, r_L = 0, r_dst = 0, r_off = 0, r_ml = 0;
		int32_t ns = 0, pieces = 0;
		auto record = [&](int32_t lit, int32_t L, int32_t off, int32_t ml) {
			const bool mine = lane == ns;
			r_lit = mine ? lit : r_lit;
			r_L = mine ? L : r_L;
			r_dst = mine ? o : r_dst;
			r_off = mine ? off : r_off;
			r_ml = mine ? ml : r_ml;
			pieces += L > BIG ? 0 : (L + 15) >> 4;
			o += L + ml;
			++ns;
		};
		for (;;) {
			// -- the common shape, a tight scalar loop (the CU's eight waves
			// share one scalar unit, so instructions per sequence are the
			// cost): the literal length's extension bytes among the token
			// window's bytes 1..4, at most one match-length extension byte, not
			// the last sequence, well formed, the offset within the staged
			// bytes.  Anything else leaves it for the general code below.
			while (ns < NSEQ && pieces <= OWN - BIG / 16 && tv >= 5 && p + mis + 1100 <= shi) {
				const uint32_t tk = t0 & 0xffu;
				const uint32_t ex = uint32_t((uint64_t(t0) | (uint64_t(t1) << 32)) >> 8);  // bytes 1..4
				const uint32_t kb = uint32_t(__builtin_ctz(~ex | 0x80000000u)) & ~7u;  // 8 x first non-0xFF
				const bool isx = tk >= 0xf0u;
				const int32_t L = isx ? int32_t(15 + 255 * (kb >> 3) + ((ex >> kb) & 0xffu)) : int32_t(tk >> 4);
				const int32_t lit = p + 1 + (isx ? int32_t(kb >> 3) + 1 : 0);
				const int32_t x = lit + L;
				if ((isx && (~ex) == 0u) || x + 1 >= n)
					break;
				uint32_t w0, w1;
				lds8(x, w0, w1);  // offset, match-length byte, the next token
				const int32_t off = int32_t(w0 & 0xffffu);
				const int32_t M = int32_t(tk & 15u);
				const uint32_t e = (w0 >> 16) & 0xffu;
				const bool x2 = M == 15;
				const int32_t ml = M + 4 + (x2 ? int32_t(e) : 0);
				if ((x2 && e == 255u) || off == 0 || off > o + L || o + L + ml > cap)
					break;
				const int32_t used = x2 ? 3 : 2;  // the next token is in w
				const uint64_t w = (uint64_t(w0) | (uint64_t(w1) << 32)) >> (8 * used);
				t0 = uint32_t(w);
				t1 = uint32_t(w >> 32);
				tv = 8 - used;
				record(lit, L, off, ml);
				p = x + used;
			}
			if (ns >= NSEQ || pieces > OWN - BIG / 16)
				break;
			if (p >= n) {
				done = true;  // the chain ended right after a match
				break;
			}
			if (p + mis + 1100 > shi) {
				ensure(p + 1100);
				if (tv >= 5)
					continue;
			}
			// -- one sequence, the general way (rare)
			rd8(p, t0, t1);
			tv = 8;
			const uint32_t tk = t0 & 0xffu;
			int32_t L = int32_t(tk >> 4);
			int32_t lit = p + 1;
			if (L == 15) {
				lit = ext_slow(p + 1, L);
				if (lit < 0) {
					bad = true;
					break;
				}
			}
			const int32_t x = lit + L;
			int32_t M = int32_t(tk & 15u), off = 0, ml = 0, next = n;
			if (x >= n) {
				// the block's last sequence: literals only (:748-764)
				if (x > n || M != 0 || o + L > cap) {
					bad = true;
					break;
				}
				done = true;
			} else {
				if (x + 1 >= n) {
					bad = true;
					break;
				}
				uint32_t w0, w1;
				rd8(x, w0, w1);
				off = int32_t(w0 & 0xffffu);
				next = x + 2;
				if (M == 15) {
					next = ext_slow(x + 2, M);
					if (next < 0) {
						bad = true;
						break;
					}
				}
				ml = M + 4;
				// off 0, a reference before the block start (D2) or a slot
				// overflow: k_decode_pc gives the exact status
				if (off == 0 || off > o + L || int64_t(o) + L + ml > cap) {
					bad = true;
					break;
				}
			}
			record(lit, L, off, ml);
			p = next;
			if (done)
				break;
			rd8(p, t0, t1);  // the next token's window
			tv = 8;
		}
		nseq += ns;
		if (bad || ns == 0)
			break;
		if (nseq > p / DENSE_BYTES + 256) {
			bad = true;  // dense data: the two-wave decoder is faster
			break;
		}

#ifndef LZ4ADA_SP_EXP_NOLIT  // timing experiment (wrong output)
		// ---- literals (Write_Output, :790-824): runs up to BIG bytes cut
		// into 16-byte pieces dealt over the wave, piece t = 64 r + lane; its
		// run from a mark at every run's first piece and a prefix maximum
		{
			const int32_t Lr = lane < ns ? r_L : 0;
			const int32_t P = Lr <= BIG ? (Lr + 15) >> 4 : 0;
			const int32_t I = wave_incl_scan(P);
			const int32_t tot = __builtin_amdgcn_readlane(I, 63);
			const int32_t st = I - P;
			u32x4 rc;
			rc.x = uint32_t(r_lit - 16 * st);
			rc.y = uint32_t(r_dst - 16 * st);
			rc.z = uint32_t(Lr + 16 * st);
			rc.w = 0;
			S.rec[lane] = rc;
			for (int32_t z = 16 * lane; z < tot; z += 1024)
				*reinterpret_cast<u32x4*>(&S.own[z]) = u32x4{ 0, 0, 0, 0 };
			wave_lds_fence();
			if (P > 0)
				S.own[st] = uint8_t(lane);
			wave_lds_fence();
			int32_t carry = 0;
			for (int32_t r0 = 0; r0 < tot; r0 += 64 * U) {
				u32x4 v[U];
				int32_t dd[U], ln[U];
#pragma unroll
				for (int u = 0; u < U; ++u) {
					const int32_t t = r0 + 64 * u + lane;
					const int32_t m = t < tot ? int32_t(S.own[t]) : 0;
					const int32_t ow = max(wave_incl_max(m), carry);
					carry = __builtin_amdgcn_readlane(ow, 63);
					const u32x4 q = S.rec[ow];
					ln[u] = t < tot ? min(16, int32_t(q.z) - 16 * t) : 0;
					dd[u] = int32_t(q.y) + 16 * t;
					if (ln[u] > 0)
						v[u] = gload16(reinterpret_cast<uintptr_t>(in) + uintptr_t(int32_t(q.x) + 16 * t),
						               lim);
				}
#pragma unroll
				for (int u = 0; u < U; ++u)
					if (ln[u] > 0)
						gstore_n(ob + dd[u], v[u], ln[u]);
			}
			// runs over BIG bytes: the whole wave, 8 KiB per step
			uint64_t big = __ballot(lane < ns && r_L > BIG);
			while (big) {
				const int32_t j = int32_t(__builtin_ctzll(big));
				big &= big - 1;
				const int32_t Lj = __builtin_amdgcn_readlane(r_L, j);
				const int32_t sj = __builtin_amdgcn_readlane(r_lit, j);
				const int32_t dj = __builtin_amdgcn_readlane(r_dst, j);
				for (int32_t c = 0; c < Lj; c += 1024 * U) {
					u32x4 v[U];
#pragma unroll
					for (int u = 0; u < U; ++u) {
						const int32_t k = c + 1024 * u + 16 * lane;
						if (k < Lj)
							v[u] = gload16(reinterpret_cast<uintptr_t>(in) + uintptr_t(sj + k), lim);
					}
#pragma unroll
					for (int u = 0; u < U; ++u) {
						const int32_t k = c + 1024 * u + 16 * lane;
						if (k < Lj)
							gstore_n(ob + dj + k, v[u], min(16, Lj - k));
					}
				}
			}
		}
#endif
		// every literal (and earlier match) store has landed before a match
		// of this batch reads the output
		__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)

		// ---- matches in dependency rounds (Output_With_History, :845-904)
		const int32_t mdst = r_dst + r_L;
		const int32_t mend = mdst + r_ml;
		const int32_t src = mdst - r_off;
		const int32_t dep_end = src + min(r_off, r_ml);
		bool pend = lane < ns && r_ml > 0;
#ifdef LZ4ADA_SP_EXP_NOMATCH  // timing experiment (wrong output)
		pend = false;
#endif
		// lanes [j1, c2) of the batch write bytes in [src, dep_end)
		int32_t j1 = 0, c2 = 0;
#pragma unroll
		for (int stp = 32; stp >= 1; stp >>= 1) {
			if (__shfl(lane < ns ? mend : INT32_MAX, j1 + stp - 1) <= src)
				j1 += stp;
			if (__shfl(lane < ns ? mdst : INT32_MAX, c2 + stp - 1) < dep_end)
				c2 += stp;
		}
		const int32_t j2 = min(c2 - 1, lane - 1);
		uint64_t dep = 0;
		if (pend && j1 <= j2)
			dep = (j2 == 63 ? ~uint64_t(0) : ((uint64_t(2) << j2) - 1)) & ~((uint64_t(1) << j1) - 1);
		for (;;) {
			const uint64_t pending = __ballot(pend);
			if (pending == 0)
				break;
			const bool ready = pend && (dep & pending) == 0;
			// ready matches read no pending match's output: any order
			if (ready && r_ml <= LONGM)
				run_match(ob, mdst, r_off, r_ml, olim);
			uint64_t lng = __ballot(ready && r_ml > LONGM);
			while (lng) {
				const int32_t j = int32_t(__builtin_ctzll(lng));
				lng &= lng - 1;
				run_match_wave(ob, __builtin_amdgcn_readlane(mdst, j), __builtin_amdgcn_readlane(r_off, j),
				               __builtin_amdgcn_readlane(r_ml, j), olim);
			}
			if (ready)
				pend = false;
			__builtin_amdgcn_s_waitcnt(0x0F70);  // this round's stores landed
		}
	}
	if (!bad && !done)
		bad = true;
	if (lane == 0) {
		if (bad) {
			status[b].code = DS_RETRY;
		} else {
			status[b].code = DS_OK;
			status[b].aux = 0;
			status[b].detail = 0;
			status[b].err_out_pos = 0;
			status[b].out_len = uint32_t(o);
		}
	}
}

}  // namespace sparse

hipError_t launch_decode_sparse(const uint8_t* d_frame, uint64_t frame_len,
                                const lz4ada_block_desc* d_desc, uint32_t nblocks, uint8_t* d_out,
                                lz4ada_block_status* d_status, hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(sparse::k_decode_sparse, dim3(nblocks), dim3(64), 0, stream, d_frame,
	                   frame_len, d_desc, nblocks, d_out, d_status);
	return hipGetLastError();
}

}  // namespace lz4ada
