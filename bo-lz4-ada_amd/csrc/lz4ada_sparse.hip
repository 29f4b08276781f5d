// lz4ada_sparse.hip -- streaming decoder for literal-heavy ("sparse") blocks.
//
// Same reference path as the index decoder (lib/lz4ada.adb:716-904:
// Decompress_Full_Block / Decompress_Sequence / Write_Output /
// Output_With_History), for the blocks its pass 1 declines because their
// sequences are too far apart for speculative walks to merge (long literal
// runs: incompressible text, mostly-stored content in compressed blocks).
// Such a block holds few sequences (~9k per 4 MiB at 470 B each) and is a
// copy job, so one wave per block, streaming:
//
//  * staging: the compressed stream flows through a 16 KiB LDS ring in 2 KiB
//    chunks by LDS-DMA (global_load_lds_dwordx4, no registers), DEPTH chunks
//    in flight ahead of the parse;
//  * parse: the sequence chain walked wave-uniformly from the ring;
//  * literals (Write_Output, :790-824): each run is copied the moment its
//    sequence is parsed, from the ring to HBM (the bytes are staged anyway:
//    the compressed stream is read from HBM once), 1 KiB per store
//    instruction; a run longer than the staged window goes HBM -> HBM;
//  * matches (Output_With_History, :845-904): sequence j of a batch of 64
//    records its match in lane j; the batch's matches run at the end of the
//    NEXT batch, when everything the batch stored has long completed, so
//    their wait is for memory operations a whole batch old and never drains
//    the staging stream.  Lane j runs match j once no earlier match of the
//    batch writes a byte it reads (a dependency mask from two binary
//    searches over the batch's monotone match positions); sources are read
//    from the output already written (L1-bypassing loads); a match reads
//    only its first `off` source bytes -- byte i is source byte i mod off --
//    so no piece reads its own match.
//
// The wave's vector-memory counter is in order, and the LDS-DMA loads are
// invisible to the compiler's wait pass, so the waits for staged chunks and
// for a batch's stores are counted by hand: `nvm` is a lower bound of the
// vector-memory instructions issued so far (every DMA chunk 2, every literal
// store round 1, every HBM copy step 2 -- a store the compiler splits only
// adds more), and "everything issued before point X has completed" is
// vmcnt <= nvm - nvm_at_X, rounded down to an encodable count.
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

constexpr int STG = 2048;          // staged chunk (two LDS-DMA instructions)
constexpr int NSLOT = 8;           // ring slots
constexpr int RING = NSLOT * STG;  // LDS ring of compressed bytes (16 KiB)
constexpr int DEPTH = 5;           // chunks in flight beyond the landed ones
// The parse keeps [p, p + AHEAD) landed.  After a chunk is issued the ring
// still holds the NSLOT - DEPTH chunks before the newest landed one, i.e.
// every byte from p - (3 * STG - AHEAD - STG) on: the position being parsed
// and everything after it stay valid while chunks are issued.
constexpr int AHEAD = 3088;
constexpr int NSEQ = 64;           // sequences per batch (one match per lane)
constexpr int LONGM = 512;         // longer matches: copied by the whole wave
constexpr int U = 8;               // HBM -> HBM copies: pieces per lane in flight (8 KiB per wave)
constexpr int DENSE_BYTES = 48;    // fewer input bytes per sequence: decline
static_assert(AHEAD + 2 * STG <= (NSLOT - DEPTH) * STG + STG, "parse window vs ring slack");

struct alignas(16) SpLds {
	uint8_t ring[RING];  // filled by LDS-DMA, STG-byte slots
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Diagnostic build only (-DLZ4ADA_SP_STAMPS): cycles per phase and event
// counts, summed over waves (no draining: a wait is timed as it stands).
enum SpPhase { SP_TOTAL, SP_DMAWAIT, SP_MWAIT, SP_MATCH, SP_GCOPY, SP_BATCHES, SP_RESTARTS, SP_SEQ,
	           SP_SLOW, SP_NST };
#ifdef LZ4ADA_SP_STAMPS
__device__ unsigned long long g_sp_stamps[SP_NST];
#define SSTAMP_DECL uint64_t sst[SP_NST] = {}; const uint64_t sst0 = __builtin_amdgcn_s_memtime()
#define SSTAMP_BEGIN() const uint64_t _sst_t = __builtin_amdgcn_s_memtime()
#define SSTAMP_END(ph) (sst[ph] += __builtin_amdgcn_s_memtime() - _sst_t)
#define SCOUNT(ph, v) (sst[ph] += uint64_t(v))
#define SSTAMP_FLUSH()                                                       \
	do {                                                                     \
		sst[SP_TOTAL] = __builtin_amdgcn_s_memtime() - sst0;                 \
		if (lane_id() == 0)                                                  \
			for (int _i = 0; _i < SP_NST; ++_i)                              \
				atomicAdd(&g_sp_stamps[_i], (unsigned long long)sst[_i]);    \
	} while (0)
#else
#define SSTAMP_DECL
#define SSTAMP_BEGIN()
#define SSTAMP_END(ph)
#define SCOUNT(ph, v)
#define SSTAMP_FLUSH()
#endif

// Wait until at most n vector-memory instructions are outstanding, n rounded
// down to one of a few encodable counts (n is wave-uniform: scalar branches).
__device__ __forceinline__ void vm_wait_upto(uint32_t n)
{
	if (n >= 63)
		asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
	else if (n >= 48)
		asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
	else if (n >= 32)
		asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
	else if (n >= 24)
		asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
	else if (n >= 16)
		asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
	else if (n >= 12)
		asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
	else if (n >= 8)
		asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
	else if (n >= 4)
		asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
	else if (n >= 2)
		asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
	else
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void vm_wait_all()
{
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// 16 global bytes at a, never reading at or past lim.
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

// 16 bytes at byte a of the LDS ring: three 8-byte-aligned ds_read_b64 (each
// wrapped on its own), a one-bit dword select and four v_alignbyte.
__device__ __forceinline__ u32x4 ring16(const uint8_t* base, uint32_t a)
{
	constexpr uint32_t mask = RING - 1;
	const uint32_t a8 = a & ~7u;
	const uint64_t q0 = *reinterpret_cast<const uint64_t*>(base + (a8 & mask));
	const uint64_t q1 = *reinterpret_cast<const uint64_t*>(base + ((a8 + 8) & mask));
	const uint64_t q2 = *reinterpret_cast<const uint64_t*>(base + ((a8 + 16) & mask));
	const uint32_t w0 = uint32_t(q0), w1 = uint32_t(q0 >> 32), w2 = uint32_t(q1),
	               w3 = uint32_t(q1 >> 32), w4 = uint32_t(q2), w5 = uint32_t(q2 >> 32);
	const bool s1 = (a & 4u) != 0;
	const uint32_t d0 = s1 ? w1 : w0, d1 = s1 ? w2 : w1, d2 = s1 ? w3 : w2, d3 = s1 ? w4 : w3,
	               d4 = s1 ? w5 : w4;
	const uint32_t sh = a & 3u;
	u32x4 v;
	v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
	v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
	v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
	v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
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

// A literal piece of rem (>= 1) bytes at output position x: always 16 bytes
// while they stay inside the slot -- the bytes past the run belong to its
// match and the later sequences, all stored after this (in order, by this
// wave), so one store instruction per piece and no partial stores.
__device__ __forceinline__ void lit_store(g8* ob, int32_t x, u32x4 v, int32_t rem, int32_t cap)
{
	if (x + 16 <= cap)
		__builtin_memcpy(ob + x, &v, 16);
	else
		gstore_n(ob + x, v, min(16, rem));
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

// The matches of one batch (lane j: match j of cnt; ml 0: none), every
// byte they read already stored and completed -- except the batch's own
// match output, which the dependency rounds order (each later round waits
// for the earlier rounds' stores).
__device__ __forceinline__ void run_batch_matches(g8* ob, uintptr_t olim, int32_t mdst, int32_t off,
                                                  int32_t ml, int32_t cnt, uint32_t& nvm)
{
	const int32_t lane = int32_t(lane_id());
	const bool mine = lane < cnt && ml > 0;
	const int32_t mend = mdst + ml;
	const int32_t src = mdst - off;
	const int32_t dep_end = src + min(off, ml);
	bool pend = mine;
	// lanes [j1, c2) of the batch write bytes in [src, dep_end)
	int32_t j1 = 0, c2 = 0;
#pragma unroll
	for (int stp = 32; stp >= 1; stp >>= 1) {
		if (__shfl(lane < cnt ? mend : INT32_MAX, j1 + stp - 1) <= src)
			j1 += stp;
		if (__shfl(lane < cnt ? mdst : INT32_MAX, c2 + stp - 1) < dep_end)
			c2 += stp;
	}
	const int32_t j2 = min(c2 - 1, lane - 1);
	uint64_t dep = 0;
	if (pend && j1 <= j2)
		dep = (j2 == 63 ? ~uint64_t(0) : ((uint64_t(2) << j2) - 1)) & ~((uint64_t(1) << j1) - 1);
	for (bool first = true;; first = false) {
		const uint64_t pending = __ballot(pend);
		if (pending == 0)
			break;
		if (!first)
			vm_wait_all();  // the previous round's stores landed
		const bool ready = pend && (dep & pending) == 0;
		// ready matches read no pending match's output: any order
		if (ready && ml <= LONGM)
			run_match(ob, mdst, off, ml, olim);
		uint64_t lng = __ballot(ready && ml > LONGM);
		while (lng) {
			const int32_t j = int32_t(__builtin_ctzll(lng));
			lng &= lng - 1;
			run_match_wave(ob, __builtin_amdgcn_readlane(mdst, j), __builtin_amdgcn_readlane(off, j),
			               __builtin_amdgcn_readlane(ml, j), olim);
		}
		if (ready)
			pend = false;
		nvm += 2;  // at least one load and one store instruction
	}
	// settle the match loads (see copy_lit): once per batch, not per sequence
	__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
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
	SSTAMP_DECL;
	const uintptr_t lim = reinterpret_cast<uintptr_t>(frame) + frame_len;
	const uintptr_t olim = reinterpret_cast<uintptr_t>(ob) + uintptr_t(cap);
	const int32_t mis = int32_t(reinterpret_cast<uintptr_t>(in) & 15u);
	const uintptr_t abase = reinterpret_cast<uintptr_t>(in) - uintptr_t(mis);
	// A lane whose 16-byte DMA piece would cross the frame's end loads an
	// earlier piece instead (below), so ring bytes from the last 16-byte
	// boundary before the frame's end on are not the stream's: block-relative
	// bytes at or past rbad are read from HBM.
	const int32_t rbad =
	    int32_t(min(uintptr_t(lim - abase) & ~uintptr_t(15), uintptr_t(INT32_MAX / 2))) - mis;

	// ---- staging: chunk c = aligned bytes [c STG, (c + 1) STG) from abase
	// goes to ring slot c % NSLOT by LDS-DMA (global_load_lds_dwordx4, 1 KiB
	// per instruction, no registers).  Chunks [vlo, landed) are in the ring,
	// [landed, issued) in flight; issued <= landed + DEPTH.
	const uint32_t ring_lds =
	    uint32_t(uintptr_t((__attribute__((address_space(3))) uint8_t*)(&S.ring[0])));
	uint32_t nvm = 0;    // vector-memory instructions issued (lower bound)
	uint32_t dma_v = 0;  // lane s: nvm right after the DMA of the chunk in slot s was issued
	int32_t issued = 0, landed = 0, vlo = 0;
	const int32_t nchunks = (n + mis + STG - 1) / STG;
	auto issue = [&](int32_t c) {
		// the slot's previous chunk may still be read by an LDS read in flight
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
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
		nvm += STG / 1024;
		dma_v = lane == c % NSLOT ? nvm : dma_v;
		vlo = max(vlo, c + 1 - NSLOT);
	};
	const int32_t maxc = nchunks;  // one chunk past the payload: 8-byte reads at its end
	for (; issued < DEPTH && issued <= maxc; ++issued)
		issue(issued);
	int32_t shi = 0;  // = landed * STG: bytes below it (from abase) are in LDS (from vlo * STG on)
	// make block-relative bytes [.., pend) readable (pend wave-uniform)
	auto ensure = [&](int32_t pend) {
		// nothing past the payload is ever needed (the last chunk issued is
		// the one past it)
		pend = int32_t(uni(uint32_t(min(pend, n + 16))));
		const int32_t need = (pend + mis - 1) / STG;  // last chunk needed
		if (need >= issued) {
			// a long literal run jumped past the chunks in flight: settle them
			// and restart the stream two chunks before the one needed
			vm_wait_all();
			SCOUNT(SP_RESTARTS, 1);
			issued = landed = vlo = max(need - 1, 0);
			for (int k = 0; k < DEPTH && issued <= maxc; ++k)
				issue(issued++);
		}
		while (landed <= need) {
			// chunk `landed` is the oldest in flight: everything issued after
			// it may stay outstanding
			SSTAMP_BEGIN();
			vm_wait_upto(nvm - uni(uint32_t(__builtin_amdgcn_readlane(dma_v, landed % NSLOT))));
			SSTAMP_END(SP_DMAWAIT);
			++landed;
			if (issued <= maxc)
				issue(issued++);
		}
		shi = landed * STG;
	};
	// 8 bytes at block-relative pos, already readable.  pos is wave-uniform,
	// and so is the parse on it.
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
		if (pos + 8 > rbad) {
			// the stream's last bytes: from HBM, never at or past the frame's end
			uint64_t v = 0;
			for (int k = 0; k < 8; ++k)
				if (reinterpret_cast<uintptr_t>(in) + uintptr_t(pos + k) < lim)
					v |= uint64_t(in[pos + k]) << (8 * k);
			__builtin_amdgcn_s_waitcnt(0x0F70);  // settled here (see copy_lit)
			lo = uni(uint32_t(v));
			hi = uni(uint32_t(v >> 32));
			return;
		}
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
			if (x + 64 <= rbad) {
				// 64 bytes a step, one per lane: a ballot of the bytes that are
				// not 255 (RLE blocks carry runs of hundreds of them)
				if (x + mis + 64 > shi)
					ensure(x + 64);
				const uint32_t bv = S.ring[uint32_t(x + mis + lane) & (RING - 1)];
				const uint64_t nf = __ballot(bv != 0xFFu);
				if (nf == 0) {
					len += 255 * 64;
					x += 64;
					continue;
				}
				const int32_t k = int32_t(__builtin_ctzll(nf));
				if (x + k >= n)
					return -1;
				len += 255 * k + int32_t(__builtin_amdgcn_readlane(bv, k));
				return x + k + 1;
			}
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
	// Literal run [lit, lit + L) -> output [dst, dst + L) (Write_Output,
	// :790-824), now: from the ring when every byte of it is staged, else
	// HBM -> HBM (runs longer than the staged window).  The stores are left
	// in flight.
	auto copy_lit = [&](int32_t lit, int32_t L, int32_t dst) {
		if (L <= 0)
			return;
		if (lit + mis >= vlo * STG && lit + L + mis <= shi && lit + L <= rbad) {
			for (int32_t c = 0; c < L; c += 1024) {
				const int32_t k = c + 16 * lane;
				if (k < L)
					lit_store(ob, dst + k, ring16(S.ring, uint32_t(lit + mis + k)), L - k, cap);
				nvm += 1;
			}
			return;
		}
		SSTAMP_BEGIN();
		for (int32_t c = 0; c < L; c += 1024 * U) {
			u32x4 v[U];
#pragma unroll
			for (int u = 0; u < U; ++u) {
				const int32_t k = c + 1024 * u + 16 * lane;
				if (k < L)
					v[u] = gload16(reinterpret_cast<uintptr_t>(in) + uintptr_t(lit + k), lim);
			}
#pragma unroll
			for (int u = 0; u < U; ++u) {
				const int32_t k = c + 1024 * u + 16 * lane;
				if (k < L)
					lit_store(ob, dst + k, v[u], L - k, cap);
			}
			nvm += 2;
		}
		// settle this rare path's loads here: left pending (lanes past the
		// run skip the stores that wait for them), they reach the parse loop's
		// head, and the wait pass puts a vmcnt(0) -- every DMA chunk and store
		// in flight -- before each sequence's first LDS read
		__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
		SSTAMP_END(SP_GCOPY);
	};

	bool bad = false;
	int32_t why = 0;   // decline reason (status detail of a DS_RETRY block: diagnostics)
	int32_t p = 0;     // input position of the next sequence
	int32_t o = 0;     // output position
	int32_t nseq = 0;  // sequences so far
	bool done = n == 0;
	u32x4 win = {0u, 0u, 0u, 0u};  // the bytes at p (tv of them valid): the next
	int32_t tv = 0;                // token, from the previous offset read
	// the previous batch's matches (lane j: match j; ml 0: none), run at the
	// end of the current batch
	int32_t pm_dst = 0, pm_off = 1, pm_ml = 0, pm_cnt = 0;
	uint32_t nvm_b0 = 0;  // nvm when the current batch began
	if (!done)
		ensure(AHEAD);
	while (!done && !bad) {
		// ---- parse up to NSEQ sequences (Decompress_Sequence, :737-777);
		// each sequence's literals are copied at once, its match lands in
		// lane j of the batch
		int32_t m_dst = 0, m_off = 1, m_ml = 0;
		int32_t ns = 0;
		auto record = [&](int32_t L, int32_t off, int32_t ml) {
			const bool mine = lane == ns;
			m_dst = mine ? o + L : m_dst;
			m_off = mine ? off : m_off;
			m_ml = mine ? ml : m_ml;
			o += L + ml;
			++ns;
		};
		for (;;) {
			// -- the common shape: the literal length's extension among the
			// 16-byte window's bytes, at most one match-length extension byte,
			// not the last sequence, well formed, run and offset staged (runs
			// up to 3074 bytes: 99.9% of the literal class, against 91% for
			// the 8-byte window before); the literals stored branch-free.
			// Anything else leaves the sequence to the general code below.
			// The parse is wave-uniform and runs on the scalar unit; on the
			// VALU (LZ4ADA_SP_VALU: the state laundered into VGPRs, every lane
			// computing the same values) the decoder alone is faster (6.8 vs
			// 7.4 ms) but the step with the block checksums beside it slower
			// (9.4 vs 8.7 ms): their XXH32 chains wait on the same VALUs.
			{
				int32_t vp = p, vo = o, vns = ns, vtv = tv;
				u32x4 w = win;
				// (LZ4ADA_SP_VALU: kept in VGPRs, opaque to the uniformity
				// analysis, so everything derived from them stays on the VALU)
#ifdef LZ4ADA_SP_VALU
				asm volatile("" : "+v"(vp), "+v"(vo), "+v"(vns), "+v"(vtv), "+v"(w.x), "+v"(w.y), "+v"(w.z),
				             "+v"(w.w));
#endif
				for (;;) {
					const uint32_t tk = w.x & 0xffu;
					const int32_t L4 = int32_t(tk >> 4), M4 = int32_t(tk & 15u);
					// first byte != 0xFF among the window's bytes 1..15 (i = 16:
					// none): per dword the lowest set bit of its complement
					// (v_ffbl; 128 when none), the minimum over the four
					auto ff = [](uint32_t m) -> uint32_t { return m ? uint32_t(__builtin_ctz(m)) : 128u; };
					const uint32_t fb = min(min(ff(~w.x & 0xFFFFFF00u), 32u + ff(~w.y)),
					                        min(64u + ff(~w.z), 96u + ff(~w.w)));
					const int32_t i = int32_t(min(fb >> 3, 16u));
					const uint32_t wd = (i & 8) ? ((i & 4) ? w.w : w.z) : ((i & 4) ? w.y : w.x);
					const uint32_t bi = (wd >> (8 * (i & 3))) & 0xffu;
					const bool isx = L4 == 15;
					const int32_t L = isx ? 15 + 255 * (i - 1) + int32_t(bi) : L4;
					const int32_t lit = vp + 1 + (isx ? i : 0);
					const int32_t x = lit + L;
					// staged through x + 16 (a chunk at a time, every few sequences)
					// (only for a length read within the window: x stays within 3.1 KiB of
					// vp, so the chunks ensure() recycles are all behind vp)
					if (uni(uint32_t(x + mis + 16 > shi && (!isx || i < vtv))))
						ensure(int32_t(uni(uint32_t(x + 16))));
					const u32x4 y = ring16(S.ring, uint32_t(x + mis));  // offset, ML byte, next token...
					const int32_t off = int32_t(y.x & 0xffffu);
					const uint32_t e = (y.x >> 16) & 0xffu;
					const bool x2 = M4 == 15;
					const int32_t ml = M4 + 4 + (x2 ? int32_t(e) : 0);
					const int32_t used = x2 ? 3 : 2;
					const bool ok = vns < NSEQ && vtv >= 1 && (!isx || i < vtv) && x + 1 < n &&
					                x + mis + 16 <= shi && x + 16 <= rbad && lit + mis >= vlo * STG &&
					                !(x2 && e == 255u) &&
					                off != 0 && off <= vo + L && vo + L + ml + 16 <= cap;
					if (!uni(uint32_t(ok)))
						break;
					// the literals: lane j stores piece j (16 bytes; pieces past the
					// run repeat the last one, so no lane is masked off; the bytes a
					// piece spills past the run are rewritten later)
					const int32_t last = max((L - 1) >> 4, 0);
					{
						const int32_t j = min(lane, last);
						const u32x4 v = ring16(S.ring, uint32_t(lit + mis + 16 * j));
						__builtin_memcpy(ob + vo + 16 * j, &v, 16);
					}
					if (uni(uint32_t(L > 1024))) {
#pragma unroll
						for (int r = 1; r < 4; ++r) {
							const int32_t j = min(64 * r + lane, last);
							const u32x4 v = ring16(S.ring, uint32_t(lit + mis + 16 * j));
							__builtin_memcpy(ob + vo + 16 * j, &v, 16);
						}
						nvm += 3;
					}
					nvm += 1;
					const bool mine = lane == vns;
					m_dst = mine ? vo + L : m_dst;
					m_off = mine ? off : m_off;
					m_ml = mine ? ml : m_ml;
					vo += L + ml;
					vns += 1;
					vp = x + used;
					// the next window: y from byte `used` on
					const uint32_t sh = uint32_t(used);
					w.x = __builtin_amdgcn_alignbyte(y.y, y.x, sh);
					w.y = __builtin_amdgcn_alignbyte(y.z, y.y, sh);
					w.z = __builtin_amdgcn_alignbyte(y.w, y.z, sh);
					w.w = y.w >> (8 * sh);
					vtv = 16 - used;
				}
				p = int32_t(uni(uint32_t(vp)));
				o = int32_t(uni(uint32_t(vo)));
				ns = int32_t(uni(uint32_t(vns)));
				tv = int32_t(uni(uint32_t(vtv)));
				win = w;
			}
			if (ns >= NSEQ)
				break;
			if (p >= n) {
				done = true;  // the chain ended right after a match
				break;
			}
			// -- one sequence, the general way (rare)
			SCOUNT(SP_SLOW, 1);
			uint32_t t0, t1;
			rd8(p, t0, t1);
			const uint32_t tk = t0 & 0xffu;
			int32_t L = int32_t(tk >> 4);
			int32_t lit = p + 1;
			if (L == 15) {
				lit = ext_slow(p + 1, L);
				if (lit < 0) {
					why = 1;
					bad = true;
					break;
				}
			}
			const int32_t x = lit + L;
			if (x > n || int64_t(o) + L > cap) {
				why = 2;
				bad = true;  // literals past the block end (D3) or the slot
				break;
			}
			// the literals now, while they may still be in the ring
			copy_lit(lit, L, o);
			int32_t M = int32_t(tk & 15u), off = 0, ml = 0, next = n;
			if (x >= n) {
				// the block's last sequence: literals only (:748-764)
				if (M != 0) {
					why = 3;
					bad = true;
					break;
				}
				done = true;
			} else {
				if (x + 1 >= n) {
					why = 4;
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
						why = 5;
						bad = true;
						break;
					}
				}
				ml = M + 4;
				// off 0, a reference before the block start (D2) or a slot
				// overflow: k_decode_pc gives the exact status
				if (off == 0 || off > o + L || int64_t(o) + L + ml > cap) {
					why = 6;
					bad = true;
					break;
				}
			}
			record(L, off, ml);
			p = next;
			if (done)
				break;
			// the next token's window
			if (p + mis + 16 > shi)
				ensure(p + 16);
			win = ring16(S.ring, uint32_t(p + mis));
			tv = max(min(rbad - p, 16), 0);  // (0: the general path takes the rest)
		}
		nseq += ns;
		if (bad || ns == 0)
			break;
		if (nseq > p / DENSE_BYTES + 256) {
			why = 7;
			bad = true;  // dense data: the two-wave decoder is faster
			break;
		}
		// ---- the previous batch's matches: everything they read was stored
		// before this batch began
		SCOUNT(SP_BATCHES, 1);
		SCOUNT(SP_SEQ, ns);
		if (pm_cnt > 0) {
			{
				SSTAMP_BEGIN();
				vm_wait_upto(nvm - nvm_b0);
				SSTAMP_END(SP_MWAIT);
			}
			SSTAMP_BEGIN();
			run_batch_matches(ob, olim, pm_dst, pm_off, pm_ml, pm_cnt, nvm);
			SSTAMP_END(SP_MATCH);
		}
		pm_dst = m_dst;
		pm_off = m_off;
		pm_ml = m_ml;
		pm_cnt = ns;
		nvm_b0 = nvm;
	}
	if (!bad && !done) {
		why = 8;
		bad = true;
	}
	if (!bad && pm_cnt > 0) {
		vm_wait_all();
		run_batch_matches(ob, olim, pm_dst, pm_off, pm_ml, pm_cnt, nvm);
	}
	// nothing may still be landing in this workgroup's LDS when it ends
	vm_wait_all();
	SSTAMP_FLUSH();
	if (lane == 0) {
		if (bad) {
			status[b].code = DS_RETRY;
			status[b].detail = why;
			status[b].err_out_pos = uint32_t(p);
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

#ifdef LZ4ADA_SP_STAMPS
extern "C" int lz4ada_sp_stamps(unsigned long long* out, int reset)
{
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sparse::g_sp_stamps),
	                        sizeof(unsigned long long) * sparse::SP_NST) != hipSuccess)
		return -1;
	if (reset) {
		unsigned long long z[sparse::SP_NST] = {};
		if (hipMemcpyToSymbol(HIP_SYMBOL(sparse::g_sp_stamps), z, sizeof z) != hipSuccess)
			return -1;
	}
	return sparse::SP_NST;
}
#endif

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
