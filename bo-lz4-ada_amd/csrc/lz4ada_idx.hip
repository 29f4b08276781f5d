// lz4ada_idx.hip -- index-driven bulk decoder for independent blocks.
//
// Replaces the same reference path as k_decode_pc (lib/lz4ada.adb:716-904:
// Decompress_Full_Block / Decompress_Sequence / Write_Output /
// Output_With_History) with two passes that keep every lane busy instead of
// parsing one sequence chain per wave:
//
//  * k_index (pass 1, one wave per block).  The compressed payload is cut
//    into 256-byte segments, 64 per 16 KiB LDS-staged chunk, one per lane.
//    Every lane walks the sequence chain of its segment from a guessed
//    entry (its segment start; lane 0 from the exact entry carried from the
//    previous chunk), then each lane re-walks from the exit of the lane
//    before it, until no entry changes.  LZ4 chains started at a wrong byte
//    merge with the true chain within a few sequences, so this converges in
//    2-4 walks per segment.  The walk records, for every 32-byte
//    sub-segment, where the first sequence starting inside it begins
//    (1 byte; 0xFF = none).  Any malformed sequence marks the block
//    DS_RETRY.
//  * k_decode_idx (pass 2, one wave per block).  Batches of 64 sub-segments
//    (2 KiB of input): lane i walks the sequences starting in sub-segment i
//    from its index entry (LDS-staged input), a wave prefix sum places them
//    in the output, literals and matches whose source lies before the batch
//    are copied at once, lane-parallel, straight to HBM; long runs and
//    matches reading this batch's own output follow in output order
//    (a leader loop: the first pending item always runs, every other whose
//    source is already final runs with it).
//
// Blocks either pass declines (DS_RETRY: malformed data, a back-reference
// before the block start, an oversize block) are redone by k_decode_pc,
// which produces the exact statuses; so this pair never changes a result,
// only the speed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4ada_internal.h"
#include "lz4ada_dev.h"

namespace lz4ada {
namespace idx {

// Stored-block copies without a block checksum: nontemporal loads and
// stores (2; 1 = stores only, 0 = neither).  With a block checksum the copy
// stays cached: the checksum kernel beside it reads the same payload.  A/B, 2048 x 4 MiB stored blocks, twice (tools/st_ab.sh,
// DESIGN §3): 3.62 / 3.84 ms plain, 3.71 / 3.77 ms NT stores, 3.39 / 3.48 ms
// NT loads and stores (with block checksums beside: 9.32 / 9.71, 9.49 /
// 9.82, 8.68 / 8.73 ms).
#ifndef LZ4ADA_STORED_NT
#define LZ4ADA_STORED_NT 2
#endif
constexpr int SEG = 256;            // pass-1 segment per lane
constexpr int CHUNK = 64 * SEG;     // pass-1 staged chunk (16 KiB)
constexpr int SUB = 32;             // pass-2 sub-segment per lane
constexpr int NSUB = SEG / SUB;     // index records per segment
constexpr int BATCH = 64 * SUB;     // pass-2 batch (2 KiB of input)
constexpr int RING = 4 * BATCH;     // pass-2 staging ring
constexpr int LONG = 256;           // runs longer than this are copied by the whole wave
constexpr int32_t MAX_RUN = 1 << 28;  // length guard (block_max <= 4 MiB in the bulk path)
// Pass-1 lead-in (k_index): each lane first walks from this many bytes
// before its segment: about LEAD_SEQ sequences at the previous chunk's
// density (the first chunk: LEAD_IN0 bytes).
#ifndef LZ4ADA_LEAD_SEQ
#define LZ4ADA_LEAD_SEQ 60
#endif
constexpr int32_t LEAD_SEQ = LZ4ADA_LEAD_SEQ;
#ifndef LZ4ADA_LEAD_MAX
#define LZ4ADA_LEAD_MAX 1024
#endif
constexpr int32_t LEAD_IN0 = 256, LEAD_MIN = 256, LEAD_MAX = LZ4ADA_LEAD_MAX;
// Blocks with more than RLE_RATIO output bytes (slot capacity) per input
// byte are declined as sparse before any walk: few sequences with huge
// matches (runs), whose length extensions of hundreds of 255-bytes make the
// speculative walks crawl a lane per fixed-point iteration (53 per chunk,
// ~125k cycles each) -- k_decode_sparse's case (it declines dense data
// itself, so no result changes).
// (RLE_MIN_IN: the slot capacity overstates a short block's output, e.g. a
// frame's last block, and small blocks cost pass 1 little either way.)
constexpr uint64_t RLE_RATIO = 64;
constexpr uint32_t RLE_MIN_IN = 4096;

// vmcnt(0) through the builtin, so the compiler's wait pass sees it (an asm
// wait leaves the loads pending in its model: later register reuse on any
// path merging with this one then waits again)
__device__ __forceinline__ void vm_wait()
{
	asm volatile("" ::: "memory");
	__builtin_amdgcn_s_waitcnt(0x0F70);
	asm volatile("" ::: "memory");
}

// Diagnostic build only (-DLZ4ADA_IDX_STAMPS): cycles per phase, summed over
// waves (each stamp drains the wave's memory counters: read shares).
enum IdxPhase { I_STAGE, I_WALK0, I_ITER, I_CHUNKS, I_ITERS,
	            D_STAGE, D_WALK1, D_WALK2, D_TLDS, D_LIT, D_MFAR, D_NEAR, D_FLUSH, D_GLOBAL,
	            D_BATCHES, D_GBATCHES, D_ROUNDS, D_TASKS, D_LANES, I_STEPS, I_MAXST, IDX_NST };
#ifdef LZ4ADA_IDX_STAMPS
__device__ unsigned long long g_idx_stamps[IDX_NST];
#define ISTAMP_DECL uint64_t ist[IDX_NST] = {}; uint64_t ist_t = __builtin_amdgcn_s_memtime()
#define ISTAMP(ph)                                                           \
	do {                                                                     \
		asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");          \
		const uint64_t _n = __builtin_amdgcn_s_memtime();                    \
		ist[ph] += _n - ist_t;                                               \
		ist_t = _n;                                                          \
	} while (0)
#define ICOUNT(ph, v) (ist[ph] += uint64_t(v))
#define ISTAMP_FLUSH()                                                       \
	do {                                                                     \
		if (lane_id() == 0)                                                  \
			for (int _i = 0; _i < IDX_NST; ++_i)                             \
				atomicAdd(&g_idx_stamps[_i], (unsigned long long)ist[_i]);   \
	} while (0)
#else
#define ISTAMP_DECL
#define ISTAMP(ph)
#define ICOUNT(ph, v)
#define ISTAMP_FLUSH()
#endif

// Diagnostic build only (-DLZ4ADA_IDX_GATHERS): the 16-byte HBM loads of
// k_decode_idx's HBM-sourced matches: loads, 128-byte line touches (a load
// crossing a line boundary touches two; no de-duplication), batches -- to
// price the gather share of FETCH_SIZE.
#ifdef LZ4ADA_IDX_GATHERS
__device__ unsigned long long g_idx_gathers[4];  // loads, line touches, batches, input stagings
#define GCOUNT(i, v)                                                         \
	do {                                                                     \
		const uint64_t _v = uint64_t(v);                                     \
		if (lane_id() == 0 && _v)                                            \
			atomicAdd(&g_idx_gathers[i], (unsigned long long)_v);            \
	} while (0)
#else
#define GCOUNT(i, v)
#endif

// ---------------------------------------------------------------- byte access
// Block-relative byte p comes from LDS when [p, p+8) lies in the staged
// window [lo, hi), else from global memory (guarded by the frame end).
struct Src {
	const uint8_t* lds;  // LDS array; block-relative p at lds[(p + mis) & mask]
	uint32_t mask;       // LDS array size - 1 (power of two; a 16-byte mirror follows)
	int32_t mis;
	int32_t lo, hi;
	cg8* in;
	uintptr_t lim;
};

__device__ __forceinline__ uint32_t fetch4(const Src& S, int32_t p)
{
	if (p >= S.lo && p + 8 <= S.hi) {
		const uint32_t a = uint32_t(p + S.mis) & S.mask;
		const uint32_t* w = reinterpret_cast<const uint32_t*>(S.lds + (a & ~3u));
		const uint32_t w0 = w[0], w1 = w[1];  // w[1] may be in the mirror
		return __builtin_amdgcn_alignbyte(w1, w0, a & 3u);
	}
	const uintptr_t g = reinterpret_cast<uintptr_t>(S.in) + uintptr_t(intptr_t(p));
	uint32_t v = 0;
#pragma unroll
	for (int i = 0; i < 4; ++i)
		if (g + i < S.lim)
			v |= uint32_t(*reinterpret_cast<cg8*>(g + i)) << (8 * i);
	// settle this rare path's loads here: left pending, they make every
	// merge after it (the walk loops' heads) wait for all memory, the
	// in-flight next-chunk prefetch included
	__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
	return v;
}

// 16 bytes at byte a of a power-of-two LDS ring (mask = size - 1): three
// 8-byte-aligned ds_read_b64 (each wrapped on its own), a one-bit dword
// select and four v_alignbyte -- ld16u's select network costs ~4x the VALU.
__device__ __forceinline__ u32x4 ring16(const uint8_t* base, uint32_t a, uint32_t mask)
{
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

// 16 bytes at block-relative p (literal source): LDS or global.
__device__ __forceinline__ u32x4 fetch16(const Src& S, int32_t p)
{
	if (p >= S.lo && p + 16 <= S.hi)
		return ring16(S.lds, uint32_t(p + S.mis) & S.mask, S.mask);
	const uintptr_t g = reinterpret_cast<uintptr_t>(S.in) + uintptr_t(intptr_t(p));
	u32x4 v;
	if (g + 16 <= S.lim) {
		__builtin_memcpy(&v, reinterpret_cast<cg8*>(g), 16);
	} else {
		uint8_t t[16];
		for (int i = 0; i < 16; ++i)
			t[i] = (g + i < S.lim) ? *reinterpret_cast<cg8*>(g + i) : 0;
		__builtin_memcpy(&v, t, 16);
	}
	// settle the rare global read here (see fetch4): otherwise every use of
	// the LDS path's result waits for all memory -- the batch's in-flight
	// HBM match loads and flush stores included
	__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
	return v;
}

struct Seq {
	int32_t lit, L, off, ml, next;  // ml = 0: literal-only last sequence
};

// One sequence at block-relative p < n (Decompress_Sequence,
// lz4ada.adb:737-777, with the end-of-block rule of :748-764).  False on
// any malformed shape; the caller then declines the block.
__device__ __forceinline__ bool parse_seq(const Src& S, int32_t p, int32_t n, Seq& q)
{
	const uint32_t w = fetch4(S, p);
	const int32_t tk = int32_t(w & 0xffu);
	int32_t L = tk >> 4, M = tk & 15, x = p + 1;
	if (L == 15) {
		uint32_t e, k = 1, ww = w;
		do {
			if (x >= n || L > n)
				return false;
			if (k > 3) {
				ww = fetch4(S, x);
				k = 0;
			}
			e = (ww >> (8 * k)) & 0xffu;
			++k;
			++x;
			L += int32_t(e);
		} while (e == 255u);
	}
	q.lit = x;
	q.L = L;
	x += L;
	if (x >= n) {
		if (x > n || M != 0)
			return false;
		q.off = 0;
		q.ml = 0;
		q.next = n;
		return true;
	}
	if (x + 1 >= n)
		return false;
	uint32_t w2 = fetch4(S, x);
	q.off = int32_t(w2 & 0xffffu);
	if (q.off == 0)
		return false;
	x += 2;
	if (M == 15) {
		uint32_t e, k = 2;
		do {
			if (x >= n || M > MAX_RUN)
				return false;
			if (k > 3) {
				w2 = fetch4(S, x);
				k = 0;
			}
			e = (w2 >> (8 * k)) & 0xffu;
			++k;
			++x;
			M += int32_t(e);
		} while (e == 255u);
	}
	q.ml = M + 4;
	q.next = x;
	return true;
}

// parse_seq for the common shape, without branches: both length
// extensions at most one byte, every byte read in the LDS window, the
// sequence well before the block end.  Anything else (and malformed data)
// takes parse_seq; the result is the same.
__device__ __forceinline__ bool parse_fast(const Src& S, int32_t p, int32_t n, Seq& q)
{
	const uint32_t a = uint32_t(p + S.mis) & S.mask;
	const uint32_t* wa = reinterpret_cast<const uint32_t*>(S.lds + (a & ~3u));
	const uint32_t w = __builtin_amdgcn_alignbyte(wa[1], wa[0], a & 3u);
	const uint32_t tk = w & 0xffu, e1 = (w >> 8) & 0xffu;
	const bool x1 = tk >= 0xf0u, x2 = (tk & 15u) == 15u;
	const int32_t L = int32_t(tk >> 4) + (x1 ? int32_t(e1) : 0);
	const int32_t lit = p + 1 + (x1 ? 1 : 0);
	const int32_t x = lit + L;
	const uint32_t b = uint32_t(x + S.mis) & S.mask;
	const uint32_t* wb = reinterpret_cast<const uint32_t*>(S.lds + (b & ~3u));
	const uint32_t w2 = __builtin_amdgcn_alignbyte(wb[1], wb[0], b & 3u);
	const uint32_t e2 = (w2 >> 16) & 0xffu;
	q.lit = lit;
	q.L = L;
	q.off = int32_t(w2 & 0xffffu);
	q.ml = int32_t(tk & 15u) + 4 + (x2 ? int32_t(e2) : 0);
	q.next = x + 2 + (x2 ? 1 : 0);
	const bool ok = p >= S.lo && x + 8 <= S.hi && x + 8 <= n && !(x1 && e1 == 255u) &&
	                !(x2 && e2 == 255u) && q.off != 0;
	if (__builtin_expect(ok, 1))
		return true;
	return parse_seq(S, p, n, q);
}

// parse_fast's branch-free form alone: false where it does not apply (the
// caller then runs parse_seq for that sequence; q is a placeholder)
__device__ __forceinline__ bool parse_fast_try(const Src& S, int32_t p, int32_t n, Seq& q)
{
	const uint32_t a = uint32_t(p + S.mis) & S.mask;
	const uint32_t* wa = reinterpret_cast<const uint32_t*>(S.lds + (a & ~3u));
	const uint32_t w = __builtin_amdgcn_alignbyte(wa[1], wa[0], a & 3u);
	const uint32_t tk = w & 0xffu, e1 = (w >> 8) & 0xffu;
	const bool x1 = tk >= 0xf0u, x2 = (tk & 15u) == 15u;
	const int32_t L = int32_t(tk >> 4) + (x1 ? int32_t(e1) : 0);
	const int32_t lit = p + 1 + (x1 ? 1 : 0);
	const int32_t x = lit + L;
	const uint32_t b = uint32_t(x + S.mis) & S.mask;
	const uint32_t* wb = reinterpret_cast<const uint32_t*>(S.lds + (b & ~3u));
	const uint32_t w2 = __builtin_amdgcn_alignbyte(wb[1], wb[0], b & 3u);
	const uint32_t e2 = (w2 >> 16) & 0xffu;
	q.lit = lit;
	q.L = L;
	q.off = int32_t(w2 & 0xffffu);
	q.ml = int32_t(tk & 15u) + 4 + (x2 ? int32_t(e2) : 0);
	q.next = x + 2 + (x2 ? 1 : 0);
	return p >= S.lo && x + 8 <= S.hi && x + 8 <= n && !(x1 && e1 == 255u) && !(x2 && e2 == 255u) &&
	       q.off != 0;
}


// 16 bytes from global memory at byte address a, never reading at or past lim.
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

// Exact-length store of n (0..16) bytes to global memory.
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

// ------------------------------------------------------------------ pass 1

struct alignas(16) IdxLds {
	uint8_t buf[CHUNK + 16];       // staged chunk; + mirror of its first 16 bytes
	uint32_t rbm[64][NSUB + 1];    // each lane's records from its latest walk: start
	uint16_t rcnt[64][NSUB + 1];   // bitmaps and output bytes (>= 0xFFFF: in HBM)
};

// Walk the chain from e (an entry at or after this lane's segment start s)
// over the sequences starting before seg_end; returns the exit (first
// chain position >= seg_end, or n).  A malformed sequence sets err (epos:
// its position) and returns seg_end as a guess: from a wrong (speculative)
// entry that is just a dead chain, and a -1 would poison every lane after
// it one iteration at a time.
//
// Every walk rewrites the segment's NSUB records (sub-segment k = bytes
// [s + 32k, s + 32k + 32)) in LDS: rb[k] bit j = a sequence starts at byte
// j, rc[k] = the output bytes (literals + match) of the sequences starting
// there.  The lane's last walk -- from the true entry -- leaves the exact
// records; k_index writes them to HBM once per chunk.  An output count that
// does not fit 16 bits goes straight to its record's high word in HBM
// (ghi[2k]; long RLE runs).
//
// Re-walk (may_stop: the lane's previous walk, exit y_old, had no error):
// chains are deterministic, so once this walk reaches a position the
// previous walk started a sequence at, the rest is the previous walk.  It
// finishes that sub-segment (its count mixes both walks' sequences) and
// stops: later records and the exit are the previous walk's.  Chains from a
// wrong entry merge within ~14 sequences, so a re-walk costs a fraction of
// a segment.
template <int NS = NSUB>
__device__ __forceinline__ int32_t walk_segment(const Src& S, int32_t e, int32_t s, int32_t seg_end,
                                                int32_t n, uint32_t* rb, uint16_t* rc, uint32_t* ghi,
                                                bool& err, int32_t& epos, int32_t y_old,
                                                bool may_stop, int32_t& nst)
{
	nst = 0;  // sequence steps (diagnostic counts; dead in the product)
	err = false;
	epos = INT32_MAX;
	auto put = [&](int32_t k, uint32_t b, uint32_t c) {
		rb[k] = b;
		rc[k] = uint16_t(min(c, 0xFFFFu));
		if (c >= 0xFFFFu)
			ghi[2 * k] = c;
	};
	// the dword pair at pos, shifted to pos (LDS; a position outside the
	// staged window reads garbage, which parse_fast's window test rejects)
	auto pair_at = [&](int32_t pos) -> uint32_t {
		const uint32_t a = uint32_t(pos + S.mis) & S.mask;
		const uint32_t* wa = reinterpret_cast<const uint32_t*>(S.lds + (a & ~3u));
		return __builtin_amdgcn_alignbyte(wa[1], wa[0], a & 3u);
	};
	int32_t p = e;
	int32_t kc = -1, nxt = 0;  // sub-segment being counted; next record to write
	uint32_t bm = 0, cnt = 0;
	bool merged = false;
	uint32_t w = p < seg_end ? pair_at(p) : 0u;  // token pair of the sequence at p
	while (p < seg_end) {
		const int32_t k = (p - s) >> 5;
		if (k != kc) {
			if (kc >= 0)
				put(kc, bm, cnt);
			if (merged)
				return y_old;
			for (; nxt < k; ++nxt)
				if (nxt != kc)
					put(nxt, 0, 0);
			nxt = k + 1;
			kc = k;
			bm = cnt = 0;
		}
		const uint32_t bit = 1u << ((p - s) & 31);
		if (may_stop && (rb[k] & bit))
			merged = true;  // rb[k] is still the previous walk's record
		bm |= bit;
		++nst;
		// parse_fast from the token pair in hand; the offset pair at x and
		// the next sequence's token pair load together (the next position
		// needs only this token), so a step waits for one LDS round trip
		const uint32_t tk = w & 0xffu, e1 = (w >> 8) & 0xffu;
		const bool x1 = tk >= 0xf0u, x2 = (tk & 15u) == 15u;
		const int32_t L = int32_t(tk >> 4) + (x1 ? int32_t(e1) : 0);
		const int32_t x = p + 1 + (x1 ? 1 : 0) + L;
		const int32_t np = x + 2 + (x2 ? 1 : 0);
		const uint32_t w2 = pair_at(x), wn = pair_at(np);
		const uint32_t e2 = (w2 >> 16) & 0xffu;
		Seq q;
		q.L = L;
		q.ml = int32_t(tk & 15u) + 4 + (x2 ? int32_t(e2) : 0);
		q.next = np;
		const bool ok = p >= S.lo && x + 8 <= S.hi && x + 8 <= n && !(x1 && e1 == 255u) &&
		                !(x2 && e2 == 255u) && (w2 & 0xffffu) != 0;
		if (!ok) {  // rare shapes (and malformed data): the exact parse
			if (!parse_seq(S, p, n, q)) {
				err = true;
				epos = p;
				return seg_end;
			}
		}
		cnt += uint32_t(q.L + q.ml);
		p = q.next;
		w = ok ? wn : pair_at(p);
	}
	if (kc >= 0)
		put(kc, bm, cnt);
	if (!merged)
		for (; nxt < NS; ++nxt)
			put(nxt, 0, 0);
	return p;
}

// The chain position after the sequence at p, for the lead-in walk: only
// a guess, so no checks, and every length extension taken as one byte (a
// longer one just makes a wrong guess, which the re-walks fix) -- then the
// token's dword pair is the one LDS read the step waits for.
__device__ __forceinline__ int32_t skip_seq(const Src& S, int32_t p)
{
	const uint32_t a = uint32_t(p + S.mis) & S.mask;
	const uint32_t* wa = reinterpret_cast<const uint32_t*>(S.lds + (a & ~3u));
	const uint32_t w = __builtin_amdgcn_alignbyte(wa[1], wa[0], a & 3u);
	const uint32_t tk = w & 0xffu;
	const int32_t x1 = tk >= 0xf0u ? 1 : 0;
	const int32_t L = int32_t(tk >> 4) + (x1 ? int32_t((w >> 8) & 0xffu) : 0);
	return p + 3 + x1 + L + ((tk & 15u) == 15u ? 1 : 0);
}

__device__ __forceinline__ int32_t lead_in_bytes(int32_t starts)
{
	const int32_t l = LEAD_SEQ * (CHUNK / max(starts, 1));
	return __builtin_amdgcn_readfirstlane(min(max(l, LEAD_MIN), LEAD_MAX));
}

// Pass 1 of block b (the body of k_index; k_decode_idx mode 3 runs it
// before pass 2 of the same block).
__device__ __forceinline__ void index_block(IdxLds& X, const uint8_t* __restrict__ frame,
                                            uint64_t frame_len,
                                            const lz4ada_block_desc* __restrict__ desc, uint32_t b,
                                            uint8_t* __restrict__ tab_all,
                                            lz4ada_block_status* __restrict__ status)
{
	const int32_t lane = int32_t(lane_id());
	const lz4ada_block_desc d = desc[b];
	if (d.flags & LZ4ADA_BLOCK_STORED) {
		if (lane == 0)
			status[b].code = DS_OK;
		return;
	}
	if (d.in_len >= RLE_MIN_IN && uint64_t(d.in_len) * RLE_RATIO < uint64_t(d.out_cap)) {
		if (lane == 0)
			status[b].code = DS_SPARSE;
		return;
	}
	cg8* in = gptr(frame) + d.in_off;
	const int32_t n = int32_t(d.in_len);
	const uintptr_t lim = reinterpret_cast<uintptr_t>(frame) + frame_len;
	const int32_t mis = int32_t(reinterpret_cast<uintptr_t>(in) & 15u);
	uint64_t* tab = reinterpret_cast<uint64_t*>(tab_all) + (((d.in_off >> 8) + b) << 3);

	Src S;
	S.lds = X.buf;
	S.mask = CHUNK - 1;
	S.mis = mis;
	S.in = in;
	S.lim = lim;

	// 16 KiB chunk at aligned address a (lanes: 16 x 16 bytes each), the
	// next one loaded while the current one is walked
	auto load16k = [&](uintptr_t a, u32x4 (&v)[CHUNK / 1024]) {
		if (a + CHUNK <= lim) {
#pragma unroll
			for (int r = 0; r < CHUNK / 1024; ++r)
				__builtin_memcpy(&v[r], reinterpret_cast<cg8*>(a + uintptr_t(1024 * r + 16 * lane)), 16);
		} else {
#pragma unroll
			for (int r = 0; r < CHUNK / 1024; ++r)
				v[r] = gload16(a + uintptr_t(1024 * r + 16 * lane), lim);
		}
	};
	const uintptr_t abase = reinterpret_cast<uintptr_t>(in) - uintptr_t(mis);
	u32x4 pf[CHUNK / 1024];
	if (n > 0)
		load16k(abase, pf);

	ISTAMP_DECL;
	int32_t E = 0;  // exact chain entry of the current chunk
	int32_t lead = LEAD_IN0;  // lead-in bytes (from the previous chunk's density)
	bool bad = false;
	bool sparse = false;  // declined as literal-heavy (k_decode_sparse takes it)
	for (int32_t C = 0; C < n && !bad; C += CHUNK) {
		// stage block-relative [C - mis, C - mis + CHUNK) (16-byte aligned addresses)
#pragma unroll
		for (int r = 0; r < CHUNK / 1024; ++r)
			*reinterpret_cast<u32x4*>(&X.buf[1024 * r + 16 * lane]) = pf[r];
		if (lane == 0)
			*reinterpret_cast<u32x4*>(&X.buf[CHUNK]) = pf[0];
		__syncthreads();
		if (C + CHUNK < n)
			load16k(abase + uintptr_t(C + CHUNK), pf);
		S.lo = C - mis;
		S.hi = C - mis + CHUNK;
		ISTAMP(I_STAGE);
		ICOUNT(I_CHUNKS, 1);

		const int32_t s = C + SEG * lane;
		const int32_t seg_end = min(s + SEG, n);
		// Entry of lane i = max exit of lanes < i (lane 0: the exact entry E).
		// True exits never decrease along the chunk, so the fixed point is
		// the true chain, and a run of segments a long sequence jumps over
		// is crossed in one step instead of one iteration per segment.
		int32_t ein = (lane == 0) ? E : s;
		if (lane > 0 && s < n) {
			// Lead-in: walk from OV bytes before the segment to find a
			// likelier entry than s itself -- chains from a wrong start merge
			// with the true one within ~14 sequences, so by s this one mostly
			// has, and the re-walk rounds below (most of pass 1's time) are
			// rarely needed.
			int32_t p = max(s - lead, C);  // inside the staged chunk
			while (p < s)
				p = skip_seq(S, p);
			ein = p;
		}
		uint32_t* ghi = reinterpret_cast<uint32_t*>(tab + (C >> 5) + NSUB * lane) + 1;
#ifdef LZ4ADA_IDX_NO_MERGE_STOP
		constexpr bool no_stop = true;
#else
		constexpr bool no_stop = false;
#endif
		int32_t epos = INT32_MAX;
		bool err = false;
		int32_t nst = 0;
		int32_t y = (s < n) ? walk_segment(S, ein, s, seg_end, n, X.rbm[lane], X.rcnt[lane], ghi, err,
		                                   epos, 0, false, nst)
		                    : ein;
		ISTAMP(I_WALK0);
		ICOUNT(I_STEPS, __shfl(wave_incl_scan(nst), 63));
		ICOUNT(I_MAXST, __shfl(wave_incl_max(nst), 63));
		for (int it = 0; it < 64; ++it) {
			int32_t prev = __shfl_up(wave_incl_max(y), 1);
			if (lane == 0)
				prev = E;
			const bool changed = prev != ein;
			if (!__any(changed))
				break;
			ICOUNT(I_ITERS, 1);
			nst = 0;
			if (changed) {
				ein = prev;
				if (s < n) {
					y = walk_segment(S, ein, s, seg_end, n, X.rbm[lane], X.rcnt[lane], ghi, err, epos, y,
					                 !err && !no_stop, nst);
				} else {
					y = ein;
					err = false;
				}
			}
			ICOUNT(I_STEPS, __shfl(wave_incl_scan(nst), 63));
			ICOUNT(I_MAXST, __shfl(wave_incl_max(nst), 63));
		}
		ISTAMP(I_ITER);
		// converged: every entry is the true chain position, and every
		// lane's records are those of its last walk: to HBM, coalesced
		if (s < n && err)
			bad = true;

		bad = __any(bad);
		wave_lds_fence();
		int32_t starts = 0;  // sequence starts in this chunk (sizes the next lead-in)
#pragma unroll
		for (int i = 0; i < NSUB; ++i) {
			const int32_t r = 64 * i + lane, sg = r / NSUB, sb = r & (NSUB - 1);
			if (C + SEG * sg < n) {
				const uint32_t bmv = X.rbm[sg][sb], c16 = X.rcnt[sg][sb];
				starts += __popc(bmv);
				if (c16 != 0xFFFFu)
					tab[(C >> 5) + r] = uint64_t(bmv) | (uint64_t(c16) << 32);
				else  // the exact count is in the high word already
					*reinterpret_cast<uint32_t*>(tab + (C >> 5) + r) = bmv;
			}
		}
		E = __shfl(wave_incl_max(y), 63);
		lead = lead_in_bytes(__shfl(wave_incl_scan(starts), 63));
		if (C == 0 && n >= 4 * CHUNK) {
			// Sparse chains (over 64 input bytes per sequence: long literal
			// runs) defeat the speculative walks -- every segment's guess
			// misses and the entries crawl one lane per iteration -- and are
			// the one-wave scalar parse's best case: decline the block (large
			// blocks only: a short one costs a few chunks either way).
			int32_t used = 0;  // sub-segments holding a sequence start
			if (s < n)
				for (int k = 0; k < NSUB; ++k)
					used += X.rbm[lane][k] ? 1 : 0;
			if (!bad && __shfl(wave_incl_scan(used), 63) < CHUNK / SUB / 4)
				bad = sparse = true;
		}
		__syncthreads();  // the next chunk overwrites the staging buffer
	}
	if (E != n)
		bad = true;
	if (lane == 0)
		status[b].code = bad ? (sparse ? DS_SPARSE : DS_RETRY) : DS_OK;
	ISTAMP_FLUSH();
}

__global__ __launch_bounds__(64) void k_index(const uint8_t* __restrict__ frame, uint64_t frame_len,
                                               const lz4ada_block_desc* __restrict__ desc,
                                               uint32_t nblocks, uint8_t* __restrict__ tab_all,
                                               lz4ada_block_status* __restrict__ status)
{
	__shared__ IdxLds X;
	if (blockIdx.x < nblocks)
		index_block(X, frame, frame_len, desc, blockIdx.x, tab_all, status);
}

// ------------------------------------------------------------------ pass 2

// Matches: copy len bytes to ob[dst] from ob[dst - off] (Output_With_History,
// lz4ada.adb:845-904, for an in-block source).  One lane, exact stores.
// Sources must be final; for off < len the lane reads back its own first
// 16 bytes (made visible by a wave-wide wait) or fills an off < 16 pattern.
__device__ __forceinline__ void lane_match(g8* ob, uintptr_t olim, int32_t dst, int32_t off,
                                           int32_t len)
{
	const uintptr_t base = reinterpret_cast<uintptr_t>(ob);
	if (off < 16 && off < len) {
		const u32x4 s = gload16(base + uintptr_t(dst - off), olim);
		u32x4 pv;
		int32_t width, stp;
		make_pattern(uint64_t(s.x) | (uint64_t(s.y) << 32), uint64_t(s.z) | (uint64_t(s.w) << 32),
		             off, pv, width, stp);
		for (int32_t k = 0; k < len; k += stp)
			gstore_n(ob + dst + k, pv, min(width, len - k));
		return;
	}
	int32_t r = 0;
	for (int32_t k = 0; k < len; k += 16) {
		const u32x4 v = gload16(base + uintptr_t(dst - off + r), olim);
		gstore_n(ob + dst + k, v, min(16, len - k));
		if (k == 0 && off < len)
			vm_wait();  // bytes [dst, dst+16) are read back by later chunks
		r += 16;
		if (r >= off)
			r -= off;
	}
}

// Whole-wave copy of one match (any length).
__device__ __forceinline__ void wave_match(g8* ob, uintptr_t olim, int32_t dst, int32_t off,
                                           int32_t len)
{
	const int32_t lane = int32_t(lane_id());
	const uintptr_t base = reinterpret_cast<uintptr_t>(ob);
	if (off < 16 && off < len) {
		const u32x4 s = gload16(base + uintptr_t(dst - off), olim);
		u32x4 pv;
		int32_t width, stp;
		make_pattern(uint64_t(s.x) | (uint64_t(s.y) << 32), uint64_t(s.z) | (uint64_t(s.w) << 32),
		             off, pv, width, stp);
		for (int32_t c = 0; c < len; c += 64 * stp) {
			const int32_t k = c + lane * stp;
			if (k < len)
				gstore_n(ob + dst + k, pv, min(width, len - k));
		}
		return;
	}
	// each step copies span <= off bytes, so it reads only bytes already final
	const int32_t span = off >= 1024 ? 1024 : (off & ~15);
	for (int32_t c = 0; c < len; c += span) {
		const int32_t k = c + 16 * lane;
		if (16 * lane < span && k < len) {
			const u32x4 v = gload16(base + uintptr_t(dst + k - off), olim);
			gstore_n(ob + dst + k, v, min(16, len - k));
		}
		if (off < len)
			vm_wait();
	}
}

// Whole-wave copy of one literal run from the compressed input.  NT
// (stored blocks, experiment LZ4ADA_STORED_NT): 1 = nontemporal stores,
// 2 = nontemporal loads too.
template <int NT = 0>
__device__ __forceinline__ void wave_literal(g8* ob, int32_t dst, const Src& S, int32_t src,
                                             int32_t len)
{
	const int32_t lane = int32_t(lane_id());
	// 8 KiB per step, every load issued before the first store (a stored
	// block is pure copy: one memory round trip per 8 KiB, not per 1 KiB)
	constexpr int U = 8;
	for (int32_t c = 0; c < len; c += 1024 * U) {
		u32x4 v[U];
#pragma unroll
		for (int u = 0; u < U; ++u) {
			const int32_t k = c + 1024 * u + 16 * lane;
			const uintptr_t a = reinterpret_cast<uintptr_t>(S.in) + uintptr_t(src + k);
			if (NT >= 2 && k + 16 <= len && a + 16 <= S.lim)
				v[u] = __builtin_nontemporal_load(reinterpret_cast<const GLOBAL u32x4*>(a));
			else if (k < len)
				v[u] = gload16(a, S.lim);
		}
#pragma unroll
		for (int u = 0; u < U; ++u) {
			const int32_t k = c + 1024 * u + 16 * lane;
			if (NT >= 1 && k + 16 <= len)
				__builtin_nontemporal_store(v[u], reinterpret_cast<GLOBAL u32x4*>(ob + dst + k));
			else if (k < len)
				gstore_n(ob + dst + k, v[u], min(16, len - k));
		}
	}
}

// Deferred work item of one lane: a long literal run (src >= 0: input
// position) or a match (src = -offset) that is long or reads this batch.
struct Item {
	int32_t dst, len, src;
};

// Next deferred item of this lane from cursor (p, o, part); part 0 = the
// sequence's literals are next, 1 = its match.  far_end: output position
// before which every byte is final (the batch start).
__device__ __forceinline__ bool next_item(const Src& S, int32_t& p, int32_t& o, int32_t& part,
                                          int32_t sub_end, int32_t n, int32_t far_end, Item& it)
{
	while (p < sub_end) {
		Seq q;
		parse_seq(S, p, n, q);  // validated by the first walk of this batch
		if (part == 0) {
			part = 1;
			if (q.L > LONG) {
				it.dst = o;
				it.len = q.L;
				it.src = q.lit;
				return true;
			}
		}
		const int32_t mdst = o + q.L;
		p = q.next;
		o = mdst + q.ml;
		part = 0;
		if (q.ml > 0) {
			const int32_t dep_end = mdst - q.off + min(q.off, q.ml);
			if (q.ml > LONG || dep_end > far_end) {
				it.dst = mdst;
				it.len = q.ml;
				it.src = -q.off;
				return true;
			}
		}
	}
	return false;
}

// Oversized batches (a lane whose sequences decode to more than the LDS
// window, e.g. long RLE runs): the batch goes straight to HBM.  Literals
// and matches reading output older than the batch are copied at once;
// long runs and matches reading the batch itself follow in output order
// through a leader loop (the first pending item always runs; any other
// whose source is already final runs with it), with a wave-wide wait
// between rounds.  Returns false on a reference before the block start
// (hb: history bytes before it, linked frames).
__device__ __forceinline__ bool batch_global(const Src& S, g8* ob, uintptr_t olim, int32_t p0,
                                          int32_t sub_end, int32_t n, int32_t o_lane,
                                          int32_t o_batch, int32_t hb)
{
	const int32_t lane = int32_t(lane_id());
	int32_t cp = 0, co = 0, cpart = 0;
	bool has = false, pre = false;
	{
		int32_t o = o_lane;
		for (int32_t p = p0; p < sub_end;) {
			Seq q;
			parse_seq(S, p, n, q);
			if (q.L > LONG) {
				if (!has) {
					has = true;
					cp = p;
					co = o;
					cpart = 0;
				}
			} else {
				for (int32_t c = 0; c < q.L; c += 16)
					gstore_n(ob + o + c, fetch16(S, q.lit + c), min(16, q.L - c));
			}
			const int32_t mdst = o + q.L;
			if (q.ml > 0) {
				if (q.off > mdst + hb)
					pre = true;  // reference before the block start (D2)
				if (hb > 0 && q.off > mdst && q.off >= D1_OFF)
					pre = true;  // a possible quirk-D1 read: P flags / emulates those, so decline
				const int32_t dep_end = mdst - q.off + min(q.off, q.ml);
				if (q.ml > LONG || dep_end > o_batch) {
					if (!has) {
						has = true;
						cp = p;
						co = o;
						cpart = 1;
					}
				} else if (!pre) {
					lane_match(ob, olim, mdst, q.off, q.ml);
				}
			}
			o = mdst + q.ml;
			p = q.next;
		}
	}
	if (__any(pre))
		return false;
	Item it = {0, 0, 0};
	if (has)
		has = next_item(S, cp, co, cpart, sub_end, n, o_batch, it);
	if (__any(has)) {
		vm_wait();  // everything above is final
		for (;;) {
			const uint64_t m = __ballot(has);
			if (m == 0)
				break;
			const int32_t leader = __builtin_ctzll(m);
			const int32_t ldst = __shfl(it.dst, leader);
			const int32_t llen = __shfl(it.len, leader);
			const int32_t lsrc = __shfl(it.src, leader);
			bool ready;
			if (llen > LONG) {
				if (lsrc >= 0)
					wave_literal(ob, ldst, S, lsrc, llen);
				else
					wave_match(ob, olim, ldst, -lsrc, llen);
				ready = (lane == leader);
			} else {
				ready = has && it.len <= LONG &&
				        (it.src >= 0 || it.dst + it.src + min(-it.src, it.len) <= ldst);
				if (ready) {
					if (it.src >= 0)
						for (int32_t c = 0; c < it.len; c += 16)
							gstore_n(ob + it.dst + c, fetch16(S, it.src + c), min(16, it.len - c));
					else
						lane_match(ob, olim, it.dst, -it.src, it.len);
				}
			}
			vm_wait();
			if (ready)
				has = next_item(S, cp, co, cpart, sub_end, n, o_batch, it);
		}
	}
	return true;
}

// ------------------------------------------------------ LDS output window
// A batch whose output fits in OW bytes is assembled in an LDS ring that
// also keeps the 2+ KiB of output before it, then flushed to HBM with
// aligned 16-byte stores (the partial last 16 bytes go with the next batch).
constexpr int OW = 4080;        // max batch output assembled in LDS (see glo below)
constexpr int ORING = 8192;     // LDS output ring (batch + history)
constexpr int OMASK = ORING - 1;
constexpr int MAXSEQ = 128;     // sequences per batch (2 rounds: 192 VGPRs; 256 took 254 and spilled)
constexpr int RMAX = MAXSEQ / 64;  // rounds of 64 sequences per batch
constexpr int GC = 1;           // 16-byte pieces an HBM-sourced match loads in its own lane (1: fewest registers; the rest are dealt)
constexpr int FLUSH_ST = (OW + 15) / 16 / 64 + 1;  // store instructions per flush (fixed)
static_assert(2 * OW + 16 <= ORING, "batch + its HBM threshold must fit the ring");
// batch cut limits (experiments: a smaller cut with the same ring and HBM threshold)
#ifndef LZ4ADA_OW_CUT
#define LZ4ADA_OW_CUT OW
#endif
#ifndef LZ4ADA_SEQ_CUT
#define LZ4ADA_SEQ_CUT MAXSEQ
#endif

struct alignas(16) DecLds {
	uint8_t ring[RING + 16];      // staged input: 4 chunks of 2 KiB (+ mirror)
	uint8_t oring[ORING];         // output window
	uint16_t cst[MAXSEQ];         // the batch's sequence starts, in order
	uint8_t own[256];             // piece -> owning lane (dealt HBM pieces)
	uint64_t rrec[4 * 64];        // pass-1 records of the staged chunks' sub-segments
	uint64_t ldesc[2 * 64];       // literal runs of both rounds (dealt literal pieces)
	uint32_t plut[16 * 4];        // v_perm selectors of the period-off patterns (pattern_lut_init)
	uint8_t junk[16];             // target of the stores a lane does not need (lds_store_bf)
};
static_assert(sizeof(DecLds) <= 20480, "8 waves per CU: at most 20 KiB of LDS per wave");

// The output window and per-wave scratch of an LDS layout: DecLds (one
// wave per block) holds them directly; a k_decode_pp2 wave's view (WP2,
// below) picks its wave's scratch.
__device__ __forceinline__ uint8_t* oring_of(DecLds& D) { return D.oring; }
__device__ __forceinline__ const uint8_t* oring_of(const DecLds& D) { return D.oring; }
__device__ __forceinline__ uint8_t* own_of(DecLds& D) { return D.own; }
__device__ __forceinline__ uint64_t* ldesc_of(DecLds& D) { return D.ldesc; }
// Layouts with junk bytes and the pattern selectors (the one-wave decoder):
// branch-free exact stores (lds_store_bf) and period patterns by v_perm
// (pattern_perm); the two-wave layout keeps the branching forms.
template <class LD>
struct lds_fast {
	static constexpr bool value = false;
};
template <>
struct lds_fast<DecLds> {
	static constexpr bool value = true;
};
__device__ __forceinline__ uint8_t* junk_of(DecLds& D) { return D.junk; }
__device__ __forceinline__ const uint32_t* plut_of(const DecLds& D) { return D.plut; }
template <class LD>
__device__ __forceinline__ uint8_t* junk_of(LD&) { return nullptr; }
template <class LD>
__device__ __forceinline__ const uint32_t* plut_of(const LD&) { return nullptr; }
// the window's size - 1 (a power of two) for a layout: ORING unless the
// layout says otherwise (the pipelined pair's 16 KiB window)
template <class LD>
__device__ __forceinline__ constexpr uint32_t omask_of(const LD&) { return OMASK; }

// Exact store of n (0..16) bytes of v at p, without branches: each of the
// five stores (16, 8, 4, 2, 1 bytes) goes to its place or, when n does not
// take it, to the 16 junk bytes, so every lane runs the same five ds_write
// instructions (lds_store_n's four divergent branches cost a wave whose
// lanes disagree on n all of them, with their exec-mask bookkeeping).
__device__ __forceinline__ void lds_store_bf(uint8_t* p, uint8_t* junk, u32x4 v, uint32_t n)
{
	const uint64_t lo = uint64_t(v.x) | (uint64_t(v.y) << 32);
	const uint64_t hi = uint64_t(v.z) | (uint64_t(v.w) << 32);
	__builtin_memcpy(n >= 16u ? p : junk, &v, 16);
	__builtin_memcpy((n & 8u) ? p : junk, &lo, 8);
	const uint64_t r8 = (n & 8u) ? hi : lo;
	uint8_t* const p4 = p + (n & 8u);
	const uint32_t w4 = uint32_t(r8);
	__builtin_memcpy((n & 4u) ? p4 : junk, &w4, 4);
	const uint32_t r4 = (n & 4u) ? uint32_t(r8 >> 32) : w4;
	uint8_t* const p2 = p4 + (n & 4u);
	const uint16_t w2 = uint16_t(r4);
	__builtin_memcpy((n & 2u) ? p2 : junk, &w2, 2);
	*((n & 1u) ? p2 + (n & 2u) : junk) = uint8_t((n & 2u) ? (r4 >> 16) : r4);
}

// Exact-length store of n bytes (fast layouts: 0..16; else 1..16) at
// output position x into the ring.
template <class LD>
__device__ __forceinline__ void ostore(LD& L, int32_t x, u32x4 v, int32_t n)
{
	const uint32_t a = uint32_t(x) & omask_of(L);
	if constexpr (lds_fast<LD>::value) {
		// a store wrapping the ring's end (one piece every 8 KiB of output)
		// takes the byte loop below, the wave's other lanes with it
		if (__builtin_expect(!__any(a + uint32_t(n) > omask_of(L) + 1), 1)) {
			lds_store_bf(&oring_of(L)[a], junk_of(L), v, uint32_t(n));
			return;
		}
	}
	if (a + uint32_t(n) <= omask_of(L) + 1) {
		// one ds_write_b128 even when misaligned: 256 cycles against 1579
		// for four ds_write_b32 (each misaligned one is split too) and 384
		// for 16 ds_write_b8 (tools/lds_bench.hip, dependent chain)
		lds_store_n(&oring_of(L)[a], v, n);
		return;
	}
	const uint64_t lo = uint64_t(v.x) | (uint64_t(v.y) << 32);
	const uint64_t hi = uint64_t(v.z) | (uint64_t(v.w) << 32);
	for (int32_t i = 0; i < n; ++i) {
		const uint64_t w = i < 8 ? lo : hi;
		oring_of(L)[(a + uint32_t(i)) & omask_of(L)] = uint8_t(w >> (8 * (i & 7)));
	}
}

template <class LD>
__device__ __forceinline__ u32x4 oload16(const LD& L, int32_t x)
{
	return ring16(oring_of(L), uint32_t(x) & omask_of(L), omask_of(L));
}

// Store steps and phases of period-off patterns without integer division:
// bits 5(o-1).. = o * (16 / o), bits 40 + 2(o-1).. = 8 mod o, for o = 1..8.
constexpr uint64_t pattern_lut()
{
	uint64_t v = 0;
	for (int o = 1; o <= 8; ++o)
		v |= (uint64_t(o * (16 / o)) << (5 * (o - 1))) | (uint64_t(8 % o) << (40 + 2 * (o - 1)));
	return v;
}
constexpr uint64_t PAT_LUT = pattern_lut();

// 16 bytes of the period-off (1..15) sequence whose first off bytes are
// s0|s1's, and the largest multiple of off <= 16: storing it every stp
// bytes keeps the phase.
__device__ __forceinline__ void make_pattern16(uint64_t s0, uint64_t s1, int32_t off, u32x4& pv,
                                               int32_t& stp)
{
	uint64_t x, hi;
	if (off <= 8) {
		x = off == 8 ? s0 : (s0 & ((uint64_t(1) << (8 * off)) - 1));
		// doubling x |= x << 8w for w = off, 2 off, 4 off while w < 8, with
		// selects instead of a lane-divergent loop
#pragma unroll
		for (int i = 0; i < 3; ++i) {
			const int32_t w = off << i;
			x |= w < 8 ? x << (8 * w) : 0;
		}
		const uint32_t sh = uint32_t(off - 1);
		stp = int32_t((PAT_LUT >> (5 * sh)) & 31u);
		const int32_t r = int32_t((PAT_LUT >> (40 + 2 * sh)) & 3u);
		// bytes 8..15: x[r..7], then x from 8 - off on (x is off-periodic)
		hi = r == 0 ? x : (x >> (8 * r)) | ((x >> (8 * (8 - off))) << (8 * (8 - r)));
	} else {
		const int32_t r = off - 8;
		x = s0;
		hi = (s1 & ((uint64_t(1) << (8 * r)) - 1)) | (s0 << (8 * r));
		stp = off;
	}
	pv.x = uint32_t(x);
	pv.y = uint32_t(x >> 32);
	pv.z = uint32_t(hi);
	pv.w = uint32_t(hi >> 32);
}

// a's bytes j < c, b's from c on (c = 1..15)
__device__ __forceinline__ u32x4 merge_at(u32x4 a, u32x4 b, int32_t c)
{
	auto m = [c](int32_t d) -> uint32_t {
		const int32_t t = c - 4 * d;
		return t >= 4 ? ~0u : (t <= 0 ? 0u : (1u << (8 * t)) - 1u);
	};
	u32x4 v;
	v.x = (a.x & m(0)) | (b.x & ~m(0));
	v.y = (a.y & m(1)) | (b.y & ~m(1));
	v.z = (a.z & m(2)) | (b.z & ~m(2));
	v.w = (a.w & m(3)) | (b.w & ~m(3));
	return v;
}

// Store step of a period-off pattern match (make_pattern16's stp).
__device__ __forceinline__ int32_t pattern_step(int32_t off)
{
	return off <= 8 ? int32_t((PAT_LUT >> (5 * (off - 1))) & 31u) : off;
}

// v_perm_b32 selectors of the period-off patterns, off = 1..15 (entry off,
// dword d; entry 0 unused): byte t of output dword d is source byte
// (4d + t) mod off, taken from v.y:v.x (off <= 8, and dwords 0-1 -- v.x and
// v.y themselves -- of every off), v.z:v.x (dword 2, off >= 9) or
// v.w:v.x / v.y:v.x (dword 3, off >= 12 / 9..11): pattern_perm.  Written
// once per block by its wave (lane l: entry l / 4, dword l % 4).
__device__ __forceinline__ void pattern_lut_init(uint32_t* plut)
{
	const uint32_t l = lane_id(), off = l >> 2, d = l & 3u;
	uint32_t sel = 0;
	if (off > 0)
		for (uint32_t t = 0; t < 4; ++t) {
			const uint32_t idx = (4 * d + t) % off;
			uint32_t x = idx;
			if (off > 8 && d == 2 && idx >= 8)
				x = idx - 4;  // v.z byte idx - 8 (v_perm's src0 bytes are 4..7)
			if (off >= 12 && d == 3 && idx >= 12)
				x = idx - 8;  // v.w byte idx - 12
			sel |= x << (8 * t);
		}
	plut[l] = sel;
}

// The phase-0 period-off (1..15) pattern of the 16 source bytes v (the
// first off of them valid): make_pattern16's value in one LDS read, two
// selects and four v_perm_b32 instead of its 64-bit shift network.
__device__ __forceinline__ u32x4 pattern_perm(u32x4 v, int32_t off, const uint32_t* plut)
{
	const u32x4 sel = *reinterpret_cast<const u32x4*>(plut + 4 * off);
	const uint32_t h2 = off <= 8 ? v.y : v.z, h3 = off <= 11 ? v.y : v.w;
	u32x4 o;
	o.x = __builtin_amdgcn_perm(v.y, v.x, sel.x);
	o.y = __builtin_amdgcn_perm(v.y, v.x, sel.y);
	o.z = __builtin_amdgcn_perm(h2, v.x, sel.z);
	o.w = __builtin_amdgcn_perm(h3, v.x, sel.w);
	return o;
}

// Match with a final source entirely inside the ring (Output_With_History,
// lz4ada.adb:845-904).  Match byte i is source byte i mod off (the overlap
// rule), so no unit reads this match's own output: an off < 16 overlap
// stores a 16-byte period pattern every stp bytes, any other match 16
// source bytes per unit (a unit that wraps the period merges two reads).
// One loop for both forms: a wave runs max(units) over its lanes, not the
// two loops one after the other.
template <class LD>
__device__ __forceinline__ void ring_match(LD& L, int32_t dst, int32_t off, int32_t len)
{
	const int32_t src = dst - off;
	u32x4 pv = oload16(L, src);
	int32_t stp = 16;
	const bool pat = off < 16 && off < len;
	if (pat) {
		if constexpr (lds_fast<LD>::value) {
			pv = pattern_perm(pv, off, plut_of(L));
			stp = pattern_step(off);
		} else {
			make_pattern16(uint64_t(pv.x) | (uint64_t(pv.y) << 32), uint64_t(pv.z) | (uint64_t(pv.w) << 32),
			               off, pv, stp);
		}
	}
	ostore(L, dst, pv, min(16, len));
	int32_t start = 0;  // unit x of the wide form begins at source byte x mod off
	for (int32_t x = stp; x < len; x += stp) {
		u32x4 v = pv;
		if (!pat) {
			start += 16;
			if (start >= off)
				start -= off;
			v = oload16(L, src + start);
			if (off - start < 16)
				v = merge_at(v, oload16(L, src + start - off), off - start);
		}
		ostore(L, dst + x, v, min(16, len - x));
	}
}

// q = t / d and r = t mod d for 0 <= t < 2^22, 1 <= d < 2^16: float
// reciprocal (error < 1 in q) and one correction step.
__device__ __forceinline__ int32_t div_small(int32_t t, int32_t d, int32_t& r)
{
	int32_t q = int32_t(float(t) * __builtin_amdgcn_rcpf(float(d)));
	r = t - q * d;
	if (r < 0) {
		--q;
		r += d;
	}
	if (r >= d) {
		++q;
		r -= d;
	}
	return q;
}


__device__ __forceinline__ int32_t piece_owner(int32_t inc, int32_t t);

// Owner lane of piece t0 + lane, lane i holding pieces [inc_i - np_i,
// inc_i) (inc: inclusive prefix sum, monotone): each lane marks its first
// piece's slot of the 64-piece chunk in LDS, a prefix maximum fills the
// slots in between, and the chunk's first slot is seeded with the owner of
// piece t0 (the lanes with inc <= t0, counted from a ballot).  Two LDS
// round trips instead of six dependent shuffles of a binary search.
template <class LD>
__device__ __forceinline__ int32_t chunk_owner(LD& D, int32_t inc, int32_t np, int32_t t0)
{
	const int32_t lane = int32_t(lane_id());
	const int32_t seed = __popcll(__ballot(inc <= t0));
	uint8_t* own = own_of(D);
	own[lane] = uint8_t(lane == 0 ? seed : 0);
	const int32_t excl = inc - np;
	if (np > 0 && excl >= t0 && excl < t0 + 64)
		own[excl - t0] = uint8_t(lane);
	wave_lds_fence();
	const int32_t v = own[lane];
	wave_lds_fence();  // own[] is marked again for the next chunk
	return wave_incl_max(v);
}

// chunk_owner over two rounds' entries (round 0's lanes, then round 1's:
// entry 64 r + lane holds pieces [inc_r - np_r, inc_r)), owner 0..127.
template <class LD>
__device__ __forceinline__ int32_t chunk_owner2(LD& D, int32_t inc0, int32_t np0, int32_t inc1,
                                                int32_t np1, int32_t t0)
{
	const int32_t lane = int32_t(lane_id());
	const int32_t seed = __popcll(__ballot(inc0 <= t0)) + __popcll(__ballot(inc1 <= t0));
	uint8_t* own = own_of(D);
	own[lane] = uint8_t(lane == 0 ? seed : 0);
	const int32_t e0 = inc0 - np0, e1 = inc1 - np1;
	if (np0 > 0 && e0 >= t0 && e0 < t0 + 64)
		own[e0 - t0] = uint8_t(lane);
	if (np1 > 0 && e1 >= t0 && e1 < t0 + 64)
		own[e1 - t0] = uint8_t(64 + lane);
	wave_lds_fence();
	const int32_t v = own[lane];
	wave_lds_fence();  // own[] is marked again for the next chunk
	return wave_incl_max(v);
}

// Every lane's match (dst, off, ml; ml = 0: none) with a source in the LDS
// ring, cut into pieces dealt over the wave: 16 output bytes each, or stp
// bytes of a period-off pattern (off < 16 < ml would overlap: match byte i
// is source byte i mod off, so a piece never reads its own match's output).
// Pieces are in output order; one reading output of a lower lane of its
// chunk waits until that lane has stored (ballot per step).
// Pieces of one match: 16-byte pieces, or stp-byte steps of a period-off
// pattern (off < 16 < ml overlaps).
__device__ __forceinline__ int32_t match_pieces(int32_t off, int32_t ml)
{
	if (ml <= 0)
		return 0;
	if (!(off < 16 && off < ml))
		return (ml + 15) >> 4;
	const int32_t stp = pattern_step(off);
	int32_t rr;
	return stp == 16 ? (ml + 15) >> 4 : div_small(ml + stp - 1, stp, rr);
}

#ifndef LZ4ADA_FWD_ROUNDS
#define LZ4ADA_FWD_ROUNDS 5
#endif
constexpr int FWD_ROUNDS = LZ4ADA_FWD_ROUNDS;  // forwarding rounds of ring_lanes (0: none)
// ... and of ring_pieces: off (mixed 13.17 -> 13.41 ms with it, dense
// 37.07 -> 37.38: its dealt pieces rarely sit inside one producer piece,
// and the set-up runs for every 64-piece chunk; profiles/r06i_ab.txt)
#ifndef LZ4ADA_FWD_PIECES
#define LZ4ADA_FWD_PIECES 0
#endif
constexpr int FWD_PIECES = LZ4ADA_FWD_PIECES;

// Both rounds' ring-sourced matches (round r: mdst[r], off[r], ml[r]; ml 0:
// none), dealt together in output order; a piece finds its match in an LDS
// descriptor (D.ldesc, free after the literals) instead of by shuffles.
template <class LD>
__device__ __forceinline__ int32_t ring_pieces(LD& D, const int32_t (&mdst)[RMAX],
                                               const int32_t (&off)[RMAX], const int32_t (&ml)[RMAX],
                                               int32_t o_batch, int32_t glo = INT32_MIN)
{
	int32_t steps = 0;  // store steps (diagnostic count)
	const int32_t lane = int32_t(lane_id());
	const int32_t np0 = match_pieces(off[0], ml[0]), np1 = match_pieces(off[1], ml[1]);
	const int32_t inc0 = wave_incl_scan(np0);
	const int32_t tot0 = __shfl(inc0, 63);
	const int32_t inc1 = tot0 + wave_incl_scan(np1);
	const int32_t tot = __shfl(inc1, 63);
	auto pack = [&](int32_t md, int32_t of, int32_t m, int32_t excl) -> uint64_t {
		return uint64_t(uint16_t(md - o_batch)) | (uint64_t(uint16_t(of)) << 16) |
		       (uint64_t(uint16_t(m)) << 32) | (uint64_t(uint16_t(excl)) << 48);
	};
	uint64_t* ldesc = ldesc_of(D);
	ldesc[lane] = pack(mdst[0], off[0], ml[0], inc0 - np0);
	ldesc[64 + lane] = pack(mdst[1], off[1], ml[1], inc1 - np1);
	for (int32_t t0 = 0; t0 < tot; t0 += 64) {
		const int32_t t = t0 + lane;
		const bool act = t < tot;
		const int32_t lo = min(chunk_owner2(D, inc0, np0, inc1, np1, t0), 127);
		const uint64_t dd = ldesc[lo];
		const int32_t od = o_batch + int32_t(dd & 0xffffu);
		const int32_t ooff = int32_t((dd >> 16) & 0xffffu), oml = int32_t((dd >> 32) & 0xffffu);
		const int32_t k = t - int32_t(dd >> 48);
		const bool opat = ooff < 16 && ooff < oml;
		const int32_t ostp = opat ? pattern_step(ooff) : 16;
		const bool wide = !opat && oml > ooff;  // overlap with off >= 16
		const int32_t pd = od + k * ostp;
		const int32_t pn = min(16, oml - k * ostp);
		// source bytes read: the whole period for patterns and overlaps
		const int32_t s_lo = (opat || wide) ? od - ooff : od - ooff + 16 * k;
		const int32_t s_hi = (opat || wide) ? od : s_lo + pn;
		// lanes of this chunk whose piece [pd, pd + pn) meets [s_lo, s_hi):
		// pd is monotone over the lanes, so two binary searches -- skipped
		// when every source ends before the chunk's first piece
		// a piece writes [pd, pd + pn): its end, not pd + 16 (a short last piece
		// must not hold back a source that only starts after it)
		const int32_t pe = act ? pd + pn : INT32_MAX, ps = act ? pd : INT32_MAX;
		int32_t fj1 = 64, fj2 = -1;  // the chunk's pieces that write this one's source (none)
		if (!__all(!act || s_hi <= __shfl(ps, 0))) {
			int32_t j1 = 0, c2 = 0;
#pragma unroll
			for (int st = 32; st >= 1; st >>= 1) {
				if (__shfl(pe, j1 + st - 1) <= s_lo)
					j1 += st;
				if (__shfl(ps, c2 + st - 1) < s_hi)
					c2 += st;
			}
			fj1 = j1;
			fj2 = min(c2 - 1, lane - 1);
		}
		// Forwarding (ring_lanes' pointer jumping, per piece): a piece whose
		// source [s_lo, s_hi) lies inside ONE earlier piece P of the chunk, P
		// a plain copy (out[y] = out[y - sh_P] over its bytes, sh_P = its
		// offset plus its own forwarding), reads F bytes further back
		// instead and waits for P's producers; every read form shifts as a
		// whole (a pattern's period, an overlap's two reads)
		int32_t F = 0;
		if (FWD_PIECES > 0 && glo != INT32_MIN) {
			const bool plain = act && !opat && !wide;
			int32_t sh = ooff;
			const int32_t q0 = __shfl(ps, fj1), qe = __shfl(pe, fj1);
			bool fw = act && fj1 == fj2 && q0 <= s_lo && s_hi <= qe && __shfl(int32_t(plain), fj1) != 0;
			for (int r = 0; r < FWD_PIECES && __any(fw); ++r) {
				const int32_t p = fj1;
				const int32_t qs = __shfl(sh, p), q1 = __shfl(fj1, p), q2 = __shfl(fj2, p);
				const bool qf = __shfl(int32_t(fw), p) != 0;
				if (fw && s_lo - F - qs >= glo) {
					F += qs;
					sh = ooff + F;
					fj1 = q1;  // P's producers (none: q1 > q2, the source is final)
					fj2 = q2;
					fw = qf;
				} else {
					fw = false;
				}
			}
		}
		uint64_t dep = 0;
		if (act && fj1 <= fj2)
			dep = (fj2 == 63 ? ~uint64_t(0) : ((uint64_t(2) << fj2) - 1)) & ~((uint64_t(1) << fj1) - 1);
		// the piece's reads, fixed before the steps: 16 bytes at a1 and, for
		// an overlap with off >= 16 whose unit wraps the period, the bytes
		// from cut on at a1 - off (one load for every form: divergent
		// per-form loads made a step run up to three of them in turn)
		int32_t rem = 0;
		if (wide)
			div_small(16 * k, ooff, rem);
		const int32_t a1 = (opat ? od - ooff : (wide ? od - ooff + rem : s_lo)) - F;
		const int32_t cut = (wide && ooff - rem < 16) ? ooff - rem : 16;
		bool pend = act;
		for (;;) {
			const uint64_t pm = __ballot(pend);
			if (pm == 0)
				break;
			const bool ready = pend && (dep & pm) == 0;
			if constexpr (lds_fast<LD>::value) {
				// every lane loads and stores (a lane not ready stores
				// nothing: n = 0 sends its stores to the junk bytes)
				u32x4 v = oload16(D, a1);
				if (ready && cut < 16)
					v = merge_at(v, oload16(D, a1 - ooff), cut);
				if (ready && opat)
					v = pattern_perm(v, ooff, plut_of(D));
				ostore(D, pd, v, ready ? pn : 0);
			} else if (ready) {
				u32x4 v = oload16(D, a1);
				if (cut < 16)
					v = merge_at(v, oload16(D, a1 - ooff), cut);
				if (opat) {
					int32_t sstp;
					make_pattern16(uint64_t(v.x) | (uint64_t(v.y) << 32),
					               uint64_t(v.z) | (uint64_t(v.w) << 32), ooff, v, sstp);
				}
				ostore(D, pd, v, pn);
			}
			pend = pend && !ready;
			wave_lds_fence();
			++steps;
		}
	}
	return steps;
}

// Ring-sourced matches of a round of short matches, one lane each: those
// whose source is final before the round (or lies in their own literals)
// at once, a near match -- reading this round's match output -- once every
// lane whose output it reads is done (a 64-bit mask from two binary
// searches over the round's monotone match positions, one AND against a
// ballot per step).  rbeg: the round's first output position; L: this
// lane's literal length.
#ifndef LZ4ADA_RING_LANE_MAX
#define LZ4ADA_RING_LANE_MAX 32
#endif
constexpr int RING_LANE_MAX = LZ4ADA_RING_LANE_MAX;
template <class LD>
__device__ __forceinline__ int32_t ring_lanes(LD& D, int32_t mdst, int32_t off, int32_t ml,
                                           int32_t rbeg, int32_t L, int32_t glo = INT32_MIN)
{
	const int32_t lane = int32_t(lane_id());
	const int32_t src = mdst - off;
	const int32_t dep_end = src + min(off, ml);
	const bool far = ml > 0 && (dep_end <= rbeg || off <= L);
	int32_t steps = 0;  // store steps (diagnostic count)
	if (!__any(ml > 0 && !far)) {
		if (far)
			ring_match(D, mdst, off, ml);
		wave_lds_fence();
		return 0;
	}
	// with near matches, the far ones run in the first step with the near
	// ones that are ready (their sources are final: no producers), not in
	// a step of their own
	bool near = ml > 0;
	const int32_t mend = mdst + ml;
	int32_t j1 = 0, c2 = 0;
#pragma unroll
	for (int st = 32; st >= 1; st >>= 1) {
		if (__shfl(mend, j1 + st - 1) <= src)
			j1 += st;
		if (__shfl(mdst, c2 + st - 1) < dep_end)
			c2 += st;
	}
	int32_t fj1 = far ? 64 : j1, fj2 = far ? -1 : min(c2 - 1, lane - 1);
	// Forwarding (pointer jumping over the round's near matches): a plain
	// match (off >= ml) whose source lies inside ONE earlier near match P of
	// the round, P itself a plain copy, reads P's source instead -- byte x of
	// it is byte x - off - off_P -- and waits for P's producers instead of
	// for P.  Each round composes every lane's forwarding with its producer's
	// current one, so a chain of k dependent matches (text: matches copying
	// recent matches, ~17 in a row) takes ~log2 k rounds instead of k store
	// steps.  A source forwarded past glo (below the window's kept bytes)
	// stops there.
	int32_t fo = off;
	{
		const int32_t pm = __shfl(mdst, fj1), pe = __shfl(mend, fj1), po = __shfl(off, fj1);
		const bool pn = __shfl(int32_t(near), fj1) != 0;
		bool fw = FWD_ROUNDS > 0 && glo != INT32_MIN && near && off >= ml && fj1 == fj2 && pm <= src &&
		          dep_end <= pe && pn && po >= pe - pm;
		// (the producer's state is read before any lane updates its own:
		// synchronous rounds; P's identity out[y] = out[y - fo_P] holds for
		// whatever forwarding P has reached)
		for (int r = 0; r < FWD_ROUNDS && __any(fw); ++r) {
			const int32_t p = fj1;
			const int32_t qo = __shfl(fo, p), q1 = __shfl(fj1, p), q2 = __shfl(fj2, p);
			const bool qf = __shfl(int32_t(fw), p) != 0;
			if (fw && mdst - fo - qo >= glo) {
				fo += qo;
				fj1 = q1;  // P's producers (none: q1 > q2, the source is final)
				fj2 = q2;
				fw = qf;
			} else {
				fw = false;
			}
		}
	}
	uint64_t dep = 0;
	if (near && fj1 <= fj2)
		dep = (fj2 == 63 ? ~uint64_t(0) : ((uint64_t(2) << fj2) - 1)) & ~((uint64_t(1) << fj1) - 1);
	for (;;) {
		const uint64_t pending = __ballot(near);
		if (pending == 0)
			break;
		const bool ready = near && (dep & pending) == 0;
		if (ready) {
			ring_match(D, mdst, fo, ml);
			near = false;
		}
		wave_lds_fence();
		++steps;
	}
	return steps;
}

// Owner of piece t when lane i holds pieces [inc_i - cnt_i, inc_i) (inc: the
// wave's inclusive prefix sum of piece counts): the first lane with inc > t.
__device__ __forceinline__ int32_t piece_owner(int32_t inc, int32_t t)
{
	int32_t lo = 0;
#pragma unroll
	for (int st = 32; st >= 1; st >>= 1)
		if (__shfl(inc, lo + st - 1) <= t)
			lo += st;
	return lo;
}

// 2 KiB input chunk c (aligned address abase + c*BATCH), 32 bytes per lane
__device__ __forceinline__ void load_chunk2(uintptr_t abase, int32_t c, uintptr_t lim, u32x4& v0,
                                            u32x4& v1)
{
	const uintptr_t g = abase + uintptr_t(c) * BATCH + 16u * lane_id();
	if (abase + uintptr_t(c + 1) * BATCH <= lim) {
		__builtin_memcpy(&v0, reinterpret_cast<cg8*>(g), 16);
		__builtin_memcpy(&v1, reinterpret_cast<cg8*>(g + 1024), 16);
	} else {
		v0 = gload16(g, lim);
		v1 = gload16(g + 1024, lim);
	}
}

// Quirk D1 under the host's predicted round state (BLOCK_D1_ROUND: the
// last round ended at OPH in [65536, 65542] and this block starts at round
// position n1).  A match reading before the round start within 7 bytes of
// where that round ended (OPH - off < 8) reads what the reference's last
// wild copy (lib/lz4ada.adb:811-817) left past its frontier, not history:
// * after literals (L > 0): the payload bytes after them -- emulated when
//   their last chunk was wild (8 payload bytes left, k_lone_words' rule);
// * with no literals: the previous match's last Write_Output call
//   (:845-904), i.e. the output bytes right after that match's source --
//   emulated when the match was one call (no repeating part; from history,
//   no intermediate part either) whose tail read only final bytes (in the
//   round: its source ends pad bytes before its output; from history: the
//   tail stays in the previous round, and that match is no D1 read
//   itself).  `lit` then carries that position (block-relative, + D1_QBIAS,
//   << 3) and the overshoot length pad (low 3 bits) for M.
// Either way the match must read nothing of the current round.  false: a
// D1 read it does not emulate (the block is declined).  The rule was
// checked against the oracle's output over 256-block linked frames of the
// generator's uniform-offset kinds (tools/d1_model.py).
constexpr int32_t D1_QBIAS = 1 << 17;
__device__ __forceinline__ bool d1_emulable(int32_t mdst, int32_t L, int32_t& lit, int32_t off, int32_t ml,
                                            int32_t pmd, int32_t pof, int32_t pml, int32_t n1, int32_t oph,
                                            int32_t n)
{
	if (!(n1 + mdst < off && oph - off < 8))
		return true;  // no D1 read
	if (n1 + mdst + ml > off)
		return false;  // it also reads the current round
	if (L > 0)
		return lit + 8 * ((L - 1) >> 3) + 8 <= n;
	if (n1 + mdst == 0) {  // the round's first output: nothing written past its frontier yet,
		lit = D1_QBIAS << 3;  // the read is the previous round's bytes -- plain history (pad 0)
		return true;
	}
	if (pml <= 0)
		return false;  // the previous match is not known here
	const int32_t f = n1 + pmd, raw = f - pof, pad = (8 - (pml & 7)) & 7;
	bool ok = raw >= 0 ? pml <= pof && pof - pml >= pad
	                   : pof - f >= pml && oph - pof >= 8 && raw + pml + pad <= 0;
	const int32_t q = pmd - pof + pml;  // the previous match's source end
	if (ok)
		lit = ((q + D1_QBIAS) << 3) | pad;
	return ok;
}

// One block.  hist: output bytes right before this block's slot that its
// matches may read -- 0 for independent blocks; in a linked frame, the
// earlier blocks' output, contiguous when every one of them is full.
// Returns the block's status code; out_len gets its output length.
//
// ZL (the linked path's second plane, k_decode_idx_zl; a constant at each
// inlined call site, so the other decoders' code has none of it): every literal byte
// is written as 0, so an output byte is nonzero only where it came from
// the synthetic history (whose bytes there hold the history position's
// high byte); a match reading history positions below 256 (more than
// 65,280 bytes before the block: their high byte is 0 too) sets
// AUX_DEEP_HIST; a stored block is all zeros; an oversized batch (literals
// straight to HBM) declines the block, which then takes the three-plane
// decode (lz4ada_bulk_linked.cpp).
__device__ __forceinline__ int32_t decode_block(DecLds& D, const uint8_t* __restrict__ frame,
                                                uint64_t frame_len,
                                                const lz4ada_block_desc* __restrict__ desc,
                                                uint32_t b, const uint8_t* __restrict__ tab_all,
                                                uint8_t* __restrict__ out,
                                                lz4ada_block_status* __restrict__ status,
                                                int64_t hist, int32_t& out_len, const bool ZL = false,
                                                const bool D1E = false)
{
	const int32_t lane = int32_t(lane_id());
	const lz4ada_block_desc d = desc[b];
	out_len = 0;
	if (status[b].code != DS_OK)
		return DS_RETRY;  // pass 1 declined it
	cg8* in = gptr(frame) + d.in_off;
	g8* ob = gptr(out) + d.out_off;
	const int32_t n = int32_t(d.in_len);
	const int32_t cap = int32_t(d.out_cap);
	const uintptr_t lim = reinterpret_cast<uintptr_t>(frame) + frame_len;
	const uintptr_t olim = reinterpret_cast<uintptr_t>(ob) + uintptr_t(cap);

	if (d.flags & LZ4ADA_BLOCK_STORED) {
		int32_t code = DS_OK;
		if (n > cap) {
			code = DS_OUT_OVERFLOW;
		} else if (ZL) {  // every byte a literal: zeros
			for (int32_t x = 16 * lane; x < n; x += 64 * 16)
				gstore_n(ob + x, u32x4{ 0u, 0u, 0u, 0u }, min(16, n - x));
		} else {
			Src S0;
			S0.in = in;
			S0.lim = lim;
			// nontemporal copy unless the block checksum kernel beside this
			// one reads the same payload (it then finds it in the caches)
			if (d.flags & LZ4ADA_BLOCK_HAS_CKSUM)
				wave_literal<0>(ob, 0, S0, 0, n);
			else
				wave_literal<LZ4ADA_STORED_NT>(ob, 0, S0, 0, n);
		}
		if (lane == 0) {
			status[b].code = code;
			status[b].aux = 0;
			status[b].detail = 0;
			status[b].err_out_pos = 0;
			status[b].out_len = code == DS_OK ? uint32_t(n) : 0u;
		}
		out_len = code == DS_OK ? n : 0;
		return code;
	}

	const int32_t mis = int32_t(reinterpret_cast<uintptr_t>(in) & 15u);
	const int32_t hb = int32_t(min(hist, int64_t(65535)));  // reachable history
	pattern_lut_init(D.plut);  // (LDS shared with pass 1: written per block)
	if (hb > 0) {
		// the ring's history: the previous block's last bytes
		for (int32_t x = (-min(hb + 16, ORING - 16)) & ~15; x < 0; x += 64 * 16)
			if (x + 16 * lane < 0)
				*reinterpret_cast<u32x4*>(&D.oring[uint32_t(x + 16 * lane) & OMASK]) =
				    gload16(reinterpret_cast<uintptr_t>(ob) + uintptr_t(intptr_t(x + 16 * lane)), olim);
		__builtin_amdgcn_s_waitcnt(0x0F70);  // settled before the batch loop (see fetch4)
		wave_lds_fence();
	}
	const uint64_t* tab = reinterpret_cast<const uint64_t*>(tab_all) + (((d.in_off >> 8) + b) << 3);
	const int32_t nsub = (n + SUB - 1) / SUB;
	const uintptr_t abase = reinterpret_cast<uintptr_t>(in) - uintptr_t(mis);

	Src S;
	S.lds = D.ring;
	S.mask = RING - 1;
	S.mis = mis;
	S.in = in;
	S.lim = lim;

	// input chunks staged: [hi - 4, hi) are in the ring, and the records of
	// sub-segments [64 (hi - 4), 64 hi) in rrec (loaded with the input: a
	// record load of its own per batch would wait on the previous flush)
	int32_t hi = 0;
	u32x4 pf0, pf1;  // chunk hi, loaded ahead
	load_chunk2(abase, 0, lim, pf0, pf1);
	auto load_rec = [&](int32_t c) -> uint64_t {
		const int32_t k = 64 * c + lane;
		return k < nsub ? __builtin_nontemporal_load(tab + k) : 0;
	};
	uint64_t pr = load_rec(0);
	// settled before the loop: left pending, the loop head's merge would
	// make every batch's staging wait vmcnt(0) (flush stores included)
	vm_wait();

	ISTAMP_DECL;
	int32_t o_batch = 0;  // output position of the current batch
	bool bad = false;
	bool d1 = false;  // a match with offset >= D1_OFF reads before the block start
	// the host's prediction of the round state (linked bulk path): quirk D1
	// emulated under it (d1x: a D1 match it cannot emulate declines the
	// block; the status says AUX_D1_EMU: decoded under the prediction)
	const bool d1p = D1E && (d.flags & BLOCK_D1_ROUND) != 0;  // (D1E: the linked planes' kernels)
	const int32_t oph = int32_t(HISTORY_SIZE) + int32_t((d.flags >> BLOCK_D1_OPH_SHIFT) & 7u);
	const int32_t n1 = int32_t(d.flags >> BLOCK_N1_SHIFT);
	bool d1x = false;
	// the previous batch's last match (block-relative output start, offset,
	// length; pml = 0: none known) for a D1 match without literals in lane 0
	int32_t pmd_b = 0, pof_b = 0, pml_b = 0;
	bool deep = false;  // ZL: a match reads history positions below 256
	int32_t hcnt = 0;   // ZL: match bytes read straight from the history region
	for (int32_t k0 = 0; k0 < nsub && !bad;) {
		// stage input so that [k0*SUB, k0*SUB + 4 KiB) is readable
		const int32_t cf = (k0 * SUB + mis) / BATCH;
		bool staged = false;
		if (hi < cf + 3) {
			staged = true;
			auto stage_one = [&]() {
				const uint32_t a = uint32_t(hi * BATCH) & (RING - 1);
				*reinterpret_cast<u32x4*>(&D.ring[a + 16 * lane]) = pf0;
				*reinterpret_cast<u32x4*>(&D.ring[a + 1024 + 16 * lane]) = pf1;
				if (a == 0 && lane == 0)
					*reinterpret_cast<u32x4*>(&D.ring[RING]) = pf0;
				D.rrec[64 * (hi & 3) + lane] = pr;
				++hi;
				load_chunk2(abase, hi, lim, pf0, pf1);
				pr = load_rec(hi);
			};
			// the first chunk outside the loop: its prefetch is settled (M's
			// wait), and inside a loop the wait pass would put a vmcnt(0) --
			// the previous batch's flush stores included -- before it too
			stage_one();
			while (hi < cf + 3)  // the block's first batch (and rarely later)
				stage_one();
			wave_lds_fence();
		}
		S.lo = max(hi - 4, 0) * BATCH - mis;
		S.hi = hi * BATCH - mis;

		ISTAMP(D_STAGE);
		ICOUNT(D_BATCHES, 1);
		const int32_t k = k0 + lane;  // this lane's sub-segment
		const int32_t sub_s = k * SUB;
		const int32_t sub_end = min(sub_s + SUB, n);
		// this lane's sequence starts and output bytes, from pass 1's record
		const uint64_t rec = (k < nsub) ? D.rrec[k & 255] : 0;
		uint32_t bm = uint32_t(rec);
		const int32_t cnt = int32_t(min(uint32_t(rec >> 32), 1u << 24));  // > cap: rejected below
		const int32_t nseq = __popc(bm);
		const int32_t p0 = bm ? sub_s + __builtin_ctz(bm) : n;
		const int32_t incl = wave_incl_scan(cnt);
		const int32_t incl_s = wave_incl_scan(nseq);
		const int32_t o_lane = o_batch + incl - cnt;
		const bool fit = incl <= LZ4ADA_OW_CUT && incl_s <= LZ4ADA_SEQ_CUT;
		const int32_t m = __popcll(__ballot(fit));  // lanes [0, m) form an LDS batch
		ISTAMP(D_WALK1);

		if (m == 0) {
			if (ZL) {  // (literals straight to HBM: the three-plane decode takes the block)
				bad = true;
				break;
			}
			// oversized: all 64 sub-segments straight to HBM
			const int32_t total = __shfl(incl, 63);
			if (o_batch + total > cap) {
				bad = true;
				break;
			}
			const int32_t a0 = o_batch & ~15;
			if (lane == 0 && o_batch > a0)  // the ring's unflushed tail
				gstore_n(ob + a0, *reinterpret_cast<const u32x4*>(&D.oring[a0 & OMASK]), o_batch - a0);
			vm_wait();
			if (!batch_global(S, ob, olim, p0, sub_end, n, o_lane, o_batch, hb)) {
				bad = true;
				break;
			}
			o_batch += total;
			pml_b = 0;  // (its sequences are not tracked for quirk D1)
			vm_wait();
			ICOUNT(D_GBATCHES, 1);
			// reload the ring's history from HBM
			const int32_t x0 = max(o_batch - ORING + 16, -((hb + 15) & ~15)) & ~15;
			for (int32_t x = x0 + 16 * lane; x < o_batch + 15; x += 64 * 16)
				*reinterpret_cast<u32x4*>(&D.oring[uint32_t(x) & OMASK]) =
				    gload16(reinterpret_cast<uintptr_t>(ob) + uintptr_t(intptr_t(x)), olim);
			wave_lds_fence();
			ISTAMP(D_GLOBAL);
			k0 += 64;
			continue;
		}

		const int32_t o_end = o_batch + __shfl(incl, m - 1);
		if (o_end > cap) {
			bad = true;
			break;
		}
		// the batch's sequence starts, in output order
		const int32_t base = k0 * SUB;
		if (lane < m) {
			int32_t e = incl_s - nseq;
			const uint16_t rel = uint16_t(sub_s - base);
			for (; bm; bm &= bm - 1)
				D.cst[e++] = uint16_t(rel + __builtin_ctz(bm));
		}
		wave_lds_fence();
		const int32_t N = __shfl(incl_s, m - 1);
		// HBM holds every byte below align_down(o_batch, 16) (earlier
		// flushes); a match reading below glo reads HBM (its source ends
		// before o_batch - 16), anything newer is in the ring
		const int32_t glo = o_batch - OW - 16;

		// P: parse 64 sequences per round, place them by a prefix sum
		int32_t rL[RMAX], rlit[RMAX], roff[RMAX], rml[RMAX], rdst[RMAX], rbeg[RMAX];
		bool pre = false, anyg = false;
		{
			int32_t o_round = o_batch;
			// both rounds' sequences parsed first (their starts are known, so
			// the four dependent LDS reads of the two rounds overlap), the
			// rare shapes the branch-free form rejects after, then placement
			// (mixed / dense / text -0.5..-0.9% against one round at a time,
			// profiles/r06u_psplit_ab.txt; 189 VGPRs)
			bool fok[RMAX];
#pragma unroll
			for (int r = 0; r < RMAX; ++r) {
				rL[r] = rlit[r] = roff[r] = rml[r] = 0;
				fok[r] = true;
				const int32_t idx = 64 * r + lane;
				if (idx < N) {
					Seq q;
					fok[r] = parse_fast_try(S, base + int32_t(D.cst[idx]), n, q);
					rL[r] = q.L;
					rlit[r] = q.lit;
					roff[r] = q.off;
					rml[r] = q.ml;
				}
			}
#pragma unroll
			for (int r = 0; r < RMAX; ++r) {
				if (__builtin_expect(__any(!fok[r]), 0)) {
					if (!fok[r]) {
						Seq q;
						parse_seq(S, base + int32_t(D.cst[64 * r + lane]), n, q);
						rL[r] = q.L;
						rlit[r] = q.lit;
						roff[r] = q.off;
						rml[r] = q.ml;
					}
				}
			}
#pragma unroll
			for (int r = 0; r < RMAX; ++r) {
				rbeg[r] = o_round;
				if (64 * r < N) {
					const int32_t len = rL[r] + rml[r];
					const int32_t inc = wave_incl_scan(len);
					rdst[r] = o_round + inc - len;  // literal destination
					o_round += __shfl(inc, 63);
					const int32_t mdst = rdst[r] + rL[r];
					if (d1p) {
						// the previous sequence's match: lane - 1, lane 0 the
						// previous round's lane 63 or the previous batch's last
						int32_t pmd = __shfl(mdst, (lane + 63) & 63), pof = __shfl(roff[r], (lane + 63) & 63),
						        pml = __shfl(rml[r], (lane + 63) & 63);
						if (r > 0) {
							const int32_t a = __shfl(rdst[0] + rL[0], 63), b = __shfl(roff[0], 63),
							              c = __shfl(rml[0], 63);
							if (lane == 0) {
								pmd = a;
								pof = b;
								pml = c;
							}
						} else if (lane == 0) {
							pmd = pmd_b;
							pof = pof_b;
							pml = pml_b;
						}
						if (rml[r] > 0 && !d1_emulable(mdst, rL[r], rlit[r], roff[r], rml[r], pmd, pof, pml, n1,
						                               oph, n))
							d1x = true;
					}
					if (rml[r] > 0) {
						if (roff[r] > mdst + hb)
							pre = true;  // reference before the block start (D2) / history
						if (roff[r] > mdst && roff[r] >= D1_OFF)
							d1 = true;
						if (ZL && roff[r] > mdst + 65280)
							deep = true;
						if (ZL && roff[r] > mdst)
							hcnt += min(rml[r], roff[r] - mdst);
						if (mdst - roff[r] < glo)
							anyg = true;
					}
				}
			}
		}
		if (__any(pre || d1x)) {
			bad = true;
			break;
		}
		if (d1p) {  // the batch's last sequence, for the next batch's lane 0
			const int32_t l = (N - 1) & 63;
			const bool r1 = N > 64;
			pmd_b = __shfl(r1 ? rdst[1] + rL[1] : rdst[0] + rL[0], l);
			pof_b = __shfl(r1 ? roff[1] : roff[0], l);
			pml_b = __shfl(r1 ? rml[1] : rml[0], l);
		}
		ISTAMP(D_WALK2);

		// HBM-sourced matches: every load in flight before the first use.  A
		// match's first GC pieces load in its own lane; the pieces beyond
		// (long matches) of both rounds are dealt over the wave, one per
		// lane, through the LDS match descriptors (more than 64: the rest
		// load in M, rare).
		u32x4 vg[RMAX][GC], vr = u32x4{0u, 0u, 0u, 0u};
		int32_t rtot[RMAX], rfirst[RMAX];  // pieces beyond GC per round; the first not dealt here
		int32_t rpd = 0, rpn = 0;          // this lane's dealt piece
#pragma unroll
		for (int r = 0; r < RMAX; ++r)
			rtot[r] = rfirst[r] = 0;
		if (__any(anyg)) {
			// the previous batch's flush (FLUSH_ST store instructions) and
			// the input and record prefetch (3 loads, when this batch
			// staged) may stay in flight; everything older -- earlier
			// flushes -- is complete
			if (staged)
				asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FLUSH_ST + 3) : "memory");
			else
				asm volatile("s_waitcnt vmcnt(%0)" ::"n"(FLUSH_ST) : "memory");
			int32_t nc[RMAX];
#pragma unroll
			for (int r = 0; r < RMAX; ++r) {
				nc[r] = 0;
				if (64 * r < N) {
					const int32_t src = rdst[r] + rL[r] - roff[r];
					const bool g = rml[r] > 0 && src < glo;
#pragma unroll
					for (int c = 0; c < GC; ++c)
						if (g && 16 * c < rml[r])
							__builtin_memcpy(&vg[r][c], ob + src + 16 * c, 16);
					nc[r] = g ? max(((rml[r] + 15) >> 4) - GC, 0) : 0;
					GCOUNT(0, __popcll(__ballot(g)));
					GCOUNT(1, __popcll(__ballot(g)) + __popcll(__ballot(g && ((src & 127) > 112))));
				}
			}
			GCOUNT(2, 1);
			static_assert(RMAX == 2, "HBM piece dealing pairs two rounds");
			if (__any(nc[0] > 0 || nc[1] > 0)) {
				const int32_t inc0 = wave_incl_scan(nc[0]);
				const int32_t tot0 = __shfl(inc0, 63);
				const int32_t inc1 = tot0 + wave_incl_scan(nc[1]);
				const int32_t tot = __shfl(inc1, 63);
				rtot[0] = tot0;
				rtot[1] = tot - tot0;
				rfirst[0] = 64;
				rfirst[1] = max(64 - tot0, 0);
				auto pack = [&](int32_t md, int32_t of, int32_t m, int32_t excl) -> uint64_t {
					return uint64_t(uint16_t(md - o_batch)) | (uint64_t(uint16_t(of)) << 16) |
					       (uint64_t(uint16_t(m)) << 32) | (uint64_t(uint16_t(excl)) << 48);
				};
				D.ldesc[lane] = pack(rdst[0] + rL[0], roff[0], rml[0], inc0 - nc[0]);
				D.ldesc[64 + lane] = pack(rdst[1] + rL[1], roff[1], rml[1], inc1 - nc[1]);
				const int32_t lo = min(chunk_owner2(D, inc0, nc[0], inc1, nc[1], 0), 127);
				const uint64_t dd = D.ldesc[lo];
				const int32_t od = o_batch + int32_t(dd & 0xffffu);
				const int32_t ooff = int32_t((dd >> 16) & 0xffffu), oml = int32_t((dd >> 32) & 0xffffu);
				const int32_t k = GC + lane - int32_t(dd >> 48);
				GCOUNT(0, __popcll(__ballot(lane < tot)));
				GCOUNT(1, __popcll(__ballot(lane < tot)) +
				              __popcll(__ballot(lane < tot && ((od - ooff + 16 * k) & 127) > 112)));
				if (lane < tot) {
					rpd = od + 16 * k;
					rpn = min(16, oml - 16 * k);
					__builtin_memcpy(&vr, ob + (od - ooff) + 16 * k, 16);
				}
				wave_lds_fence();  // ldesc / own[] are written again later
			}
		}
		ISTAMP(D_TLDS);

		// L: literals (input ring -> output ring).  Every run's first 16
		// bytes in its own lane; the pieces beyond (runs over 16 bytes) of
		// both rounds are dealt over the wave together, each piece reading
		// its run from an LDS descriptor.  (Storing a short last piece as 16
		// bytes that spill into its own match, rewritten in M, measured no
		// faster.)
		static_assert(RMAX == 2, "literal dealing pairs two rounds");
		{
#pragma unroll
			for (int r = 0; r < RMAX; ++r)  // (rL = 0 also where a round has no sequence: n = 0)
				ostore(D, rdst[r], ZL ? u32x4{ 0u, 0u, 0u, 0u } : fetch16(S, rL[r] > 0 ? rlit[r] : S.lo),
				       min(16, rL[r]));
			const int32_t nc0 = rL[0] > 16 ? (rL[0] - 1) >> 4 : 0;
			const int32_t nc1 = rL[1] > 16 ? (rL[1] - 1) >> 4 : 0;
			if (__any(nc0 > 0 || nc1 > 0)) {
				const int32_t inc0 = wave_incl_scan(nc0);
				const int32_t tot0 = __shfl(inc0, 63);
				const int32_t inc1 = tot0 + wave_incl_scan(nc1);
				const int32_t tot = __shfl(inc1, 63);
				auto pack = [&](int32_t lit, int32_t dst, int32_t L, int32_t excl) -> uint64_t {
					return uint64_t(uint16_t(lit - base)) | (uint64_t(uint16_t(dst - o_batch)) << 16) |
					       (uint64_t(uint16_t(L)) << 32) | (uint64_t(uint16_t(excl)) << 48);
				};
				D.ldesc[lane] = pack(rlit[0], rdst[0], rL[0], inc0 - nc0);
				D.ldesc[64 + lane] = pack(rlit[1], rdst[1], rL[1], inc1 - nc1);
				for (int32_t t0 = 0; t0 < tot; t0 += 64) {
					const int32_t t = t0 + lane;
					const int32_t lo = min(chunk_owner2(D, inc0, nc0, inc1, nc1, t0), 127);
					const uint64_t dd = D.ldesc[lo];
					const int32_t lit = base + int32_t(dd & 0xffffu);
					const int32_t dst = o_batch + int32_t((dd >> 16) & 0xffffu);
					const int32_t L = int32_t((dd >> 32) & 0xffffu);
					const int32_t k = 1 + t - int32_t(dd >> 48);  // piece 0 went in-lane
					const bool has = t < tot;
					ostore(D, dst + 16 * k, ZL ? u32x4{ 0u, 0u, 0u, 0u } : fetch16(S, has ? lit + 16 * k : S.lo),
					       has ? min(16, L - 16 * k) : 0);
				}
			}
		}
		wave_lds_fence();
		ISTAMP(D_LIT);

		// M: matches.  HBM-sourced matches store the pieces loaded in P,
		// both rounds first.  Every match whose source is in the LDS ring --
		// before the batch, in its own literals, or in this batch's match
		// output (near) -- is then cut into pieces dealt over the wave, both
		// rounds together in output order, 16 bytes each (a period-off
		// pattern: stp bytes, so every piece starts at phase 0), so a batch
		// costs its piece count / 64, not its longest match.  A piece
		// reading this chunk's output runs once every lower lane it reads
		// from has stored (one AND against a ballot per step; pieces of one
		// match never read each other: match byte i is source byte i mod
		// off).
		int32_t mring[RMAX], oring[RMAX], lring[RMAX];  // the rounds' ring-sourced matches
		// settle the HBM match loads in every lane: their first uses below
		// are lane-divergent, and a load left pending on the path that skips
		// them makes each later reuse of its registers wait vmcnt(0) (one
		// showed up inside the near-match loop)
		__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
		// pieces of HBM-sourced matches beyond the first GC, dealt and
		// loaded in P (the first 64 of the batch)
		ostore(D, rpd, vr, rpn);  // (rpn = 0: none)
#pragma unroll
		for (int r = 0; r < RMAX; ++r) {
			mring[r] = oring[r] = lring[r] = 0;
			if (64 * r < N) {
				const int32_t mdst = rdst[r] + rL[r], off = roff[r], ml = rml[r];
				const bool hbm = ml > 0 && mdst - off < glo;
				static_assert(GC == 1, "one own HBM piece per match");
				ostore(D, mdst, vg[r][0], hbm ? min(16, ml) : 0);
				int32_t xoff = off, xml = (ml > 0 && !hbm) ? ml : 0;  // its ring copy, if any
				if (d1p) {
					// quirk D1 (d1_emulable): the match's first k1 bytes are
					// what the last wild copy left past the frontier, from d =
					// OPH - off on -- the payload bytes after its literals, or
					// (no literals) the output bytes after the previous
					// match's source, which P put in rlit (a D1 match reads
					// >= 65,529 back: always HBM-sourced, stored above).  Those
					// output bytes: from HBM when flushed (below glo), else a
					// ring copy of their own (offset mdst - q, k1 bytes) among
					// the batch's ring matches, which orders it after the
					// bytes' producers and before their readers
					int32_t k1 = 0, sp = S.lo, gq = 0;
					bool fo = false;
					if (ml > 0 && n1 + mdst < off && oph - off < 8) {
						const int32_t dd = oph - off;
						const int32_t ovs = rL[r] > 0 ? 8 * ((rL[r] + 7) >> 3) - rL[r] : rlit[r] & 7;
						if (dd < ovs) {
							k1 = min(ovs - dd, ml);
							if (rL[r] > 0) {
								sp = rlit[r] + rL[r] + dd;
							} else {
								gq = (rlit[r] >> 3) - D1_QBIAS + dd;
								fo = true;
							}
						}
					}
					if (fo && gq >= glo) {
						xoff = mdst - gq;
						xml = k1;
						k1 = 0;
						fo = false;
					}
					u32x4 v = ZL ? u32x4{ 0u, 0u, 0u, 0u } : fetch16(S, sp);
					if (fo)
						__builtin_memcpy(&v, ob + gq, 16);
					ostore(D, mdst, v, k1);
				}
				if (rtot[r] > rfirst[r]) {  // rare: more than 64 dealt pieces; the rest now
					const int32_t nc = hbm ? max(((ml + 15) >> 4) - GC, 0) : 0;
					const int32_t inc = wave_incl_scan(nc);
					for (int32_t t0 = rfirst[r]; t0 < rtot[r]; t0 += 64) {
						const int32_t t = t0 + lane;
						const int32_t lo = piece_owner(inc, t);
						const int32_t k = GC + t - (__shfl(inc, lo) - __shfl(nc, lo));
						const int32_t osrc = __shfl(mdst - off, lo), odst = __shfl(mdst, lo);
						const int32_t oml = __shfl(ml, lo);
						if (t < rtot[r]) {
							u32x4 v;
							__builtin_memcpy(&v, ob + osrc + 16 * k, 16);
							ostore(D, odst + 16 * k, v, min(16, oml - 16 * k));
						}
					}
					// settle this rare path's loads (see fetch4)
					__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
				}
				mring[r] = mdst;
				oring[r] = xoff;
				lring[r] = xml;
			}
		}
		// every HBM-sourced match of the batch is stored before the ring
		// matches run (none reads another's output: their sources are in HBM)
		wave_lds_fence();
		ISTAMP(D_MFAR);
		// ring-sourced matches: with a long one (over RING_LANE_MAX bytes) in
		// the batch, the pieces of both rounds are dealt over the wave
		// together; rounds of short ones only (e.g. dense data) keep one lane
		// per match -- the dealing's fixed cost (owner search, dependency
		// masks) would dominate there
		static_assert(RMAX == 2, "ring dealing pairs two rounds");
		if (__any(lring[0] > RING_LANE_MAX || lring[1] > RING_LANE_MAX)) {
			const int32_t st = ring_pieces(D, mring, oring, lring, o_batch, glo);
			ICOUNT(D_TASKS, 1);
			ICOUNT(D_ROUNDS, st);
			(void)st;
		} else {
#pragma unroll
			for (int r = 0; r < RMAX; ++r) {
				if (64 * r < N) {
					const int32_t st = ring_lanes(D, mring[r], oring[r], lring[r], rbeg[r], rL[r], glo);
					ICOUNT(D_GBATCHES, 1);
					ICOUNT(D_LANES, st);
					(void)st;
				}
			}
		}
		ISTAMP(D_NEAR);

		// flush whole 16-byte units of [o_batch, o_end) (the first may start
		// before o_batch: those bytes are in the ring too); always FLUSH_ST
		// store instructions, so the wait above can count them
		{
			const int32_t u0 = o_batch >> 4, u1 = o_end >> 4;
#pragma unroll
			for (int i = 0; i < FLUSH_ST; ++i) {
				const int32_t u = u0 + lane + 64 * i;
				if (u < u1)
					*reinterpret_cast<GLOBAL u32x4*>(ob + (u << 4)) =
					    *reinterpret_cast<const u32x4*>(&D.oring[(u << 4) & OMASK]);
			}
		}
		o_batch = o_end;
		k0 += m;
		ISTAMP(D_FLUSH);
	}
	d1 = __any(d1);
	deep = __any(deep);
	if (ZL)
		hcnt = __shfl(wave_incl_scan(hcnt), 63);
	if (!bad && lane == 0 && (o_batch & 15))  // last partial unit
		gstore_n(ob + (o_batch & ~15), *reinterpret_cast<const u32x4*>(&D.oring[(o_batch & ~15) & OMASK]),
		         o_batch & 15);
	if (lane == 0) {
		if (bad) {
			status[b].code = DS_RETRY;
		} else {
			status[b].code = DS_OK;
			status[b].aux = (d1 ? AUX_D1_RISK : 0) | (d1p ? AUX_D1_EMU : 0) | (deep ? AUX_DEEP_HIST : 0);
			status[b].detail = ZL ? hcnt : 0;  // ZL: the linked path's density estimate
			status[b].err_out_pos = 0;
			status[b].out_len = uint32_t(o_batch);
		}
	}
	ISTAMP_FLUSH();
	out_len = bad ? 0 : o_batch;
	return bad ? DS_RETRY : DS_OK;
}

// Independent blocks (linked 0): one wave per block.  Linked frames in the
// history layout of lz4ada_linked.hip (linked 2): one wave per block, each
// slot preceded by LINK_HIST readable bytes.  Linked frames in contiguous
// slots (linked 1, launched as one workgroup): the blocks in order, each
// reading the previous ones' output as history while every block so far is
// full (its slot then continues the previous one); a declined or short
// block leaves every later block DS_RETRY for the exact path.  Pinned to two waves per
// SIMD (at most 256 registers, so the allocator never reaches for AGPRs):
// LDS allows 8 waves per CU, and the bench's 2048 blocks are all resident.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_decode_idx(const uint8_t* __restrict__ frame,
                                                    uint64_t frame_len,
                                                    const lz4ada_block_desc* __restrict__ desc,
                                                    uint32_t nblocks, uint8_t* __restrict__ tab_all,
                                                    uint8_t* __restrict__ out,
                                                    lz4ada_block_status* __restrict__ status,
                                                    int linked)
{
	__shared__ union {
		DecLds d;
		IdxLds x;
	} U;
	DecLds& D = U.d;
	if (linked == 3) {
		// fused: pass 1 of this block first (its table and status, read
		// below by this same wave, made visible to it first), so a block's pass 2
		// starts when its own pass 1 is done, not when every block's is
		if (blockIdx.x < nblocks)
			index_block(U.x, frame, frame_len, desc, blockIdx.x, tab_all, status);
		// workgroup scope is enough (the same wave reads it back); an agent
		// fence here wrote the whole L2 back once per block
		vm_wait();
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
		__syncthreads();
		linked = 0;
	}
	// one call site of decode_block for every mode (code size)
	int64_t hist = linked == 2 ? LINK_HIST : 0;
	uint32_t b = linked == 1 ? 0u : blockIdx.x;
	const uint32_t bend = linked == 1 ? nblocks : min(blockIdx.x + 1u, nblocks);
	for (; b < bend; ++b) {
		int32_t len;
		const int32_t code = decode_block(D, frame, frame_len, desc, b, tab_all, out, status,
		                                  hist, len);
		if (linked != 1)
			return;
		vm_wait();  // the next block reads this output as history
		__syncthreads();
		if (code != DS_OK)
			break;
		if (b + 1 < nblocks && (uint32_t(len) != desc[b].out_cap ||
		                        desc[b + 1].out_off != desc[b].out_off + uint64_t(len))) {
			++b;  // the next block's history would not be contiguous
			break;
		}
		hist += len;
	}
	if (linked != 1)
		return;
	for (uint32_t r = b + lane_id(); r < nblocks; r += 64)
		if (status[r].code == DS_OK || r > b)
			status[r].code = DS_RETRY;
}


// The linked path's literal-zero plane (decode_block<true>): pass 2 of every
// block in the history layout, one wave per block.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_decode_idx_zl(
        const uint8_t* __restrict__ frame, uint64_t frame_len, const lz4ada_block_desc* __restrict__ desc,
        uint32_t nblocks, uint8_t* __restrict__ tab_all, uint8_t* __restrict__ out,
        lz4ada_block_status* __restrict__ status)
{
	__shared__ DecLds D;
	if (blockIdx.x >= nblocks)
		return;
	int32_t len;
	decode_block(D, frame, frame_len, desc, blockIdx.x, tab_all, out, status, LINK_HIST, len, true, true);
}

// The linked path's byte planes (x, and y / h when a block needs them):
// pass 2 of every block in the history layout with quirk D1 emulated under
// the host's predicted round state (decode_block's D1E; k_decode_idx's
// linked 2 mode without it).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_decode_idx_lk(
        const uint8_t* __restrict__ frame, uint64_t frame_len, const lz4ada_block_desc* __restrict__ desc,
        uint32_t nblocks, uint8_t* __restrict__ tab_all, uint8_t* __restrict__ out,
        lz4ada_block_status* __restrict__ status)
{
	__shared__ DecLds D;
	if (blockIdx.x >= nblocks)
		return;
	int32_t len;
	decode_block(D, frame, frame_len, desc, blockIdx.x, tab_all, out, status, LINK_HIST, len, false, true);
}

// ============================================================ two waves
// Pass 1 by the two waves of a 128-lane workgroup (k_decode_pp2's): 128
// lanes walk one 16 KiB chunk, 128 bytes each; wave 0's lane 0 enters at
// the exact chain position, wave 1's lane 0 at its lead-in guess until wave
// 0's exit is known (one exchange per chunk).  (Round 4's k_decode_idx2,
// which also split each pass-2 batch between the two waves, was retired in
// round 6: k_decode_pp2 pipelining whole batches replaced it where two
// waves per block pay, docs/DESIGN_LOG.md §3.)

constexpr int SEG2 = 128;          // pass-1 segment per lane: 128 lanes per 16 KiB chunk
constexpr int NSUB2 = SEG2 / SUB;  // records per segment
static_assert(128 * SEG2 == CHUNK, "two waves walk one pass-1 chunk");
#ifndef LZ4ADA_LEAD_SEQ2
#define LZ4ADA_LEAD_SEQ2 60
#endif
constexpr int32_t LEAD_SEQ2 = LZ4ADA_LEAD_SEQ2;

struct alignas(16) IdxLds2 {
	uint8_t buf[CHUNK + 16];
	uint32_t rbm[128][NSUB2 + 1];
	uint16_t rcnt[128][NSUB2 + 1];
	int32_t xa;        // wave 0's largest exit (wave 1's lane-0 entry)
	int32_t xs[2][4];  // per wave: largest exit, sequence starts, bad, used sub-segments
};

__device__ __forceinline__ int32_t lead_in_bytes2(int32_t starts)
{
	const int32_t l = LEAD_SEQ2 * (CHUNK / max(starts, 1));
	return __builtin_amdgcn_readfirstlane(min(max(l, LEAD_MIN), LEAD_MAX));
}

// Pass 1 of block b by both waves of the workgroup (index_block's rules).
__device__ __forceinline__ void index_block2(IdxLds2& X, const uint8_t* __restrict__ frame,
                                             uint64_t frame_len,
                                             const lz4ada_block_desc* __restrict__ desc, uint32_t b,
                                             uint8_t* __restrict__ tab_all,
                                             lz4ada_block_status* __restrict__ status)
{
	const int32_t tid = int32_t(threadIdx.x), w = tid >> 6, lane = tid & 63;
	const lz4ada_block_desc d = desc[b];
	if (d.flags & LZ4ADA_BLOCK_STORED) {
		if (tid == 0)
			status[b].code = DS_OK;
		return;
	}
	if (d.in_len >= RLE_MIN_IN && uint64_t(d.in_len) * RLE_RATIO < uint64_t(d.out_cap)) {
		if (tid == 0)
			status[b].code = DS_SPARSE;
		return;
	}
	cg8* in = gptr(frame) + d.in_off;
	const int32_t n = int32_t(d.in_len);
	const uintptr_t lim = reinterpret_cast<uintptr_t>(frame) + frame_len;
	const int32_t mis = int32_t(reinterpret_cast<uintptr_t>(in) & 15u);
	uint64_t* tab = reinterpret_cast<uint64_t*>(tab_all) + (((d.in_off >> 8) + b) << 3);

	Src S;
	S.lds = X.buf;
	S.mask = CHUNK - 1;
	S.mis = mis;
	S.in = in;
	S.lim = lim;
	constexpr int PF = CHUNK / 2048;  // 16-byte loads per thread per chunk
	auto load16k = [&](uintptr_t a, u32x4 (&v)[PF]) {
		if (a + CHUNK <= lim) {
#pragma unroll
			for (int r = 0; r < PF; ++r)
				__builtin_memcpy(&v[r], reinterpret_cast<cg8*>(a + uintptr_t(2048 * r + 16 * tid)), 16);
		} else {
#pragma unroll
			for (int r = 0; r < PF; ++r)
				v[r] = gload16(a + uintptr_t(2048 * r + 16 * tid), lim);
		}
	};
	const uintptr_t abase = reinterpret_cast<uintptr_t>(in) - uintptr_t(mis);
	u32x4 pf[PF];
	if (n > 0)
		load16k(abase, pf);

	int32_t E = 0, lead = LEAD_IN0;
	bool bad = false, sparse = false;
	for (int32_t C = 0; C < n && !bad; C += CHUNK) {
#pragma unroll
		for (int r = 0; r < PF; ++r)
			*reinterpret_cast<u32x4*>(&X.buf[2048 * r + 16 * tid]) = pf[r];
		if (tid == 0)
			*reinterpret_cast<u32x4*>(&X.buf[CHUNK]) = pf[0];
		__syncthreads();
		if (C + CHUNK < n)
			load16k(abase + uintptr_t(C + CHUNK), pf);
		S.lo = C - mis;
		S.hi = C - mis + CHUNK;

		const int32_t s = C + SEG2 * tid;
		const int32_t seg_end = min(s + SEG2, n);
		int32_t ein = (tid == 0) ? E : s;
		if (tid > 0 && s < n) {  // lead-in (index_block)
			int32_t p = max(s - lead, C);
			while (p < s)
				p = skip_seq(S, p);
			ein = p;
		}
		uint32_t* ghi = reinterpret_cast<uint32_t*>(tab + (C >> 5) + NSUB2 * tid) + 1;
		int32_t epos = INT32_MAX;
		bool err = false;
		int32_t nst = 0;
		int32_t y = (s < n) ? walk_segment<NSUB2>(S, ein, s, seg_end, n, X.rbm[tid], X.rcnt[tid], ghi, err,
		                                          epos, 0, false, nst)
		                    : ein;
		// this wave's lane-0 entry: exact for wave 0, wave 1's lead-in guess
		// until wave 0's largest exit is known
		int32_t e0 = __shfl(ein, 0);
		auto converge = [&]() {
			for (int it = 0; it < 64; ++it) {
				int32_t prev = __shfl_up(wave_incl_max(y), 1);
				if (lane == 0)
					prev = e0;
				const bool changed = prev != ein;
				if (!__any(changed))
					break;
				if (changed) {
					ein = prev;
					if (s < n) {
						y = walk_segment<NSUB2>(S, ein, s, seg_end, n, X.rbm[tid], X.rcnt[tid], ghi, err,
						                        epos, y, !err, nst);
					} else {
						y = ein;
						err = false;
					}
				}
			}
		};
		converge();
		{
			const int32_t mx = __shfl(wave_incl_max(y), 63);
			if (tid == 0)
				X.xa = mx;
		}
		__syncthreads();
		if (w == 1) {
			const int32_t ea = X.xa;
			if (ea != e0) {  // the guess missed: the lanes it reached walk again
				e0 = ea;
				converge();
			}
		}
		// converged: every lane's records are its last walk's, to HBM
		bad = __any(s < n && err);
		wave_lds_fence();
		int32_t starts = 0;
#pragma unroll
		for (int i = 0; i < NSUB2; ++i) {
			const int32_t r = 64 * i + lane, sg = 64 * w + r / NSUB2, sb = r & (NSUB2 - 1);
			if (C + SEG2 * sg < n) {
				const uint32_t bmv = X.rbm[sg][sb], c16 = X.rcnt[sg][sb];
				starts += __popc(bmv);
				if (c16 != 0xFFFFu)
					tab[(C >> 5) + 256 * w + r] = uint64_t(bmv) | (uint64_t(c16) << 32);
				else
					*reinterpret_cast<uint32_t*>(tab + (C >> 5) + 256 * w + r) = bmv;
			}
		}
		int32_t used = 0;
		if (C == 0 && s < n)
			for (int k = 0; k < NSUB2; ++k)
				used += X.rbm[tid][k] ? 1 : 0;
		starts = __shfl(wave_incl_scan(starts), 63);
		used = __shfl(wave_incl_scan(used), 63);
		const int32_t mx = __shfl(wave_incl_max(y), 63);
		if (lane == 0) {
			X.xs[w][0] = mx;
			X.xs[w][1] = starts;
			X.xs[w][2] = bad ? 1 : 0;
			X.xs[w][3] = used;
		}
		__syncthreads();  // also: every read of this chunk's staging is done
		E = max(X.xs[0][0], X.xs[1][0]);
		bad = (X.xs[0][2] | X.xs[1][2]) != 0;
		lead = lead_in_bytes2(X.xs[0][1] + X.xs[1][1]);
		if (C == 0 && n >= 4 * CHUNK && !bad && X.xs[0][3] + X.xs[1][3] < CHUNK / SUB / 4)
			bad = sparse = true;  // literal-heavy (index_block)
	}
	if (E != n)
		bad = true;
	if (tid == 0)
		status[b].code = bad ? (sparse ? DS_SPARSE : DS_RETRY) : DS_OK;
}

// ============================================================ pipelined pair
// k_decode_pp2 (round 5): two waves per block that pipeline consecutive
// batches instead of splitting each one (k_decode_idx2), for launches of at
// most one block per SIMD -- a configs[3] shard at N = 8 (1,024 blocks) --
// where a block has the LDS (~30 KiB) and the VGPRs (two waves per SIMD at
// <= 256) for two-round batches of up to 128 sequences in each wave.  Each
// block's chain is latency-bound: wave w takes batches j = w,
// w + 2, ...; batch j's staging, cut, parse, HBM-sourced loads, literals and
// HBM-sourced stores run while the other wave is still inside batch j - 1,
// and only the ring-sourced matches (which may read batch j - 1's output)
// wait for batch j - 1's to be stored -- an LDS token, no barrier in the
// batch loop.  Both waves compute every cut from the staged pass-1 records
// (each its own batch and the next), so they agree on the batch sequence,
// on who stages which input chunk and on the HBM threshold; spin waits on
// LDS counters carry the hand-offs, each bounded (a hand-off that never
// comes declines the block instead of hanging the grid).
//
// Window discipline (16 KiB output window, batches of <= OW bytes): while
// batch j runs its ring-sourced matches, batch j + 1 may write its literals
// and HBM-sourced bytes, so the window keeps [o_j - RFLOOR2, o_j + OW)
// intact.  A match reads HBM for its source bytes below glo_j =
// align16(o_{j-1}) rounded down to a 128-byte line (written by the flushes
// of batches <= j - 2, whose completion each wave publishes after its own
// vmcnt wait; a CU's L1 never gets a line holding bytes not yet flushed) in
// whole 16-byte pieces, and the window for the rest (a match straddling the
// threshold is split in two).  A first try with one-round batches and four
// waves per SIMD at 2,048 blocks (k_decode_pp, commit dd280ab) ran 15.6 ms
// against k_decode_idx's 13.3: 64-sequence batches cost ~0.7 of a
// 128-sequence one (tools/time_decode.py, LZ4ADA_SEQ_CUT=64), and four
// waves per SIMD slow each one ~1.3x.

constexpr int ORING2 = 16384;                 // output window of the pipelined pair
constexpr int32_t RFLOOR2 = ORING2 - 2 * OW;  // window bytes kept below a batch through its ring phase
static_assert(OW + 16 + 128 + 16 < RFLOOR2, "the HBM threshold must lie inside the kept window");

struct alignas(16) PpLds2 {
	uint8_t ring[RING + 16];   // staged input: 4 chunks of 2 KiB (+ mirror), shared
	uint8_t oring[ORING2];     // output window, shared
	uint64_t rrec[4 * 64];     // pass-1 records of the staged chunks
	uint64_t ldesc[2][2 * 64]; // per wave: run / match descriptors of both rounds
	uint16_t cst[2][MAXSEQ];   // per wave: its batch's sequence starts
	uint8_t own[2][256];       // per wave: piece owners
	int32_t tok;               // last batch whose ring-sourced matches are stored
	int32_t staged;            // input chunks staged so far
	int32_t abort_;            // a wave declined the block
	int32_t pad;
	int32_t done[2];           // per wave: last own batch whose flush has completed
};

struct WP2 {
	PpLds2& L;
	int32_t w;
};
__device__ __forceinline__ uint8_t* oring_of(WP2& V) { return V.L.oring; }
__device__ __forceinline__ const uint8_t* oring_of(const WP2& V) { return V.L.oring; }
__device__ __forceinline__ uint8_t* own_of(WP2& V) { return V.L.own[V.w]; }
__device__ __forceinline__ uint64_t* ldesc_of(WP2& V) { return V.L.ldesc[V.w]; }
__device__ __forceinline__ constexpr uint32_t omask_of(const WP2&) { return ORING2 - 1; }

__device__ __forceinline__ int32_t lds_peek(const int32_t* p)
{
	return __builtin_amdgcn_readfirstlane(*reinterpret_cast<const volatile int32_t*>(p));
}

// Publish v at p after every LDS write of this wave so far (the other wave
// reads those once it sees v): lgkmcnt(0) only, the flush stores in flight
// are not waited for.
__device__ __forceinline__ void lds_publish(int32_t* p, int32_t v)
{
	asm volatile("" ::: "memory");
	__builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt/expcnt untouched
	*reinterpret_cast<volatile int32_t*>(p) = v;
	asm volatile("" ::: "memory");
}

// Wait until *p >= want; false if the block was aborted meanwhile -- or
// after ~2^24 polls (~0.5 s): a hand-off that never comes declines the
// block (DS_RETRY: k_decode_pc redoes it) instead of hanging the grid.
__device__ __forceinline__ bool lds_wait_ge(int32_t* abort_flag, const int32_t* p, int32_t want)
{
	for (uint32_t it = 0; lds_peek(p) < want; ++it) {
		if (lds_peek(abort_flag))
			return false;
		if (it >= (1u << 24)) {
			lds_publish(abort_flag, 1);
			return false;
		}
		__builtin_amdgcn_s_sleep(1);
	}
	asm volatile("" ::: "memory");
	return true;
}

// One batch cut from the staged records (decode_block's rule: <= OW output
// bytes, <= MAXSEQ sequences): sub-segments [k0, k0 + m).  over: the first
// sub-segment alone exceeds a limit -- the 64 from k0 go straight to HBM.
struct PpCut {
	int32_t m, bytes;
	bool over;
};
__device__ __forceinline__ PpCut pp_cut(const PpLds2& L, int32_t k0, int32_t nsub)
{
	const int32_t k = k0 + int32_t(lane_id());
	const uint64_t rec = k < nsub ? L.rrec[k & 255] : 0;
	const int32_t cnt = int32_t(min(uint32_t(rec >> 32), 1u << 24));
	const int32_t incl = wave_incl_scan(cnt);
	const int32_t incl_s = wave_incl_scan(__popc(uint32_t(rec)));
	PpCut c;
	c.m = __popcll(__ballot(incl <= OW && incl_s <= MAXSEQ));
	c.over = c.m == 0;
	c.m = c.over ? 64 : c.m;
	c.bytes = __shfl(incl, c.m - 1);
	return c;
}

__device__ __forceinline__ void pp_load_chunk(uintptr_t abase, int32_t c, uintptr_t lim, const uint64_t* tab,
                                              int32_t nsub, u32x4& v0, u32x4& v1, uint64_t& r)
{
	load_chunk2(abase, c, lim, v0, v1);
	const int32_t k = 64 * c + int32_t(lane_id());
	r = k < nsub ? __builtin_nontemporal_load(tab + k) : 0;
}

__device__ __forceinline__ void pp_stage_chunk(PpLds2& L, int32_t c, const u32x4& v0, const u32x4& v1,
                                               uint64_t r)
{
	const uint32_t lane = lane_id();
	const uint32_t a = uint32_t(c * BATCH) & (RING - 1);
	*reinterpret_cast<u32x4*>(&L.ring[a + 16 * lane]) = v0;
	*reinterpret_cast<u32x4*>(&L.ring[a + 1024 + 16 * lane]) = v1;
	if (a == 0 && lane == 0)
		*reinterpret_cast<u32x4*>(&L.ring[RING]) = v0;
	L.rrec[64 * (c & 3) + lane] = r;
}

// Pass 2 of block b (independent; pass 1's verdict DS_OK) by both waves.
// Returns the output length, or -1 when the block is declined.
__device__ __forceinline__ int32_t decode_block_pp2(PpLds2& L, const uint8_t* __restrict__ frame,
                                                    uint64_t frame_len,
                                                    const lz4ada_block_desc* __restrict__ desc, uint32_t b,
                                                    const uint8_t* __restrict__ tab_all,
                                                    uint8_t* __restrict__ out)
{
	const int32_t tid = int32_t(threadIdx.x), w = tid >> 6, lane = tid & 63;
	WP2 V{ L, w };
	const lz4ada_block_desc d = desc[b];
	cg8* in = gptr(frame) + d.in_off;
	g8* ob = gptr(out) + d.out_off;
	const int32_t n = int32_t(d.in_len);
	const int32_t cap = int32_t(d.out_cap);
	const uintptr_t lim = reinterpret_cast<uintptr_t>(frame) + frame_len;
	const uintptr_t olim = reinterpret_cast<uintptr_t>(ob) + uintptr_t(cap);
	const int32_t mis = int32_t(reinterpret_cast<uintptr_t>(in) & 15u);
	const uint64_t* tab = reinterpret_cast<const uint64_t*>(tab_all) + (((d.in_off >> 8) + b) << 3);
	const int32_t nsub = (n + SUB - 1) / SUB;
	const uintptr_t abase = reinterpret_cast<uintptr_t>(in) - uintptr_t(mis);
	constexpr uint32_t WMASK = ORING2 - 1;
	int32_t* const abort_flag = &L.abort_;

	Src S;
	S.lds = L.ring;
	S.mask = RING - 1;
	S.mis = mis;
	S.in = in;
	S.lim = lim;

	// The cut cursor: the next batch to cut is j, at sub-segment k0 and
	// output byte o; hi = input chunks staged once the batches cut so far
	// have staged theirs (the owner of batch j stages [hi_before, cf_j + 3)).
	// o_prev / over_prev: batch j - 1's output start and whether it went
	// straight to HBM.  Each wave cuts its own batch and the next one.
	int32_t j = 0, k0 = 0, o = 0, hi = 0, o_prev = 0;
	bool over_prev = false;
	auto advance = [&](PpCut& c) {
		c = pp_cut(L, k0, nsub);
		o_prev = o;
		over_prev = c.over;
		o += c.bytes;
		k0 += c.m;
		++j;
	};
	auto chunk_of = [&](int32_t k) { return (k * SUB + mis) / BATCH; };
	u32x4 pf0 = u32x4{ 0u, 0u, 0u, 0u }, pf1 = pf0;  // this wave's prefetched chunk pfc
	uint64_t pr = 0;
	int32_t pfc = -1;
	bool bad = false;
	if (w == 1 && k0 < nsub) {  // batch 0 is wave 0's: cut it once staged
		hi = chunk_of(0) + 3;
		PpCut c0;
		if (lds_wait_ge(abort_flag, &L.staged, hi))
			advance(c0);
		else
			bad = true;
	}

	while (!bad && k0 < nsub) {
		// ---- batch j is this wave's
		const int32_t jb = j, ob0 = o, kb = k0;
		const bool prev_over = over_prev;
		// HBM holds, complete, every byte below glo: batches <= j - 2, or all
		// of batch j - 1 when it went straight to HBM
		const int32_t glo = jb == 0 ? 0 : ((prev_over ? ob0 : o_prev) & ~15);
		const int32_t cf = chunk_of(kb);
		const int32_t hi_before = hi;
		hi = max(hi, cf + 3);
		if (!lds_wait_ge(abort_flag, &L.staged, hi_before)) {
			bad = true;
			break;
		}
		for (int32_t c = hi_before; c < hi; ++c) {
			if (c != pfc) {
				pp_load_chunk(abase, c, lim, tab, nsub, pf0, pf1, pr);
				__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): a rare path's loads settle here
			}
			pp_stage_chunk(L, c, pf0, pf1, pr);
			pfc = -1;
		}
		if (hi > hi_before)
			lds_publish(&L.staged, hi);
		S.lo = cf * BATCH - mis;
		S.hi = hi * BATCH - mis;
		// this batch's cut, then the next one's (its records are staged:
		// chunks <= cf + 2), which places this wave's next batch: prefetch the
		// chunk that batch will stage
		PpCut cb;
		advance(cb);
		const int32_t oe = o;
		bool next_over = false;
		int32_t npf = 0;  // vector loads issued after this wave's last flush
		if (k0 < nsub) {
			hi = max(hi, chunk_of(k0) + 3);
			PpCut cn;
			advance(cn);
			next_over = cn.over;
			if (k0 < nsub && chunk_of(k0) + 3 > hi) {
				pfc = hi;
				pp_load_chunk(abase, pfc, lim, tab, nsub, pf0, pf1, pr);
				npf = 3;
			}
		}
		if (oe > cap) {
			bad = true;
			lds_publish(abort_flag, 1);
			break;
		}
		if (cb.over) {
			// ---- a sub-segment alone exceeds the batch limits: the 64
			// sub-segments go straight to HBM (batch_global), alone -- after
			// every earlier batch's bytes are final in HBM and in the window
			if (!lds_wait_ge(abort_flag, &L.tok, jb - 1) || !lds_wait_ge(abort_flag, &L.done[w ^ 1], jb - 1)) {
				bad = true;
				break;
			}
			vm_wait();
			const int32_t k = kb + lane;
			const int32_t sub_s = k * SUB;
			const int32_t sub_end = min(sub_s + SUB, n);
			const uint64_t rec = (k < nsub) ? L.rrec[k & 255] : 0;
			const uint32_t bm = uint32_t(rec);
			const int32_t cnt = int32_t(min(uint32_t(rec >> 32), 1u << 24));
			const int32_t p0 = bm ? sub_s + __builtin_ctz(bm) : n;
			const int32_t incl = wave_incl_scan(cnt);
			const int32_t a0 = ob0 & ~15;
			if (lane == 0 && ob0 > a0)  // the window's unflushed tail
				gstore_n(ob + a0, *reinterpret_cast<const u32x4*>(&L.oring[a0 & WMASK]), ob0 - a0);
			vm_wait();
			const bool ok = !__any(!batch_global(S, ob, olim, p0, sub_end, n, ob0 + incl - cnt, ob0, 0));
			vm_wait();
			if (!ok) {
				bad = true;
				lds_publish(abort_flag, 1);
				break;
			}
			// the window's history again, from HBM (nontemporal: past the L1,
			// which may hold lines of this batch from before their stores)
			const int32_t x0 = max(oe - ORING2 + 16, 0) & ~15;
			for (int32_t x = x0 + 16 * lane; x < oe + 15; x += 64 * 16)
				*reinterpret_cast<u32x4*>(&L.oring[uint32_t(x) & WMASK]) =
				    x + 16 <= cap ? __builtin_nontemporal_load(reinterpret_cast<const GLOBAL u32x4*>(ob + x))
				                  : gload16(reinterpret_cast<uintptr_t>(ob) + uintptr_t(intptr_t(x)), olim);
			__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
			lds_publish(&L.done[w], jb);
			lds_publish(&L.tok, jb);
			continue;
		}
		if (prev_over && !lds_wait_ge(abort_flag, &L.tok, jb - 1)) {
			bad = true;  // (the batch before went straight to HBM: its window reload first)
			break;
		}

		// ---- the batch's sequence starts, in output order
		const int32_t base = kb * SUB;
		int32_t N;
		{
			const int32_t k = kb + lane;
			const int32_t sub_s = k * SUB;
			const uint64_t rec = (k < nsub) ? L.rrec[k & 255] : 0;
			uint32_t bm = uint32_t(rec);
			const int32_t nseq = __popc(bm);
			const int32_t incl_s = wave_incl_scan(nseq);
			if (lane < cb.m) {
				int32_t e = incl_s - nseq;
				const uint16_t rel = uint16_t(sub_s - base);
				for (; bm; bm &= bm - 1)
					L.cst[w][e++] = uint16_t(rel + __builtin_ctz(bm));
			}
			N = __shfl(incl_s, cb.m - 1);
		}
		wave_lds_fence();
		const int32_t gl = glo & ~127;  // HBM pieces end in whole lines below this

		// ---- P: up to 64 sequences per round, placed by a prefix sum; each
		// match split into its HBM part (hml bytes) and its window part
		int32_t rL[RMAX], rlit[RMAX], roff[RMAX], rml[RMAX], rdst[RMAX], rbeg[RMAX], hml[RMAX];
		bool pre = false, anyg = false;
		{
			int32_t o_round = ob0;
			// both rounds parsed first, then the rare shapes, then placement
			// (as decode_block)
			bool fok[RMAX];
#pragma unroll
			for (int r = 0; r < RMAX; ++r) {
				rL[r] = rlit[r] = roff[r] = rml[r] = hml[r] = 0;
				fok[r] = true;
				const int32_t idx = 64 * r + lane;
				if (idx < N) {
					Seq q;
					fok[r] = parse_fast_try(S, base + int32_t(L.cst[w][idx]), n, q);
					rL[r] = q.L;
					rlit[r] = q.lit;
					roff[r] = q.off;
					rml[r] = q.ml;
				}
			}
#pragma unroll
			for (int r = 0; r < RMAX; ++r) {
				if (__builtin_expect(__any(!fok[r]), 0)) {
					if (!fok[r]) {
						Seq q;
						parse_seq(S, base + int32_t(L.cst[w][64 * r + lane]), n, q);
						rL[r] = q.L;
						rlit[r] = q.lit;
						roff[r] = q.off;
						rml[r] = q.ml;
					}
				}
			}
#pragma unroll
			for (int r = 0; r < RMAX; ++r) {
				rbeg[r] = o_round;
				if (64 * r < N) {
					const int32_t len = rL[r] + rml[r];
					const int32_t inc = wave_incl_scan(len);
					rdst[r] = o_round + inc - len;
					o_round += __shfl(inc, 63);
					const int32_t mdst = rdst[r] + rL[r];
					if (rml[r] > 0) {
						if (roff[r] > mdst)
							pre = true;  // a reference before the block start (D2)
						const int32_t room = gl - (mdst - roff[r]);
						hml[r] = ((rml[r] + 15) & ~15) <= room ? rml[r] : max(room & ~15, 0);
						if (hml[r] > 0)
							anyg = true;
					}
				}
			}
		}
		if (__any(pre)) {
			bad = true;
			lds_publish(abort_flag, 1);
			break;
		}

		// ---- HBM-sourced parts: this wave's flush of batch j - 2 first (the
		// prefetch loads issued after it may stay in flight), then the other
		// wave's of batch j - 3; every load in flight before the first use: a
		// part's first piece in its own lane, the rest of both rounds dealt
		if (npf)
			asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
		else
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		lds_publish(&L.done[w], max(jb - 2, -1));
		u32x4 vg[RMAX], vr = u32x4{ 0u, 0u, 0u, 0u };
		int32_t rtot[RMAX], rfirst[RMAX];
		int32_t rpd = 0, rpn = 0;
#pragma unroll
		for (int r = 0; r < RMAX; ++r) {
			vg[r] = vr;
			rtot[r] = rfirst[r] = 0;
		}
		if (__any(anyg)) {
			if (!lds_wait_ge(abort_flag, &L.done[w ^ 1], jb - 3)) {
				bad = true;
				break;
			}
			int32_t nc[RMAX];
#pragma unroll
			for (int r = 0; r < RMAX; ++r) {
				nc[r] = 0;
				if (64 * r < N) {
					const int32_t src = rdst[r] + rL[r] - roff[r];
					if (hml[r] > 0)
						__builtin_memcpy(&vg[r], ob + src, 16);
					nc[r] = hml[r] > 0 ? max(((hml[r] + 15) >> 4) - 1, 0) : 0;
				}
			}
			if (__any(nc[0] > 0 || nc[1] > 0)) {
				const int32_t inc0 = wave_incl_scan(nc[0]);
				const int32_t tot0 = __shfl(inc0, 63);
				const int32_t inc1 = tot0 + wave_incl_scan(nc[1]);
				const int32_t tot = __shfl(inc1, 63);
				rtot[0] = tot0;
				rtot[1] = tot - tot0;
				rfirst[0] = 64;
				rfirst[1] = max(64 - tot0, 0);
				auto pack = [&](int32_t md, int32_t of, int32_t m, int32_t excl) -> uint64_t {
					return uint64_t(uint16_t(md - ob0)) | (uint64_t(uint16_t(of)) << 16) |
					       (uint64_t(uint16_t(m)) << 32) | (uint64_t(uint16_t(excl)) << 48);
				};
				uint64_t* ldesc = ldesc_of(V);
				ldesc[lane] = pack(rdst[0] + rL[0], roff[0], hml[0], inc0 - nc[0]);
				ldesc[64 + lane] = pack(rdst[1] + rL[1], roff[1], hml[1], inc1 - nc[1]);
				const int32_t lo = min(chunk_owner2(V, inc0, nc[0], inc1, nc[1], 0), 127);
				const uint64_t dd = ldesc[lo];
				const int32_t od = ob0 + int32_t(dd & 0xffffu);
				const int32_t ooff = int32_t((dd >> 16) & 0xffffu), oml = int32_t((dd >> 32) & 0xffffu);
				const int32_t k = 1 + lane - int32_t(dd >> 48);
				if (lane < tot) {
					rpd = od + 16 * k;
					rpn = min(16, oml - 16 * k);
					__builtin_memcpy(&vr, ob + (od - ooff) + 16 * k, 16);
				}
				wave_lds_fence();  // ldesc / own are written again later
			}
		}

		// ---- L: literals (input ring -> window), first pieces in-lane, the
		// rest of both rounds dealt
		{
#pragma unroll
			for (int r = 0; r < RMAX; ++r)
				if (rL[r] > 0)
					ostore(V, rdst[r], fetch16(S, rlit[r]), min(16, rL[r]));
			const int32_t nc0 = rL[0] > 16 ? (rL[0] - 1) >> 4 : 0;
			const int32_t nc1 = rL[1] > 16 ? (rL[1] - 1) >> 4 : 0;
			if (__any(nc0 > 0 || nc1 > 0)) {
				const int32_t inc0 = wave_incl_scan(nc0);
				const int32_t tot0 = __shfl(inc0, 63);
				const int32_t inc1 = tot0 + wave_incl_scan(nc1);
				const int32_t tot = __shfl(inc1, 63);
				auto pack = [&](int32_t lit, int32_t dst, int32_t Lx, int32_t excl) -> uint64_t {
					return uint64_t(uint16_t(lit - base)) | (uint64_t(uint16_t(dst - ob0)) << 16) |
					       (uint64_t(uint16_t(Lx)) << 32) | (uint64_t(uint16_t(excl)) << 48);
				};
				uint64_t* ldesc = ldesc_of(V);
				ldesc[lane] = pack(rlit[0], rdst[0], rL[0], inc0 - nc0);
				ldesc[64 + lane] = pack(rlit[1], rdst[1], rL[1], inc1 - nc1);
				for (int32_t t0 = 0; t0 < tot; t0 += 64) {
					const int32_t t = t0 + lane;
					const int32_t lo = min(chunk_owner2(V, inc0, nc0, inc1, nc1, t0), 127);
					const uint64_t dd = ldesc[lo];
					const int32_t lit = base + int32_t(dd & 0xffffu);
					const int32_t dst = ob0 + int32_t((dd >> 16) & 0xffffu);
					const int32_t Lx = int32_t((dd >> 32) & 0xffffu);
					const int32_t k = 1 + t - int32_t(dd >> 48);
					if (t < tot)
						ostore(V, dst + 16 * k, fetch16(S, lit + 16 * k), min(16, Lx - 16 * k));
				}
			}
		}
		wave_lds_fence();

		// ---- M: the HBM-sourced parts (sources in HBM: no order among them)
		int32_t mring[RMAX], oring[RMAX], lring[RMAX];
		__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
		if (rpn > 0)
			ostore(V, rpd, vr, rpn);
#pragma unroll
		for (int r = 0; r < RMAX; ++r) {
			mring[r] = oring[r] = lring[r] = 0;
			if (64 * r < N) {
				const int32_t mdst = rdst[r] + rL[r];
				if (hml[r] > 0)
					ostore(V, mdst, vg[r], min(16, hml[r]));
				if (rtot[r] > rfirst[r]) {  // rare: more than 64 dealt pieces; the rest now
					const int32_t nc = hml[r] > 0 ? max(((hml[r] + 15) >> 4) - 1, 0) : 0;
					const int32_t inc = wave_incl_scan(nc);
					for (int32_t t0 = rfirst[r]; t0 < rtot[r]; t0 += 64) {
						const int32_t t = t0 + lane;
						const int32_t lo = piece_owner(inc, t);
						const int32_t k = 1 + t - (__shfl(inc, lo) - __shfl(nc, lo));
						const int32_t osrc = __shfl(mdst - roff[r], lo), odst = __shfl(mdst, lo);
						const int32_t oml = __shfl(hml[r], lo);
						if (t < rtot[r]) {
							u32x4 v;
							__builtin_memcpy(&v, ob + osrc + 16 * k, 16);
							ostore(V, odst + 16 * k, v, min(16, oml - 16 * k));
						}
					}
					__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
				}
				// the window part: the match's bytes from hml on
				mring[r] = mdst + hml[r];
				oring[r] = roff[r];
				lring[r] = rml[r] - hml[r];
			}
		}
		wave_lds_fence();

		// ---- window-sourced matches, after batch j - 1's
		if (!lds_wait_ge(abort_flag, &L.tok, jb - 1)) {
			bad = true;
			break;
		}
		static_assert(RMAX == 2, "ring dealing pairs two rounds");
		if (__any(lring[0] > RING_LANE_MAX || lring[1] > RING_LANE_MAX)) {
			ring_pieces(V, mring, oring, lring, ob0, ob0 - RFLOOR2);
		} else {
#pragma unroll
			for (int r = 0; r < RMAX; ++r)
				if (64 * r < N)
					ring_lanes(V, mring[r], oring[r], lring[r], rbeg[r], rL[r], ob0 - RFLOOR2);
		}
		lds_publish(&L.tok, jb);

		// ---- flush whole 16-byte units of [ob0, oe) (the first may start
		// before ob0: batch j - 1's bytes, final since its token)
		{
			const int32_t u0 = ob0 >> 4, u1 = oe >> 4;
#pragma unroll
			for (int i = 0; i < FLUSH_ST; ++i) {
				const int32_t u = u0 + lane + 64 * i;
				if (u < u1)
					*reinterpret_cast<GLOBAL u32x4*>(ob + (u << 4)) =
					    *reinterpret_cast<const u32x4*>(&L.oring[(u << 4) & WMASK]);
			}
		}
		if (next_over) {
			// the next batch goes straight to HBM once this flush is complete
			vm_wait();
			lds_publish(&L.done[w], jb);
		}
	}
	// the last partial unit (after both waves' batches), by wave 0
	__syncthreads();
	bad = bad || lds_peek(abort_flag) != 0;
	if (!bad && tid == 0 && (o & 15))
		gstore_n(ob + (o & ~15), *reinterpret_cast<const u32x4*>(&L.oring[(o & ~15) & WMASK]), o & 15);
	return bad ? -1 : o;
}

// Independent blocks, both passes, two waves per block pipelining batches
// (pass 1: index_block2, both waves walking each chunk).  Two waves per SIMD
// (<= 256 VGPRs; the block checksum kernel's 118 still fit beside them at
// one block per SIMD).
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void k_decode_pp2(
        const uint8_t* __restrict__ frame, uint64_t frame_len, const lz4ada_block_desc* __restrict__ desc,
        uint32_t nblocks, uint8_t* __restrict__ tab_all, uint8_t* __restrict__ out,
        lz4ada_block_status* __restrict__ status)
{
	__shared__ union {
		PpLds2 d;
		IdxLds2 x;
	} U;
	if (blockIdx.x >= nblocks)
		return;
	const uint32_t b = blockIdx.x;
	const int32_t tid = int32_t(threadIdx.x), w = tid >> 6;
	index_block2(U.x, frame, frame_len, desc, b, tab_all, status);
	// the table and status this block's pass 1 wrote are read back by both waves
	vm_wait();
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
	__syncthreads();
	const lz4ada_block_desc d = desc[b];
	if (status[b].code != DS_OK)
		return;  // declined: its status says so
	if (d.flags & LZ4ADA_BLOCK_STORED) {
		const int32_t n = int32_t(d.in_len);
		int32_t c = DS_OK;
		if (n > int32_t(d.out_cap)) {
			c = DS_OUT_OVERFLOW;
		} else {  // each wave copies half
			Src S0;
			S0.in = gptr(frame) + d.in_off;
			S0.lim = reinterpret_cast<uintptr_t>(frame) + frame_len;
			const int32_t mid = (n >> 1) & ~1023;
			const int32_t c0 = w == 0 ? 0 : mid, c1 = w == 0 ? mid : n;
			if (d.flags & LZ4ADA_BLOCK_HAS_CKSUM)
				wave_literal<0>(gptr(out) + d.out_off, c0, S0, c0, c1 - c0);
			else
				wave_literal<LZ4ADA_STORED_NT>(gptr(out) + d.out_off, c0, S0, c0, c1 - c0);
		}
		if (tid == 0) {
			status[b].code = c;
			status[b].aux = 0;
			status[b].detail = 0;
			status[b].err_out_pos = 0;
			status[b].out_len = c == DS_OK ? uint32_t(n) : 0u;
		}
		return;
	}
	PpLds2& L = U.d;
	if (tid == 0) {
		L.tok = -1;  // "batches <= -1 done"
		L.staged = 0;
		L.abort_ = 0;
		L.done[0] = L.done[1] = -1;
	}
	__syncthreads();
	const int32_t len = decode_block_pp2(L, frame, frame_len, desc, b, tab_all, out);
	if (tid == 0) {
		if (len < 0) {
			status[b].code = DS_RETRY;
		} else {
			status[b].code = DS_OK;
			status[b].aux = 0;
			status[b].detail = 0;
			status[b].err_out_pos = 0;
			status[b].out_len = uint32_t(len);
		}
	}
}

}  // namespace idx

#ifdef LZ4ADA_IDX_STAMPS
extern "C" int lz4ada_idx_stamps(unsigned long long* out, int reset)
{
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(idx::g_idx_stamps),
	                        sizeof(unsigned long long) * idx::IDX_NST) != hipSuccess)
		return -1;
	if (reset) {
		unsigned long long z[idx::IDX_NST] = {};
		if (hipMemcpyToSymbol(HIP_SYMBOL(idx::g_idx_stamps), z, sizeof z) != hipSuccess)
			return -1;
	}
	return idx::IDX_NST;
}
#endif

#ifdef LZ4ADA_IDX_GATHERS
extern "C" int lz4ada_idx_gathers(unsigned long long* out, int reset)
{
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(idx::g_idx_gathers), sizeof(unsigned long long) * 4) != hipSuccess)
		return -1;
	if (reset) {
		unsigned long long z[4] = {};
		if (hipMemcpyToSymbol(HIP_SYMBOL(idx::g_idx_gathers), z, sizeof z) != hipSuccess)
			return -1;
	}
	return 4;
}
#endif

// index table: 8 records of 8 bytes per 256-byte segment, per block at
// record ((in_off >> 8) + b) * 8
size_t index_table_bytes(uint64_t frame_len, uint32_t nblocks)
{
	return ((size_t(frame_len) >> 8) + size_t(nblocks) + 2) * 64;
}

hipError_t launch_index(const uint8_t* d_frame, uint64_t frame_len, const lz4ada_block_desc* d_desc,
                        uint32_t nblocks, uint8_t* d_tab, lz4ada_block_status* d_status,
                        hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(idx::k_index, dim3(nblocks), dim3(64), 0, stream, d_frame, frame_len, d_desc,
	                   nblocks, d_tab, d_status);
	return hipGetLastError();
}

hipError_t launch_decode_idx_tab(const uint8_t* d_frame, uint64_t frame_len,
                                 const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                 const uint8_t* d_tab, uint8_t* d_out,
                                 lz4ada_block_status* d_status, int mode, hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	if (mode == 6) {  // pass 2, linked layout, literals as zeros (k_decode_idx_zl)
		hipLaunchKernelGGL(idx::k_decode_idx_zl, dim3(nblocks), dim3(64), 0, stream, d_frame, frame_len,
		                   d_desc, nblocks, const_cast<uint8_t*>(d_tab), d_out, d_status);
		return hipGetLastError();
	}
	if (mode == 2) {  // pass 2, linked layout (k_decode_idx_lk: quirk D1 emulated)
		hipLaunchKernelGGL(idx::k_decode_idx_lk, dim3(nblocks), dim3(64), 0, stream, d_frame, frame_len,
		                   d_desc, nblocks, const_cast<uint8_t*>(d_tab), d_out, d_status);
		return hipGetLastError();
	}
	if (mode == 5 || mode == 4) {  // both passes, two waves per block pipelining batches (k_decode_pp2;
		                           // 4: round 4's k_decode_idx2, retired -- its callers get pp2)
		hipLaunchKernelGGL(idx::k_decode_pp2, dim3(nblocks), dim3(128), 0, stream, d_frame, frame_len,
		                   d_desc, nblocks, const_cast<uint8_t*>(d_tab), d_out, d_status);
		return hipGetLastError();
	}
	hipLaunchKernelGGL(idx::k_decode_idx, dim3(mode == 1 ? 1 : nblocks), dim3(64), 0, stream, d_frame,
	                   frame_len, d_desc, nblocks, const_cast<uint8_t*>(d_tab), d_out, d_status, mode);
	return hipGetLastError();
}

// The fused launch for independent blocks.  One wave per block
// (k_decode_idx, mode 3) while the blocks fill the chip's SIMDs twice; two
// waves per block pipelining batches (k_decode_pp2, mode 5) for at most 4
// blocks per CU (measured, docs/DESIGN_LOG.md §3: 1,024 x 4 MiB mixed 12.0
// -> 8.7 ms, but at 2,048 blocks 13.3 -> 18.0 ms).  LZ4ADA_IDX_WAVES=1 / p
// (or 2, which meant the retired k_decode_idx2) forces one or the other.
int idx_fused_mode(uint32_t nblocks)
{
	static const int forced = [] {
		const char* e = getenv("LZ4ADA_IDX_WAVES");
		return e ? (e[0] == '1' ? 3 : ((e[0] == '2' || e[0] == 'p') ? 5 : 0)) : 0;
	}();
	if (forced)
		return forced;
	int dev = 0, cus = 256;
	if (hipGetDevice(&dev) == hipSuccess)
		(void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
	return nblocks <= uint32_t(4 * cus) ? 5 : 3;
}

const char* idx_fused_kernel_name(uint32_t nblocks)
{
	const int m = idx_fused_mode(nblocks);
	return m == 5 ? "k_decode_pp2" : "k_decode_idx";
}

hipError_t launch_decode_idx(const uint8_t* d_frame, uint64_t frame_len,
                             const lz4ada_block_desc* d_desc, uint32_t nblocks, uint8_t* d_out,
                             lz4ada_block_status* d_status, hipStream_t stream, int linked)
{
	if (nblocks == 0)
		return hipSuccess;
	void* tab = nullptr;
	hipError_t err = hipMallocAsync(&tab, index_table_bytes(frame_len, nblocks), stream);
	if (err != hipSuccess)
		return err;
	const bool split = linked == -4;  // the two passes as two launches (diagnostic: per-pass counters)
	if (linked <= 0 && !split) {  // both passes in one launch (-1: one wave per block, -2: two, -3: pipelined pair)
		const int mode = linked == -1 ? 3 : (linked == -2 ? 4 : (linked == -3 ? 5 : idx_fused_mode(nblocks)));
		err = launch_decode_idx_tab(d_frame, frame_len, d_desc, nblocks,
		                            static_cast<const uint8_t*>(tab), d_out, d_status, mode, stream);
	} else {
		err = launch_index(d_frame, frame_len, d_desc, nblocks, static_cast<uint8_t*>(tab), d_status,
		                   stream);
		if (err == hipSuccess)
			err = launch_decode_idx_tab(d_frame, frame_len, d_desc, nblocks,
			                            static_cast<const uint8_t*>(tab), d_out, d_status, split ? 0 : linked,
			                            stream);
	}
	const hipError_t e2 = hipFreeAsync(tab, stream);
	return err != hipSuccess ? err : e2;
}

}  // namespace lz4ada
