// lz4ada_kernels.hip -- gfx950 kernels of the MI355X LZ4Ada decompressor.
//
// Replaces the reference's hot path (lib/lz4ada.adb):
//   Decompress_Full_Block / Decompress_Sequence      :716-788
//   Write_Output (8-byte wild copy)                  :790-824
//   Output_With_History (overlap-safe match copy)    :845-904
//
// (XXH32: lz4ada_xxh32.hip.)  Design (DESIGN.md has the long form):
//  * k_decode_pc -- two waves per block (producer parses windows of
//    sequences speculatively, consumer copies them); the bulk path's
//    decoder for the blocks the index-driven decoder (lz4ada_idx.hip) and
//    the literal-heavy decoder (lz4ada_sparse.hip) decline, and the lone
//    facade's small blocks.
//    Long or unusual tokens (multi-byte length extensions, anything
//    malformed) go through a wave-cooperative one-token path that also
//    produces the precise error.
//  * k_serial_block -- reference-exact single-lane emulation of one block
//    on a device mirror of the caller's Buffer (Output_Pos wrap, history,
//    8-byte wild-copy overshoot and its D1 side effect).  Used by the
//    streaming Update facade and by the bulk path's exact fallback.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <utility>

#include "lz4ada_internal.h"
#include "lz4ada_dev.h"

namespace lz4ada {


// --------------------------------------------------------- block decoder

constexpr int INB = 8192;        // compressed staging ring per wave (LDS)
constexpr int INB_MASK = INB - 1;
constexpr int WIN = 256;         // speculative parse window (4 candidates per lane)
constexpr int LOOK = WIN + 288;  // bytes past s a window's tokens may touch
constexpr int OUTB = 4096;       // batch output bytes
constexpr int MAXTOK = 64;       // tokens per batch (one per lane)
constexpr int WTOK = 64;         // tokens taken from one window (one per lane)
constexpr int BIG = 1024;        // longer sequences take the one-token path
constexpr int SPAN = 2048;       // compressed bytes a batch may span
constexpr int STAGE_AHEAD = 2112;  // staged bytes kept ahead of the chain (>= 64 + LOOK, > BIG)
static_assert(STAGE_AHEAD >= 64 + LOOK && STAGE_AHEAD > BIG + 16, "staging lead too short");
// ring occupancy bound: batch span + one token's advance + lead + chunk
static_assert(SPAN + BIG + 64 + STAGE_AHEAD + 1024 + 16 <= INB, "input ring too small");

enum TokKind : int { TK_NORMAL = 0, TK_LAST = 1, TK_COMPLEX = 2, TK_ERR = 3 };

// Diagnostic build only (make stamps -> liblz4ada_hip_stamps.so): per-phase
// s_memtime sums of the decoders' phases, read back by tools/stamps.py.  The
// product library is built without LZ4ADA_STAMPS and executes no stamp.
enum StampPhase { SP_STAGE, SP_CAND, SP_DOUBLE, SP_SELECT, SP_LIT, SP_MATCH, SP_FLUSH, SP_ONE,
	          SP_WAIT, SP_DEP, SP_BATCHES, SP_WINDOWS, SP_TOKENS, SP_ROUNDS, SP_N };
#ifdef LZ4ADA_STAMPS
__device__ unsigned long long g_stamps[SP_N];
#define STAMP_DECL uint64_t st_acc[SP_N] = {}; uint64_t st_t = __builtin_amdgcn_s_memtime()
#define STAMP(ph)                                                                  \
	do {                                                                       \
		asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");        \
		const uint64_t _t = __builtin_amdgcn_s_memtime();                  \
		st_acc[ph] += _t - st_t;                                           \
		st_t = _t;                                                         \
	} while (0)
#define STAMP_COUNT(ph, v) (st_acc[ph] += uint64_t(v))
#define STAMP_PARAM , uint64_t(&st_acc)[SP_N], uint64_t& st_t
#define STAMP_ARGS , st_acc, st_t
#define STAMP_FLUSH()                                                              \
	do {                                                                       \
		if (lane_id() == 0)                                                \
			for (int _i = 0; _i < SP_N; ++_i)                          \
				atomicAdd(&g_stamps[_i], (unsigned long long)st_acc[_i]); \
	} while (0)
#else
#define STAMP_DECL
#define STAMP(ph)
#define STAMP_COUNT(ph, v)
#define STAMP_PARAM
#define STAMP_ARGS
#define STAMP_FLUSH()
#endif

// Sum of a length extension (Process_Variable_Length, lz4ada.adb:724-735)
// starting at block-relative p, 64 bytes per step.  Returns false when the
// block ends first (D4).  Whole-wave, uniform.
__device__ bool wave_ext_sum(cg8* in, int64_t n, int64_t& p, int64_t& sum)
{
	const uint32_t lane = lane_id();
	for (;;) {
		const int64_t q = p + lane;
		const bool valid = q < n;
		const uint32_t byte = valid ? in[q] : 0u;
		const uint64_t stop = __ballot(valid && byte != 255u);
		const uint64_t inval = __ballot(!valid);
		if (stop) {
			const int first = __ffsll((long long)stop) - 1;
			if (inval && (__ffsll((long long)inval) - 1) < first)
				return false;
			const uint32_t fb = uint32_t(__shfl(int(byte), first));
			sum += int64_t(255) * first + fb;
			p += first + 1;
			return true;
		}
		if (inval)
			return false;
		sum += int64_t(255) * 64;
		p += 64;
	}
}

// Wave-cooperative copy of n bytes global -> global (no overlap).
__device__ void wave_copy(g8* __restrict__ dst, cg8* __restrict__ src, int64_t n)
{
	const uint32_t lane = lane_id();
	int64_t head = int64_t((16 - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u);
	if (head > n)
		head = n;
	if (int64_t(lane) < head)
		dst[lane] = src[lane];
	dst += head;
	src += head;
	n -= head;
	const int64_t nv = n / 16;
	for (int64_t i = lane; i < nv; i += 64) {
		cg8* sp = src + 16 * i;
		u32x4 v;
		v.x = ld32u_cached(sp);
		v.y = ld32u_cached(sp + 4);
		v.z = ld32u_cached(sp + 8);
		v.w = ld32u_cached(sp + 12);
		*reinterpret_cast<GLOBAL u32x4*>(dst + 16 * i) = v;
	}
	for (int64_t i = nv * 16 + lane; i < n; i += 64)
		dst[i] = src[i];
}

// One token at block-relative s, wave-cooperative, global -> global.
// Handles every shape, including the malformed ones (exact statuses).
// Returns false with st filled on error; advances s and o.
// Every global store and LDS op of this wave done (one-token path; the
// path is run by a single wave, also inside the two-wave decoder, so it
// must not use a workgroup barrier).
__device__ __forceinline__ void wave_mem_fence()
{
	asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// hist: output bytes readable right before the block's slot (0 for
// independent blocks; 65535 in the linked-frame layout of lz4ada_linked.hip).
// d1: set when a match with offset >= D1_OFF reads before the block start
// (the only matches the reference's wild-copy overshoot can corrupt, D1).
__device__ bool one_token(cg8* __restrict__ in, int64_t n, g8* __restrict__ ob,
                          int64_t cap, int64_t& s, int64_t& o, lz4ada_block_status& st,
                          int32_t hist, bool& d1)
{
	const uint32_t lane = lane_id();
	int64_t p = s;
	const uint32_t tk = in[p];
	int64_t L = tk >> 4, M = tk & 15;
	++p;
	if (L == 15 && !wave_ext_sum(in, n, p, L)) {
		st.code = DS_TRUNCATED;
		st.err_out_pos = o;
		return false;
	}
	if (L > 0) {
		if (o + L > cap) {
			st.code = DS_OUT_OVERFLOW;
			st.err_out_pos = o;
			return false;
		}
		if (p + L > n) {  // literal run overruns the block
			st.code = (M != 0) ? DS_ML_AFTER_LIT : DS_LIT_OVERRUN;
			st.aux = int32_t(M);
			st.err_out_pos = o + L;
			return false;
		}
		wave_copy(ob + o, in + p, L);
		o += L;
		p += L;
	}
	if (p >= n) {
		if (M != 0) {
			st.code = DS_ML_AFTER_LIT;
			st.aux = int32_t(M);
			st.err_out_pos = o;
			return false;
		}
		s = p;
		wave_mem_fence();
		return true;
	}
	if (p + 1 >= n) {
		st.code = DS_TRUNCATED;
		st.err_out_pos = o;
		return false;
	}
	const int64_t off = int64_t(in[p]) | (int64_t(in[p + 1]) << 8);
	p += 2;
	if (off == 0) {
		st.code = DS_OFFSET0;
		st.err_out_pos = o;
		return false;
	}
	if (M == 15 && !wave_ext_sum(in, n, p, M)) {
		st.code = DS_TRUNCATED;
		st.err_out_pos = o;
		return false;
	}
	const int64_t ml = M + 4;
	const int64_t q0 = o - off;
	if (q0 < 0 && off >= D1_OFF)
		d1 = true;
	if (q0 < -int64_t(hist)) {
		st.code = DS_PRE_BLOCK_REF;
		st.detail = q0;
		st.err_out_pos = o;
		return false;
	}
	if (o + ml > cap) {
		st.code = DS_OUT_OVERFLOW;
		st.err_out_pos = o;
		return false;
	}
	wave_mem_fence();  // literals above are visible to every lane
	if (off >= ml) {
		wave_copy(ob + o, ob + q0, ml);
	} else {
		// Overlap: byte k repeats source byte (k mod off); every source
		// byte precedes the match, so all lanes run at once.
		const uint32_t offu = uint32_t(off);
		uint32_t k = lane, r = lane % offu;
		const uint32_t step = 64u % offu;
		for (; int64_t(k) < ml; k += 64) {
			ob[o + k] = ob[q0 + r];
			r += step;
			if (r >= offu)
				r -= offu;
		}
	}
	o += ml;
	s = p;
	wave_mem_fence();
	return true;
}

// ---------------------------------------------------------- V3 decoder
//
// One wavefront per block.  State: s = block-relative compressed position
// of the token chain, o = block-relative output already flushed to HBM.
//
//  1. stage: compressed bytes live in an LDS ring (16-byte global chunks,
//     1 KiB per refill, the next refill already in flight in registers).
//  2. parse window [s, s+64): every lane evaluates a token at s + lane
//     (branch-free, two LDS reads), ds_bpermute pointer doubling finds the
//     chain from s, lane j picks up the j-th token.  Tokens accumulate into
//     a batch of up to 64 (one per lane) in LDS records.
//  3. copy the batch into an LDS output buffer, lane per token, 16 bytes
//     per step: literals from the ring, matches from HBM (pre-batch) or the
//     buffer (in-batch, in dependency rounds), then flush with 16-byte
//     stores.
//  4. anything unusual -> one_token (wave-cooperative, exact statuses).

constexpr int MIRROR = 16;

struct Cand {
	int32_t L, lit, off, ml, next, kind;
};

__device__ __forceinline__ uint32_t lds_u16(const uint8_t* p)
{
	uint16_t v;
	__builtin_memcpy(&v, p, 2);
	return v;
}
__device__ __forceinline__ uint32_t lds_u32(const uint8_t* p)
{
	uint32_t v;
	__builtin_memcpy(&v, p, 4);
	return v;
}

// Branch-free token parse at block-relative c from the staging ring
// (Decompress_Sequence, lz4ada.adb:737-777).  Only single-byte length
// extensions are resolved here; longer ones are TK_COMPLEX, malformed
// shapes TK_ERR -- both go to one_token, which reports them exactly.
__device__ __forceinline__ Cand parse_cand(const uint8_t* inb, int32_t mis, int32_t c, int32_t n)
{
	const uint32_t t2 = lds_u16(inb + ((c + mis) & INB_MASK));
	const int32_t tk = int32_t(t2 & 0xffu), e1 = int32_t(t2 >> 8);
	const int32_t L0 = tk >> 4, M0 = tk & 15;
	const bool x1 = (L0 == 15), x2 = (M0 == 15);
	const int32_t L = L0 + (x1 ? e1 : 0);
	const int32_t lit = c + 1 + (x1 ? 1 : 0);
	const int32_t p = lit + L;  // offset position
	const uint32_t w = lds_u32(inb + ((p + mis) & INB_MASK));
	const int32_t off = int32_t(w & 0xffffu), e2 = int32_t((w >> 16) & 0xffu);
	const int32_t ml = M0 + 4 + (x2 ? e2 : 0);
	const int32_t next = p + 2 + (x2 ? 1 : 0);
	const bool last = (p == n) && (M0 == 0);
	const bool err = (c >= n) || (x1 && c + 1 >= n) || (p > n) || (p == n && M0 != 0) ||
	                 (p < n && (p + 1 >= n || off == 0 || (x2 && p + 2 >= n)));
	const bool cx = (x1 && e1 == 255) || (x2 && e2 == 255);
	Cand t;
	t.L = L;
	t.lit = lit;
	t.off = off;
	t.ml = ml;
	t.next = next;
	t.kind = err ? TK_ERR : (cx ? TK_COMPLEX : (last ? TK_LAST : TK_NORMAL));
	if (last) {
		t.ml = 0;
		t.off = 0;
		t.next = n;
	}
	if (x1 && e1 == 255)  // L, p and everything after are meaningless
		t.kind = (c + 1 >= n) ? TK_ERR : TK_COMPLEX;
	return t;
}

// parse_cand for a token at least 2 x 272 bytes before the block end, where
// only a zero offset or a 255 extension byte (TK_ERR here; one_token
// classifies it exactly) can make it other than TK_NORMAL.  Branch-free.
__device__ __forceinline__ Cand parse_cand_far(const uint8_t* inb, int32_t mis, int32_t c)
{
	const uint32_t t2 = lds_u16(inb + ((c + mis) & INB_MASK));
	const bool x1 = (t2 & 0xf0u) == 0xf0u, x2 = (t2 & 15u) == 15u;
	const int32_t L = int32_t((t2 >> 4) & 15u) + int32_t(x1 ? (t2 >> 8) : 0u);
	const int32_t lit = c + 1 + (x1 ? 1 : 0);
	const int32_t p = lit + L;
	const uint32_t w = lds_u32(inb + ((p + mis) & INB_MASK));
	const uint32_t e2 = (w >> 16) & 0xffu;
	Cand t;
	t.L = L;
	t.lit = lit;
	t.off = int32_t(w & 0xffffu);
	t.ml = int32_t(t2 & 15u) + 4 + int32_t(x2 ? e2 : 0u);
	t.next = p + 2 + (x2 ? 1 : 0);
	const bool ok = (t.off != 0) & !(x1 & ((t2 >> 8) == 255u)) & !(x2 & (e2 == 255u));
	t.kind = ok ? TK_NORMAL : TK_ERR;
	return t;
}

// Wave-uniform value: every lane holds the same; tell the compiler so it
// keeps the serial parse in SGPRs with scalar branches.
__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Uniform (scalar) parse of the token at s from the staging ring, with
// length extensions of any size, for tokens the speculative window cannot
// take (long literal runs).  Returns false when the token is malformed or
// not fully staged; one_token then handles it.
__device__ __forceinline__ bool parse_serial(const uint8_t* inb, int32_t mis, int32_t s, int32_t n,
                                             int32_t hi, Cand& t)
{
	s = uni(s);
	n = uni(n);
	hi = uni(hi);
	mis = uni(mis);
	if (s >= n || s + 2 > hi)
		return false;
	const int32_t tk = uni(inb[(s + mis) & INB_MASK]);
	int32_t L = tk >> 4, M = tk & 15, p = s + 1;
	bool ok = true;
	if (L == 15) {
		int32_t e = 255;
		while (ok && e == 255) {
			if (p >= n || p >= hi) {
				ok = false;
			} else {
				e = uni(inb[(p + mis) & INB_MASK]);
				++p;
				L += e;
			}
		}
	}
	const int32_t lit = p;
	p += L;
	int32_t off = 0, ml = 0, next = n, kind = TK_ERR;
	if (ok) {
		if (p >= n) {
			if (p == n && M == 0 && p <= hi)
				kind = TK_LAST;
		} else if (p + 3 <= hi && p + 1 < n) {
			off = uni(inb[(p + mis) & INB_MASK]) | (uni(inb[(p + 1 + mis) & INB_MASK]) << 8);
			p += 2;
			if (off != 0) {
				bool okm = true;
				if (M == 15) {
					int32_t e = 255;
					while (okm && e == 255) {
						if (p >= n || p >= hi) {
							okm = false;
						} else {
							e = uni(inb[(p + mis) & INB_MASK]);
							++p;
							M += e;
						}
					}
				}
				if (okm) {
					ml = M + 4;
					next = p;
					kind = TK_NORMAL;
				}
			}
		}
	}
	t.lit = lit;
	t.L = L;
	t.off = kind == TK_NORMAL ? off : 0;
	t.ml = kind == TK_NORMAL ? ml : 0;
	t.next = next;
	t.kind = kind;
	return kind == TK_NORMAL || kind == TK_LAST;
}

// Index of the last batch token whose output starts at or before x
// (tokens live one per lane, ts ascending).
__device__ __forceinline__ int32_t owner_of(int32_t ts_reg, int32_t nb, int32_t x)
{
	int32_t lo = 0, hi = nb - 1;
#pragma unroll
	for (int i = 0; i < 6; ++i) {
		const int32_t mid = (lo + hi + 1) >> 1;
		const int32_t t = __shfl(ts_reg, mid);
		if (t <= x)
			lo = mid;
		else
			hi = mid - 1;
	}
	return lo;
}

// Cross-lane hand-off through LDS inside one wavefront: LDS executes a
// wave's operations in order, so only the compiler must not reorder.

// Stage compressed bytes so that block-relative [lo, need) is in the ring.
// `pf` holds the 1 KiB chunk at `hi`, loaded ahead; writing it to LDS is
// the first use, so its load latency overlaps the work since the last call.
__device__ __forceinline__ u32x4 load_chunk(cg8* in, uintptr_t lim_addr, int32_t at)
{
	const uint32_t lane = lane_id();
	const uintptr_t ga = reinterpret_cast<uintptr_t>(in) + uintptr_t(intptr_t(at)) + 16u * lane;
	u32x4 v;
	if (ga + 16 <= lim_addr) {
		v = *reinterpret_cast<const GLOBAL u32x4*>(ga);
	} else {
		uint8_t t[16];
		for (int i = 0; i < 16; ++i)
			t[i] = (ga + i < lim_addr) ? *reinterpret_cast<cg8*>(ga + i) : 0;
		__builtin_memcpy(&v, t, 16);
	}
	return v;
}

template <class LdsT>
__device__ __forceinline__ void stage_to(LdsT& L, cg8* in, uintptr_t lim_addr, int32_t mis,
                                         int32_t& hi, u32x4& pf0, u32x4& pf1, int32_t lo,
                                         int32_t need)
{
	const uint32_t lane = lane_id();
	if (hi < lo) {  // jumped ahead (one-token path): restart the stream at lo
		hi = ((lo + mis) & ~15) - mis;
		pf0 = load_chunk(in, lim_addr, hi);
		pf1 = load_chunk(in, lim_addr, hi + 1024);
	}
	bool any = false;
	while (hi < need) {
		const uint32_t idx = uint32_t(hi + mis + 16 * int32_t(lane)) & INB_MASK;
		*reinterpret_cast<u32x4*>(&L.inb[idx]) = pf0;
		if (idx == 0)
			*reinterpret_cast<u32x4*>(&L.inb[INB]) = pf0;  // mirror for wrap-free reads
		hi += 1024;
		pf0 = pf1;
		pf1 = load_chunk(in, lim_addr, hi + 1024);  // two chunks in flight
		any = true;
	}
	if (any)
		wave_lds_fence();
}

// Exact-length store of n (0..16) bytes of v to LDS.

// ------------------------------------------- producer/consumer decoder
// k_decode_pc: the per-wave decoder split over two waves of one workgroup
// per block.  Wave 0 (producer) stages the compressed stream and parses
// windows into batches of sequence records; wave 1 (consumer) copies the
// previous batch (literals, dependency-ordered matches, 16-byte flush to
// HBM).  The two run in lockstep, one barrier per step, with the records
// double-buffered, so a step costs max(parse, copy) instead of their sum,
// and each CU holds 16 waves instead of 8.  Anything unusual goes through
// the same one-token path, run by the producer once every batch is out.

constexpr int PC_BIG = BIG;            // longer sequences take the one-token path
constexpr int PC_SPAN = SPAN;          // compressed bytes a batch may span
constexpr int PC_STAGE_AHEAD = STAGE_AHEAD;
#ifndef LZ4ADA_PC_SER_MIN
#define LZ4ADA_PC_SER_MIN 64
#endif
// sequences averaging at least this many compressed bytes are parsed one at
// a time (scalar); denser streams use the speculative window.  The scalar
// parse is LDS-latency bound (~1300 cycles per sequence under load, against
// ~420 for the window on mixed data), so only long literal runs take it.
constexpr int PC_SER_MIN = LZ4ADA_PC_SER_MIN;
#ifndef LZ4ADA_PC_ANCH
#define LZ4ADA_PC_ANCH 3
#endif
// window walk anchors every 2^PC_ANCH sequences
constexpr int PC_ANCH = LZ4ADA_PC_ANCH;
// The ring also holds the batch the consumer is copying: the producer ends
// its batch early (or waits a step) rather than stage over those bytes.

constexpr int PC_OUTX = 16 + OUTB + 32;
static_assert(PC_OUTX % 16 == 0, "outx is read as aligned 16-byte pairs");

#ifndef LZ4ADA_PC_SLOTS
#define LZ4ADA_PC_SLOTS 4
#endif
// record slots between producer and consumer (a power of two)
constexpr int PC_SLOTS = LZ4ADA_PC_SLOTS;
static_assert((PC_SLOTS & (PC_SLOTS - 1)) == 0 && PC_SLOTS >= 2, "PC_SLOTS: power of two >= 2");

struct alignas(16) PcLds {
	uint8_t inb[INB + MIRROR];
	uint8_t outx[PC_OUTX];  // [0, 16): the 16 output bytes before the batch; batch at 16
	int32_t r_tstart[PC_SLOTS][MAXTOK];
	int32_t r_L[PC_SLOTS][MAXTOK];
	int32_t r_lit[PC_SLOTS][MAXTOK];
	int32_t r_off[PC_SLOTS][MAXTOK];
	int32_t r_ml[PC_SLOTS][MAXTOK];
	int32_t m_nb[PC_SLOTS], m_blen[PC_SLOTS], m_o[PC_SLOTS], m_bcomp0[PC_SLOTS];
	int32_t full[PC_SLOTS];  // 1: the slot's records wait for (or are being copied by) the consumer
	int32_t pdone;           // producer finished: no slot will be filled again
	int32_t tail_end;        // block output position of outx[16] (consumer)
};

__device__ __forceinline__ int32_t lds_poll(const int32_t* p)
{
	return *reinterpret_cast<const volatile int32_t*>(p);
}

// 8 ring bytes at block-relative x as a wave-uniform u64: three aligned
// dword reads (the ring's 16-byte mirror covers the wrap) and a shift.
__device__ __forceinline__ uint64_t ring_u64s(const uint8_t* inb, int32_t mis, int32_t x)
{
	const uint32_t a = uint32_t(x + mis) & INB_MASK;
	const uint32_t* w = reinterpret_cast<const uint32_t*>(inb + (a & ~3u));
	const uint32_t w0 = uint32_t(uni(int32_t(w[0])));
	const uint32_t w1 = uint32_t(uni(int32_t(w[1])));
	const uint32_t w2 = uint32_t(uni(int32_t(w[2])));
	const uint32_t sh = 8u * (a & 3u);
	const uint64_t lo = uint64_t(w0) | (uint64_t(w1) << 32);
	return sh ? (lo >> sh) | (uint64_t(w2) << (64u - sh)) : lo;
}

// parse_serial for the common shapes with two dependent ring reads (token
// and <= 1 extension byte, then offset and <= 1 extension byte); anything
// else -- longer extensions, the block end, malformed data, bytes not yet
// staged -- is left to parse_serial, so the result is the same.
__device__ __forceinline__ bool parse_fast(const uint8_t* inb, int32_t mis, int32_t s, int32_t n,
                                           int32_t hi, Cand& t)
{
	s = uni(s);
	n = uni(n);
	hi = uni(hi);
	if (s + 16 > hi || s + 16 > n)
		return parse_serial(inb, mis, s, n, hi, t);
	const uint64_t A = ring_u64s(inb, mis, s);
	const int32_t tk = int32_t(A & 0xffu);
	int32_t L = tk >> 4, p = s + 1;
	const int32_t e1 = int32_t((A >> 8) & 0xffu);
	if (L == 15) {
		if (e1 == 255)
			return parse_serial(inb, mis, s, n, hi, t);
		L += e1;
		++p;
	}
	const int32_t lit = p;
	p += L;
	if (p + 8 > n || p + 8 > hi)
		return parse_serial(inb, mis, s, n, hi, t);
	const uint64_t B = (p + 3 <= s + 8) ? (A >> (8 * (p - s))) : ring_u64s(inb, mis, p);
	const int32_t off = int32_t(B & 0xffffu), e2 = int32_t((B >> 16) & 0xffu);
	int32_t M = tk & 15, next = p + 2;
	if (off == 0 || (M == 15 && e2 == 255))
		return parse_serial(inb, mis, s, n, hi, t);
	if (M == 15) {
		M += e2;
		++next;
	}
	t.lit = lit;
	t.L = L;
	t.off = off;
	t.ml = M + 4;
	t.next = next;
	t.kind = TK_NORMAL;
	return true;
}

// Window successor tables hold one byte per position, four positions per
// lane (position k: lane k & 63, byte k >> 6; 0 = none).  Entry of table
// `t` for position p, for every lane at once (p < WIN).
__device__ __forceinline__ uint32_t win_look(uint32_t t, uint32_t p)
{
	const uint32_t w = uint32_t(__builtin_amdgcn_ds_bpermute(int32_t((p & 63u) << 2), int32_t(t)));
	return (w >> (8 * ((p >> 6) & 3u))) & 0xffu;
}
// ... where p is itself a table entry (0 = none stays none)
__device__ __forceinline__ uint32_t win_next(uint32_t t, uint32_t p)
{
	const uint32_t v = win_look(t, p);
	return p ? v : 0u;
}

// Consumer: copy batch `c` (records, output at o) into outb and flush it.
#define PC_STORE_N(p, v, n) lds_store_n((p), (v), (n))
#define PC_LOAD16(dst, p) __builtin_memcpy((dst), (p), 16)

__device__ __forceinline__ void pc_copy_batch(PcLds& L, int c, int32_t mis, g8* __restrict__ ob,
                                              int32_t hist STAMP_PARAM)
{
	const int lane = int(lane_id());
	const int32_t nb = L.m_nb[c], blen = L.m_blen[c], o = L.m_o[c];
	uint8_t* const outb = L.outx + 16;
	if (L.tail_end != o) {  // first batch, or output written by the one-token path
		if (lane < 16)
			L.outx[lane] = (o - 16 + lane >= -hist) ? ob[o - 16 + lane] : 0;
		if (lane == 0)
			L.tail_end = o;
		wave_mem_fence();
	}
	const bool tl = lane < nb;
	const int32_t ts = tl ? L.r_tstart[c][lane] : 0;
	const int32_t tL = tl ? L.r_L[c][lane] : 0;
	const int32_t tlit = tl ? L.r_lit[c][lane] : 0;
	const int32_t toff = tl ? L.r_off[c][lane] : 1;
	const int32_t tml = tl ? L.r_ml[c][lane] : 0;
	const int32_t d0 = ts + tL;        // batch-relative
	const int32_t q0 = o + d0 - toff;  // block-relative source
	u32x4 pv0 = {0, 0, 0, 0}, pv1 = {0, 0, 0, 0};
	const bool pre0 = tl && tml > 0 && toff >= 16 && q0 + 16 <= o;
	const bool pre1 = pre0 && tml > 16 && q0 + 32 <= o;
	if (pre0)
		__builtin_memcpy(&pv0, (const uint8_t*)(ob + q0), 16);
	if (pre1)
		__builtin_memcpy(&pv1, (const uint8_t*)(ob + q0 + 16), 16);
	constexpr int32_t LONG = 48;
	if (tL <= LONG) {
		for (int32_t i = 0; i < tL; i += 16) {
			u32x4 v;
			PC_LOAD16(&v, &L.inb[(tlit + i + mis) & INB_MASK]);
			PC_STORE_N(&outb[ts + i], v, tL - i);
		}
	}
	for (uint64_t lm = __ballot(tl && tL > LONG); lm; lm &= lm - 1) {
		const int k = __ffsll((long long)lm) - 1;
		const int32_t Lk = __shfl(tL, k), litk = __shfl(tlit, k), tsk = __shfl(ts, k);
		for (int32_t i = 16 * lane; i < Lk; i += 1024) {
			u32x4 v;
			PC_LOAD16(&v, &L.inb[(litk + i + mis) & INB_MASK]);
			PC_STORE_N(&outb[tsk + i], v, Lk - i);
		}
	}
	wave_lds_fence();
	STAMP(SP_LIT);
	const int32_t sb = (q0 + tml < o + d0 ? q0 + tml : o + d0) - o;
	const int32_t sa = (q0 - o > 0) ? q0 - o : 0;
	const bool inbatch = tl && tml > 0 && sb > 0;
	uint64_t dep = 0;
	if (__ballot(inbatch)) {
		const int32_t ka = owner_of(ts, nb, inbatch ? sa : 0);
		const int32_t kb = owner_of(ts, nb, inbatch ? sb - 1 : 0);
		const int32_t d0_ka = __shfl(d0, ka), ml_ka = __shfl(tml, ka);
		const int32_t d0_kb = __shfl(d0, kb), ml_kb = __shfl(tml, kb);
		if (inbatch) {
			if (kb > ka + 1)
				dep = ((1ull << kb) - 1) & ~((2ull << ka) - 1);
			if (ml_ka > 0 && d0_ka < sb && d0_ka + ml_ka > sa)
				dep |= 1ull << ka;
			if (kb != ka && ml_kb > 0 && d0_kb < sb)
				dep |= 1ull << kb;
			dep &= (1ull << lane) - 1;
		}
	}
	STAMP(SP_DEP);
	bool pend = tl && tml > 0;
	for (int guard = 0;; ++guard) {
		const uint64_t pm = __ballot(pend);
		if (!pm)
			break;
		const bool ready = pend && (!(pm & dep) || guard > MAXTOK);
		if (ready) {
			if (toff >= 16) {
				for (int32_t i = 0; i < tml; i += 16) {
					const int32_t sp = q0 + i;
					const int32_t nn = tml - i < 16 ? tml - i : 16;
					u32x4 v;
					if (i == 0 && pre0) {
						v = pv0;
					} else if (i == 16 && pre1) {
						v = pv1;
					} else if (sp >= o - 16) {  // this batch or the tail before it
						v = ld16u(L.outx, uint32_t(sp - o + 16), PC_OUTX);
					} else {
						__builtin_memcpy(&v, (const uint8_t*)(ob + sp), 16);
					}
					PC_STORE_N(&outb[d0 + i], v, nn);
				}
			} else {
				// the toff (< 16) source bytes are in this batch or in the
				// 16-byte tail of the previous one: a periodic fill from LDS
				const u32x4 sv = ld16u(L.outx, uint32_t(q0 - o + 16), PC_OUTX);
				u32x4 pv;
				int32_t width, stp;
				make_pattern(uint64_t(sv.x) | (uint64_t(sv.y) << 32),
				             uint64_t(sv.z) | (uint64_t(sv.w) << 32), toff, pv, width, stp);
				for (int32_t k = 0; k < tml; k += stp)
					PC_STORE_N(&outb[d0 + k], pv, tml - k < width ? tml - k : width);
			}
		}
		pend = pend && !ready;
		wave_lds_fence();
		STAMP_COUNT(SP_ROUNDS, 1);
	}
	STAMP(SP_MATCH);
	{
		g8* dst = ob + o;
		const int32_t head = int32_t((16 - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u);
		const int32_t h = head < blen ? head : blen;
		if (lane < h)
			dst[lane] = outb[lane];
		const int32_t nv = (blen - h) / 16;
		for (int32_t i = lane; i < nv; i += 64) {
			u32x4 v;
			__builtin_memcpy(&v, &outb[h + 16 * i], 16);
			*reinterpret_cast<GLOBAL u32x4*>(dst + h + 16 * i) = v;
		}
		for (int32_t i = h + nv * 16 + lane; i < blen; i += 64)
			dst[i] = outb[i];
		// keep the last 16 output bytes in front of the next batch
		uint32_t tb = 0;
		if (lane < 16)
			tb = L.outx[blen + lane];
		wave_lds_fence();
		if (lane < 16)
			L.outx[lane] = uint8_t(tb);
		if (lane == 0)
			L.tail_end = o + blen;
	}
	// later batches (either wave) read this output back from HBM
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	STAMP(SP_FLUSH);
	STAMP_COUNT(SP_BATCHES, 1);
}

__global__ __launch_bounds__(128) void k_decode_pc(const uint8_t* __restrict__ frame,
                                                    uint64_t frame_len,
                                                    const lz4ada_block_desc* __restrict__ desc,
                                                    uint32_t nblocks, uint8_t* __restrict__ out,
                                                    lz4ada_block_status* __restrict__ status,
                                                    int retry_only, int32_t hist)
{
	__shared__ PcLds L;

	const uint32_t b = blockIdx.x;
	if (b >= nblocks)
		return;
	if (retry_only && status[b].code != DS_RETRY && status[b].code != DS_SPARSE)
		return;
	const int wave = int(threadIdx.x >> 6);
	const int lane = int(lane_id());
	const lz4ada_block_desc d = desc[b];
	cg8* __restrict__ in = gptr(frame) + d.in_off;
	g8* __restrict__ ob = gptr(out) + d.out_off;
	const int32_t n = int32_t(d.in_len);
	const int32_t cap = int32_t(d.out_cap);

	lz4ada_block_status st;
	st.code = DS_OK;
	st.aux = 0;
	st.detail = 0;
	st.err_out_pos = 0;
	st.out_len = 0;

	if (d.flags & LZ4ADA_BLOCK_STORED) {
		if (wave == 0) {
			if (n > cap) {
				st.code = DS_OUT_OVERFLOW;
			} else {
				wave_copy(ob, in, n);
				st.out_len = uint32_t(n);
			}
			if (lane == 0) {
				status[b].code = st.code;
				status[b].aux = 0;
				status[b].detail = 0;
				status[b].err_out_pos = 0;
				status[b].out_len = st.out_len;
			}
		}
		return;
	}

	const uintptr_t lim_addr = reinterpret_cast<uintptr_t>(frame) + frame_len;
	const int32_t mis = int32_t(reinterpret_cast<uintptr_t>(in) & 15u);
	// producer state (wave 0)
	int32_t s = 0, o = 0, hi = -mis;
	u32x4 pf0 = {0, 0, 0, 0}, pf1 = {0, 0, 0, 0};
	if (wave == 0) {
		pf0 = load_chunk(in, lim_addr, hi);
		pf1 = load_chunk(in, lim_addr, hi + 1024);
	}
	bool ok = true;
	bool d1 = false;  // a match with offset >= D1_OFF reads before the block start
	bool pdone = (n == 0);
	bool smode = false;  // sequences are long: parse them one at a time
	if (threadIdx.x < PC_SLOTS)
		L.full[threadIdx.x] = 0;
	if (threadIdx.x == 0) {
		L.pdone = pdone ? 1 : 0;
		L.tail_end = -1;
	}
	__syncthreads();
	STAMP_DECL;
	// The waves share only the slot queue: the producer fills slot pseq
	// (mod PC_SLOTS) once the consumer has released it and raises its
	// `full` flag; the consumer copies the slots in order and lowers the
	// flag after its flush has reached memory.  No workgroup barriers.
	if (wave == 0) {
		// ---------------------------------------------------- producer
		int32_t pseq = 0;
		while (!pdone) {
			const int ps = pseq & (PC_SLOTS - 1);
			while (lds_poll(&L.full[ps]))
				__builtin_amdgcn_s_sleep(1);
			STAMP(SP_WAIT);
			int32_t nb = 0, blen = 0, bcomp0 = s;
			bool stop = false, end_block = false;
			for (int32_t iter = 0;; ++iter) {
				if (iter > 4 * n + 64) {
					st.code = DS_INTERNAL;
					ok = false;
					pdone = true;
					break;
				}
				// oldest compressed byte a queued batch may still read
				int32_t keep = INT32_MAX;
#pragma unroll
				for (int k = 1; k < PC_SLOTS; ++k) {
					const int q = (pseq - k) & (PC_SLOTS - 1);
					if (lds_poll(&L.full[q]))
						keep = L.m_bcomp0[q] < keep ? L.m_bcomp0[q] : keep;
				}
				keep = uni(keep);
				if (keep != INT32_MAX && s + PC_STAGE_AHEAD + 1024 + MIRROR - keep > INB) {
					// staging further would overwrite a queued batch's input
					if (nb > 0)
						break;
					__builtin_amdgcn_s_sleep(2);
					--iter;
					continue;
				}
				bool force_flush = false;
				{
					int32_t lo = nb ? bcomp0 : s;
					lo = keep < lo ? keep : lo;
					stage_to(L, in, lim_addr, mis, hi, pf0, pf1, lo, s + PC_STAGE_AHEAD);
					STAMP(SP_STAGE);
					STAMP_COUNT(SP_WINDOWS, 1);
				}
				const uint32_t peek =
				    uint32_t(uni(int32_t(lds_u16(L.inb + ((s + mis) & INB_MASK)))));
				if (((peek & 0xf0u) == 0xf0u && (peek >> 8) == 255u && s + 1 < n) || smode) {
					// serial run: one sequence at a time in scalar registers
					// while sequences average >= PC_SER_MIN compressed bytes
					const int32_t s_run = s;
					int32_t took = 0;
					for (;;) {
						Cand t = {};
						bool okp = parse_fast(L.inb, mis, s, n, hi, t);
						const int32_t klen = t.L + t.ml;
						const int32_t d0 = o + blen + t.L;
						okp = okp && nb < MAXTOK && klen <= PC_BIG && blen + klen <= OUTB &&
						      o + blen + klen <= cap && (t.kind != TK_NORMAL || d0 - t.off >= -hist) &&
						      (t.off >= 16 || t.ml <= 64);
						d1 = d1 || (okp && t.kind == TK_NORMAL && d0 < t.off && t.off >= D1_OFF);
						if (!okp) {
							if (nb == 0)
								stop = true;
							else
								force_flush = true;
							smode = false;
							break;
						}
						if (lane == 0) {
							L.r_tstart[ps][nb] = blen;
							L.r_L[ps][nb] = t.L;
							L.r_lit[ps][nb] = t.lit;
							L.r_off[ps][nb] = t.off;
							L.r_ml[ps][nb] = t.ml;
						}
						if (nb == 0)
							bcomp0 = s;
						++nb;
						++took;
						blen += klen;
						STAMP_COUNT(SP_TOKENS, 1);
						if (t.kind == TK_LAST || t.next >= n) {
							end_block = true;
							s = t.next;
							break;
						}
						s = t.next;
						smode = (s - s_run) >= PC_SER_MIN * took;
						if (!smode || nb >= MAXTOK || blen > OUTB - PC_BIG ||
						    (s - bcomp0) >= PC_SPAN || s + PC_BIG + 64 > hi)
							break;
					}
				} else {
					const int32_t s_win = s;
					// next-token offsets of the window's WIN positions, one
					// byte each (0: no in-window normal successor), packed
					// four to a lane: position k in lane k & 63, byte k >> 6
					uint32_t pk = 0;
					if (s + WIN + 2 * 272 < n) {
						// far from the block end only a zero offset or a
						// 255 extension byte can stop a chain: branch-free,
						// all reads of a kind issued together
						uint32_t t2[WIN / 64], w4[WIN / 64];
						int32_t pp[WIN / 64];
#pragma unroll
						for (int q = 0; q < WIN / 64; ++q)
							t2[q] = lds_u16(L.inb + ((s + 64 * q + lane + mis) & INB_MASK));
#pragma unroll
						for (int q = 0; q < WIN / 64; ++q) {
							const uint32_t x1 = ((t2[q] & 0xf0u) == 0xf0u) ? 1u : 0u;
							pp[q] = 64 * q + lane + 1 + int32_t(x1) + int32_t((t2[q] >> 4) & 15u) +
							        int32_t(x1 ? (t2[q] >> 8) : 0u);
						}
#pragma unroll
						for (int q = 0; q < WIN / 64; ++q)
							w4[q] = lds_u32(L.inb + ((s + pp[q] + mis) & INB_MASK));
#pragma unroll
						for (int q = 0; q < WIN / 64; ++q) {
							const bool x1 = (t2[q] & 0xf0u) == 0xf0u, x2 = (t2[q] & 15u) == 15u;
							const uint32_t e2 = (w4[q] >> 16) & 0xffu;
							const int32_t rel = pp[q] + 2 + (x2 ? 1 : 0);
							const bool ok = ((w4[q] & 0xffffu) != 0) & !(x1 & ((t2[q] >> 8) == 255u)) &
							                !(x2 & (e2 == 255u)) & (rel < WIN);
							pk |= uint32_t(ok ? rel : 0) << (8 * q);
						}
					} else {
#pragma unroll
						for (int q = 0; q < WIN / 64; ++q) {
							const int k = 64 * q + lane;
							const Cand t = parse_cand(L.inb, mis, s + k, n);
							const int32_t rel = t.next - s;
							pk |= uint32_t((t.kind == TK_NORMAL && rel < WIN) ? rel : 0) << (8 * q);
						}
					}
					STAMP(SP_CAND);
					// PC_ANCH doubling levels in registers (tables 2, 4, ..
					// 2^PC_ANCH sequences ahead), a scalar walk over the last
					// placing every 2^PC_ANCH-th sequence in its lane group,
					// then each lane steps from that anchor by the binary
					// digits of its index: lane i gets sequence i's position
					uint32_t jt[PC_ANCH + 1];
					jt[0] = pk;
#pragma unroll
					for (int r = 1; r <= PC_ANCH; ++r) {
						uint32_t j = 0;
#pragma unroll
						for (int q = 0; q < WIN / 64; ++q)
							j |= win_next(jt[r - 1], (jt[r - 1] >> (8 * q)) & 0xffu) << (8 * q);
						jt[r] = j;
					}
					const int32_t wl = uni(MAXTOK - nb < 64 ? MAXTOK - nb : 64);
					uint32_t cj = 0xffffu;
					int32_t cur = 0, walked = 0;
					do {
						cj = ((lane >> PC_ANCH) == walked) ? uint32_t(cur) : cj;
						++walked;
						const uint32_t w =
						    uint32_t(__builtin_amdgcn_readlane(int32_t(jt[PC_ANCH]), cur & 63));
						cur = uni(int32_t((w >> (8 * (cur >> 6))) & 0xffu));
					} while (cur != 0 && (walked << PC_ANCH) < wl);
#pragma unroll
					for (int r = PC_ANCH - 1; r >= 0; --r) {
						const uint32_t x = win_look(jt[r], cj & 0xffu);
						if ((lane >> r) & 1)
							cj = (cj < WIN && x) ? x : 0xffffu;
					}
					STAMP(SP_DOUBLE);
					const bool inwin = cj < WIN;
					const Cand tk = (s + WIN + 2 * 272 < n)
					                    ? parse_cand_far(L.inb, mis, s + (inwin ? int32_t(cj) : 0))
					                    : parse_cand(L.inb, mis, s + (inwin ? int32_t(cj) : 0), n);
					const int32_t kL = tk.L, klit = tk.lit, koff = tk.off, kml = tk.ml;
					const int32_t knext = tk.next, kkind = tk.kind;
					const bool good = inwin && (kkind == TK_NORMAL || kkind == TK_LAST);
					const int32_t klen = kL + kml;
					const int32_t incl = wave_incl_scan(good ? klen : 0);
					const int32_t tstart = blen + incl - klen;
					const int32_t d0 = o + tstart + kL;
					const bool fits = good && lane < MAXTOK - nb && klen <= PC_BIG &&
					                  blen + incl <= OUTB && o + blen + incl <= cap &&
					                  (kkind != TK_NORMAL || d0 - koff >= -hist) &&
					                  (koff >= 16 || kml <= 64);
					const uint64_t badm = __ballot(!fits);
					const int cnt = badm ? (__ffsll((long long)badm) - 1) : 64;
					d1 = d1 || (lane < cnt && kkind == TK_NORMAL && d0 < koff && koff >= D1_OFF);
					const int32_t cnext = cnt > 0 ? __shfl(knext, cnt - 1) : s;
					const int32_t ckind_last = cnt > 0 ? __shfl(kkind, cnt - 1) : TK_NORMAL;
					if (lane < cnt) {
						L.r_tstart[ps][nb + lane] = tstart;
						L.r_L[ps][nb + lane] = kL;
						L.r_lit[ps][nb + lane] = klit;
						L.r_off[ps][nb + lane] = koff;
						L.r_ml[ps][nb + lane] = kml;
					}
					STAMP_COUNT(SP_TOKENS, cnt);
					smode = cnt > 0 && cnext - s_win >= PC_SER_MIN * cnt;
					const bool was_empty = (nb == 0);
					if (was_empty && cnt > 0)
						bcomp0 = s;
					nb += cnt;
					blen += cnt > 0 ? __shfl(incl, cnt - 1) : 0;
					if (cnt > 0 && ckind_last == TK_LAST) {
						end_block = true;
						s = n;
					} else if (cnt > 0 && cnext >= n) {
						end_block = true;  // block ends right after a match (lz4ada.adb:780)
						s = cnext;
					} else if (cnt > 0) {
						s = cnext;
					} else if (was_empty) {
						stop = true;
					} else {
						force_flush = true;
					}
				}
				wave_lds_fence();
				STAMP(SP_SELECT);
				if (end_block || stop || force_flush ||
				    nb > (smode ? MAXTOK - 1 : MAXTOK - WTOK / 2) || blen > OUTB - PC_BIG ||
				    (s - bcomp0) >= PC_SPAN)
					break;
			}
			if (nb > 0) {
				if (lane == 0) {
					L.m_nb[ps] = nb;
					L.m_blen[ps] = blen;
					L.m_o[ps] = o;
					L.m_bcomp0[ps] = bcomp0;
				}
				wave_lds_fence();
				if (lane == 0)
					L.full[ps] = 1;
				o += blen;
				++pseq;
			}
			if (end_block)
				pdone = true;
			if (stop && !pdone) {
				// every queued batch must be in HBM: the one-token path reads
				// its history there
				for (int k = 0; k < PC_SLOTS; ++k)
					while (lds_poll(&L.full[k]))
						__builtin_amdgcn_s_sleep(1);
				STAMP(SP_WAIT);
				int64_t s64 = s, o64 = o;
				if (!one_token(in, n, ob, cap, s64, o64, st, hist, d1)) {
					ok = false;
					pdone = true;
				} else {
					s = int32_t(s64);
					o = int32_t(o64);
					if (s >= n)
						pdone = true;
				}
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				STAMP(SP_ONE);
			}
		}
		d1 = __any(d1);
		wave_lds_fence();
		if (lane == 0)
			L.pdone = 1;
	} else {
		// ---------------------------------------------------- consumer
		for (int32_t cseq = 0;; ++cseq) {
			const int cs = cseq & (PC_SLOTS - 1);
			bool have = true;
			while (!lds_poll(&L.full[cs])) {
				if (lds_poll(&L.pdone) && !lds_poll(&L.full[cs])) {
					have = false;
					break;
				}
				__builtin_amdgcn_s_sleep(1);
			}
			STAMP(SP_WAIT);
			if (!have)
				break;
			asm volatile("" ::: "memory");
			pc_copy_batch(L, cs, mis, ob, hist STAMP_ARGS);
			wave_lds_fence();
			if (lane == 0)
				L.full[cs] = 0;
		}
	}
	__syncthreads();
	STAMP_FLUSH();

	if (threadIdx.x == 0) {
		status[b].code = ok ? int32_t(DS_OK) : st.code;
		status[b].aux = ok ? (d1 ? AUX_D1_RISK : 0) : st.aux;
		status[b].detail = st.detail;
		status[b].err_out_pos = st.err_out_pos;
		status[b].out_len = uint32_t(o);
	}
}

// Gather variable-length slots into a contiguous buffer.
__global__ __launch_bounds__(256) void k_compact(const uint8_t* __restrict__ src,
                                                  const lz4ada_block_desc* __restrict__ desc,
                                                  const uint64_t* __restrict__ dst_off,
                                                  const lz4ada_block_status* __restrict__ st,
                                                  uint32_t nblocks, uint8_t* __restrict__ dst)
{
	const uint32_t b = blockIdx.x;
	if (b >= nblocks)
		return;
	const uint8_t* s = src + desc[b].out_off;
	uint8_t* t = dst + dst_off[b];
	const uint32_t n = st[b].out_len;
	for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
		t[i] = s[i];
}

// ------------------------------------------ reference-exact serial kernel
//
// Single-lane emulation of Decode_Full_Block_With_Trailer after the block
// checksum (lz4ada.adb:678-695) on a device mirror of the caller's Buffer.
// Every Write_Output (:790-824) moves 8-byte chunks while 8 source bytes
// remain before Data'Last -- each chunk an Ada slice assignment (memmove) --
// then an exact tail, so it overshoots past Output_Pos exactly like the
// reference.  That overshoot is what corrupts linked history in quirk D1,
// and this kernel reproduces it.

struct SerialCtx {
	uint8_t* buf;
	int64_t buflen;
	SerialState* st;
	int64_t output_pos;
	uint64_t size_remaining;
	int has_content_size;
};

// Write_Output: copy data[first..last] (data spans [0, data_len)) to
// buf[output_pos..].  Returns false (status set) on error.
__device__ bool ser_write(SerialCtx& c, const uint8_t* data, int64_t data_len,
                          int64_t first, int64_t last)
{
	const int64_t num = last - first + 1;
	int64_t co = c.output_pos, ci = first;
	if (co + num > c.buflen) {
		c.st->code = DS_OUT_OVERFLOW;
		return false;
	}
	while ((data_len - 1) - ci + 1 >= 8 && ci <= last) {
		uint8_t tmp[8];
#pragma unroll
		for (int i = 0; i < 8; ++i)
			tmp[i] = data[ci + i];
		const int64_t lim = (co + 8 <= c.buflen) ? 8 : c.buflen - co;
		for (int i = 0; i < lim; ++i)
			c.buf[co + i] = tmp[i];
		co += 8;
		ci += 8;
	}
	if (ci <= last) {
		const int64_t cnt = last - ci + 1;
		int64_t avail = data_len - ci;
		if (avail < 0)
			avail = 0;
		if (avail > cnt)
			avail = cnt;
		// memmove semantics: copy forward when dst < src, else backward.
		if (c.buf + co <= data + ci) {
			for (int64_t i = 0; i < avail; ++i)
				c.buf[co + i] = data[ci + i];
		} else {
			for (int64_t i = avail - 1; i >= 0; --i)
				c.buf[co + i] = data[ci + i];
		}
		for (int64_t i = avail; i < cnt; ++i)  // D3: bytes past Data'Last
			c.buf[co + i] = 0;
	}
	c.output_pos += num;
	if (c.has_content_size) {  // Decrease_Data_Size_Remaining (:826-839)
		if (c.size_remaining < uint64_t(num)) {
			c.st->code = DS_CONTENT_SIZE;
			return false;
		}
		c.size_remaining -= uint64_t(num);
	}
	return true;
}

__global__ __launch_bounds__(64) void k_serial_block(uint8_t* buf, int64_t buflen,
                                                      const uint8_t* __restrict__ blk,
                                                      int64_t raw_len, int64_t data_len,
                                                      int compressed, SerialState* st)
{
	if (threadIdx.x != 0)
		return;
	SerialCtx c;
	c.buf = buf;
	c.buflen = buflen;
	c.st = st;
	c.output_pos = st->output_pos;
	c.size_remaining = st->size_remaining;
	c.has_content_size = st->has_content_size;
	st->code = DS_OK;
	st->aux = 0;
	st->detail = 0;
	int64_t oph = st->output_pos_history;
	if (c.output_pos >= HISTORY_SIZE)  // :678-680
		c.output_pos = 0;
	bool ok = true;
	int64_t first = c.output_pos;
	if (!compressed) {  // stored block (:685-694), Data = payload + trailer
		ok = ser_write(c, blk, data_len, 0, raw_len - 1);
		if (ok) {
			if (c.output_pos >= HISTORY_SIZE)
				oph = c.output_pos;
			first = c.output_pos - raw_len;
		}
	} else {
		const uint8_t* raw = blk;
		const int64_t n = raw_len;
		int64_t idx = 0;
		while (ok && idx <= n - 1) {  // Decompress_Sequence (:737-777)
			const uint32_t token = raw[idx];
			int64_t nlit = token >> 4, ml = token & 15;
			idx += 1;
			if (nlit == 15) {
				uint32_t t;
				do {
					if (idx > n - 1) { st->code = DS_TRUNCATED; ok = false; break; }
					t = raw[idx];
					nlit += t;
					idx += 1;
				} while (t == 255);
				if (!ok) break;
			}
			if (nlit > 0) {
				ok = ser_write(c, raw, n, idx, idx + nlit - 1);
				if (!ok) break;
				idx += nlit;
			}
			if (idx > n - 1) {
				if (ml != 0) {
					st->code = DS_ML_AFTER_LIT;
					st->aux = int32_t(ml);
					ok = false;
				} else if (idx > n) {
					st->code = DS_LIT_OVERRUN;
					ok = false;
				}
				break;
			}
			if (idx + 1 > n - 1) { st->code = DS_TRUNCATED; ok = false; break; }
			const int64_t offset = int64_t(raw[idx]) | (int64_t(raw[idx + 1]) << 8);
			idx += 2;
			if (offset == 0) { st->code = DS_OFFSET0; ok = false; break; }
			if (ml == 15) {
				uint32_t t;
				do {
					if (idx > n - 1) { st->code = DS_TRUNCATED; ok = false; break; }
					t = raw[idx];
					ml += t;
					idx += 1;
				} while (t == 255);
				if (!ok) break;
			}
			ml += 4;
			// Output_With_History (:845-904)
			const int64_t raw_off = c.output_pos - offset;
			int64_t remaining = ml, i_off, i_len;
			if (raw_off >= 0) {
				i_off = raw_off;
				i_len = ml < offset ? ml : offset;
			} else {
				const int64_t h_off = raw_off + oph;
				int64_t h_len = offset - c.output_pos;
				if (ml < h_len)
					h_len = ml;
				if (h_off < 0) {
					st->code = DS_BACKREF;
					st->detail = h_off;
					ok = false;
					break;
				}
				if (h_len > 0) {
					ok = ser_write(c, buf, buflen, h_off, h_off + h_len - 1);
					if (!ok) break;
					remaining = ml - h_len;
				}
				i_off = 0;
				i_len = remaining < c.output_pos ? remaining : c.output_pos;
			}
			if (i_len > 0) {
				ok = ser_write(c, buf, buflen, i_off, i_off + i_len - 1);
				if (!ok) break;
				remaining -= i_len;
			}
			if (remaining > 0) {
				const int64_t r_start = c.output_pos - offset;
				int64_t done = 0;
				while (done < remaining) {
					int64_t r_len = c.output_pos - r_start;
					if (remaining - done < r_len)
						r_len = remaining - done;
					ok = ser_write(c, buf, buflen, r_start, r_start + r_len - 1);
					if (!ok) break;
					done += r_len;
				}
				if (!ok) break;
			}
		}
		if (ok && c.output_pos >= HISTORY_SIZE)  // :785-787
			oph = c.output_pos;
	}
	st->first = first;
	st->last = c.output_pos - 1;
	st->output_pos = c.output_pos;
	st->output_pos_history = oph;
	st->size_remaining = c.size_remaining;
	__threadfence_system();
}

// -------------------------------------------------------------- launchers

#ifdef LZ4ADA_STAMPS
extern "C" int lz4ada_debug_stamps(unsigned long long* out, int reset)
{
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * SP_N) !=
	    hipSuccess)
		return -1;
	if (reset) {
		unsigned long long z[SP_N] = {};
		if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z) != hipSuccess)
			return -1;
	}
	return SP_N;
}
#endif

hipError_t launch_decode_variant(const uint8_t* d_frame, uint64_t frame_len,
                                 const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                 uint8_t* d_out, lz4ada_block_status* d_status, int variant,
                                 hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	if (variant == DEC_PC) {
		hipLaunchKernelGGL(k_decode_pc, dim3(nblocks), dim3(128), 0, stream, d_frame, frame_len,
		                   d_desc, nblocks, d_out, d_status, 0, 0);
		return hipGetLastError();
	}
	if (variant == DEC_IDX_LINKED)
		return launch_decode_idx(d_frame, frame_len, d_desc, nblocks, d_out, d_status, stream, 1);
	if (variant == DEC_IDX_SPLIT)
		return launch_decode_idx(d_frame, frame_len, d_desc, nblocks, d_out, d_status, stream, -4);
	if (variant == DEC_IDX1_ALONE || variant == DEC_IDX2_ALONE || variant == DEC_PP2_ALONE)
		return launch_decode_idx(d_frame, frame_len, d_desc, nblocks, d_out, d_status, stream,
		                         variant == DEC_IDX1_ALONE ? -1 : (variant == DEC_IDX2_ALONE ? -2 : -3));
	if (variant == DEC_IDX || variant == DEC_IDX_ALONE || variant == DEC_IDX_SPARSE) {
		const hipError_t err = launch_decode_idx(d_frame, frame_len, d_desc, nblocks, d_out,
		                                         d_status, stream);
		if (err != hipSuccess || variant == DEC_IDX_ALONE)
			return err;
		const hipError_t e2 = launch_decode_sparse(d_frame, frame_len, d_desc, nblocks, d_out,
		                                           d_status, stream);
		if (e2 != hipSuccess || variant == DEC_IDX_SPARSE)
			return e2;
		hipLaunchKernelGGL(k_decode_pc, dim3(nblocks), dim3(128), 0, stream, d_frame, frame_len,
		                   d_desc, nblocks, d_out, d_status, 1, 0);
		return hipGetLastError();
	}
	// 1 (the round-1 one-wave decoder) and 2 (the workgroup decoder, retired
	// in round 4: no faster than k_decode_pc on the facade's small blocks)
	return hipErrorInvalidValue;
}

hipError_t launch_decode_pc(const uint8_t* d_frame, uint64_t frame_len,
                            const lz4ada_block_desc* d_desc, uint32_t nblocks, uint8_t* d_out,
                            lz4ada_block_status* d_status, int retry_only, int32_t hist,
                            hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(k_decode_pc, dim3(nblocks), dim3(128), 0, stream, d_frame, frame_len, d_desc,
	                   nblocks, d_out, d_status, retry_only, hist);
	return hipGetLastError();
}

static int decoder_variant();

hipError_t launch_decode_blocks(const uint8_t* d_frame, uint64_t frame_len,
                                const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                uint8_t* d_out, lz4ada_block_status* d_status,
                                hipStream_t stream)
{
	return launch_decode_variant(d_frame, frame_len, d_desc, nblocks, d_out, d_status,
	                             decoder_variant(), stream);
}

static int decoder_variant()
{
	// Default: the index-driven decoder (lz4ada_idx.hip), the two-wave
	// decoder for the blocks it declines.  LZ4ADA_DECODER=pc selects the
	// two-wave decoder alone.
	static const int variant = [] {
		const char* e = getenv("LZ4ADA_DECODER");
		if (e && e[0] == 'p')
			return int(DEC_PC);
		return int(DEC_IDX);
	}();
	return variant;
}

// A side stream and its fork / join events per device and host thread,
// created on first use and kept for the process.
struct SideStream {
	hipStream_t s = nullptr;
	hipEvent_t fork = nullptr, join = nullptr, fill = nullptr;
};

static hipError_t side_stream(SideStream*& out)
{
	constexpr int MAXDEV = 64;
	static thread_local SideStream cache[MAXDEV];
	int dev = 0;
	hipError_t err = hipGetDevice(&dev);
	if (err != hipSuccess)
		return err;
	if (dev < 0 || dev >= MAXDEV)
		return hipErrorInvalidDevice;
	SideStream& c = cache[dev];
	if (!c.s) {
		SideStream n;
		err = hipStreamCreateWithFlags(&n.s, hipStreamNonBlocking);
		if (err == hipSuccess)
			err = hipEventCreateWithFlags(&n.fork, hipEventDisableTiming);
		if (err == hipSuccess)
			err = hipEventCreateWithFlags(&n.join, hipEventDisableTiming);
		if (err == hipSuccess)
			err = hipEventCreateWithFlags(&n.fill, hipEventDisableTiming);
		if (err != hipSuccess) {
			if (n.fill)
				(void)hipEventDestroy(n.fill);
			if (n.join)
				(void)hipEventDestroy(n.join);
			if (n.fork)
				(void)hipEventDestroy(n.fork);
			if (n.s)
				(void)hipStreamDestroy(n.s);
			return err;
		}
		c = n;
	}
	out = &c;
	return hipSuccess;
}

hipError_t launch_block_checksums_beside(const uint8_t* d_frame, const lz4ada_block_desc* d_desc,
                                        uint32_t nblocks, lz4ada_block_status* d_status, hipStream_t stream)
{
	SideStream* side = nullptr;
	hipError_t err = side_stream(side);
	if (err == hipSuccess)
		err = hipEventRecord(side->fork, stream);
	if (err == hipSuccess)
		err = hipStreamWaitEvent(side->s, side->fork, 0);
	if (err == hipSuccess)
		err = launch_block_checksums(d_frame, d_desc, nblocks, d_status, side->s);
	if (err == hipSuccess)
		err = hipEventRecord(side->join, side->s);
	return err;
}

hipError_t join_block_checksums(hipStream_t stream)
{
	SideStream* side = nullptr;
	const hipError_t err = side_stream(side);
	return err != hipSuccess ? err : hipStreamWaitEvent(stream, side->join, 0);
}

hipError_t side_fork(hipStream_t stream, hipStream_t* side_s)
{
	SideStream* side = nullptr;
	hipError_t err = side_stream(side);
	if (err == hipSuccess)
		err = hipEventRecord(side->fork, stream);
	if (err == hipSuccess)
		err = hipStreamWaitEvent(side->s, side->fork, 0);
	if (err == hipSuccess)
		*side_s = side->s;
	return err;
}

hipError_t side_join(hipStream_t stream)
{
	SideStream* side = nullptr;
	hipError_t err = side_stream(side);
	if (err == hipSuccess)
		err = hipEventRecord(side->join, side->s);
	return err != hipSuccess ? err : hipStreamWaitEvent(stream, side->join, 0);
}

hipError_t launch_link_fill_beside(uint8_t* x, uint8_t* y, uint8_t* h, const lz4ada_block_desc* d_desc,
                                   uint32_t nblocks, hipStream_t stream)
{
	SideStream* side = nullptr;
	hipError_t err = side_stream(side);
	if (err == hipSuccess)
		err = hipEventRecord(side->fork, stream);
	if (err == hipSuccess)
		err = hipStreamWaitEvent(side->s, side->fork, 0);
	if (err == hipSuccess)
		err = launch_link_fill(x, y, h, d_desc, nblocks, side->s);
	if (err == hipSuccess)
		err = hipEventRecord(side->fill, side->s);
	return err;
}

hipError_t join_link_fill(hipStream_t stream)
{
	SideStream* side = nullptr;
	const hipError_t err = side_stream(side);
	return err != hipSuccess ? err : hipStreamWaitEvent(stream, side->fill, 0);
}

hipError_t launch_decode_checked(const uint8_t* d_frame, uint64_t frame_len,
                                 const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                 uint8_t* d_out, lz4ada_block_status* d_status,
                                 hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	if (decoder_variant() != DEC_IDX || getenv("LZ4ADA_NO_OVERLAP")) {
		hipError_t err = launch_block_checksums(d_frame, d_desc, nblocks, d_status, stream);
		return err != hipSuccess ? err
		                         : launch_decode_blocks(d_frame, frame_len, d_desc, nblocks, d_out,
		                                                d_status, stream);
	}
	// k_index (2 waves/SIMD, LDS-bound, 168 VGPRs) leaves VGPRs for one
	// k_xxh32_rows wave per SIMD (no LDS): both chains are latency-bound,
	// so the checksums ride in k_index's idle issue slots
	SideStream* side = nullptr;
	hipError_t err = side_stream(side);
	if (err != hipSuccess)
		return err;
	void* tab = nullptr;
	err = hipMallocAsync(&tab, index_table_bytes(frame_len, nblocks), stream);
	if (err != hipSuccess)
		return err;
	err = hipEventRecord(side->fork, stream);
	if (err == hipSuccess)
		err = hipStreamWaitEvent(side->s, side->fork, 0);
	// pass 1 and pass 2 in one launch (k_decode_idx mode 3), or as two
	// (LZ4ADA_NO_FUSE, for A/B)
	static const bool fuse = getenv("LZ4ADA_NO_FUSE") == nullptr;
	if (err == hipSuccess)
		err = fuse ? launch_decode_idx_tab(d_frame, frame_len, d_desc, nblocks,
		                                   static_cast<const uint8_t*>(tab), d_out, d_status,
		                                   idx_fused_mode(nblocks), stream)
		           : launch_index(d_frame, frame_len, d_desc, nblocks, static_cast<uint8_t*>(tab),
		                          d_status, stream);
	if (err == hipSuccess)
		err = launch_block_checksums(d_frame, d_desc, nblocks, d_status, side->s);
	if (err == hipSuccess)
		err = hipEventRecord(side->join, side->s);
	if (err == hipSuccess && !fuse)
		err = launch_decode_idx_tab(d_frame, frame_len, d_desc, nblocks,
		                            static_cast<const uint8_t*>(tab), d_out, d_status, 0, stream);
	// literal-heavy blocks pass 1 declined, then every other declined block
	if (err == hipSuccess)
		err = launch_decode_sparse(d_frame, frame_len, d_desc, nblocks, d_out, d_status, stream);
	if (err == hipSuccess)
		err = launch_decode_pc(d_frame, frame_len, d_desc, nblocks, d_out, d_status, 1, 0, stream);
	const hipError_t e2 = hipFreeAsync(tab, stream);
	const hipError_t e3 = hipStreamWaitEvent(stream, side->join, 0);
	return err != hipSuccess ? err : (e2 != hipSuccess ? e2 : e3);
}

hipError_t launch_serial_block(uint8_t* d_buf, int64_t buflen, const uint8_t* d_blk,
                               int64_t raw_len, int64_t data_len, int compressed,
                               SerialState* d_state, hipStream_t stream)
{
	hipLaunchKernelGGL(k_serial_block, dim3(1), dim3(64), 0, stream, d_buf, buflen, d_blk,
	                   raw_len, data_len, compressed, d_state);
	return hipGetLastError();
}

hipError_t launch_compact(const uint8_t* d_src, const lz4ada_block_desc* d_desc,
                          const uint64_t* d_dst_off, const lz4ada_block_status* d_status,
                          uint32_t nblocks, uint8_t* d_dst, hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(k_compact, dim3(nblocks), dim3(256), 0, stream, d_src, d_desc, d_dst_off,
	                   d_status, nblocks, d_dst);
	return hipGetLastError();
}

}  // namespace lz4ada
