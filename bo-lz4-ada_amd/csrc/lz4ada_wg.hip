// lz4ada_wg.hip -- workgroup-per-block LZ4 block decoder for gfx950.
//
// Same contract as k_decode_blocks (lz4ada_kernels.hip): decodes every
// independent block of a device-resident frame into its output slot,
// following lib/lz4ada.adb:716-904 (Decompress_Full_Block, Write_Output,
// Output_With_History) for valid data.  Anything it does not handle -- an
// invalid token, a reference before the block start, a slot overflow, a
// single sequence longer than a batch -- is marked DS_RETRY and redone by
// k_decode_blocks, which reports the exact reference error.
//
// One 256-lane workgroup owns one block, so the block's last 64 KiB of
// output lives in LDS and every match copy is LDS -> LDS:
//
//  * batch: 16 KiB of compressed input (256 lane regions of 64 B) staged
//    in LDS with 16 B/lane loads;
//  * own walk: every lane parses tokens from the start of its region to the
//    region end, recording the visited positions (64-bit mask);
//  * continuation: from its exit, each lane keeps parsing until it lands on
//    a position another lane's walk visited -- from there on that lane's
//    walk is the same chain (parsing is deterministic);
//  * path: from lane 0 (which starts at the exact chain position) the
//    lanes whose walks lie on the true chain are found by pointer doubling
//    over the "synced into lane k" links; each gets its exact entry point;
//  * a workgroup prefix sum of decoded lengths gives every lane its output
//    offset;
//  * copy: each path lane copies its sequences into the LDS output ring;
//    a match whose source lies in another lane's output waits until that
//    lane's published progress covers it (dataflow, no barriers; a lane
//    only ever waits on earlier output, so it always completes);
//  * flush: the batch output goes to HBM with 16-byte coalesced stores.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4ada_dev.h"
#include "lz4ada_internal.h"

namespace lz4ada {

namespace wg {

constexpr int LANES = 512;                  // lanes per workgroup (8 waves)
constexpr int WAVES = LANES / 64;
constexpr int REG = 32;                     // compressed bytes per lane region
constexpr int BATCH_IN = LANES * REG;       // 16 KiB compressed per batch
constexpr int IN_OVH = 1024;                // staged bytes past the batch
constexpr int IN_STAGE = BATCH_IN + IN_OVH + 32;
constexpr int RING = 96 * 1024;             // output ring: 64 KiB window + a batch
constexpr int OUT_CAP = 32 * 1024;          // output bytes per batch
constexpr int RING_HIST = RING - OUT_CAP;   // history bytes always still in the ring
static_assert(RING_HIST >= 65536, "every match source stays in the ring");
constexpr int CMAX = 48;                    // continuation steps before a batch is cut
constexpr int LONG = 64;                    // longer literal/match runs: whole-wave copies
constexpr int NDONE = OUT_CAP / 32 + 1;     // done-bitmap words
constexpr int MAXTOK = 4096;                // sequences per batch
constexpr int TERM = LANES;                 // path terminal node
constexpr int LEVELS = 9;                   // log2(LANES)
static_assert((1 << LEVELS) == LANES, "doubling levels");
static_assert(REG == 32, "vis masks are 32-bit");

// link types of a lane's continuation
enum Link : uint8_t { LK_LANE = 0, LK_END = 1, LK_TRUNC = 2, LK_BAD = 3, LK_NONE = 4 };

struct alignas(16) Lds {
	uint8_t ring[RING];     // output: position x at ring[x mod RING]
	uint8_t inb[IN_STAGE];  // staged compressed bytes of the batch
	uint32_t rec[MAXTOK];   // batch sequences: (start - s) | (output offset << 16)
	uint32_t vis[LANES];    // positions each lane's own walk visited
	int32_t X[LANES];       // own-walk exit (-1: malformed sequence)
	int32_t sp[LANES];      // where the continuation stopped
	int32_t entry[LANES];   // exact chain entry of path lanes, else -1
	int32_t eR[LANES];      // first true sequence starting in each region
	int32_t O[LANES + 1];   // output offset of each region's first sequence
	int32_t TB[LANES + 1];  // index of each region's first sequence
	uint16_t J[LEVELS + 1][LANES + 1];
	uint16_t node[LANES];
	uint8_t link[LANES];
	uint32_t done[NDONE];   // batch output bytes written (bitmap)
	int32_t wsum[WAVES];
	int32_t wsum2[WAVES];
	int32_t first_term, lastp, next_s, total, ntok, fail, cut_idx;
};

struct Tok {
	int32_t lit;   // first literal byte
	int32_t L;     // literal length
	int32_t off;   // match offset (0: last sequence)
	int32_t ml;    // match length (0: last sequence)
	int32_t next;  // next token, or -1 when the token is invalid
};

// Compressed byte at block-relative p: LDS when staged, else HBM.
struct Src {
	cg8* in;
	const uint8_t* inb;
	int32_t s;      // batch start (block-relative)
	int32_t mis;    // (in + s) & 15
	int32_t hi;     // staged end (block-relative, exclusive)

	__device__ __forceinline__ uint32_t rd(int32_t p) const
	{
		return p < hi ? uint32_t(inb[p - s + mis]) : uint32_t(in[p]);
	}
};

// One LZ4 sequence at p (lz4ada.adb:716-788).  Valid sequences only; any
// malformed one returns next = -1 and the block is redone by the exact
// per-wave decoder.  A block may end right after a match (the reference's
// loop exits when Idx passes Raw_Data'Last, :742) or after a literal-only
// last sequence whose match nibble is 0 (:752-764).
__device__ __noinline__ Tok parse_slow(const Src& S, int32_t p, int32_t n)
{
	Tok t;
	t.off = 0;
	t.ml = 0;
	t.next = -1;
	const uint32_t tk = S.rd(p);
	int32_t L = int32_t(tk >> 4);
	int32_t M = int32_t(tk & 15u);
	int32_t q = p + 1;
	t.lit = q;
	t.L = L;
	if (L == 15) {
		uint32_t e;
		do {
			if (q >= n)
				return t;
			e = S.rd(q);
			++q;
			L += int32_t(e);
		} while (e == 255u);
		t.lit = q;
		t.L = L;
	}
	q += L;
	if (q >= n) {
		if (q == n && M == 0)
			t.next = n;
		return t;
	}
	if (q + 2 > n)
		return t;
	const int32_t off = int32_t(S.rd(q) | (S.rd(q + 1) << 8));
	q += 2;
	if (off == 0)
		return t;
	if (M == 15) {
		uint32_t e;
		do {
			if (q >= n)
				return t;
			e = S.rd(q);
			++q;
			M += int32_t(e);
		} while (e == 255u);
	}
	t.off = off;
	t.ml = M + 4;
	t.next = q;
	return t;
}

// parse() common case: staged in LDS, at most one extension byte per
// length, not at the block end.  Byte reads: the token and the first
// extension byte together, then the offset and match extension together.
__device__ __forceinline__ Tok parse(const Src& S, int32_t p, int32_t n)
{
	const uint8_t* b = S.inb + (S.mis - S.s);
	if (p + 3 <= S.hi) {
		const uint32_t tk = b[p];
		const uint32_t e1 = b[p + 1];
		int32_t L = int32_t(tk >> 4);
		int32_t M = int32_t(tk & 15u);
		const bool xl = L == 15;
		L += xl ? int32_t(e1) : 0;
		const int32_t lit = p + 1 + (xl ? 1 : 0);
		const int32_t q = lit + L;
		if (q + 3 <= S.hi && q + 3 < n && !(xl && e1 == 255u)) {
			const uint32_t o0 = b[q], o1 = b[q + 1], e2 = b[q + 2];
			const bool xm = M == 15;
			const int32_t off = int32_t(o0 | (o1 << 8));
			if (!(xm && e2 == 255u) && off != 0) {
				M += xm ? int32_t(e2) : 0;
				Tok t;
				t.lit = lit;
				t.L = L;
				t.off = off;
				t.ml = M + 4;
				t.next = q + 2 + (xm ? 1 : 0);
				return t;
			}
		}
	}
	return parse_slow(S, p, n);
}

// Next sequence start and decoded length of the sequence at p, for the
// speculative walks (no offset read: a zero offset on the real chain is
// caught when the copy phase parses it).  next = -1: malformed.
struct Step {
	int32_t next;
	int32_t dec;
};

__device__ __noinline__ Step step_slow(const Src& S, int32_t p, int32_t n)
{
	Step r;
	r.next = -1;
	r.dec = 0;
	const uint32_t tk = S.rd(p);
	int32_t L = int32_t(tk >> 4);
	int32_t M = int32_t(tk & 15u);
	int32_t q = p + 1;
	if (L == 15) {
		uint32_t e;
		do {
			if (q >= n)
				return r;
			e = S.rd(q);
			++q;
			L += int32_t(e);
		} while (e == 255u);
	}
	q += L;
	if (q >= n) {
		if (q == n && M == 0) {
			r.next = n;
			r.dec = L;
		}
		return r;
	}
	q += 2;
	if (q > n)
		return r;
	if (M == 15) {
		uint32_t e;
		do {
			if (q >= n)
				return r;
			e = S.rd(q);
			++q;
			M += int32_t(e);
		} while (e == 255u);
	}
	r.next = q;
	r.dec = L + M + 4;
	return r;
}

// Common case of step(): token, at most one length-extension byte per
// length, everything staged in LDS and not at the block end.  Two LDS
// round trips at most; anything else takes step_slow.
__device__ __forceinline__ Step step(const Src& S, int32_t p, int32_t n)
{
	const uint8_t* b = S.inb + (S.mis - S.s);  // b[p] = compressed byte p
	if (p + 3 <= S.hi) {
		const uint32_t tk = b[p];
		const uint32_t e1 = b[p + 1];
		int32_t L = int32_t(tk >> 4);
		int32_t M = int32_t(tk & 15u);
		const bool xl = L == 15;
		L += xl ? int32_t(e1) : 0;
		const int32_t q = p + 1 + (xl ? 1 : 0) + L;  // offset bytes at q, q+1
		if (q + 3 <= S.hi && q + 3 < n && !(xl && e1 == 255u)) {
			const uint32_t e2 = b[q + 2];
			const bool xm = M == 15;
			if (!(xm && e2 == 255u)) {
				M += xm ? int32_t(e2) : 0;
				Step r;
				r.next = q + 2 + (xm ? 1 : 0);
				r.dec = L + M + 4;
				return r;
			}
		}
	}
	return step_slow(S, p, n);
}

// ring index of output position o + rel; callers pass oring = o mod RING
// and -RING < rel < RING
__device__ __forceinline__ uint32_t ridx(int32_t oring, int32_t rel)
{
	int32_t i = oring + rel;
	i += (i < 0) ? RING : 0;
	i -= (i >= RING) ? RING : 0;
	return uint32_t(i);
}

__device__ __forceinline__ u32x4 ring_ld16(const uint8_t* ring, uint32_t i)
{
	return ld16u(ring, i, RING);
}

__device__ __forceinline__ void ring_st(uint8_t* ring, uint32_t i, u32x4 v, int32_t nb)
{
	if (i + uint32_t(nb) <= uint32_t(RING)) {
		lds_store_n(ring + i, v, nb);
	} else {
		uint8_t t[16];
		__builtin_memcpy(t, &v, 16);
		for (int k = 0; k < nb; ++k) {
			uint32_t j = i + k;
			j -= (j >= uint32_t(RING)) ? uint32_t(RING) : 0u;
			ring[j] = t[k];
		}
	}
}

// Next sequence start from the batch table, or parsed when the table has
// no entry (long extensions, block end, positions past the batch).  -1:
// malformed.
__device__ __forceinline__ int32_t nstep(const Lds& W, const Src& S, int32_t p, int32_t n)
{
	(void)W;
	return step(S, p, n).next;
}

// Workgroup exclusive prefix sums of two values (lane order).
__device__ __forceinline__ void wg_excl_scan2(Lds& W, int32_t v0, int32_t v1, int32_t& x0,
                                              int32_t& x1, int32_t& t0, int32_t& t1)
{
	const int32_t tid = int32_t(threadIdx.x);
	const int32_t lane = tid & 63, wave = tid >> 6;
	const int32_t i0 = wave_incl_scan(v0), i1 = wave_incl_scan(v1);
	__syncthreads();
	if (lane == 63) {
		W.wsum[wave] = i0;
		W.wsum2[wave] = i1;
	}
	__syncthreads();
	int32_t b0 = 0, b1 = 0, a0 = 0, a1 = 0;
#pragma unroll
	for (int w = 0; w < WAVES; ++w) {
		const int32_t y0 = W.wsum[w], y1 = W.wsum2[w];
		b0 += (w < wave) ? y0 : 0;
		b1 += (w < wave) ? y1 : 0;
		a0 += y0;
		a1 += y1;
	}
	x0 = b0 + i0 - v0;
	x1 = b1 + i1 - v1;
	t0 = a0;
	t1 = a1;
}

// Batch output bytes [a, b) marked written (LDS bitmap, one bit per byte).
__device__ __forceinline__ void done_mark(uint32_t* done, int32_t a, int32_t b)
{
	for (int32_t w = a >> 5; (w << 5) < b; ++w) {
		const int32_t lo = (a > (w << 5)) ? a - (w << 5) : 0;
		const int32_t hi = (b < (w << 5) + 32) ? b - (w << 5) : 32;
		const uint32_t m = (hi == 32 ? 0xffffffffu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
		atomicOr(&done[w], m);
	}
}

__device__ __forceinline__ bool done_check(const uint32_t* done, int32_t a, int32_t b)
{
	bool ok = true;
	for (int32_t w = a >> 5; ok && (w << 5) < b; ++w) {
		const int32_t lo = (a > (w << 5)) ? a - (w << 5) : 0;
		const int32_t hi = (b < (w << 5) + 32) ? b - (w << 5) : 32;
		const uint32_t m = (hi == 32 ? 0xffffffffu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
		const uint32_t v = __hip_atomic_load(&done[w], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
		ok = (v & m) == m;
	}
	return ok;
}

// 16 compressed bytes at block-relative sp (staged LDS, else HBM dwords).
__device__ __forceinline__ u32x4 lit16(const Lds& W, const Src& S, int32_t sp, int32_t n)
{
	if (sp + 16 <= S.hi)
		return ld16u(W.inb, uint32_t(sp - S.s + S.mis), 1u << 30);
	cg8* g = S.in + sp;
	u32x4 v;
	v.x = ld32u_cached(g);
	v.y = sp + 4 < n ? ld32u_cached(g + 4) : 0u;
	v.z = sp + 8 < n ? ld32u_cached(g + 8) : 0u;
	v.w = sp + 12 < n ? ld32u_cached(g + 12) : 0u;
	return v;
}

// Match with offset off < 16 (period off): its bytes repeat the off source
// bytes before dm.  The phase-0 pattern (8 bytes when off <= 8, else 16) is
// stored every off*floor(width/off) bytes; overlapping stores write equal
// bytes.  Lanes li, li+cnt, ... of the cooperating group take the stores.
__device__ __forceinline__ void pattern_fill(Lds& W, int32_t oring, int32_t dm, int32_t q,
                                             int32_t off, int32_t ml, int32_t li, int32_t cnt)
{
	const u32x4 sv = ring_ld16(W.ring, ridx(oring, q));
	u32x4 pv;
	int32_t width, stp;
	make_pattern(uint64_t(sv.x) | (uint64_t(sv.y) << 32), uint64_t(sv.z) | (uint64_t(sv.w) << 32),
	             off, pv, width, stp);
	for (int32_t k = stp * li; k < ml; k += stp * cnt) {
		const int32_t nb = (ml - k < width) ? ml - k : width;
		ring_st(W.ring, ridx(oring, dm + k), pv, nb);
	}
}

// One lane copies a match of ml bytes from batch-relative q to dm
// (lz4ada.adb:845-904, overlap-safe).
__device__ __forceinline__ void match_copy_lane(Lds& W, int32_t oring, int32_t dm, int32_t q,
                                                int32_t off, int32_t ml)
{
	if (off >= 16) {
		for (int32_t k = 0; k < ml; k += 16) {
			const int32_t nb = (ml - k < 16) ? ml - k : 16;
			ring_st(W.ring, ridx(oring, dm + k), ring_ld16(W.ring, ridx(oring, q + k)), nb);
		}
	} else {
		pattern_fill(W, oring, dm, q, off, ml, 0, 1);
	}
}

// The whole wave copies one long match: steps of P = min(off rounded down
// to 16, 1024) bytes, whose sources all precede the step.
__device__ __forceinline__ void match_copy_wave(Lds& W, int32_t oring, int32_t dm, int32_t q,
                                                int32_t off, int32_t ml)
{
	const int32_t lane = int32_t(threadIdx.x & 63u);
	if (off >= 16) {
		const int32_t P = (off & ~15) < 1024 ? (off & ~15) : 1024;
		for (int32_t b = 0; b < ml; b += P) {
			const int32_t c = b + 16 * lane;
			if (16 * lane < P && c < ml) {
				const int32_t nb = (ml - c < 16) ? ml - c : 16;
				ring_st(W.ring, ridx(oring, dm + c), ring_ld16(W.ring, ridx(oring, q + c)), nb);
			}
			asm volatile("" ::: "memory");  // in-order LDS: next step sees these
		}
	} else {
		pattern_fill(W, oring, dm, q, off, ml, lane, 64);
	}
}

// Diagnostic build only (make stamps): per-phase s_memtime sums taken by
// thread 0 right after each phase's barrier (phase wall time), plus counts.
enum WgStamp { WS_STAGE, WS_WALK, WS_CONT, WS_PATH, WS_OFFS, WS_COPY, WS_FLUSH, WS_BATCHES,
	       WS_SLOWPATH, WS_ITERS, WS_CUTS, WS_CP_PARSE, WS_CP_READY, WS_CP_LIT, WS_CP_MATCH,
	       WS_CP_REST, WS_N };
#ifdef LZ4ADA_STAMPS
__device__ unsigned long long g_wg_stamps[WS_N];
#define WSTAMP_DECL uint64_t ws_acc[WS_N] = {}; uint64_t ws_t = __builtin_amdgcn_s_memtime()
#define WSTAMP(ph)                                                          \
	do {                                                                \
		const uint64_t _t = __builtin_amdgcn_s_memtime();           \
		ws_acc[ph] += _t - ws_t;                                    \
		ws_t = _t;                                                  \
	} while (0)
#define WSTAMP_COUNT(ph, v) (ws_acc[ph] += uint64_t(v))
#define CSTAMP(ph)                                                          \
	do {                                                                \
		asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
		const uint64_t _t = __builtin_amdgcn_s_memtime();           \
		cs_acc[ph - WS_CP_PARSE] += _t - cs_t;                      \
		cs_t = _t;                                                  \
	} while (0)
#define WSTAMP_FLUSH()                                                      \
	do {                                                                \
		if (threadIdx.x == 0)                                       \
			for (int _i = 0; _i < WS_N; ++_i)                   \
				atomicAdd(&g_wg_stamps[_i], (unsigned long long)ws_acc[_i]); \
	} while (0)
#else
#define WSTAMP_DECL
#define WSTAMP(ph)
#define WSTAMP_COUNT(ph, v)
#define CSTAMP(ph)
#define WSTAMP_FLUSH()
#endif

}  // namespace wg

using namespace wg;

__global__ __launch_bounds__(LANES) void k_decode_wg(const uint8_t* __restrict__ frame,
                                                     uint64_t frame_len,
                                                     const lz4ada_block_desc* __restrict__ desc,
                                                     uint32_t nblocks, uint8_t* __restrict__ out,
                                                     lz4ada_block_status* __restrict__ status)
{
	__shared__ Lds W;
	const uint32_t b = blockIdx.x;
	if (b >= nblocks)
		return;
	const int32_t tid = int32_t(threadIdx.x);
	const lz4ada_block_desc d = desc[b];
	cg8* __restrict__ in = gptr(frame) + d.in_off;
	g8* __restrict__ ob = gptr(out) + d.out_off;
	const int32_t n = int32_t(d.in_len);
	const int32_t cap = int32_t(d.out_cap);
	const uintptr_t lim_addr = reinterpret_cast<uintptr_t>(frame) + frame_len;

	if (d.flags & LZ4ADA_BLOCK_STORED) {
		// stored block: plain copy (lz4ada.adb:686-694)
		if (n <= cap) {
			for (int32_t i = tid; i < n; i += LANES)
				ob[i] = in[i];
		}
		if (tid == 0) {
			status[b].code = n <= cap ? int32_t(DS_OK) : int32_t(DS_RETRY);
			status[b].aux = 0;
			status[b].detail = 0;
			status[b].err_out_pos = 0;
			status[b].out_len = n <= cap ? uint32_t(n) : 0u;
		}
		return;
	}

	int32_t s = 0;  // exact chain position (block-relative), uniform
	int32_t o = 0;  // output bytes flushed, uniform
	int32_t code = DS_OK;
	int32_t guard = 0;
	WSTAMP_DECL;

	while (s < n) {
		if (++guard > n + 8) {  // every batch advances s
			code = DS_INTERNAL;
			break;
		}
		// ------------------------------------------------------ stage
		Src S;
		S.in = in;
		S.inb = W.inb;
		S.s = s;
		S.mis = int32_t((reinterpret_cast<uintptr_t>(in) + uint32_t(s)) & 15u);
		S.hi = (n - s < BATCH_IN + IN_OVH) ? n : s + BATCH_IN + IN_OVH;
		{
			const uintptr_t base = (reinterpret_cast<uintptr_t>(in) + uint32_t(s)) & ~uintptr_t(15);
			const int32_t nchunk = (S.hi - s + S.mis + 15) >> 4;
			for (int32_t c = tid; c < nchunk; c += LANES) {
				const uintptr_t ga = base + 16u * uint32_t(c);
				u32x4 v;
				if (ga + 16 <= lim_addr) {
					v = *reinterpret_cast<const GLOBAL u32x4*>(ga);
				} else {
					uint8_t t[16];
					for (int k = 0; k < 16; ++k)
						t[k] = (ga + k < lim_addr) ? *reinterpret_cast<cg8*>(ga + k) : 0;
					__builtin_memcpy(&v, t, 16);
				}
				*reinterpret_cast<u32x4*>(&W.inb[16 * c]) = v;
			}
		}
		if (tid == 0) {
			W.first_term = LANES;
			W.fail = 0;
			W.cut_idx = INT32_MAX;
		}
		__syncthreads();
		WSTAMP(WS_STAGE);
		WSTAMP_COUNT(WS_BATCHES, 1);

		const int32_t bend = (n - s < BATCH_IN) ? n : s + BATCH_IN;
		const int32_t bi = s + tid * REG;
		const bool live = bi < bend;
		const int32_t ei = (bi + REG < bend) ? bi + REG : bend;

		// ------------------------------------------------------ own walk
		int32_t x = -1;
		{
			uint32_t v = 0;
			if (live) {
				int32_t p = bi;
				while (p < ei) {
					v |= 1u << (p - bi);
					p = nstep(W, S, p, n);
					if (p < 0)
						break;
				}
				x = p;
			}
			W.vis[tid] = v;
		}
		__syncthreads();
		WSTAMP(WS_WALK);

		// ------------------------------------------------------ continuation
		{
			uint8_t lk = LK_NONE;
			int32_t p = x, tgt = TERM;
			if (live && x >= 0) {
				int32_t kc = -1;
				uint32_t vk = 0;
				for (int32_t steps = 0;; ++steps) {
					if (p >= bend) {
						lk = LK_END;
						break;
					}
					const int32_t k = (p - s) >> 5;
					if (k != kc) {
						kc = k;
						vk = W.vis[k];
					}
					if ((vk >> ((p - s) & 31)) & 1u) {
						lk = LK_LANE;
						tgt = k;
						break;
					}
					if (steps >= CMAX) {
						lk = LK_TRUNC;
						break;
					}
					p = nstep(W, S, p, n);
					if (p < 0) {
						lk = LK_BAD;
						break;
					}
				}
			} else if (live) {
				lk = LK_BAD;  // own walk hit a malformed sequence
			}
			W.X[tid] = x;
			W.sp[tid] = p;
			W.link[tid] = lk;
			W.J[0][tid] = uint16_t(tgt);
			W.entry[tid] = -1;
			W.eR[tid] = INT32_MAX;
			if (tid == 0) {
				for (int l = 0; l <= LEVELS; ++l)
					W.J[l][TERM] = TERM;
			}
			if (live && lk != LK_LANE)
				atomicMin(&W.first_term, tid);
		}
		__syncthreads();
		WSTAMP(WS_CONT);

		// ------------------------------------------------------ path
		// Lane 0 starts on the chain; lane i's continuation links it to the
		// lane whose walk it joined.  Following the links from lane 0 gives
		// the path; each path lane's entry is its predecessor's stop.
		{
			const int32_t ft = W.first_term;
			const bool chain = (tid >= ft) || (W.J[0][tid] == uint16_t(tid + 1));
			if (__syncthreads_and(chain)) {
				if (tid <= ft)
					W.entry[tid] = tid == 0 ? s : W.sp[tid - 1];
				if (tid == 0)
					W.lastp = ft;
			} else {
				WSTAMP_COUNT(WS_SLOWPATH, 1);
				for (int l = 0; l < LEVELS; ++l) {
					const uint16_t j = W.J[l][tid];
					W.J[l + 1][tid] = W.J[l][j];
					__syncthreads();
				}
				int32_t xnode = 0;  // path node number tid
#pragma unroll
				for (int l = 0; l < LEVELS; ++l)
					if ((tid >> l) & 1)
						xnode = W.J[l][xnode];
				W.node[tid] = uint16_t(xnode);
				__syncthreads();
				if (xnode != TERM) {
					W.entry[xnode] = tid ? W.sp[W.node[tid - 1]] : s;
					if (tid == LANES - 1 || W.node[tid + 1] == TERM)
						W.lastp = xnode;
				}
			}
		}
		__syncthreads();
		const int32_t lastp = W.lastp;  // last lane of the path
		if (W.link[lastp] == LK_BAD || W.link[lastp] == LK_NONE) {
			code = DS_RETRY;  // the chain meets a malformed sequence
			break;
		}
		WSTAMP(WS_PATH);

		// ------------------------------------------------------ regions
		// Lane k takes the true sequences starting in its region; the first
		// one is the smaller of its own path entry and the first stop any
		// path continuation made in the region.
		const int32_t nexts0 = W.sp[lastp];  // end of this batch's chain
		{
			const int32_t e = W.entry[tid];
			if (e >= 0) {
				atomicMin(&W.eR[(e - s) >> 5], e);
				if (W.link[tid] == LK_LANE || tid == lastp) {
					int32_t p = W.X[tid];
					const int32_t stop = W.sp[tid];
					int32_t lastr = -1;
					while (p < stop) {
						const int32_t r = (p - s) >> 5;
						if (r != lastr) {
							atomicMin(&W.eR[r], p);
							lastr = r;
						}
						p = nstep(W, S, p, n);
					}
				}
			}
		}
		__syncthreads();
		const int32_t ek = W.eR[tid];
		const int32_t pend = (bi + REG < nexts0) ? bi + REG : nexts0;
		int32_t mydec = 0, myn = 0;
		bool fail = false;
		if (ek < pend) {
			int32_t p = ek;
			while (p < pend) {
				const Tok t = parse(S, p, n);
				if (t.next < 0) {
					fail = true;
					break;
				}
				mydec += t.L + t.ml;
				++myn;
				p = t.next;
			}
		}
		int32_t O, TBk, total, ntot;
		wg_excl_scan2(W, mydec, myn, O, TBk, total, ntot);
		// records (and the batch cut: the first sequence past MAXTOK or OUT_CAP)
		if (!fail && myn) {
			int32_t p = ek, xo = O, idx = TBk;
			for (int32_t j = 0; j < myn; ++j) {
				const Tok t = parse(S, p, n);
				if (idx >= MAXTOK || xo + t.L + t.ml > OUT_CAP) {
					atomicMin(&W.cut_idx, idx);
					break;
				}
				W.rec[idx] = uint32_t(p - s) | (uint32_t(xo) << 16);
				xo += t.L + t.ml;
				++idx;
				p = t.next;
			}
		}
		for (int32_t w = tid; w < NDONE; w += LANES)
			W.done[w] = 0u;
		if (fail)
			atomicOr(&W.fail, 1);
		__syncthreads();
		if (W.fail) {
			code = DS_RETRY;
			break;
		}
		const int32_t cut = W.cut_idx;
		if (cut != INT32_MAX && myn && cut >= TBk && cut < TBk + myn) {
			// this region holds the first sequence that does not fit
			int32_t p = ek, xo = O;
			for (int32_t j = TBk; j < cut; ++j) {
				const Tok t = parse(S, p, n);
				xo += t.L + t.ml;
				p = t.next;
			}
			W.next_s = p;
			W.total = xo;
			W.ntok = cut;
		}
		if (tid == 0 && cut == INT32_MAX) {
			W.next_s = nexts0;
			W.total = total;
			W.ntok = ntot;
		}
		__syncthreads();
		const int32_t T = W.total, nexts = W.next_s, nseq = W.ntok;
		if (nseq == 0 || o + T > cap) {
			code = DS_RETRY;  // a sequence larger than a batch, or a slot overflow
			break;
		}
		WSTAMP(WS_OFFS);

		const int32_t oring = o % RING;

		// ------------------------------------------------------ copy
		// Rounds of LANES sequences in output order.  Literals first (no
		// dependencies), then the match once every source byte it reads from
		// this batch is marked done; bytes before the batch always are.
#ifdef LZ4ADA_STAMPS
		uint64_t cs_acc[5] = {};
		uint64_t cs_t = __builtin_amdgcn_s_memtime();
#endif
		for (int32_t base = 0; base < nseq; base += LANES) {
			const int32_t i = base + tid;
			const bool act = i < nseq;
			Tok t = {};
			int32_t xo = 0;
			if (act) {
				const uint32_t r = W.rec[i];
				t = parse(S, s + int32_t(r & 0xffffu), n);
				xo = int32_t(r >> 16);
			}
			CSTAMP(WS_CP_PARSE);
			if (act && t.L <= LONG) {
				for (int32_t k = 0; k < t.L; k += 16) {
					const int32_t nb = (t.L - k < 16) ? t.L - k : 16;
					ring_st(W.ring, ridx(oring, xo + k), lit16(W, S, t.lit + k, n), nb);
				}
			}
			// long literal runs: the whole wave, one run at a time
			for (uint64_t lm = __ballot(act && t.L > LONG); lm; lm &= lm - 1) {
				const int k = __ffsll((long long)lm) - 1;
				const int32_t Lk = __shfl(t.L, k), litk = __shfl(t.lit, k), xk = __shfl(xo, k);
				for (int32_t c = 16 * (tid & 63); c < Lk; c += 1024) {
					const int32_t nb = (Lk - c < 16) ? Lk - c : 16;
					ring_st(W.ring, ridx(oring, xk + c), lit16(W, S, litk + c, n), nb);
				}
			}
			CSTAMP(WS_CP_LIT);
			if (act) {
				if (t.L) {
					asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
					done_mark(W.done, xo, xo + t.L);
				}
				if (t.ml && o + xo + t.L - t.off < 0)
					fail = true;  // reference before the block start (D2)
			}
			CSTAMP(WS_CP_READY);
			bool pend_m = act && t.ml && !fail;
			int32_t iters = 0;
			asm volatile("; MARK_MATCH_BEGIN" ::: "memory");
			while (__any(pend_m)) {
				if (++iters > (1 << 22)) {
					fail = true;
					break;
				}
				bool progressed = false;
				const int32_t dm = xo + t.L;
				const int32_t q = dm - t.off;
				bool ready = false;
				if (pend_m) {
					const int32_t e = (q + t.ml < dm) ? q + t.ml : dm;
#ifdef LZ4ADA_WG_EXP_NODEPS
					ready = true;
					(void)e;
#else
					ready = done_check(W.done, q > 0 ? q : 0, e);
#endif
				}
				if (pend_m && ready && t.ml <= LONG) {
					match_copy_lane(W, oring, dm, q, t.off, t.ml);
					asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
					done_mark(W.done, dm, dm + t.ml);
					pend_m = false;
					progressed = true;
				}
				// long matches: the whole wave, one at a time
				for (uint64_t lm = __ballot(pend_m && ready && t.ml > LONG); lm; lm &= lm - 1) {
					const int k = __ffsll((long long)lm) - 1;
					const int32_t dk = __shfl(dm, k), qk = __shfl(q, k);
					const int32_t ok = __shfl(t.off, k), mk = __shfl(t.ml, k);
					match_copy_wave(W, oring, dk, qk, ok, mk);
					if ((tid & 63) == k) {
						asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
						done_mark(W.done, dk, dk + mk);
						pend_m = false;
						progressed = true;
					}
				}
				if (!__any(progressed))
					__builtin_amdgcn_s_sleep(1);
			}
#ifdef LZ4ADA_STAMPS
			WSTAMP_COUNT(WS_ITERS, iters);
#endif
			asm volatile("; MARK_MATCH_END" ::: "memory");
			CSTAMP(WS_CP_MATCH);
			// no barrier: a wave moves on to its next sequences at once (they
			// only ever wait on lower-numbered ones, which always complete)
			CSTAMP(WS_CP_REST);
		}
#ifdef LZ4ADA_STAMPS
		for (int k = 0; k < 5; ++k)
			ws_acc[WS_CP_PARSE + k] += cs_acc[k];
#endif
		if (fail)
			atomicOr(&W.fail, 1);
		__syncthreads();
		if (W.fail) {
			code = DS_RETRY;
			break;
		}
		WSTAMP(WS_COPY);
		WSTAMP_COUNT(WS_CUTS, nexts != nexts0);

		// ------------------------------------------------------ flush
		{
			g8* dst = ob + o;
			const int32_t head = int32_t((16 - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u);
			const int32_t h = head < T ? head : T;
			if (tid < h)
				dst[tid] = W.ring[ridx(oring, tid)];
			const int32_t nv = (T - h) >> 4;
			for (int32_t i = tid; i < nv; i += LANES) {
				const u32x4 v = ring_ld16(W.ring, ridx(oring, h + 16 * i));
				*reinterpret_cast<GLOBAL u32x4*>(dst + h + 16 * i) = v;
			}
			for (int32_t i = h + nv * 16 + tid; i < T; i += LANES)
				dst[i] = W.ring[ridx(oring, i)];
		}
		// later batches read old output back from HBM (sources > 32 KiB back)
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		__syncthreads();
		WSTAMP(WS_FLUSH);
		o += T;
		s = nexts;
	}
	WSTAMP_FLUSH();

	if (tid == 0) {
		status[b].code = code;
		status[b].aux = 0;
		status[b].detail = 0;
		status[b].err_out_pos = 0;
		status[b].out_len = uint32_t(o);
	}
}

#ifdef LZ4ADA_STAMPS
extern "C" int lz4ada_debug_wg_stamps(unsigned long long* out, int reset)
{
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg_stamps), sizeof(unsigned long long) * WS_N) !=
	    hipSuccess)
		return -1;
	if (reset) {
		unsigned long long z[WS_N] = {};
		if (hipMemcpyToSymbol(HIP_SYMBOL(g_wg_stamps), z, sizeof z) != hipSuccess)
			return -1;
	}
	return WS_N;
}
#endif

hipError_t launch_decode_wg(const uint8_t* d_frame, uint64_t frame_len,
                            const lz4ada_block_desc* d_desc, uint32_t nblocks, uint8_t* d_out,
                            lz4ada_block_status* d_status, hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(k_decode_wg, dim3(nblocks), dim3(LANES), 0, stream, d_frame, frame_len,
	                   d_desc, nblocks, d_out, d_status);
	return hipGetLastError();
}

}  // namespace lz4ada
