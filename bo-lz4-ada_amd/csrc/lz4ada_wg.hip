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
constexpr int RING = 96 * 1024;             // output ring: 64 KiB history + batch
constexpr int OUT_CAP = 32 * 1024;          // output bytes per batch
constexpr int HIST = 65536;
static_assert(RING >= HIST + OUT_CAP, "ring must hold the window and a batch");
constexpr int CMAX = 96;                    // continuation steps before a batch is cut
constexpr int NDONE = OUT_CAP / 32 + 1;     // done-bitmap words
constexpr int TERM = LANES;                 // path terminal node
constexpr int LEVELS = 9;                   // log2(LANES)
static_assert((1 << LEVELS) == LANES, "doubling levels");

// link types of a lane's continuation
enum Link : uint8_t { LK_LANE = 0, LK_END = 1, LK_TRUNC = 2, LK_BAD = 3, LK_NONE = 4 };

struct alignas(16) Lds {
	uint8_t ring[RING];
	uint8_t inb[IN_STAGE];
	uint64_t vis[LANES];
	int32_t X[LANES];       // own-walk exit (-1: invalid token)
	int32_t sp[LANES];      // where the continuation stopped
	int32_t dec[LANES];     // decoded bytes of the own walk / of the path part
	int32_t cdec[LANES];    // decoded bytes of the continuation
	int32_t O[LANES + 1];   // batch-relative output start of each region's sequences
	int32_t eR[LANES];      // first true sequence starting in each region
	int32_t entry[LANES];   // exact chain entry (path lanes), else -1
	uint16_t J[LEVELS + 1][LANES + 1];
	uint16_t node[LANES];
	uint32_t done[NDONE];   // batch output bytes written (phase bitmap)
	uint8_t link[LANES];
	int32_t wsum[WAVES];
	int32_t first_term;
	int32_t lastp;
	int32_t next_s;
	int32_t total;
	int32_t fail;
	int32_t cutlane;  // first path lane starting at or past OUT_CAP
	int32_t cutdone;  // a lane cut the batch inside its sequences
	int32_t fail_dbg;
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

// ring index of batch-relative output position rel (rel >= -HIST)
__device__ __forceinline__ int32_t ridx(int32_t oring, int32_t rel)
{
	int32_t i = oring + rel;
	i += (i < 0) ? RING : 0;
	i -= (i >= RING) ? RING : 0;
	return i;
}

__device__ __forceinline__ u32x4 ring_ld16(const uint8_t* ring, int32_t i)
{
	return ld16u(ring, uint32_t(i), RING);
}

__device__ __forceinline__ void ring_st(uint8_t* ring, int32_t i, u32x4 v, int32_t nb)
{
	if (i + nb <= RING) {
		lds_store_n(ring + i, v, nb);
	} else {
		uint8_t t[16];
		__builtin_memcpy(t, &v, 16);
		for (int k = 0; k < nb; ++k) {
			int32_t j = i + k;
			j -= (j >= RING) ? RING : 0;
			ring[j] = t[k];
		}
	}
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

// Workgroup exclusive prefix sum (lane order); returns the total in *tot.
__device__ __forceinline__ int32_t wg_excl_scan(Lds& W, int32_t v, int32_t* tot)
{
	const int32_t tid = int32_t(threadIdx.x);
	const int32_t lane = tid & 63, wave = tid >> 6;
	const int32_t inc = wave_incl_scan(v);
	if (lane == 63)
		W.wsum[wave] = inc;
	__syncthreads();
	int32_t base = 0, all = 0;
#pragma unroll
	for (int w = 0; w < WAVES; ++w) {
		const int32_t x = W.wsum[w];
		base += (w < wave) ? x : 0;
		all += x;
	}
	*tot = all;
	return base + inc - v;
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
			W.cutlane = LANES;
			W.cutdone = 0;
			W.fail_dbg = 0;
		}
		__syncthreads();
		WSTAMP(WS_STAGE);
		WSTAMP_COUNT(WS_BATCHES, 1);

		// ------------------------------------------------------ own walk
		const int32_t bend = (n - s < BATCH_IN) ? n : s + BATCH_IN;
		const int32_t bi = s + tid * REG;
		const bool live = bi < bend;
		int32_t x = -1, dsum = 0;
		{
			uint64_t v = 0;
			if (live) {
				const int32_t ei = (bi + REG < bend) ? bi + REG : bend;
				int32_t p = bi;
				while (p < ei) {
					v |= uint64_t(1) << (p - bi);
					const Step t = step(S, p, n);
					if (t.next < 0) {
						p = -1;
						break;
					}
					dsum += t.dec;
					p = t.next;
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
			int32_t p = x, cd = 0, tgt = TERM;
			if (live && x >= 0) {
				for (int32_t steps = 0;; ++steps) {
					if (p >= bend) {
						lk = LK_END;
						break;
					}
					const int32_t k = (p - s) / REG;
					if ((W.vis[k] >> (p - (s + k * REG))) & 1u) {
						lk = LK_LANE;
						tgt = k;
						break;
					}
					if (steps >= CMAX) {
						lk = LK_TRUNC;
						break;
					}
					const Step t = step(S, p, n);
					if (t.next < 0) {
						lk = LK_BAD;
						break;
					}
					cd += t.dec;
					p = t.next;
				}
			} else if (live) {
				lk = LK_BAD;  // own walk hit an invalid token
			}
			W.X[tid] = x;
			W.sp[tid] = p;
			W.dec[tid] = dsum;
			W.cdec[tid] = cd;
			W.link[tid] = lk;
			W.J[0][tid] = uint16_t(tgt);
			W.entry[tid] = -1;
			W.eR[tid] = INT32_MAX;
			if (tid == 0) {
				W.J[0][TERM] = TERM;
				for (int l = 1; l <= LEVELS; ++l)
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
				// common case: every lane up to the first terminal links to the next
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
		WSTAMP(WS_PATH);
		{
			const uint8_t lk = W.link[lastp];
			if (lk == LK_BAD || lk == LK_NONE) {
				code = DS_RETRY;  // the chain meets a malformed sequence
				break;
			}
		}

		// ------------------------------------------------------ region entries
		// Re-base the work on regions: lane k copies the true sequences that
		// start in [b_k, b_{k+1}).  Their first one is the smaller of the
		// lane's own path entry and the first stop a path continuation made
		// in region k.
		const int32_t nexts0 = W.sp[lastp];  // end of this batch's chain
		{
			const int32_t e = W.entry[tid];
			if (e >= 0) {
				atomicMin(&W.eR[(e - s) / REG], e);
				const uint8_t lk = W.link[tid];
				if (lk == LK_LANE || tid == lastp) {
					int32_t p = W.X[tid];
					const int32_t stop = W.sp[tid];
					int32_t lastr = -1;
					while (p < stop) {
						const int32_t r = (p - s) / REG;
						if (r != lastr) {
							atomicMin(&W.eR[r], p);
							lastr = r;
						}
						p = step(S, p, n).next;
					}
				}
			}
		}
		__syncthreads();
		const int32_t ek = W.eR[tid];
		const int32_t pend = (bi + REG < nexts0) ? bi + REG : nexts0;
		int32_t mydec = 0;
		if (ek < pend) {
			int32_t p = ek;
			while (p < pend) {
				const Step t = step(S, p, n);
				mydec += t.dec;
				p = t.next;
			}
		}
		int32_t total;
		const int32_t O = wg_excl_scan(W, mydec, &total);
		if (tid == 0) {
			W.next_s = nexts0;
			W.total = total;
		}
		W.O[tid] = O;
		if (O >= OUT_CAP && mydec > 0)
			atomicMin(&W.cutlane, tid);
		for (int32_t w = tid; w < NDONE; w += LANES)
			W.done[w] = 0u;
		if (tid == 0)
			W.O[LANES] = total;
		__syncthreads();
		WSTAMP(WS_OFFS);
#ifdef LZ4ADA_WG_CHECK
		if (tid == 0) {
			int32_t p = s, sum = 0, nt = 0;
			while (p < nexts0) {
				const Tok t = parse(S, p, n);
				if (t.next < 0)
					break;
				sum += t.L + t.ml;
				p = t.next;
				++nt;
			}
			if (p != nexts0 || sum != total)
				printf("[wgcheck] b=%u s=%d o=%d lastp=%d link=%d next=%d walk=%d total=%d "
				       "walksum=%d ntok=%d fast=%d\n",
				       b, s, o, lastp, int(W.link[lastp]), nexts0, p, total, sum, nt,
				       int(W.first_term));
		}
#endif
		if (o + (total < OUT_CAP ? total : OUT_CAP) > cap) {
			code = DS_RETRY;  // slot overflow: exact path reports D5
			break;
		}

		// ------------------------------------------------------ copy
		// Phase A: every lane copies the literals of its region's sequences
		// (no dependencies) and marks those output bytes done in a bitmap.
		// Phase B: matches, in order per lane; a match runs once every
		// source byte it reads is marked done (bytes before the batch always
		// are), then marks its own bytes.  A lane only waits on earlier
		// output, so the batch always completes.
		const int32_t oring = o % RING;
		// stores never pass the lane's range (or the batch cap)
		const int32_t lim = (O + mydec < OUT_CAP) ? O + mydec : OUT_CAP;
		int32_t ntok = 0;  // sequences this lane owns in this batch (after a cut)
		bool fail = false;
		{
			int32_t p = ek, xo = O;
			bool go = (mydec > 0) && O < OUT_CAP;
			while (go && p < pend) {
				const Tok t = parse(S, p, n);
				if (t.next < 0 || (t.ml && o + xo + t.L - t.off < 0)) {
					fail = true;  // malformed, or reaches before the block (D2)
					break;
				}
				if (xo + t.L + t.ml > OUT_CAP) {
					if (xo == 0)
						fail = true;  // one sequence larger than a batch
					W.next_s = p;
					W.total = xo;
					W.cutdone = 1;
					break;
				}
				for (int32_t k = 0; k < t.L; k += 16) {
					const int32_t sp = t.lit + k;
					u32x4 v;
					if (sp + 16 <= S.hi) {
						v = ld16u(W.inb, uint32_t(sp - s + S.mis), 1u << 30);
					} else {
						uint8_t tb[16];
						for (int j = 0; j < 16; ++j)
							tb[j] = (sp + j < n) ? uint8_t(S.rd(sp + j)) : 0;
						__builtin_memcpy(&v, tb, 16);
					}
					const int32_t room = lim - (xo + k);
					ring_st(W.ring, ridx(oring, xo + k), v, room < 16 ? room : 16);
				}
				xo += t.L + t.ml;
				p = t.next;
				++ntok;
			}
		}
		__syncthreads();
		// literal bytes done (a separate pass keeps the atomics off the copy)
		{
			int32_t p = ek, xo = O;
			for (int32_t i = 0; i < ntok; ++i) {
				const Tok t = parse(S, p, n);
				if (t.L)
					done_mark(W.done, xo, xo + t.L);
				xo += t.L + t.ml;
				p = t.next;
			}
		}
		__syncthreads();
		WSTAMP(WS_CP_LIT);
		{
			int32_t p = ek, xo = O, left = ntok;
			int32_t iters = 0;
			bool have = false;
			Tok t = {};
			while (__any(left > 0)) {
				if (++iters > (1 << 22)) {
					fail = true;
					break;
				}
				bool progressed = false;
				if (left > 0) {
					if (!have) {
						t = parse(S, p, n);
						have = true;
					}
					const int32_t dm = xo + t.L;   // match start (batch-relative)
					const int32_t q = dm - t.off;  // match source
					bool ready = true;
					if (t.ml) {
						// source bytes before the match start: [q, min(q+ml, dm))
						const int32_t e = (q + t.ml < dm) ? q + t.ml : dm;
						ready = done_check(W.done, q > 0 ? q : 0, e);
					}
					if (ready) {
						if (t.ml) {
							const int32_t off = t.off;
							if (off >= 16) {
								for (int32_t k = 0; k < t.ml; k += 16) {
									const int32_t nb = (t.ml - k < 16) ? t.ml - k : 16;
									const u32x4 v = ring_ld16(W.ring, ridx(oring, q + k));
									ring_st(W.ring, ridx(oring, dm + k), v, nb);
								}
							} else {
								// period off < 16: the 16-byte pattern of phase 0,
								// stored every off*floor(16/off) bytes
								const u32x4 sv = ring_ld16(W.ring, ridx(oring, q));
								unsigned __int128 x;
								__builtin_memcpy(&x, &sv, 16);
								x &= (((unsigned __int128)1) << (8 * off)) - 1;
								for (int32_t w = off; w < 16; w <<= 1)
									x |= x << (8 * w);
								u32x4 pv;
								__builtin_memcpy(&pv, &x, 16);
								const int32_t stp = off * (16 / off);
								for (int32_t k = 0; k < t.ml; k += stp) {
									const int32_t nb = (t.ml - k < 16) ? t.ml - k : 16;
									ring_st(W.ring, ridx(oring, dm + k), pv, nb);
								}
							}
							asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
							done_mark(W.done, dm, dm + t.ml);
						}
						xo += t.L + t.ml;
						p = t.next;
						have = false;
						--left;
						progressed = true;
					}
				}
				if (!__any(progressed))
					__builtin_amdgcn_s_sleep(1);
			}
#ifdef LZ4ADA_STAMPS
			atomicMax(&W.fail_dbg, iters);
#endif
		}
		if (fail)
			atomicOr(&W.fail, 1);
		__syncthreads();
		if (W.fail) {
			code = DS_RETRY;
			break;
		}
		WSTAMP(WS_COPY);
		WSTAMP_COUNT(WS_CUTS, W.cutdone || W.cutlane < LANES);
#ifdef LZ4ADA_STAMPS
		WSTAMP_COUNT(WS_ITERS, W.fail_dbg);
#endif
		int32_t T = W.total, nexts = W.next_s;
		if (!W.cutdone && W.cutlane < LANES) {
			// the batch is full exactly at a region boundary
			T = W.O[W.cutlane];
			nexts = W.eR[W.cutlane];
		}

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
		__syncthreads();
#ifdef LZ4ADA_WG_CHECK
		if (tid == 0 && b == 0)
			printf("[wgbatch] s=%d o=%d T=%d next=%d lastp=%d ft=%d\n", s, o, T, nexts, lastp,
			       W.first_term);
#endif
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
