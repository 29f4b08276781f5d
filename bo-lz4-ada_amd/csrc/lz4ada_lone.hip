// lz4ada_lone.hip -- one LZ4 block decoded by the whole GPU (a "lone" block:
// the streaming facade's Update hands over one block at a time, SURVEY §8f
// item 1, lib/lz4ada.adb:630-659).  The per-block decoders give a block one
// wave or one workgroup, so a lone 4 MiB block takes milliseconds; here every
// step is parallel over the block's bytes instead.
//
// Replaces lib/lz4ada.adb:716-904 (Decompress_Full_Block, Decompress_Sequence,
// Write_Output, Output_With_History) for a block that reads no history: any
// sequence the reference would reject, a reference before the block start or
// an output over the slot makes the block DS_RETRY, and the caller's exact
// path then gives the reference's result.
//
//  1. k_lone_windows -- one workgroup per window (512 B - 4 KiB) of the compressed
//     block.  Every byte position is parsed as if a sequence started there
//     (Decompress_Sequence's shape rules, lz4ada.adb:737-777), giving the
//     position after it and its output bytes; pointer jumping in LDS then
//     gives, for every position, the first chain position at or past the
//     window end (its exit) and the output bytes on the way.
//  2. k_lone_chain -- one workgroup: the true chain's entry into every
//     window.  Entry w+1 is the exit of entry w; all windows are guessed at
//     once (chains started at a wrong byte merge within a few sequences) and
//     the recurrence is iterated until nothing changes, then a prefix sum of
//     the windows' output bytes places each window in the output.
//  3. k_lone_words -- one workgroup per window: marks the true chain from the
//     window's entry (pointer doubling), places each sequence by a prefix
//     sum and writes one word per output byte, in tiles of consecutive words
//     (coalesced stores): a literal (bit 31 | byte) or the output position
//     the byte copies (Output_With_History's byte i = byte i - offset, which
//     also gives the overlap rule).
//  4. k_lone_resolve -- the copies resolved by pointer jumping over the
//     words (W[i] = W[W[i]] until every word is a literal), each workgroup
//     over its own slice of the output, reading the others' slices as they
//     go; then the bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4ada_internal.h"
#include "lz4ada_dev.h"

namespace lz4ada {

// Window size LW (compressed bytes per workgroup in steps 1 and 3): 512 B
// to 4 KiB by the block's compressed size and ratio (lone_window, host side).  Small
// windows give a small block more workgroups; large ones keep the chain
// step short where speculative chains do not merge (literal-heavy data).
constexpr int32_t LW_MIN = 512;
constexpr int32_t LT = 256;               // threads per workgroup
constexpr uint32_t NX_BAD = 0xFFFFFFFFu;  // not a sequence (or beyond what a window parses)
constexpr uint32_t LIT = 0x80000000u;     // word: a literal byte
constexpr int32_t RES_SLICE = 4096;       // largest output slice per workgroup in k_lone_resolve
constexpr int32_t MAX_RUN_L = 1 << 28;
static_assert(RES_SLICE % (4 * LT) == 0, "lone-decoder tiling");

struct LoneCtl {
	int32_t code;     // DS_OK, or DS_RETRY once any step declines
	uint32_t total;   // output bytes
	uint32_t nwin;
	uint32_t iters;   // k_lone_chain iterations (diagnostics)
};

// 16 bytes at byte a of the staged copy (a + 20 within the array): aligned
// dword reads and v_alignbyte.
__device__ __forceinline__ u32x4 lds16(const uint8_t* s, uint32_t a)
{
	const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (a & ~3u));
	const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4], sh = a & 3u;
	u32x4 v;
	v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
	v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
	v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
	v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
	return v;
}

__device__ __forceinline__ u32x4 gld16(cg8* p)
{
	u32x4 v;
	v.x = ld32u_cached(p);
	v.y = ld32u_cached(p + 4);
	v.z = ld32u_cached(p + 8);
	v.w = ld32u_cached(p + 12);
	return v;
}

// Byte x of the block (x < n): the staged copy or global memory.
struct LoneSrc {
	const uint8_t* s;  // LDS: bytes [ws, shi)
	int32_t ws, shi;
	cg8* in;
	__device__ __forceinline__ uint32_t at(int32_t x) const
	{
		if (__builtin_expect(x < shi, 1))
			return uint32_t(s[x - ws]);
		return uint32_t(in[x]);
	}
	// dword at x (x + 4 <= n)
	__device__ __forceinline__ uint32_t at4(int32_t x) const
	{
		if (__builtin_expect(x + 4 <= shi, 1)) {
			const uint32_t a = uint32_t(x - ws);
			const uint32_t* w = reinterpret_cast<const uint32_t*>(s + (a & ~3u));
			return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
		}
		return ld32u_cached(in + x);
	}
};

struct LoneSeq {
	uint32_t nx;  // position after the sequence (n: the last one), NX_BAD if malformed
	uint32_t os;  // output bytes
	int32_t lit, L, off, ml;
};

// A length extension at x (Process_Variable_Length, lz4ada.adb:724-735):
// bytes of 255 and one below, added to len; x ends past the last.  Scans 16
// bytes a step.  False if the block ends first, the length passes
// MAX_RUN_L, or more than gmax bytes would be read past the staged copy.
__device__ __forceinline__ bool lone_ext(const LoneSrc& S, int32_t& x, int32_t& len, int32_t n,
                                         int32_t gmax)
{
	int32_t g = 0;
	for (;;) {
		u32x4 v;
		if (x + 16 <= S.shi) {
			v = lds16(S.s, uint32_t(x - S.ws));
		} else if (x + 16 <= n) {
			g += 16;
			if (g > gmax)
				return false;
			v = gld16(S.in + x);
		} else {
			while (x < n) {
				const uint32_t e = S.at(x++);
				len += int32_t(e);
				if (e != 255u)
					return true;
				if (++g > gmax + 16)
					return false;
			}
			return false;
		}
		const uint32_t t0 = ~v.x, t1 = ~v.y, t2 = ~v.z, t3 = ~v.w;
		const int32_t j = t0 ? int32_t(__builtin_ctz(t0) >> 3)
		                     : t1 ? 4 + int32_t(__builtin_ctz(t1) >> 3)
		                          : t2 ? 8 + int32_t(__builtin_ctz(t2) >> 3)
		                               : t3 ? 12 + int32_t(__builtin_ctz(t3) >> 3) : 16;
		if (j == 16) {
			len += 16 * 255;
			x += 16;
			if (len > MAX_RUN_L)
				return false;
			continue;
		}
		const uint32_t c = j < 4 ? v.x : j < 8 ? v.y : j < 12 ? v.z : v.w;
		len += 255 * j + int32_t((c >> (8 * (j & 3))) & 0xFFu);
		x += j + 1;
		return true;
	}
}

// Decompress_Sequence's shape at p (the rules of parse_seq in
// lz4ada_idx.hip: lz4ada.adb:737-777 with the end-of-block rule :748-764).
// gmax bounds the extension bytes read past the staged copy: a speculative
// position in a run of 255s must not walk the block (k_lone_windows: a
// sequence over the bound is declined, NX_BAD); the true chain's sequences
// are parsed without bound (k_lone_words).
__device__ __forceinline__ LoneSeq lone_parse(const LoneSrc& S, int32_t p, int32_t n, int32_t gmax)
{
	LoneSeq q;
	q.nx = NX_BAD;
	q.os = 0;
	q.off = 0;
	q.ml = 0;
	const uint32_t t = S.at(p);
	int32_t L = int32_t(t >> 4), M = int32_t(t & 15u), x = p + 1;
	if (L == 15 && !lone_ext(S, x, L, n, gmax))
		return q;
	q.lit = x;
	q.L = L;
	x += L;
	if (x >= n) {
		if (x > n || M != 0)
			return q;
		q.nx = uint32_t(n);
		q.os = uint32_t(L);
		return q;
	}
	if (x + 1 >= n)
		return q;
	const int32_t off = int32_t(S.at(x) | (S.at(x + 1) << 8));
	if (off == 0)
		return q;
	x += 2;
	if (M == 15 && !lone_ext(S, x, M, n, gmax))
		return q;
	q.off = off;
	q.ml = M + 4;
	q.nx = uint32_t(x);
	q.os = uint32_t(L + q.ml);
	return q;
}

constexpr int32_t GMAX_SPEC = 4096;     // speculative parse: extension bytes past the stage
constexpr int32_t GMAX_TRUE = 1 << 24;  // true chain

__device__ __forceinline__ void lone_stage(uint8_t* s, cg8* in, int32_t ws, int32_t shi)
{
	for (int32_t i = int32_t(threadIdx.x) * 4; i < shi - ws; i += LT * 4) {
		if (ws + i + 4 <= shi) {
			const uint32_t v = ld32u_cached(in + ws + i);
			__builtin_memcpy(s + i, &v, 4);
		} else {
			for (int32_t k = 0; ws + i + k < shi; ++k)
				s[i + k] = in[ws + i + k];
		}
	}
	__syncthreads();
}

__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b)
{
	const uint32_t s = a + b;
	return (s < a || s > 0x7FFFFFFFu) ? 0x7FFFFFFFu : s;
}

// ---------------------------------------------------------------- step 2
constexpr int32_t CT = 1024;  // k_lone_chain threads

// The chain step's body for NT threads (CK windows per thread at most), E:
// nwin + 1 entries of LDS.
template <int32_t LW, int32_t NT, int32_t CK>
__device__ __forceinline__ void lone_chain_body(uint32_t* E, const uint32_t* __restrict__ exit_tab,
                                                const uint32_t* __restrict__ osum_tab,
                                                const uint32_t* __restrict__ guess, int32_t n, int32_t nwin,
                                                uint32_t cap, uint32_t* __restrict__ entry,
                                                uint32_t* __restrict__ obase, LoneCtl* __restrict__ ctl,
                                                lz4ada_block_status* __restrict__ st)
{
	constexpr int32_t CT = NT;
	__shared__ uint32_t wsum[CT / 64];
	__shared__ unsigned long long total64;
	__shared__ int32_t first_ch;  // the first window whose successor changed this pass
	const int32_t tid = int32_t(threadIdx.x);
	// entry w: the first chain position >= w * LW.  Guess: the exit most
	// positions of window w-1 reach (k_lone_windows).
	for (int32_t w = tid; w <= nwin; w += CT)
		E[w] = w > 0 ? guess[w] : 0u;
	if (tid == 0)
		total64 = 0;
	__syncthreads();
	// entry w+1 = the exit of entry w (or entry w itself when a sequence
	// jumps over window w); after k passes entries 1..k are exact
	uint32_t it = 0;
	for (;;) {
		++it;
		if (tid == 0)
			first_ch = INT32_MAX;
		uint32_t nv[CK];
#pragma unroll
		for (int32_t k = 0; k < CK; ++k) {
			const int32_t w = tid + k * CT;
			nv[k] = 0;
			if (w < nwin) {
				const uint32_t e = E[w];
				const uint32_t lim = uint32_t(min((w + 1) * LW, n));
				nv[k] = e == NX_BAD ? NX_BAD : (e < lim ? exit_tab[e] : e);
			}
		}
		__syncthreads();
		int ch = 0;
		int32_t lo = INT32_MAX;  // this thread's lowest window whose successor changed
#pragma unroll
		for (int32_t k = 0; k < CK; ++k) {
			const int32_t w = tid + k * CT;
			if (w < nwin && E[w + 1] != nv[k]) {
				E[w + 1] = nv[k];
				lo = min(lo, w);
				ch = 1;
			}
		}
		if (ch)
			atomicMin(&first_ch, lo);
		if (!__syncthreads_or(ch) || it > uint32_t(nwin) + 2)
			break;
		// still changing after two passes: the guesses are poor (sequences
		// too far apart for speculative chains to merge, e.g. long literal
		// runs).  One lane walks the first run of wrong entries, one
		// dependent lookup per window instead of one pass per window, up to
		// where its entry meets the stored one (the rest of that run was
		// already right); the next pass confirms, or finds the next run
		// (profiles/r04o_chain_walk.txt: a linked 256 KiB frame at 512-byte
		// windows 24 -> 11 us against walking every remaining window).  The
		// short walks are capped: from pass 2 + SHORT_WALKS on the
		// lane walks every remaining window, so inputs with many short wrong
		// runs cost at most a few passes more than the walk-to-the-end did.
		constexpr uint32_t SHORT_WALKS = 3;
		if (it >= 2) {
			if (tid == 0) {
				const bool to_end = it >= 2 + SHORT_WALKS;
				for (int32_t w = first_ch; w < nwin; ++w) {
					const uint32_t e = E[w];
					const uint32_t lim = uint32_t(min((w + 1) * LW, n));
					const uint32_t x = e == NX_BAD ? NX_BAD : (e < lim ? exit_tab[e] : e);
					if (!to_end && w > first_ch && E[w + 1] == x)
						break;
					E[w + 1] = x;
				}
			}
			__syncthreads();
		}
	}
	// each window's output bytes along the chain; an exclusive scan places
	// the windows (exact in 32 bits once the 64-bit total fits the slot)
	const int32_t per = (nwin + CT - 1) / CT;
	const int32_t w0 = tid * per;
	uint64_t mine = 0;
	bool bad = false;
	uint32_t os[CK];  // the windows' output bytes, kept for the placement (per <= CK)
#pragma unroll
	for (int32_t k = 0; k < CK; ++k) {
		const int32_t w = w0 + k;
		os[k] = 0;
		if (k < per && w < nwin) {
			const uint32_t e = E[w];
			if (e == NX_BAD)
				bad = true;
			else if (e < uint32_t(min((w + 1) * LW, n)))
				os[k] = osum_tab[e];
		}
	}
#pragma unroll
	for (int32_t k = 0; k < CK; ++k)
		mine += os[k];
	if (mine)
		atomicAdd(&total64, (unsigned long long)mine);
	const uint32_t m32 = uint32_t(min<uint64_t>(mine, 0x3FFFFFFFull));
	const uint32_t lane = lane_id(), wv = uint32_t(tid) >> 6;
	const uint32_t inc = uint32_t(wave_incl_scan(int32_t(m32)));
	if (lane == 63)
		wsum[wv] = inc;
	const bool anybad = __syncthreads_or(bad);
	uint32_t run = inc - m32;
	for (uint32_t j = 0; j < wv; ++j)
		run += wsum[j];
#pragma unroll
	for (int32_t k = 0; k < CK; ++k) {
		const int32_t w = w0 + k;
		if (k < per && w < nwin) {
			obase[w] = run;
			entry[w] = E[w];
			run += os[k];
		}
	}
	if (tid == 0) {
		const uint64_t total = total64;
		const bool ok = !anybad && E[nwin] == uint32_t(n) && total <= uint64_t(cap);
		ctl->code = ok ? int32_t(DS_OK) : int32_t(DS_RETRY);
		ctl->total = ok ? uint32_t(total) : 0u;
		ctl->nwin = uint32_t(nwin);
		ctl->iters = it;
		st->code = ctl->code;
		st->out_len = ctl->total;
	}
}

template <int32_t LW>
__global__ __launch_bounds__(CT) void k_lone_chain(const uint32_t* __restrict__ exit_tab,
                                                   const uint32_t* __restrict__ osum_tab,
                                                   const uint32_t* __restrict__ guess,
                                                   int32_t n, int32_t nwin, uint32_t cap,
                                                   uint32_t* __restrict__ entry,
                                                   uint32_t* __restrict__ obase,
                                                   LoneCtl* __restrict__ ctl,
                                                   lz4ada_block_status* __restrict__ st)
{
	extern __shared__ uint32_t E[];  // entries 0..nwin
	lone_chain_body<LW, CT, (int32_t(16) << 20) / LW / CT>(E, exit_tab, osum_tab, guess, n, nwin, cap, entry,
	                                                      obase, ctl, st);
}

// ---------------------------------------------------------------- step 1
// Also the entry guess for the next window: the exit most positions of this
// window reach (chains started at wrong bytes mostly merge into the true
// one before the window ends), counted in an LDS hash table.
//
// copy (not null): blk is pinned host memory, read here once; each window
// also writes its bytes -- the last one up to ncopy, the block's trailer --
// to the device copy that step 3 reads.
//
// done (not null, zero at launch): the windows count themselves off there,
// and the last one runs the chain step (lone_chain_body; nwin <= 2 LW, so
// its entries fit in X) and zeroes the count again -- one launch less for
// a small block.
template <int32_t LW>
__global__ __launch_bounds__(LT) void k_lone_windows(const uint8_t* __restrict__ blk, int32_t n,
                                                     uint32_t* __restrict__ exit_tab,
                                                     uint32_t* __restrict__ osum_tab,
                                                     uint32_t* __restrict__ nxt_tab,
                                                     uint32_t* __restrict__ guess,
                                                     uint8_t* __restrict__ copy, int32_t ncopy,
                                                     uint32_t* __restrict__ done, uint32_t cap,
                                                     uint32_t* __restrict__ entry,
                                                     uint32_t* __restrict__ obase, LoneCtl* __restrict__ ctl,
                                                     lz4ada_block_status* __restrict__ st)
{
	constexpr int32_t LP = LW / LT, LSTG = 2 * LW;
	__shared__ alignas(16) uint8_t s[LSTG + 32];
	__shared__ uint64_t X[LW];  // nx | os << 32
	__shared__ uint32_t best[LT / 64][2];
	const int32_t ws = int32_t(blockIdx.x) * LW, we = min(ws + LW, n);
	const int32_t shi = min(ws + LSTG, n);
	cg8* in = gptr(blk);
	lone_stage(s, in, ws, shi);
	if (copy) {
		const int32_t ce = blockIdx.x + 1 == gridDim.x ? ncopy : we;
		for (int32_t i = ws + int32_t(threadIdx.x); i < ce; i += LT)
			copy[i] = i < shi ? s[i - ws] : in[i];
	}
	const LoneSrc S{ s, ws, shi, in };
	const int32_t t0 = int32_t(threadIdx.x) * LP;
	for (int32_t k = 0; k < LP; ++k) {
		const int32_t p = ws + t0 + k;
		uint64_t v = uint64_t(NX_BAD);
		if (p < we) {
			const LoneSeq q = lone_parse(S, p, n, GMAX_SPEC);
			v = uint64_t(q.nx) | (uint64_t(q.os) << 32);
			nxt_tab[p] = q.nx;
		}
		X[t0 + k] = v;
	}
	__syncthreads();
	// pointer jumping: a position whose next lies inside the window takes
	// the next's next and adds its bytes (NX_BAD and exits stay)
	for (int r = 0; r < 12; ++r) {
		uint64_t nv[LP];
		int any = 0;
#pragma unroll
		for (int k = 0; k < LP; ++k) {
			const uint64_t v = X[t0 + k];
			const uint32_t nx = uint32_t(v);
			nv[k] = v;
			if (nx >= uint32_t(ws) && nx < uint32_t(we)) {
				const uint64_t u = X[nx - uint32_t(ws)];
				nv[k] = (u & 0xFFFFFFFFull) |
				        (uint64_t(sat_add(uint32_t(v >> 32), uint32_t(u >> 32))) << 32);
				any = 1;
			}
		}
		if (!__syncthreads_or(any))
			break;
#pragma unroll
		for (int k = 0; k < LP; ++k)
			X[t0 + k] = nv[k];
		__syncthreads();
	}
	uint32_t ex[LP];
#pragma unroll
	for (int k = 0; k < LP; ++k)
		ex[k] = uint32_t(X[t0 + k]);
	for (int32_t i = int32_t(threadIdx.x); i < we - ws; i += LT) {
		const uint64_t v = X[i];
		exit_tab[ws + i] = uint32_t(v);
		osum_tab[ws + i] = uint32_t(v >> 32);
	}
	__syncthreads();
	// the most common exit: keys and counts in the (now free) X array
	uint32_t* key = reinterpret_cast<uint32_t*>(X);
	uint32_t* cnt = key + LW;
	for (int32_t i = int32_t(threadIdx.x); i < LW; i += LT) {
		key[i] = NX_BAD;
		cnt[i] = 0;
	}
	__syncthreads();
#pragma unroll
	for (int k = 0; k < LP; ++k) {
		const uint32_t e = ex[k];
		if (e == NX_BAD)
			continue;
		uint32_t h = (e * 2654435761u) >> (32 - __builtin_ctz(uint32_t(LW)));  // log2(LW) bits
		for (int probe = 0; probe < LW; ++probe, h = (h + 1) & (LW - 1)) {
			const uint32_t old = atomicCAS(&key[h], NX_BAD, e);
			if (old == NX_BAD || old == e) {
				atomicAdd(&cnt[h], 1u);
				break;
			}
		}
	}
	__syncthreads();
	uint32_t bc = 0, bk = NX_BAD;
	for (int32_t i = int32_t(threadIdx.x); i < LW; i += LT)
		if (cnt[i] > bc) {
			bc = cnt[i];
			bk = key[i];
		}
	for (int m = 32; m >= 1; m >>= 1) {
		const uint32_t oc = __shfl_xor(bc, m), ok = __shfl_xor(bk, m);
		if (oc > bc) {
			bc = oc;
			bk = ok;
		}
	}
	if (lane_id() == 0) {
		best[threadIdx.x >> 6][0] = bc;
		best[threadIdx.x >> 6][1] = bk;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int j = 1; j < LT / 64; ++j)
			if (best[j][0] > bc) {
				bc = best[j][0];
				bk = best[j][1];
			}
		guess[blockIdx.x + 1] = bc ? bk : uint32_t(min(we, n));
	}
	if (!done)
		return;
	// the tables of this window out (release), counted; the last window in
	// sees every window's (acquire) and chains them
	__shared__ uint32_t last;
	// every thread's table stores released at agent scope before the count
	// (the last workgroup may run on another XCD's L2; thread 0's release
	// alone would lean on the barrier's fence being cumulative)
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
	__syncthreads();
	if (threadIdx.x == 0)
		last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1u ==
		       gridDim.x;
	__syncthreads();
	if (!last)
		return;
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
	if (threadIdx.x == 0)
		__hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	const int32_t nwin = int32_t(gridDim.x);
	lone_chain_body<LW, LT, 2 * LW / LT>(reinterpret_cast<uint32_t*>(X), exit_tab, osum_tab, guess, n, nwin,
	                                      cap, entry, obase, ctl, st);
}

// ---------------------------------------------------------------- step 3
// One workgroup per window.  The true chain is marked from the window's
// entry (pointer doubling), its sequences are parsed once into an LDS table
// in chain order (output start, literal position, literal length, offset),
// and the window's output words are written in tiles of OT consecutive
// words: every sequence starting in the tile marks its first word, a prefix
// maximum gives every word its sequence, and lane i of a wave writes word
// i -- each store instruction covers 256 contiguous bytes.  A word is a
// literal (bit 31 | the byte) or the output position the byte copies
// (Output_With_History's byte i = byte i - offset, which also gives the
// overlap rule); H history words precede output byte 0.
constexpr int32_t OT = 4096;            // output words per emission tile
constexpr int32_t OTP = OT / LT;        // per thread in the tile's prefix maximum

struct SeqRec {
	uint32_t o;    // first output byte, from the window's first
	int32_t lit;   // block position of the first literal
	int32_t L;     // literal bytes
	uint32_t off;  // match offset (0: none) | k1 << 16 (quirk D1, below)
	int32_t ml;    // match bytes
};

// Quirk D1 (lz4ada.adb:790-824, 845-904), emulated.  Right after a round
// that ended at Output_Pos_History = OPH in [65536, 65542], the new round
// writes from Buffer position 0 and a history match at output position p
// reads Buffer(p - off + OPH ...) = Buffer(p + d ...), d = OPH - off.  The
// reference's wild copies leave up to 7 bytes past the write frontier:
// after this sequence's literal Write_Output (Data = the block payload, 8
// bytes a chunk while 8 payload bytes remain), Buffer(p .. p + ovs - 1)
// holds the payload bytes right after the literals, ovs = 8 ceil(L / 8) - L
// (every older write ended before p - L, its overshoot before p).  So the
// match's first k1 = ovs - d bytes (d < ovs) are those payload bytes -- lit
// + L + d + j -- and the rest are history; its own chunks read ahead of
// what they write.  With no literals the last write was the previous
// match's last Write_Output call, whose overshoot is the Buffer bytes right
// after its source: emulated (as pointer words to those output positions,
// kept in the record's lit) when that match was one call whose tail read
// only final bytes -- the rule of lz4ada_idx.hip d1_emulable.  Declined
// (exact path) instead: a literal run whose last chunk was not wild (the
// payload's last 8 bytes), a match that also reads the current round (p +
// ml > off), a no-literal read after any other previous match (or the
// window's first sequence).

template <int32_t LW>
__global__ __launch_bounds__(LT) void k_lone_words(const uint8_t* __restrict__ blk, int32_t n,
                                                   const uint32_t* __restrict__ nxt_tab,
                                                   const uint32_t* __restrict__ entry,
                                                   const uint32_t* __restrict__ obase,
                                                   LoneCtl* __restrict__ ctl,
                                                   lz4ada_block_status* __restrict__ st,
                                                   uint32_t* __restrict__ Wbase, int32_t H,
                                                   int32_t d1, int32_t n1, int32_t nwin,
                                                   const uint8_t* __restrict__ h0, int32_t n0,
                                                   const uint8_t* __restrict__ h1)
{
	// the workgroups past the windows write the history words (round 4: a
	// launch of its own, k_lone_hist)
	if (int32_t(blockIdx.x) >= nwin) {
		for (int32_t i = (int32_t(blockIdx.x) - nwin) * LT * 4 + int32_t(threadIdx.x); i < H &&
		     i < (int32_t(blockIdx.x) - nwin + 1) * LT * 4; i += LT)
			Wbase[i] = LIT | uint32_t(i < n0 ? h0[i] : h1[i - n0]);
		return;
	}
	// d1: 0, or 1 (decline every match >= D1_OFF back before the block), or
	// the round's OPH (>= 65536: emulate quirk D1); n1: the block's position
	// in the round (its history's current-round part)
	// words [0, H): the history (literals); output byte x is word H + x
	constexpr int32_t LP = LW / LT, LSTG = 2 * LW;
	constexpr int32_t MAXSEQ = LW / 3 + 2;  // chain sequences starting in a window (>= 3 bytes but the last)
	uint32_t* __restrict__ W = Wbase + H;
	__shared__ alignas(16) uint8_t s[LSTG + 32];
	__shared__ uint16_t J[LW];
	__shared__ uint8_t mark[LW];
	__shared__ SeqRec R[MAXSEQ + 1];
	__shared__ uint16_t T16[OT];
	__shared__ uint32_t wred[3][LT / 64];
	if (ctl->code != DS_OK)
		return;
	const int32_t w = int32_t(blockIdx.x);
	const int32_t ws = w * LW, we = min(ws + LW, n);
	const uint32_t e = entry[w];
	if (e >= uint32_t(we))
		return;  // a sequence started earlier covers this window
	const int32_t shi = min(ws + LSTG, n);
	cg8* in = gptr(blk);
	const int32_t tid = int32_t(threadIdx.x), t0 = tid * LP;
	const uint32_t lane = lane_id(), wv = uint32_t(tid) >> 6;
	constexpr uint16_t EXIT = 0xFFFFu;
	for (int32_t i = tid; i < LW; i += LT) {
		const int32_t p = ws + i;
		uint16_t j = EXIT;
		if (p < we) {
			const uint32_t nx = nxt_tab[p];
			if (nx >= uint32_t(ws) && nx < uint32_t(we))
				j = uint16_t(nx - uint32_t(ws));
		}
		J[i] = j;
		mark[i] = uint8_t(p == int32_t(e));
	}
	lone_stage(s, in, ws, shi);  // ends with a barrier
	const LoneSrc S{ s, ws, shi, in };
	// mark the chain from e: after round r every position within 2^(r+1)
	// steps of e is marked
	for (int r = 0; r < 12; ++r) {
		int any = 0;
#pragma unroll
		for (int32_t k = 0; k < LP; ++k) {
			const uint16_t j = J[t0 + k];
			if (j != EXIT) {
				any = 1;
				if (mark[t0 + k])
					mark[j] = 1;
			}
		}
		if (!__syncthreads_or(any))
			break;
		uint16_t nj[LP];
#pragma unroll
		for (int32_t k = 0; k < LP; ++k) {
			const uint16_t j = J[t0 + k];
			nj[k] = j == EXIT ? EXIT : J[j];
		}
		__syncthreads();
#pragma unroll
		for (int32_t k = 0; k < LP; ++k)
			J[t0 + k] = nj[k];
		__syncthreads();
	}
	// this thread's chain sequences, in order: table index by a prefix sum
	uint32_t mk = 0;
#pragma unroll
	for (int32_t k = 0; k < LP; ++k)
		mk |= uint32_t(mark[t0 + k] != 0) << k;
	const int32_t cnt = __builtin_popcount(mk);
	const int32_t ci = wave_incl_scan(cnt);
	if (lane == 63)
		wred[0][wv] = uint32_t(ci);
	// parsed without bound (the true chain); output bytes relative to the
	// thread's first sequence until the second prefix sum
	bool bad = false;
	uint32_t mine = 0;
	__syncthreads();
	int32_t si = ci - cnt, ns = 0;
	for (uint32_t j = 0; j < LT / 64; ++j) {
		si += j < wv ? int32_t(wred[0][j]) : 0;
		ns += int32_t(wred[0][j]);
	}
	int32_t sj = si;
	for (uint32_t m = mk; m; m &= m - 1u, ++sj) {
		const int32_t k = __builtin_ctz(m);
		const LoneSeq q = lone_parse(S, ws + t0 + k, n, GMAX_TRUE);
		if (q.nx == NX_BAD || sj >= MAXSEQ) {
			bad = true;  // never expected: k_lone_chain accepted this chain
			continue;
		}
		R[sj] = SeqRec{ mine, q.lit, q.L, uint32_t(q.off), q.ml };
		mine += q.os;
	}
	const uint32_t oi = uint32_t(wave_incl_scan(int32_t(mine)));
	if (lane == 63)
		wred[1][wv] = oi;
	__syncthreads();
	uint32_t ob = oi - mine, tw = 0;
	for (uint32_t j = 0; j < LT / 64; ++j) {
		ob += j < wv ? wred[1][j] : 0u;
		tw += wred[1][j];
	}
	const uint32_t wo = obase[w];
	for (int32_t j = si; j < min(sj, MAXSEQ); ++j)
		R[j].o += ob;
	if (d1 > 1)
		__syncthreads();  // R[j - 1] of another thread, for quirk D1 below
	for (int32_t j = si; j < min(sj, MAXSEQ); ++j) {
		const uint32_t o = R[j].o;
		const int32_t L = R[j].L;
		const int64_t off = int64_t(R[j].off), oa = int64_t(wo) + o;
		if (off && oa + L + H < off) {
			bad = true;  // a reference before the history it was given (exact path)
		} else if (d1 == 1 && off && oa + L < off && off >= D1_OFF) {
			bad = true;  // quirk D1 (not emulated by this caller)
		} else if (d1 > 1 && off && n1 + oa + L < off && int64_t(d1) - off < 8) {
			// quirk D1: a read before the round start, which may see what the
			// literals' wild copy left
			const int32_t d = d1 - int32_t(off);
			const int32_t c_last = R[j].lit + 8 * ((L - 1) / 8);  // the literal copy's last chunk
			const int32_t ovs = 8 * ((L + 7) / 8) - L;
			if (n1 + oa + L + R[j].ml > off || (L > 0 && c_last + 8 > n)) {
				bad = true;  // the cases not emulated: the exact path
			} else if (L == 0 && n1 + oa == 0) {
				// the round's first output: nothing written past its frontier
				// yet, so the read is the previous round's bytes (plain history)
			} else if (L == 0) {
				// the previous match's overshoot: output bytes q + d + i
				const int32_t pml = j > 0 ? R[j - 1].ml : 0, pof = j > 0 ? int32_t(R[j - 1].off & 0xFFFFu) : 0;
				const int32_t pmd = j > 0 ? int32_t(wo + R[j - 1].o) + R[j - 1].L : 0;
				const int32_t f = n1 + pmd, raw = f - pof, pad = (8 - (pml & 7)) & 7;
				const bool ok = pml > 0 && (raw >= 0 ? pml <= pof && pof - pml >= pad
				                                     : pof - f >= pml && d1 - pof >= 8 && raw + pml + pad <= 0);
				if (!ok) {
					bad = true;
				} else if (d < pad) {
					const int32_t k1 = min(pad - d, R[j].ml);
					R[j].lit = H + pmd - pof + pml + d;  // the word of output byte q + d
					R[j].off = uint32_t(off) | (uint32_t(k1) << 16);
				}
			} else if (d < ovs) {
				const int32_t k1 = min(ovs - d, R[j].ml);
				R[j].off = uint32_t(off) | (uint32_t(k1) << 16);
			}
		}
	}
	if (__syncthreads_or(bad)) {
		if (tid == 0) {
			ctl->code = DS_RETRY;
			st->code = DS_RETRY;
			st->out_len = 0;
		}
		return;
	}
	// tiles of the window's output words [wo, wo + tw)
	uint32_t cur = 0;  // 1 + the sequence covering the tile's first word
	for (uint32_t tb = 0; tb < tw; tb += OT) {
#pragma unroll
		for (int32_t k = 0; k < OTP; ++k)
			T16[tid + LT * k] = 0;
		__syncthreads();
		for (int32_t j = tid; j < ns; j += LT) {
			const uint32_t o = R[j].o;
			if (o >= tb && o - tb < uint32_t(OT) && o < tw)
				T16[o - tb] = uint16_t(j + 1);
		}
		__syncthreads();
		uint32_t v[OTP], run = 0;
#pragma unroll
		for (int32_t k = 0; k < OTP; ++k) {
			run = max(run, uint32_t(T16[tid * OTP + k]));
			v[k] = run;
		}
		const uint32_t inc = uint32_t(wave_incl_max(int32_t(run)));
		if (lane == 63)
			wred[2][wv] = inc;
		uint32_t pre = uint32_t(__shfl_up(int32_t(inc), 1));
		pre = lane ? pre : 0u;
		__syncthreads();
		uint32_t tmax = cur;
		for (uint32_t j = 0; j < LT / 64; ++j) {
			pre = j < wv ? max(pre, wred[2][j]) : pre;
			tmax = max(tmax, wred[2][j]);
		}
		pre = max(pre, cur);
#pragma unroll
		for (int32_t k = 0; k < OTP; ++k)
			T16[tid * OTP + k] = uint16_t(max(v[k], pre) - 1u);
		cur = tmax;
		__syncthreads();
		const uint32_t lim = min(uint32_t(OT), tw - tb);
#pragma unroll 4
		for (int32_t k = 0; k < OTP; ++k) {
			const uint32_t i = uint32_t(tid + LT * k);
			if (i < lim) {
				const SeqRec r = R[T16[i]];
				const uint32_t x = tb + i - r.o;
				const uint32_t oa = wo + tb + i;
				const uint32_t off = r.off & 0xFFFFu, k1 = r.off >> 16;
				const int32_t j = int32_t(x) - r.L;  // match byte
				uint32_t v;
				if (j < 0)
					v = LIT | S.at(r.lit + int32_t(x));
				else if (uint32_t(j) < k1)  // quirk D1: the last wild copy's overshoot
					v = r.L > 0 ? LIT | S.at(r.lit + r.L + (d1 - int32_t(off)) + j) : uint32_t(r.lit + j);
				else
					v = uint32_t(H) + oa - off;
				W[oa] = v;
			}
		}
		__syncthreads();
	}
}

// ---------------------------------------------------------------- step 4
// Words are read and written with agent-scope relaxed atomics: another
// workgroup's progress on its slice becomes visible while this one jumps
// through it (a stale word is still a valid pointer along the same chain,
// so visibility only changes the speed, never the result).
__device__ __forceinline__ uint32_t w_load(const uint32_t* p)
{
	return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void w_store(uint32_t* p, uint32_t v)
{
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// SL output words per workgroup: a small block takes small slices, so its
// jump rounds spread over more CUs with fewer gathers per lane each.
// hout (not null): pinned host memory that takes the bytes too.
template <int32_t SL>
__global__ __launch_bounds__(LT) void k_lone_resolve(uint32_t* __restrict__ W,
                                                     const LoneCtl* __restrict__ ctl,
                                                     lz4ada_block_status* __restrict__ st,
                                                     uint8_t* __restrict__ out, uint32_t H,
                                                     uint8_t* __restrict__ hout)
{
	static_assert(SL % (4 * LT) == 0 && SL <= RES_SLICE, "lone-decoder tiling");
	constexpr int32_t RPT = SL / LT;  // words per thread
	if (ctl->code != DS_OK)
		return;
	const uint32_t total = ctl->total;
	const uint32_t base = blockIdx.x * uint32_t(SL);
	if (base >= total)
		return;
	// thread t owns words base + 4 (t + LT k) .. +3 for k < RPT / 4: its
	// own words it alone writes, so its reads of them need no atomics
	const uint32_t tid = threadIdx.x;
	uint32_t v[RPT];
#pragma unroll
	for (int32_t k = 0; k < RPT / 4; ++k) {
		const uint32_t i = base + 4u * (tid + uint32_t(LT) * uint32_t(k));
#pragma unroll
		for (int32_t j = 0; j < 4; ++j)
			v[4 * k + j] = (i + uint32_t(j) < total) ? W[H + i + uint32_t(j)] : LIT;
	}
	int pend = 1;
	for (int32_t round = 0; round < 1024 && pend; ++round) {
		// every lane issues all its gathers before the first use (a resolved
		// word re-reads itself: branch-free, so one wait covers the round)
		uint32_t nv[RPT];
#pragma unroll
		for (int32_t k = 0; k < RPT; ++k) {
			const uint32_t i = base + 4u * (tid + uint32_t(LT) * uint32_t(k >> 2)) + uint32_t(k & 3);
			const uint32_t a = (v[k] & LIT) ? H + min(i, total - 1) : v[k];
			nv[k] = w_load(W + a);
		}
		pend = 0;
#pragma unroll
		for (int32_t k = 0; k < RPT; ++k) {
			const uint32_t i = base + 4u * (tid + uint32_t(LT) * uint32_t(k >> 2)) + uint32_t(k & 3);
			if (!(v[k] & LIT)) {
				v[k] = nv[k];
				pend |= !(nv[k] & LIT);
				if (i < total)
					w_store(W + H + i, v[k]);
			}
		}
		pend = __syncthreads_or(pend);
	}
	if (pend) {  // never expected: pointer chains halve every round
		if (threadIdx.x == 0) {
			__hip_atomic_store(&st->code, int32_t(DS_RETRY), __ATOMIC_RELAXED,
			                   __HIP_MEMORY_SCOPE_AGENT);
			__hip_atomic_store(&st->out_len, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		return;
	}
#pragma unroll
	for (int32_t k = 0; k < RPT / 4; ++k) {
		const uint32_t i = base + 4u * (tid + uint32_t(LT) * uint32_t(k));
		if (i + 4 <= total) {
			const uint32_t b = (v[4 * k] & 0xFFu) | ((v[4 * k + 1] & 0xFFu) << 8) |
			                   ((v[4 * k + 2] & 0xFFu) << 16) | ((v[4 * k + 3] & 0xFFu) << 24);
			*reinterpret_cast<uint32_t*>(out + i) = b;
			if (hout)
				*reinterpret_cast<uint32_t*>(hout + i) = b;
		} else {
			for (int32_t j = 0; j < 4; ++j)
				if (i + uint32_t(j) < total) {
					out[i + uint32_t(j)] = uint8_t(v[4 * k + j]);
					if (hout)
						hout[i + uint32_t(j)] = uint8_t(v[4 * k + j]);
				}
		}
	}
}

// ---------------------------------------------------------------- host side
constexpr int64_t LONE_HDR = 256;  // the scratch's fixed header: the windows' done count

int64_t lone_scratch_bytes(int64_t n, int64_t cap)
{
	const int64_t nwin = (n + LW_MIN - 1) / LW_MIN;
	return LONE_HDR + 12 * std::max<int64_t>(n, 1) + 12 * (nwin + 2) + 64 + 4 * std::max<int64_t>(cap, 1) +
	       4 * 65536 + 512;
}

hipError_t lone_scratch_init(void* d_scratch, hipStream_t stream)
{
	return hipMemsetAsync(d_scratch, 0, size_t(LONE_HDR), stream);
}

// Window size by compressed size n and output capacity cap, swept with
// the first-run chain walk (tools/r04_sw.sh, profiles/r04p_window_sweep.txt;
// earlier sweeps profiles/r04m_lone_window.txt).  Blocks with matches take
// 512-byte windows up to ~800 KB compressed (256 KiB mixed / dense 0.045 /
// 0.051 ms against 0.051 / 0.058 at 1 KiB) and 1 KiB above (4 MiB 0.164 /
// 0.280 ms against 0.171 / 0.402 at 4 KiB); literal-heavy blocks (n >= 0.9
// cap) take 1 KiB windows up to 160 KB and 2 KiB above (4 MiB 0.278 ms
// against 0.300 at 4 KiB and 0.418 at 1 KiB).  LZ4ADA_LONE_LW forces one.
static int32_t lone_window(int64_t n, int64_t cap)
{
	static const int32_t forced = [] {
		const char* e = getenv("LZ4ADA_LONE_LW");
		const int v = e ? atoi(e) : 0;
		return (v == 512 || v == 1024 || v == 2048 || v == 4096) ? v : 0;
	}();
	if (forced)
		return forced;
	if (10 * n >= 9 * cap)  // literal-heavy
		return n <= (int64_t(160) << 10) ? 1024 : 2048;
	return n <= (int64_t(800) << 10) ? 512 : 1024;
}

// Resolve slice by output capacity (tools/r04_sl.sh, profiles/r04k_resolve_slice.txt:
// lone decode of mixed / dense 64 KiB blocks 0.050 / 0.052 -> 0.042 / 0.042 ms
// at 1024-word slices, 256 KiB 0.058 / 0.067 -> 0.052 / 0.058; 1 MiB even;
// 4 MiB 0.171 / 0.403 -> 0.175 / 0.420, so large blocks keep 4096).
// LZ4ADA_LONE_SLICE forces one.
static int32_t resolve_slice(int64_t cap)
{
	static const int32_t forced = [] {
		const char* e = getenv("LZ4ADA_LONE_SLICE");
		const int v = e ? atoi(e) : 0;
		return (v == 1024 || v == 2048 || v == 4096) ? v : 0;
	}();
	if (forced)
		return forced;
	return cap <= (int64_t(512) << 10) ? 1024 : RES_SLICE;
}

// The scratch: per-position tables, per-window entries, the control block
// and the words (H history words, then one per output byte).
struct LoneLayout {
	uint32_t *done, *exit_tab, *osum_tab, *nxt_tab, *entry, *obase, *guess, *W;
	LoneCtl* ctl;
	LoneLayout(uint8_t* sc, int64_t n, int64_t nwin)
	{
		done = reinterpret_cast<uint32_t*>(sc);  // first: the same place for every block size
		exit_tab = reinterpret_cast<uint32_t*>(sc + LONE_HDR);
		osum_tab = exit_tab + n;
		nxt_tab = osum_tab + n;
		entry = nxt_tab + n;
		obase = entry + (nwin + 1);
		guess = obase + (nwin + 1);
		ctl = reinterpret_cast<LoneCtl*>((reinterpret_cast<uintptr_t>(guess + (nwin + 1)) + 63) &
		                                 ~uintptr_t(63));
		W = reinterpret_cast<uint32_t*>((reinterpret_cast<uintptr_t>(ctl + 1) + 255) & ~uintptr_t(255));
	}
};

template <int32_t LW>
static hipError_t lone_steps(const uint8_t* d_blk, int64_t n, int64_t cap, lz4ada_block_status* d_st,
                             uint8_t* sc, hipStream_t stream, const uint8_t* d_h0, int32_t n0,
                             const uint8_t* d_h1, int32_t n1, int d1, uint8_t* d_copy, int64_t ncopy,
                             bool fused)
{
	constexpr int32_t CK = (int32_t(16) << 20) / LW / CT;
	static_assert(int64_t(CK) * CT * LW >= LONE_MAX_IN, "the chain step covers every window");
	const int64_t nwin = (n + LW - 1) / LW;
	if (nwin > int64_t(CK) * CT)
		return hipErrorInvalidValue;
	const int32_t H = n0 + n1;
	const LoneLayout Lo(sc, n, nwin);
	uint32_t *exit_tab = Lo.exit_tab, *osum_tab = Lo.osum_tab, *nxt_tab = Lo.nxt_tab, *entry = Lo.entry,
	         *obase = Lo.obase, *guess = Lo.guess, *W = Lo.W;
	LoneCtl* ctl = Lo.ctl;
	// a small block's chain step runs in its last window's workgroup
	// (done: the count, zeroed by lone_scratch_init and again by each use)
	uint32_t* done = fused && nwin < 2 * LW ? Lo.done : nullptr;
	hipLaunchKernelGGL(k_lone_windows<LW>, dim3(uint32_t(nwin)), dim3(LT), 0, stream, d_blk, int32_t(n),
	                   exit_tab, osum_tab, nxt_tab, guess, d_copy, int32_t(ncopy), done, uint32_t(cap), entry,
	                   obase, ctl, d_st);
	if (d_copy)
		d_blk = d_copy;  // step 3 reads the device copy
	hipError_t err = hipGetLastError();
	if (err != hipSuccess)
		return err;
	if (!done) {
		hipLaunchKernelGGL(k_lone_chain<LW>, dim3(1), dim3(CT), size_t(nwin + 2) * 4, stream, exit_tab,
		                   osum_tab, guess, int32_t(n), int32_t(nwin), uint32_t(cap), entry, obase, ctl,
		                   d_st);
		err = hipGetLastError();
		if (err != hipSuccess)
			return err;
	}
	// the history words ride in the words launch (workgroups past nwin)
	const uint32_t nh = uint32_t((H + 4 * LT - 1) / (4 * LT));
	hipLaunchKernelGGL(k_lone_words<LW>, dim3(uint32_t(nwin) + nh), dim3(LT), 0, stream, d_blk, int32_t(n),
	                   nxt_tab, entry, obase, ctl, d_st, W, H, d1, n1, int32_t(nwin), d_h0, n0, d_h1);
	return hipGetLastError();
}

hipError_t launch_decode_lone_parse(const uint8_t* d_blk, int64_t n, int64_t cap,
                                    lz4ada_block_status* d_st, void* d_scratch, int64_t scratch_bytes,
                                    hipStream_t stream, const uint8_t* d_h0, int32_t n0,
                                    const uint8_t* d_h1, int32_t n1, int d1, uint8_t* d_copy, int64_t ncopy,
                                    bool fused)
{
	if (n <= 0 || n > LONE_MAX_IN || cap <= 0 || cap > (int64_t(1) << 30) ||
	    scratch_bytes < lone_scratch_bytes(n, cap) || n0 < 0 || n1 < 0 || n0 + n1 > 65535 ||
	    (d_copy && (ncopy < n || ncopy > INT32_MAX)))
		return hipErrorInvalidValue;
	uint8_t* sc = static_cast<uint8_t*>(d_scratch);
	switch (lone_window(n, cap)) {
	case 512: return lone_steps<512>(d_blk, n, cap, d_st, sc, stream, d_h0, n0, d_h1, n1, d1, d_copy, ncopy, fused);
	case 1024: return lone_steps<1024>(d_blk, n, cap, d_st, sc, stream, d_h0, n0, d_h1, n1, d1, d_copy, ncopy, fused);
	case 2048: return lone_steps<2048>(d_blk, n, cap, d_st, sc, stream, d_h0, n0, d_h1, n1, d1, d_copy, ncopy, fused);
	default: return lone_steps<4096>(d_blk, n, cap, d_st, sc, stream, d_h0, n0, d_h1, n1, d1, d_copy, ncopy, fused);
	}
}

hipError_t launch_decode_lone_emit(int64_t n, uint8_t* d_out, int64_t cap, lz4ada_block_status* d_st,
                                   void* d_scratch, hipStream_t stream, int32_t H, uint8_t* h_out)
{
	const int32_t lw = lone_window(n, cap);
	const int64_t nwin = (n + lw - 1) / lw;
	const LoneLayout Lo(static_cast<uint8_t*>(d_scratch), n, nwin);
	const int32_t sl = resolve_slice(cap);
	const uint32_t nres = uint32_t((cap + sl - 1) / sl);
	switch (sl) {
	case 1024:
		hipLaunchKernelGGL(k_lone_resolve<1024>, dim3(nres), dim3(LT), 0, stream, Lo.W, Lo.ctl, d_st, d_out,
		                   uint32_t(H), h_out);
		break;
	case 2048:
		hipLaunchKernelGGL(k_lone_resolve<2048>, dim3(nres), dim3(LT), 0, stream, Lo.W, Lo.ctl, d_st, d_out,
		                   uint32_t(H), h_out);
		break;
	default:
		hipLaunchKernelGGL(k_lone_resolve<RES_SLICE>, dim3(nres), dim3(LT), 0, stream, Lo.W, Lo.ctl, d_st,
		                   d_out, uint32_t(H), h_out);
	}
	return hipGetLastError();
}

hipError_t launch_decode_lone(const uint8_t* d_blk, int64_t n, uint8_t* d_out, int64_t cap,
                              lz4ada_block_status* d_st, void* d_scratch, int64_t scratch_bytes,
                              hipStream_t stream, const uint8_t* d_h0, int32_t n0, const uint8_t* d_h1,
                              int32_t n1, int d1)
{
	const hipError_t err = launch_decode_lone_parse(d_blk, n, cap, d_st, d_scratch, scratch_bytes, stream,
	                                                d_h0, n0, d_h1, n1, d1);
	if (err != hipSuccess)
		return err;
	return launch_decode_lone_emit(n, d_out, cap, d_st, d_scratch, stream, n0 + n1);
}

}  // namespace lz4ada
