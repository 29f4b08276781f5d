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
//  1. k_lone_windows -- one workgroup per 4 KiB window of the compressed
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
//     sum and writes one word per output byte: a literal (bit 31 | byte) or
//     the output position the byte copies (Output_With_History's byte i =
//     byte i - offset, which also gives the overlap rule).
//  4. k_lone_resolve -- the copies resolved by pointer jumping over the
//     words (W[i] = W[W[i]] until every word is a literal), each workgroup
//     over its own slice of the output, reading the others' slices as they
//     go; then the bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4ada_internal.h"
#include "lz4ada_dev.h"

namespace lz4ada {

constexpr int32_t LW = 4096;        // compressed bytes per window
constexpr int32_t LT = 256;         // threads per workgroup
constexpr int32_t LP = LW / LT;     // positions per thread
constexpr int32_t LSTG = 2 * LW;    // staged input bytes (window + 4 KiB lookahead)
constexpr uint32_t NX_BAD = 0xFFFFFFFFu;  // not a sequence (or beyond what a window parses)
constexpr uint32_t LIT = 0x80000000u;     // word: a literal byte
constexpr int32_t LONG_SEQ = 64;          // sequences over this many output bytes: whole workgroup
constexpr int32_t RES_SLICE = 16384;      // output words per workgroup in k_lone_resolve
constexpr int32_t MAX_RUN_L = 1 << 28;

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

// ---------------------------------------------------------------- step 1
// Also the entry guess for the next window: the exit most positions of this
// window reach (chains started at wrong bytes mostly merge into the true
// one before the window ends), counted in an LDS hash table.
__global__ __launch_bounds__(LT) void k_lone_windows(const uint8_t* __restrict__ blk, int32_t n,
                                                     uint32_t* __restrict__ exit_tab,
                                                     uint32_t* __restrict__ osum_tab,
                                                     uint32_t* __restrict__ nxt_tab,
                                                     uint32_t* __restrict__ guess)
{
	__shared__ alignas(16) uint8_t s[LSTG + 32];
	__shared__ uint64_t X[LW];  // nx | os << 32
	__shared__ uint32_t best[LT / 64][2];
	const int32_t ws = int32_t(blockIdx.x) * LW, we = min(ws + LW, n);
	const int32_t shi = min(ws + LSTG, n);
	cg8* in = gptr(blk);
	lone_stage(s, in, ws, shi);
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
		uint32_t h = (e * 2654435761u) >> 20;  // 12 bits
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
}

// ---------------------------------------------------------------- step 2
constexpr int32_t CT = 1024;  // k_lone_chain threads
constexpr int32_t CK = 4;     // windows per thread (nwin <= CT * CK: 16 MiB blocks)

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
	__shared__ uint32_t wsum[CT / 64];
	__shared__ unsigned long long total64;
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
#pragma unroll
		for (int32_t k = 0; k < CK; ++k) {
			const int32_t w = tid + k * CT;
			if (w < nwin && E[w + 1] != nv[k]) {
				E[w + 1] = nv[k];
				ch = 1;
			}
		}
		if (!__syncthreads_or(ch) || it > uint32_t(nwin) + 2)
			break;
		// still changing after two passes: the guesses are poor (sequences
		// too far apart for speculative chains to merge, e.g. long literal
		// runs).  Entries 0..it are exact; one lane walks the rest, one
		// dependent lookup per window instead of one pass per window, and
		// the next pass confirms.
		if (it == 2) {
			if (tid == 0) {
				for (int32_t w = int32_t(it); w < nwin; ++w) {
					const uint32_t e = E[w];
					const uint32_t lim = uint32_t(min((w + 1) * LW, n));
					E[w + 1] = e == NX_BAD ? NX_BAD : (e < lim ? exit_tab[e] : e);
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
	for (int32_t w = w0; w < min(w0 + per, nwin); ++w) {
		const uint32_t e = E[w];
		if (e == NX_BAD)
			bad = true;
		else if (e < uint32_t(min((w + 1) * LW, n)))
			mine += osum_tab[e];
	}
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
	for (int32_t w = w0; w < min(w0 + per, nwin); ++w) {
		obase[w] = run;
		const uint32_t e = E[w];
		entry[w] = e;
		if (e != NX_BAD && e < uint32_t(min((w + 1) * LW, n)))
			run += osum_tab[e];
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

// ---------------------------------------------------------------- step 3
// Words of output bytes [o, o + q.os) of sequence q: literals (bit 31 | the
// byte, four per input dword) then the match (the position each byte
// copies).  Threads j = j0, j0 + js, ... of the caller share the work.
__device__ __forceinline__ void lone_emit(const LoneSrc& S, const LoneSeq& q, uint32_t o,
                                          uint32_t* __restrict__ W, int32_t j0, int32_t js,
                                          int32_t n, uint32_t hb)
{
	for (int32_t b = 4 * j0; b < q.L; b += 4 * js) {
		const int32_t x = q.lit + b;
		uint32_t d;
		if (x + 4 <= n) {
			d = S.at4(x);
		} else {
			d = 0;
			for (int32_t k = 0; k < 4 && x + k < n; ++k)
				d |= S.at(x + k) << (8 * k);
		}
		const int32_t m = min(4, q.L - b);
#pragma unroll
		for (int32_t k = 0; k < 4; ++k)
			if (k < m)
				W[o + uint32_t(b + k)] = LIT | ((d >> (8 * k)) & 0xFFu);
	}
	const uint32_t m0 = o + uint32_t(q.L);
	for (int32_t b = j0; b < q.ml; b += js)
		W[m0 + uint32_t(b)] = hb + m0 + uint32_t(b) - uint32_t(q.off);
}

__global__ __launch_bounds__(LT) void k_lone_words(const uint8_t* __restrict__ blk, int32_t n,
                                                   const uint32_t* __restrict__ nxt_tab,
                                                   const uint32_t* __restrict__ entry,
                                                   const uint32_t* __restrict__ obase,
                                                   LoneCtl* __restrict__ ctl,
                                                   lz4ada_block_status* __restrict__ st,
                                                   uint32_t* __restrict__ Wbase, int32_t H,
                                                   int32_t d1_guard)
{
	// words [0, H): the history (literals); output byte x is word H + x
	uint32_t* __restrict__ W = Wbase + H;
	__shared__ alignas(16) uint8_t s[LSTG + 32];
	__shared__ uint16_t J[LW];
	__shared__ uint8_t mark[LW];
	__shared__ uint32_t tsum[LT / 64];
	__shared__ int32_t nlong;
	__shared__ int32_t lpos[LW / 4];
	__shared__ uint32_t lout[LW / 4];
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
	if (tid == 0)
		nlong = 0;
	lone_stage(s, in, ws, shi);  // ends with a barrier
	const LoneSrc S{ s, ws, shi, in };
	// mark the chain from e: after round r every position within 2^(r+1)
	// steps of e is marked
	for (int r = 0; r < 12; ++r) {
		int any = 0;
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
		for (int32_t k = 0; k < LP; ++k) {
			const uint16_t j = J[t0 + k];
			nj[k] = j == EXIT ? EXIT : J[j];
		}
		__syncthreads();
		for (int32_t k = 0; k < LP; ++k)
			J[t0 + k] = nj[k];
		__syncthreads();
	}
	// this thread's marked sequences (the true chain: parsed without bound)
	LoneSeq qs[LP];
	uint32_t mine = 0;
	uint32_t mk = 0;
	for (int32_t k = 0; k < LP; ++k) {
		if (mark[t0 + k]) {
			qs[k] = lone_parse(S, ws + t0 + k, n, GMAX_TRUE);
			mine += qs[k].os;
			mk |= 1u << k;
		}
	}
	const uint32_t lane = lane_id(), wv = uint32_t(tid) >> 6;
	const uint32_t inc = uint32_t(wave_incl_scan(int32_t(mine)));
	if (lane == 63)
		tsum[wv] = inc;
	__syncthreads();
	uint32_t o = obase[w] + inc - mine;
	for (uint32_t j = 0; j < wv; ++j)
		o += tsum[j];
	bool bad = false;
	for (int32_t k = 0; k < LP; ++k) {
		if (!(mk >> k & 1u))
			continue;
		const LoneSeq& q = qs[k];
		if (q.nx == NX_BAD)
			bad = true;  // never expected: k_lone_chain accepted this chain
		else if (q.ml && int64_t(o) + q.L + H < int64_t(q.off))
			bad = true;  // a reference before the history it was given (exact path)
		else if (d1_guard && q.ml && int64_t(o) + q.L < int64_t(q.off) && q.off >= D1_OFF)
			bad = true;  // quirk D1: the reference's wild copy may have clobbered it
		else if (int32_t(q.os) > LONG_SEQ) {
			const int32_t i = atomicAdd(&nlong, 1);
			if (i < LW / 4) {
				lpos[i] = ws + t0 + k;
				lout[i] = o;
			} else {
				bad = true;  // never expected (a window holds < LW/4 long sequences)
			}
		} else {
			lone_emit(S, q, o, W, 0, 1, n, uint32_t(H));
		}
		o += q.os;
	}
	if (__syncthreads_or(bad)) {
		if (tid == 0) {
			ctl->code = DS_RETRY;
			st->code = DS_RETRY;
			st->out_len = 0;
		}
		return;
	}
	// long sequences: the whole workgroup, one after the other
	const int32_t nl = nlong;
	for (int32_t i = 0; i < nl; ++i) {
		const LoneSeq q = lone_parse(S, lpos[i], n, GMAX_TRUE);
		lone_emit(S, q, lout[i], W, tid, LT, n, uint32_t(H));
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

constexpr int32_t RPT = RES_SLICE / LT;  // words per thread (64)

__global__ __launch_bounds__(LT) void k_lone_resolve(uint32_t* __restrict__ W,
                                                     const LoneCtl* __restrict__ ctl,
                                                     lz4ada_block_status* __restrict__ st,
                                                     uint8_t* __restrict__ out, uint32_t H)
{
	if (ctl->code != DS_OK)
		return;
	const uint32_t total = ctl->total;
	const uint32_t base = blockIdx.x * uint32_t(RES_SLICE);
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
		} else {
			for (int32_t j = 0; j < 4; ++j)
				if (i + uint32_t(j) < total)
					out[i + uint32_t(j)] = uint8_t(v[4 * k + j]);
		}
	}
}

// History words: the H bytes before the block (a linked frame's earlier
// output) as literals, so matches reaching back resolve like any other.
__global__ __launch_bounds__(LT) void k_lone_hist(uint32_t* __restrict__ W, const uint8_t* __restrict__ h0,
                                                  int32_t n0, const uint8_t* __restrict__ h1, int32_t n1)
{
	const int32_t i = int32_t(blockIdx.x) * LT + int32_t(threadIdx.x);
	if (i < n0)
		W[i] = LIT | uint32_t(h0[i]);
	else if (i < n0 + n1)
		W[i] = LIT | uint32_t(h1[i - n0]);
}

// ---------------------------------------------------------------- host side
int64_t lone_scratch_bytes(int64_t n, int64_t cap)
{
	const int64_t nwin = (n + LW - 1) / LW;
	return 12 * std::max<int64_t>(n, 1) + 12 * (nwin + 2) + 64 + 4 * std::max<int64_t>(cap, 1) +
	       4 * 65536 + 512;
}

hipError_t launch_decode_lone(const uint8_t* d_blk, int64_t n, uint8_t* d_out, int64_t cap,
                              lz4ada_block_status* d_st, void* d_scratch, int64_t scratch_bytes,
                              hipStream_t stream, const uint8_t* d_h0, int32_t n0, const uint8_t* d_h1,
                              int32_t n1, int d1_guard)
{
	const int64_t nwin = (n + LW - 1) / LW;
	const int32_t H = n0 + n1;
	if (n <= 0 || n > (int64_t(1) << 30) || cap <= 0 || cap > (int64_t(1) << 30) ||
	    nwin > CK * CT || scratch_bytes < lone_scratch_bytes(n, cap) || n0 < 0 || n1 < 0 ||
	    H > 65535)
		return hipErrorInvalidValue;
	uint8_t* sc = static_cast<uint8_t*>(d_scratch);
	uint32_t* exit_tab = reinterpret_cast<uint32_t*>(sc);
	uint32_t* osum_tab = exit_tab + n;
	uint32_t* nxt_tab = osum_tab + n;
	uint32_t* entry = nxt_tab + n;
	uint32_t* obase = entry + (nwin + 1);
	uint32_t* guess = obase + (nwin + 1);
	LoneCtl* ctl = reinterpret_cast<LoneCtl*>(
	        (reinterpret_cast<uintptr_t>(guess + (nwin + 1)) + 63) & ~uintptr_t(63));
	uint32_t* W = reinterpret_cast<uint32_t*>(
	        (reinterpret_cast<uintptr_t>(ctl + 1) + 255) & ~uintptr_t(255));
	hipLaunchKernelGGL(k_lone_windows, dim3(uint32_t(nwin)), dim3(LT), 0, stream, d_blk, int32_t(n),
	                   exit_tab, osum_tab, nxt_tab, guess);
	hipError_t err = hipGetLastError();
	if (err != hipSuccess)
		return err;
	hipLaunchKernelGGL(k_lone_chain, dim3(1), dim3(CT), size_t(nwin + 2) * 4, stream, exit_tab,
	                   osum_tab, guess, int32_t(n), int32_t(nwin), uint32_t(cap), entry, obase, ctl,
	                   d_st);
	err = hipGetLastError();
	if (err != hipSuccess)
		return err;
	if (H > 0) {
		hipLaunchKernelGGL(k_lone_hist, dim3(uint32_t((H + LT - 1) / LT)), dim3(LT), 0, stream, W, d_h0,
		                   n0, d_h1, n1);
		err = hipGetLastError();
		if (err != hipSuccess)
			return err;
	}
	hipLaunchKernelGGL(k_lone_words, dim3(uint32_t(nwin)), dim3(LT), 0, stream, d_blk, int32_t(n),
	                   nxt_tab, entry, obase, ctl, d_st, W, H, d1_guard);
	err = hipGetLastError();
	if (err != hipSuccess)
		return err;
	const uint32_t nres = uint32_t((cap + RES_SLICE - 1) / RES_SLICE);
	hipLaunchKernelGGL(k_lone_resolve, dim3(nres), dim3(LT), 0, stream, W, ctl, d_st, d_out,
	                   uint32_t(H));
	return hipGetLastError();
}

}  // namespace lz4ada
