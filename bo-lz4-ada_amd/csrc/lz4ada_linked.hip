// lz4ada_linked.hip -- every block of a LINKED frame at once (SURVEY §8f
// item 3).  gfx950 / MI355X.
//
// In a linked frame a block's matches may read up to 65535 bytes of the
// output before it (lz4ada.adb:845-904 with the Output_Pos_History scheme
// of :678-690, 785-787).  That makes the blocks one serial chain if they are
// decoded with real history.  Here each block is decoded with a SYNTHETIC
// history instead, so every block runs at once:
//
//  * layout: every block's output slot is preceded by a 64 KiB history
//    region (desc.out_off - 65536), so the decoders read "before the block
//    start" like any other output byte (k_decode_idx mode 2, k_decode_pc
//    with hist = LINK_HIST);
//  * two decodes of the whole batch with different history patterns at
//    position k of the region: plane X holds k & 255 there; plane Z has
//    every literal written as 0 and k >> 8 in the region.  Decoding only
//    moves bytes, so a byte that is 0 in Z is a constant (a literal, maybe
//    copied on) and any other came from history position k = X | Z << 8 --
//    byte (k - 65536) relative to its block start.  Blocks that read
//    history positions below 256 (their high byte is 0 too) or that Z's
//    decoder declined also take Y = ~X (and H = k >> 8): the three-plane rule;
//  * k_link_init turns the planes into the output bytes and, for a byte
//    that came from history, a word: a pointer to an earlier position of
//    the frame -- taken two steps already from the source bytes' own planes
//    (final before init runs), which resolve most of them;
//  * k_link_jump resolves the pointers by pointer jumping (each round
//    replaces a pointer by its target's word, so chains through many
//    blocks finish in ~log2(length) rounds), reading positions before the
//    batch from the previous batch's last 64 KiB; k_link_init writes the
//    constant bytes and each round the bytes it resolves, so the last
//    round leaves the output (a separate emit pass until round 4).
//
// The result equals decoding the frame with contiguous history.  The
// reference differs from that only in quirk D1 (wild-copy overshoot into
// history), which the host detects from the decoders' AUX_D1_RISK flags and
// the Output_Pos_History sequence, and in references before the frame
// start, which k_link_jump reports; both send the frame to the exact path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "lz4ada_internal.h"
#include "lz4ada_dev.h"

namespace lz4ada {

namespace link {

constexpr uint32_t RES = 0x80000000u;  // resolved: low byte is the value
constexpr int TPB = 256;

// *flag = 1 when any thread of the workgroup has v: one plain store per
// workgroup at most (the host only asks whether any thread had it).  Round
// 4 summed the counts with one atomic per wave -- up to 262,144 atomics on
// one word per launch, which serialise at its L2 channel (~88 per us,
// MI355X_MICROARCH "dequeue"): most of k_link_init's 3.1 ms.
__device__ __forceinline__ void flag_any(uint32_t* flag, bool v)
{
	if (__syncthreads_or(v) && threadIdx.x == 0)
		__hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// History regions of the decode buffers (a null plane is skipped): x = k &
// 255, y = ~x, h = k >> 8 at region byte k (the literal-zero plane z takes
// h's pattern).
__global__ __launch_bounds__(TPB) void k_link_fill(uint8_t* __restrict__ x, uint8_t* __restrict__ y,
                                                   uint8_t* __restrict__ h,
                                                   const lz4ada_block_desc* __restrict__ desc,
                                                   uint32_t nblocks)
{
	const uint32_t b = blockIdx.x;
	if (b >= nblocks)
		return;
	const uint64_t base = desc[b].out_off - uint64_t(HISTORY_SIZE);
	for (uint32_t c = blockIdx.y * TPB + threadIdx.x; c < HISTORY_SIZE / 16; c += gridDim.y * TPB) {
		const uint32_t k0 = 16u * c;
		u32x4 vx;
		uint32_t w[4];
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const uint32_t k = (k0 + 4u * i) & 255u;
			w[i] = k | ((k + 1u) << 8) | ((k + 2u) << 16) | ((k + 3u) << 24);
		}
		vx = u32x4{ w[0], w[1], w[2], w[3] };
		const uint32_t hi = (k0 >> 8) * 0x01010101u;
		if (x)
			*reinterpret_cast<GLOBAL u32x4*>(gptr(x) + base + k0) = vx;
		if (y)
			*reinterpret_cast<GLOBAL u32x4*>(gptr(y) + base + k0) = ~vx;
		if (h)
			*reinterpret_cast<GLOBAL u32x4*>(gptr(h) + base + k0) = u32x4{ hi, hi, hi, hi };
	}
}

// One word per output byte of the batch (batch-relative position a =
// A[b] + q): RES | byte, or the encoded position of the byte it copies,
// (source position) + 65536 -- always >= 0, and below a.  Every byte also
// goes to F (a history-derived one as a placeholder, rewritten by the jump
// round that resolves it), so no emit pass reads the words again.
//
// Each pointer is taken LZ4ADA_LINK_STEPS (2) steps here already, from the
// planes of its source byte (all final before this launch; the words of
// other blocks are not: they are being written by this launch): a source
// in one of the three blocks before b whose planes are x and z (mode 0) is
// a constant (z = 0: its x byte) or a pointer one step further back; a
// source before the batch is the tail's byte.  Anything else (a source
// further back, a mode 1 / 2 block) keeps its pointer for the jump rounds.
// Words are written only for a quad with a byte still open, and M says
// which bytes are final (1: no word written, 2: word written) -- unless
// `full` (a history-heavy batch, whose rounds then read words alone):
// every word, no M.  On the bench's linked frame (mixed) the two steps
// leave almost nothing to the rounds, so the 4 GiB of words are never
// written.
constexpr int64_t SPAN = 4 * TPB;  // positions per activity flag (k_link_jump)
#ifndef LZ4ADA_LINK_STEPS
#define LZ4ADA_LINK_STEPS 2  // pointer steps taken in init from the planes
#endif
#ifndef LZ4ADA_LINK_XCD
#define LZ4ADA_LINK_XCD 1
#endif
#ifndef LZ4ADA_LINK_LJ
#define LZ4ADA_LINK_LJ 4  // 256-position quads per lane and wave pass (a wave takes 256 LJ positions)
#endif
constexpr int LJ = LZ4ADA_LINK_LJ;
static_assert(256 * LJ <= 1024, "a wave pass meets at most two activity spans");
#ifndef LZ4ADA_LINK_J_UNROLL
#define LZ4ADA_LINK_J_UNROLL 1  // 0: a lane's four quads one after the other (fewer registers)
#endif

__global__ __launch_bounds__(TPB) void k_link_init(const uint8_t* __restrict__ x,
                                                   const uint8_t* __restrict__ z,
                                                   const uint8_t* __restrict__ y3,
                                                   const uint8_t* __restrict__ h3,
                                                   const uint8_t* __restrict__ three,
                                                   const lz4ada_block_desc* __restrict__ desc,
                                                   const lz4ada_block_status* __restrict__ st,
                                                   const int64_t* __restrict__ A, uint32_t nblocks,
                                                   const uint8_t* __restrict__ tail, int32_t tail_valid,
                                                   uint32_t* __restrict__ P, uint8_t* __restrict__ F,
                                                   uint8_t* __restrict__ M, uint8_t* __restrict__ act,
                                                   bool full, uint32_t gy)
{
	// gy parts per block.  Workgroups are dealt round-robin over the 8 XCDs
	// (MI355X_MICROARCH: blocks b and b + 8 share one), so workgroup L takes
	// unit (L % 8) x per + L / 8 of the nblocks x gy units: each XCD runs a
	// contiguous range of blocks in order, and a block's history sources --
	// the previous block's last 64 KiB of both planes, read a moment before
	// by the same XCD -- are likely still in that XCD's L2 (LZ4ADA_LINK_XCD=0
	// at build: blocks in launch order over all XCDs, for A/B)
	const uint32_t units = gy * nblocks;
#if LZ4ADA_LINK_XCD
	const uint32_t per = (units + 7) / 8;
	const uint32_t u = (blockIdx.x % 8) * per + blockIdx.x / 8;
#else
	const uint32_t u = blockIdx.x;
#endif
	if (u >= units)
		return;
	const uint32_t b = u / gy, part = u % gy;
	const uint64_t ob = desc[b].out_off;  // 256-byte aligned slot
	const int64_t len = st[b].out_len;
	const int64_t ab = A[b];
	const int32_t lane = int32_t(lane_id());
	const bool aligned = (ab & 3) == 0;
	const uint32_t hb = uint32_t(ab);  // + k: history position k's source, encoded + 65536
	// mode 0, planes x and z: a byte came from history iff z != 0, k = x |
	// z << 8; mode 1 (history positions below 256 read), x, z and y: iff z
	// != 0 or x != y, k = x | z << 8; mode 2 (z not decoded), x, y and h:
	// iff x != y, k = x | h << 8
	const uint32_t md = three ? three[b] : 0u;
	const bool tri = md != 0;
	const uint8_t* __restrict__ y = tri ? y3 : z;
	const uint8_t* __restrict__ h = md == 2 ? h3 : z;
	// the three blocks before b (a source is at most 65535 bytes back):
	// batch position (INT32_MAX: none, or not mode 0) and slot
	int32_t pa[3];
	uint64_t po[3];
	bool more = true;  // stop at the first block before b that is not mode 0
#pragma unroll
	for (int r = 0; r < 3; ++r) {
		const int32_t bb = int32_t(b) - 1 - r;
		more = more && bb >= 0 && (!three || three[bb] == 0);
		pa[r] = more ? int32_t(A[bb]) : INT32_MAX;
		po[r] = more ? desc[bb].out_off : 0;
	}
	// a wave takes 256 LJ positions of the block at a time, lane l its bytes
	// g0 + 4 l + 256 j (j < LJ): every load (a dword of each copy), word store (16 bytes)
	// and byte store (a dword) of the wave is one contiguous run (round 4
	// gave each lane 16 consecutive bytes: its four 16-byte word stores were
	// 64 bytes apart across the lanes)
	constexpr int64_t CH = 256 * LJ;  // positions per wave pass
	const int64_t wave0 = CH * (int64_t(part) * (TPB / 64) + (threadIdx.x >> 6));
	for (int64_t g0 = wave0; g0 < len; g0 += CH * int64_t(gy) * (TPB / 64)) {
		uint32_t wx[LJ], wy[LJ], wh[LJ];
#pragma unroll
		for (int j = 0; j < LJ; ++j) {
			const int64_t q = g0 + 256 * j + 4 * lane;
			wx[j] = wy[j] = wh[j] = 0;
			if (q + 4 <= len) {
				wx[j] = *reinterpret_cast<const GLOBAL uint32_t*>(gptr(x) + ob + q);
				if (tri)
					wy[j] = *reinterpret_cast<const GLOBAL uint32_t*>(gptr(y) + ob + q);
				wh[j] = *reinterpret_cast<const GLOBAL uint32_t*>(gptr(h) + ob + q);
			} else {
				for (int i = 0; i < 4; ++i)
					if (q + i < len) {
						wx[j] |= uint32_t(x[ob + q + i]) << (8 * i);
						wy[j] |= tri ? uint32_t(y[ob + q + i]) << (8 * i) : 0u;
						wh[j] |= uint32_t(h[ob + q + i]) << (8 * i);
					}
			}
		}
		// the spans (SPAN positions each) this wave pass meets: at most two
		const int64_t sA = (ab + g0) / SPAN;
		bool inA = false, inB = false;
		auto which = [&](int32_t t) { return t >= pa[0] ? 0 : (t >= pa[1] ? 1 : (t >= pa[2] ? 2 : 3)); };
#if LZ4ADA_LINK_J_UNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
		for (int j = 0; j < LJ; ++j) {
			const int64_t q = g0 + 256 * j + 4 * lane;
			const int32_t nv = int32_t(min<int64_t>(4, max<int64_t>(len - q, 0)));
			// words: branch-free per byte; positions fit 31 bits (bulk_linked
			// checks), so the words are 32-bit sums
			uint32_t v[4];
#pragma unroll
			for (int i = 0; i < 4; ++i) {
				const uint32_t bx = (wx[j] >> (8 * i)) & 255u;
				const uint32_t by = (wy[j] >> (8 * i)) & 255u;
				const uint32_t bh = (wh[j] >> (8 * i)) & 255u;
				const bool from_hist = md == 2 ? bx != by : (bh != 0u || (md == 1 && bx != by));
				const uint32_t hist = (from_hist && i < nv) ? 0xFFFFFFFFu : 0u;
				const uint32_t lit = RES | bx, ptr = hb + (bx | (bh << 8));
				v[i] = lit ^ ((lit ^ ptr) & hist);
			}
			// LZ4ADA_LINK_STEPS steps of every pointer: its source's planes (or
			// the tail's byte), a step's loads issued before any is used
			// (loading a quad's four consecutive source bytes as two dwords per
			// plane instead measured slower: mixed init 2.17 -> 2.60 ms)
#pragma unroll
			for (int stp = 0; stp < LZ4ADA_LINK_STEPS; ++stp) {
				uint32_t sx[4], sz[4];
#pragma unroll
				for (int i = 0; i < 4; ++i) {
					sx[i] = 0;
					sz[i] = 1;
					if (v[i] & RES)
						continue;
					const int32_t t = int32_t(v[i]) - int32_t(HISTORY_SIZE);
					if (t < 0) {
						if (t >= -tail_valid) {
							sx[i] = tail[HISTORY_SIZE + t];
							sz[i] = 0;
						}
					} else {
						const int r = which(t);
						if (r < 3) {
							const uint64_t o = (r == 0 ? po[0] : (r == 1 ? po[1] : po[2])) +
							                   uint64_t(t - (r == 0 ? pa[0] : (r == 1 ? pa[1] : pa[2])));
							sx[i] = x[o];
							sz[i] = z[o];
						}
					}
				}
#pragma unroll
				for (int i = 0; i < 4; ++i) {
					if (v[i] & RES)
						continue;
					const int32_t t = int32_t(v[i]) - int32_t(HISTORY_SIZE);
					const int r = which(t);
					const uint32_t base = uint32_t(r == 0 ? pa[0] : (r == 1 ? pa[1] : pa[2]));
					if (sz[i] == 0)
						v[i] = RES | sx[i];  // a constant (or the tail's byte)
					else if (t >= 0 && r < 3)
						v[i] = base + (sx[i] | (sz[i] << 8));  // its source's own pointer
				}
			}
			uint32_t u = 0;
#pragma unroll
			for (int i = 0; i < 4; ++i)
				u += (v[i] & RES) ? 0u : 1u;
			if (u) {  // the first jump round visits only the spans flagged here
				inA |= (ab + q) / SPAN == sA;
				inB |= (ab + q + nv - 1) / SPAN != sA;
			}
			// M: 0 open (its word written), 1 final with no word written, 2
			// final with its word written (RES | byte).  A quad's words are
			// written when one of them is open, or every word when `full`
			const bool wr = u != 0 || full;
			const uint32_t mf = wr ? 2u : 1u;
			if (nv == 4 && aligned) {
				if (wr)
					*reinterpret_cast<GLOBAL u32x4*>(gptr(P) + ab + q) = u32x4{ v[0], v[1], v[2], v[3] };
				*reinterpret_cast<GLOBAL uint32_t*>(gptr(F) + ab + q) =
				        (v[0] & 255u) | ((v[1] & 255u) << 8) | ((v[2] & 255u) << 16) | ((v[3] & 255u) << 24);
				if (!full)  // (full: the rounds never read M)
					*reinterpret_cast<GLOBAL uint32_t*>(gptr(M) + ab + q) =
					        ((v[0] >> 31) * mf) | (((v[1] >> 31) * mf) << 8) | (((v[2] >> 31) * mf) << 16) |
					        (((v[3] >> 31) * mf) << 24);
			} else {
				for (int i = 0; i < nv; ++i) {
					if (wr)
						P[ab + q + i] = v[i];
					F[ab + q + i] = uint8_t(v[i]);
					if (!full)
						M[ab + q + i] = uint8_t((v[i] >> 31) * mf);
				}
			}
		}
		const bool fA = __ballot(inA) != 0, fB = __ballot(inB) != 0;
		if (lane == 0) {
			if (fA)
				act[sA] = 1;
			if (fB)
				act[sA + 1] = 1;
		}
	}
}

// One pointer-jumping round over P[0, n).  ctr[0] = 1: a word is still
// unresolved after the round; ctr[1] = 1: a reference before the frame
// start (a position below -tail_valid).  tail: the 65536 output bytes
// before the batch.  Every unresolved word is replaced by its target's
// word; where a word changes, its four-byte group of F is rewritten (the
// last round to touch them leaves the final bytes).
//
// Activity flags: one per SPAN consecutive positions; act_out gets 1 for a
// span that still holds an unresolved word after the round, and a later
// round given act_in skips every span flagged 0 (most of the frame after
// the first round) instead of reading its words again.

// A whole span (SPAN positions) in one wave: lane l takes positions s0 +
// 256 j + 4 l + i (j, i < 4).  Its quads' M bytes first (1: final since
// init, whose word was never written), then the words of the quads that
// have an open position, then every open word's target together -- M, F
// and the word of the target, selected by its M -- four times the loads in
// flight of round 4's quad per thread.  Returns the words still unresolved.
template <bool full>
__device__ __forceinline__ uint32_t jump_span(GLOBAL uint32_t* Pg, const uint8_t* __restrict__ M, int64_t s0,
                                              int64_t n, const uint8_t* __restrict__ tail, int64_t tail_valid,
                                              uint8_t* __restrict__ F, uint32_t& bad)
{
	const int64_t l4 = 4 * int64_t(lane_id());

	uint32_t m[4];  // full: every word was written, M was not (all 0 here)
#pragma unroll
	for (int j = 0; j < 4; ++j) {
		const int64_t a0 = s0 + 256 * j + l4;  // 4-aligned: spans are SPAN-aligned positions
		if (full) {
			m[j] = 0;
		} else if (a0 + 4 <= n) {
			m[j] = *reinterpret_cast<const GLOBAL uint32_t*>(gptr(M) + a0);
		} else {
			m[j] = 0;
#pragma unroll
			for (int i = 0; i < 4; ++i)
				m[j] |= uint32_t(a0 + i < n ? M[a0 + i] : 1u) << (8 * i);
		}
	}
	auto all_final = [](uint32_t q) {  // every M byte of the quad nonzero
		return ((q & 0xffu) != 0u) & ((q & 0xff00u) != 0u) & ((q & 0xff0000u) != 0u) & ((q & 0xff000000u) != 0u);
	};
	if (!full && all_final(m[0]) && all_final(m[1]) && all_final(m[2]) && all_final(m[3]))
		return 0;  // every byte final since init
	uint32_t w[16];
#pragma unroll
	for (int j = 0; j < 4; ++j) {
		const int64_t a0 = s0 + 256 * j + l4;
#pragma unroll
		for (int i = 0; i < 4; ++i)
			w[4 * j + i] = RES;
		if (!full && all_final(m[j]))
			continue;
		if (a0 + 4 <= n) {
			const u32x4 v = *reinterpret_cast<const GLOBAL u32x4*>(Pg + a0);
			w[4 * j] = v.x;
			w[4 * j + 1] = v.y;
			w[4 * j + 2] = v.z;
			w[4 * j + 3] = v.w;
		} else {
#pragma unroll
			for (int i = 0; i < 4; ++i)
				w[4 * j + i] = a0 + i < n ? Pg[a0 + i] : RES;
		}
#pragma unroll
		for (int i = 0; i < 4; ++i)
			if ((m[j] >> (8 * i)) & 255u)
				w[4 * j + i] = RES;  // final since init (F has the byte)
	}
	// the source's word, and (sparse words) its M beside it; its F byte
	// only where M = 1 says the word was never written.  The M gathers
	// double a round's time where many words stay open after init (dense:
	// round 1 3.7 -> 6.1 ms), so such batches write every word (`full`)
	uint32_t rs = RES;
#pragma unroll
	for (int k = 0; k < 16; ++k)
		rs &= w[k];
	if (rs & RES)
		return 0;  // all final (their bytes are in F already)
	uint32_t f[16], mt[16];
#pragma unroll
	for (int k = 0; k < 16; ++k) {
		const int64_t t = int64_t(w[k] & ~RES) - HISTORY_SIZE;
		f[k] = w[k];
		mt[k] = 0;
		if (w[k] & RES)
			continue;
		if (t >= s0 + 256 * (k >> 2) + l4 + (k & 3)) {
			f[k] = ~0u;  // never expected: every pointer goes strictly back (reported as bad)
		} else if (t >= 0) {
			mt[k] = full ? 0u : M[t];  // full: every word was written
			f[k] = Pg[t];
		} else if (t >= -tail_valid) {
			f[k] = RES | tail[HISTORY_SIZE + t];
		} else {
			f[k] = ~0u;  // before the frame start
		}
	}
#pragma unroll
	for (int k = 0; k < 16; ++k)
		if (mt[k] == 1u)
			f[k] = RES | F[int64_t(w[k] & ~RES) - HISTORY_SIZE];  // final since init, no word
	uint32_t unres = 0;
#pragma unroll
	for (int j = 0; j < 4; ++j) {
		const int64_t a0 = s0 + 256 * j + l4;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const int k = 4 * j + i;
			if (w[k] & RES)
				continue;  // final (since init or an earlier round): F has its byte
			uint32_t x = f[k];
			if (x == ~0u) {
				++bad;
				x = w[k];
			}
			if (x != w[k]) {
				Pg[a0 + i] = x;
				if (x & RES)
					F[a0 + i] = uint8_t(x);
			}
			unres += (x & RES) ? 0u : 1u;
		}
	}
	return unres;
}

// Each wave takes 64 consecutive spans at a time: one coalesced load of
// their activity flags, then only the active ones, a span per step with no
// workgroup barrier (round 4 read each span's flag in its loop, one
// dependent load per span, which made a round that skips 94% of the spans
// cost 0.5 ms; until late round 5 a span was one quad per thread of the
// workgroup, a __syncthreads per span).
constexpr int32_t SPW = TPB;  // spans per workgroup pass (64 per wave)

// (one instance per word mode: `full` leaves out every M access, and the
// registers they take: 81 VGPRs against 50, 5 waves per SIMD against 8)
template <bool full>
__global__ __launch_bounds__(TPB) void k_link_jump(uint32_t* __restrict__ P, const uint8_t* __restrict__ M,
                                                   int64_t n, const uint8_t* __restrict__ tail,
                                                   int64_t tail_valid, uint8_t* __restrict__ F,
                                                   const uint8_t* __restrict__ act_in,
                                                   uint8_t* __restrict__ act_out,
                                                   uint32_t* __restrict__ ctr)
{
	uint32_t unres = 0, bad = 0;
	GLOBAL uint32_t* Pg = gptr(P);
	const int64_t nsp = (n + SPAN - 1) / SPAN;
	const int32_t lane = int32_t(lane_id());
	// groups of SPW spans; as in k_link_init each XCD takes a contiguous
	// range of them (workgroup L on XCD L % 8, the grid a multiple of 8), so
	// a span's sources -- mostly in the spans just before it -- were read by
	// the same XCD's L2
	const int64_t ng = (nsp + SPW - 1) / SPW;
#if LZ4ADA_LINK_XCD
	const int64_t per = (ng + 7) / 8, g_end = min<int64_t>(ng, (blockIdx.x % 8 + 1) * per);
	const int64_t g0 = (blockIdx.x % 8) * per + blockIdx.x / 8, gs = gridDim.x / 8;
#else
	const int64_t g_end = ng, g0 = blockIdx.x, gs = gridDim.x;
#endif
	for (int64_t g = g0; g < g_end; g += gs) {
		const int64_t sb = g * SPW + 64 * int64_t(threadIdx.x >> 6);
		const int64_t my = sb + lane;
		const bool a = my < nsp && (!act_in || act_in[my]);
		if (my < nsp && !a)
			act_out[my] = 0;
		for (uint64_t mm = __ballot(a); mm; mm &= mm - 1) {
			const int64_t span = sb + __builtin_ctzll(mm);
			const uint32_t u = jump_span<full>(Pg, M, span * SPAN, n, tail, tail_valid, F, bad);
			unres += u;
			const bool any = __ballot(u != 0) != 0;
			if (lane == 0)
				act_out[span] = uint8_t(any);
		}
	}
	flag_any(&ctr[0], unres != 0);
	flag_any(&ctr[1], bad != 0);
}


// tail_new = the last 65536 bytes of (tail_old ++ F[0, n)).
__global__ __launch_bounds__(TPB) void k_link_tail(const uint8_t* __restrict__ F, int64_t n,
                                                   const uint8_t* __restrict__ tail_old,
                                                   uint8_t* __restrict__ tail_new)
{
	for (int64_t i = int64_t(blockIdx.x) * TPB + threadIdx.x; i < HISTORY_SIZE;
	     i += int64_t(gridDim.x) * TPB) {
		const int64_t p = n - HISTORY_SIZE + i;
		tail_new[i] = p >= 0 ? F[p] : tail_old[HISTORY_SIZE + p];
	}
}

}  // namespace link

hipError_t launch_link_fill(uint8_t* x, uint8_t* y, uint8_t* h, const lz4ada_block_desc* d_desc,
                            uint32_t nblocks, hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(link::k_link_fill, dim3(nblocks, 4), dim3(link::TPB), 0, stream, x, y, h, d_desc,
	                   nblocks);
	return hipGetLastError();
}

hipError_t launch_link_init(const uint8_t* x, const uint8_t* z, const uint8_t* y, const uint8_t* h,
                            const uint8_t* d_three, const lz4ada_block_desc* d_desc,
                            const lz4ada_block_status* d_st, const int64_t* d_A, uint32_t nblocks,
                            int64_t block_max, const uint8_t* d_tail, int64_t tail_valid, uint32_t* d_P,
                            uint8_t* d_F, uint8_t* d_M, uint8_t* d_act, bool full, hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	// ~16 KiB of output per workgroup (each lane loops ~4 times): a
	// million 1 KiB workgroups cost more in dispatch than in work
	const int64_t per = 4 * 16 * link::TPB;
	const uint32_t gy = uint32_t(std::min<int64_t>(64, std::max<int64_t>(1, (block_max + per - 1) / per)));
	const uint32_t units = gy * nblocks;
	const uint32_t grid = LZ4ADA_LINK_XCD ? 8 * ((units + 7) / 8) : units;
	hipLaunchKernelGGL(link::k_link_init, dim3(grid), dim3(link::TPB), 0, stream, x, z, y, h, d_three, d_desc,
	                   d_st, d_A, nblocks, d_tail, int32_t(tail_valid), d_P, d_F, d_M, d_act, full, gy);
	return hipGetLastError();
}

static uint32_t grid_for(int64_t n, int64_t per_thread)
{
	const int64_t per = per_thread * link::TPB;
	return uint32_t(std::min<int64_t>(8192, std::max<int64_t>(1, (n + per - 1) / per)));
}

int64_t link_spans(int64_t n) { return (n + link::SPAN - 1) / link::SPAN; }

hipError_t launch_link_jump(uint32_t* d_P, const uint8_t* d_M, int64_t n, const uint8_t* d_tail,
                            int64_t tail_valid, uint8_t* d_F, const uint8_t* d_act_in, uint8_t* d_act_out,
                            uint32_t* d_ctr, bool full, hipStream_t stream)
{
	if (n <= 0)
		return hipSuccess;
	const uint32_t grid = (grid_for(n, 4 * link::SPW) + 7) / 8 * 8;  // (a multiple of 8: k_link_jump's XCD ranges)
	if (full)
		hipLaunchKernelGGL(link::k_link_jump<true>, dim3(grid), dim3(link::TPB), 0, stream,
		                   d_P, d_M, n, d_tail, tail_valid, d_F, d_act_in, d_act_out, d_ctr);
	else
		hipLaunchKernelGGL(link::k_link_jump<false>, dim3(grid), dim3(link::TPB), 0, stream,
		                   d_P, d_M, n, d_tail, tail_valid, d_F, d_act_in, d_act_out, d_ctr);
	return hipGetLastError();
}

hipError_t launch_link_tail(const uint8_t* d_F, int64_t n, const uint8_t* d_tail_old, uint8_t* d_tail_new,
                            hipStream_t stream)
{
	hipLaunchKernelGGL(link::k_link_tail, dim3(64), dim3(link::TPB), 0, stream, d_F, n, d_tail_old,
	                   d_tail_new);
	return hipGetLastError();
}

}  // namespace lz4ada
