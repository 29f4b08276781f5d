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
//  * three decodes of the whole batch with different history patterns at
//    position k of the region: X = k & 255, Y = ~X, H = k >> 8.  Decoding
//    only moves bytes, so an output byte equal in X and Y is a constant (a
//    literal, maybe copied on), and one that differs came from history
//    position k = X | H << 8 -- byte (k - 65536) relative to its block start;
//  * k_link_init turns the three outputs into one word per output byte, a
//    resolved byte or a pointer to an earlier position of the frame;
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
// round that resolves it), so no emit pass reads the words again.  16 bytes
// per lane: dwordx4 loads of the three copies, four 16-byte word stores.
constexpr int64_t SPAN = 4 * TPB;  // positions per activity flag (k_link_jump)

__global__ __launch_bounds__(TPB) void k_link_init(const uint8_t* __restrict__ x,
                                                   const uint8_t* __restrict__ z,
                                                   const uint8_t* __restrict__ y3,
                                                   const uint8_t* __restrict__ h3,
                                                   const uint8_t* __restrict__ three,
                                                   const lz4ada_block_desc* __restrict__ desc,
                                                   const lz4ada_block_status* __restrict__ st,
                                                   const int64_t* __restrict__ A, uint32_t nblocks,
                                                   uint32_t* __restrict__ P, uint8_t* __restrict__ F,
                                                   uint8_t* __restrict__ act)
{
	// grid (parts, blocks): consecutive workgroups take consecutive parts
	// of one block, so the waves in flight share pages of the five arrays
	const uint32_t b = blockIdx.y;
	if (b >= nblocks)
		return;
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
	// a wave takes 1 KiB of the block at a time, lane l its bytes g0 + 4 l +
	// 256 j (j < 4): every load (a dword of each copy), word store (16 bytes)
	// and byte store (a dword) of the wave is one contiguous run (round 4
	// gave each lane 16 consecutive bytes: its four 16-byte word stores were
	// 64 bytes apart across the lanes)
	const int64_t wave0 = 1024 * (int64_t(blockIdx.x) * (TPB / 64) + (threadIdx.x >> 6));
	for (int64_t g0 = wave0; g0 < len; g0 += 1024 * int64_t(gridDim.x) * (TPB / 64)) {
		uint32_t wx[4], wy[4], wh[4];
#pragma unroll
		for (int j = 0; j < 4; ++j) {
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
		// the spans (SPAN positions each) this wave's kilobyte meets: at most two
		const int64_t sA = (ab + g0) / SPAN;
		bool inA = false, inB = false;
#pragma unroll
		for (int j = 0; j < 4; ++j) {
			const int64_t q = g0 + 256 * j + 4 * lane;
			const int32_t nv = int32_t(min<int64_t>(4, max<int64_t>(len - q, 0)));
			// branch-free per byte; positions fit 31 bits (bulk_linked checks),
			// so the words are 32-bit sums
			uint32_t v[4], u = 0;
#pragma unroll
			for (int i = 0; i < 4; ++i) {
				const uint32_t bx = (wx[j] >> (8 * i)) & 255u;
				const uint32_t by = (wy[j] >> (8 * i)) & 255u;
				const uint32_t bh = (wh[j] >> (8 * i)) & 255u;
				const bool from_hist = md == 2 ? bx != by : (bh != 0u || (md == 1 && bx != by));
				const uint32_t hist = (from_hist && i < nv) ? 0xFFFFFFFFu : 0u;
				const uint32_t lit = RES | bx, ptr = hb + (bx | (bh << 8));
				v[i] = lit ^ ((lit ^ ptr) & hist);
				u += hist & 1u;
			}
			if (u) {  // the first jump round visits only the spans flagged here
				inA |= (ab + q) / SPAN == sA;
				inB |= (ab + q + nv - 1) / SPAN != sA;
			}
			if (nv == 4 && aligned) {
				*reinterpret_cast<GLOBAL u32x4*>(gptr(P) + ab + q) = u32x4{ v[0], v[1], v[2], v[3] };
				*reinterpret_cast<GLOBAL uint32_t*>(gptr(F) + ab + q) =
				        (v[0] & 255u) | ((v[1] & 255u) << 8) | ((v[2] & 255u) << 16) | ((v[3] & 255u) << 24);
			} else {
				for (int i = 0; i < nv; ++i) {
					P[ab + q + i] = v[i];
					F[ab + q + i] = uint8_t(v[i]);
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
// start (a position below -tail_valid).  tail: the 65536 output bytes before the batch.  A
// lane takes four positions: their words, then every unresolved one's
// target word, loaded together before any is used; where a word changes the
// lane rewrites its four bytes of F (the last round to touch them leaves the
// final bytes).
//
// Activity flags: a workgroup pass covers SPAN consecutive positions; act_out
// gets 1 for a span that still holds an unresolved word after the round, and
// a later round given act_in skips every span flagged 0 (most of the frame
// after the first round) instead of reading its words again.

// Positions a0 .. a0+3 (a0 < n): one jump of every unresolved word, their
// bytes to F.  Returns the words still unresolved.
__device__ __forceinline__ uint32_t jump4(GLOBAL uint32_t* Pg, int64_t a0, int64_t n,
                                          const uint8_t* __restrict__ tail, int64_t tail_valid,
                                          uint8_t* __restrict__ F, uint32_t& bad)
{
	uint32_t w[4];
	const bool full = a0 + 4 <= n;
	if (full) {
		const u32x4 v = *reinterpret_cast<const GLOBAL u32x4*>(Pg + a0);
		w[0] = v.x;
		w[1] = v.y;
		w[2] = v.z;
		w[3] = v.w;
	} else {
#pragma unroll
		for (int i = 0; i < 4; ++i)
			w[i] = a0 + i < n ? Pg[a0 + i] : RES;
	}
	if ((w[0] & w[1] & w[2] & w[3]) & RES)
		return 0;  // all resolved (their bytes are in F already)
	uint32_t f[4];
#pragma unroll
	for (int i = 0; i < 4; ++i) {
		const int64_t t = int64_t(w[i] & ~RES) - HISTORY_SIZE;
		f[i] = w[i];
		if (w[i] & RES)
			continue;
		if (t >= 0)
			f[i] = Pg[t];  // the source's word: resolved, or a pointer further back
		else if (t >= -tail_valid)
			f[i] = RES | tail[HISTORY_SIZE + t];
		else
			f[i] = ~0u;  // before the frame start
	}
	uint32_t o = 0, unres = 0;
#pragma unroll
	for (int i = 0; i < 4; ++i) {
		if (f[i] == ~0u) {
			++bad;
			f[i] = w[i];
		}
		if (f[i] != w[i])
			Pg[a0 + i] = f[i];
		unres += (f[i] & RES) ? 0u : 1u;
		o |= (f[i] & 255u) << (8 * i);
	}
	GLOBAL uint8_t* fb = gptr(F) + a0;
	if (full && (reinterpret_cast<uintptr_t>(fb) & 3u) == 0) {
		*reinterpret_cast<GLOBAL uint32_t*>(fb) = o;
	} else {
#pragma unroll
		for (int i = 0; i < 4; ++i)
			if (a0 + i < n)
				fb[i] = uint8_t(o >> (8 * i));
	}
	return unres;
}

// A workgroup takes SPW consecutive spans: it loads their SPW activity
// flags at once (one coalesced load), then visits only the active ones --
// round 4 read each span's flag in its loop, one dependent load per span,
// which made a round that skips 94% of the spans cost 0.5 ms.
constexpr int32_t SPW = TPB;  // spans per workgroup

__global__ __launch_bounds__(TPB) void k_link_jump(uint32_t* __restrict__ P, int64_t n,
                                                   const uint8_t* __restrict__ tail,
                                                   int64_t tail_valid, uint8_t* __restrict__ F,
                                                   const uint8_t* __restrict__ act_in,
                                                   uint8_t* __restrict__ act_out,
                                                   uint32_t* __restrict__ ctr)
{
	__shared__ uint64_t on[SPW / 64];
	uint32_t unres = 0, bad = 0;
	GLOBAL uint32_t* Pg = gptr(P);
	const int64_t nsp = (n + SPAN - 1) / SPAN;
	const int32_t tid = int32_t(threadIdx.x);
	for (int64_t sb = int64_t(blockIdx.x) * SPW; sb < nsp; sb += int64_t(gridDim.x) * SPW) {
		const int64_t my = sb + tid;
		const bool a = my < nsp && (!act_in || act_in[my]);
		const uint64_t m = __ballot(a);
		if (lane_id() == 0)
			on[tid >> 6] = m;
		if (my < nsp && !a)
			act_out[my] = 0;
		__syncthreads();
		for (int q = 0; q < SPW / 64; ++q) {
			for (uint64_t mm = on[q]; mm; mm &= mm - 1) {
				const int64_t span = sb + 64 * q + __builtin_ctzll(mm);
				const int64_t a0 = span * SPAN + 4 * int64_t(tid);
				const uint32_t u = a0 < n ? jump4(Pg, a0, n, tail, tail_valid, F, bad) : 0u;
				unres += u;
				const int any = __syncthreads_or(u != 0);
				if (tid == 0)
					act_out[span] = uint8_t(any);
			}
		}
		__syncthreads();  // on[] is rewritten for the next spans
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
                            int64_t block_max, uint32_t* d_P, uint8_t* d_F, uint8_t* d_act,
                            hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	// ~16 KiB of output per workgroup (each lane loops ~4 times): a
	// million 1 KiB workgroups cost more in dispatch than in work
	const int64_t per = 4 * 16 * link::TPB;
	const uint32_t gy = uint32_t(std::min<int64_t>(64, std::max<int64_t>(1, (block_max + per - 1) / per)));
	hipLaunchKernelGGL(link::k_link_init, dim3(gy, nblocks), dim3(link::TPB), 0, stream, x, z, y, h, d_three,
	                   d_desc, d_st, d_A, nblocks, d_P, d_F, d_act);
	return hipGetLastError();
}

static uint32_t grid_for(int64_t n, int64_t per_thread)
{
	const int64_t per = per_thread * link::TPB;
	return uint32_t(std::min<int64_t>(8192, std::max<int64_t>(1, (n + per - 1) / per)));
}

int64_t link_spans(int64_t n) { return (n + link::SPAN - 1) / link::SPAN; }

hipError_t launch_link_jump(uint32_t* d_P, int64_t n, const uint8_t* d_tail, int64_t tail_valid,
                            uint8_t* d_F, const uint8_t* d_act_in, uint8_t* d_act_out, uint32_t* d_ctr,
                            hipStream_t stream)
{
	if (n <= 0)
		return hipSuccess;
	hipLaunchKernelGGL(link::k_link_jump, dim3(grid_for(n, 4 * link::SPW)), dim3(link::TPB), 0, stream, d_P, n, d_tail,
	                   tail_valid, d_F, d_act_in, d_act_out, d_ctr);
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
