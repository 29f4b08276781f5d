// lz4ada_kernels.hip -- gfx950 kernels of the MI355X LZ4Ada decompressor.
//
// Replaces the reference's hot path (lib/lz4ada.adb):
//   Decompress_Full_Block / Decompress_Sequence      :716-788
//   Write_Output (8-byte wild copy)                  :790-824
//   Output_With_History (overlap-safe match copy)    :845-904
//   Check_Checksum / Update_Checksum / XXHash32      :698-714, :923-1026
//
// Design (DESIGN.md has the long form):
//  * k_decode_blocks -- one 64-lane wavefront per independent block.  The
//    compressed stream is staged through a 1 KiB LDS window with 16 B/lane
//    loads.  Token boundaries are found speculatively: every lane parses a
//    token at 4 of the next 256 byte positions, the chain from the known
//    start is resolved by pointer doubling (6 LDS jump tables) and lane j
//    picks up the j-th token -- up to 64 sequences per step instead of one.
//    Output offsets come from a wave prefix scan; literals are copied into
//    a 4 KiB LDS batch buffer, matches are copied lane-parallel in
//    dependency rounds (a lane runs once every earlier match it reads from
//    is final), then the batch is flushed to HBM.  Overlapping matches use
//    src = start - off + (k mod off), so a lane never waits on its own
//    output.  Long or unusual tokens (multi-byte length extensions, runs
//    over 256 B, anything malformed) go through a wave-cooperative
//    one-token path that also produces the precise error.
//  * k_block_checksums / k_xxh32_update -- XXH32 with the four accumulator
//    lanes mapped onto lanes 0-3 of a wavefront; all 64 lanes load and
//    pre-multiply 256 B per step, ds_bpermute feeds the serial chain.
//  * k_serial_block -- reference-exact single-lane emulation of one block
//    on a device mirror of the caller's Buffer (Output_Pos wrap, history,
//    8-byte wild-copy overshoot and its D1 side effect).  Used by the
//    streaming Update facade and by the bulk path's exact fallback.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4ada_internal.h"

namespace lz4ada {

// ------------------------------------------------------------------ XXH32

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r)
{
	return (x << r) | (x >> (32 - r));
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Unaligned little-endian dword from global memory.  Reads only the aligned
// dwords that contain wanted bytes, so it never touches a page the data
// does not.
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p)
{
	uintptr_t a = reinterpret_cast<uintptr_t>(p);
	const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
	uint32_t sh = uint32_t(a & 3u);
	uint32_t lo = __builtin_nontemporal_load(q);
	if (sh == 0)
		return lo;
	uint32_t hi = __builtin_nontemporal_load(q + 1);
	return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

__device__ __forceinline__ uint32_t ld32u_cached(const uint8_t* p)
{
	uintptr_t a = reinterpret_cast<uintptr_t>(p);
	const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
	uint32_t sh = uint32_t(a & 3u);
	uint32_t lo = q[0];
	if (sh == 0)
		return lo;
	uint32_t hi = q[1];
	return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Advance the four XXH32 accumulators over `nstripes` 16-byte stripes at p.
// Whole-wave call; lane l carries accumulator (l & 3); every lane returns
// its (l & 3) accumulator.  (Process, lz4ada.adb:979-991.)
__device__ uint32_t wave_xxh32_stripes(uint32_t acc, const uint8_t* p, uint64_t nstripes)
{
	const uint32_t lane = lane_id();
	const uint64_t nwords = nstripes * 4;
	for (uint64_t w0 = 0; w0 < nwords; w0 += 256) {
		uint32_t prod[4];
#pragma unroll
		for (int r = 0; r < 4; ++r) {
			uint64_t w = w0 + uint64_t(r) * 64 + lane;
			uint32_t word = 0;
			if (w < nwords)
				word = ld32u(p + 4 * w);
			prod[r] = word * P2;
		}
		const uint64_t left = (nwords - w0) / 4;  // stripes left from w0
#pragma unroll
		for (int r = 0; r < 4; ++r) {
			uint32_t xs[16];
#pragma unroll
			for (int k = 0; k < 16; ++k)
				xs[k] = __shfl(prod[r], 4 * k + int(lane & 3u));
#pragma unroll
			for (int k = 0; k < 16; ++k) {
				if (uint64_t(r) * 16 + k < left)
					acc = rotl32(acc + xs[k], 13) * P1;
			}
		}
	}
	return acc;
}

// XXHash32.Final (lz4ada.adb:993-1017) from the 4 lanes + tail buffer.
__device__ uint32_t xxh32_final_dev(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3,
                                    const uint8_t* buf, int32_t bufsize, uint64_t total)
{
	uint32_t ret = uint32_t(total & 0xffffffffu);
	if (total >= 16)
		ret += rotl32(v0, 1) + rotl32(v1, 7) + rotl32(v2, 12) + rotl32(v3, 18);
	else
		ret += v2 + P5;
	int d = 0;
	while (d + 3 < bufsize) {
		uint32_t w = uint32_t(buf[d]) | (uint32_t(buf[d + 1]) << 8) |
		             (uint32_t(buf[d + 2]) << 16) | (uint32_t(buf[d + 3]) << 24);
		ret = rotl32(ret + w * P3, 17) * P4;
		d += 4;
	}
	while (d < bufsize) {
		ret = rotl32(ret + uint32_t(buf[d]) * P5, 11) * P1;
		d += 1;
	}
	ret = (ret ^ (ret >> 15)) * P2;
	ret = (ret ^ (ret >> 13)) * P3;
	return ret ^ (ret >> 16);
}

// One-shot XXH32 (seed 0) of [p, p+n) by a whole wave (XXHash32.Hash).
__device__ uint32_t wave_xxh32(const uint8_t* p, uint64_t n)
{
	const uint32_t lane = lane_id();
	const uint32_t init[4] = { P1 + P2, P2, 0u, 0u - P1 };
	uint32_t acc = init[lane & 3u];
	const uint64_t ns = n / 16;
	acc = wave_xxh32_stripes(acc, p, ns);
	uint32_t v0 = __shfl(acc, 0), v1 = __shfl(acc, 1), v2 = __shfl(acc, 2),
	         v3 = __shfl(acc, 3);
	uint8_t tail[16];
	const int32_t tl = int32_t(n - ns * 16);
	for (int i = 0; i < tl; ++i)
		tail[i] = p[ns * 16 + i];
	return xxh32_final_dev(v0, v1, v2, v3, tail, tl, n);
}

__global__ __launch_bounds__(64) void k_block_checksums(const uint8_t* __restrict__ frame,
                                                         const lz4ada_block_desc* __restrict__ desc,
                                                         uint32_t nblocks,
                                                         lz4ada_block_status* __restrict__ st)
{
	const uint32_t b = blockIdx.x;
	if (b >= nblocks)
		return;
	const lz4ada_block_desc d = desc[b];
	if (!(d.flags & LZ4ADA_BLOCK_HAS_CKSUM))
		return;
	uint32_t h = wave_xxh32(frame + d.in_off, d.in_len);
	if (lane_id() == 0)
		st[b].cksum = h;
}

__global__ __launch_bounds__(64) void k_output_checksums(const uint8_t* __restrict__ out,
                                                          const lz4ada_block_desc* __restrict__ desc,
                                                          uint32_t nblocks,
                                                          const lz4ada_block_status* __restrict__ st,
                                                          uint32_t* __restrict__ hash)
{
	const uint32_t b = blockIdx.x;
	if (b >= nblocks)
		return;
	uint32_t h = wave_xxh32(out + desc[b].out_off, st[b].out_len);
	if (lane_id() == 0)
		hash[b] = h;
}

// Streaming XXHash32.Update (lz4ada.adb:942-977) on a device-resident state.
__global__ __launch_bounds__(64) void k_xxh32_update(lz4ada_xxh32_state* __restrict__ s,
                                                      const uint8_t* __restrict__ data,
                                                      uint64_t len)
{
	const uint32_t lane = lane_id();
	uint32_t acc = s->state[lane & 3u];
	uint8_t buf[16];
	int32_t bs = s->buffer_size;
	for (int i = 0; i < 16; ++i)
		buf[i] = s->buffer[i];
	uint64_t total = s->total_length + len;
	uint64_t pos = 0;
	// Refill a partially filled stripe byte by byte (Update1, :965-977).
	if (bs > 0) {
		while (bs < 16 && pos < len)
			buf[bs++] = data[pos++];
		if (bs == 16) {
			uint32_t w = uint32_t(buf[4 * (lane & 3u)]) |
			             (uint32_t(buf[4 * (lane & 3u) + 1]) << 8) |
			             (uint32_t(buf[4 * (lane & 3u) + 2]) << 16) |
			             (uint32_t(buf[4 * (lane & 3u) + 3]) << 24);
			acc = rotl32(acc + w * P2, 13) * P1;
			bs = 0;
		}
	}
	if (bs == 0) {
		const uint64_t ns = (len - pos) / 16;
		acc = wave_xxh32_stripes(acc, data + pos, ns);
		pos += ns * 16;
		while (pos < len)
			buf[bs++] = data[pos++];
	}
	uint32_t v0 = __shfl(acc, 0), v1 = __shfl(acc, 1), v2 = __shfl(acc, 2), v3 = __shfl(acc, 3);
	uint32_t h = xxh32_final_dev(v0, v1, v2, v3, buf, bs, total);
	if (lane == 0) {
		s->state[0] = v0;
		s->state[1] = v1;
		s->state[2] = v2;
		s->state[3] = v3;
		for (int i = 0; i < 16; ++i)
			s->buffer[i] = buf[i];
		s->buffer_size = bs;
		s->total_length = total;
		s->hash = h;
	}
}

// --------------------------------------------------------- block decoder

constexpr int WIN = 1024;        // LDS window of compressed bytes
constexpr int NC = 256;          // speculative token candidates per step
constexpr int TERM = 0xffff;     // jump-table terminal
constexpr int LOOKAHEAD = 544;   // bytes a candidate token may touch
constexpr int OUTB = 4096;       // LDS batch output capacity
constexpr int BIG = 256;         // longer sequences take the one-token path

enum TokKind : int { TK_NORMAL = 0, TK_LAST = 1, TK_COMPLEX = 2, TK_ERR = 3 };

struct Tok {
	int32_t lit;   // block-relative literal start
	int32_t L;     // literal count
	int32_t ml;    // match length incl. +4 (0 for TK_LAST)
	int32_t off;   // match offset
	int32_t next;  // block-relative position of the next token
	int32_t kind;
};

// Parse the token at block-relative position c from the LDS window.
// wofs maps block-relative x to window index x + wofs; wend is the
// block-relative end of the window.  Only single-byte length extensions
// are resolved here (TK_COMPLEX otherwise).  Mirrors Decompress_Sequence
// (lz4ada.adb:737-777) for the non-error cases; every malformed shape is
// TK_ERR and left to the one-token path, which raises precisely.
__device__ __forceinline__ Tok parse_tok(const uint8_t* win, int64_t wofs, int64_t c,
                                         int64_t n, int64_t wend)
{
	Tok t;
	t.lit = 0;
	t.L = 0;
	t.ml = 0;
	t.off = 0;
	t.next = 0;
	t.kind = TK_ERR;
	if (c >= n || c >= wend)
		return t;
	const uint32_t tk = win[c + wofs];
	int64_t L = tk >> 4, M = tk & 15, p = c + 1;
	if (L == 15) {
		if (p >= n) return t;
		if (p >= wend) { t.kind = TK_COMPLEX; return t; }
		uint32_t e = win[p + wofs];
		++p;
		if (e == 255) { t.kind = TK_COMPLEX; return t; }
		L += e;
	}
	t.lit = int32_t(p);
	t.L = int32_t(L);
	p += L;
	if (p > wend) { t.kind = TK_COMPLEX; return t; }
	if (p >= n) {
		if (p == n && M == 0) {
			t.kind = TK_LAST;
			t.next = int32_t(n);
		}
		return t;  // else ML-after-literals / overrun: TK_ERR
	}
	if (p + 1 >= n) return t;
	if (p + 1 >= wend) { t.kind = TK_COMPLEX; return t; }
	const uint32_t off = uint32_t(win[p + wofs]) | (uint32_t(win[p + 1 + wofs]) << 8);
	p += 2;
	if (off == 0) return t;
	if (M == 15) {
		if (p >= n) return t;
		if (p >= wend) { t.kind = TK_COMPLEX; return t; }
		uint32_t e = win[p + wofs];
		++p;
		if (e == 255) { t.kind = TK_COMPLEX; return t; }
		M += e;
	}
	t.off = int32_t(off);
	t.ml = int32_t(M + 4);
	t.next = int32_t(p);
	t.kind = TK_NORMAL;
	return t;
}

__device__ __forceinline__ int64_t wave_min_i64(int64_t v)
{
#pragma unroll
	for (int m = 32; m >= 1; m >>= 1) {
		int64_t o = __shfl_xor(v, m);
		v = o < v ? o : v;
	}
	return v;
}

// Inclusive prefix sum over the wave.
__device__ __forceinline__ int32_t wave_incl_scan(int32_t v)
{
	const int lane = int(lane_id());
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		int32_t o = __shfl_up(v, d);
		if (lane >= d)
			v += o;
	}
	return v;
}

// Sum of a length extension (Process_Variable_Length, lz4ada.adb:724-735)
// starting at block-relative p, 64 bytes per step.  Returns false when the
// block ends first (D4).  Whole-wave, uniform.
__device__ bool wave_ext_sum(const uint8_t* in, int64_t n, int64_t& p, int64_t& sum)
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
__device__ void wave_copy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int64_t n)
{
	const uint32_t lane = lane_id();
	// Align the destination to 16 B, then move 16 B per lane per step.
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
		const uint8_t* s = src + 16 * i;
		uint4 v;
		v.x = ld32u(s);
		v.y = ld32u(s + 4);
		v.z = ld32u(s + 8);
		v.w = ld32u(s + 12);
		*reinterpret_cast<uint4*>(dst + 16 * i) = v;
	}
	for (int64_t i = nv * 16 + lane; i < n; i += 64)
		dst[i] = src[i];
}

// One token at block-relative s, wave-cooperative, straight to global
// memory.  Handles every shape, including the malformed ones.
// Returns false with st filled on error; advances s and o.
__device__ bool one_token(const uint8_t* __restrict__ in, int64_t n, uint8_t* __restrict__ ob,
                          int64_t cap, int64_t& s, int64_t& o, lz4ada_block_status& st)
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
		__syncthreads();
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
	if (q0 < 0) {
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
	__syncthreads();  // literals above are visible to every lane
	if (off >= ml) {
		wave_copy(ob + o, ob + q0, ml);
	} else {
		// Overlap: byte k repeats source byte (k mod off); every source
		// byte precedes the match, so all lanes run at once.
		for (int64_t k = lane; k < ml; k += 64)
			ob[o + k] = ob[q0 + (k % off)];
	}
	o += ml;
	s = p;
	__syncthreads();
	return true;
}

__global__ __launch_bounds__(64) void k_decode_blocks(const uint8_t* __restrict__ frame,
                                                       uint64_t frame_len,
                                                       const lz4ada_block_desc* __restrict__ desc,
                                                       uint32_t nblocks, uint8_t* __restrict__ out,
                                                       lz4ada_block_status* __restrict__ status)
{
	__shared__ __attribute__((aligned(16))) uint8_t win[WIN];
	__shared__ uint16_t J[6][NC];
	__shared__ __attribute__((aligned(16))) uint8_t outb[OUTB];

	const uint32_t b = blockIdx.x;
	if (b >= nblocks)
		return;
	const uint32_t lane = lane_id();
	const lz4ada_block_desc d = desc[b];
	const uint8_t* __restrict__ in = frame + d.in_off;
	uint8_t* __restrict__ ob = out + d.out_off;
	const int64_t n = d.in_len;
	const int64_t cap = d.out_cap;

	lz4ada_block_status st;
	st.code = DS_OK;
	st.aux = 0;
	st.detail = 0;
	st.err_out_pos = 0;
	st.out_len = 0;

	if (d.flags & LZ4ADA_BLOCK_STORED) {
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
		return;
	}

	const uintptr_t in_addr = reinterpret_cast<uintptr_t>(in);
	const uintptr_t lim_addr = reinterpret_cast<uintptr_t>(frame) + frame_len;
	int64_t s = 0, o = 0;
	int64_t wofs = 0, wend = -1;  // window: block-relative [wend - WIN, wend)
	bool ok = true;

	while (s < n) {
		// ---- (re)stage the compressed window so [s, s + LOOKAHEAD) is in it
		if (s + LOOKAHEAD > wend || s + wofs < 0) {
			const uintptr_t wg = (in_addr + uintptr_t(s)) & ~uintptr_t(15);
			const uintptr_t ga = wg + 16u * lane;
			uint4 v;
			if (ga + 16 <= lim_addr) {
				v = *reinterpret_cast<const uint4*>(ga);
			} else {
				uint8_t t[16];
				for (int i = 0; i < 16; ++i)
					t[i] = (ga + i < lim_addr) ? *reinterpret_cast<const uint8_t*>(ga + i) : 0;
				v.x = t[0] | (t[1] << 8) | (t[2] << 16) | (uint32_t(t[3]) << 24);
				v.y = t[4] | (t[5] << 8) | (t[6] << 16) | (uint32_t(t[7]) << 24);
				v.z = t[8] | (t[9] << 8) | (t[10] << 16) | (uint32_t(t[11]) << 24);
				v.w = t[12] | (t[13] << 8) | (t[14] << 16) | (uint32_t(t[15]) << 24);
			}
			*reinterpret_cast<uint4*>(&win[16 * lane]) = v;
			wofs = int64_t(in_addr - wg);
			wend = WIN - wofs;
			__syncthreads();
		}

		// ---- speculative candidates: next-token pointer for s + [0, 256)
#pragma unroll
		for (int i = 0; i < NC / 64; ++i) {
			const int k = int(lane) + 64 * i;
			const Tok t = parse_tok(win, wofs, s + k, n, wend);
			int nx = TERM;
			if (t.kind == TK_NORMAL) {
				const int64_t rel = int64_t(t.next) - s;
				if (rel < NC)
					nx = int(rel);
			}
			J[0][k] = uint16_t(nx);
		}
		__syncthreads();
		// ---- pointer doubling: J[r+1][k] = J[r][J[r][k]]
#pragma unroll
		for (int r = 0; r < 5; ++r) {
#pragma unroll
			for (int i = 0; i < NC / 64; ++i) {
				const int k = int(lane) + 64 * i;
				const int a = J[r][k];
				J[r + 1][k] = uint16_t(a == TERM ? TERM : J[r][a]);
			}
			__syncthreads();
		}
		// ---- lane j finds the j-th token of the chain that starts at s
		int c = 0;
#pragma unroll
		for (int r = 0; r < 6; ++r) {
			if (((lane >> r) & 1u) && c != TERM)
				c = J[r][c];
		}
		const bool inchain = (c != TERM);
		Tok t = parse_tok(win, wofs, s + (inchain ? c : 0), n, wend);
		const int32_t len = (t.kind == TK_NORMAL) ? t.L + t.ml : (t.kind == TK_LAST ? t.L : 0);
		bool good = inchain && (t.kind == TK_NORMAL || t.kind == TK_LAST) && len <= BIG;
		// batch = longest prefix of good lanes that fits OUTB, the block
		// slot, and references nothing before the block start
		const uint64_t bad0 = __ballot(!good);
		int cnt = bad0 ? (__ffsll((long long)bad0) - 1) : 64;
		const int32_t lenm = (int(lane) < cnt) ? len : 0;
		const int32_t incl = wave_incl_scan(lenm);
		const int32_t ostart = incl - lenm;
		const int64_t d0 = o + ostart + t.L;           // match destination
		const int64_t q0 = d0 - t.off;                  // match source start
		const bool fits = (incl <= OUTB) && (o + incl <= cap) &&
		                  (t.kind != TK_NORMAL || q0 >= 0);
		const uint64_t bad1 = __ballot(!(fits) && int(lane) < cnt);
		if (bad1) {
			const int f = __ffsll((long long)bad1) - 1;
			cnt = f < cnt ? f : cnt;
		}
		if (cnt == 0) {
			__syncthreads();
			if (!one_token(in, n, ob, cap, s, o, st)) {
				ok = false;
				break;
			}
			continue;
		}
		const bool mine = int(lane) < cnt;
		const int32_t blen = __shfl(incl, cnt - 1);
		const int32_t last_next = __shfl(t.next, cnt - 1);

		// ---- literals: window -> batch buffer
		if (mine) {
			const int64_t src = t.lit + wofs;
			for (int32_t i = 0; i < t.L; ++i)
				outb[ostart + i] = win[src + i];
		}
		__syncthreads();
		// ---- matches, in dependency rounds
		bool pend = mine && t.kind == TK_NORMAL;
		const int64_t srcend = (q0 + t.ml < d0) ? q0 + t.ml : d0;
		while (__ballot(pend)) {
			const int64_t m = wave_min_i64(pend ? d0 : INT64_MAX);
			const bool ready = pend && srcend <= m;
			if (ready) {
				const int32_t ml = t.ml, off = t.off;
				int32_t r = 0;
				for (int32_t k = 0; k < ml; ++k) {
					const int64_t sp = q0 + r;
					const uint8_t v = (sp < o) ? ob[sp] : outb[sp - o];
					outb[d0 - o + k] = v;
					if (++r == off)
						r = 0;
				}
			}
			pend = pend && !ready;
			__syncthreads();
		}
		// ---- flush the batch to HBM
		for (int32_t i = int32_t(lane); i < blen; i += 64)
			ob[o + i] = outb[i];
		__syncthreads();
		o += blen;
		s = last_next;
	}

	if (lane == 0) {
		status[b].code = ok ? int32_t(DS_OK) : st.code;
		status[b].aux = st.aux;
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

hipError_t launch_decode_blocks(const uint8_t* d_frame, uint64_t frame_len,
                                const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                uint8_t* d_out, lz4ada_block_status* d_status,
                                hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(k_decode_blocks, dim3(nblocks), dim3(64), 0, stream, d_frame, frame_len,
	                   d_desc, nblocks, d_out, d_status);
	return hipGetLastError();
}

hipError_t launch_block_checksums(const uint8_t* d_frame, const lz4ada_block_desc* d_desc,
                                  uint32_t nblocks, lz4ada_block_status* d_status,
                                  hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(k_block_checksums, dim3(nblocks), dim3(64), 0, stream, d_frame, d_desc,
	                   nblocks, d_status);
	return hipGetLastError();
}

hipError_t launch_output_checksums(const uint8_t* d_out, const lz4ada_block_desc* d_desc,
                                   uint32_t nblocks, const lz4ada_block_status* d_status,
                                   uint32_t* d_hash, hipStream_t stream)
{
	if (nblocks == 0)
		return hipSuccess;
	hipLaunchKernelGGL(k_output_checksums, dim3(nblocks), dim3(64), 0, stream, d_out, d_desc,
	                   nblocks, d_status, d_hash);
	return hipGetLastError();
}

hipError_t launch_xxh32_update(lz4ada_xxh32_state* d_state, const uint8_t* d_data, uint64_t len,
                               hipStream_t stream)
{
	hipLaunchKernelGGL(k_xxh32_update, dim3(1), dim3(64), 0, stream, d_state, d_data, len);
	return hipGetLastError();
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
