// lz4ada_bulk.cpp -- the bulk frame paths of the MI355X LZ4Ada decompressor
// (SURVEY §8a-a5, §8f): the frame indexer (the size-word walk of
// lib/lz4ada.adb:525-585), independent blocks in one device pass (block
// checksums + the index-driven decoder, lz4ada_idx.hip), linked frames
// against synthetic history resolved on the GPU (lz4ada_linked.hip), the
// reference-exact resume at a failing block, and their C-ABI
// (lz4ada_decode_frame / _stream / _alloc / _partial, the device-resident
// entries).
#include "lz4ada_host_common.h"

using namespace lz4ada;

// ------------------------------------------------------------ bulk path

namespace lz4ada {

// Walk one frame's block size words (Try_Detect_Input_Length semantics,
// lz4ada.adb:525-585, under Init_With_Header(Single_Frame)).
static void index_frame(const uint8_t* f, int64_t len, lz4ada_frame_info& info,
                        std::vector<lz4ada_block_desc>* descs)
{
	memset(&info, 0, sizeof info);
	if (len < 7)
		raise(LZ4ADA_ASSERTION_ERROR, "failed precondition from lz4ada.ads:243");
	Meta mt;
	mt.memory_reservation = LZ4ADA_USE_FIRST;
	uint8_t hb[20];
	int64_t pos = 0;
	while (mt.header_parsing != HDR_DONE) {
		if (pos >= len)
			raise(LZ4ADA_TOO_FEW_HEADER_BYTES,
			      "Expected at least " + img_u(mt.size_remaining) +
			              " more bytes but header input has already ended.");
		pos += header_bytes(mt, hb, f + pos, len - pos);
	}
	info.header_len = pos;
	const int64_t bmax = block_size_of(mt.memory_reservation);
	info.block_max = bmax;
	if (mt.is_format == F_SKIPPABLE) {
		info.format = LZ4ADA_FORMAT_SKIPPABLE;
		info.frame_len = pos + int64_t(mt.size_remaining);
		info.nblocks = 0;
		return;
	}
	info.format = mt.is_format == F_LEGACY ? LZ4ADA_FORMAT_LEGACY : LZ4ADA_FORMAT_MODERN;
	info.flg = mt.flg;
	info.bd = mt.bd;
	info.block_checksum = mt.block_checksum_length ? 1 : 0;
	info.content_checksum = mt.content_checksum_length ? 1 : 0;
	info.has_content_size = mt.has_content_size ? 1 : 0;
	info.independent = (mt.is_format == F_LEGACY) || (mt.flg & 0x20u) ? 1 : 0;
	info.content_size = mt.has_content_size ? mt.size_remaining : 0;
	const int64_t inbuf = bmax + mt.block_checksum_length + BLOCK_SIZE_BYTES;
	const int64_t additional = BLOCK_SIZE_BYTES + mt.block_checksum_length;
	int64_t nb = 0;
	for (;;) {
		if (pos + 4 > len) {
			if (mt.is_format == F_LEGACY && pos == len)
				break;  // legacy frames end with the input
			raise(LZ4ADA_DATA_CORRUPTION, "Frame truncated: block size word missing.");
		}
		uint32_t word = load32(f + pos);
		if (mt.is_format == F_MODERN && word == 0) {
			pos += 4;
			if (mt.content_checksum_length) {
				if (pos + 4 > len)
					raise(LZ4ADA_DATA_CORRUPTION, "Frame truncated: content checksum missing.");
				info.content_checksum_declared = load32(f + pos);
				pos += 4;
			}
			break;
		}
		if (mt.is_format == F_LEGACY && is_any_magic(word))
			break;  // next frame starts here
		bool stored = false;
		if (mt.is_format == F_MODERN) {
			stored = (word & 0x80000000u) != 0;
			word &= 0x7ffffffu;
		}
		if (int64_t(word) + additional > inbuf)
			raise(LZ4ADA_DATA_CORRUPTION,
			      "Declared maximum data length exceeded. Buffer has " + img(inbuf) +
			              " bytes, current block requires " + img_u(word) + " bytes + " +
			              img(additional) + " bytes for metadata.");
		const int64_t payload = pos + 4;
		const int64_t end = payload + int64_t(word) + mt.block_checksum_length;
		if (end > len)
			raise(LZ4ADA_DATA_CORRUPTION, "Frame truncated inside a block.");
		if (descs) {
			lz4ada_block_desc d{};
			d.in_off = uint64_t(payload);
			d.in_len = word;
			d.flags = (stored ? LZ4ADA_BLOCK_STORED : 0u) |
			          (mt.block_checksum_length ? LZ4ADA_BLOCK_HAS_CKSUM : 0u);
			d.out_off = uint64_t(nb) * uint64_t(bmax);
			d.out_cap = uint32_t(bmax);
			d.cksum = mt.block_checksum_length ? load32(f + payload + word) : 0u;
			descs->push_back(d);
		}
		++nb;
		pos = end;
	}
	info.nblocks = nb;
	info.frame_len = pos;
}


// Independent blocks, batch by batch: block checksums + the bulk decoder
// over slots, then the batch's bytes (compacted if a block is short) to the
// sink, hashed on the way when the frame has a content checksum.
// BULK_FAIL_AT: block `fail` has a bad status or checksum; the blocks before
// it are committed (their lengths in `lens`), so the exact path can resume
// there instead of redoing the frame.
static BulkResult bulk_independent(const uint8_t* d_frame, const uint8_t* host_frame,
                                   const lz4ada_frame_info& info,
                                   const std::vector<lz4ada_block_desc>& descs, Sink& out,
                                   lz4ada_xxh32_state* h, uint64_t& total,
                                   std::vector<uint32_t>& lens, int64_t& fail)
{
	lens.clear();
	fail = -1;
	hipStream_t stream = nullptr;
	uint64_t budget = uint64_t(env_bytes("LZ4ADA_BATCH_BYTES", int64_t(4) << 30));
	uint32_t lo = 0;
	total = 0;
	while (lo < descs.size()) {
		const auto bt = batches_of(std::vector<lz4ada_block_desc>(descs.begin() + lo, descs.end()),
		                           info.block_max, 0, budget);
		const uint32_t hi = lo + bt[0].second;
		uint32_t nb = hi - lo;
		std::vector<lz4ada_block_desc> d(descs.begin() + lo, descs.begin() + hi);
		uint64_t slots = 0;
		for (auto& x : d) {
			x.out_cap = slot_cap(x, info.block_max);
			x.out_off = slots;
			slots += round256(x.out_cap);
		}
		DevBuf<lz4ada_block_desc> d_desc;
		DevBuf<lz4ada_block_status> d_st;
		uint8_t* const d_out = scratch(SC_OUT, size_t(slots));
		if (!d_out) {
			if (budget > (uint64_t(64) << 20) && nb > 1) {
				budget /= 2;  // retry this batch smaller
				continue;
			}
			return BULK_EXACT;
		}
		d_desc.reserve(nb);
		d_st.reserve(nb);
		vec_h2d(d_desc, d, nullptr);
		std::vector<lz4ada_block_status> st(nb);
		if (!(host_frame && few_large_blocks(d) &&
		      decode_lone_blocks(host_frame, d_frame, d, d_out, d_st.p, st,
		                         scratch_cache().b[SC_LONE], stream))) {
			HIP_OK(hipMemset(d_st.p, 0, nb * sizeof(lz4ada_block_status)));
			HIP_OK(launch_decode_checked(d_frame, uint64_t(info.frame_len), d_desc.p, nb, d_out,
			                             d_st.p, stream));
			vec_d2h(st, d_st, nullptr);
		}
		uint64_t bt_total = 0;
		bool contiguous = true;
		std::vector<uint64_t> dst_off(nb);
		uint32_t ok_n = nb;  // the blocks before the first failing one
		for (uint32_t i = 0; i < nb; ++i) {
			// the block checksum is checked before decoding (lz4ada.adb:672-676)
			if ((d[i].flags & LZ4ADA_BLOCK_HAS_CKSUM) && st[i].cksum != d[i].cksum) {
				ok_n = i;
				break;
			}
			if (st[i].code == DS_PRE_BLOCK_REF)
				return BULK_PRE_REF;  // B.Indep set, but the block reads earlier blocks (D2)
			if (st[i].code != DS_OK) {
				ok_n = i;
				break;
			}
			dst_off[i] = bt_total;
			if (bt_total != d[i].out_off)
				contiguous = false;
			bt_total += st[i].out_len;
		}
		const uint32_t nb_all = nb;
		nb = ok_n;
		const uint8_t* d_res = d_out;
		if (!contiguous) {
			DevBuf<uint64_t> d_off;
			uint8_t* const d_compact = scratch(SC_COMPACT, size_t(std::max<uint64_t>(bt_total, 1)));
			if (!d_compact)
				return BULK_EXACT;
			d_off.reserve(nb);
			HIP_OK(hipMemcpy(d_off.p, dst_off.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice));
			HIP_OK(launch_compact(d_out, d_desc.p, d_off.p, d_st.p, nb, d_compact, stream));
			HIP_OK(hipDeviceSynchronize());
			d_res = d_compact;
		}
		uint8_t* dst = out.room(int64_t(bt_total));
		if (h)  // D2H overlapped with the host XXH32 chain (content_xxh32_d2h)
			content_xxh32_d2h(*h, d_res, int64_t(bt_total), dst, stream);
		else if (bt_total)
			HIP_OK(hipMemcpy(dst, d_res, size_t(bt_total), hipMemcpyDeviceToHost));
		out.commit(int64_t(bt_total));
		total += bt_total;
		for (uint32_t i = 0; i < nb; ++i)
			lens.push_back(st[i].out_len);
		if (nb < nb_all) {
			fail = int64_t(lo) + nb;
			return BULK_FAIL_AT;
		}
		lo = hi;
	}
	return BULK_OK;
}


// Which paths the last lz4ada_decode_* call on this thread took
// (LZ4ADA_PATH_* bits; tests and diagnostics).
static thread_local int g_last_path = 0;

// for lz4ada_multi.cpp (lz4ada_internal.h)
void set_thread_error(const std::string& msg) { g_thread_error = msg; }
void set_last_path(int bits) { g_last_path = bits; }

// The stream state before block `fail`, the first one the bulk path could
// not take (its predecessors are committed): Output_Pos and
// Output_Pos_History as lz4ada.adb:678-690 and 785-787 leave them.
static void resume_state(const std::vector<uint32_t>& lens, Resume& rs)
{
	int64_t pos = 0, oph = 0;
	for (uint32_t n : lens) {
		if (pos >= HISTORY_SIZE)  // :678-680
			pos = 0;
		pos += n;
		if (pos >= HISTORY_SIZE)  // :688-690, 785-787
			oph = pos;
	}
	rs.output_pos = pos;
	rs.output_pos_history = oph;
}

// One frame from host memory (Single_Frame semantics): the bulk path when
// the frame indexes cleanly, else -- or when the bulk path finds anything
// the reference would report or treat differently -- the exact path, which
// raises the reference's exception in the reference's order.
static void decode_one_frame(const uint8_t* f, int64_t len, Sink& out, int64_t& consumed)
{
	lz4ada_frame_info info;
	std::vector<lz4ada_block_desc> descs;
	bool indexed = true;
	try {
		index_frame(f, len, info, &descs);
	} catch (const Error&) {
		indexed = false;  // the exact path raises the reference's error in order
	}
	if (indexed && info.format == LZ4ADA_FORMAT_SKIPPABLE && info.frame_len <= len) {
		consumed = info.frame_len;  // Skip (lz4ada.adb:420-433): nothing to decode
		return;
	}
	const int64_t base = out.len;
	// LZ4ADA_TRACE_FRAME=1: phase times (synchronised) to stderr
	static const bool trace = getenv("LZ4ADA_TRACE_FRAME") != nullptr;
	auto t0 = std::chrono::steady_clock::now();
	auto phase = [&](const char* name) {
		if (!trace)
			return;
		HIP_OK(hipDeviceSynchronize());
		const auto t1 = std::chrono::steady_clock::now();
		fprintf(stderr, "[frame] %-10s %8.3f ms\n", name,
		        std::chrono::duration<double, std::milli>(t1 - t0).count());
		t0 = t1;
	};
	if (indexed && info.frame_len <= len && info.format != LZ4ADA_FORMAT_SKIPPABLE &&
	    !getenv("LZ4ADA_EXACT_ONLY")) {
		device_check_or_raise();
		struct {
			uint8_t* p;
		} d_frame{ scratch(SC_FRAME, size_t(info.frame_len)) };
		phase("index");
		if (d_frame.p) {
			HIP_OK(hipMemcpy(d_frame.p, f, size_t(info.frame_len), hipMemcpyHostToDevice));
			phase("h2d");
			lz4ada_xxh32_state hs;
			lz4ada_xxh32_reset(&hs, 0);
			lz4ada_xxh32_state* h = info.content_checksum ? &hs : nullptr;
			uint64_t total = 0;
			// the reference decodes every frame as linked (B.Indep is never
			// read, lz4ada.adb:267-275); independent blocks are the fast case
			BulkResult r = BULK_PRE_REF;
			std::vector<uint32_t> lens;
			int64_t fail = -1;
			if (info.independent && !getenv("LZ4ADA_FORCE_LINKED"))
				r = bulk_independent(d_frame.p, f, info, descs, out, h, total, lens, fail);
			phase("bulk");
			const bool linked = r == BULK_PRE_REF;
			if (linked) {
				out.len = base;
				lz4ada_xxh32_reset(&hs, 0);
				LinkedSink ls;
				ls.dst = [&](int64_t n) -> uint8_t* {
					return scratch(SC_F, size_t(std::max<int64_t>(n, 1)));
				};
				ls.done = [&](const uint8_t* F, int64_t n) {
					uint8_t* dst = out.room(n);
					if (h)
						content_xxh32_d2h(*h, F, n, dst, nullptr);
					else if (n)
						HIP_OK(hipMemcpy(dst, F, size_t(n), hipMemcpyDeviceToHost));
					out.commit(n);
				};
				r = bulk_linked(d_frame.p, uint64_t(info.frame_len), info.block_max, descs, ls, total,
				                lens, fail, nullptr);
			}
			// blocks before `fail` that already decode past the declared content
			// size: the reference raises inside the first block that overruns
			// (lz4ada.adb:830-835), which a resume at `fail` would skip -- the
			// whole frame goes to the exact path instead
			const bool overrun = info.has_content_size && total > info.content_size;
			if (r == BULK_FAIL_AT && !overrun && !getenv("LZ4ADA_NO_RESUME")) {
				// the reference outputs blocks 0 .. fail-1 and then raises in
				// block `fail` (lz4ada.adb:672-676: each block is checked when it
				// is reached): the exact path resumes at that block, over the
				// Buffer the committed blocks leave, not at byte 0
				Resume rs;
				resume_state(lens, rs);
				rs.committed = total;
				rs.hash = hs;  // the blocks before `fail`, hashed on their way out
				rs.output = out.p + base;
				rs.lens = &lens;
				rs.at = int64_t(descs[size_t(fail)].in_off) - BLOCK_SIZE_BYTES;
				rs.checksum_first = info.block_checksum != 0;
				g_last_path |= LZ4ADA_PATH_EXACT |
				               (linked ? LZ4ADA_PATH_LINKED : LZ4ADA_PATH_INDEPENDENT);
				phase("state");
				try {
					exact_frame(f, len, out, consumed, &rs);
				} catch (...) {
					phase("resume");
					throw;
				}
				phase("resume");
				return;
			}
			if (trace)
				fprintf(stderr, "[frame] bulk result %d fail %lld total %llu hash %08x declared %08x\n", int(r),
				        (long long)fail, (unsigned long long)total, h ? (total ? hs.hash : 0x02cc5d05u) : 0u,
				        h ? info.content_checksum_declared : 0u);
			if (r == BULK_OK && (!info.has_content_size || total == info.content_size) &&
			    (!h || (total == 0 ? 0x02cc5d05u : hs.hash) == info.content_checksum_declared)) {
				consumed = info.frame_len;
				g_last_path |= linked ? LZ4ADA_PATH_LINKED : LZ4ADA_PATH_INDEPENDENT;
				return;
			}
			out.len = base;
		}
	}
	// A legacy frame has no end mark: it ends where the next magic starts
	// (what tool_unlz4ada's per-frame re-init achieves), so hand the exact
	// path only this frame's bytes.
	const int64_t flen = (indexed && info.format == LZ4ADA_FORMAT_LEGACY) ? info.frame_len : len;
	g_last_path |= LZ4ADA_PATH_EXACT;
	exact_frame(f, flen, out, consumed);
}
}  // namespace lz4ada

extern "C" {

int lz4ada_frame_index(const uint8_t* frame, int64_t len, lz4ada_frame_info* info,
                       lz4ada_block_desc* descs, int64_t desc_cap)
{
	return guarded(nullptr, [&] {
		std::vector<lz4ada_block_desc> v;
		index_frame(frame, len, *info, descs ? &v : nullptr);
		if (descs) {
			if (int64_t(v.size()) > desc_cap)
				raise(LZ4ADA_CONSTRAINT_ERROR, "descriptor capacity exceeded");
			memcpy(descs, v.data(), v.size() * sizeof(lz4ada_block_desc));
		}
	});
}

int lz4ada_launch_decode(const void* d_frame, uint64_t frame_len, const lz4ada_block_desc* d_descs,
                         int64_t nblocks, void* d_out, lz4ada_block_status* d_status, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_decode_blocks(static_cast<const uint8_t*>(d_frame), frame_len, d_descs,
		                            uint32_t(nblocks), static_cast<uint8_t*>(d_out), d_status,
		                            static_cast<hipStream_t>(stream)));
	});
}

int lz4ada_launch_decode_variant(const void* d_frame, uint64_t frame_len,
                                 const lz4ada_block_desc* d_descs, int64_t nblocks, void* d_out,
                                 lz4ada_block_status* d_status, int variant, void* stream)
{
	return guarded(nullptr, [&] {
		if (variant < 0 || variant > 10)
			raise(LZ4ADA_ASSERTION_ERROR, "unknown decoder variant");
		HIP_OK(launch_decode_variant(static_cast<const uint8_t*>(d_frame), frame_len, d_descs,
		                             uint32_t(nblocks), static_cast<uint8_t*>(d_out), d_status,
		                             variant, static_cast<hipStream_t>(stream)));
	});
}


int64_t lz4ada_lone_scratch_bytes(int64_t n, int64_t cap) { return lone_scratch_bytes(n, cap); }

int lz4ada_launch_decode_lone(const void* d_blk, int64_t n, void* d_out, int64_t cap,
                              lz4ada_block_status* d_status, void* d_scratch,
                              int64_t scratch_bytes, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_decode_lone(static_cast<const uint8_t*>(d_blk), n, static_cast<uint8_t*>(d_out),
		                          cap, d_status, d_scratch, scratch_bytes,
		                          static_cast<hipStream_t>(stream)));
	});
}

int lz4ada_launch_block_checksums(const void* d_frame, const lz4ada_block_desc* d_descs,
                                  int64_t nblocks, lz4ada_block_status* d_status, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_block_checksums(static_cast<const uint8_t*>(d_frame), d_descs,
		                              uint32_t(nblocks), d_status,
		                              static_cast<hipStream_t>(stream)));
	});
}

int lz4ada_decode_blocks_device(const void* d_frame, uint64_t frame_len,
                                const lz4ada_block_desc* d_descs, int64_t nblocks, void* d_out,
                                lz4ada_block_status* d_status, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_decode_checked(static_cast<const uint8_t*>(d_frame), frame_len, d_descs,
		                             uint32_t(nblocks), static_cast<uint8_t*>(d_out), d_status,
		                             static_cast<hipStream_t>(stream)));
	});
}

int lz4ada_output_checksums_device(const void* d_out, const lz4ada_block_desc* d_descs,
                                   const lz4ada_block_status* d_status, int64_t nblocks,
                                   uint32_t* d_hash, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_output_checksums(static_cast<const uint8_t*>(d_out), d_descs,
		                               uint32_t(nblocks), d_status, d_hash,
		                               static_cast<hipStream_t>(stream)));
	});
}

// A stream's next frame starts with fewer than 7 bytes left: what the
// reference CLI raises there (tool_unlz4ada/unlz4ada.adb:65-76), before
// Init_With_Header's precondition (lz4ada.ads:243) would.
static void partial_frame_check(int64_t left)
{
	if (left < 7)
		raise(LZ4ADA_CONSTRAINT_ERROR, "Partial frame detected. Unable to process all data");
}

int lz4ada_decode_frame(const uint8_t* frame, int64_t len, uint8_t* out, int64_t out_cap,
                        int64_t* out_len, int64_t* frame_consumed)
{
	*out_len = 0;
	*frame_consumed = 0;
	g_last_path = 0;
	return guarded(nullptr, [&] {
		Sink s;
		s.p = out;
		s.cap = out_cap;
		decode_one_frame(frame, len, s, *frame_consumed);
		*out_len = s.len;
	});
}

int lz4ada_decode_stream(const uint8_t* input, int64_t len, uint8_t* out, int64_t out_cap,
                         int64_t* out_len)
{
	*out_len = 0;
	g_last_path = 0;
	return guarded(nullptr, [&] {
		Sink s;
		s.p = out;
		s.cap = out_cap;
		int64_t pos = 0;
		while (pos < len) {
			int64_t c = 0;
			partial_frame_check(len - pos);
			decode_one_frame(input + pos, len - pos, s, c);
			*out_len = s.len;
			if (c <= 0)
				raise(LZ4ADA_CONSTRAINT_ERROR, "decoder made no progress");
			pos += c;
		}
	});
}

// The same into a buffer the library allocates and grows (no bound needed
// up front); release it with lz4ada_buffer_free.  On failure *out is NULL.
static int decode_alloc(const uint8_t* input, int64_t len, bool stream, uint8_t** out,
                        int64_t* out_len, int64_t* consumed, bool keep_partial = false)
{
	*out = nullptr;
	*out_len = 0;
	if (consumed)
		*consumed = 0;
	Sink s;
	s.growable = true;
	g_last_path = 0;
	const int st = guarded(nullptr, [&] {
		int64_t pos = 0;
		do {
			int64_t c = 0;
			if (stream)
				partial_frame_check(len - pos);
			decode_one_frame(input + pos, len - pos, s, c);
			if (c <= 0)
				raise(LZ4ADA_CONSTRAINT_ERROR, "decoder made no progress");
			pos += c;
		} while (stream && pos < len);
		if (consumed)
			*consumed = pos;
	});
	if (st != LZ4ADA_OK) {
		if (keep_partial) {  // what the reference had output before it raised
			*out = s.p ? s.p : static_cast<uint8_t*>(malloc(1));
			*out_len = s.len;
			return st;
		}
		free(s.p);
		return st;
	}
	*out = s.p ? s.p : static_cast<uint8_t*>(malloc(1));
	*out_len = s.len;
	return LZ4ADA_OK;
}

int lz4ada_decode_frame_alloc(const uint8_t* frame, int64_t len, uint8_t** out, int64_t* out_len,
                              int64_t* frame_consumed)
{
	return decode_alloc(frame, len, false, out, out_len, frame_consumed);
}

int lz4ada_decode_stream_alloc(const uint8_t* input, int64_t len, uint8_t** out, int64_t* out_len)
{
	return decode_alloc(input, len, true, out, out_len, nullptr);
}

int lz4ada_decode_frame_partial(const uint8_t* frame, int64_t len, uint8_t** out, int64_t* out_len,
                                int64_t* frame_consumed)
{
	return decode_alloc(frame, len, false, out, out_len, frame_consumed, true);
}

void lz4ada_buffer_free(uint8_t* p) { free(p); }

int lz4ada_decode_linked_device(const void* d_frame, uint64_t frame_len,
                                const lz4ada_block_desc* descs, int64_t nblocks, int64_t block_max,
                                void* d_out, int64_t out_cap, int64_t* out_len, void* stream)
{
	*out_len = 0;
	return guarded(nullptr, [&] {
		device_check_or_raise();
		std::vector<lz4ada_block_desc> v(descs, descs + nblocks);
		hipStream_t s = static_cast<hipStream_t>(stream);
		int64_t pos = 0;
		LinkedSink ls;
		ls.dst = [&](int64_t n) -> uint8_t* {
			return pos + n <= out_cap ? static_cast<uint8_t*>(d_out) + pos : nullptr;
		};
		ls.done = [&](const uint8_t*, int64_t n) { pos += n; };
		uint64_t total = 0;
		std::vector<uint32_t> lens;
		int64_t fail = -1;
		if (bulk_linked(static_cast<const uint8_t*>(d_frame), frame_len, block_max, v, ls, total,
		                lens, fail, s) != BULK_OK)
			raise(LZ4ADA_EXACT_PATH,
			      "the frame needs the reference-exact path (lz4ada_decode_frame): a block "
			      "error or checksum mismatch, quirk D1, or too little output room");
		HIP_OK(hipStreamSynchronize(s));
		*out_len = pos;
	});
}

int lz4ada_last_path(void) { return g_last_path; }

const char* lz4ada_bulk_decoder_kernel(int64_t nblocks)
{
	return idx_fused_kernel_name(uint32_t(std::max<int64_t>(nblocks, 0)));
}

void lz4ada_release_device_cache(void)
{
	scratch_release();
	dev_pool().release_all();
	pin_pool().release_all();
	// the facade's pooled streams and events too
	std::vector<StreamSet> sets;
	{
		std::lock_guard<std::mutex> l(g_stream_mu);
		sets.swap(stream_pool());
	}
	int cur = 0;
	(void)hipGetDevice(&cur);
	for (auto& x : sets) {
		(void)hipSetDevice(x.device);
		(void)hipStreamDestroy(x.side);
		(void)hipEventDestroy(x.ev);
		(void)hipStreamDestroy(x.stream);
	}
	(void)hipSetDevice(cur);
}

int64_t lz4ada_decoded_bound(const uint8_t* input, int64_t len)
{
	int64_t pos = 0, bound = 0;
	while (pos < len) {
		lz4ada_frame_info info;
		if (lz4ada_frame_index(input + pos, len - pos, &info, nullptr, 0) != LZ4ADA_OK)
			return -1;
		if (info.frame_len <= 0)
			return -1;
		bound += info.nblocks * info.block_max;
		pos += info.frame_len;
	}
	return bound;
}

}  // extern "C"

