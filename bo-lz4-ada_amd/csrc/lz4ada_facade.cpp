// lz4ada_facade.cpp -- the streaming facade of the MI355X LZ4Ada
// decompressor: the Update state machine of lib/lz4ada.adb
// (LZ4Ada.Init / Init_With_Header / Init_For_Block / Update /
// Is_End_Of_Frame, lz4ada.ads:189-321; lz4ada.adb:383-714) over a device
// mirror of the caller's Buffer, every block decoded on the GPU (read-ahead
// bulk batches, the lone-block decoder, the reference-exact serial kernel),
// and the XXHash32 C-ABI (lz4ada.ads:335-343).
#include "lz4ada_host_common.h"

using namespace lz4ada;

// ----------------------------------------------------------- Decompressor

struct lz4ada_decompressor {
	Meta m;
	bool is_at_end_mark = false;
	std::vector<uint8_t> input_buffer;  // Input_Buffer(0 .. In_Last)
	int64_t output_pos = 0;
	int64_t output_pos_history = 0;
	int64_t input_length = -1;
	std::string err;
	int64_t exact_blocks = 0;  // blocks decoded by the reference-exact serial kernel (diagnostics)

	// device side (lazily created at the first block)
	bool dev_ready = false;
	// check the next block's checksum before launching the speculative
	// decode (the block a bulk path stopped at: a decode of a corrupted
	// payload may be long, and would have to finish before the raise)
	bool checksum_first = false;
	int device = -1;
	hipStream_t stream = nullptr;
	DevBuf<uint8_t> d_buf;  // mirror of the caller's Buffer (history lives here)
	int64_t d_buf_len = 0;
	DevBuf<uint8_t> d_blk;
	lz4ada_xxh32_state hash_all{};  // Hash_All_Data, over the bytes the GPU decoded
	// A large block's content hash runs on a helper thread while the caller
	// feeds the next block, over the pinned staging copy of its output (our
	// memory, so the caller may reuse its Buffer); every reader of hash_all
	// joins it first.  The staging ping-pongs: a block handed to the hasher
	// leaves in stage_hashed, so the next block's copy never waits for it
	// (the hasher runs one job at a time, and submit() joins the previous one).
	Worker hasher;
	void hash_wait() { hasher.wait(); }
	PinBuf stage;  // a block's output on its way to the caller's Buffer
	PinBuf stage_hashed;  // the staging the hasher may be reading
	PinBuf stage_st;  // its status (the lone-block decoder writes it there itself)
	PinBuf pin_blk;   // a lone block's compressed bytes, read by its first kernel
	std::vector<uint8_t> blk_tmp;  // a block assembled from cached + new input
	DevBuf<lz4ada_xxh32_state> d_tmp_hash;
	DevBuf<SerialState> d_serial;
	DevBuf<lz4ada_block_desc> d_desc;  // one-block fast path
	DevBuf<lz4ada_block_status> d_bst;
	DevBuf<uint8_t> d_scr;  // its output, until the block checksum has passed
	DevBuf<uint8_t> d_lone;  // the lone-block decoder's tables and words
	bool lone_hdr_zeroed = false;  // its header (the fused chain step's count) is zero
	hipStream_t side = nullptr;  // the block checksum, beside the fast decode
	hipEvent_t ev_in = nullptr;

	// Read-ahead: when one Update call hands over several
	// complete blocks, they are decoded together by the bulk decoder and
	// then served one per call, as the reference returns them.
	struct Ahead {
		std::vector<uint8_t> input;  // the batch's compressed bytes (identity check)
		std::vector<lz4ada_block_desc> descs;
		std::vector<lz4ada_block_status> st;
		DevBuf<uint8_t> d_in, d_out, d_lone;
		DevBuf<lz4ada_block_desc> d_desc;
		DevBuf<lz4ada_block_status> d_st;
		uint64_t slot = 0;
		size_t next = 0;  // next block to serve
		void clear()
		{
			descs.clear();
			st.clear();
			next = 0;
		}
	} ahead;
	int64_t linked_cap = int64_t(512) << 20;  // input bytes of a linked read-ahead batch

	lz4ada_decompressor() { lz4ada_xxh32_reset(&hash_all, 0); }
	~lz4ada_decompressor()
	{
		hash_wait();
		if (!stream)
			return;
		// idle streams go back to the pool for the next context
		const bool idle = hipStreamSynchronize(side) == hipSuccess && hipStreamSynchronize(stream) == hipSuccess;
		if (idle) {
			std::lock_guard<std::mutex> l(g_stream_mu);
			stream_pool().push_back(StreamSet{ device, stream, side, ev_in });
		} else {
			(void)hipStreamDestroy(side);
			(void)hipEventDestroy(ev_in);
			(void)hipStreamDestroy(stream);
		}
	}

	void ensure_device()
	{
		if (dev_ready)
			return;
		device_check_or_raise();
		HIP_OK(hipGetDevice(&device));
		{
			std::lock_guard<std::mutex> l(g_stream_mu);
			auto& pool = stream_pool();
			for (size_t i = 0; i < pool.size(); ++i)
				if (pool[i].device == device) {
					stream = pool[i].stream;
					side = pool[i].side;
					ev_in = pool[i].ev;
					pool[i] = pool.back();
					pool.pop_back();
					break;
				}
		}
		if (!stream) {
			HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
			HIP_OK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
			HIP_OK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
		}
		d_tmp_hash.reserve(1);
		d_serial.reserve(1);
		d_desc.reserve(1);
		d_bst.reserve(1);
		dev_ready = true;
	}

	void reset_content_hash()  // XXHash32.Reset(0)
	{
		hash_wait();
		lz4ada_xxh32_reset(&hash_all, 0);
	}

	// ---------------------------------------------------- Update pieces
	void reset_outer()  // lz4ada.adb:451-461
	{
		ahead.clear();
		is_at_end_mark = false;
		input_length = -1;
		output_pos = 0;
		output_pos_history = 0;
		reset_content_hash();
	}

	int64_t reset_for_next_frame(const uint8_t* in, int64_t len)  // :435-449
	{
		if (m.memory_reservation == LZ4ADA_SINGLE_FRAME)
			raise(LZ4ADA_DATA_CORRUPTION,
			      "Requested Single_Frame operation but data was provided after End of Frame "
			      "was detected");
		m.status_eof = LZ4ADA_EOF_NO;
		m.header_parsing = NEED_MAGIC;
		m.size_remaining = 4;
		reset_outer();
		return header_bytes(m, input_buffer.data(), in, len);
	}

	int64_t skip(const uint8_t* in, int64_t len)  // :420-433
	{
		const uint64_t remain = m.size_remaining;
		const uint64_t cons = std::min<uint64_t>(uint64_t(len), remain);
		if (m.status_eof == LZ4ADA_EOF_YES && cons == 0)
			return reset_for_next_frame(in, len);
		m.size_remaining = remain - cons;
		m.status_eof = m.size_remaining == 0 ? LZ4ADA_EOF_YES : LZ4ADA_EOF_NO;
		return int64_t(cons);
	}

	void frame_has_ended()  // :465-477
	{
		m.status_eof = LZ4ADA_EOF_YES;
		m.input_buffer_filled = 0;
		if (m.has_content_size && m.size_remaining != 0)
			raise(LZ4ADA_DATA_CORRUPTION,
			      "Frame has ended, but according to content size, there should be " +
			              img_u(m.size_remaining) + " bytes left to output.");
	}

	uint32_t content_hash_final()
	{
		hash_wait();
		return host_xxh32_final(hash_all);
	}

	void check_end_mark(const uint8_t* in, int64_t len, int64_t& consumed)  // :463-523
	{
		const int64_t provided = len - consumed;
		const int64_t required = m.content_checksum_length - m.input_buffer_filled;
		if (m.content_checksum_length == 0 || m.status_eof == LZ4ADA_EOF_YES || required <= 0) {
			if (m.status_eof == LZ4ADA_EOF_YES) {
				if (consumed != 0)
					raise(LZ4ADA_ASSERTION_ERROR, "lz4ada.adb:486");
				consumed = reset_for_next_frame(in, len);
			} else {
				frame_has_ended();
			}
		} else if (provided >= required) {
			uint8_t tmp[8];
			memcpy(tmp, input_buffer.data(), size_t(m.input_buffer_filled));
			memcpy(tmp + m.input_buffer_filled, in + consumed, size_t(required));
			const uint32_t declared = load32(tmp);
			const uint32_t computed = content_hash_final();
			consumed += required;
			if (declared != computed)
				raise(LZ4ADA_CHECKSUM_ERROR, "Computed content checksum 0x" + hex32(computed) +
				                                     " does not match declared content checksum 0x" +
				                                     hex32(declared) + ".");
			frame_has_ended();
		} else {
			memcpy(input_buffer.data() + m.input_buffer_filled, in + consumed, size_t(provided));
			m.input_buffer_filled += provided;
			consumed += provided;
		}
	}

	int64_t try_detect_input_length(const uint8_t* in, int64_t len)  // :525-585
	{
		const int64_t additional = BLOCK_SIZE_BYTES + m.block_checksum_length;
		const int64_t n = std::min<int64_t>(BLOCK_SIZE_BYTES - m.input_buffer_filled, len);
		memcpy(input_buffer.data() + m.input_buffer_filled, in, size_t(n));
		m.input_buffer_filled += n;
		if (m.input_buffer_filled == BLOCK_SIZE_BYTES) {
			uint32_t word = load32(input_buffer.data());
			if (m.is_format == F_MODERN && word == 0) {
				is_at_end_mark = true;
				m.input_buffer_filled = 0;
			} else if (m.is_format == F_LEGACY && is_any_magic(word)) {
				if (m.memory_reservation == LZ4ADA_SINGLE_FRAME)
					raise(LZ4ADA_DATA_CORRUPTION,
					      "Requested Single_Frame operation but data provided what looks "
					      "like the beginning of another frame.");
				reset_outer();
				header_magic(m, word);
			} else {
				if (m.is_format == F_MODERN) {
					m.is_compressed = (word & 0x80000000u) == 0;
					word &= 0x7ffffffu;  // 27-bit mask, quirk Q2
				}
				input_length = int64_t(word);
				if (input_length + additional > int64_t(input_buffer.size())) {
					input_length = -1;
					raise(LZ4ADA_DATA_CORRUPTION,
					      "Declared maximum data length exceeded. Buffer has " +
					              img(int64_t(input_buffer.size())) +
					              " bytes, current block requires " + img_u(word) +
					              " bytes + " + img(additional) + " bytes for metadata.");
				}
			}
		}
		return n;
	}

	void grow_mirror(int64_t buflen)  // the Buffer mirror, keeping history
	{
		DevBuf<uint8_t> nb;
		nb.reserve(size_t(buflen));
		HIP_OK(hipMemsetAsync(nb.p, 0, size_t(buflen), stream));
		if (d_buf_len)
			HIP_OK(hipMemcpyAsync(nb.p, d_buf.p, size_t(d_buf_len), hipMemcpyDeviceToDevice,
			                      stream));
		HIP_OK(hipStreamSynchronize(stream));
		std::swap(nb.p, d_buf.p);
		std::swap(nb.n, d_buf.n);
		std::swap(nb.bytes, d_buf.bytes);
		d_buf_len = buflen;
	}

	// Decode_Full_Block_With_Trailer (lz4ada.adb:661-714) on the GPU.
	void decode_full_block(const uint8_t* blk, int64_t blen, uint8_t* buf, int64_t buflen,
	                       int64_t& first, int64_t& last)
	{
		ensure_device();
		const int bcl = m.block_checksum_length;
		const int64_t raw_len = blen - bcl;
		if (buflen > d_buf_len)
			grow_mirror(buflen);
		static const bool trace = getenv("LZ4ADA_TRACE_FACADE") != nullptr;
		auto t0 = std::chrono::steady_clock::now();
		auto phase = [&](const char* name) {
			if (!trace)
				return;
			const auto t1 = std::chrono::steady_clock::now();
			fprintf(stderr, "[facade] %-8s %8.3f ms\n", name,
			        std::chrono::duration<double, std::milli>(t1 - t0).count());
			t0 = t1;
		};
		d_blk.reserve(size_t(std::max<int64_t>(blen, 1)));
		// Check_Checksum comes before decoding (:672-676, quirk Q8).  The
		// payload is host memory here: its XXH32 runs on this thread (one
		// serial chain, ~10x the GPU chain's rate) while the GPU decodes
		// into a scratch slot; the mirror takes the output only once the
		// checksum has passed.  A block known to fail (the bulk path stopped
		// at it) is checked before anything is launched.
		auto check = [&] { return block_checksum(blk, blen); };
		if (checksum_first && bcl > 0) {
			checksum_first = false;
			const auto c = check();
			if (!c.first)
				raise(LZ4ADA_CHECKSUM_ERROR, c.second);
		}
		// a lone block goes over without a DMA copy: its first kernel reads the
		// pinned bytes and leaves the device copy the other paths read
		LonePlan lp;
		const bool lone = lone_plan(blen, buflen, lp);
		if (blen > 0 && lone) {
			pin_blk.reserve(size_t(blen));
			memcpy(pin_blk.p, blk, size_t(blen));
		} else if (blen > 0) {
			HIP_OK(hipMemcpyAsync(d_blk.p, blk, size_t(blen), hipMemcpyHostToDevice, stream));
		}
		phase("h2d");
		const LoneResult lr = lone ? lone_block(lp, blk, blen, buf, first, last) : LONE_NOT_TAKEN;
		phase("lone");
		if (lr == LONE_DONE)
			return;
		const int64_t fast_start = lr == LONE_DECLINED ? -1 : launch_fast_block(raw_len, blen, buflen);
		if (bcl > 0 && lr != LONE_DECLINED) {
			const auto c = check();
			phase("cksum");
			if (!c.first) {
				HIP_OK(hipStreamSynchronize(stream));  // the scratch decode, discarded
				raise(LZ4ADA_CHECKSUM_ERROR, c.second);
			}
		}
		if (fast_start >= 0 && finish_fast_block(fast_start, first, last)) {
			phase("decode");
			deliver(buf, first, last);
			phase("deliver");
			return;
		}
		SerialState s{};
		s.output_pos = output_pos;
		s.output_pos_history = output_pos_history;
		s.size_remaining = m.size_remaining;
		s.has_content_size = m.has_content_size ? 1 : 0;
		HIP_OK(hipMemcpyAsync(d_serial.p, &s, sizeof s, hipMemcpyHostToDevice, stream));
		++exact_blocks;
		HIP_OK(launch_serial_block(d_buf.p, buflen, d_blk.p, raw_len,
		                           m.is_compressed ? raw_len : blen, m.is_compressed ? 1 : 0,
		                           d_serial.p, stream));
		HIP_OK(hipMemcpyAsync(&s, d_serial.p, sizeof s, hipMemcpyDeviceToHost, stream));
		HIP_OK(hipStreamSynchronize(stream));
		// state changes before a raise persist, as with the Ada record
		output_pos = s.output_pos;
		output_pos_history = s.output_pos_history;
		if (m.has_content_size)
			m.size_remaining = s.size_remaining;
		if (s.code != DS_OK)
			raise_device_status(s);
		first = s.first;
		last = s.last;
		deliver(buf, first, last);
	}

	// The block's output, in the Buffer mirror at [first, last], to the
	// caller's Buffer, and into the content checksum (Update_Checksum,
	// :709-714) on the way.
	void deliver(uint8_t* buf, int64_t first, int64_t last)
	{
		const int64_t nout = last - first + 1;
		if (nout <= 0)
			return;
		static const bool trace = getenv("LZ4ADA_TRACE_FACADE") != nullptr;
		const auto t0 = std::chrono::steady_clock::now();
		stage.reserve(size_t(nout));
		HIP_OK(hipMemcpyAsync(stage.p, d_buf.p + first, size_t(nout), hipMemcpyDeviceToHost, stream));
		HIP_OK(hipStreamSynchronize(stream));
		const auto t1 = std::chrono::steady_clock::now();
		to_caller(buf + first, nout);
		if (trace)
			fprintf(stderr, "[facade]   d2h %.3f ms, content hash %.3f ms\n",
			        std::chrono::duration<double, std::milli>(t1 - t0).count(),
			        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1)
			                .count());
	}

	// The staged output (stage.p, nout bytes) to the caller's Buffer and into
	// the content checksum -- on the helper thread for a large block.
	void to_caller(uint8_t* dst, int64_t nout)
	{
		memcpy(dst, stage.p, size_t(nout));
		if (m.content_checksum_length == 0)
			return;
		const uint8_t* p = stage.p;
		if (nout >= (int64_t(64) << 10)) {
			hasher.submit([this, p, nout] { host_xxh32_update(hash_all, p, size_t(nout)); });
			stage.swap(stage_hashed);
		} else {
			hash_wait();  // the previous block's share first
			host_xxh32_update(hash_all, p, size_t(nout));
		}
	}

	// A lone block is latency-bound: the lone-block decoder (every step
	// parallel over the block's bytes, lz4ada_lone.hip) decodes a 4 MiB mixed
	// block in ~0.2 ms against ~21 ms for k_decode_pc's one workgroup
	// (tools/lone_time.py).  Below LONE_MIN compressed bytes k_decode_pc's
	// single launch wins (16 KiB mixed blocks, 8 KB compressed: lone 0.051 ms,
	// pc 0.090; pc's time grows with the block, lone's ~0.045 ms floor is its
	// five launches).  LZ4ADA_FACADE_DECODER=pc / lone forces one.
	static constexpr int64_t LONE_MIN = 6 << 10;
	static int facade_variant()
	{
		const char* e = getenv("LZ4ADA_FACADE_DECODER");
		if (e && !strcmp(e, "pc"))
			return DEC_PC;
		if (e && !strcmp(e, "lone"))
			return -2;  // the lone-block decoder at every size
		return -1;  // lone (large blocks), else k_decode_pc
	}

	// Decompress_Full_Block through the bulk decoder for one block, into a
	// scratch slot; a clean result moves to the Buffer mirror at the
	// position the reference would use.  Any status but OK -- including a
	// reference before the block start, which only the exact path resolves
	// (history scheme, D1) -- or a content-size overrun leaves the block to
	// k_serial_block, which redoes it from the same state on an untouched
	// mirror.  launch_fast_block enqueues the decode and returns the block's
	// Output_Pos (-1: not tried); finish_fast_block waits for it.
	// The output room a decoder slot needs for one block: what the Buffer
	// leaves, but no more than the frame's block maximum (BD for modern
	// frames, 8 MiB for legacy ones, lz4ada.adb:65-77, 225-239) or 255 bytes
	// per payload byte.  A block that would decode to more is the exact
	// path's (the reference bounds it by the Buffer alone, D5) -- so a large
	// caller Buffer never sizes the device scratch.
	int64_t block_room(int64_t buflen_left, int64_t raw_len, bool compressed) const
	{
		int64_t cap = std::min<int64_t>(buflen_left, INT32_MAX);
		if (compressed)
			cap = std::min<int64_t>(cap, 255 * std::max<int64_t>(raw_len, 1) + 16);
		else
			cap = std::min<int64_t>(cap, raw_len);
		if (m.is_format == F_MODERN)
			cap = std::min<int64_t>(cap, int64_t(1) << (8 + 2 * ((m.bd & 0x70u) >> 4)));
		else if (m.is_format == F_LEGACY)
			cap = std::min<int64_t>(cap, int64_t(8) << 20);
		return cap;
	}

	// The history a block of a linked frame may read (lz4ada.adb:678-690,
	// 862-883) when it starts at Buffer position `start`: the current round's
	// bytes Buffer(0 .. start-1) (n1), and before them the previous round's
	// tail Buffer(OPH - n0 .. OPH - 1) -- up to 65535 bytes in all, the
	// largest offset.  Before the first round ends there is none beyond n1.
	void history_of(int64_t start, int64_t& n0, int64_t& n1) const
	{
		n1 = start;
		n0 = std::min<int64_t>(65535, start + output_pos_history) - n1;
	}
	// Quirk D1 can only strike right after a round that ended within the
	// reference's 8-byte wild copy of 64 KiB (lz4ada.adb:811-817, 862-879).
	bool d1_window() const
	{
		return output_pos_history >= HISTORY_SIZE && output_pos_history <= HISTORY_SIZE + 6;
	}

	std::pair<bool, std::string> block_checksum(const uint8_t* blk, int64_t blen) const
	{
		const int bcl = m.block_checksum_length;
		lz4ada_xxh32_state h;
		lz4ada_xxh32_reset(&h, 0);
		host_xxh32_update(h, blk, size_t(blen - bcl));
		const uint32_t got = host_xxh32_final(h);
		const uint32_t expect = load32(blk + blen - bcl);
		return std::make_pair(got == expect, "Declared checksum is 0x" + hex32(expect) +
		                                             ", but computed one is 0x" + hex32(got) + ".");
	}

	// A compressed block for the lone-block decoder: every block of a linked
	// frame (the reference's history as readable words in front of its
	// output), an independent frame's from LONE_MIN compressed bytes.  Its
	// two halves run around the host checksum (Check_Checksum before any
	// output, :672-676), and the emit writes straight into the mirror at the
	// reference's Output_Pos -- only when the block decoded cleanly, so a
	// decline (a reference past the history, D1 risk, a content-size or
	// slot overrun, anything the reference would reject) leaves the mirror
	// untouched for the exact path.  The status and the output come back in
	// one round trip through pinned staging.
	enum LoneResult { LONE_NOT_TAKEN, LONE_DONE, LONE_DECLINED };
	struct LonePlan {
		int64_t raw_len, start, cap, n0, n1;
		bool linked;
	};
	// Whether the lone-block decoder takes this block, and where its output goes.
	bool lone_plan(int64_t blen, int64_t buflen, LonePlan& p)
	{
		const int bcl = m.block_checksum_length;
		const int64_t raw_len = blen - bcl;
		if (!m.is_compressed || raw_len <= 0 || raw_len > LONE_MAX_IN || getenv("LZ4ADA_FACADE_EXACT"))
			return false;
		const bool linked = m.is_format == F_MODERN && !(m.flg & 0x20u);
		const int fv = facade_variant();
		if (!linked && !(fv < 0 && (raw_len >= LONE_MIN || fv == -2)))
			return false;
		const int64_t start = output_pos >= HISTORY_SIZE ? 0 : output_pos;  // :678-680
		if (buflen - start <= 0)
			return false;
		int64_t cap = block_room(buflen - start, raw_len, true);
		if (m.has_content_size)  // more output: the exact path raises mid-block, as the reference does
			cap = int64_t(std::min<uint64_t>(uint64_t(cap), m.size_remaining));
		if (cap <= 0 || cap > (int64_t(1) << 30))
			return false;
		p.raw_len = raw_len;
		p.start = start;
		p.cap = cap;
		p.linked = linked;
		p.n0 = p.n1 = 0;
		if (linked)
			history_of(start, p.n0, p.n1);
		return true;
	}

	// The block's pinned bytes (pin_blk) through the lone-block decoder: its
	// first kernel copies them to d_blk (for the exact path, should it
	// decline), its last writes the output to the mirror and to the pinned
	// staging, and the status comes back in pinned memory too -- one stream
	// synchronisation, no DMA copy (a DMA transfer costs ~10 us of latency
	// each way for a 64 KiB block).
	LoneResult lone_block(const LonePlan& lp, const uint8_t* blk, int64_t blen, uint8_t* buf, int64_t& first,
	                      int64_t& last)
	{
		const int bcl = m.block_checksum_length;
		const int64_t raw_len = lp.raw_len, start = lp.start, cap = lp.cap, n0 = lp.n0, n1 = lp.n1;
		const bool linked = lp.linked;
		static const bool trace = getenv("LZ4ADA_TRACE_FACADE") != nullptr;
		auto t0 = std::chrono::steady_clock::now();
		auto lap = [&](const char* name) {
			if (!trace)
				return;
			const auto t1 = std::chrono::steady_clock::now();
			fprintf(stderr, "[facade]   lone %-7s %8.3f ms\n", name,
			        std::chrono::duration<double, std::milli>(t1 - t0).count());
			t0 = t1;
		};
		const int64_t sb = lone_scratch_bytes(raw_len, cap);
		const size_t had = d_lone.n;
		d_lone.reserve(size_t(sb));
		if (d_lone.n != had || !lone_hdr_zeroed) {  // a new scratch: its header zeroed once
			HIP_OK(lone_scratch_init(d_lone.p, stream));
			lone_hdr_zeroed = true;
		}
		stage.reserve(size_t(cap));
		stage_st.reserve(sizeof(lz4ada_block_status));
		lz4ada_block_status* hst = reinterpret_cast<lz4ada_block_status*>(stage_st.p);
		HIP_OK(launch_decode_lone_parse(pin_blk.p, raw_len, cap, hst, d_lone.p, sb, stream,
		                                linked ? d_buf.p + output_pos_history - n0 : nullptr, int32_t(n0),
		                                linked ? d_buf.p : nullptr, int32_t(n1),
		                                linked && d1_window() ? int(output_pos_history) : 0, d_blk.p, blen,
		                                true));
		lap("parse");
		if (bcl > 0) {
			const auto c = block_checksum(blk, blen);
			if (!c.first) {
				HIP_OK(hipStreamSynchronize(stream));
				raise(LZ4ADA_CHECKSUM_ERROR, c.second);
			}
		}
		lap("cksum");
		HIP_OK(launch_decode_lone_emit(raw_len, d_buf.p + start, cap, hst, d_lone.p, stream,
		                               int32_t(n0 + n1), stage.p));
		lap("enqueue");
		HIP_OK(hipStreamSynchronize(stream));
		lap("wait");
		lz4ada_block_status st;
		memcpy(&st, hst, sizeof st);
		if (st.code != DS_OK)
			return LONE_DECLINED;
		const int64_t nout = int64_t(st.out_len);
		if (m.has_content_size)
			m.size_remaining -= uint64_t(nout);
		output_pos = start + nout;
		if (output_pos >= HISTORY_SIZE)  // :785-787
			output_pos_history = output_pos;
		first = start;
		last = start + nout - 1;
		if (nout > 0)
			to_caller(buf + first, nout);
		lap("deliver");
		return LONE_DONE;
	}

	int64_t launch_fast_block(int64_t raw_len, int64_t blen, int64_t buflen)
	{
		const bool linked = m.is_format == F_MODERN && !(m.flg & 0x20u);
		if (getenv("LZ4ADA_FACADE_EXACT"))
			return -1;
		const int64_t start = output_pos >= HISTORY_SIZE ? 0 : output_pos;  // :678-680
		if (buflen - start <= 0 || raw_len > INT32_MAX)
			return -1;
		const int64_t cap = std::max<int64_t>(block_room(buflen - start, raw_len, m.is_compressed), 1);
		if (linked && m.is_compressed)
			return -1;  // lone_block declined it: the exact path
		d_scr.reserve(size_t(cap));
		lz4ada_block_desc d{};
		d.in_off = 0;
		d.in_len = uint32_t(raw_len);
		d.flags = m.is_compressed ? 0u : LZ4ADA_BLOCK_STORED;
		d.out_off = 0;
		d.out_cap = uint32_t(cap);
		HIP_OK(hipMemcpyAsync(d_desc.p, &d, sizeof d, hipMemcpyHostToDevice, stream));
		HIP_OK(launch_decode_variant(d_blk.p, uint64_t(std::max<int64_t>(blen, 1)), d_desc.p, 1,
		                             d_scr.p, d_bst.p, DEC_PC, stream));
		return start;
	}

	bool finish_fast_block(int64_t start, int64_t& first, int64_t& last)
	{
		lz4ada_block_status st;
		HIP_OK(hipMemcpyAsync(&st, d_bst.p, sizeof st, hipMemcpyDeviceToHost, stream));
		HIP_OK(hipStreamSynchronize(stream));
		if (st.code != DS_OK)
			return false;
		const int64_t nout = int64_t(st.out_len);
		if (m.has_content_size && uint64_t(nout) > m.size_remaining)
			return false;  // the exact path raises mid-block, as the reference does
		if (m.has_content_size)
			m.size_remaining -= uint64_t(nout);
		if (nout > 0)  // deliver() reads it from the mirror, after this copy
			HIP_OK(hipMemcpyAsync(d_buf.p + start, d_scr.p, size_t(nout), hipMemcpyDeviceToDevice,
			                      stream));
		output_pos = start + nout;
		if (output_pos >= HISTORY_SIZE)  // :785-787 (:688-690 for stored blocks)
			output_pos_history = output_pos;
		first = start;
		last = start + nout - 1;
		return true;
	}

	// Decode the current block (payload at blk, `total` bytes with its
	// checksum) and every complete block after it in [blk, end), up to the
	// end mark, in one bulk launch.  False when fewer than two are there.
	bool build_ahead(const uint8_t* blk, int64_t total, const uint8_t* end, int64_t buflen)
	{
		ahead.clear();
		if (m.is_format != F_MODERN && m.is_format != F_LEGACY)
			return false;
		const bool linked = m.is_format == F_MODERN && !(m.flg & 0x20u);
		const int bcl = m.block_checksum_length;
		const int64_t avail = end - blk;
		// a slot holds one block: the Buffer's room, at most the block maximum
		// (block_room with the largest payload, so every block of the batch fits)
		const int64_t room = std::max<int64_t>(
		        block_room(buflen, m.is_format == F_LEGACY ? (int64_t(8) << 20) : (int64_t(4) << 20), true), 1);
		const uint64_t slot = (uint64_t(room) + 255) & ~uint64_t(255);
		const uint64_t max_blocks = std::max<uint64_t>(1, (uint64_t(2) << 30) / slot);
		auto add = [&](int64_t off, int64_t sz, bool stored) {
			lz4ada_block_desc d{};
			d.in_off = uint64_t(off);
			d.in_len = uint32_t(sz);
			d.flags = (stored ? LZ4ADA_BLOCK_STORED : 0u) | (bcl ? LZ4ADA_BLOCK_HAS_CKSUM : 0u);
			d.out_off = uint64_t(ahead.descs.size()) * slot;
			d.out_cap = uint32_t(room);
			d.cksum = bcl ? load32(blk + off + sz) : 0u;
			ahead.descs.push_back(d);
		};
		add(0, total - bcl, !m.is_compressed);
		int64_t pos = total;
		while (pos + BLOCK_SIZE_BYTES <= avail && ahead.descs.size() < max_blocks &&
		       pos < (linked ? linked_cap : (int64_t(512) << 20))) {
			uint32_t w = load32(blk + pos);
			bool stored = false;
			if (m.is_format == F_MODERN) {
				if (w == 0)
					break;  // end mark
				stored = (w & 0x80000000u) != 0;
				w &= 0x7ffffffu;
			} else if (is_any_magic(w)) {
				break;  // the next frame
			}
			const int64_t sz = int64_t(w);
			if (sz + BLOCK_SIZE_BYTES + bcl > int64_t(input_buffer.size()) ||
			    pos + BLOCK_SIZE_BYTES + sz + bcl > avail)
				break;  // the exact path reports it, or the rest comes later
			add(pos + BLOCK_SIZE_BYTES, sz, stored);
			pos += BLOCK_SIZE_BYTES + sz + bcl;
		}
		const size_t nb = ahead.descs.size();
		if (nb < 2) {
			ahead.clear();
			return false;
		}
		ahead.input.assign(blk, blk + pos);
		ahead.slot = slot;
		ahead.st.assign(nb, lz4ada_block_status{});
		ahead.d_in.reserve(size_t(pos));
		ahead.d_out.reserve(size_t(nb * slot));
		ahead.d_desc.reserve(nb);
		ahead.d_st.reserve(nb);
		HIP_OK(hipMemcpyAsync(ahead.d_in.p, blk, size_t(pos), hipMemcpyHostToDevice, stream));
		vec_h2d(ahead.d_desc, ahead.descs, stream);
		HIP_OK(hipMemsetAsync(ahead.d_st.p, 0, nb * sizeof(lz4ada_block_status), stream));
		if (linked)
			return build_ahead_linked(nb, pos, buflen);
		if (few_large_blocks(ahead.descs) &&
		    decode_lone_blocks(blk, ahead.d_in.p, ahead.descs, ahead.d_out.p, ahead.d_st.p, ahead.st,
		                       ahead.d_lone, stream))
			return true;
		HIP_OK(hipMemsetAsync(ahead.d_st.p, 0, nb * sizeof(lz4ada_block_status), stream));
		if (bcl)
			HIP_OK(launch_block_checksums(ahead.d_in.p, ahead.d_desc.p, uint32_t(nb), ahead.d_st.p,
			                              stream));
		HIP_OK(launch_decode_blocks(ahead.d_in.p, uint64_t(pos), ahead.d_desc.p, uint32_t(nb),
		                            ahead.d_out.p, ahead.d_st.p, stream));
		vec_d2h(ahead.st, ahead.d_st, stream);
		return true;
	}

	// Read-ahead of a linked frame's blocks: all of them at once against
	// synthetic history, resolved on the GPU (bulk_linked, §7 of DESIGN),
	// seeded with the reference's history before the first one and its
	// Output_Pos / Output_Pos_History (quirk D1).  The blocks up to the
	// first one it cannot take are served; that one goes to the exact path.
	bool build_ahead_linked(size_t nb, int64_t in_len, int64_t buflen)
	{
		if (buflen > d_buf_len)
			grow_mirror(buflen);
		const int64_t start = output_pos >= HISTORY_SIZE ? 0 : output_pos;
		LinkedHist lh;
		history_of(start, lh.n0, lh.n1);
		lh.h0 = d_buf.p + output_pos_history - lh.n0;
		lh.h1 = d_buf.p;
		lh.output_pos = output_pos;
		lh.output_pos_history = output_pos_history;
		const int64_t bmax = int64_t(1) << (8 + 2 * ((m.bd & 0x70u) >> 4));
		int64_t room = 0;
		for (const auto& d : ahead.descs)
			room += std::max<int64_t>(d.out_cap, 1);
		ahead.d_out.reserve(size_t(room));
		int64_t used = 0;
		LinkedSink ls;
		ls.dst = [&](int64_t n) -> uint8_t* { return used + n <= room ? ahead.d_out.p + used : nullptr; };
		ls.done = [&](const uint8_t*, int64_t n) { used += n; };
		uint64_t total = 0;
		std::vector<uint32_t> lens;
		int64_t fail = -1;
		const BulkResult r = bulk_linked(ahead.d_in.p, uint64_t(in_len), bmax, ahead.descs, ls, total, lens,
		                                 fail, stream, &lh);
		HIP_OK(hipStreamSynchronize(stream));
		if (r != BULK_OK && r != BULK_FAIL_AT) {
			ahead.clear();
			return false;  // each block alone (lone decoder with history, else exact)
		}
		// A batch that stops early (quirk D1, an error) is decoded again from
		// the failing block on: the next batch is kept to about twice what this
		// one served, so frames with many such blocks are not re-decoded to
		// the end each time; a clean batch lets it grow back.
		if (r == BULK_OK) {
			linked_cap = std::min<int64_t>(int64_t(512) << 20, 2 * linked_cap);
		} else {
			int64_t served = 0;
			for (size_t k = 0; k < lens.size() && k < nb; ++k)
				served += int64_t(ahead.descs[k].in_len) + BLOCK_SIZE_BYTES + m.block_checksum_length;
			linked_cap = std::max<int64_t>(int64_t(1) << 20, 2 * served);
		}
		uint64_t off = 0;
		for (size_t k = 0; k < nb; ++k) {
			lz4ada_block_status& st = ahead.st[k];
			st = lz4ada_block_status{};
			if (k < lens.size()) {
				st.code = DS_OK;
				st.out_len = lens[k];
				st.cksum = ahead.descs[k].cksum;  // checked by bulk_linked
				ahead.descs[k].out_off = off;
				off += lens[k];
			} else {
				st.code = DS_RETRY;
			}
		}
		return true;
	}

	// Serve the current block from the read-ahead batch when it is the
	// batch's next block (same bytes) and decoded cleanly; the state moves
	// exactly as Decode_Full_Block_With_Trailer would move it.
	bool serve_ahead(const uint8_t* blk, int64_t total, const uint8_t* end, uint8_t* buf,
	                 int64_t buflen, int64_t& first, int64_t& last)
	{
		if (getenv("LZ4ADA_FACADE_EXACT"))
			return false;
		ensure_device();
		const int bcl = m.block_checksum_length;
		auto same = [&](size_t k) {
			const lz4ada_block_desc& d = ahead.descs[k];
			return int64_t(d.in_len) + bcl == total &&
			       memcmp(ahead.input.data() + d.in_off, blk, size_t(total)) == 0;
		};
		if (ahead.next >= ahead.descs.size() || !same(ahead.next)) {
			if (!build_ahead(blk, total, end, buflen))
				return false;
		}
		const size_t k = ahead.next++;
		const lz4ada_block_desc& d = ahead.descs[k];
		const lz4ada_block_status& st = ahead.st[k];
		const int64_t start = output_pos >= HISTORY_SIZE ? 0 : output_pos;  // :678-680
		const int64_t nout = int64_t(st.out_len);
		if (st.code != DS_OK || (bcl && st.cksum != d.cksum) || start + nout > buflen ||
		    (m.has_content_size && uint64_t(nout) > m.size_remaining)) {
			ahead.clear();  // the exact path takes this block (and reports it)
			return false;
		}
		if (buflen > d_buf_len)
			grow_mirror(buflen);
		const uint8_t* src = ahead.d_out.p + d.out_off;
		if (nout > 0) {  // the mirror keeps the history for a later exact block
			// a helper thread may still be hashing an earlier block's bytes in
			// this Buffer range (deliver() hands large blocks to it): join it
			// before the copy overwrites them
			hash_wait();
			HIP_OK(hipMemcpyAsync(d_buf.p + start, src, size_t(nout), hipMemcpyDeviceToDevice,
			                      stream));
			HIP_OK(hipMemcpyAsync(buf + start, src, size_t(nout), hipMemcpyDeviceToHost, stream));
			HIP_OK(hipStreamSynchronize(stream));
			if (m.content_checksum_length != 0)
				host_xxh32_update(hash_all, buf + start, size_t(nout));
		}
		if (m.has_content_size)
			m.size_remaining -= uint64_t(nout);
		output_pos = start + nout;
		if (output_pos >= HISTORY_SIZE)
			output_pos_history = output_pos;
		first = start;
		last = start + nout - 1;
		return true;
	}

	void cache_and_process(const uint8_t* in, int64_t len, int64_t& consumed, uint8_t* buf,
	                       int64_t buflen, int64_t& first, int64_t& last)  // :630-659
	{
		const int64_t avail = len - consumed;
		const int64_t want = input_length + m.block_checksum_length - m.input_buffer_filled +
		                     (m.is_format == F_BLOCK ? 0 : BLOCK_SIZE_BYTES);
		const int64_t fill = m.input_buffer_filled;
		const uint8_t* src = in + consumed;
		if (want > avail) {
			if (fill + avail > int64_t(input_buffer.size()))
				raise(LZ4ADA_CONSTRAINT_ERROR, "lz4ada.adb:644 index check failed");
			memcpy(input_buffer.data() + fill, src, size_t(avail));
			m.input_buffer_filled += avail;
			consumed += avail;
		} else {
			consumed += want;
			m.input_buffer_filled = 0;
			input_length = -1;
			// Input_Buffer(4 .. Fill-1) & Input(...): drops 4 cached bytes for
			// the raw-block format (quirk Q5), like the reference.
			const int64_t head = std::max<int64_t>(fill - BLOCK_SIZE_BYTES, 0);
			if (fill >= BLOCK_SIZE_BYTES && fill + want <= int64_t(input_buffer.size())) {
				// the rest of the block right after the cached bytes: no copy
				memcpy(input_buffer.data() + fill, src, size_t(want));
				decode_full_block(input_buffer.data() + BLOCK_SIZE_BYTES, head + want, buf, buflen,
				                  first, last);
				return;
			}
			blk_tmp.resize(size_t(head + want));
			if (head)
				memcpy(blk_tmp.data(), input_buffer.data() + BLOCK_SIZE_BYTES, size_t(head));
			memcpy(blk_tmp.data() + head, src, size_t(want));
			decode_full_block(blk_tmp.data(), head + want, buf, buflen, first, last);
		}
	}

	void update(const uint8_t* in, int64_t len, int64_t& consumed, uint8_t* buf, int64_t buflen,
	            int64_t& first, int64_t& last)  // lz4ada.adb:383-418
	{
		consumed = 0;
		first = 1;
		last = 0;
		if (m.header_parsing != HDR_DONE) {
			consumed = header_bytes(m, input_buffer.data(), in, len);
		} else if (m.is_format == F_SKIPPABLE) {
			consumed = skip(in, len);
		} else if (is_at_end_mark) {
			check_end_mark(in, len, consumed);
		} else if (input_length != -1) {
			cache_and_process(in, len, consumed, buf, buflen, first, last);
		} else {
			consumed = try_detect_input_length(in, len);
			if (is_at_end_mark) {
				check_end_mark(in, len, consumed);
			} else if (input_length != -1) {
				const int64_t total = input_length + m.block_checksum_length;
				if (len - consumed >= total) {  // :603-617, no copy
					const uint8_t* blk = in + consumed;
					consumed += total;
					m.input_buffer_filled = 0;
					input_length = -1;
					if (!serve_ahead(blk, total, in + len, buf, buflen, first, last))
						decode_full_block(blk, total, buf, buflen, first, last);
				} else {
					cache_and_process(in, len, consumed, buf, buflen, first, last);
				}
			}
		}
	}

	int is_end_of_frame() const  // :906-915
	{
		switch (m.is_format) {
		case F_LEGACY: return is_at_end_mark ? LZ4ADA_EOF_MAYBE : m.status_eof;
		case F_BLOCK: return input_length == -1 ? LZ4ADA_EOF_YES : LZ4ADA_EOF_NO;
		default: return m.status_eof;
		}
	}
};

// ---------------------------------------------------------------- C-ABI

static lz4ada_decompressor* new_ctx(int64_t in_last)
{
	auto* c = new lz4ada_decompressor();
	c->input_buffer.assign(size_t(std::max<int64_t>(in_last + 1, 0)), 0);
	return c;
}

extern "C" {

int lz4ada_abi_version(void) { return LZ4ADA_HIP_ABI_VERSION; }

const char* lz4ada_error_name(int status)
{
	static const char* const names[] = { "",
		                             "LZ4ADA.CHECKSUM_ERROR",
		                             "LZ4ADA.DATA_CORRUPTION",
		                             "LZ4ADA.NOT_SUPPORTED",
		                             "LZ4ADA.TOO_FEW_HEADER_BYTES",
		                             "LZ4ADA.TOO_LITTLE_MEMORY",
		                             "ADA.ASSERTIONS.ASSERTION_ERROR",
		                             "CONSTRAINT_ERROR",
		                             "LZ4ADA.DEVICE_ERROR",
		                             "LZ4ADA.EXACT_PATH" };
	if (status < 0 || status > LZ4ADA_EXACT_PATH)
		return "UNKNOWN";
	return names[status];
}

const char* lz4ada_thread_last_error(void) { return g_thread_error.c_str(); }

const char* lz4ada_last_error(const lz4ada_decompressor* ctx) { return ctx ? ctx->err.c_str() : ""; }

int64_t lz4ada_exact_blocks(const lz4ada_decompressor* ctx) { return ctx ? ctx->exact_blocks : -1; }

int lz4ada_device_check(void)
{
	return guarded(nullptr, [] { device_check_or_raise(); });
}

void lz4ada_to_hex8(uint8_t v, char out[3]) { snprintf(out, 3, "%02x", v); }
void lz4ada_to_hex32(uint32_t v, char out[9]) { snprintf(out, 9, "%08x", v); }

int lz4ada_init(int reservation, int64_t* min_buffer_size, lz4ada_decompressor** ctx)
{
	*ctx = nullptr;
	return guarded(nullptr, [&] {  // lz4ada.adb:48-63
		if (!concrete(reservation))
			raise(LZ4ADA_CONSTRAINT_ERROR, "Init requires a Memory_Reservation (SZ_*)");
		const int64_t bmax = block_size_of(reservation);
		*min_buffer_size = bmax + HISTORY_SIZE + 8;
		auto* c = new_ctx(bmax + 4 + BLOCK_SIZE_BYTES - 1);
		c->m.memory_reservation = reservation;
		*ctx = c;
	});
}

int lz4ada_init_with_header(const uint8_t* input, int64_t len, int reservation,
                            int64_t* num_consumed, int64_t* min_buffer_size,
                            lz4ada_decompressor** ctx)
{
	*ctx = nullptr;
	*num_consumed = 0;
	return guarded(nullptr, [&] {  // lz4ada.adb:79-125
		if (len < 7)
			raise(LZ4ADA_ASSERTION_ERROR, "failed precondition from lz4ada.ads:243");
		if (reservation < LZ4ADA_SZ_64_KIB || reservation > LZ4ADA_SINGLE_FRAME)
			raise(LZ4ADA_CONSTRAINT_ERROR, "bad reservation");
		uint8_t hb[20];
		Meta mt;
		mt.memory_reservation =
		        reservation == LZ4ADA_SINGLE_FRAME ? int(LZ4ADA_USE_FIRST) : reservation;
		int64_t pos = 0;
		while (mt.header_parsing != HDR_DONE) {
			if (pos >= len)
				raise(LZ4ADA_TOO_FEW_HEADER_BYTES,
				      "Expected at least " + img_u(mt.size_remaining) +
				              " more bytes but header input has already ended.");
			const int64_t c = header_bytes(mt, hb, input + pos, len - pos);
			pos += c;
			*num_consumed += c;
		}
		const int64_t bmax = block_size_of(mt.memory_reservation);
		*min_buffer_size = bmax + HISTORY_SIZE + 8;
		if (reservation == LZ4ADA_SINGLE_FRAME)
			mt.memory_reservation = LZ4ADA_SINGLE_FRAME;
		auto* c = new_ctx(bmax + mt.block_checksum_length + BLOCK_SIZE_BYTES - 1);
		c->m = mt;
		*ctx = c;
	});
}

int lz4ada_init_for_block(int64_t compressed_length, int reservation, int64_t* min_buffer_size,
                          lz4ada_decompressor** ctx)
{
	*ctx = nullptr;
	return guarded(nullptr, [&] {  // lz4ada.adb:127-147
		if (!concrete(reservation))
			raise(LZ4ADA_CONSTRAINT_ERROR, "Init_For_Block requires a Memory_Reservation");
		const int64_t bmax = block_size_of(reservation);
		*min_buffer_size = bmax + HISTORY_SIZE + 8;
		auto* c = new_ctx(bmax - 1);
		c->m.is_format = F_BLOCK;
		c->m.is_compressed = true;
		c->m.header_parsing = HDR_DONE;
		c->m.memory_reservation = reservation;
		c->input_length = compressed_length;
		*ctx = c;
	});
}

int lz4ada_update(lz4ada_decompressor* ctx, const uint8_t* input, int64_t len,
                  int64_t* num_consumed, uint8_t* buffer, int64_t buffer_len,
                  int64_t* output_first, int64_t* output_last)
{
	*num_consumed = 0;
	*output_first = 1;
	*output_last = 0;
	return guarded(&ctx->err, [&] {
		ctx->update(input, len, *num_consumed, buffer, buffer_len, *output_first, *output_last);
	});
}

int lz4ada_is_end_of_frame(const lz4ada_decompressor* ctx) { return ctx->is_end_of_frame(); }

void lz4ada_free(lz4ada_decompressor* ctx) { delete ctx; }

// -------------------------------------------------------------- XXHash32

void lz4ada_xxh32_reset(lz4ada_xxh32_state* h, uint32_t seed)  // lz4ada.adb:932-940
{
	h->state[0] = seed + P1 + P2;
	h->state[1] = seed + P2;
	h->state[2] = seed;
	h->state[3] = seed - P1;
	memset(h->buffer, 0, sizeof h->buffer);
	h->buffer_size = 0;
	h->total_length = 0;
	h->hash = 0;
}

void lz4ada_xxh32_init(lz4ada_xxh32_state* h, uint32_t seed)  // :925-930 (Q1)
{
	(void)seed;
	lz4ada_xxh32_reset(h, 0);
}

static int xxh32_update_dev(lz4ada_xxh32_state* h, const void* d_data, int64_t len,
                            hipStream_t stream)
{
	return guarded(nullptr, [&] {
		device_check_or_raise();
		DevBuf<lz4ada_xxh32_state> ds;
		ds.reserve(1);
		HIP_OK(hipMemcpyAsync(ds.p, h, sizeof *h, hipMemcpyHostToDevice, stream));
		HIP_OK(launch_xxh32_update(ds.p, static_cast<const uint8_t*>(d_data), uint64_t(len), stream));
		HIP_OK(hipMemcpyAsync(h, ds.p, sizeof *h, hipMemcpyDeviceToHost, stream));
		HIP_OK(hipStreamSynchronize(stream));
	});
}

int lz4ada_xxh32_update_device(lz4ada_xxh32_state* h, const void* d_data, int64_t len,
                               void* stream)
{
	return xxh32_update_dev(h, d_data, len, static_cast<hipStream_t>(stream));
}

// XXHash32.Update over HOST bytes (lz4ada.adb:942-991) runs on the calling
// host thread: the chain is serial, a host core runs it ~10x
// faster than one GPU wave, and the bytes are already on the host -- a
// device round trip per call (allocation, H2D, one-wave kernel, D2H, sync)
// only added latency.  Device-resident bytes keep the GPU kernel
// (lz4ada_xxh32_update_device) or the D2H pipeline (lz4ada_content_xxh32_d2h).
int lz4ada_xxh32_update(lz4ada_xxh32_state* h, const uint8_t* data, int64_t len)
{
	return guarded(nullptr, [&] {
		if (len < 0 || (len > 0 && !data))
			raise(LZ4ADA_ASSERTION_ERROR, "failed precondition: XXHash32.Update input");
		if (len > 0)
			host_xxh32_update(*h, data, size_t(len));
		h->hash = host_xxh32_final(*h);
	});
}

// XXHash32.Final (lz4ada.adb:993-1017): a pure function of the state.
uint32_t lz4ada_xxh32_final(const lz4ada_xxh32_state* h) { return host_xxh32_final(*h); }


int lz4ada_content_xxh32_d2h(lz4ada_xxh32_state* h, const void* d_data, int64_t len,
                             uint8_t* host_out, void* stream)
{
	return guarded(nullptr, [&] {
		content_xxh32_d2h(*h, static_cast<const uint8_t*>(d_data), len, host_out,
		                  static_cast<hipStream_t>(stream));
	});
}

int lz4ada_xxh32_hash(const uint8_t* data, int64_t len, uint32_t* out)  // :1019-1024
{
	lz4ada_xxh32_state h;
	lz4ada_xxh32_init(&h, 0);
	int st = lz4ada_xxh32_update(&h, data, len);
	if (st == LZ4ADA_OK)
		*out = h.hash;
	return st;
}

}  // extern "C"

// ------------------------------------------- shared with the bulk paths

// Content checksum pipeline: the frame-wide XXH32 is
// one serial chain that one GPU wave runs at ~1.3 GB/s, so
// for output that is headed to the host anyway the chain runs on the host
// core, chunk by chunk, while the next chunk is still in flight over PCIe.
// The bytes hashed are the ones the GPU decoded; nothing is decoded here.
void lz4ada::content_xxh32_d2h(lz4ada_xxh32_state& h, const uint8_t* d_data, int64_t len,
                              uint8_t* host_out, hipStream_t stream)
{
	device_check_or_raise();
	constexpr size_t CH = size_t(32) << 20;
	struct Pinned {
		uint8_t* p[2] = { nullptr, nullptr };
		hipEvent_t ev[2] = { nullptr, nullptr };
		~Pinned()
		{
			for (int i = 0; i < 2; ++i) {
				if (p[i])
					(void)hipHostFree(p[i]);
				if (ev[i])
					(void)hipEventDestroy(ev[i]);
			}
		}
	} pin;
	const size_t n = size_t(std::max<int64_t>(len, 0));
	const size_t chunks = (n + CH - 1) / CH;
	for (int i = 0; i < 2 && size_t(i) < chunks; ++i) {
		HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&pin.p[i]), CH, hipHostMallocDefault));
		HIP_OK(hipEventCreateWithFlags(&pin.ev[i], hipEventDisableTiming));
	}
	auto issue = [&](size_t k) {
		const size_t off = k * CH, c = std::min(CH, n - off);
		HIP_OK(hipMemcpyAsync(pin.p[k & 1], d_data + off, c, hipMemcpyDeviceToHost, stream));
		HIP_OK(hipEventRecord(pin.ev[k & 1], stream));
	};
	if (chunks)
		issue(0);
	for (size_t k = 0; k < chunks; ++k) {
		if (k + 1 < chunks)
			issue(k + 1);  // in flight while chunk k is hashed
		HIP_OK(hipEventSynchronize(pin.ev[k & 1]));
		const size_t off = k * CH, c = std::min(CH, n - off);
		host_xxh32_update(h, pin.p[k & 1], c);
		if (host_out)
			memcpy(host_out + off, pin.p[k & 1], c);
	}
	h.hash = host_xxh32_final(h);
}

namespace lz4ada {
// The reference's Buffer as it stands before the resume block: blocks form
// "rounds" -- one starts at Buffer position 0 whenever Output_Pos has
// reached 64 KiB (lz4ada.adb:678-680) and appends otherwise -- so Buffer(x)
// holds byte x of the newest round longer than x (zero if none is).
static void buffer_image(const Resume& rs, uint8_t* img, int64_t size)
{
	memset(img, 0, size_t(size));
	const auto& lens = *rs.lens;
	std::vector<std::pair<int64_t, int64_t>> rounds;  // (output offset, length)
	int64_t pos = 0, off = 0;
	for (size_t j = 0; j < lens.size(); ++j) {
		if (rounds.empty() || pos >= HISTORY_SIZE) {
			rounds.emplace_back(off, 0);
			pos = 0;
		}
		pos += lens[j];
		off += lens[j];
		rounds.back().second = pos;
	}
	int64_t filled = 0;
	for (size_t r = rounds.size(); r-- > 0 && filled < size;) {
		const int64_t hi = std::min(rounds[r].second, size);
		if (hi > filled)
			memcpy(img + filled, rs.output + rounds[r].first + filled, size_t(hi - filled));
		filled = std::max(filled, hi);
	}
}

// Reference-exact path for one frame: the unlz4ada loop
// (tool_unlz4ada/unlz4ada.adb:84-103) over the streaming engine, from the
// frame start or from `resume`.
}  // namespace lz4ada

void lz4ada::exact_frame(const uint8_t* f, int64_t len, Sink& out, int64_t& consumed_total,
                         const Resume* resume)
{
	int64_t consumed = 0, mbs = 0;
	lz4ada_decompressor* raw = nullptr;
	int st = lz4ada_init_with_header(f, len, LZ4ADA_SINGLE_FRAME, &consumed, &mbs, &raw);
	if (st)
		raise(st, g_thread_error);
	std::unique_ptr<lz4ada_decompressor> ctx(raw);
	std::vector<uint8_t> buf(size_t(mbs), 0);
	int eof = LZ4ADA_EOF_NO;
	int64_t pos = consumed;
	if (resume) {
		ctx->output_pos = resume->output_pos;
		ctx->output_pos_history = resume->output_pos_history;
		if (ctx->m.has_content_size)
			ctx->m.size_remaining -= resume->committed;
		ctx->hash_all = resume->hash;
		ctx->checksum_first = resume->checksum_first;
		pos = resume->at;
		if (resume->lens && !resume->lens->empty()) {
			// the history the resume block may read: Buffer and its mirror
			buffer_image(*resume, buf.data(), int64_t(buf.size()));
			ctx->ensure_device();
			if (ctx->d_buf_len < int64_t(buf.size()))
				ctx->grow_mirror(int64_t(buf.size()));
			HIP_OK(hipMemcpy(ctx->d_buf.p, buf.data(), buf.size(), hipMemcpyHostToDevice));
		}
	}
	while (pos < len) {
		int64_t c = 0, first = 1, last = 0;
		ctx->update(f + pos, len - pos, c, buf.data(), mbs, first, last);
		if (last >= first) {
			const int64_t nout = last - first + 1;
			memcpy(out.room(nout), buf.data() + first, size_t(nout));
			out.commit(nout);
		}
		pos += c;
		eof = ctx->is_end_of_frame();
		if (eof == LZ4ADA_EOF_YES)
			break;
		if (c == 0 && last < first)
			raise(LZ4ADA_CONSTRAINT_ERROR, "decoder made no progress");
	}
	if (eof == LZ4ADA_EOF_NO)
		raise(LZ4ADA_CONSTRAINT_ERROR, "End not signalled by library. Unable to process all data");
	consumed_total = pos;
}
