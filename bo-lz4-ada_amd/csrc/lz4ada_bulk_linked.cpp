// lz4ada_bulk_linked.cpp -- the linked-frame bulk path of the MI355X LZ4Ada
// decompressor (BASELINE configs[4]): every block of a
// linked frame (B.Indep = 0, the LZ4F default) decoded at once against
// synthetic history, which lz4ada_linked.hip then resolves on the GPU by
// pointer jumping; quirk D1 (lib/lz4ada.adb:811-817, 862-879)
// and references before the frame start go to the exact path.
#include "lz4ada_host_common.h"

namespace lz4ada {

// Linked frames (and independent ones whose blocks read earlier blocks,
// D2): every block at once with synthetic history, resolved on the GPU
// (lz4ada_linked.hip), batch by batch with the previous batch's last
// 64 KiB carried as real history.  BULK_EXACT: the frame needs the exact
// path (a block error or checksum mismatch, quirk D1, a reference before
// the frame start, no device memory).
BulkResult bulk_linked(const uint8_t* d_frame, uint64_t frame_len, int64_t block_max,
                              const std::vector<lz4ada_block_desc>& descs, LinkedSink& sink,
                              uint64_t& total, std::vector<uint32_t>& lens, int64_t& fail,
                              hipStream_t stream, const LinkedHist* hist)
{
	lens.clear();
	fail = -1;
	// a batch holds 3 decode buffers (slots + 64 KiB regions) and one 4-byte
	// word per output byte: ~7x its slot bytes
	uint64_t budget = uint64_t(env_bytes("LZ4ADA_LINKED_BATCH_BYTES", int64_t(2) << 30));
	// LZ4ADA_TRACE_LINKED=1: phase times (synchronised) to stderr; =2: the
	// host's own time between the phases (no synchronisation)
	static const int trace = [] {
		const char* e = getenv("LZ4ADA_TRACE_LINKED");
		return e ? std::max(1, atoi(e)) : 0;
	}();
	auto t0 = std::chrono::steady_clock::now();
	auto phase = [&](const char* name) {
		if (!trace)
			return;
		if (trace == 1)
			HIP_OK(hipStreamSynchronize(stream));
		const auto t1 = std::chrono::steady_clock::now();
		fprintf(stderr, "[linked] %-10s %8.3f ms\n", name,
		        std::chrono::duration<double, std::milli>(t1 - t0).count());
		t0 = t1;
	};
	auto why = [&](BulkResult r, const char* reason) {  // (trace) why the batch loop ends
		if (trace)
			fprintf(stderr, "[linked] result %d: %s\n", int(r), reason);
		return r;
	};
	// the small per-call buffers -- both history tails, and per batch the
	// descriptors, both planes' statuses, A, the modes and the round counters
	// -- carved from one thread-cached device buffer, and their host sides
	// from one thread-cached pinned buffer: a pooled buffer's release costs
	// a device synchronisation (round 5: ~8 per call)
	const size_t nmax = descs.size();
	auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
	const size_t o_desc = 2 * size_t(HISTORY_SIZE), o_st = o_desc + al(nmax * sizeof(lz4ada_block_desc)),
	             o_A = o_st + al(2 * nmax * sizeof(lz4ada_block_status)), o_mode = o_A + al(nmax * sizeof(int64_t)),
	             o_ctr = o_mode + al(nmax), link_bytes = o_ctr + 256;
	uint8_t* const lk = scratch(SC_LINK, link_bytes);
	if (!lk)
		return why(BULK_EXACT, "exit at line 61");
	PinBuf& pin = scratch_cache().pin;
	pin.reserve(link_bytes);
	uint8_t* const hp = pin.p;  // host twin of lk: hp + o is the host side of lk + o
	struct {
		uint8_t* p;
	} d_tail[2]{ { lk }, { lk + HISTORY_SIZE } };
	HIP_OK(hipMemsetAsync(d_tail[0].p, 0, size_t(HISTORY_SIZE), stream));
	int cur = 0;
	// the reference's Output_Pos / Output_Pos_History (lz4ada.adb:678-690,
	// 785-787), for quirk D1
	int64_t opos = 0, oph = 0;
	int64_t hist0 = 0;  // history bytes before the first block (mid-frame batch)
	if (hist) {
		hist0 = std::min<int64_t>(hist->n0 + hist->n1, HISTORY_SIZE);
		if (hist->n1 > 0)
			HIP_OK(hipMemcpyAsync(d_tail[0].p + HISTORY_SIZE - hist->n1, hist->h1, size_t(hist->n1),
			                      hipMemcpyDeviceToDevice, stream));
		if (hist->n0 > 0)
			HIP_OK(hipMemcpyAsync(d_tail[0].p + HISTORY_SIZE - hist->n1 - hist->n0, hist->h0,
			                      size_t(hist->n0), hipMemcpyDeviceToDevice, stream));
		opos = hist->output_pos;
		oph = hist->output_pos_history;
	}
	uint32_t lo = 0;
	total = 0;
	while (lo < descs.size()) {
		const auto bt = batches_of(std::vector<lz4ada_block_desc>(descs.begin() + lo, descs.end()),
		                           block_max, uint64_t(HISTORY_SIZE), budget);
		const uint32_t hi = lo + bt[0].second;
		uint32_t nb = hi - lo;
		std::vector<lz4ada_block_desc> d(descs.begin() + lo, descs.begin() + hi);
		phase("batch");
		uint64_t bytes = 0;
		for (auto& x : d) {
			x.out_cap = slot_cap(x, block_max);
			x.out_off = bytes + uint64_t(HISTORY_SIZE);
			bytes += uint64_t(HISTORY_SIZE) + round256(x.out_cap);
		}
		// quirk D1's round state, predicted with every block filling its
		// slot (Output_Pos / Output_Pos_History, lz4ada.adb:678-690,
		// 785-787): the index decoder emulates D1 under it, and the replay
		// below accepts a block only if the real state is the predicted one
		{
			int64_t po = opos, ph = oph;
			for (auto& x : d) {
				if (po >= HISTORY_SIZE)
					po = 0;
				x.flags &= LZ4ADA_BLOCK_STORED | LZ4ADA_BLOCK_HAS_CKSUM;
				if (ph >= HISTORY_SIZE && ph <= HISTORY_SIZE + 6)
					x.flags |= BLOCK_D1_ROUND | (uint32_t(ph - HISTORY_SIZE) << BLOCK_D1_OPH_SHIFT) |
					           (uint32_t(po) << BLOCK_N1_SHIFT);
				po += int64_t(x.out_cap);
				if (po >= HISTORY_SIZE)
					ph = po;
			}
		}
		// two planes for every block (x: history k -> k & 255; z: literals
		// as zeros, history k -> k >> 8), two more (y, h) only for the blocks
		// z cannot serve
		struct {
			uint8_t* p;
		} bx{ scratch(SC_X, size_t(bytes)) }, bz{ bx.p ? scratch(SC_Z, size_t(bytes)) : nullptr },
		    tab{ bz.p ? scratch(SC_TAB, index_table_bytes(frame_len, nb)) : nullptr };
		if (!tab.p) {
			if (budget > (uint64_t(64) << 20) && nb > 1) {
				budget /= 2;
				continue;
			}
			return why(BULK_EXACT, "exit at line 130");
		}
		// planes x's and z's statuses side by side: one copy back
		struct {
			lz4ada_block_desc* p;
		} d_desc{ reinterpret_cast<lz4ada_block_desc*>(lk + o_desc) };
		struct {
			lz4ada_block_status* p;
		} s2{ reinterpret_cast<lz4ada_block_status*>(lk + o_st) }, sx{ s2.p }, sz{ s2.p + nb };
		const size_t sb = nb * sizeof(lz4ada_block_status);
		const size_t db = nb * sizeof(lz4ada_block_desc);
		phase("alloc");
		memcpy(hp + o_desc, d.data(), db);
		HIP_OK(hipMemcpyAsync(d_desc.p, hp + o_desc, db, hipMemcpyHostToDevice, stream));
		phase("desc h2d");
		HIP_OK(hipMemsetAsync(sx.p, 0, sb, stream));
		// the history regions' fill and the checksums ride beside the index
		// (side stream); the decodes wait for the fill, the status read for
		// the checksums
		HIP_OK(launch_link_fill_beside(bx.p, nullptr, bz.p, d_desc.p, nb, stream));
		HIP_OK(launch_block_checksums_beside(d_frame, d_desc.p, nb, sx.p, stream));
		HIP_OK(launch_index(d_frame, frame_len, d_desc.p, nb, tab.p, sx.p, stream));
		HIP_OK(join_link_fill(stream));
		phase("launches");
		HIP_OK(hipMemcpyAsync(sz.p, sx.p, sb, hipMemcpyDeviceToDevice, stream));
		// plane z's decode on the side stream beside plane x's: each launch
		// has more blocks than resident slots, and the other one's blocks
		// fill the slots its last ones leave idle
		// (LZ4ADA_LINK_SERIAL=1: one after the other, for A/B)
		static const bool serial = getenv("LZ4ADA_LINK_SERIAL") != nullptr;
		hipStream_t side = stream;
		if (!serial)
			HIP_OK(side_fork(stream, &side));
		HIP_OK(launch_decode_idx_tab(d_frame, frame_len, d_desc.p, nb, tab.p, bz.p, sz.p, 6, side));
		HIP_OK(launch_decode_idx_tab(d_frame, frame_len, d_desc.p, nb, tab.p, bx.p, sx.p, 2, stream));
		HIP_OK(launch_decode_pc(d_frame, frame_len, d_desc.p, nb, bx.p, sx.p, 1, LINK_HIST, stream));
		HIP_OK(side_join(stream));  // plane z and the checksums
		phase("decodes");
		std::vector<lz4ada_block_status> st(nb), stz(nb);
		d2h(hp + o_st, s2.p, 2 * sb, stream);
		memcpy(st.data(), hp + o_st, sb);
		memcpy(stz.data(), hp + o_st + sb, sb);
		int64_t* A = reinterpret_cast<int64_t*>(hp + o_A);
		int64_t n = 0;
		const int64_t opos0 = opos, oph0 = oph;  // this batch's start (a smaller retry rescans)
		// the first block the exact path has to take: a block error, a
		// checksum mismatch, or quirk D1 (a match reaching
		// >= D1_OFF back into the history right after a block that ended at
		// 65536..65542).  The blocks before it only point backwards, so they
		// resolve on their own and the exact path resumes at it.
		uint32_t ok_n = nb;
		for (uint32_t i = 0; i < nb; ++i) {
			if (opos >= HISTORY_SIZE)
				opos = 0;
			// quirk D1: a block with a match >= D1_OFF back before its start
			// (AUX_D1_RISK) in a round after one that ended at 65536..65542
			// is the decoders' only if the index decoder (which emulates D1)
			// decoded it under the real round state; one decoded under a D1
			// prediction the real state does not have goes too (without
			// such a match, neither the quirk nor the emulation changes a byte)
			const bool in_d1 = oph >= HISTORY_SIZE && oph <= HISTORY_SIZE + 6;
			const bool emu = (st[i].aux & AUX_D1_EMU) != 0;
			// (plane z declined: planes y and h come from k_decode_pc, which
			// does not emulate D1 -- the planes would disagree)
			const bool pred_ok = emu && in_d1 && (d[i].flags & BLOCK_D1_ROUND) && stz[i].code == DS_OK &&
			                     int64_t((d[i].flags >> BLOCK_D1_OPH_SHIFT) & 7u) == oph - HISTORY_SIZE &&
			                     int64_t(d[i].flags >> BLOCK_N1_SHIFT) == opos;
			const bool d1_bad = (st[i].aux & AUX_D1_RISK) && (in_d1 ? !pred_ok : emu);
			if (trace > 2)
				fprintf(stderr, "[linked] block %u: code %d aux %d len %u z %d | opos %lld oph %lld pred %s%u/%u%s\n",
				        lo + i, st[i].code, st[i].aux, st[i].out_len, stz[i].code, (long long)opos, (long long)oph,
				        (d[i].flags & BLOCK_D1_ROUND) ? "" : "-", (d[i].flags >> BLOCK_D1_OPH_SHIFT) & 7u,
				        d[i].flags >> BLOCK_N1_SHIFT, d1_bad ? " D1 STOP" : "");
			if (st[i].code != DS_OK ||
			    ((d[i].flags & LZ4ADA_BLOCK_HAS_CKSUM) && st[i].cksum != d[i].cksum) || d1_bad) {
				ok_n = i;
				break;
			}
			opos += st[i].out_len;
			if (opos >= HISTORY_SIZE)
				oph = opos;
			A[i] = n;
			n += st[i].out_len;
		}
		if (ok_n < nb) {
			fail = int64_t(lo) + ok_n;
			nb = ok_n;
			if (nb == 0)
				return why(BULK_FAIL_AT, "fail-at exit at line 211");
		}
		if (n >= (int64_t(1) << 31) - HISTORY_SIZE) {  // words hold positions + 65536 in 31 bits
			if (nb > 1) {
				// the smaller batch rescans from this batch's start: its own
				// first failing block (if any) and the replayed positions
				budget /= 2;
				fail = -1;
				opos = opos0;
				oph = oph0;
				continue;
			}
			return why(BULK_EXACT, "exit at line 223");
		}
		// blocks plane z cannot serve alone: one that reads history positions
		// below 256 (AUX_DEEP_HIST: their high byte is 0, like a literal's)
		// takes plane y too (x != y marks a history byte, k = x | z << 8);
		// one z's decoder declined (oversized batches, anything pass 1
		// declined) takes y and h -- the three-plane rule.  Every other block
		// is DS_SKIP in those launches.
		uint8_t* mode = hp + o_mode;
		memset(mode, 0, nb);
		uint32_t ny = 0, nh = 0;
		for (uint32_t i = 0; i < nb; ++i) {
			if (stz[i].code != DS_OK)
				mode[i] = 2;
			else if (stz[i].aux & AUX_DEEP_HIST)
				mode[i] = 1;
			ny += mode[i] != 0;
			nh += mode[i] == 2;
		}
		uint8_t *py = nullptr, *ph = nullptr;
		struct {
			uint8_t* p;
		} d_mode{ lk + o_mode };
		if (ny) {
			py = scratch(SC_Y, size_t(bytes));
			ph = py && nh ? scratch(SC_H, size_t(bytes)) : nullptr;
			if (!py || (nh && !ph))
				return why(BULK_EXACT, "exit at line 250");
			HIP_OK(hipMemcpyAsync(d_mode.p, mode, nb, hipMemcpyHostToDevice, stream));
			HIP_OK(launch_link_fill(nullptr, py, ph, d_desc.p, nb, stream));
			std::vector<lz4ada_block_status> s_plane[2];
			// (nb may be smaller than when sb was taken: the blocks before a
			// failing one)
			const size_t sbn = nb * sizeof(lz4ada_block_status);
			for (int k = 0; k < (nh ? 2 : 1); ++k) {
				std::vector<lz4ada_block_status> s3(stz);
				for (uint32_t i = 0; i < nb; ++i)
					if (mode[i] <= k)  // y: modes 1 and 2; h: mode 2
						s3[i].code = DS_SKIP;
				// the plane's statuses in plane z's half of the status scratch
				// (free: stz is on the host), not a pooled buffer -- releasing
				// one costs a device-wide synchronisation
				lz4ada_block_status* const s_dev = sz.p;
				HIP_OK(hipMemcpyAsync(s_dev, s3.data(), sbn, hipMemcpyHostToDevice, stream));
				uint8_t* buf = k == 0 ? py : ph;
				HIP_OK(launch_decode_idx_tab(d_frame, frame_len, d_desc.p, nb, tab.p, buf, s_dev, 2, stream));
				HIP_OK(launch_decode_pc(d_frame, frame_len, d_desc.p, nb, buf, s_dev, 1, LINK_HIST, stream));
				s_plane[k].resize(nb);
				d2h(s_plane[k].data(), s_dev, sbn, stream);
				for (uint32_t i = 0; i < nb; ++i)
					if (mode[i] > k &&
					    (s_plane[k][i].code != DS_OK || s_plane[k][i].out_len != st[i].out_len))
						return why(BULK_EXACT, "never expected: plane x decoded it");
			}
			phase("more planes");
		}
		struct {
			int64_t* p;
		} d_A{ reinterpret_cast<int64_t*>(lk + o_A) };
		struct {
			uint32_t* p;
		} d_ctr{ reinterpret_cast<uint32_t*>(lk + o_ctr) };
		struct {
			uint32_t* p;
		} d_P{ reinterpret_cast<uint32_t*>(scratch(SC_P, size_t(std::max<int64_t>(n, 1)) * 4)) };
		if (!d_P.p)
			return why(BULK_EXACT, "exit at line 289");
		HIP_OK(hipMemcpyAsync(d_A.p, A, nb * sizeof(int64_t), hipMemcpyHostToDevice, stream));
		const int64_t tail_valid = std::min<int64_t>(int64_t(total) + hist0, HISTORY_SIZE);
		uint8_t* F = nullptr;
		// a word per output byte (resolving only the history-derived bytes,
		// round 4's sparse form, measured slower -- three gathers per target
		// instead of one word -- DESIGN §7)
		{
			// the constant bytes go to F with the words, each round writes the
			// bytes it resolves: the last round leaves the output
			F = sink.dst(n);
			if (!F)
				return why(BULK_EXACT, "exit at line 301");
			// span activity flags, double-buffered across rounds (an init that
			// also stepped every history-derived byte one pointer forward was
			// measured and dropped: mixed 10.32 vs 10.35 ms, chain 13.5 vs
			// 15.4, dense 31.0 vs 23.7 -- its byte gathers cost what the round
			// saves)
			const int64_t ns = link_spans(n);
			uint8_t* act = scratch(SC_U, size_t(2 * ns + 64));
			uint8_t* M = act ? scratch(SC_M, size_t(n) + 64) : nullptr;
			if (!M)
				return why(BULK_EXACT, "exit at line 311");
			// init flags the spans that hold a history-derived byte: the
			// first round reads only those
			HIP_OK(hipMemsetAsync(act + ns, 0, size_t(ns), stream));
			// words everywhere (`full`) or only where a byte is still open
			// after init's steps: the latter saves most of init's writes but
			// costs the rounds a gather per word (a source's M), which only
			// pays where few stay open.  The z decoder counts the match bytes
			// each block reads straight from history: above 1/12 of the
			// batch's bytes (measured: dense 0.102, mixed 0.058, chain 0),
			// full.
			// LZ4ADA_LINK_WORDS=full / sparse forces one.
			int64_t hbytes = 0;
			for (uint32_t i = 0; i < nb; ++i)
				hbytes += stz[i].detail;
			const char* we = getenv("LZ4ADA_LINK_WORDS");  // (per call: the tests force both)
			const int words_env = we ? (we[0] == 'f' ? 1 : (we[0] == 's' ? 2 : 0)) : 0;
			const bool full = words_env ? words_env == 1 : 12 * hbytes > n;
			if (trace)
				fprintf(stderr, "[linked] history   %.3f of the bytes read straight from history: %s words\n",
				        double(hbytes) / double(std::max<int64_t>(n, 1)), full ? "full" : "sparse");
			HIP_OK(launch_link_init(bx.p, bz.p, py, ph, ny ? d_mode.p : nullptr, d_desc.p, sx.p, d_A.p, nb,
			                        block_max, d_tail[cur].p, tail_valid, d_P.p, F, M, act + ns, full, stream));
			phase("init");
			auto spans_flagged = [&](const uint8_t* a) {  // (trace only) spans a round will visit
				if (!trace)
					return;
				std::vector<uint8_t> h(static_cast<size_t>(ns));
				d2h(h.data(), a, size_t(ns), stream);
				size_t c = 0;
				for (uint8_t v : h)
					c += v != 0;
				fprintf(stderr, "[linked] spans     %zu of %lld flagged\n", c, (long long)ns);
			};
			spans_flagged(act + ns);
			// the rounds run in pairs, one host round trip per pair (a mixed
			// frame needs two rounds; a round after the last one finds every
			// span flagged 0 and reads only the flags).  The first pair always
			// runs: init's span flags leave it nothing to read when no byte
			// came from history (a count would cost an atomic per wave and a
			// round trip)
			uint32_t left = 1;
			for (int round = 0; left > 0; round += 2) {
				if (round > 64)
					return why(BULK_EXACT, "never expected: every pointer goes strictly back");
				HIP_OK(hipMemsetAsync(d_ctr.p, 0, 4 * sizeof(uint32_t), stream));
				for (int k = 0; k < 2; ++k) {
					uint8_t* a_out = act + ((round + k) & 1) * ns;
					const uint8_t* a_in = act + ((round + k + 1) & 1) * ns;
					HIP_OK(launch_link_jump(d_P.p, M, n, d_tail[cur].p, tail_valid, F, a_in, a_out,
					                        d_ctr.p + 2 * k, full, stream));
					spans_flagged(a_out);
				}
				// the next batch's history, enqueued before the round trip (a
				// later pair, if any, writes it again)
				HIP_OK(launch_link_tail(F, n, d_tail[cur].p, d_tail[cur ^ 1].p, stream));
				uint32_t* c4 = reinterpret_cast<uint32_t*>(hp + o_ctr);
				d2h(c4, d_ctr.p, 4 * sizeof(uint32_t), stream);
				if (c4[1] || c4[3])
					return why(BULK_EXACT, "a reference before the frame start: the exact error");
				left = c4[2];  // words still unresolved after the pair's second round
			}
			phase("jumps");
		}
		cur ^= 1;
		phase("emit");
		sink.done(F, n);
		phase("sink");
		total += uint64_t(n);
		for (uint32_t i = 0; i < nb; ++i)
			lens.push_back(st[i].out_len);
		if (fail >= 0)
			return why(BULK_FAIL_AT, "fail-at exit at line 383");
		lo = hi;
	}
	return BULK_OK;
}

}  // namespace lz4ada
