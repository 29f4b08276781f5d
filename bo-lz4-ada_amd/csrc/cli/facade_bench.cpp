// facade_bench -- the streaming facade timed from C (tool_unlz4ada's loop,
// tool_unlz4ada/unlz4ada.adb:16, 84-103, over the C-ABI): Init_With_Header,
// then Update with `feed`-byte reads until End_Of_Frame, the delivered bytes
// appended to an output buffer and compared with the expected output once.
// No Python in the loop, so the per-call cost is the library's own.  Built
// by csrc/Makefile as bo-lz4-ada_amd/facade_bench; bench.py's `facade` key
// runs it (the last line of its output is one JSON object).
//   facade_bench frame.lz4 4096 5     (frame.lz4.out: the expected bytes)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "lz4ada_hip.h"

static std::vector<uint8_t> slurp(const char* path)
{
	std::vector<uint8_t> v;
	FILE* f = fopen(path, "rb");
	if (!f)
		return v;
	uint8_t b[1 << 16];
	size_t n;
	while ((n = fread(b, 1, sizeof b, f)) > 0)
		v.insert(v.end(), b, b + n);
	fclose(f);
	return v;
}

static int64_t g_exact = 0;  // blocks the last pass sent to the exact path

// One pass; returns seconds, or -1 on an error or a wrong output.
// reservation: LZ4ADA_SINGLE_FRAME (one context per frame, as timed by
// tools/facade_time.py) or LZ4ADA_USE_FIRST with `frame` holding several
// copies of the frame (one context for all: no per-frame device setup).
static double run(const std::vector<uint8_t>& frame, const std::vector<uint8_t>& expect, int64_t feed,
                  std::vector<uint8_t>& out, int reservation = LZ4ADA_SINGLE_FRAME)
{
	out.assign(expect.size(), 0);  // touch the pages first: no page faults inside the timed loop
	out.clear();
	const auto t0 = std::chrono::steady_clock::now();
	int64_t pos = 0, mbs = 0;
	lz4ada_decompressor* ctx = nullptr;
	if (lz4ada_init_with_header(frame.data(), int64_t(frame.size()), reservation, &pos, &mbs, &ctx) !=
	    LZ4ADA_OK) {
		fprintf(stderr, "init: %s\n", lz4ada_thread_last_error());
		return -1;
	}
	std::vector<uint8_t> buf(static_cast<size_t>(mbs));
	while (pos < int64_t(frame.size())) {
		const int64_t len = feed > 0 ? std::min<int64_t>(feed, int64_t(frame.size()) - pos)
		                             : int64_t(frame.size()) - pos;
		int64_t c = 0, first = 1, last = 0;
		if (lz4ada_update(ctx, frame.data() + pos, len, &c, buf.data(), mbs, &first, &last) != LZ4ADA_OK) {
			fprintf(stderr, "update: %s\n", lz4ada_last_error(ctx));
			lz4ada_free(ctx);
			return -1;
		}
		if (last >= first)
			out.insert(out.end(), buf.begin() + first, buf.begin() + last + 1);
		pos += c;
		if (reservation == LZ4ADA_SINGLE_FRAME && lz4ada_is_end_of_frame(ctx) == LZ4ADA_EOF_YES)
			break;
	}
	// the context's teardown (stream and device memory release) is not the
	// loop's cost: timed up to the last Update, like the Python loop
	const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
	g_exact = lz4ada_exact_blocks(ctx);
	lz4ada_free(ctx);
	return out == expect ? dt : -1;
}

int main(int argc, char** argv)
{
	if (argc < 2) {
		fprintf(stderr, "usage: %s frame.lz4 [feed] [reps]\n", argv[0]);
		return 2;
	}
	const std::vector<uint8_t> frame = slurp(argv[1]);
	const std::vector<uint8_t> expect = slurp((std::string(argv[1]) + ".out").c_str());
	const int64_t feed = argc > 2 ? atoll(argv[2]) : 4096;
	const int reps = argc > 3 ? atoi(argv[3]) : 5;
	if (frame.empty()) {
		perror(argv[1]);
		return 2;
	}
	std::vector<uint8_t> out;
	if (run(frame, expect, feed, out) < 0)  // warm (device setup, scratch)
		return 1;
	std::vector<double> ts;
	for (int r = 0; r < reps; ++r) {
		const double t = run(frame, expect, feed, out);
		if (t < 0)
			return 1;
		ts.push_back(t);
	}
	std::sort(ts.begin(), ts.end());
	const double mib = double(expect.size()) / (1 << 20);
	printf("facade_c %s feed=%lld: median of %d %.2f ms  %.1f MiB/s (best %.1f), a context per frame, "
	       "%lld exact blocks\n",
	       argv[1], (long long)feed, reps, ts[ts.size() / 2] * 1e3, mib / ts[ts.size() / 2], mib / ts[0],
	       (long long)g_exact);
	// the same frames back to back through one context (Use_First)
	constexpr int K = 8;
	std::vector<uint8_t> frames, expects;
	for (int k = 0; k < K; ++k) {
		frames.insert(frames.end(), frame.begin(), frame.end());
		expects.insert(expects.end(), expect.begin(), expect.end());
	}
	const double t = run(frames, expects, feed, out, LZ4ADA_USE_FIRST);
	if (t < 0)
		return 1;
	printf("facade_c %s feed=%lld: %d frames through one context %.2f ms per frame  %.1f MiB/s, "
	       "%lld exact blocks\n", argv[1], (long long)feed, K, t * 1e3 / K, mib * K / t, (long long)g_exact);
	printf("{\"mib_s\": %.1f, \"mib_s_best\": %.1f, \"ms_per_frame\": %.3f, \"reps\": %d, "
	       "\"mib_s_one_context\": %.1f, \"exact_blocks\": %lld}\n",
	       mib / ts[ts.size() / 2], mib / ts[0], ts[ts.size() / 2] * 1e3, reps, mib * K / t,
	       (long long)g_exact);
	return 0;
}
