// unlz4ada_simple -- counterpart of tool_unlz4ada_simple/unlz4ada_simple.adb:
// the library-simple path, one Init(For_All) context and an Update loop over
// 4 KiB reads of stdin (lz4ada.ads:189-191, 281-287), so every frame of the
// stream goes through the streaming facade (lz4ada_update: read-ahead bulk
// decode or single blocks on the GPU).  Errors print the reference's
// Exception_Information line and exit 1; input ending mid-frame is the
// tool's own Constraint_Error.
#include <cstdint>
#include <cstdio>
#include <vector>

#include "lz4ada_hip.h"

static int fail(int st, const char* msg)
{
	fprintf(stderr, "raised %s : %s\n", lz4ada_error_name(st), msg);
	return 1;
}

int main()
{
	int64_t bufsz = 0;
	lz4ada_decompressor* ctx = nullptr;
	int st = lz4ada_init(LZ4ADA_FOR_ALL, &bufsz, &ctx);
	if (st != LZ4ADA_OK)
		return fail(st, lz4ada_thread_last_error());
	std::vector<uint8_t> out(static_cast<size_t>(bufsz)), in(4096);
	int64_t last = -1, total = 0;
	for (;;) {
		if (total > last) {
			const size_t n = fread(in.data(), 1, in.size(), stdin);
			if (n == 0)
				break;
			last = int64_t(n) - 1;
			total = 0;
		}
		int64_t consumed = 0, first = 1, olast = 0;
		st = lz4ada_update(ctx, in.data() + total, last - total + 1, &consumed, out.data(), bufsz,
		                   &first, &olast);
		if (st != LZ4ADA_OK) {
			const int rc = fail(st, lz4ada_last_error(ctx));
			lz4ada_free(ctx);
			return rc;
		}
		if (olast >= first && fwrite(out.data() + first, 1, size_t(olast - first + 1), stdout) !=
		                              size_t(olast - first + 1)) {
			perror("stdout");
			return 2;
		}
		total += consumed;
	}
	const bool mid = lz4ada_is_end_of_frame(ctx) == LZ4ADA_EOF_NO;
	lz4ada_free(ctx);
	if (mid)
		return fail(LZ4ADA_CONSTRAINT_ERROR, "Input ended mid-frame.");
	return fflush(stdout) == 0 ? 0 : 2;
}
