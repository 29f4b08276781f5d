// unlz4ada -- counterpart of the reference CLI (tool_unlz4ada/unlz4ada.adb):
// decompress every frame of stdin (or of the file named by argv[1]) to
// stdout.  Frames go through the library's bulk GPU path one at a time
// (lz4ada_decode_frame_partial: Init_With_Header(Single_Frame) + Update
// semantics per frame, as the reference tool re-inits per frame,
// unlz4ada.adb:84-87); each frame's bytes are written before the next
// frame is decoded, and a failing frame's blocks before the failing block
// are written before the error, as the reference's per-block writes leave
// them.  An error prints the reference's Exception_Information
// line ("raised LZ4ADA.<NAME> : <message>") to stderr and exits 1; fewer
// than 7 bytes left at a frame start is the tool's own
// "Partial frame detected" Constraint_Error (unlz4ada.adb:65-76).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "lz4ada_hip.h"

static bool read_all(FILE* f, std::vector<uint8_t>& v)
{
	uint8_t buf[1 << 16];
	size_t n;
	while ((n = fread(buf, 1, sizeof buf, f)) > 0)
		v.insert(v.end(), buf, buf + n);
	return !ferror(f);
}

static int fail(int st, const char* msg)
{
	fprintf(stderr, "raised %s : %s\n", lz4ada_error_name(st), msg);
	return 1;
}

int main(int argc, char** argv)
{
	std::vector<uint8_t> in;
	FILE* f = argc > 1 ? fopen(argv[1], "rb") : stdin;
	if (!f || !read_all(f, in)) {
		perror(argc > 1 ? argv[1] : "stdin");
		return 2;
	}
	if (f != stdin)
		fclose(f);
	const int64_t len = int64_t(in.size());
	int64_t pos = 0;
	while (pos < len) {
		if (len - pos < 7)
			return fail(LZ4ADA_CONSTRAINT_ERROR, "Partial frame detected. Unable to process all data");
		uint8_t* out = nullptr;
		int64_t out_len = 0, consumed = 0;
		// on an error, the blocks the reference wrote before raising come
		// back too (unlz4ada.adb:41 writes each block as Update returns it)
		const int st = lz4ada_decode_frame_partial(in.data() + pos, len - pos, &out, &out_len, &consumed);
		const bool ok = out_len == 0 || fwrite(out, 1, size_t(out_len), stdout) == size_t(out_len);
		lz4ada_buffer_free(out);
		if (st != LZ4ADA_OK) {
			fflush(stdout);
			return fail(st, lz4ada_thread_last_error());
		}
		if (!ok) {
			perror("stdout");
			return 2;
		}
		pos += consumed;
	}
	return fflush(stdout) == 0 ? 0 : 2;
}
