// xxhash32ada -- counterpart of the reference demo CLI
// (tool_xxhash32ada/xxhash32ada.adb): prints the XXHash32 (seed 0) of stdin
// as "xxhash32(0, stdin) = 0x<hex>" (To_Hex, lz4ada.ads:306-307).  The
// hasher lanes advance on the GPU (lz4ada_xxh32_update).
#include <cstdint>
#include <cstdio>
#include <vector>

#include "lz4ada_hip.h"

int main()
{
	std::vector<uint8_t> in;
	uint8_t buf[1 << 16];
	size_t n;
	while ((n = fread(buf, 1, sizeof buf, stdin)) > 0)
		in.insert(in.end(), buf, buf + n);
	lz4ada_xxh32_state h;
	lz4ada_xxh32_init(&h, 0);
	const int st = lz4ada_xxh32_update(&h, in.data(), int64_t(in.size()));
	if (st != LZ4ADA_OK) {
		fprintf(stderr, "raised %s : %s\n", lz4ada_error_name(st), lz4ada_thread_last_error());
		return 1;
	}
	char hex[9];
	lz4ada_to_hex32(lz4ada_xxh32_final(&h), hex);
	printf("xxhash32(0, stdin) = 0x%s\n", hex);
	return 0;
}
