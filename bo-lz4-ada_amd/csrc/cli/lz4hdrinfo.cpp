// lz4hdrinfo -- counterpart of tool_lz4hdrinfo/lz4hdrinfo.adb: prints the
// frame header fields of the first frame on stdin (a debug aid with its own
// copy of the header parse, lz4hdrinfo.adb:70-145; it does not link the
// library there either).  Same lines, same Ada 'Image spellings (TRUE /
// FALSE, a leading blank before numbers).
#include <cinttypes>
#include <cstdint>
#include <cstdio>
#include <cstring>

static const char* tf(bool b) { return b ? "TRUE" : "FALSE"; }

static uint32_t load32(const uint8_t* p)
{
	return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}

int main()
{
	printf("Ma_Sys.ma LZ4 Header Info 1.0.0, (c) 2023 Ma_Sys.ma <info@masysma.net>\n\n");
	uint8_t in[64];
	memset(in, 0, sizeof in);
	const size_t n = fread(in, 1, sizeof in, stdin);
	if (n < 7) {
		fflush(stdout);
		fprintf(stderr, "raised CONSTRAINT_ERROR : Partial frame detected. Unable to process all data\n");
		return 1;
	}
	const uint32_t magic = load32(in);
	const uint8_t flg = in[4], bd = in[5];
	if (magic == 0x184d2204u) {
		printf("Declared Format        = %08x (modern)\n", magic);
		printf("FLG                    = %02x\n", flg);
		printf("    Version:64|128     = %02x\n", (flg & 0xc0) >> 6);
		printf("    Block_Checksum:16  = %s\n", tf(flg & 16));
		printf("    Content_Size:8     = %s\n", tf(flg & 8));
		printf("    Content_Checksum:4 = %s\n", tf(flg & 4));
		printf("    Reserved:2         = %s\n", tf(flg & 2));
		printf("    Dictionary_ID:1    = %s\n", tf(flg & 1));
		printf("BD                     = %02x\n", bd);
		printf("    Has_Reserved       = %s\n", tf(bd & 0x8f));
		const uint8_t bms = (bd & 0x70) >> 4;
		static const char* const sizes[] = { "64 KiB", "256 KiB", "1 MiB", "4 MiB" };
		printf("    Block_Max_Size     = %s (%02x)\n", bms >= 4 && bms <= 7 ? sizes[bms - 4] : "INVALID",
		       bms);
		int cursor = 6;
		if (flg & 8) {
			uint64_t cs = 0;
			memcpy(&cs, in + cursor, 8);
			printf("Content_Size           =  %" PRIu64 "\n", cs);
			cursor += 8;
		}
		cursor += (flg & 1) ? 4 : 0;
		printf("Header_Checksum        = %02x\n", in[cursor]);
	} else if (magic == 0x184c2102u) {
		printf("Declared Format        = %08x (legacy)\n", magic);
	} else if (magic >= 0x184d2a50u && magic <= 0x184d2a5fu) {
		printf("Declared Format        = %08x (skippable)\n", magic);
		printf("Content_Size           =  %" PRIu32 "\n", load32(in + 4));
	} else {
		printf("Declared Format        = %08x (UNSUPPORTED)\n", magic);
	}
	return 0;
}
