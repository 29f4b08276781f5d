/*
 * lz4ada_oracle.h -- CPU restatement of the reference LZ4Ada library.
 *
 * TEST INFRASTRUCTURE ONLY.  This oracle is the parity checker for the
 * MI355X decoder in bo-lz4-ada_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  It is never linked into, or
 * called by, the product library (bo-lz4-ada_amd/liblz4ada_hip.so).
 *
 * It restates /root/reference/lib/lz4ada.adb (+ lz4ada.ads) in plain C:
 * header parser, streaming Update state machine, block decoder with the
 * reference's 8-byte wild copy and Output_Pos / Output_Pos_History buffer
 * scheme, and the streaming XXHash32.  Exceptions become status codes plus
 * the exact Exception_Information text of the reference.
 *
 * Parity pinning: the reference is Ada and cannot be compiled here (no
 * GNAT).  The oracle is pinned by the reference's own
 * fixtures: all test_vectors_lz4 .lz4 -> .bin digests (4 KiB and 1-byte
 * feed), all .err -> .eds exception strings, and the in-source KATs of
 * test_suite/lz4test.adb (tests/test_oracle_*.py).
 */
#ifndef LZ4ADA_ORACLE_H
#define LZ4ADA_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: one per reference exception (lz4ada.ads:133-162). */
enum {
	OR_OK = 0,
	OR_CHECKSUM_ERROR = 1,
	OR_DATA_CORRUPTION = 2,
	OR_NOT_SUPPORTED = 3,
	OR_TOO_FEW_HEADER_BYTES = 4,
	OR_TOO_LITTLE_MEMORY = 5,
	OR_ASSERTION_ERROR = 6, /* Ada Pre/Assert failure (API misuse) */
	OR_CONSTRAINT_ERROR = 7 /* library-bug branch (lz4ada.adb:184-188) */
};

/* Flexible_Memory_Reservation (lz4ada.ads:79-80), same order. */
enum {
	OR_SZ_64_KIB = 0,
	OR_SZ_256_KIB = 1,
	OR_SZ_1_MIB = 2,
	OR_SZ_4_MIB = 3,
	OR_SZ_8_MIB = 4,
	OR_USE_FIRST = 5,
	OR_SINGLE_FRAME = 6
};

/* End_Of_Frame (lz4ada.ads:124), same order. */
enum { OR_EOF_YES = 0, OR_EOF_NO = 1, OR_EOF_MAYBE = 2 };

typedef struct oracle_ctx oracle_ctx;

/* LZ4Ada.Init (lz4ada.adb:48-63). reservation must be SZ_*. */
int oracle_init(int reservation, int64_t *min_buffer_size, oracle_ctx **out);

/* LZ4Ada.Init_With_Header (lz4ada.adb:79-125).  On error *out is NULL and
 * the message goes to errbuf. */
int oracle_init_with_header(const uint8_t *input, int64_t len, int reservation,
                            int64_t *num_consumed, int64_t *min_buffer_size,
                            oracle_ctx **out, char *errbuf, size_t errcap);

/* LZ4Ada.Init_For_Block (lz4ada.adb:127-147). */
int oracle_init_for_block(int64_t compressed_length, int reservation,
                          int64_t *min_buffer_size, oracle_ctx **out);

/* LZ4Ada.Update, Octets form (lz4ada.adb:383-418).  buf is the caller's
 * 0-based Buffer; first/last are inclusive indices (first=1,last=0: none). */
int oracle_update(oracle_ctx *ctx, const uint8_t *input, int64_t len,
                  int64_t *num_consumed, uint8_t *buf, int64_t buflen,
                  int64_t *first, int64_t *last);

/* LZ4Ada.Is_End_Of_Frame (lz4ada.adb:906-915). */
int oracle_is_end_of_frame(const oracle_ctx *ctx);

/* Exception name ("LZ4ADA.DATA_CORRUPTION") and message of the last error. */
const char *oracle_error_name(int status);
const char *oracle_last_error(const oracle_ctx *ctx);
void oracle_free(oracle_ctx *ctx);

/* XXHash32 package (lz4ada.adb:923-1026). */
typedef struct {
	uint32_t state[4];
	uint8_t buffer[16];
	int32_t buffer_size;
	uint64_t total_length;
} oracle_xxh32;
void oracle_xxh32_init(oracle_xxh32 *h, uint32_t seed); /* seed ignored (Q1) */
void oracle_xxh32_reset(oracle_xxh32 *h, uint32_t seed);
void oracle_xxh32_update(oracle_xxh32 *h, const uint8_t *data, int64_t len);
uint32_t oracle_xxh32_final(const oracle_xxh32 *h);
uint32_t oracle_xxh32_hash(const uint8_t *data, int64_t len);

/*
 * Whole-stream convenience used by tests and the CPU baseline: runs the
 * reference test harness loop (lz4test.adb:32-83) -- Init(reservation) then
 * Update with `chunk`-byte reads until the input is exhausted -- and appends
 * every produced output slice to out.  Returns a status; *out_len gets the
 * produced length, *eof the final Is_End_Of_Frame.  errbuf gets the message.
 */
int oracle_decode_stream(const uint8_t *input, int64_t len, int64_t chunk,
                         int reservation, uint8_t *out, int64_t out_cap,
                         int64_t *out_len, int *eof, char *errbuf, size_t errcap);

/*
 * The reference error-test harness (lz4test.adb:280-308):
 * Init_With_Header(Single_Frame) then Update over the rest until an
 * exception.  Returns the status of the raised exception (OR_OK if none).
 */
int oracle_error_harness(const uint8_t *input, int64_t len, char *errbuf,
                         size_t errcap);

/*
 * The reference CLI loop (tool_unlz4ada/unlz4ada.adb:63-105): one
 * Init_With_Header(Single_Frame) context per frame, 4 KiB reads, output
 * appended.  Used for config C1 and as the 1-core CPU baseline.
 */
int oracle_unlz4ada(const uint8_t *input, int64_t len, uint8_t *out,
                    int64_t out_cap, int64_t *out_len, char *errbuf,
                    size_t errcap);

#ifdef __cplusplus
}
#endif
#endif
