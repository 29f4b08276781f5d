/*
 * lz4ada_hip.h -- C-ABI of the MI355X-native LZ4Ada decompressor.
 *
 * Drop-in boundary for the reference's public Ada API (lib/lz4ada.ads):
 * every entry point below names the reference subprogram it replaces.  An
 * Ada caller binds them with pragma Import (bindings/ada/lz4ada.ads,
 * INTEGRATION.md); Python binds them with ctypes (bo-lz4-ada_amd/lz4ada.py).
 *
 * Plain pointers and sizes only.  Lengths are int64_t so that both the
 * Integer and the Stream_Element_Offset overloads map onto one entry point.
 * Status codes are 1:1 with the reference's exceptions (lz4ada.ads:133-162);
 * the exact Exception_Information message is available from
 * lz4ada_last_error() / lz4ada_thread_last_error().
 *
 * Block decode and block XXH32 run on the GPU (HIP kernels for gfx950).
 * Frame-header parsing, the Update state machine and the serial XXH32 chain
 * over host-resident bytes (content checksums, the XXHash32 API) are host
 * code.  There is no CPU fallback: without a usable GPU,
 * calls that would decode return LZ4ADA_DEVICE_ERROR.
 */
#ifndef LZ4ADA_HIP_H
#define LZ4ADA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LZ4ADA_HIP_ABI_VERSION 1

/* ---------------------------------------------------------------- enums */

/* Exceptions (lz4ada.ads:133-162). */
typedef enum {
	LZ4ADA_OK = 0,
	LZ4ADA_CHECKSUM_ERROR = 1,       /* LZ4Ada.Checksum_Error */
	LZ4ADA_DATA_CORRUPTION = 2,      /* LZ4Ada.Data_Corruption */
	LZ4ADA_NOT_SUPPORTED = 3,        /* LZ4Ada.Not_Supported */
	LZ4ADA_TOO_FEW_HEADER_BYTES = 4, /* LZ4Ada.Too_Few_Header_Bytes */
	LZ4ADA_TOO_LITTLE_MEMORY = 5,    /* LZ4Ada.Too_Little_Memory */
	LZ4ADA_ASSERTION_ERROR = 6,      /* Pre/Assert violated (API misuse) */
	LZ4ADA_CONSTRAINT_ERROR = 7,     /* library-internal check */
	LZ4ADA_DEVICE_ERROR = 8,         /* HIP error / no GPU (no reference twin) */
	LZ4ADA_EXACT_PATH = 9            /* device-only call: the frame needs lz4ada_decode_frame */
} lz4ada_status;

/* Flexible_Memory_Reservation (lz4ada.ads:79-106), same order. */
typedef enum {
	LZ4ADA_SZ_64_KIB = 0,
	LZ4ADA_SZ_256_KIB = 1,
	LZ4ADA_SZ_1_MIB = 2,
	LZ4ADA_SZ_4_MIB = 3,
	LZ4ADA_SZ_8_MIB = 4,
	LZ4ADA_USE_FIRST = 5,
	LZ4ADA_SINGLE_FRAME = 6,
	LZ4ADA_FOR_MODERN = LZ4ADA_SZ_4_MIB, /* lz4ada.ads:92 */
	LZ4ADA_FOR_LEGACY = LZ4ADA_SZ_8_MIB, /* lz4ada.ads:100 */
	LZ4ADA_FOR_ALL = LZ4ADA_SZ_8_MIB     /* lz4ada.ads:106 */
} lz4ada_reservation;

/* End_Of_Frame (lz4ada.ads:124). */
typedef enum { LZ4ADA_EOF_YES = 0, LZ4ADA_EOF_NO = 1, LZ4ADA_EOF_MAYBE = 2 } lz4ada_end_of_frame;

/* ------------------------------------------------- streaming decompressor */

/* Opaque Decompressor context (lz4ada.ads:126, 440-449).  Owns device
 * buffers (Buffer mirror holding the 64 KiB history, block staging, content
 * hash state); not copyable; one thread at a time. */
typedef struct lz4ada_decompressor lz4ada_decompressor;

/* LZ4Ada.Init (lz4ada.ads:189-191, 218-220; lz4ada.adb:48-63).
 * reservation: one of LZ4ADA_SZ_*. */
int lz4ada_init(int reservation, int64_t *min_buffer_size, lz4ada_decompressor **ctx);

/* LZ4Ada.Init_With_Header (lz4ada.ads:238-243; lz4ada.adb:79-125).
 * Requires len >= 7 (Pre).  On failure *ctx is NULL and the message is in
 * lz4ada_thread_last_error(). */
int lz4ada_init_with_header(const uint8_t *input, int64_t len, int reservation,
                            int64_t *num_consumed, int64_t *min_buffer_size,
                            lz4ada_decompressor **ctx);

/* LZ4Ada.Init_For_Block (lz4ada.ads:255-258; lz4ada.adb:127-147). */
int lz4ada_init_for_block(int64_t compressed_length, int reservation,
                          int64_t *min_buffer_size, lz4ada_decompressor **ctx);

/* LZ4Ada.Update (lz4ada.ads:211-216, 281-287; lz4ada.adb:383-418).
 * buffer is the caller-owned 0-based Buffer (length >= min_buffer_size);
 * it must not be modified between calls.  At most one block of output is
 * returned, as inclusive indices [*output_first, *output_last]
 * (first = 1, last = 0 when nothing was produced). */
int lz4ada_update(lz4ada_decompressor *ctx, const uint8_t *input, int64_t len,
                  int64_t *num_consumed, uint8_t *buffer, int64_t buffer_len,
                  int64_t *output_first, int64_t *output_last);

/* LZ4Ada.Is_End_Of_Frame (lz4ada.ads:303; lz4ada.adb:906-915). */
int lz4ada_is_end_of_frame(const lz4ada_decompressor *ctx);

/* Exception message of the last failed call on ctx, and the reference
 * exception name for a status ("LZ4ADA.DATA_CORRUPTION"). */
const char *lz4ada_last_error(const lz4ada_decompressor *ctx);
/* Blocks this context sent through the reference-exact single-lane path
 * (k_serial_block: errors, quirk D1, anything the GPU decoders decline);
 * every other block was decoded by the parallel GPU decoders.  Diagnostic,
 * no reference twin. */
int64_t lz4ada_exact_blocks(const lz4ada_decompressor *ctx);
const char *lz4ada_error_name(int status);
/* Message of the last failed context-less call on this thread. */
const char *lz4ada_thread_last_error(void);

void lz4ada_free(lz4ada_decompressor *ctx);

/* LZ4Ada.To_Hex (lz4ada.ads:306-307); writes 3 / 9 bytes incl. NUL. */
void lz4ada_to_hex8(uint8_t v, char out[3]);
void lz4ada_to_hex32(uint32_t v, char out[9]);

/* ---------------------------------------------------------------- XXHash32 */

/* LZ4Ada.XXHash32.Hasher (lz4ada.ads:335-343).  Plain struct so callers can
 * embed it.  Host bytes are hashed on the calling thread (the chain is one
 * serial dependency); device-resident bytes by the GPU kernel or
 * the D2H pipeline below, on the same state.  `hash` caches Final(). */
typedef struct {
	uint32_t state[4];
	uint8_t buffer[16];
	int32_t buffer_size;
	uint32_t hash;
	uint64_t total_length;
} lz4ada_xxh32_state;

/* XXHash32.Init (lz4ada.adb:925-930): Seed is ignored (quirk Q1). */
void lz4ada_xxh32_init(lz4ada_xxh32_state *h, uint32_t seed);
/* XXHash32.Reset (lz4ada.adb:932-940). */
void lz4ada_xxh32_reset(lz4ada_xxh32_state *h, uint32_t seed);
/* XXHash32.Update (lz4ada.adb:942-963) over host bytes (host chain, no
 * device round trip). */
int lz4ada_xxh32_update(lz4ada_xxh32_state *h, const uint8_t *data, int64_t len);
/* Same over device-resident bytes; stream is a hipStream_t (0 = default). */
int lz4ada_xxh32_update_device(lz4ada_xxh32_state *h, const void *d_data, int64_t len,
                               void *stream);
/* Content checksum pipeline: XXHash32.Update over
 * device-resident bytes copied to the host in 32 MiB chunks, each chunk
 * hashed on the calling host thread while the next one is in flight; the
 * bytes also land in host_out when it is not NULL.  The serial chain runs
 * ~5x faster on a host core than on one GPU wave. */
int lz4ada_content_xxh32_d2h(lz4ada_xxh32_state *h, const void *d_data, int64_t len,
                             uint8_t *host_out, void *stream);
/* XXHash32.Final (lz4ada.adb:993-1017). */
uint32_t lz4ada_xxh32_final(const lz4ada_xxh32_state *h);
/* XXHash32.Hash (lz4ada.adb:1019-1024), seed 0, host bytes. */
int lz4ada_xxh32_hash(const uint8_t *data, int64_t len, uint32_t *out);

/* ------------------------------------------------------- bulk frame decode */
/*
 * The hot path.  A whole LZ4 frame is indexed on the host (a serial walk of
 * the 4-byte block size words, lz4ada.adb:525-585) and every block is then
 * decoded by its own wavefront on the GPU, with block checksums
 * (lz4ada.adb:698-707) verified on the GPU.  Output lands in per-block
 * slots of block_max bytes (desc.out_off), contiguous whenever every
 * non-last block is full.  lz4ada_decode_frame() decodes independent
 * blocks this way; linked frames (and independent ones whose blocks read
 * earlier blocks, quirk D2) decode every block at once against a synthetic
 * history that the GPU then resolves (quirk D1
 * emulated there, section 6).  A non-zero block status, a failed checksum,
 * a D1 read the GPU does not emulate or a reference before the frame start
 * sends the frame (from that block on) down the reference-exact serial
 * path, which reproduces the reference's output and exception.
 */

typedef struct {
	uint64_t in_off;  /* payload offset inside the frame */
	uint32_t in_len;  /* payload bytes (size word & 0x7FFFFFF) */
	uint32_t flags;   /* LZ4ADA_BLOCK_* */
	uint64_t out_off; /* output slot offset */
	uint32_t out_cap; /* slot capacity (block_max) */
	uint32_t cksum;   /* declared block checksum (if present) */
} lz4ada_block_desc;

#define LZ4ADA_BLOCK_STORED 1u    /* size word bit 31 set */
#define LZ4ADA_BLOCK_HAS_CKSUM 2u /* FLG.B.Checksum */

typedef struct {
	int32_t code;        /* 0 = ok; else device status */
	int32_t aux;
	int64_t detail;
	int64_t err_out_pos; /* block-relative output count at the error */
	uint32_t out_len;    /* decoded bytes */
	uint32_t cksum;      /* XXH32 of the compressed payload */
} lz4ada_block_status;

#define LZ4ADA_FORMAT_MODERN 1
#define LZ4ADA_FORMAT_LEGACY 2
#define LZ4ADA_FORMAT_SKIPPABLE 3

typedef struct {
	int32_t format;           /* LZ4ADA_FORMAT_* */
	uint8_t flg, bd;          /* frame descriptor bytes (modern) */
	uint8_t block_checksum;   /* FLG bit 4 */
	uint8_t content_checksum; /* FLG bit 2 */
	uint8_t has_content_size; /* FLG bit 3 */
	uint8_t independent;      /* FLG bit 5 (B.Indep; ignored by the reference) */
	uint8_t pad[2];
	int64_t block_max;        /* BD block maximum (8 MiB for legacy) */
	int64_t header_len;
	int64_t nblocks;
	int64_t frame_len;        /* bytes of this frame incl. end mark + checksum */
	uint64_t content_size;
	uint32_t content_checksum_declared;
	uint32_t pad2;
} lz4ada_frame_info;

/* Index one frame starting at frame[0].  descs may be NULL to count blocks
 * (then info->nblocks is set and LZ4ADA_OK returned).  Slots are laid out
 * at i * block_max.  Errors carry the reference's header messages. */
int lz4ada_frame_index(const uint8_t *frame, int64_t len, lz4ada_frame_info *info,
                       lz4ada_block_desc *descs, int64_t desc_cap);

/* Launch the per-block kernels over a device-resident frame: block XXH32
 * (when LZ4ADA_BLOCK_HAS_CKSUM) and decode into d_out.  Asynchronous on
 * `stream` (hipStream_t).  d_frame must stay readable up to frame_len.
 * The checksums run on a library-owned side stream beside the decoder's
 * first pass (forked from and joined back into `stream` by events; set
 * LZ4ADA_NO_OVERLAP to serialise them). */
int lz4ada_decode_blocks_device(const void *d_frame, uint64_t frame_len,
                                const lz4ada_block_desc *d_descs, int64_t nblocks,
                                void *d_out, lz4ada_block_status *d_status,
                                void *stream);

/* Decode-only / checksum-only halves of the above (for profiling). */
int lz4ada_launch_decode(const void *d_frame, uint64_t frame_len,
                         const lz4ada_block_desc *d_descs, int64_t nblocks, void *d_out,
                         lz4ada_block_status *d_status, void *stream);
/* Decoder variants of the bulk path: the two-wave
 * producer/consumer decoder (1, the round-1 one-wave decoder, and 2, the
 * workgroup decoder, are retired: LZ4ADA_DEVICE_ERROR). */
#define LZ4ADA_DECODE_PC 0
/* Index-driven two-pass decoder (k_index + k_decode_idx, lz4ada_idx.hip),
 * then the two-wave decoder for the blocks it declines; _ALONE skips that
 * second step (declined blocks keep status code 10). */
#define LZ4ADA_DECODE_IDX 3
#define LZ4ADA_DECODE_IDX_ALONE 4
/* The blocks of one LINKED frame (slots contiguous, block_max >= 256 KiB):
 * sequence index of every block at once, then the blocks in order with the
 * earlier output as history; from the first declined or short block on,
 * every block is left with status code 10 (the exact path takes over). */
#define LZ4ADA_DECODE_IDX_LINKED 5
/* The index-driven decoder, then the literal-heavy decoder (k_decode_sparse)
 * for the blocks pass 1 declines as sparse; no two-wave pass: blocks either
 * declines keep status code 10 (retry). */
#define LZ4ADA_DECODE_IDX_SPARSE 6
/* The fused index decoder alone with one wave per block (k_decode_idx) or
 * two pipelining batches (k_decode_pp2; _IDX2_ALONE named round 4's
 * k_decode_idx2, retired in round 6, and now runs k_decode_pp2); declined
 * blocks keep status code 10.  The default of LZ4ADA_DECODE_IDX / _ALONE
 * picks by launch size: k_decode_pp2 for at most 4x the CU count in
 * blocks, k_decode_idx above; LZ4ADA_IDX_WAVES=1 / p forces k_decode_idx /
 * k_decode_pp2 (lz4ada_bulk_decoder_kernel() names the one a launch uses). */
#define LZ4ADA_DECODE_IDX1_ALONE 7
#define LZ4ADA_DECODE_IDX2_ALONE 8
/* The pipelined two-wave decoder (k_decode_pp2: two waves per block taking
 * alternate batches) alone; declined blocks keep status code 10 / 11. */
#define LZ4ADA_DECODE_PP2_ALONE 9
/* The index decoder's two passes as two launches (k_index, then
 * k_decode_idx's pass 2): per-pass timing and counters. */
#define LZ4ADA_DECODE_IDX_SPLIT 10

int lz4ada_launch_decode_variant(const void *d_frame, uint64_t frame_len,
                                 const lz4ada_block_desc *d_descs, int64_t nblocks, void *d_out,
                                 lz4ada_block_status *d_status, int variant, void *stream);
/* The name of the kernel the fused bulk decode (LZ4ADA_DECODE_IDX, the
 * product call lz4ada_decode_blocks_device) launches for nblocks blocks --
 * it depends on how the block count fills the chip (for benches and
 * profiles; a static string). */
const char *lz4ada_bulk_decoder_kernel(int64_t nblocks);

/* One block (payload d_blk, n bytes, no history) decoded by the whole GPU
 * (lz4ada_lone.hip: every byte position parsed, the sequence chain found by
 * pointer jumping, copies resolved by pointer jumping over one word per
 * output byte) into d_out (cap bytes); *d_status gets code 0 and out_len, or
 * 10 (declined: malformed data, a reference before the block start, an
 * output over cap -- the exact path gives the reference's result).  The
 * streaming facade's decoder for lone blocks.  d_scratch: device memory of
 * lz4ada_lone_scratch_bytes(n, cap) bytes.  Asynchronous on stream. */
int64_t lz4ada_lone_scratch_bytes(int64_t n, int64_t cap);
int lz4ada_launch_decode_lone(const void *d_blk, int64_t n, void *d_out, int64_t cap,
                              lz4ada_block_status *d_status, void *d_scratch,
                              int64_t scratch_bytes, void *stream);

int lz4ada_launch_block_checksums(const void *d_frame, const lz4ada_block_desc *d_descs,
                                  int64_t nblocks, lz4ada_block_status *d_status,
                                  void *stream);

/* XXH32 of each decoded slot (golden checks). */
int lz4ada_output_checksums_device(const void *d_out, const lz4ada_block_desc *d_descs,
                                   const lz4ada_block_status *d_status, int64_t nblocks,
                                   uint32_t *d_hash, void *stream);

/* Decode one complete single frame (Init_With_Header(Single_Frame) + Update
 * semantics, as tool_unlz4ada does per frame) from host memory into host
 * memory.  *frame_consumed = bytes of this frame; *out_len = decoded bytes.
 * On failure the reference's exception message is in
 * lz4ada_thread_last_error().  out_cap must be >= the decoded size. */
int lz4ada_decode_frame(const uint8_t *frame, int64_t len, uint8_t *out, int64_t out_cap,
                        int64_t *out_len, int64_t *frame_consumed);

/* Decode every frame of a concatenated stream (skippable frames skipped). */
int lz4ada_decode_stream(const uint8_t *input, int64_t len, uint8_t *out, int64_t out_cap,
                         int64_t *out_len);

/* The same two calls into a buffer the library allocates and grows, so no
 * bound is needed up front (a stream that fails to index part-way still
 * raises the reference's own exception); release it with
 * lz4ada_buffer_free().  On failure *out is NULL. */
int lz4ada_decode_frame_alloc(const uint8_t *frame, int64_t len, uint8_t **out, int64_t *out_len,
                              int64_t *frame_consumed);
int lz4ada_decode_stream_alloc(const uint8_t *input, int64_t len, uint8_t **out,
                               int64_t *out_len);
void lz4ada_buffer_free(uint8_t *p);

/* lz4ada_decode_frame_alloc, except that on failure *out / *out_len hold
 * what the reference would have output before raising: every block before
 * the failing one, each returned by its own Update call (lz4ada.adb:383-418,
 * 661-714; tool_unlz4ada/unlz4ada.adb:41 writes each at once).  The exact
 * path resumes at (or just before) the failing block with the stream state
 * replayed from the decoded lengths, so the error comes in about the time
 * the bulk path needs, not after a redo of the frame.  Free *out with
 * lz4ada_buffer_free() in both cases. */
int lz4ada_decode_frame_partial(const uint8_t *frame, int64_t len, uint8_t **out,
                                int64_t *out_len, int64_t *frame_consumed);

/* The linked-frame bulk path over a device-resident frame (BASELINE
 * configs[4]): every block at once against a synthetic history, resolved
 * on the GPU, into contiguous device output d_out
 * (out_cap bytes); descs are the HOST descriptors from lz4ada_frame_index.
 * Synchronous on `stream`.  Returns LZ4ADA_EXACT_PATH when the reference
 * would raise or diverge in a way the GPU does not reproduce (block error,
 * checksum mismatch, a quirk-D1 read it does not emulate, a reference
 * before the frame start) -- lz4ada_decode_frame() then gives
 * the reference's result.  The content checksum is the caller's. */
int lz4ada_decode_linked_device(const void *d_frame, uint64_t frame_len,
                                const lz4ada_block_desc *descs, int64_t nblocks, int64_t block_max,
                                void *d_out, int64_t out_cap, int64_t *out_len, void *stream);

/* Paths the last lz4ada_decode_* call on this thread took (bit mask):
 * independent blocks in bulk, linked blocks in bulk (synthetic history
 * resolved on the GPU), the reference-exact serial path. */
#define LZ4ADA_PATH_INDEPENDENT 1
#define LZ4ADA_PATH_LINKED 2
#define LZ4ADA_PATH_EXACT 4
#define LZ4ADA_PATH_MULTI 8 /* lz4ada_decode_frame_multi* took the call */
int lz4ada_last_path(void);

/* The bulk path keeps its large device scratch (output slots, linked-frame
 * decode copies) per thread between calls; this frees the calling thread's. */
void lz4ada_release_device_cache(void);

/* Upper bound of the decoded size of a stream (sum of block maxima); -1 if
 * some frame does not index (then use the _alloc calls). */
int64_t lz4ada_decoded_bound(const uint8_t *input, int64_t len);

/* ------------------------------------------------- multi-GPU bulk decode */
/*
 * One frame over n_gpus devices from ONE process (no
 * reference twin -- it replaces the caller's whole Update loop
 * (lz4ada.ads:281-287, tool_unlz4ada/unlz4ada.adb:84-103) for a frame, like
 * lz4ada_decode_frame, and spreads it over GPUs).  An independent-block
 * modern frame is split into contiguous block ranges balanced by compressed
 * bytes (lz4ada_plan_shards); one host worker thread per device copies its
 * range in and decodes it; RCCL (ncclCommInitAll over the devices) carries
 * one all-reduce of the block verdict and the per-device output sizes, and
 * for the _gather variant the bytes to the first device.  The content
 * checksum is one XXH32 chain in frame order.  Linked, legacy and skippable
 * frames, and any frame the bulk path would not take (block error, checksum
 * mismatch, cross-block references, failed frame checks), are decoded by
 * lz4ada_decode_frame on the first device, which gives the reference's
 * output or exception.  devices: n_gpus HIP ordinals, or NULL for
 * 0 .. n_gpus-1.  Calls are serialised (the communicators are shared).
 */
int lz4ada_decode_frame_multi(const uint8_t *frame, int64_t len, int n_gpus, const int *devices,
                              uint8_t *out, int64_t out_cap, int64_t *out_len,
                              int64_t *frame_consumed);
/* The same with the output gathered into d_out on the first device
 * (out_cap bytes, device memory) instead of host memory. */
int lz4ada_decode_frame_multi_gather(const uint8_t *frame, int64_t len, int n_gpus,
                                     const int *devices, void *d_out, int64_t out_cap,
                                     int64_t *out_len, int64_t *frame_consumed);
/* The block split of the above (and of bo-lz4-ada_amd/shard.py): rank r
 * decodes blocks [bounds[r], bounds[r+1]) (bounds has n_gpus + 1 entries);
 * the blocks whose compressed-prefix midpoint falls in
 * [r, r+1) * total / n_gpus.  Host-only. */
int lz4ada_plan_shards(const lz4ada_block_desc *descs, int64_t nblocks, int n_gpus,
                       int64_t *bounds);
/* Device allocations the multi-GPU workers made so far for HIP ordinal
 * `device` (each worker keeps its buffers and pinned staging between calls:
 * a repeated call of the same size adds none); -1 if it has no worker yet. */
int64_t lz4ada_multi_device_allocs(int device);
/* The RCCL version the process actually bound (ncclGetVersion, e.g. 22606
 * for 2.26.6): in a process that loaded another librccl.so.1 first (a torch
 * job loads its bundled one), that library serves this one's calls too;
 * a plain C / Ada program gets /opt/rocm/lib's (the library's RUNPATH). */
int lz4ada_rccl_version(void);

/* ------------------------------------------------------------------ misc */

/* 0 when a HIP device is usable, else LZ4ADA_DEVICE_ERROR (message in
 * lz4ada_thread_last_error()). */
int lz4ada_device_check(void);
int lz4ada_abi_version(void);

/*
 * Deterministic synthetic LZ4 block generator for benches and tests
 * (SURVEY §8d): emits one valid compressed block whose decoded size is
 * exactly raw_len.  kind: 0 dense (~5 B/sequence), 1 mixed (~32 B/seq,
 * ratio ~2), 2 rle (zeros, offset 1), 3 literal-heavy, 4 chain (matches
 * only, offsets <= 16), 5 mixed with offsets <= 65528 (no match can meet
 * quirk D1 in a linked frame).  Writes the decoded
 * bytes to raw (raw_len bytes) and the block payload to comp; returns the
 * payload length, or -1 if comp_cap is too small.
 */
int64_t lz4ada_gen_block(int kind, uint64_t seed, uint8_t *raw, int64_t raw_len,
                         uint8_t *comp, int64_t comp_cap);
/* The same for one block of a linked frame: buf holds `hist` bytes of the
 * frame's earlier output, then room for raw_len decoded bytes (written at
 * buf + hist); offsets may reach back into the history (up to 65535). */
int64_t lz4ada_gen_block_linked(int kind, uint64_t seed, uint8_t *buf, int64_t hist,
                                int64_t raw_len, uint8_t *comp, int64_t comp_cap);

#ifdef __cplusplus
}
#endif
#endif
