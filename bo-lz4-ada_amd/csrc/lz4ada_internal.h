// lz4ada_internal.h -- types shared by the host units (lz4ada_host_common.h, lz4ada_facade.cpp, lz4ada_bulk.cpp, lz4ada_bulk_linked.cpp)
// and the gfx950 kernels (lz4ada_kernels.hip).  Not part of the public C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "lz4ada_hip.h"

namespace lz4ada {

// XXH32 primes (lz4ada.ads:323-328).
constexpr uint32_t P1 = 2654435761u;
constexpr uint32_t P2 = 2246822519u;
constexpr uint32_t P3 = 3266489917u;
constexpr uint32_t P4 = 668265263u;
constexpr uint32_t P5 = 374761393u;

constexpr int64_t HISTORY_SIZE = 65536;  // lz4ada.ads:350
constexpr int64_t BLOCK_SIZE_BYTES = 4;  // lz4ada.ads:351

// Linked frames (lz4ada_linked.hip): every block slot is preceded by this
// many readable history bytes (the largest LZ4 offset).
constexpr int32_t LINK_HIST = 65535;
// Quirk D1: the reference's 8-byte wild copy (lz4ada.adb:811-817) may
// clobber history bytes [Output_Pos + 1, Output_Pos + 7] before a match
// reads them; that needs Output_Pos_History in [65536, 65542] and an offset
// >= Output_Pos_History - 7 >= D1_OFF.  The decoders flag every block with
// such a match reaching before its start (status aux bit AUX_D1_RISK on a
// DS_OK block) and the host sends those frames to the exact path.
constexpr int32_t D1_OFF = int32_t(HISTORY_SIZE) - 7;
constexpr int32_t AUX_D1_RISK = 1;
// Quirk D1 in the linked bulk path, emulated (round 6): the host predicts
// each block's round state from the slot sizes (every block full) and
// passes it in the descriptor's flags -- BLOCK_D1_ROUND: the block's round
// follows one that ended at Output_Pos_History = 65536 + the 3 bits at
// BLOCK_D1_OPH_SHIFT; bits from BLOCK_N1_SHIFT: Output_Pos at the block's
// start (its place in the round).  The index decoder then writes a D1
// match's first bytes as the reference's wild literal copy leaves them
// (lz4ada.adb:811-817, 862-879; the lone decoder's k_lone_words does the
// same); its status carries AUX_D1_EMU (decoded under a prediction), and
// the host accepts such a block only if the real round state equals the
// prediction.  (Bits 0-1 are the public flags.)
constexpr uint32_t BLOCK_D1_ROUND = 8u;
constexpr int BLOCK_D1_OPH_SHIFT = 4;
constexpr int BLOCK_N1_SHIFT = 16;
constexpr int32_t AUX_D1_EMU = 4;
// the linked path's literal-zero decode (k_decode_idx_zl): a match reads
// history positions below 256, whose high byte is 0 like a literal's
constexpr int32_t AUX_DEEP_HIST = 2;

// Device status codes written by the decode kernels (per block).
enum DevStatus : int32_t {
	DS_OK = 0,
	DS_OFFSET0 = 1,        // lz4ada.adb:769-772
	DS_ML_AFTER_LIT = 2,   // lz4ada.adb:752-762 (aux = Match_Length nibble)
	DS_LIT_OVERRUN = 3,    // D3
	DS_TRUNCATED = 4,      // D4
	DS_OUT_OVERFLOW = 5,   // D5 (bulk: block_max slot; serial: Buffer)
	DS_PRE_BLOCK_REF = 6,  // back-reference before the block start (bulk)
	DS_BACKREF = 7,        // lz4ada.adb:867-874 (detail = H_Offset)
	DS_CONTENT_SIZE = 8,   // lz4ada.adb:830-835
	DS_INTERNAL = 9,       // decoder invariant broken (never expected)
	DS_RETRY = 10,         // a fast decoder declined the block: k_decode_pc (or the exact path) redoes it
	DS_SPARSE = 11,        // pass 1 declined a literal-heavy block: k_decode_sparse takes it
	                       // (k_decode_pc, retry_only, takes it like DS_RETRY)
	DS_SKIP = 12,          // not part of this launch: every decoder leaves the block alone
};

// State of the serial reference-exact block kernel (emulates one
// Decode_Full_Block_With_Trailer step on a device mirror of Buffer).
struct SerialState {
	int64_t output_pos;          // Ctx.Output_Pos
	int64_t output_pos_history;  // Ctx.Output_Pos_History
	int64_t first, last;         // Output_First / Output_Last
	uint64_t size_remaining;     // Ctx.M.Size_Remaining
	int32_t has_content_size;
	int32_t code;   // DevStatus
	int32_t aux;
	int32_t pad;
	int64_t detail;
};

// ---- launchers (lz4ada_kernels.hip) ----
// All launch on `stream` and never synchronise.

// Bulk independent-block decoders (LZ4ADA_DECODE_* in lz4ada_hip.h).
enum DecVariant : int { DEC_PC = 0, DEC_IDX = 3, DEC_IDX_ALONE = 4,
                        DEC_IDX_LINKED = 5, DEC_IDX_SPARSE = 6,
                        // the fused index decoder alone with one / two waves per block
                        DEC_IDX1_ALONE = 7, DEC_IDX2_ALONE = 8,
                        // the pipelined two-wave decoder (k_decode_pp2) alone
                        DEC_PP2_ALONE = 9,
                        // k_index then k_decode_idx's pass 2, two launches (per-pass counters)
                        DEC_IDX_SPLIT = 10 };
int idx_fused_mode(uint32_t nblocks);  // 3: k_decode_idx, 5: k_decode_pp2 (4, round 4's k_decode_idx2, is retired) (lz4ada_idx.hip)
const char* idx_fused_kernel_name(uint32_t nblocks);  // the kernel idx_fused_mode picks

hipError_t launch_decode_variant(const uint8_t* d_frame, uint64_t frame_len,
                                 const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                 uint8_t* d_out, lz4ada_block_status* d_status, int variant,
                                 hipStream_t stream);

// The default decoder: the index-driven decoder, then the literal-heavy and
// two-wave decoders for the blocks it declines; LZ4ADA_DECODER=pc / wg
// select the others.
hipError_t launch_decode_blocks(const uint8_t* d_frame, uint64_t frame_len,
                                const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                uint8_t* d_out, lz4ada_block_status* d_status,
                                hipStream_t stream);

// Index-driven decoder alone (lz4ada_idx.hip): k_index + k_decode_idx;
// declined blocks keep status DS_RETRY and are not decoded.  linked: the
// blocks of one linked frame (slots contiguous), decoded in order with the
// earlier output as history; from the first declined or short block on,
// every block is left DS_RETRY.
hipError_t launch_decode_idx(const uint8_t* d_frame, uint64_t frame_len,
                             const lz4ada_block_desc* d_desc, uint32_t nblocks, uint8_t* d_out,
                             lz4ada_block_status* d_status, hipStream_t stream, int linked = 0);

// Two-wave decoder alone (k_decode_pc).  retry_only: only blocks whose
// status is DS_RETRY.  hist: output bytes readable right before every slot
// (0 independent; LINK_HIST in the linked-frame layout).
hipError_t launch_decode_pc(const uint8_t* d_frame, uint64_t frame_len,
                            const lz4ada_block_desc* d_desc, uint32_t nblocks, uint8_t* d_out,
                            lz4ada_block_status* d_status, int retry_only, int32_t hist,
                            hipStream_t stream);

// Pass 1 of the index-driven decoder alone: the sequence-index table of
// every block (index_table_bytes() of device memory at d_tab); declined
// blocks get status DS_RETRY.
size_t index_table_bytes(uint64_t frame_len, uint32_t nblocks);
hipError_t launch_index(const uint8_t* d_frame, uint64_t frame_len, const lz4ada_block_desc* d_desc,
                        uint32_t nblocks, uint8_t* d_tab, lz4ada_block_status* d_status,
                        hipStream_t stream);
// Pass 2 over a table from launch_index.  mode 0: independent blocks; 1:
// the serial linked decoder (one workgroup, blocks in order); 2: every
// block at once with LINK_HIST readable history bytes before its slot; 3:
// independent blocks, each wave running pass 1 of its block first (d_tab
// is written: no launch_index needed).
hipError_t launch_decode_idx_tab(const uint8_t* d_frame, uint64_t frame_len,
                                 const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                 const uint8_t* d_tab, uint8_t* d_out,
                                 lz4ada_block_status* d_status, int mode, hipStream_t stream);

// Literal-heavy blocks pass 1 declined (status DS_SPARSE; lz4ada_sparse.hip):
// decoded straight to HBM, one wave per block; anything unusual leaves the
// block DS_RETRY for k_decode_pc.
hipError_t launch_decode_sparse(const uint8_t* d_frame, uint64_t frame_len,
                                const lz4ada_block_desc* d_desc, uint32_t nblocks, uint8_t* d_out,
                                lz4ada_block_status* d_status, hipStream_t stream);

// Per-block XXH32 of the compressed payloads (block checksums).
hipError_t launch_block_checksums(const uint8_t* d_frame,
                                  const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                  lz4ada_block_status* d_status, hipStream_t stream);

// Block checksums and the default decoder together: the checksum kernel
// (latency-bound, no LDS) runs on a side stream beside pass 1 of the
// index-driven decoder, fork and join by events; `stream` sees both done.
hipError_t launch_decode_checked(const uint8_t* d_frame, uint64_t frame_len,
                                 const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                 uint8_t* d_out, lz4ada_block_status* d_status,
                                 hipStream_t stream);

// Per-block XXH32 of decoded output slots (golden checks).
hipError_t launch_output_checksums(const uint8_t* d_out,
                                   const lz4ada_block_desc* d_desc, uint32_t nblocks,
                                   const lz4ada_block_status* d_status,
                                   uint32_t* d_hash, hipStream_t stream);

// Streaming XXH32 update of a device-resident state over device data.
// Also refreshes state->hash with the Final() value.
hipError_t launch_xxh32_update(lz4ada_xxh32_state* d_state, const uint8_t* d_data,
                               uint64_t len, hipStream_t stream);

// Reference-exact serial decode of one block into the Buffer mirror.
hipError_t launch_serial_block(uint8_t* d_buf, int64_t buflen, const uint8_t* d_blk,
                               int64_t raw_len, int64_t data_len, int compressed,
                               SerialState* d_state, hipStream_t stream);

// Linked frames, every block at once (lz4ada_linked.hip).  Slots of the
// three decode buffers are preceded by 64 KiB history regions.
hipError_t launch_link_fill(uint8_t* x, uint8_t* y, uint8_t* h, const lz4ada_block_desc* d_desc,
                            uint32_t nblocks, hipStream_t stream);
// The block checksums on this thread's side stream, forked from stream
// (they write only the statuses' cksum fields, so kernels on stream may
// fill the other fields meanwhile); join_block_checksums makes stream wait
// for them.
hipError_t launch_block_checksums_beside(const uint8_t* d_frame, const lz4ada_block_desc* d_desc,
                                        uint32_t nblocks, lz4ada_block_status* d_status, hipStream_t stream);
hipError_t join_block_checksums(hipStream_t stream);
// k_link_fill on the same side stream (after everything already on
// stream), so it runs beside k_index; join_link_fill makes stream wait for
// it (before the decodes that read the history regions).
hipError_t launch_link_fill_beside(uint8_t* x, uint8_t* y, uint8_t* h, const lz4ada_block_desc* d_desc,
                                   uint32_t nblocks, hipStream_t stream);
hipError_t join_link_fill(hipStream_t stream);
// The same side stream for any launch: side_fork gives it, ordered after
// everything already on stream; side_join makes stream wait for everything
// on it so far (the checksums included).
hipError_t side_fork(hipStream_t stream, hipStream_t* side);
hipError_t side_join(hipStream_t stream);
// Words from the planes: x (history k -> k & 255) and z (literals 0,
// history k -> k >> 8) for every block; d_three (nullable) gives a block's
// mode -- 1: y (~x) as well, 2: x, y and h (k >> 8) instead.
// Each pointer is stepped twice from its source's planes (d_tail: the
// tail_valid bytes before the batch, for sources there).  d_P gets a word
// for every quad with a byte still open and d_M a byte per position (0
// open, 1 final with no word, 2 final with its word) -- or, `full` (batches
// where many words stay open, whose rounds then read a source's word
// alone), every word and no d_M.
hipError_t launch_link_init(const uint8_t* x, const uint8_t* z, const uint8_t* y, const uint8_t* h,
                            const uint8_t* d_three, const lz4ada_block_desc* d_desc,
                            const lz4ada_block_status* d_st, const int64_t* d_A, uint32_t nblocks,
                            int64_t block_max, const uint8_t* d_tail, int64_t tail_valid, uint32_t* d_P,
                            uint8_t* d_F, uint8_t* d_M, uint8_t* d_act, bool full, hipStream_t stream);
// One pointer-jumping round; d_act_in (nullptr: every span) / d_act_out:
// a byte per span of positions, 1 while the span holds an unresolved word.
int64_t link_spans(int64_t n);
hipError_t launch_link_jump(uint32_t* d_P, const uint8_t* d_M, int64_t n, const uint8_t* d_tail,
                            int64_t tail_valid, uint8_t* d_F, const uint8_t* d_act_in, uint8_t* d_act_out,
                            uint32_t* d_ctr, bool full, hipStream_t stream);
hipError_t launch_link_tail(const uint8_t* d_F, int64_t n, const uint8_t* d_tail_old,
                            uint8_t* d_tail_new, hipStream_t stream);

// Gather variable-length slots into a contiguous buffer (short blocks).
// One block decoded by the whole GPU (lz4ada_lone.hip): d_st gets DS_OK and
// out_len, or DS_RETRY (the exact path then decides).  d_scratch holds
// lone_scratch_bytes(n, cap) bytes.  History (a linked frame's block): the
// n0 + n1 <= 65535 bytes before the block, h0 then h1 (device memory; the
// reference's Buffer keeps them in two places), readable by its matches;
// d1: 0; 1 -- a match reaching >= D1_OFF back before the block start
// declines it (quirk D1); or the round's Output_Pos_History (>= 65536) --
// the block follows a round that ended there, and quirk D1's overshoot
// bytes are emulated (lz4ada_lone.hip).  Without history such a match
// declines it.  At most LONE_MAX_IN compressed bytes: the chain step keeps
// every window's entry in one workgroup's registers (16 MiB of windows at
// every window size); larger blocks return hipErrorInvalidValue, and the
// facade sends them to the exact path instead (lone_plan).
constexpr int64_t LONE_MAX_IN = int64_t(16) << 20;
int64_t lone_scratch_bytes(int64_t n, int64_t cap);
hipError_t launch_decode_lone(const uint8_t* d_blk, int64_t n, uint8_t* d_out, int64_t cap,
                              lz4ada_block_status* d_st, void* d_scratch, int64_t scratch_bytes,
                              hipStream_t stream, const uint8_t* d_h0 = nullptr, int32_t n0 = 0,
                              const uint8_t* d_h1 = nullptr, int32_t n1 = 0, int d1 = 0);
// The same in two halves: the parse (steps 1-3: nothing written to d_out,
// the status set to DS_RETRY on a decline) and the emit (step 4: the bytes
// to d_out when the status is still OK).  A caller may check something on
// the host between them, e.g. the block checksum before d_out is touched.
// Zero-copy form (the streaming facade): d_blk may be pinned host memory
// that step 1 reads once and copies to d_copy (ncopy >= n bytes: the
// block's trailer too), which step 3 then reads; d_st may be pinned host
// memory; h_out, when not null, is pinned host memory that step 4 writes
// the bytes to as well -- no DMA copy on the block's critical path.
hipError_t launch_decode_lone_parse(const uint8_t* d_blk, int64_t n, int64_t cap,
                                    lz4ada_block_status* d_st, void* d_scratch, int64_t scratch_bytes,
                                    hipStream_t stream, const uint8_t* d_h0, int32_t n0,
                                    const uint8_t* d_h1, int32_t n1, int d1, uint8_t* d_copy = nullptr,
                                    int64_t ncopy = 0, bool fused = false);
// fused: a small block's chain step runs inside its windows launch, which
// needs the scratch's header zeroed once (lone_scratch_init) before the
// scratch's first fused use; every fused use leaves it zeroed again.
hipError_t lone_scratch_init(void* d_scratch, hipStream_t stream);
hipError_t launch_decode_lone_emit(int64_t n, uint8_t* d_out, int64_t cap, lz4ada_block_status* d_st,
                                   void* d_scratch, hipStream_t stream, int32_t H, uint8_t* h_out = nullptr);

// host side (lz4ada_bulk.cpp): the calling thread's message for
// lz4ada_thread_last_error() and its lz4ada_last_path() bits
void set_thread_error(const std::string& msg);
void set_last_path(int bits);

hipError_t launch_compact(const uint8_t* d_src, const lz4ada_block_desc* d_desc,
                          const uint64_t* d_dst_off, const lz4ada_block_status* d_status,
                          uint32_t nblocks, uint8_t* d_dst, hipStream_t stream);

}  // namespace lz4ada
