/*
 * lz4ada_oracle.c -- CPU restatement of /root/reference/lib/lz4ada.adb.
 *
 * TEST INFRASTRUCTURE ONLY (see lz4ada_oracle.h).  Never part of the
 * product.  Each function names the reference lines it restates.  Ada
 * exceptions are modelled with setjmp/longjmp: state changes made before a
 * raise persist, exactly as with the reference's in-out limited record.
 *
 * Deliberate, documented divergences (DESIGN.md "Reference quirks"): where the
 * reference has undefined behaviour (checks suppressed, lz4ada.adb:798-801)
 * or raises a non-library Constraint_Error, the oracle raises
 * DATA_CORRUPTION with its own message:
 *   D3  literal run past the block end with Match_Length = 0
 *   D4  length-extension / offset bytes missing at the block end
 *   D5  decoded bytes would not fit the caller's Buffer
 * Everything else -- including the D1 wild-copy clobber of linked-block
 * history -- is reproduced bit for bit.
 */
#include "lz4ada_oracle.h"

#include <setjmp.h>
#include <stdarg.h>
#include <stdbool.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- consts */
/* lz4ada.ads:348-353 */
#define MAGIC_MODERN 0x184d2204u
#define MAGIC_LEGACY 0x184c2102u
#define MAGIC_SKIP_LO 0x184d2a50u
#define MAGIC_SKIP_HI 0x184d2a5fu
#define HISTORY_SIZE 65536
#define BLOCK_SIZE_BYTES 4

/* lz4ada.ads:323-328 */
#define P1 2654435761u
#define P2 2246822519u
#define P3 3266489917u
#define P4 668265263u
#define P5 374761393u

enum fmt { F_TBD, F_LEGACY, F_MODERN, F_BLOCK, F_SKIPPABLE };           /* ads:355 */
enum hps { NEED_MAGIC, NEED_MODERN, NEED_FLAGS, NEED_SKIP_LEN, HDR_DONE }; /* ads:356 */

/* Decompressor_Meta (lz4ada.ads:359-370) */
typedef struct {
	int is_format;
	int header_parsing;
	int memory_reservation;
	int content_checksum_length;
	int block_checksum_length;
	int status_eof;
	int64_t input_buffer_filled;
	bool is_compressed;
	bool has_content_size;
	uint64_t size_remaining;
} meta_t;

/* Decompressor (lz4ada.ads:440-449) */
struct oracle_ctx {
	meta_t m;
	bool is_at_end_mark;
	uint8_t *input_buffer;
	int64_t input_buffer_len; /* In_Last + 1 */
	int64_t output_pos;
	int64_t output_pos_history;
	int64_t input_length;
	oracle_xxh32 hash_all_data;
	/* error state */
	int err_code;
	char err[512];
};

/* ------------------------------------------------------------ exceptions */
static const char *const ERROR_NAMES[] = {
	"",
	"LZ4ADA.CHECKSUM_ERROR",
	"LZ4ADA.DATA_CORRUPTION",
	"LZ4ADA.NOT_SUPPORTED",
	"LZ4ADA.TOO_FEW_HEADER_BYTES",
	"LZ4ADA.TOO_LITTLE_MEMORY",
	"ADA.ASSERTIONS.ASSERTION_ERROR",
	"CONSTRAINT_ERROR",
};

const char *oracle_error_name(int status)
{
	if (status < 0 || status > OR_CONSTRAINT_ERROR)
		return "UNKNOWN";
	return ERROR_NAMES[status];
}

typedef struct {
	jmp_buf jb;
	int code;
	char msg[512];
} raise_t;

__attribute__((noreturn, format(printf, 3, 4))) static void
raise_err(raise_t *r, int code, const char *fmt, ...)
{
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(r->msg, sizeof(r->msg), fmt, ap);
	va_end(ap);
	r->code = code;
	longjmp(r->jb, 1);
}

/* Ada 'Image of a non-negative integer has a leading blank, negative a '-'. */
static const char *img(char *b, int64_t v)
{
	if (v >= 0)
		sprintf(b, " %lld", (long long)v);
	else
		sprintf(b, "%lld", (long long)v);
	return b;
}
static const char *img_u(char *b, uint64_t v)
{
	sprintf(b, " %llu", (unsigned long long)v);
	return b;
}

/* Memory_Reservation'Image (upper case, lz4ada.ads:79-80). */
static const char *RES_IMAGE[] = { "SZ_64_KIB", "SZ_256_KIB", "SZ_1_MIB",
	                           "SZ_4_MIB", "SZ_8_MIB", "USE_FIRST",
	                           "SINGLE_FRAME" };

static uint32_t load32(const uint8_t *p)
{
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
	       ((uint32_t)p[3] << 24);
}
static uint64_t load64(const uint8_t *p)
{
	return (uint64_t)load32(p) | ((uint64_t)load32(p + 4) << 32);
}

/* ---------------------------------------------------------------- XXH32 */
static inline uint32_t rotl32(uint32_t x, int r)
{
	return (x << r) | (x >> (32 - r));
}

/* Reset (lz4ada.adb:932-940) */
void oracle_xxh32_reset(oracle_xxh32 *h, uint32_t seed)
{
	h->state[0] = seed + P1 + P2;
	h->state[1] = seed + P2;
	h->state[2] = seed;
	h->state[3] = seed - P1;
	h->buffer_size = 0;
	h->total_length = 0;
}

/* Init ignores its Seed argument (lz4ada.adb:925-930, quirk Q1). */
void oracle_xxh32_init(oracle_xxh32 *h, uint32_t seed)
{
	(void)seed;
	oracle_xxh32_reset(h, 0);
}

/* Process (lz4ada.adb:979-991) */
static void xxh_process(oracle_xxh32 *h, const uint8_t *d)
{
	for (int i = 0; i < 4; i++)
		h->state[i] = rotl32(h->state[i] + load32(d + 4 * i) * P2, 13) * P1;
}

/* Update1 (lz4ada.adb:965-977) */
static bool xxh_update1(oracle_xxh32 *h, uint8_t b)
{
	h->buffer[h->buffer_size] = b;
	h->total_length += 1;
	h->buffer_size += 1;
	if (h->buffer_size == 16) {
		h->buffer_size = 0;
		xxh_process(h, h->buffer);
		return true;
	}
	return false;
}

/* Update (lz4ada.adb:942-963) */
void oracle_xxh32_update(oracle_xxh32 *h, const uint8_t *data, int64_t len)
{
	bool fast = (h->buffer_size == 0);
	int64_t start = 0;
	while (start < len) {
		int64_t n = len - start < 16 ? len - start : 16;
		if (n == 16 && fast) {
			h->total_length += 16;
			xxh_process(h, data + start);
			start += 16;
		} else {
			fast = xxh_update1(h, data[start]);
			start += 1;
		}
	}
}

/* Final (lz4ada.adb:993-1017) */
uint32_t oracle_xxh32_final(const oracle_xxh32 *h)
{
	uint32_t ret = (uint32_t)(h->total_length & 0xffffffffu);
	if (h->total_length >= 16)
		ret += rotl32(h->state[0], 1) + rotl32(h->state[1], 7) +
		       rotl32(h->state[2], 12) + rotl32(h->state[3], 18);
	else
		ret += h->state[2] + P5;
	int d = 0;
	while (d + 3 < h->buffer_size) {
		ret = rotl32(ret + load32(h->buffer + d) * P3, 17) * P4;
		d += 4;
	}
	while (d < h->buffer_size) {
		ret = rotl32(ret + (uint32_t)h->buffer[d] * P5, 11) * P1;
		d += 1;
	}
	ret = (ret ^ (ret >> 15)) * P2;
	ret = (ret ^ (ret >> 13)) * P3;
	return ret ^ (ret >> 16);
}

/* Hash (lz4ada.adb:1019-1024) */
uint32_t oracle_xxh32_hash(const uint8_t *data, int64_t len)
{
	oracle_xxh32 h;
	oracle_xxh32_init(&h, 0);
	oracle_xxh32_update(&h, data, len);
	return oracle_xxh32_final(&h);
}

/* ------------------------------------------------------------ reservation */
/* Get_Block_Size (lz4ada.adb:65-77) */
static int64_t get_block_size(int r)
{
	static const int64_t lut[] = { 64 * 1024, 256 * 1024, 1024 * 1024,
		                       4 * 1024 * 1024, 8 * 1024 * 1024 };
	return lut[r];
}

static bool is_concrete(int r) { return r >= OR_SZ_64_KIB && r <= OR_SZ_8_MIB; }

/* Check_Reservation (lz4ada.adb:241-260) */
static void check_reservation(raise_t *R, int requested, int *effective)
{
	if (is_concrete(requested)) {
		if (*effective > requested)
			raise_err(R, OR_TOO_LITTLE_MEMORY,
			          "LZ4 header requres reservation %s, but API call "
			          "requested that only %s be used. This frame "
			          "cannot be processed under the given constraints.",
			          RES_IMAGE[*effective], RES_IMAGE[requested]);
		*effective = requested;
	}
}

/* ----------------------------------------------------------------- header */
/* Process_Legacy_End_Of_Header (lz4ada.adb:225-239) */
static void legacy_end_of_header(raise_t *R, meta_t *m)
{
	int eff = OR_SZ_8_MIB; /* For_Legacy */
	m->input_buffer_filled = 0;
	m->is_format = F_LEGACY;
	m->header_parsing = HDR_DONE;
	m->size_remaining = 0;
	m->status_eof = OR_EOF_MAYBE;
	m->block_checksum_length = 0;
	m->content_checksum_length = 0;
	m->has_content_size = false;
	m->is_compressed = true;
	check_reservation(R, m->memory_reservation, &eff);
	m->memory_reservation = eff;
}

/* Process_Header_Magic (lz4ada.adb:199-223) */
static void header_magic(raise_t *R, meta_t *m, uint32_t magic)
{
	if (magic == MAGIC_MODERN) {
		m->is_format = F_MODERN;
		m->header_parsing = NEED_FLAGS;
		m->size_remaining = 2;
	} else if (magic == MAGIC_LEGACY) {
		legacy_end_of_header(R, m);
	} else if (magic >= MAGIC_SKIP_LO && magic <= MAGIC_SKIP_HI) {
		m->is_format = F_SKIPPABLE;
		m->header_parsing = NEED_SKIP_LEN;
		m->size_remaining = 4;
		m->block_checksum_length = 0;
		m->content_checksum_length = 0;
	} else {
		raise_err(R, OR_NOT_SUPPORTED,
		          "Invalid or unsupported magic: 0x%08x", magic);
	}
}

/* Get_Block_Size_Reservation (lz4ada.adb:316-328) */
static int bd_reservation(raise_t *R, unsigned v)
{
	switch (v) {
	case 4: return OR_SZ_64_KIB;
	case 5: return OR_SZ_256_KIB;
	case 6: return OR_SZ_1_MIB;
	case 7: return OR_SZ_4_MIB;
	default:
		raise_err(R, OR_NOT_SUPPORTED,
		          "Unknown maximum block size flag: 0x%02x", v);
	}
}

/* Process_Header_Flags + Check_Flag_Validity (lz4ada.adb:262-314) */
static void header_flags(raise_t *R, meta_t *m, const uint8_t *hb)
{
	uint8_t flg = hb[4], bd = hb[5];
	bool bchk = (flg & 16) != 0, cchk = (flg & 4) != 0;
	bool reserved = (flg & 2) != 0, dict = (flg & 1) != 0;
	unsigned version = (flg & 0xc0) >> 6;
	unsigned bmax = (bd & 0x70) >> 4;
	bool bd_res = (bd & 0x8f) != 0;
	if (version != 1)
		raise_err(R, OR_NOT_SUPPORTED,
		          "Only LZ4 frame format version 01 supported. "
		          "Detected 0x%02x instead.", version);
	if (reserved || bd_res)
		raise_err(R, OR_NOT_SUPPORTED,
		          "Found reserved bits /= 0. Data might be too new to be "
		          "processed by this implementation!");
	m->status_eof = OR_EOF_NO;
	int required = bd_reservation(R, bmax);
	m->block_checksum_length = bchk ? 4 : 0;
	m->content_checksum_length = cchk ? 4 : 0;
	m->has_content_size = (flg & 8) != 0;
	m->header_parsing = NEED_MODERN;
	m->size_remaining = 1 + (m->has_content_size ? 8 : 0) + (dict ? 4 : 0);
	check_reservation(R, m->memory_reservation, &required);
	if (m->memory_reservation != OR_SINGLE_FRAME)
		m->memory_reservation = required;
}

/* Process_Modern_End_Of_Header + Check_Header_Checksum (lz4ada.adb:330-361) */
static void header_modern_end(raise_t *R, meta_t *m, const uint8_t *hb)
{
	uint8_t hc = hb[m->input_buffer_filled - 1];
	if (m->has_content_size)
		m->size_remaining = load64(hb + 6);
	uint8_t computed = (uint8_t)((oracle_xxh32_hash(hb + 4,
	                               m->input_buffer_filled - 1 - 4) >> 8) & 0xff);
	if (hc != computed)
		raise_err(R, OR_CHECKSUM_ERROR,
		          "Computed Header Checksum 0x%02x does not match expected "
		          "Header Checksum 0x%02x", computed, hc);
	m->header_parsing = HDR_DONE;
	m->input_buffer_filled = 0;
}

/* Process_Header_Bytes (lz4ada.adb:155-191) */
static void header_bytes(raise_t *R, meta_t *m, uint8_t *hb,
                         const uint8_t *in, int64_t len, int64_t *consumed)
{
	int64_t copy = len < (int64_t)m->size_remaining ? len
	                                               : (int64_t)m->size_remaining;
	if (!(copy > 0))
		raise_err(R, OR_ASSERTION_ERROR, "lz4ada.adb:161");
	memcpy(hb + m->input_buffer_filled, in, (size_t)copy);
	m->input_buffer_filled += copy;
	m->size_remaining -= (uint64_t)copy;
	*consumed = copy;
	if (m->size_remaining == 0) {
		switch (m->header_parsing) {
		case NEED_MAGIC: header_magic(R, m, load32(hb)); break;
		case NEED_FLAGS: header_flags(R, m, hb); break;
		case NEED_MODERN: header_modern_end(R, m, hb); break;
		case NEED_SKIP_LEN:
			m->memory_reservation = OR_SZ_64_KIB; /* quirk Q3 */
			m->header_parsing = HDR_DONE;
			m->size_remaining = load32(hb + 4);
			m->status_eof = m->size_remaining == 0 ? OR_EOF_YES : OR_EOF_NO;
			m->input_buffer_filled = 0;
			break;
		default:
			raise_err(R, OR_CONSTRAINT_ERROR,
			          "Header_Complete case must not be reached while "
			          "processing header bytes. Library bug detected.");
		}
	}
}

/* ------------------------------------------------------------------- init */
static oracle_ctx *ctx_alloc(int64_t in_last)
{
	oracle_ctx *c = calloc(1, sizeof(*c));
	c->input_buffer_len = in_last + 1;
	c->input_buffer = calloc((size_t)(in_last + 1 > 0 ? in_last + 1 : 1), 1);
	c->output_pos = 0;
	c->output_pos_history = 0;
	c->input_length = -1;
	c->is_at_end_mark = false;
	oracle_xxh32_init(&c->hash_all_data, 0);
	c->m.is_format = F_TBD;
	c->m.header_parsing = NEED_MAGIC;
	c->m.content_checksum_length = 0;
	c->m.block_checksum_length = 0;
	c->m.status_eof = OR_EOF_NO;
	c->m.input_buffer_filled = 0;
	c->m.is_compressed = false;
	c->m.has_content_size = false;
	c->m.size_remaining = 4;
	return c;
}

/* Init (lz4ada.adb:48-63) */
int oracle_init(int reservation, int64_t *min_buffer_size, oracle_ctx **out)
{
	if (!is_concrete(reservation)) {
		*out = NULL;
		return OR_CONSTRAINT_ERROR;
	}
	int64_t bmax = get_block_size(reservation);
	*min_buffer_size = bmax + HISTORY_SIZE + 8;
	oracle_ctx *c = ctx_alloc(bmax + 4 + BLOCK_SIZE_BYTES - 1);
	c->m.memory_reservation = reservation;
	*out = c;
	return OR_OK;
}

/* Init_With_Header (lz4ada.adb:79-125) */
int oracle_init_with_header(const uint8_t *input, int64_t len, int reservation,
                            int64_t *num_consumed, int64_t *min_buffer_size,
                            oracle_ctx **out, char *errbuf, size_t errcap)
{
	raise_t R;
	uint8_t hb[20];
	meta_t mt;
	memset(&mt, 0, sizeof(mt));
	mt.is_format = F_TBD;
	mt.header_parsing = NEED_MAGIC;
	mt.memory_reservation =
	        reservation == OR_SINGLE_FRAME ? OR_USE_FIRST : reservation;
	mt.status_eof = OR_EOF_NO;
	mt.size_remaining = 4;
	*out = NULL;
	*num_consumed = 0;
	if (setjmp(R.jb)) {
		if (errbuf && errcap)
			snprintf(errbuf, errcap, "%s", R.msg);
		return R.code;
	}
	if (len < 7) /* Pre => Input'Length >= 7 (lz4ada.ads:243) */
		raise_err(&R, OR_ASSERTION_ERROR, "failed precondition from lz4ada.ads:243");
	int64_t pos = 0;
	while (mt.header_parsing != HDR_DONE) {
		if (pos >= len) {
			char b[32];
			raise_err(&R, OR_TOO_FEW_HEADER_BYTES,
			          "Expected at least %s more bytes but header input "
			          "has already ended.", img_u(b, mt.size_remaining));
		}
		int64_t c;
		header_bytes(&R, &mt, hb, input + pos, len - pos, &c);
		pos += c;
		*num_consumed += c;
	}
	int64_t bmax = get_block_size(mt.memory_reservation);
	int64_t in_last = bmax + mt.block_checksum_length + BLOCK_SIZE_BYTES - 1;
	*min_buffer_size = bmax + HISTORY_SIZE + 8;
	if (reservation == OR_SINGLE_FRAME)
		mt.memory_reservation = OR_SINGLE_FRAME;
	oracle_ctx *c = ctx_alloc(in_last);
	c->m = mt;
	*out = c;
	return OR_OK;
}

/* Init_For_Block (lz4ada.adb:127-147) */
int oracle_init_for_block(int64_t compressed_length, int reservation,
                          int64_t *min_buffer_size, oracle_ctx **out)
{
	if (!is_concrete(reservation)) {
		*out = NULL;
		return OR_CONSTRAINT_ERROR;
	}
	int64_t bmax = get_block_size(reservation);
	*min_buffer_size = bmax + HISTORY_SIZE + 8;
	oracle_ctx *c = ctx_alloc(bmax - 1);
	c->m.is_format = F_BLOCK;
	c->m.is_compressed = true;
	c->m.header_parsing = HDR_DONE;
	c->m.memory_reservation = reservation;
	c->input_length = compressed_length;
	*out = c;
	return OR_OK;
}

void oracle_free(oracle_ctx *c)
{
	if (!c)
		return;
	free(c->input_buffer);
	free(c);
}

const char *oracle_last_error(const oracle_ctx *c) { return c ? c->err : ""; }

/* Is_End_Of_Frame (lz4ada.adb:906-915) */
int oracle_is_end_of_frame(const oracle_ctx *c)
{
	switch (c->m.is_format) {
	case F_LEGACY: return c->is_at_end_mark ? OR_EOF_MAYBE : c->m.status_eof;
	case F_BLOCK: return c->input_length == -1 ? OR_EOF_YES : OR_EOF_NO;
	default: return c->m.status_eof;
	}
}

/* ------------------------------------------------------------ block decode */
typedef struct {
	raise_t *R;
	oracle_ctx *c;
	uint8_t *buf;
	int64_t buflen;
} dec_t;

/* Decrease_Data_Size_Remaining (lz4ada.adb:826-839) */
static void debit(dec_t *d, uint64_t n)
{
	meta_t *m = &d->c->m;
	if (m->has_content_size) {
		if (m->size_remaining < n)
			raise_err(d->R, OR_DATA_CORRUPTION,
			          "Produced content size exceeds declared content "
			          "size. The supplied data is inconsistent.");
		m->size_remaining -= n;
	}
}

/*
 * Write_Output (lz4ada.adb:790-824): the 8-byte wild copy.  `data` spans
 * indices [0, data_len) (Data'Last = data_len - 1); copy data[first..last]
 * to buf[output_pos..].  Each 8-byte step is an Ada slice assignment, i.e.
 * memmove semantics, and writes past `last` (overshoot, up to 7 bytes).
 * When data == buf the same memory is both source and destination.
 * Bytes the reference would read past Data'Last (D3) read as zero here.
 */
static void write_output(dec_t *d, const uint8_t *data, int64_t data_len,
                         int64_t first, int64_t last)
{
	oracle_ctx *c = d->c;
	int64_t num = last - first + 1;
	int64_t co = c->output_pos, ci = first;
	if (co + num > d->buflen)
		raise_err(d->R, OR_DATA_CORRUPTION,
		          "Corrupted Block: decompressed data exceeds the output "
		          "buffer.");
	while ((data_len - 1) - ci + 1 >= 8 && ci <= last) {
		uint8_t tmp[8];
		memcpy(tmp, data + ci, 8);
		int64_t n = co + 8 <= d->buflen ? 8 : d->buflen - co;
		memcpy(d->buf + co, tmp, (size_t)n);
		co += 8;
		ci += 8;
	}
	if (ci <= last) {
		int64_t n = last - ci + 1;
		int64_t avail = data_len - ci; /* in-bounds source bytes */
		if (avail < 0)
			avail = 0;
		if (avail > n)
			avail = n;
		memmove(d->buf + co, data + ci, (size_t)avail);
		if (n > avail) /* D3: reference reads past Data'Last */
			memset(d->buf + co + avail, 0, (size_t)(n - avail));
	}
	c->output_pos += num;
	debit(d, (uint64_t)num);
}

/* Output_With_History (lz4ada.adb:845-904) */
static void output_with_history(dec_t *d, int64_t offset, int64_t match_length)
{
	oracle_ctx *c = d->c;
	int64_t raw_offset = c->output_pos - offset;
	int64_t remaining = match_length;
	int64_t i_offset, i_length;
	if (raw_offset >= 0) {
		i_offset = raw_offset;
		i_length = match_length < offset ? match_length : offset;
	} else {
		int64_t h_offset = raw_offset + c->output_pos_history;
		int64_t h_length = offset - c->output_pos;
		if (match_length < h_length)
			h_length = match_length;
		if (h_offset < 0) {
			char b[32];
			raise_err(d->R, OR_DATA_CORRUPTION,
			          "Backreference location out of range. Read from "
			          "offset %s not possible (earliest available index "
			          "is 0).", img(b, h_offset));
		}
		if (h_length > 0) {
			write_output(d, d->buf, d->buflen, h_offset,
			             h_offset + h_length - 1);
			remaining = match_length - h_length;
		}
		i_offset = 0;
		i_length = remaining < c->output_pos ? remaining : c->output_pos;
	}
	if (i_length > 0) {
		write_output(d, d->buf, d->buflen, i_offset, i_offset + i_length - 1);
		remaining -= i_length;
	}
	if (remaining > 0) {
		int64_t r_start = c->output_pos - offset;
		int64_t done = 0;
		while (done < remaining) {
			int64_t r_len = c->output_pos - r_start;
			if (remaining - done < r_len)
				r_len = remaining - done;
			write_output(d, d->buf, d->buflen, r_start, r_start + r_len - 1);
			done += r_len;
		}
	}
}

/* Update_Checksum (lz4ada.adb:709-714) */
static void update_checksum(oracle_ctx *c, const uint8_t *p, int64_t n)
{
	if (c->m.content_checksum_length != 0)
		oracle_xxh32_update(&c->hash_all_data, p, n);
}

/* Decompress_Full_Block (lz4ada.adb:716-788).  raw = Raw_Data, 0-based. */
static void decompress_full_block(dec_t *d, const uint8_t *raw, int64_t n,
                                  int64_t *out_first, int64_t *out_last)
{
	oracle_ctx *c = d->c;
	int64_t idx = 0;
	*out_first = c->output_pos;
	while (idx <= n - 1) {
		/* Decompress_Sequence (lz4ada.adb:737-777) */
		uint8_t token = raw[idx];
		int64_t nlit = token >> 4, ml = token & 15;
		idx += 1;
		if (nlit == 15) { /* Process_Variable_Length (lz4ada.adb:724-735) */
			uint8_t t;
			do {
				if (idx > n - 1) /* D4: reference raises Constraint_Error */
					raise_err(d->R, OR_DATA_CORRUPTION,
					          "Corrupted Block: sequence truncated at the "
					          "end of the block.");
				t = raw[idx];
				nlit += t;
				idx += 1;
			} while (t == 255);
		}
		if (nlit > 0) {
			write_output(d, raw, n, idx, idx + nlit - 1);
			idx += nlit;
		}
		if (idx > n - 1) {
			if (ml != 0) {
				char b[32];
				raise_err(d->R, OR_DATA_CORRUPTION,
				          "Match_Length=%s suggests compressed data but "
				          "this sequence already ends after the literals. "
				          "This might also happen with an untypical encoder?",
				          img(b, ml));
			}
			if (idx > n) /* D3: literal run overran the block */
				raise_err(d->R, OR_DATA_CORRUPTION,
				          "Corrupted Block: literal run exceeds the end of "
				          "the block.");
			break;
		}
		if (idx + 1 > n - 1) /* D4 */
			raise_err(d->R, OR_DATA_CORRUPTION,
			          "Corrupted Block: sequence truncated at the end of "
			          "the block.");
		int64_t offset = (int64_t)raw[idx] | ((int64_t)raw[idx + 1] << 8);
		idx += 2;
		if (offset == 0)
			raise_err(d->R, OR_DATA_CORRUPTION,
			          "Corrupted Block: Offset = 0 detected.");
		if (ml == 15) {
			uint8_t t;
			do {
				if (idx > n - 1) /* D4 */
					raise_err(d->R, OR_DATA_CORRUPTION,
					          "Corrupted Block: sequence truncated at the "
					          "end of the block.");
				t = raw[idx];
				ml += t;
				idx += 1;
			} while (t == 255);
		}
		output_with_history(d, offset, ml + 4);
	}
	*out_last = c->output_pos - 1;
	update_checksum(c, d->buf + *out_first, *out_last - *out_first + 1);
	if (c->output_pos >= HISTORY_SIZE)
		c->output_pos_history = c->output_pos;
}

/* Decode_Full_Block_With_Trailer (lz4ada.adb:661-707).  blk holds the
 * payload plus the optional 4-byte block checksum. */
static void decode_full_block(dec_t *d, const uint8_t *blk, int64_t blen,
                              int64_t *out_first, int64_t *out_last)
{
	oracle_ctx *c = d->c;
	int bcl = c->m.block_checksum_length;
	int64_t raw_len = blen - bcl;
	if (bcl > 0) {
		uint32_t expect = load32(blk + blen - bcl);
		uint32_t comp = oracle_xxh32_hash(blk, raw_len);
		if (comp != expect)
			raise_err(d->R, OR_CHECKSUM_ERROR,
			          "Declared checksum is 0x%08x, but computed one is "
			          "0x%08x.", expect, comp);
	}
	if (c->output_pos >= HISTORY_SIZE)
		c->output_pos = 0;
	if (c->m.is_compressed) {
		decompress_full_block(d, blk, raw_len, out_first, out_last);
	} else {
		write_output(d, blk, blen, 0, raw_len - 1);
		if (c->output_pos >= HISTORY_SIZE)
			c->output_pos_history = c->output_pos;
		*out_first = c->output_pos - raw_len;
		*out_last = c->output_pos - 1;
		update_checksum(c, d->buf + *out_first, *out_last - *out_first + 1);
	}
}

/* ----------------------------------------------------------------- update */
typedef struct {
	dec_t d;
	const uint8_t *in;
	int64_t len;
	int64_t *consumed;
	int64_t *first, *last;
} upd_t;

static void reset_outer(oracle_ctx *c) /* lz4ada.adb:451-461 */
{
	c->is_at_end_mark = false;
	c->input_length = -1;
	c->output_pos = 0;
	c->output_pos_history = 0;
	oracle_xxh32_reset(&c->hash_all_data, 0);
}

/* Reset_For_Next_Frame (lz4ada.adb:435-449) */
static void reset_for_next_frame(upd_t *u, int64_t *consumed)
{
	oracle_ctx *c = u->d.c;
	if (c->m.memory_reservation == OR_SINGLE_FRAME)
		raise_err(u->d.R, OR_DATA_CORRUPTION,
		          "Requested Single_Frame operation but data was provided "
		          "after End of Frame was detected");
	c->m.status_eof = OR_EOF_NO;
	c->m.header_parsing = NEED_MAGIC;
	c->m.size_remaining = 4;
	reset_outer(c);
	header_bytes(u->d.R, &c->m, c->input_buffer, u->in, u->len, consumed);
}

/* Skip (lz4ada.adb:420-433) */
static void skip(upd_t *u)
{
	oracle_ctx *c = u->d.c;
	uint64_t remain = c->m.size_remaining;
	uint64_t cons = (uint64_t)u->len < remain ? (uint64_t)u->len : remain;
	if (c->m.status_eof == OR_EOF_YES && cons == 0) {
		reset_for_next_frame(u, u->consumed);
	} else {
		*u->consumed = (int64_t)cons;
		c->m.size_remaining = remain - cons;
		c->m.status_eof = c->m.size_remaining == 0 ? OR_EOF_YES : OR_EOF_NO;
	}
}

/* Set_Frame_Has_Ended (lz4ada.adb:465-477) */
static void frame_has_ended(upd_t *u)
{
	oracle_ctx *c = u->d.c;
	c->m.status_eof = OR_EOF_YES;
	c->m.input_buffer_filled = 0;
	if (c->m.has_content_size && c->m.size_remaining != 0) {
		char b[32];
		raise_err(u->d.R, OR_DATA_CORRUPTION,
		          "Frame has ended, but according to content size, there "
		          "should be %s bytes left to output.",
		          img_u(b, c->m.size_remaining));
	}
}

/* Check_End_Mark (lz4ada.adb:463-523) */
static void check_end_mark(upd_t *u)
{
	oracle_ctx *c = u->d.c;
	int64_t provided = u->len - *u->consumed;
	int64_t required = c->m.content_checksum_length - c->m.input_buffer_filled;
	if (c->m.content_checksum_length == 0 || c->m.status_eof == OR_EOF_YES ||
	    required <= 0) {
		if (c->m.status_eof == OR_EOF_YES) {
			if (*u->consumed != 0)
				raise_err(u->d.R, OR_ASSERTION_ERROR, "lz4ada.adb:486");
			reset_for_next_frame(u, u->consumed);
		} else {
			frame_has_ended(u);
		}
	} else if (provided >= required) {
		uint8_t tmp[8];
		memcpy(tmp, c->input_buffer, (size_t)c->m.input_buffer_filled);
		memcpy(tmp + c->m.input_buffer_filled, u->in + *u->consumed,
		       (size_t)required);
		uint32_t declared = load32(tmp);
		uint32_t computed = oracle_xxh32_final(&c->hash_all_data);
		*u->consumed += required;
		if (declared != computed)
			raise_err(u->d.R, OR_CHECKSUM_ERROR,
			          "Computed content checksum 0x%08x does not match "
			          "declared content checksum 0x%08x.", computed, declared);
		frame_has_ended(u);
	} else {
		memcpy(c->input_buffer + c->m.input_buffer_filled,
		       u->in + *u->consumed, (size_t)provided);
		c->m.input_buffer_filled += provided;
		*u->consumed += provided;
	}
}

static bool is_any_magic(uint32_t v) /* lz4ada.adb:587-593 */
{
	return v == MAGIC_MODERN || v == MAGIC_LEGACY ||
	       (v >= MAGIC_SKIP_LO && v <= MAGIC_SKIP_HI);
}

/* Try_Detect_Input_Length (lz4ada.adb:525-585) */
static void try_detect_input_length(upd_t *u)
{
	oracle_ctx *c = u->d.c;
	int64_t additional = BLOCK_SIZE_BYTES + c->m.block_checksum_length;
	int64_t n = BLOCK_SIZE_BYTES - c->m.input_buffer_filled;
	if (u->len < n)
		n = u->len;
	*u->consumed = n;
	memcpy(c->input_buffer + c->m.input_buffer_filled, u->in, (size_t)n);
	c->m.input_buffer_filled += n;
	if (c->m.input_buffer_filled != BLOCK_SIZE_BYTES)
		return;
	uint32_t word = load32(c->input_buffer);
	if (c->m.is_format == F_MODERN && word == 0) {
		c->is_at_end_mark = true;
		c->m.input_buffer_filled = 0;
	} else if (c->m.is_format == F_LEGACY && is_any_magic(word)) {
		if (c->m.memory_reservation == OR_SINGLE_FRAME)
			raise_err(u->d.R, OR_DATA_CORRUPTION,
			          "Requested Single_Frame operation but data provided "
			          "what looks like the beginning of another frame.");
		reset_outer(c);
		header_magic(u->d.R, &c->m, word);
	} else { /* Detect_Modern */
		if (c->m.is_format == F_MODERN) {
			c->m.is_compressed = (word & 0x80000000u) == 0;
			word &= 0x7ffffffu; /* 27-bit mask, quirk Q2 */
		}
		c->input_length = (int64_t)word;
		if (c->input_length + additional > c->input_buffer_len) {
			char b1[32], b2[32], b3[32];
			c->input_length = -1;
			raise_err(u->d.R, OR_DATA_CORRUPTION,
			          "Declared maximum data length exceeded. Buffer has "
			          "%s bytes, current block requires %s bytes + %s bytes "
			          "for metadata.", img(b1, c->input_buffer_len),
			          img_u(b2, word), img(b3, additional));
		}
	}
}

/* Cache_Data_And_Process_If_Full (lz4ada.adb:630-659) */
static void cache_and_process(upd_t *u)
{
	oracle_ctx *c = u->d.c;
	int64_t avail = u->len - *u->consumed;
	int64_t want = c->input_length + c->m.block_checksum_length -
	               c->m.input_buffer_filled +
	               (c->m.is_format == F_BLOCK ? 0 : BLOCK_SIZE_BYTES);
	int64_t fill = c->m.input_buffer_filled;
	const uint8_t *src = u->in + *u->consumed;
	if (want > avail) {
		if (fill + avail > c->input_buffer_len) /* Ada index check */
			raise_err(u->d.R, OR_CONSTRAINT_ERROR,
			          "lz4ada.adb:644 index check failed");
		memcpy(c->input_buffer + fill, src, (size_t)avail);
		c->m.input_buffer_filled += avail;
		*u->consumed += avail;
	} else {
		*u->consumed += want;
		c->m.input_buffer_filled = 0;
		c->input_length = -1;
		/* Input_Buffer(Block_Size_Bytes .. Fill - 1) & Input(...): for the
		 * raw-block format this drops 4 cached bytes (quirk Q5). */
		int64_t head = fill - BLOCK_SIZE_BYTES;
		if (head < 0)
			head = 0;
		int64_t blen = head + want;
		uint8_t *blk = malloc((size_t)(blen > 0 ? blen : 1));
		if (head)
			memcpy(blk, c->input_buffer + BLOCK_SIZE_BYTES, (size_t)head);
		memcpy(blk + head, src, (size_t)want);
		decode_full_block(&u->d, blk, blen, u->first, u->last);
		free(blk);
	}
}

/* Handle_Newly_Known_Input_Length (lz4ada.adb:595-628) */
static void handle_new_length(upd_t *u)
{
	oracle_ctx *c = u->d.c;
	int64_t total = c->input_length + c->m.block_checksum_length;
	if (u->len - *u->consumed >= total) {
		const uint8_t *blk = u->in + *u->consumed;
		*u->consumed += total;
		c->m.input_buffer_filled = 0;
		c->input_length = -1;
		decode_full_block(&u->d, blk, total, u->first, u->last);
	} else {
		cache_and_process(u);
	}
}

/* Update (lz4ada.adb:383-418) */
int oracle_update(oracle_ctx *c, const uint8_t *input, int64_t len,
                  int64_t *num_consumed, uint8_t *buf, int64_t buflen,
                  int64_t *first, int64_t *last)
{
	raise_t R;
	upd_t u = { { &R, c, buf, buflen }, input, len, num_consumed, first, last };
	*num_consumed = 0;
	*first = 1;
	*last = 0;
	c->err_code = OR_OK;
	c->err[0] = 0;
	if (setjmp(R.jb)) {
		c->err_code = R.code;
		snprintf(c->err, sizeof(c->err), "%s", R.msg);
		return R.code;
	}
	if (c->m.header_parsing != HDR_DONE) {
		header_bytes(&R, &c->m, c->input_buffer, input, len, num_consumed);
	} else if (c->m.is_format == F_SKIPPABLE) {
		skip(&u);
	} else {
		if (c->is_at_end_mark) {
			check_end_mark(&u);
		} else if (c->input_length != -1) {
			cache_and_process(&u);
		} else {
			try_detect_input_length(&u);
			if (c->is_at_end_mark)
				check_end_mark(&u);
			else if (c->input_length != -1)
				handle_new_length(&u);
		}
	}
	return OR_OK;
}

/* -------------------------------------------------------------- harnesses */
int oracle_decode_stream(const uint8_t *input, int64_t len, int64_t chunk,
                         int reservation, uint8_t *out, int64_t out_cap,
                         int64_t *out_len, int *eof, char *errbuf, size_t errcap)
{
	int64_t osz;
	oracle_ctx *c;
	int st = oracle_init(reservation, &osz, &c);
	*out_len = 0;
	*eof = OR_EOF_NO;
	if (st)
		return st;
	uint8_t *buf = calloc((size_t)osz, 1);
	int64_t pos = 0; /* start of the current read window */
	int64_t wlen = 0, used = 0;
	*eof = oracle_is_end_of_frame(c);
	for (;;) {
		if (used >= wlen) { /* Read(LZS, Buf_Input, Last) */
			pos += wlen;
			wlen = len - pos < chunk ? len - pos : chunk;
			used = 0;
			if (wlen <= 0)
				break;
		}
		int64_t cons, f, l;
		st = oracle_update(c, input + pos + used, wlen - used, &cons, buf,
		                   osz, &f, &l);
		if (st) {
			if (errbuf && errcap)
				snprintf(errbuf, errcap, "%s", c->err);
			break;
		}
		if (l >= f) {
			int64_t n = l - f + 1;
			if (*out_len + n > out_cap) {
				st = OR_ASSERTION_ERROR;
				if (errbuf && errcap)
					snprintf(errbuf, errcap, "output capacity exceeded");
				break;
			}
			memcpy(out + *out_len, buf + f, (size_t)n);
			*out_len += n;
		}
		used += cons;
		*eof = oracle_is_end_of_frame(c);
	}
	free(buf);
	oracle_free(c);
	return st;
}

int oracle_error_harness(const uint8_t *input, int64_t len, char *errbuf,
                         size_t errcap)
{
	int64_t total, mbs;
	oracle_ctx *c;
	int st = oracle_init_with_header(input, len, OR_SINGLE_FRAME, &total, &mbs,
	                                 &c, errbuf, errcap);
	if (st)
		return st;
	uint8_t *bo = calloc((size_t)mbs, 1);
	while (total < len) {
		int64_t cons, f, l;
		st = oracle_update(c, input + total, len - total, &cons, bo, mbs, &f, &l);
		if (st) {
			if (errbuf && errcap)
				snprintf(errbuf, errcap, "%s", c->err);
			break;
		}
		if (cons == 0)
			break;
		total += cons;
	}
	free(bo);
	oracle_free(c);
	return st;
}

/* tool_unlz4ada/unlz4ada.adb:63-105 over an in-memory stdin. */
int oracle_unlz4ada(const uint8_t *input, int64_t len, uint8_t *out,
                    int64_t out_cap, int64_t *out_len, char *errbuf,
                    size_t errcap)
{
	enum { BUFSZ = 4096 };
	uint8_t bin[BUFSZ];
	int64_t rpos = 0; /* stdin read position */
	int64_t last = -1, total = 0;
	bool end_of_input = false;
	int st = OR_OK;
	*out_len = 0;
#define READ_INTO(dst, cap, lastvar, base)                                     \
	do {                                                                   \
		int64_t _n = len - rpos < (cap) ? len - rpos : (cap);          \
		memcpy((dst), input + rpos, (size_t)_n);                        \
		rpos += _n;                                                     \
		(lastvar) = (base) + _n - 1;                                    \
	} while (0)
	while (!end_of_input) {
		if (last - total < 6) {
			int64_t keep = last - total + 1;
			memmove(bin, bin + total, (size_t)keep);
			READ_INTO(bin + keep, BUFSZ - keep, last, keep);
			if (last < 0)
				break;
			if (last < 6) {
				if (errbuf && errcap)
					snprintf(errbuf, errcap, "Partial frame detected. "
					         "Unable to process all data");
				return OR_CONSTRAINT_ERROR;
			}
			total = 0;
		}
		int eof_status = OR_EOF_NO;
		int64_t cons0, rbs;
		oracle_ctx *c;
		st = oracle_init_with_header(bin + total, last - total + 1,
		                             OR_SINGLE_FRAME, &cons0, &rbs, &c, errbuf,
		                             errcap);
		if (st)
			return st;
		uint8_t *buf = calloc((size_t)rbs, 1);
		total += cons0;
		while (eof_status == OR_EOF_NO && !end_of_input) {
			int64_t cons, f, l;
			st = oracle_update(c, bin + total, last - total + 1, &cons, buf,
			                   rbs, &f, &l);
			if (st) {
				if (errbuf && errcap)
					snprintf(errbuf, errcap, "%s", c->err);
				free(buf);
				oracle_free(c);
				return st;
			}
			total += cons;
			eof_status = oracle_is_end_of_frame(c);
			if (eof_status == OR_EOF_YES || total > last || l - f >= 0) {
				if (l >= f) {
					int64_t n = l - f + 1;
					if (*out_len + n > out_cap) {
						free(buf);
						oracle_free(c);
						return OR_ASSERTION_ERROR;
					}
					memcpy(out + *out_len, buf + f, (size_t)n);
					*out_len += n;
				}
				if (eof_status != OR_EOF_YES && total > last) {
					READ_INTO(bin, BUFSZ, last, 0);
					if (last < 0) {
						end_of_input = true;
						if (eof_status == OR_EOF_NO) {
							if (errbuf && errcap)
								snprintf(errbuf, errcap,
								         "End not signalled by library. "
								         "Unable to process all data");
							free(buf);
							oracle_free(c);
							return OR_CONSTRAINT_ERROR;
						}
					}
					total = 0;
				}
			}
		}
		free(buf);
		oracle_free(c);
	}
#undef READ_INTO
	return st;
}
