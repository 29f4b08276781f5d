// lz4gen.cpp -- deterministic synthetic LZ4 block generator (SURVEY §8d,
// hard part H6): emits valid LZ4 blocks directly from a seeded sequence
// model, together with their decoded bytes, so that benches and GPU tests
// need no external compressor on the GPU box.  Block rules honoured: the
// last sequence is literal-only with >= 12 literals when the block allows,
// offsets lie in [1, min(pos, 65535)].  kind 4 (chain) is for linked frames,
// kind 5 is mixed with offsets <= 65528 (no quirk-D1 matches).
#include <stdint.h>
#include <string.h>

#include "lz4ada_hip.h"

namespace {

struct Rng {  // xorshift64*
	uint64_t s;
	explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x4C5A3441ull) { next(); }
	uint64_t next()
	{
		s ^= s >> 12;
		s ^= s << 25;
		s ^= s >> 27;
		return s * 2685821657736338717ull;
	}
	uint32_t below(uint32_t n) { return n ? uint32_t((next() >> 32) % n) : 0; }
	// geometric with the given mean (>= 0)
	uint32_t geo(double mean)
	{
		if (mean <= 0)
			return 0;
		const double p = 1.0 / (mean + 1.0);
		uint32_t k = 0;
		while (k < 1000000 && double(next() >> 11) * (1.0 / 9007199254740992.0) > p)
			++k;
		return k;
	}
};

struct Out {
	uint8_t* p;
	int64_t n, cap;
	bool ok = true;
	void put(uint8_t b)
	{
		if (n < cap)
			p[n] = b;
		else
			ok = false;
		++n;
	}
	void len_ext(int64_t v)  // 15 + 255* + rest
	{
		v -= 15;
		while (v >= 255) {
			put(255);
			v -= 255;
		}
		put(uint8_t(v));
	}
};

uint8_t lit_byte(Rng& r, int kind)
{
	if (kind == 3)
		return uint8_t(r.next() >> 56);
	// text-like alphabet
	static const char alpha[] = "etaoinshrdlucmfwypvbgkjqxz ETAOINSHRDLU.,;:0123456789\n";
	return uint8_t(alpha[r.below(sizeof(alpha) - 1)]);
}

}  // namespace

// hist: bytes raw[-hist .. -1] precede the block (a linked frame's earlier
// output); offsets may reach back into them.
static int64_t gen_block(int kind, uint64_t seed, uint8_t* raw, int64_t raw_len, int64_t hist,
                         uint8_t* comp, int64_t comp_cap)
{
	Rng r(seed);
	Out o{ comp, 0, comp_cap };
	int64_t pos = 0;
	const int64_t tail = raw_len >= 13 ? 12 : raw_len;  // final literal-only run
	const int64_t body = raw_len - tail;
	while (pos < body) {
		int64_t L = 0, ml = 0, off = 0;
		switch (kind) {
		case 0:  // dense: ~5 B/sequence
			L = r.geo(0.9);
			ml = 4 + r.geo(0.4);
			break;
		case 1:  // mixed: ~32 B/sequence, ratio ~2
			L = r.geo(12.0);
			ml = 4 + r.geo(16.0);
			break;
		case 2:  // rle zeros: one literal, then offset-1 runs
			L = pos == 0 ? 1 : 0;
			ml = 4 + r.geo(60000.0);
			break;
		case 4:  // chain: matches only (short offsets), so in a linked frame
		         // every byte copies the previous block's tail -- pointer
		         // chains through every block (lz4ada_linked.hip worst case)
			L = 0;
			ml = 4 + r.geo(100.0);
			break;
		case 5:  // mixed, offsets below 65529: no match can meet quirk D1
			L = r.geo(12.0);
			ml = 4 + r.geo(16.0);
			break;
		default:  // literal-heavy
			L = 64 + r.geo(400.0);
			ml = 4 + r.geo(3.0);
			break;
		}
		if (pos == 0 && L == 0 && hist == 0)
			L = 1;
		if (pos + L > body)
			L = body - pos;
		const int64_t room = body - pos - L;
		if (room < 4)  // no room for a match: the final literal run takes it
			break;
		if (ml > room)
			ml = room;
		const int64_t lit0 = pos;
		for (int64_t i = 0; i < L; ++i) {
			const uint8_t b = kind == 2 ? 0 : lit_byte(r, kind);
			if (raw)
				raw[pos + i] = b;
		}
		pos += L;
		if (ml) {
			const int64_t cap = kind == 5 ? 65528 : 65535;
			const int64_t maxoff = pos + hist < cap ? pos + hist : cap;
			if (kind == 2)
				off = 1;
			else if (kind == 4)
				off = 1 + r.below(uint32_t(maxoff < 16 ? maxoff : 16));
			else if ((kind == 1 || kind == 5) && r.below(4) == 0)
				off = 1 + r.below(uint32_t(maxoff < 64 ? maxoff : 64));
			else
				off = 1 + r.below(uint32_t(maxoff));
			for (int64_t k = 0; k < ml; ++k)
				if (raw)
					raw[pos + k] = raw[pos - off + k];
		}
		// emit: literal bytes come from raw (or regenerate when raw == NULL)
		{
			const int64_t m4 = ml ? ml - 4 : 0;
			o.put(uint8_t(((L >= 15 ? 15 : L) << 4) | (ml ? (m4 >= 15 ? 15 : m4) : 0)));
			if (L >= 15)
				o.len_ext(L);
			for (int64_t i = 0; i < L; ++i)
				o.put(raw ? raw[lit0 + i] : 0);
			if (ml) {
				o.put(uint8_t(off & 0xff));
				o.put(uint8_t(off >> 8));
				if (m4 >= 15)
					o.len_ext(m4);
			}
		}
		pos += ml;
	}
	// final literal-only sequence
	{
		const int64_t L = raw_len - pos;
		for (int64_t i = 0; i < L; ++i) {
			const uint8_t b = kind == 2 ? 0 : lit_byte(r, kind);
			if (raw)
				raw[pos + i] = b;
		}
		if (L > 0 || raw_len == 0) {
			o.put(uint8_t((L >= 15 ? 15 : L) << 4));
			if (L >= 15)
				o.len_ext(L);
			for (int64_t i = 0; i < L; ++i)
				o.put(raw ? raw[pos + i] : 0);
		}
	}
	return o.ok ? o.n : -1;
}

extern "C" int64_t lz4ada_gen_block(int kind, uint64_t seed, uint8_t* raw, int64_t raw_len,
                                    uint8_t* comp, int64_t comp_cap)
{
	return gen_block(kind, seed, raw, raw_len, 0, comp, comp_cap);
}

extern "C" int64_t lz4ada_gen_block_linked(int kind, uint64_t seed, uint8_t* buf, int64_t hist,
                                           int64_t raw_len, uint8_t* comp, int64_t comp_cap)
{
	if (!buf || hist < 0)
		return -1;
	return gen_block(kind, seed, buf + hist, raw_len, hist, comp, comp_cap);
}
