// lz4ada_host.cpp -- host side of the MI355X LZ4Ada decompressor: the frame
// engine (header parser and Update state machine of lib/lz4ada.adb, L2 of
// SURVEY §1), the bulk frame indexer, and the C-ABI of include/lz4ada_hip.h.
//
// The host only parses framing.  Every block byte is produced on the GPU:
// the streaming Update path runs k_serial_block (reference-exact, one
// block per call) on a device mirror of the caller's Buffer; the bulk path
// runs k_decode_blocks (one wavefront per block) over a whole frame.  There
// is no CPU decoder here: without a GPU, decoding calls fail with
// LZ4ADA_DEVICE_ERROR.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <future>
#include <tuple>
#include <mutex>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "lz4ada_hip.h"
#include "lz4ada_internal.h"

namespace lz4ada {

// ------------------------------------------------------------------ errors

struct Error {
	int code;
	std::string msg;
};

[[noreturn]] static void raise(int code, std::string msg) { throw Error{ code, std::move(msg) }; }

// Ada 'Image: leading blank for non-negative numbers.
static std::string img(int64_t v)
{
	return v >= 0 ? " " + std::to_string(v) : std::to_string(v);
}
static std::string img_u(uint64_t v) { return " " + std::to_string(v); }
static std::string hex8(uint32_t v)
{
	char b[8];
	snprintf(b, sizeof b, "%02x", v & 0xffu);
	return b;
}
static std::string hex32(uint32_t v)
{
	char b[16];
	snprintf(b, sizeof b, "%08x", v);
	return b;
}

static const char* const RES_IMAGE[] = { "SZ_64_KIB", "SZ_256_KIB", "SZ_1_MIB",    "SZ_4_MIB",
	                                 "SZ_8_MIB",  "USE_FIRST",  "SINGLE_FRAME" };

static thread_local std::string g_thread_error;

static uint32_t load32(const uint8_t* p)
{
	return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) |
	       (uint32_t(p[3]) << 24);
}
static uint64_t load64(const uint8_t* p) { return uint64_t(load32(p)) | (uint64_t(load32(p + 4)) << 32); }

// XXH32 of the 2..14-byte frame descriptor for the header checksum byte
// (lz4ada.adb:351-361).  Framing, not block data: it runs on the host.
static uint32_t descriptor_xxh32(const uint8_t* p, size_t n)
{
	auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
	uint32_t h = uint32_t(n) + P5;  // n < 16: no stripes
	size_t d = 0;
	for (; d + 4 <= n; d += 4)
		h = rotl(h + load32(p + d) * P3, 17) * P4;
	for (; d < n; ++d)
		h = rotl(h + uint32_t(p[d]) * P5, 11) * P1;
	h = (h ^ (h >> 15)) * P2;
	h = (h ^ (h >> 13)) * P3;
	return h ^ (h >> 16);
}

// ------------------------------------------------------------------ device

#define HIP_OK(expr)                                                                          \
	do {                                                                                  \
		hipError_t _e = (expr);                                                       \
		if (_e != hipSuccess)                                                         \
			raise(LZ4ADA_DEVICE_ERROR,                                            \
			      std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr); \
	} while (0)

static void device_check_or_raise()
{
	int n = 0;
	hipError_t e = hipGetDeviceCount(&n);
	if (e != hipSuccess || n <= 0)
		raise(LZ4ADA_DEVICE_ERROR,
		      "no usable HIP device: the LZ4Ada MI355X decoder has no CPU fallback");
}

// Process-wide pools of the small device and pinned host allocations and
// of the facade's streams.  A streaming context per frame (tool_unlz4ada
// re-inits per frame, unlz4ada.adb:84-87) otherwise pays stream creation
// and a dozen hipMalloc / hipHostMalloc calls per frame -- ~3.5 ms, more
// than a 4 MiB frame of 64 KiB blocks takes to decode (tools/facade_c).
// Blocks up to POOL_MAX bytes are kept by power-of-two size class, at most
// keep_limit() bytes per kind and device; a block is pooled only after a
// device synchronisation (the implicit one of the hipFree it replaces), so
// no queued work still uses it.  lz4ada_release_device_cache() empties them.
struct MemPool {
	static constexpr size_t POOL_MAX = size_t(256) << 20;
	// idle bytes kept per pool (device / pinned): 1 GiB, or LZ4ADA_POOL_KEEP_MB
	static size_t keep_limit()
	{
		static const size_t k = [] {
			const char* e = getenv("LZ4ADA_POOL_KEEP_MB");
			return e ? size_t(strtoull(e, nullptr, 10)) << 20 : size_t(1) << 30;
		}();
		return k;
	}
	std::mutex mu;
	std::vector<std::tuple<int, size_t, void*>> free;  // (device, class bytes, block)
	size_t kept = 0;
	bool pinned;
	explicit MemPool(bool pin) : pinned(pin) {}
	static size_t size_class(size_t b)
	{
		size_t c = 4096;
		while (c < b)
			c <<= 1;
		return c;
	}
	void raw_free(void* p) { (void)(pinned ? hipHostFree(p) : hipFree(p)); }
	// A block and the device that was current when it was taken: put() syncs
	// and files it under THAT device (a buffer released after the
	// caller switched GPUs must not be pooled under the new one).  Pinned
	// blocks are pooled for any device but still sync the device they served.
	struct Block {
		void* p;
		size_t bytes;
		int dev;
	};
	Block get(size_t bytes)
	{
		int dev = 0;
		(void)hipGetDevice(&dev);
		const int key = pinned ? 0 : dev;
		const size_t c = bytes <= POOL_MAX ? size_class(bytes) : bytes;
		if (c <= POOL_MAX) {
			std::lock_guard<std::mutex> l(mu);
			for (size_t i = 0; i < free.size(); ++i)
				if (std::get<0>(free[i]) == key && std::get<1>(free[i]) == c) {
					void* p = std::get<2>(free[i]);
					free[i] = free.back();
					free.pop_back();
					kept -= c;
					return { p, c, dev };
				}
		}
		void* p = nullptr;
		hipError_t e = pinned ? hipHostMalloc(&p, c, hipHostMallocDefault) : hipMalloc(&p, c);
		if (e != hipSuccess) {  // the pool's idle blocks first, then once more
			(void)hipGetLastError();
			release_all();
			e = pinned ? hipHostMalloc(&p, c, hipHostMallocDefault) : hipMalloc(&p, c);
		}
		HIP_OK(e);
		return { p, c, dev };
	}
	void put(void* p, size_t c, int dev)
	{
		if (!p)
			return;
		// the implicit synchronisation of the hipFree this replaces, on the
		// block's own device
		int cur = 0;
		(void)hipGetDevice(&cur);
		if (cur != dev)
			(void)hipSetDevice(dev);
		const bool synced = hipDeviceSynchronize() == hipSuccess;
		if (cur != dev)
			(void)hipSetDevice(cur);
		if (c > POOL_MAX || c != size_class(c) || !synced) {
			raw_free(p);
			return;
		}
		std::lock_guard<std::mutex> l(mu);
		if (kept + c > keep_limit()) {
			raw_free(p);
			return;
		}
		free.emplace_back(pinned ? 0 : dev, c, p);
		kept += c;
	}
	void release_all()
	{
		std::lock_guard<std::mutex> l(mu);
		int cur = 0;
		(void)hipGetDevice(&cur);
		for (auto& f : free) {
			if (!pinned)
				(void)hipSetDevice(std::get<0>(f));
			raw_free(std::get<2>(f));
		}
		if (!pinned)
			(void)hipSetDevice(cur);
		free.clear();
		kept = 0;
	}
};
static MemPool& dev_pool()
{
	static MemPool* p = new MemPool(false);  // never destroyed: process lifetime
	return *p;
}
static MemPool& pin_pool()
{
	static MemPool* p = new MemPool(true);
	return *p;
}

template <class T>
struct DevBuf {
	T* p = nullptr;
	size_t n = 0;      // elements
	size_t bytes = 0;  // the block's usable bytes
	int dev = 0;       // the device it was allocated on
	DevBuf() = default;
	DevBuf(const DevBuf&) = delete;
	DevBuf& operator=(const DevBuf&) = delete;
	~DevBuf() { release(); }
	void release()
	{
		if (p)
			dev_pool().put(p, bytes, dev);
		p = nullptr;
		n = bytes = 0;
	}
	void reserve(size_t count)
	{
		if (count <= n && p)
			return;
		release();
		const auto b = dev_pool().get(std::max<size_t>(count, 1) * sizeof(T) + 64);
		p = static_cast<T*>(b.p);
		bytes = b.bytes;
		dev = b.dev;
		n = count;
	}
};

// Pinned host memory, grow-only (the facade's output staging).
struct PinBuf {
	uint8_t* p = nullptr;
	size_t n = 0, bytes = 0;
	int dev = 0;  // the device current when it was taken (synced on release)
	PinBuf() = default;
	PinBuf(const PinBuf&) = delete;
	PinBuf& operator=(const PinBuf&) = delete;
	~PinBuf() { pin_pool().put(p, bytes, dev); }
	void reserve(size_t count)
	{
		if (count <= n && p)
			return;
		pin_pool().put(p, bytes, dev);
		p = nullptr;
		n = bytes = 0;
		const auto b = pin_pool().get(std::max<size_t>(count, 1));
		p = static_cast<uint8_t*>(b.p);
		bytes = b.bytes;
		dev = b.dev;
		n = count;
	}
	void swap(PinBuf& o)
	{
		std::swap(p, o.p);
		std::swap(n, o.n);
		std::swap(bytes, o.bytes);
		std::swap(dev, o.dev);
	}
};

// The facade's streams and event, reused across contexts.
struct StreamSet {
	int device = -1;
	hipStream_t stream = nullptr, side = nullptr;
	hipEvent_t ev = nullptr;
};
static std::mutex g_stream_mu;
static std::vector<StreamSet>& stream_pool()
{
	static std::vector<StreamSet>* v = new std::vector<StreamSet>;  // process lifetime
	return *v;
}

// One long-lived helper thread running one job at a time (the facade's
// content checksum of a large block while the caller feeds the next one);
// wait() joins the current job.
struct Worker {
	std::thread th;
	std::mutex mu;
	std::condition_variable cv, done_cv;
	std::function<void()> job;
	bool busy = false, stop = false;
	Worker() = default;
	Worker(const Worker&) = delete;
	Worker& operator=(const Worker&) = delete;
	~Worker()
	{
		{
			std::lock_guard<std::mutex> l(mu);
			stop = true;
		}
		cv.notify_one();
		if (th.joinable())
			th.join();
	}
	void submit(std::function<void()> f)
	{
		wait();
		if (!th.joinable())
			th = std::thread([this] { loop(); });
		{
			std::lock_guard<std::mutex> l(mu);
			job = std::move(f);
			busy = true;
		}
		cv.notify_one();
	}
	void wait()
	{
		std::unique_lock<std::mutex> l(mu);
		done_cv.wait(l, [this] { return !busy; });
	}
	void loop()
	{
		std::unique_lock<std::mutex> l(mu);
		for (;;) {
			cv.wait(l, [this] { return (busy && job) || stop; });
			if (!(busy && job))
				return;  // stop, nothing pending
			std::function<void()> f = std::move(job);
			job = nullptr;
			l.unlock();
			f();
			l.lock();
			busy = false;
			done_cv.notify_all();
		}
	}
};

// ------------------------------------------------------------------ meta

enum Fmt { F_TBD, F_LEGACY, F_MODERN, F_BLOCK, F_SKIPPABLE };               // lz4ada.ads:355
enum Hps { NEED_MAGIC, NEED_MODERN, NEED_FLAGS, NEED_SKIP_LEN, HDR_DONE };  // lz4ada.ads:356

constexpr uint32_t MAGIC_MODERN = 0x184d2204u;  // lz4ada.ads:348-353
constexpr uint32_t MAGIC_LEGACY = 0x184c2102u;
constexpr uint32_t MAGIC_SKIP_LO = 0x184d2a50u, MAGIC_SKIP_HI = 0x184d2a5fu;

struct Meta {  // Decompressor_Meta, lz4ada.ads:359-370
	int is_format = F_TBD;
	int header_parsing = NEED_MAGIC;
	int memory_reservation = LZ4ADA_FOR_ALL;
	int content_checksum_length = 0;
	int block_checksum_length = 0;
	int status_eof = LZ4ADA_EOF_NO;
	int64_t input_buffer_filled = 0;
	bool is_compressed = false;
	bool has_content_size = false;
	uint64_t size_remaining = 4;
	// frame descriptor facts the reference does not keep (bulk path)
	uint8_t flg = 0, bd = 0;
};

static bool concrete(int r) { return r >= LZ4ADA_SZ_64_KIB && r <= LZ4ADA_SZ_8_MIB; }

static int64_t block_size_of(int r)  // Get_Block_Size, lz4ada.adb:65-77
{
	static const int64_t lut[] = { 64 << 10, 256 << 10, 1 << 20, 4 << 20, 8 << 20 };
	return lut[r];
}

static void check_reservation(int requested, int& effective)  // lz4ada.adb:241-260
{
	if (concrete(requested)) {
		if (effective > requested)
			raise(LZ4ADA_TOO_LITTLE_MEMORY,
			      std::string("LZ4 header requres reservation ") + RES_IMAGE[effective] +
			              ", but API call requested that only " + RES_IMAGE[requested] +
			              " be used. This frame cannot be processed under the given "
			              "constraints.");
		effective = requested;
	}
}

static void legacy_end_of_header(Meta& m)  // lz4ada.adb:225-239
{
	int eff = LZ4ADA_FOR_LEGACY;
	m.input_buffer_filled = 0;
	m.is_format = F_LEGACY;
	m.header_parsing = HDR_DONE;
	m.size_remaining = 0;
	m.status_eof = LZ4ADA_EOF_MAYBE;
	m.block_checksum_length = 0;
	m.content_checksum_length = 0;
	m.has_content_size = false;
	m.is_compressed = true;
	check_reservation(m.memory_reservation, eff);
	m.memory_reservation = eff;
}

static void header_magic(Meta& m, uint32_t magic)  // lz4ada.adb:199-223
{
	if (magic == MAGIC_MODERN) {
		m.is_format = F_MODERN;
		m.header_parsing = NEED_FLAGS;
		m.size_remaining = 2;
	} else if (magic == MAGIC_LEGACY) {
		legacy_end_of_header(m);
	} else if (magic >= MAGIC_SKIP_LO && magic <= MAGIC_SKIP_HI) {
		m.is_format = F_SKIPPABLE;
		m.header_parsing = NEED_SKIP_LEN;
		m.size_remaining = 4;
		m.block_checksum_length = 0;
		m.content_checksum_length = 0;
	} else {
		raise(LZ4ADA_NOT_SUPPORTED, "Invalid or unsupported magic: 0x" + hex32(magic));
	}
}

static void header_flags(Meta& m, const uint8_t* hb)  // lz4ada.adb:262-328
{
	const uint8_t flg = hb[4], bd = hb[5];
	const unsigned version = (flg & 0xc0u) >> 6, bmax = (bd & 0x70u) >> 4;
	if (version != 1)
		raise(LZ4ADA_NOT_SUPPORTED, "Only LZ4 frame format version 01 supported. Detected 0x" +
		                                    hex8(version) + " instead.");
	if ((flg & 2u) || (bd & 0x8fu))
		raise(LZ4ADA_NOT_SUPPORTED,
		      "Found reserved bits /= 0. Data might be too new to be processed by this "
		      "implementation!");
	m.status_eof = LZ4ADA_EOF_NO;
	int required;
	switch (bmax) {
	case 4: required = LZ4ADA_SZ_64_KIB; break;
	case 5: required = LZ4ADA_SZ_256_KIB; break;
	case 6: required = LZ4ADA_SZ_1_MIB; break;
	case 7: required = LZ4ADA_SZ_4_MIB; break;
	default: raise(LZ4ADA_NOT_SUPPORTED, "Unknown maximum block size flag: 0x" + hex8(bmax));
	}
	m.flg = flg;
	m.bd = bd;
	m.block_checksum_length = (flg & 16u) ? 4 : 0;
	m.content_checksum_length = (flg & 4u) ? 4 : 0;
	m.has_content_size = (flg & 8u) != 0;
	m.header_parsing = NEED_MODERN;
	m.size_remaining = 1 + (m.has_content_size ? 8 : 0) + ((flg & 1u) ? 4 : 0);
	check_reservation(m.memory_reservation, required);
	if (m.memory_reservation != LZ4ADA_SINGLE_FRAME)
		m.memory_reservation = required;
}

static void header_modern_end(Meta& m, const uint8_t* hb)  // lz4ada.adb:330-361
{
	const uint8_t hc = hb[m.input_buffer_filled - 1];
	if (m.has_content_size)
		m.size_remaining = load64(hb + 6);
	const uint8_t computed =
	        uint8_t((descriptor_xxh32(hb + 4, size_t(m.input_buffer_filled - 1 - 4)) >> 8) & 0xffu);
	if (hc != computed)
		raise(LZ4ADA_CHECKSUM_ERROR, "Computed Header Checksum 0x" + hex8(computed) +
		                                     " does not match expected Header Checksum 0x" +
		                                     hex8(hc));
	m.header_parsing = HDR_DONE;
	m.input_buffer_filled = 0;
}

// Process_Header_Bytes (lz4ada.adb:155-191)
static int64_t header_bytes(Meta& m, uint8_t* hb, const uint8_t* in, int64_t len)
{
	const int64_t copy = std::min<int64_t>(len, int64_t(m.size_remaining));
	if (!(copy > 0))
		raise(LZ4ADA_ASSERTION_ERROR, "lz4ada.adb:161");
	memcpy(hb + m.input_buffer_filled, in, size_t(copy));
	m.input_buffer_filled += copy;
	m.size_remaining -= uint64_t(copy);
	if (m.size_remaining == 0) {
		switch (m.header_parsing) {
		case NEED_MAGIC: header_magic(m, load32(hb)); break;
		case NEED_FLAGS: header_flags(m, hb); break;
		case NEED_MODERN: header_modern_end(m, hb); break;
		case NEED_SKIP_LEN:
			m.memory_reservation = LZ4ADA_SZ_64_KIB;  // quirk Q3
			m.header_parsing = HDR_DONE;
			m.size_remaining = load32(hb + 4);
			m.status_eof = m.size_remaining == 0 ? LZ4ADA_EOF_YES : LZ4ADA_EOF_NO;
			m.input_buffer_filled = 0;
			break;
		default:
			raise(LZ4ADA_CONSTRAINT_ERROR,
			      "Header_Complete case must not be reached while processing header bytes. "
			      "Library bug detected.");
		}
	}
	return copy;
}

static bool is_any_magic(uint32_t v)
{
	return v == MAGIC_MODERN || v == MAGIC_LEGACY || (v >= MAGIC_SKIP_LO && v <= MAGIC_SKIP_HI);
}

// XXHash32.Update / Final (lz4ada.adb:942-1017) on host bytes the GPU
// decoded (content checksums: the facade's Hash_All_Data and the bulk
// path's pipeline).  The state layout is the one the GPU kernel
// k_xxh32_update advances, so the two can continue each other.
static inline uint32_t rotl32h(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t xxh_round(uint32_t acc, uint32_t w) { return rotl32h(acc + w * P2, 13) * P1; }

static void host_xxh32_update(lz4ada_xxh32_state& h, const uint8_t* p, size_t n)
{
	h.total_length += n;
	size_t bs = size_t(h.buffer_size);
	if (bs + n < 16) {
		if (n)
			memcpy(h.buffer + bs, p, n);
		h.buffer_size = int32_t(bs + n);
		return;
	}
	if (bs) {  // complete the buffered stripe (Update1, :965-991)
		const size_t k = 16 - bs;
		memcpy(h.buffer + bs, p, k);
		p += k;
		n -= k;
		for (int i = 0; i < 4; ++i)
			h.state[i] = xxh_round(h.state[i], load32(h.buffer + 4 * i));
	}
	uint32_t v0 = h.state[0], v1 = h.state[1], v2 = h.state[2], v3 = h.state[3];
	for (; n >= 16; p += 16, n -= 16) {  // stripes (Process, :951-958)
		v0 = xxh_round(v0, load32(p));
		v1 = xxh_round(v1, load32(p + 4));
		v2 = xxh_round(v2, load32(p + 8));
		v3 = xxh_round(v3, load32(p + 12));
	}
	h.state[0] = v0;
	h.state[1] = v1;
	h.state[2] = v2;
	h.state[3] = v3;
	if (n)
		memcpy(h.buffer, p, n);
	h.buffer_size = int32_t(n);
}

static uint32_t host_xxh32_final(const lz4ada_xxh32_state& h)  // :993-1017
{
	uint32_t acc = h.total_length >= 16 ? rotl32h(h.state[0], 1) + rotl32h(h.state[1], 7) +
	                                          rotl32h(h.state[2], 12) + rotl32h(h.state[3], 18)
	                                    : h.state[2] + P5;
	acc += uint32_t(h.total_length);
	const uint8_t* p = h.buffer;
	size_t n = size_t(h.buffer_size);
	for (; n >= 4; p += 4, n -= 4)
		acc = rotl32h(acc + load32(p) * P3, 17) * P4;
	for (; n; ++p, --n)
		acc = rotl32h(acc + uint32_t(*p) * P5, 11) * P1;
	acc ^= acc >> 15;
	acc *= P2;
	acc ^= acc >> 13;
	acc *= P3;
	acc ^= acc >> 16;
	return acc;
}

// Device status of a decode kernel -> the reference's exception.
[[noreturn]] static void raise_device_status(const SerialState& s)
{
	switch (s.code) {
	case DS_OFFSET0: raise(LZ4ADA_DATA_CORRUPTION, "Corrupted Block: Offset = 0 detected.");
	case DS_ML_AFTER_LIT:
		raise(LZ4ADA_DATA_CORRUPTION,
		      "Match_Length=" + img(s.aux) +
		              " suggests compressed data but this sequence already ends after the "
		              "literals. This might also happen with an untypical encoder?");
	case DS_LIT_OVERRUN:
		raise(LZ4ADA_DATA_CORRUPTION, "Corrupted Block: literal run exceeds the end of the block.");
	case DS_TRUNCATED:
		raise(LZ4ADA_DATA_CORRUPTION,
		      "Corrupted Block: sequence truncated at the end of the block.");
	case DS_OUT_OVERFLOW:
		raise(LZ4ADA_DATA_CORRUPTION,
		      "Corrupted Block: decompressed data exceeds the output buffer.");
	case DS_BACKREF:
		raise(LZ4ADA_DATA_CORRUPTION, "Backreference location out of range. Read from offset " +
		                                      img(s.detail) +
		                                      " not possible (earliest available index is 0).");
	case DS_CONTENT_SIZE:
		raise(LZ4ADA_DATA_CORRUPTION,
		      "Produced content size exceeds declared content size. The supplied data is "
		      "inconsistent.");
	default: raise(LZ4ADA_CONSTRAINT_ERROR, "unexpected device status " + std::to_string(s.code));
	}
}

}  // namespace lz4ada

using namespace lz4ada;

// ----------------------------------------------------------- Decompressor

namespace lz4ada {
// A few large blocks: one block at a time through the lone-block decoder
// (lz4ada_lone.hip, the whole GPU per block: ~0.4 ms per 4 MiB mixed block)
// beats the bulk decoder's one wave per block (~13 ms per 4 MiB block, at
// any count up to the chip's 2,048 resident waves) below ~30 blocks.
static bool few_large_blocks(const std::vector<lz4ada_block_desc>& d)
{
	static const bool off = getenv("LZ4ADA_NO_LONE") != nullptr;
	if (off || d.empty() || d.size() > 24)
		return false;
	uint32_t mx = 0;
	for (const auto& x : d)
		mx = std::max(mx, x.in_len);
	return mx >= (512u << 10);
}
static bool decode_lone_blocks(const uint8_t* host_in, const uint8_t* d_in,
                               const std::vector<lz4ada_block_desc>& d, uint8_t* d_out,
                               lz4ada_block_status* d_st, std::vector<lz4ada_block_status>& st,
                               DevBuf<uint8_t>& scr, hipStream_t stream);
enum BulkResult { BULK_OK, BULK_EXACT, BULK_PRE_REF, BULK_FAIL_AT };
// Where a linked batch's resolved bytes go: dst(n) returns the device
// buffer for the batch's n bytes (nullptr: no room), done(p, n) runs once
// they are there.
struct LinkedSink {
	std::function<uint8_t*(int64_t)> dst;
	std::function<void(const uint8_t*, int64_t)> done;
};

// A linked batch that starts mid-frame (the facade's read-ahead): the
// history before its first block, as device bytes oldest first (the
// reference's Buffer keeps it in two places), and the reference's
// Output_Pos / Output_Pos_History there (quirk D1).
struct LinkedHist {
	const uint8_t* h0 = nullptr;
	int64_t n0 = 0;
	const uint8_t* h1 = nullptr;
	int64_t n1 = 0;
	int64_t output_pos = 0, output_pos_history = 0;
};
static BulkResult bulk_linked(const uint8_t* d_frame, uint64_t frame_len, int64_t block_max,
                              const std::vector<lz4ada_block_desc>& descs, LinkedSink& sink,
                              uint64_t& total, std::vector<uint32_t>& lens, int64_t& fail,
                              hipStream_t stream, const LinkedHist* hist = nullptr);
}  // namespace lz4ada

struct lz4ada_decompressor {
	Meta m;
	bool is_at_end_mark = false;
	std::vector<uint8_t> input_buffer;  // Input_Buffer(0 .. In_Last)
	int64_t output_pos = 0;
	int64_t output_pos_history = 0;
	int64_t input_length = -1;
	std::string err;
	int64_t exact_blocks = 0;  // blocks decoded by the reference-exact serial kernel (diagnostics)

	// device side (lazily created at the first block)
	bool dev_ready = false;
	// check the next block's checksum before launching the speculative
	// decode (the block a bulk path stopped at: a decode of a corrupted
	// payload may be long, and would have to finish before the raise)
	bool checksum_first = false;
	int device = -1;
	hipStream_t stream = nullptr;
	DevBuf<uint8_t> d_buf;  // mirror of the caller's Buffer (history lives here)
	int64_t d_buf_len = 0;
	DevBuf<uint8_t> d_blk;
	lz4ada_xxh32_state hash_all{};  // Hash_All_Data, over the bytes the GPU decoded
	// A large block's content hash runs on a helper thread while the caller
	// feeds the next block, over the pinned staging copy of its output (our
	// memory, so the caller may reuse its Buffer); every reader of hash_all
	// joins it first.  The staging ping-pongs: a block handed to the hasher
	// leaves in stage_hashed, so the next block's copy never waits for it
	// (the hasher runs one job at a time, and submit() joins the previous one).
	Worker hasher;
	void hash_wait() { hasher.wait(); }
	PinBuf stage;  // a block's output on its way to the caller's Buffer
	PinBuf stage_hashed;  // the staging the hasher may be reading
	PinBuf stage_st;  // its status
	std::vector<uint8_t> blk_tmp;  // a block assembled from cached + new input
	DevBuf<lz4ada_xxh32_state> d_tmp_hash;
	DevBuf<SerialState> d_serial;
	DevBuf<lz4ada_block_desc> d_desc;  // one-block fast path
	DevBuf<lz4ada_block_status> d_bst;
	DevBuf<uint8_t> d_scr;  // its output, until the block checksum has passed
	DevBuf<uint8_t> d_lone;  // the lone-block decoder's tables and words
	hipStream_t side = nullptr;  // the block checksum, beside the fast decode
	hipEvent_t ev_in = nullptr;

	// Read-ahead: when one Update call hands over several
	// complete blocks, they are decoded together by the bulk decoder and
	// then served one per call, as the reference returns them.
	struct Ahead {
		std::vector<uint8_t> input;  // the batch's compressed bytes (identity check)
		std::vector<lz4ada_block_desc> descs;
		std::vector<lz4ada_block_status> st;
		DevBuf<uint8_t> d_in, d_out, d_lone;
		DevBuf<lz4ada_block_desc> d_desc;
		DevBuf<lz4ada_block_status> d_st;
		uint64_t slot = 0;
		size_t next = 0;  // next block to serve
		void clear()
		{
			descs.clear();
			st.clear();
			next = 0;
		}
	} ahead;
	int64_t linked_cap = int64_t(512) << 20;  // input bytes of a linked read-ahead batch

	lz4ada_decompressor() { lz4ada_xxh32_reset(&hash_all, 0); }
	~lz4ada_decompressor()
	{
		hash_wait();
		if (!stream)
			return;
		// idle streams go back to the pool for the next context
		const bool idle = hipStreamSynchronize(side) == hipSuccess && hipStreamSynchronize(stream) == hipSuccess;
		if (idle) {
			std::lock_guard<std::mutex> l(g_stream_mu);
			stream_pool().push_back(StreamSet{ device, stream, side, ev_in });
		} else {
			(void)hipStreamDestroy(side);
			(void)hipEventDestroy(ev_in);
			(void)hipStreamDestroy(stream);
		}
	}

	void ensure_device()
	{
		if (dev_ready)
			return;
		device_check_or_raise();
		HIP_OK(hipGetDevice(&device));
		{
			std::lock_guard<std::mutex> l(g_stream_mu);
			auto& pool = stream_pool();
			for (size_t i = 0; i < pool.size(); ++i)
				if (pool[i].device == device) {
					stream = pool[i].stream;
					side = pool[i].side;
					ev_in = pool[i].ev;
					pool[i] = pool.back();
					pool.pop_back();
					break;
				}
		}
		if (!stream) {
			HIP_OK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
			HIP_OK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
			HIP_OK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
		}
		d_tmp_hash.reserve(1);
		d_serial.reserve(1);
		d_desc.reserve(1);
		d_bst.reserve(1);
		dev_ready = true;
	}

	void reset_content_hash()  // XXHash32.Reset(0)
	{
		hash_wait();
		lz4ada_xxh32_reset(&hash_all, 0);
	}

	// ---------------------------------------------------- Update pieces
	void reset_outer()  // lz4ada.adb:451-461
	{
		ahead.clear();
		is_at_end_mark = false;
		input_length = -1;
		output_pos = 0;
		output_pos_history = 0;
		reset_content_hash();
	}

	int64_t reset_for_next_frame(const uint8_t* in, int64_t len)  // :435-449
	{
		if (m.memory_reservation == LZ4ADA_SINGLE_FRAME)
			raise(LZ4ADA_DATA_CORRUPTION,
			      "Requested Single_Frame operation but data was provided after End of Frame "
			      "was detected");
		m.status_eof = LZ4ADA_EOF_NO;
		m.header_parsing = NEED_MAGIC;
		m.size_remaining = 4;
		reset_outer();
		return header_bytes(m, input_buffer.data(), in, len);
	}

	int64_t skip(const uint8_t* in, int64_t len)  // :420-433
	{
		const uint64_t remain = m.size_remaining;
		const uint64_t cons = std::min<uint64_t>(uint64_t(len), remain);
		if (m.status_eof == LZ4ADA_EOF_YES && cons == 0)
			return reset_for_next_frame(in, len);
		m.size_remaining = remain - cons;
		m.status_eof = m.size_remaining == 0 ? LZ4ADA_EOF_YES : LZ4ADA_EOF_NO;
		return int64_t(cons);
	}

	void frame_has_ended()  // :465-477
	{
		m.status_eof = LZ4ADA_EOF_YES;
		m.input_buffer_filled = 0;
		if (m.has_content_size && m.size_remaining != 0)
			raise(LZ4ADA_DATA_CORRUPTION,
			      "Frame has ended, but according to content size, there should be " +
			              img_u(m.size_remaining) + " bytes left to output.");
	}

	uint32_t content_hash_final()
	{
		hash_wait();
		return host_xxh32_final(hash_all);
	}

	void check_end_mark(const uint8_t* in, int64_t len, int64_t& consumed)  // :463-523
	{
		const int64_t provided = len - consumed;
		const int64_t required = m.content_checksum_length - m.input_buffer_filled;
		if (m.content_checksum_length == 0 || m.status_eof == LZ4ADA_EOF_YES || required <= 0) {
			if (m.status_eof == LZ4ADA_EOF_YES) {
				if (consumed != 0)
					raise(LZ4ADA_ASSERTION_ERROR, "lz4ada.adb:486");
				consumed = reset_for_next_frame(in, len);
			} else {
				frame_has_ended();
			}
		} else if (provided >= required) {
			uint8_t tmp[8];
			memcpy(tmp, input_buffer.data(), size_t(m.input_buffer_filled));
			memcpy(tmp + m.input_buffer_filled, in + consumed, size_t(required));
			const uint32_t declared = load32(tmp);
			const uint32_t computed = content_hash_final();
			consumed += required;
			if (declared != computed)
				raise(LZ4ADA_CHECKSUM_ERROR, "Computed content checksum 0x" + hex32(computed) +
				                                     " does not match declared content checksum 0x" +
				                                     hex32(declared) + ".");
			frame_has_ended();
		} else {
			memcpy(input_buffer.data() + m.input_buffer_filled, in + consumed, size_t(provided));
			m.input_buffer_filled += provided;
			consumed += provided;
		}
	}

	int64_t try_detect_input_length(const uint8_t* in, int64_t len)  // :525-585
	{
		const int64_t additional = BLOCK_SIZE_BYTES + m.block_checksum_length;
		const int64_t n = std::min<int64_t>(BLOCK_SIZE_BYTES - m.input_buffer_filled, len);
		memcpy(input_buffer.data() + m.input_buffer_filled, in, size_t(n));
		m.input_buffer_filled += n;
		if (m.input_buffer_filled == BLOCK_SIZE_BYTES) {
			uint32_t word = load32(input_buffer.data());
			if (m.is_format == F_MODERN && word == 0) {
				is_at_end_mark = true;
				m.input_buffer_filled = 0;
			} else if (m.is_format == F_LEGACY && is_any_magic(word)) {
				if (m.memory_reservation == LZ4ADA_SINGLE_FRAME)
					raise(LZ4ADA_DATA_CORRUPTION,
					      "Requested Single_Frame operation but data provided what looks "
					      "like the beginning of another frame.");
				reset_outer();
				header_magic(m, word);
			} else {
				if (m.is_format == F_MODERN) {
					m.is_compressed = (word & 0x80000000u) == 0;
					word &= 0x7ffffffu;  // 27-bit mask, quirk Q2
				}
				input_length = int64_t(word);
				if (input_length + additional > int64_t(input_buffer.size())) {
					input_length = -1;
					raise(LZ4ADA_DATA_CORRUPTION,
					      "Declared maximum data length exceeded. Buffer has " +
					              img(int64_t(input_buffer.size())) +
					              " bytes, current block requires " + img_u(word) +
					              " bytes + " + img(additional) + " bytes for metadata.");
				}
			}
		}
		return n;
	}

	void grow_mirror(int64_t buflen)  // the Buffer mirror, keeping history
	{
		DevBuf<uint8_t> nb;
		nb.reserve(size_t(buflen));
		HIP_OK(hipMemsetAsync(nb.p, 0, size_t(buflen), stream));
		if (d_buf_len)
			HIP_OK(hipMemcpyAsync(nb.p, d_buf.p, size_t(d_buf_len), hipMemcpyDeviceToDevice,
			                      stream));
		HIP_OK(hipStreamSynchronize(stream));
		std::swap(nb.p, d_buf.p);
		std::swap(nb.n, d_buf.n);
		std::swap(nb.bytes, d_buf.bytes);
		d_buf_len = buflen;
	}

	// Decode_Full_Block_With_Trailer (lz4ada.adb:661-714) on the GPU.
	void decode_full_block(const uint8_t* blk, int64_t blen, uint8_t* buf, int64_t buflen,
	                       int64_t& first, int64_t& last)
	{
		ensure_device();
		const int bcl = m.block_checksum_length;
		const int64_t raw_len = blen - bcl;
		if (buflen > d_buf_len)
			grow_mirror(buflen);
		static const bool trace = getenv("LZ4ADA_TRACE_FACADE") != nullptr;
		auto t0 = std::chrono::steady_clock::now();
		auto phase = [&](const char* name) {
			if (!trace)
				return;
			const auto t1 = std::chrono::steady_clock::now();
			fprintf(stderr, "[facade] %-8s %8.3f ms\n", name,
			        std::chrono::duration<double, std::milli>(t1 - t0).count());
			t0 = t1;
		};
		d_blk.reserve(size_t(std::max<int64_t>(blen, 1)));
		// Check_Checksum comes before decoding (:672-676, quirk Q8).  The
		// payload is host memory here: its XXH32 runs on this thread (one
		// serial chain, ~10x the GPU chain's rate) while the GPU decodes
		// into a scratch slot; the mirror takes the output only once the
		// checksum has passed.  A block known to fail (the bulk path stopped
		// at it) is checked before anything is launched.
		auto check = [&] { return block_checksum(blk, blen); };
		if (checksum_first && bcl > 0) {
			checksum_first = false;
			const auto c = check();
			if (!c.first)
				raise(LZ4ADA_CHECKSUM_ERROR, c.second);
		}
		if (blen > 0)
			HIP_OK(hipMemcpyAsync(d_blk.p, blk, size_t(blen), hipMemcpyHostToDevice, stream));
		phase("h2d");
		const LoneResult lr = lone_block(blk, blen, buf, buflen, first, last);
		phase("lone");
		if (lr == LONE_DONE)
			return;
		const int64_t fast_start = lr == LONE_DECLINED ? -1 : launch_fast_block(raw_len, blen, buflen);
		if (bcl > 0 && lr != LONE_DECLINED) {
			const auto c = check();
			phase("cksum");
			if (!c.first) {
				HIP_OK(hipStreamSynchronize(stream));  // the scratch decode, discarded
				raise(LZ4ADA_CHECKSUM_ERROR, c.second);
			}
		}
		if (fast_start >= 0 && finish_fast_block(fast_start, first, last)) {
			phase("decode");
			deliver(buf, first, last);
			phase("deliver");
			return;
		}
		SerialState s{};
		s.output_pos = output_pos;
		s.output_pos_history = output_pos_history;
		s.size_remaining = m.size_remaining;
		s.has_content_size = m.has_content_size ? 1 : 0;
		HIP_OK(hipMemcpyAsync(d_serial.p, &s, sizeof s, hipMemcpyHostToDevice, stream));
		++exact_blocks;
		HIP_OK(launch_serial_block(d_buf.p, buflen, d_blk.p, raw_len,
		                           m.is_compressed ? raw_len : blen, m.is_compressed ? 1 : 0,
		                           d_serial.p, stream));
		HIP_OK(hipMemcpyAsync(&s, d_serial.p, sizeof s, hipMemcpyDeviceToHost, stream));
		HIP_OK(hipStreamSynchronize(stream));
		// state changes before a raise persist, as with the Ada record
		output_pos = s.output_pos;
		output_pos_history = s.output_pos_history;
		if (m.has_content_size)
			m.size_remaining = s.size_remaining;
		if (s.code != DS_OK)
			raise_device_status(s);
		first = s.first;
		last = s.last;
		deliver(buf, first, last);
	}

	// The block's output, in the Buffer mirror at [first, last], to the
	// caller's Buffer, and into the content checksum (Update_Checksum,
	// :709-714) on the way.
	void deliver(uint8_t* buf, int64_t first, int64_t last)
	{
		const int64_t nout = last - first + 1;
		if (nout <= 0)
			return;
		static const bool trace = getenv("LZ4ADA_TRACE_FACADE") != nullptr;
		const auto t0 = std::chrono::steady_clock::now();
		stage.reserve(size_t(nout));
		HIP_OK(hipMemcpyAsync(stage.p, d_buf.p + first, size_t(nout), hipMemcpyDeviceToHost, stream));
		HIP_OK(hipStreamSynchronize(stream));
		const auto t1 = std::chrono::steady_clock::now();
		to_caller(buf + first, nout);
		if (trace)
			fprintf(stderr, "[facade]   d2h %.3f ms, content hash %.3f ms\n",
			        std::chrono::duration<double, std::milli>(t1 - t0).count(),
			        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1)
			                .count());
	}

	// The staged output (stage.p, nout bytes) to the caller's Buffer and into
	// the content checksum -- on the helper thread for a large block.
	void to_caller(uint8_t* dst, int64_t nout)
	{
		memcpy(dst, stage.p, size_t(nout));
		if (m.content_checksum_length == 0)
			return;
		const uint8_t* p = stage.p;
		if (nout >= (int64_t(64) << 10)) {
			hasher.submit([this, p, nout] { host_xxh32_update(hash_all, p, size_t(nout)); });
			stage.swap(stage_hashed);
		} else {
			hash_wait();  // the previous block's share first
			host_xxh32_update(hash_all, p, size_t(nout));
		}
	}

	// A lone block is latency-bound: the lone-block decoder (every step
	// parallel over the block's bytes, lz4ada_lone.hip) decodes a 4 MiB mixed
	// block in ~0.2 ms against ~21 ms for k_decode_pc's one workgroup
	// (tools/lone_time.py).  Below LONE_MIN compressed bytes k_decode_pc's
	// single launch wins (16 KiB mixed blocks, 8 KB compressed: lone 0.051 ms,
	// pc 0.090; pc's time grows with the block, lone's ~0.045 ms floor is its
	// five launches).  LZ4ADA_FACADE_DECODER=pc / lone forces one.
	static constexpr int64_t LONE_MIN = 6 << 10;
	static int facade_variant()
	{
		const char* e = getenv("LZ4ADA_FACADE_DECODER");
		if (e && !strcmp(e, "pc"))
			return DEC_PC;
		if (e && !strcmp(e, "lone"))
			return -2;  // the lone-block decoder at every size
		return -1;  // lone (large blocks), else k_decode_pc
	}

	// Decompress_Full_Block through the bulk decoder for one block, into a
	// scratch slot; a clean result moves to the Buffer mirror at the
	// position the reference would use.  Any status but OK -- including a
	// reference before the block start, which only the exact path resolves
	// (history scheme, D1) -- or a content-size overrun leaves the block to
	// k_serial_block, which redoes it from the same state on an untouched
	// mirror.  launch_fast_block enqueues the decode and returns the block's
	// Output_Pos (-1: not tried); finish_fast_block waits for it.
	// The output room a decoder slot needs for one block: what the Buffer
	// leaves, but no more than the frame's block maximum (BD for modern
	// frames, 8 MiB for legacy ones, lz4ada.adb:65-77, 225-239) or 255 bytes
	// per payload byte.  A block that would decode to more is the exact
	// path's (the reference bounds it by the Buffer alone, D5) -- so a large
	// caller Buffer never sizes the device scratch.
	int64_t block_room(int64_t buflen_left, int64_t raw_len, bool compressed) const
	{
		int64_t cap = std::min<int64_t>(buflen_left, INT32_MAX);
		if (compressed)
			cap = std::min<int64_t>(cap, 255 * std::max<int64_t>(raw_len, 1) + 16);
		else
			cap = std::min<int64_t>(cap, raw_len);
		if (m.is_format == F_MODERN)
			cap = std::min<int64_t>(cap, int64_t(1) << (8 + 2 * ((m.bd & 0x70u) >> 4)));
		else if (m.is_format == F_LEGACY)
			cap = std::min<int64_t>(cap, int64_t(8) << 20);
		return cap;
	}

	// The history a block of a linked frame may read (lz4ada.adb:678-690,
	// 862-883) when it starts at Buffer position `start`: the current round's
	// bytes Buffer(0 .. start-1) (n1), and before them the previous round's
	// tail Buffer(OPH - n0 .. OPH - 1) -- up to 65535 bytes in all, the
	// largest offset.  Before the first round ends there is none beyond n1.
	void history_of(int64_t start, int64_t& n0, int64_t& n1) const
	{
		n1 = start;
		n0 = std::min<int64_t>(65535, start + output_pos_history) - n1;
	}
	// Quirk D1 can only strike right after a round that ended within the
	// reference's 8-byte wild copy of 64 KiB (lz4ada.adb:811-817, 862-879).
	bool d1_window() const
	{
		return output_pos_history >= HISTORY_SIZE && output_pos_history <= HISTORY_SIZE + 6;
	}

	std::pair<bool, std::string> block_checksum(const uint8_t* blk, int64_t blen) const
	{
		const int bcl = m.block_checksum_length;
		lz4ada_xxh32_state h;
		lz4ada_xxh32_reset(&h, 0);
		host_xxh32_update(h, blk, size_t(blen - bcl));
		const uint32_t got = host_xxh32_final(h);
		const uint32_t expect = load32(blk + blen - bcl);
		return std::make_pair(got == expect, "Declared checksum is 0x" + hex32(expect) +
		                                             ", but computed one is 0x" + hex32(got) + ".");
	}

	// A compressed block for the lone-block decoder: every block of a linked
	// frame (the reference's history as readable words in front of its
	// output), an independent frame's from LONE_MIN compressed bytes.  Its
	// two halves run around the host checksum (Check_Checksum before any
	// output, :672-676), and the emit writes straight into the mirror at the
	// reference's Output_Pos -- only when the block decoded cleanly, so a
	// decline (a reference past the history, D1 risk, a content-size or
	// slot overrun, anything the reference would reject) leaves the mirror
	// untouched for the exact path.  The status and the output come back in
	// one round trip through pinned staging.
	enum LoneResult { LONE_NOT_TAKEN, LONE_DONE, LONE_DECLINED };
	LoneResult lone_block(const uint8_t* blk, int64_t blen, uint8_t* buf, int64_t buflen, int64_t& first,
	                      int64_t& last)
	{
		const int bcl = m.block_checksum_length;
		const int64_t raw_len = blen - bcl;
		if (!m.is_compressed || raw_len <= 0 || raw_len > INT32_MAX || getenv("LZ4ADA_FACADE_EXACT"))
			return LONE_NOT_TAKEN;
		const bool linked = m.is_format == F_MODERN && !(m.flg & 0x20u);
		const int fv = facade_variant();
		if (!linked && !(fv < 0 && (raw_len >= LONE_MIN || fv == -2)))
			return LONE_NOT_TAKEN;
		const int64_t start = output_pos >= HISTORY_SIZE ? 0 : output_pos;  // :678-680
		if (buflen - start <= 0)
			return LONE_NOT_TAKEN;
		int64_t cap = block_room(buflen - start, raw_len, true);
		if (m.has_content_size)  // more output: the exact path raises mid-block, as the reference does
			cap = int64_t(std::min<uint64_t>(uint64_t(cap), m.size_remaining));
		if (cap <= 0 || cap > (int64_t(1) << 30))
			return LONE_NOT_TAKEN;
		int64_t n0 = 0, n1 = 0;
		if (linked)
			history_of(start, n0, n1);
		static const bool trace = getenv("LZ4ADA_TRACE_FACADE") != nullptr;
		auto t0 = std::chrono::steady_clock::now();
		auto lap = [&](const char* name) {
			if (!trace)
				return;
			const auto t1 = std::chrono::steady_clock::now();
			fprintf(stderr, "[facade]   lone %-7s %8.3f ms\n", name,
			        std::chrono::duration<double, std::milli>(t1 - t0).count());
			t0 = t1;
		};
		const int64_t sb = lone_scratch_bytes(raw_len, cap);
		d_lone.reserve(size_t(sb));
		HIP_OK(launch_decode_lone_parse(d_blk.p, raw_len, cap, d_bst.p, d_lone.p, sb, stream,
		                                linked ? d_buf.p + output_pos_history - n0 : nullptr, int32_t(n0),
		                                linked ? d_buf.p : nullptr, int32_t(n1),
		                                linked && d1_window() ? int(output_pos_history) : 0));
		lap("parse");
		if (bcl > 0) {
			const auto c = block_checksum(blk, blen);
			if (!c.first) {
				HIP_OK(hipStreamSynchronize(stream));
				raise(LZ4ADA_CHECKSUM_ERROR, c.second);
			}
		}
		lap("cksum");
		HIP_OK(launch_decode_lone_emit(raw_len, d_buf.p + start, cap, d_bst.p, d_lone.p, stream,
		                               int32_t(n0 + n1)));
		// the likely share of the output comes back with the status
		const int64_t spec = std::min<int64_t>(cap, std::max<int64_t>(4 * raw_len, int64_t(64) << 10));
		stage.reserve(size_t(cap));
		stage_st.reserve(sizeof(lz4ada_block_status));
		HIP_OK(hipMemcpyAsync(stage_st.p, d_bst.p, sizeof(lz4ada_block_status), hipMemcpyDeviceToHost,
		                      stream));
		HIP_OK(hipMemcpyAsync(stage.p, d_buf.p + start, size_t(spec), hipMemcpyDeviceToHost, stream));
		lap("enqueue");
		HIP_OK(hipStreamSynchronize(stream));
		lap("wait");
		lz4ada_block_status st;
		memcpy(&st, stage_st.p, sizeof st);
		if (st.code != DS_OK)
			return LONE_DECLINED;
		const int64_t nout = int64_t(st.out_len);
		if (nout > spec) {
			HIP_OK(hipMemcpyAsync(stage.p + spec, d_buf.p + start + spec, size_t(nout - spec),
			                      hipMemcpyDeviceToHost, stream));
			HIP_OK(hipStreamSynchronize(stream));
		}
		if (m.has_content_size)
			m.size_remaining -= uint64_t(nout);
		output_pos = start + nout;
		if (output_pos >= HISTORY_SIZE)  // :785-787
			output_pos_history = output_pos;
		first = start;
		last = start + nout - 1;
		if (nout > 0)
			to_caller(buf + first, nout);
		lap("deliver");
		return LONE_DONE;
	}

	int64_t launch_fast_block(int64_t raw_len, int64_t blen, int64_t buflen)
	{
		const bool linked = m.is_format == F_MODERN && !(m.flg & 0x20u);
		if (getenv("LZ4ADA_FACADE_EXACT"))
			return -1;
		const int64_t start = output_pos >= HISTORY_SIZE ? 0 : output_pos;  // :678-680
		if (buflen - start <= 0 || raw_len > INT32_MAX)
			return -1;
		const int64_t cap = std::max<int64_t>(block_room(buflen - start, raw_len, m.is_compressed), 1);
		if (linked && m.is_compressed)
			return -1;  // lone_block declined it: the exact path
		d_scr.reserve(size_t(cap));
		lz4ada_block_desc d{};
		d.in_off = 0;
		d.in_len = uint32_t(raw_len);
		d.flags = m.is_compressed ? 0u : LZ4ADA_BLOCK_STORED;
		d.out_off = 0;
		d.out_cap = uint32_t(cap);
		HIP_OK(hipMemcpyAsync(d_desc.p, &d, sizeof d, hipMemcpyHostToDevice, stream));
		HIP_OK(launch_decode_variant(d_blk.p, uint64_t(std::max<int64_t>(blen, 1)), d_desc.p, 1,
		                             d_scr.p, d_bst.p, DEC_PC, stream));
		return start;
	}

	bool finish_fast_block(int64_t start, int64_t& first, int64_t& last)
	{
		lz4ada_block_status st;
		HIP_OK(hipMemcpyAsync(&st, d_bst.p, sizeof st, hipMemcpyDeviceToHost, stream));
		HIP_OK(hipStreamSynchronize(stream));
		if (st.code != DS_OK)
			return false;
		const int64_t nout = int64_t(st.out_len);
		if (m.has_content_size && uint64_t(nout) > m.size_remaining)
			return false;  // the exact path raises mid-block, as the reference does
		if (m.has_content_size)
			m.size_remaining -= uint64_t(nout);
		if (nout > 0)  // deliver() reads it from the mirror, after this copy
			HIP_OK(hipMemcpyAsync(d_buf.p + start, d_scr.p, size_t(nout), hipMemcpyDeviceToDevice,
			                      stream));
		output_pos = start + nout;
		if (output_pos >= HISTORY_SIZE)  // :785-787 (:688-690 for stored blocks)
			output_pos_history = output_pos;
		first = start;
		last = start + nout - 1;
		return true;
	}

	// Decode the current block (payload at blk, `total` bytes with its
	// checksum) and every complete block after it in [blk, end), up to the
	// end mark, in one bulk launch.  False when fewer than two are there.
	bool build_ahead(const uint8_t* blk, int64_t total, const uint8_t* end, int64_t buflen)
	{
		ahead.clear();
		if (m.is_format != F_MODERN && m.is_format != F_LEGACY)
			return false;
		const bool linked = m.is_format == F_MODERN && !(m.flg & 0x20u);
		const int bcl = m.block_checksum_length;
		const int64_t avail = end - blk;
		// a slot holds one block: the Buffer's room, at most the block maximum
		// (block_room with the largest payload, so every block of the batch fits)
		const int64_t room = std::max<int64_t>(
		        block_room(buflen, m.is_format == F_LEGACY ? (int64_t(8) << 20) : (int64_t(4) << 20), true), 1);
		const uint64_t slot = (uint64_t(room) + 255) & ~uint64_t(255);
		const uint64_t max_blocks = std::max<uint64_t>(1, (uint64_t(2) << 30) / slot);
		auto add = [&](int64_t off, int64_t sz, bool stored) {
			lz4ada_block_desc d{};
			d.in_off = uint64_t(off);
			d.in_len = uint32_t(sz);
			d.flags = (stored ? LZ4ADA_BLOCK_STORED : 0u) | (bcl ? LZ4ADA_BLOCK_HAS_CKSUM : 0u);
			d.out_off = uint64_t(ahead.descs.size()) * slot;
			d.out_cap = uint32_t(room);
			d.cksum = bcl ? load32(blk + off + sz) : 0u;
			ahead.descs.push_back(d);
		};
		add(0, total - bcl, !m.is_compressed);
		int64_t pos = total;
		while (pos + BLOCK_SIZE_BYTES <= avail && ahead.descs.size() < max_blocks &&
		       pos < (linked ? linked_cap : (int64_t(512) << 20))) {
			uint32_t w = load32(blk + pos);
			bool stored = false;
			if (m.is_format == F_MODERN) {
				if (w == 0)
					break;  // end mark
				stored = (w & 0x80000000u) != 0;
				w &= 0x7ffffffu;
			} else if (is_any_magic(w)) {
				break;  // the next frame
			}
			const int64_t sz = int64_t(w);
			if (sz + BLOCK_SIZE_BYTES + bcl > int64_t(input_buffer.size()) ||
			    pos + BLOCK_SIZE_BYTES + sz + bcl > avail)
				break;  // the exact path reports it, or the rest comes later
			add(pos + BLOCK_SIZE_BYTES, sz, stored);
			pos += BLOCK_SIZE_BYTES + sz + bcl;
		}
		const size_t nb = ahead.descs.size();
		if (nb < 2) {
			ahead.clear();
			return false;
		}
		ahead.input.assign(blk, blk + pos);
		ahead.slot = slot;
		ahead.st.assign(nb, lz4ada_block_status{});
		ahead.d_in.reserve(size_t(pos));
		ahead.d_out.reserve(size_t(nb * slot));
		ahead.d_desc.reserve(nb);
		ahead.d_st.reserve(nb);
		HIP_OK(hipMemcpyAsync(ahead.d_in.p, blk, size_t(pos), hipMemcpyHostToDevice, stream));
		HIP_OK(hipMemcpyAsync(ahead.d_desc.p, ahead.descs.data(), nb * sizeof(lz4ada_block_desc),
		                      hipMemcpyHostToDevice, stream));
		HIP_OK(hipMemsetAsync(ahead.d_st.p, 0, nb * sizeof(lz4ada_block_status), stream));
		if (linked)
			return build_ahead_linked(nb, pos, buflen);
		if (few_large_blocks(ahead.descs) &&
		    decode_lone_blocks(blk, ahead.d_in.p, ahead.descs, ahead.d_out.p, ahead.d_st.p, ahead.st,
		                       ahead.d_lone, stream))
			return true;
		HIP_OK(hipMemsetAsync(ahead.d_st.p, 0, nb * sizeof(lz4ada_block_status), stream));
		if (bcl)
			HIP_OK(launch_block_checksums(ahead.d_in.p, ahead.d_desc.p, uint32_t(nb), ahead.d_st.p,
			                              stream));
		HIP_OK(launch_decode_blocks(ahead.d_in.p, uint64_t(pos), ahead.d_desc.p, uint32_t(nb),
		                            ahead.d_out.p, ahead.d_st.p, stream));
		HIP_OK(hipMemcpyAsync(ahead.st.data(), ahead.d_st.p, nb * sizeof(lz4ada_block_status),
		                      hipMemcpyDeviceToHost, stream));
		HIP_OK(hipStreamSynchronize(stream));
		return true;
	}

	// Read-ahead of a linked frame's blocks: all of them at once against
	// synthetic history, resolved on the GPU (bulk_linked, §7 of DESIGN),
	// seeded with the reference's history before the first one and its
	// Output_Pos / Output_Pos_History (quirk D1).  The blocks up to the
	// first one it cannot take are served; that one goes to the exact path.
	bool build_ahead_linked(size_t nb, int64_t in_len, int64_t buflen)
	{
		if (buflen > d_buf_len)
			grow_mirror(buflen);
		const int64_t start = output_pos >= HISTORY_SIZE ? 0 : output_pos;
		LinkedHist lh;
		history_of(start, lh.n0, lh.n1);
		lh.h0 = d_buf.p + output_pos_history - lh.n0;
		lh.h1 = d_buf.p;
		lh.output_pos = output_pos;
		lh.output_pos_history = output_pos_history;
		const int64_t bmax = int64_t(1) << (8 + 2 * ((m.bd & 0x70u) >> 4));
		int64_t room = 0;
		for (const auto& d : ahead.descs)
			room += std::max<int64_t>(d.out_cap, 1);
		ahead.d_out.reserve(size_t(room));
		int64_t used = 0;
		LinkedSink ls;
		ls.dst = [&](int64_t n) -> uint8_t* { return used + n <= room ? ahead.d_out.p + used : nullptr; };
		ls.done = [&](const uint8_t*, int64_t n) { used += n; };
		uint64_t total = 0;
		std::vector<uint32_t> lens;
		int64_t fail = -1;
		const BulkResult r = bulk_linked(ahead.d_in.p, uint64_t(in_len), bmax, ahead.descs, ls, total, lens,
		                                 fail, stream, &lh);
		HIP_OK(hipStreamSynchronize(stream));
		if (r != BULK_OK && r != BULK_FAIL_AT) {
			ahead.clear();
			return false;  // each block alone (lone decoder with history, else exact)
		}
		// A batch that stops early (quirk D1, an error) is decoded again from
		// the failing block on: the next batch is kept to about twice what this
		// one served, so frames with many such blocks are not re-decoded to
		// the end each time; a clean batch lets it grow back.
		if (r == BULK_OK) {
			linked_cap = std::min<int64_t>(int64_t(512) << 20, 2 * linked_cap);
		} else {
			int64_t served = 0;
			for (size_t k = 0; k < lens.size() && k < nb; ++k)
				served += int64_t(ahead.descs[k].in_len) + BLOCK_SIZE_BYTES + m.block_checksum_length;
			linked_cap = std::max<int64_t>(int64_t(1) << 20, 2 * served);
		}
		uint64_t off = 0;
		for (size_t k = 0; k < nb; ++k) {
			lz4ada_block_status& st = ahead.st[k];
			st = lz4ada_block_status{};
			if (k < lens.size()) {
				st.code = DS_OK;
				st.out_len = lens[k];
				st.cksum = ahead.descs[k].cksum;  // checked by bulk_linked
				ahead.descs[k].out_off = off;
				off += lens[k];
			} else {
				st.code = DS_RETRY;
			}
		}
		return true;
	}

	// Serve the current block from the read-ahead batch when it is the
	// batch's next block (same bytes) and decoded cleanly; the state moves
	// exactly as Decode_Full_Block_With_Trailer would move it.
	bool serve_ahead(const uint8_t* blk, int64_t total, const uint8_t* end, uint8_t* buf,
	                 int64_t buflen, int64_t& first, int64_t& last)
	{
		if (getenv("LZ4ADA_FACADE_EXACT"))
			return false;
		ensure_device();
		const int bcl = m.block_checksum_length;
		auto same = [&](size_t k) {
			const lz4ada_block_desc& d = ahead.descs[k];
			return int64_t(d.in_len) + bcl == total &&
			       memcmp(ahead.input.data() + d.in_off, blk, size_t(total)) == 0;
		};
		if (ahead.next >= ahead.descs.size() || !same(ahead.next)) {
			if (!build_ahead(blk, total, end, buflen))
				return false;
		}
		const size_t k = ahead.next++;
		const lz4ada_block_desc& d = ahead.descs[k];
		const lz4ada_block_status& st = ahead.st[k];
		const int64_t start = output_pos >= HISTORY_SIZE ? 0 : output_pos;  // :678-680
		const int64_t nout = int64_t(st.out_len);
		if (st.code != DS_OK || (bcl && st.cksum != d.cksum) || start + nout > buflen ||
		    (m.has_content_size && uint64_t(nout) > m.size_remaining)) {
			ahead.clear();  // the exact path takes this block (and reports it)
			return false;
		}
		if (buflen > d_buf_len)
			grow_mirror(buflen);
		const uint8_t* src = ahead.d_out.p + d.out_off;
		if (nout > 0) {  // the mirror keeps the history for a later exact block
			// a helper thread may still be hashing an earlier block's bytes in
			// this Buffer range (deliver() hands large blocks to it): join it
			// before the copy overwrites them
			hash_wait();
			HIP_OK(hipMemcpyAsync(d_buf.p + start, src, size_t(nout), hipMemcpyDeviceToDevice,
			                      stream));
			HIP_OK(hipMemcpyAsync(buf + start, src, size_t(nout), hipMemcpyDeviceToHost, stream));
			HIP_OK(hipStreamSynchronize(stream));
			if (m.content_checksum_length != 0)
				host_xxh32_update(hash_all, buf + start, size_t(nout));
		}
		if (m.has_content_size)
			m.size_remaining -= uint64_t(nout);
		output_pos = start + nout;
		if (output_pos >= HISTORY_SIZE)
			output_pos_history = output_pos;
		first = start;
		last = start + nout - 1;
		return true;
	}

	void cache_and_process(const uint8_t* in, int64_t len, int64_t& consumed, uint8_t* buf,
	                       int64_t buflen, int64_t& first, int64_t& last)  // :630-659
	{
		const int64_t avail = len - consumed;
		const int64_t want = input_length + m.block_checksum_length - m.input_buffer_filled +
		                     (m.is_format == F_BLOCK ? 0 : BLOCK_SIZE_BYTES);
		const int64_t fill = m.input_buffer_filled;
		const uint8_t* src = in + consumed;
		if (want > avail) {
			if (fill + avail > int64_t(input_buffer.size()))
				raise(LZ4ADA_CONSTRAINT_ERROR, "lz4ada.adb:644 index check failed");
			memcpy(input_buffer.data() + fill, src, size_t(avail));
			m.input_buffer_filled += avail;
			consumed += avail;
		} else {
			consumed += want;
			m.input_buffer_filled = 0;
			input_length = -1;
			// Input_Buffer(4 .. Fill-1) & Input(...): drops 4 cached bytes for
			// the raw-block format (quirk Q5), like the reference.
			const int64_t head = std::max<int64_t>(fill - BLOCK_SIZE_BYTES, 0);
			if (fill >= BLOCK_SIZE_BYTES && fill + want <= int64_t(input_buffer.size())) {
				// the rest of the block right after the cached bytes: no copy
				memcpy(input_buffer.data() + fill, src, size_t(want));
				decode_full_block(input_buffer.data() + BLOCK_SIZE_BYTES, head + want, buf, buflen,
				                  first, last);
				return;
			}
			blk_tmp.resize(size_t(head + want));
			if (head)
				memcpy(blk_tmp.data(), input_buffer.data() + BLOCK_SIZE_BYTES, size_t(head));
			memcpy(blk_tmp.data() + head, src, size_t(want));
			decode_full_block(blk_tmp.data(), head + want, buf, buflen, first, last);
		}
	}

	void update(const uint8_t* in, int64_t len, int64_t& consumed, uint8_t* buf, int64_t buflen,
	            int64_t& first, int64_t& last)  // lz4ada.adb:383-418
	{
		consumed = 0;
		first = 1;
		last = 0;
		if (m.header_parsing != HDR_DONE) {
			consumed = header_bytes(m, input_buffer.data(), in, len);
		} else if (m.is_format == F_SKIPPABLE) {
			consumed = skip(in, len);
		} else if (is_at_end_mark) {
			check_end_mark(in, len, consumed);
		} else if (input_length != -1) {
			cache_and_process(in, len, consumed, buf, buflen, first, last);
		} else {
			consumed = try_detect_input_length(in, len);
			if (is_at_end_mark) {
				check_end_mark(in, len, consumed);
			} else if (input_length != -1) {
				const int64_t total = input_length + m.block_checksum_length;
				if (len - consumed >= total) {  // :603-617, no copy
					const uint8_t* blk = in + consumed;
					consumed += total;
					m.input_buffer_filled = 0;
					input_length = -1;
					if (!serve_ahead(blk, total, in + len, buf, buflen, first, last))
						decode_full_block(blk, total, buf, buflen, first, last);
				} else {
					cache_and_process(in, len, consumed, buf, buflen, first, last);
				}
			}
		}
	}

	int is_end_of_frame() const  // :906-915
	{
		switch (m.is_format) {
		case F_LEGACY: return is_at_end_mark ? LZ4ADA_EOF_MAYBE : m.status_eof;
		case F_BLOCK: return input_length == -1 ? LZ4ADA_EOF_YES : LZ4ADA_EOF_NO;
		default: return m.status_eof;
		}
	}
};

// ---------------------------------------------------------------- C-ABI

template <class F>
static int guarded(std::string* err, F&& f)
{
	try {
		f();
		if (err)
			err->clear();
		return LZ4ADA_OK;
	} catch (const Error& e) {
		if (err)
			*err = e.msg;
		g_thread_error = e.msg;
		return e.code;
	} catch (const std::bad_alloc&) {
		if (err)
			*err = "out of host memory";
		g_thread_error = "out of host memory";
		return LZ4ADA_CONSTRAINT_ERROR;
	}
}

static lz4ada_decompressor* new_ctx(int64_t in_last)
{
	auto* c = new lz4ada_decompressor();
	c->input_buffer.assign(size_t(std::max<int64_t>(in_last + 1, 0)), 0);
	return c;
}

extern "C" {

int lz4ada_abi_version(void) { return LZ4ADA_HIP_ABI_VERSION; }

const char* lz4ada_error_name(int status)
{
	static const char* const names[] = { "",
		                             "LZ4ADA.CHECKSUM_ERROR",
		                             "LZ4ADA.DATA_CORRUPTION",
		                             "LZ4ADA.NOT_SUPPORTED",
		                             "LZ4ADA.TOO_FEW_HEADER_BYTES",
		                             "LZ4ADA.TOO_LITTLE_MEMORY",
		                             "ADA.ASSERTIONS.ASSERTION_ERROR",
		                             "CONSTRAINT_ERROR",
		                             "LZ4ADA.DEVICE_ERROR",
		                             "LZ4ADA.EXACT_PATH" };
	if (status < 0 || status > LZ4ADA_EXACT_PATH)
		return "UNKNOWN";
	return names[status];
}

const char* lz4ada_thread_last_error(void) { return g_thread_error.c_str(); }

const char* lz4ada_last_error(const lz4ada_decompressor* ctx) { return ctx ? ctx->err.c_str() : ""; }

int64_t lz4ada_exact_blocks(const lz4ada_decompressor* ctx) { return ctx ? ctx->exact_blocks : -1; }

int lz4ada_device_check(void)
{
	return guarded(nullptr, [] { device_check_or_raise(); });
}

void lz4ada_to_hex8(uint8_t v, char out[3]) { snprintf(out, 3, "%02x", v); }
void lz4ada_to_hex32(uint32_t v, char out[9]) { snprintf(out, 9, "%08x", v); }

int lz4ada_init(int reservation, int64_t* min_buffer_size, lz4ada_decompressor** ctx)
{
	*ctx = nullptr;
	return guarded(nullptr, [&] {  // lz4ada.adb:48-63
		if (!concrete(reservation))
			raise(LZ4ADA_CONSTRAINT_ERROR, "Init requires a Memory_Reservation (SZ_*)");
		const int64_t bmax = block_size_of(reservation);
		*min_buffer_size = bmax + HISTORY_SIZE + 8;
		auto* c = new_ctx(bmax + 4 + BLOCK_SIZE_BYTES - 1);
		c->m.memory_reservation = reservation;
		*ctx = c;
	});
}

int lz4ada_init_with_header(const uint8_t* input, int64_t len, int reservation,
                            int64_t* num_consumed, int64_t* min_buffer_size,
                            lz4ada_decompressor** ctx)
{
	*ctx = nullptr;
	*num_consumed = 0;
	return guarded(nullptr, [&] {  // lz4ada.adb:79-125
		if (len < 7)
			raise(LZ4ADA_ASSERTION_ERROR, "failed precondition from lz4ada.ads:243");
		if (reservation < LZ4ADA_SZ_64_KIB || reservation > LZ4ADA_SINGLE_FRAME)
			raise(LZ4ADA_CONSTRAINT_ERROR, "bad reservation");
		uint8_t hb[20];
		Meta mt;
		mt.memory_reservation =
		        reservation == LZ4ADA_SINGLE_FRAME ? int(LZ4ADA_USE_FIRST) : reservation;
		int64_t pos = 0;
		while (mt.header_parsing != HDR_DONE) {
			if (pos >= len)
				raise(LZ4ADA_TOO_FEW_HEADER_BYTES,
				      "Expected at least " + img_u(mt.size_remaining) +
				              " more bytes but header input has already ended.");
			const int64_t c = header_bytes(mt, hb, input + pos, len - pos);
			pos += c;
			*num_consumed += c;
		}
		const int64_t bmax = block_size_of(mt.memory_reservation);
		*min_buffer_size = bmax + HISTORY_SIZE + 8;
		if (reservation == LZ4ADA_SINGLE_FRAME)
			mt.memory_reservation = LZ4ADA_SINGLE_FRAME;
		auto* c = new_ctx(bmax + mt.block_checksum_length + BLOCK_SIZE_BYTES - 1);
		c->m = mt;
		*ctx = c;
	});
}

int lz4ada_init_for_block(int64_t compressed_length, int reservation, int64_t* min_buffer_size,
                          lz4ada_decompressor** ctx)
{
	*ctx = nullptr;
	return guarded(nullptr, [&] {  // lz4ada.adb:127-147
		if (!concrete(reservation))
			raise(LZ4ADA_CONSTRAINT_ERROR, "Init_For_Block requires a Memory_Reservation");
		const int64_t bmax = block_size_of(reservation);
		*min_buffer_size = bmax + HISTORY_SIZE + 8;
		auto* c = new_ctx(bmax - 1);
		c->m.is_format = F_BLOCK;
		c->m.is_compressed = true;
		c->m.header_parsing = HDR_DONE;
		c->m.memory_reservation = reservation;
		c->input_length = compressed_length;
		*ctx = c;
	});
}

int lz4ada_update(lz4ada_decompressor* ctx, const uint8_t* input, int64_t len,
                  int64_t* num_consumed, uint8_t* buffer, int64_t buffer_len,
                  int64_t* output_first, int64_t* output_last)
{
	*num_consumed = 0;
	*output_first = 1;
	*output_last = 0;
	return guarded(&ctx->err, [&] {
		ctx->update(input, len, *num_consumed, buffer, buffer_len, *output_first, *output_last);
	});
}

int lz4ada_is_end_of_frame(const lz4ada_decompressor* ctx) { return ctx->is_end_of_frame(); }

void lz4ada_free(lz4ada_decompressor* ctx) { delete ctx; }

// -------------------------------------------------------------- XXHash32

void lz4ada_xxh32_reset(lz4ada_xxh32_state* h, uint32_t seed)  // lz4ada.adb:932-940
{
	h->state[0] = seed + P1 + P2;
	h->state[1] = seed + P2;
	h->state[2] = seed;
	h->state[3] = seed - P1;
	memset(h->buffer, 0, sizeof h->buffer);
	h->buffer_size = 0;
	h->total_length = 0;
	h->hash = 0;
}

void lz4ada_xxh32_init(lz4ada_xxh32_state* h, uint32_t seed)  // :925-930 (Q1)
{
	(void)seed;
	lz4ada_xxh32_reset(h, 0);
}

static int xxh32_update_dev(lz4ada_xxh32_state* h, const void* d_data, int64_t len,
                            hipStream_t stream)
{
	return guarded(nullptr, [&] {
		device_check_or_raise();
		DevBuf<lz4ada_xxh32_state> ds;
		ds.reserve(1);
		HIP_OK(hipMemcpyAsync(ds.p, h, sizeof *h, hipMemcpyHostToDevice, stream));
		HIP_OK(launch_xxh32_update(ds.p, static_cast<const uint8_t*>(d_data), uint64_t(len), stream));
		HIP_OK(hipMemcpyAsync(h, ds.p, sizeof *h, hipMemcpyDeviceToHost, stream));
		HIP_OK(hipStreamSynchronize(stream));
	});
}

int lz4ada_xxh32_update_device(lz4ada_xxh32_state* h, const void* d_data, int64_t len,
                               void* stream)
{
	return xxh32_update_dev(h, d_data, len, static_cast<hipStream_t>(stream));
}

// XXHash32.Update over HOST bytes (lz4ada.adb:942-991) runs on the calling
// host thread: the chain is serial, a host core runs it ~10x
// faster than one GPU wave, and the bytes are already on the host -- a
// device round trip per call (allocation, H2D, one-wave kernel, D2H, sync)
// only added latency.  Device-resident bytes keep the GPU kernel
// (lz4ada_xxh32_update_device) or the D2H pipeline (lz4ada_content_xxh32_d2h).
int lz4ada_xxh32_update(lz4ada_xxh32_state* h, const uint8_t* data, int64_t len)
{
	return guarded(nullptr, [&] {
		if (len < 0 || (len > 0 && !data))
			raise(LZ4ADA_ASSERTION_ERROR, "failed precondition: XXHash32.Update input");
		if (len > 0)
			host_xxh32_update(*h, data, size_t(len));
		h->hash = host_xxh32_final(*h);
	});
}

// XXHash32.Final (lz4ada.adb:993-1017): a pure function of the state.
uint32_t lz4ada_xxh32_final(const lz4ada_xxh32_state* h) { return host_xxh32_final(*h); }

// Content checksum pipeline: the frame-wide XXH32 is
// one serial chain that one GPU wave runs at ~1.3 GB/s, so
// for output that is headed to the host anyway the chain runs on the host
// core, chunk by chunk, while the next chunk is still in flight over PCIe.
// The bytes hashed are the ones the GPU decoded; nothing is decoded here.
static void content_xxh32_d2h(lz4ada_xxh32_state& h, const uint8_t* d_data, int64_t len,
                              uint8_t* host_out, hipStream_t stream)
{
	device_check_or_raise();
	constexpr size_t CH = size_t(32) << 20;
	struct Pinned {
		uint8_t* p[2] = { nullptr, nullptr };
		hipEvent_t ev[2] = { nullptr, nullptr };
		~Pinned()
		{
			for (int i = 0; i < 2; ++i) {
				if (p[i])
					(void)hipHostFree(p[i]);
				if (ev[i])
					(void)hipEventDestroy(ev[i]);
			}
		}
	} pin;
	const size_t n = size_t(std::max<int64_t>(len, 0));
	const size_t chunks = (n + CH - 1) / CH;
	for (int i = 0; i < 2 && size_t(i) < chunks; ++i) {
		HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&pin.p[i]), CH, hipHostMallocDefault));
		HIP_OK(hipEventCreateWithFlags(&pin.ev[i], hipEventDisableTiming));
	}
	auto issue = [&](size_t k) {
		const size_t off = k * CH, c = std::min(CH, n - off);
		HIP_OK(hipMemcpyAsync(pin.p[k & 1], d_data + off, c, hipMemcpyDeviceToHost, stream));
		HIP_OK(hipEventRecord(pin.ev[k & 1], stream));
	};
	if (chunks)
		issue(0);
	for (size_t k = 0; k < chunks; ++k) {
		if (k + 1 < chunks)
			issue(k + 1);  // in flight while chunk k is hashed
		HIP_OK(hipEventSynchronize(pin.ev[k & 1]));
		const size_t off = k * CH, c = std::min(CH, n - off);
		host_xxh32_update(h, pin.p[k & 1], c);
		if (host_out)
			memcpy(host_out + off, pin.p[k & 1], c);
	}
	h.hash = host_xxh32_final(h);
}

int lz4ada_content_xxh32_d2h(lz4ada_xxh32_state* h, const void* d_data, int64_t len,
                             uint8_t* host_out, void* stream)
{
	return guarded(nullptr, [&] {
		content_xxh32_d2h(*h, static_cast<const uint8_t*>(d_data), len, host_out,
		                  static_cast<hipStream_t>(stream));
	});
}

int lz4ada_xxh32_hash(const uint8_t* data, int64_t len, uint32_t* out)  // :1019-1024
{
	lz4ada_xxh32_state h;
	lz4ada_xxh32_init(&h, 0);
	int st = lz4ada_xxh32_update(&h, data, len);
	if (st == LZ4ADA_OK)
		*out = h.hash;
	return st;
}

}  // extern "C"

// ------------------------------------------------------------ bulk path

namespace lz4ada {

// Walk one frame's block size words (Try_Detect_Input_Length semantics,
// lz4ada.adb:525-585, under Init_With_Header(Single_Frame)).
static void index_frame(const uint8_t* f, int64_t len, lz4ada_frame_info& info,
                        std::vector<lz4ada_block_desc>* descs)
{
	memset(&info, 0, sizeof info);
	if (len < 7)
		raise(LZ4ADA_ASSERTION_ERROR, "failed precondition from lz4ada.ads:243");
	Meta mt;
	mt.memory_reservation = LZ4ADA_USE_FIRST;
	uint8_t hb[20];
	int64_t pos = 0;
	while (mt.header_parsing != HDR_DONE) {
		if (pos >= len)
			raise(LZ4ADA_TOO_FEW_HEADER_BYTES,
			      "Expected at least " + img_u(mt.size_remaining) +
			              " more bytes but header input has already ended.");
		pos += header_bytes(mt, hb, f + pos, len - pos);
	}
	info.header_len = pos;
	const int64_t bmax = block_size_of(mt.memory_reservation);
	info.block_max = bmax;
	if (mt.is_format == F_SKIPPABLE) {
		info.format = LZ4ADA_FORMAT_SKIPPABLE;
		info.frame_len = pos + int64_t(mt.size_remaining);
		info.nblocks = 0;
		return;
	}
	info.format = mt.is_format == F_LEGACY ? LZ4ADA_FORMAT_LEGACY : LZ4ADA_FORMAT_MODERN;
	info.flg = mt.flg;
	info.bd = mt.bd;
	info.block_checksum = mt.block_checksum_length ? 1 : 0;
	info.content_checksum = mt.content_checksum_length ? 1 : 0;
	info.has_content_size = mt.has_content_size ? 1 : 0;
	info.independent = (mt.is_format == F_LEGACY) || (mt.flg & 0x20u) ? 1 : 0;
	info.content_size = mt.has_content_size ? mt.size_remaining : 0;
	const int64_t inbuf = bmax + mt.block_checksum_length + BLOCK_SIZE_BYTES;
	const int64_t additional = BLOCK_SIZE_BYTES + mt.block_checksum_length;
	int64_t nb = 0;
	for (;;) {
		if (pos + 4 > len) {
			if (mt.is_format == F_LEGACY && pos == len)
				break;  // legacy frames end with the input
			raise(LZ4ADA_DATA_CORRUPTION, "Frame truncated: block size word missing.");
		}
		uint32_t word = load32(f + pos);
		if (mt.is_format == F_MODERN && word == 0) {
			pos += 4;
			if (mt.content_checksum_length) {
				if (pos + 4 > len)
					raise(LZ4ADA_DATA_CORRUPTION, "Frame truncated: content checksum missing.");
				info.content_checksum_declared = load32(f + pos);
				pos += 4;
			}
			break;
		}
		if (mt.is_format == F_LEGACY && is_any_magic(word))
			break;  // next frame starts here
		bool stored = false;
		if (mt.is_format == F_MODERN) {
			stored = (word & 0x80000000u) != 0;
			word &= 0x7ffffffu;
		}
		if (int64_t(word) + additional > inbuf)
			raise(LZ4ADA_DATA_CORRUPTION,
			      "Declared maximum data length exceeded. Buffer has " + img(inbuf) +
			              " bytes, current block requires " + img_u(word) + " bytes + " +
			              img(additional) + " bytes for metadata.");
		const int64_t payload = pos + 4;
		const int64_t end = payload + int64_t(word) + mt.block_checksum_length;
		if (end > len)
			raise(LZ4ADA_DATA_CORRUPTION, "Frame truncated inside a block.");
		if (descs) {
			lz4ada_block_desc d{};
			d.in_off = uint64_t(payload);
			d.in_len = word;
			d.flags = (stored ? LZ4ADA_BLOCK_STORED : 0u) |
			          (mt.block_checksum_length ? LZ4ADA_BLOCK_HAS_CKSUM : 0u);
			d.out_off = uint64_t(nb) * uint64_t(bmax);
			d.out_cap = uint32_t(bmax);
			d.cksum = mt.block_checksum_length ? load32(f + payload + word) : 0u;
			descs->push_back(d);
		}
		++nb;
		pos = end;
	}
	info.nblocks = nb;
	info.frame_len = pos;
}

// Where decoded bytes go: the caller's fixed buffer, or a malloc'd buffer
// that grows (lz4ada_decode_*_alloc).  `len` is what is committed so far.
struct Sink {
	uint8_t* p = nullptr;
	int64_t cap = 0;
	bool growable = false;
	int64_t len = 0;
	// Room for n more bytes after len.
	uint8_t* room(int64_t n)
	{
		if (len + n > cap) {
			if (!growable)
				raise(LZ4ADA_CONSTRAINT_ERROR, "output capacity exceeded");
			int64_t c = std::max<int64_t>(len + n, std::max<int64_t>(2 * cap, 1 << 16));
			void* q = realloc(p, size_t(c));
			if (!q)
				raise(LZ4ADA_CONSTRAINT_ERROR, "output allocation failed");
			p = static_cast<uint8_t*>(q);
			cap = c;
		}
		return p + len;
	}
	void commit(int64_t n) { len += n; }
};

// Where the exact path resumes a frame the bulk path decoded up to a failing
// block: the stream state Decode_Full_Block_With_Trailer would have there
// (lz4ada.adb:661-714) -- Output_Pos / Output_Pos_History replayed from the
// decoded lengths (:678-690, 785-787), the content size left (:826-839) and
// the content hash (:709-714) over the bytes already committed.
struct Resume {
	int64_t at = 0;          // frame offset of the resume block's size word
	int64_t output_pos = 0;  // Ctx.Output_Pos before it
	int64_t output_pos_history = 0;
	uint64_t committed = 0;  // bytes of the blocks before it
	lz4ada_xxh32_state hash{};
	const uint8_t* output = nullptr;  // those bytes, and each block's length
	const std::vector<uint32_t>* lens = nullptr;
	bool checksum_first = false;  // check the resume block's checksum before decoding it
};

// The reference's Buffer as it stands before the resume block: blocks form
// "rounds" -- one starts at Buffer position 0 whenever Output_Pos has
// reached 64 KiB (lz4ada.adb:678-680) and appends otherwise -- so Buffer(x)
// holds byte x of the newest round longer than x (zero if none is).
static void buffer_image(const Resume& rs, uint8_t* img, int64_t size)
{
	memset(img, 0, size_t(size));
	const auto& lens = *rs.lens;
	std::vector<std::pair<int64_t, int64_t>> rounds;  // (output offset, length)
	int64_t pos = 0, off = 0;
	for (size_t j = 0; j < lens.size(); ++j) {
		if (rounds.empty() || pos >= HISTORY_SIZE) {
			rounds.emplace_back(off, 0);
			pos = 0;
		}
		pos += lens[j];
		off += lens[j];
		rounds.back().second = pos;
	}
	int64_t filled = 0;
	for (size_t r = rounds.size(); r-- > 0 && filled < size;) {
		const int64_t hi = std::min(rounds[r].second, size);
		if (hi > filled)
			memcpy(img + filled, rs.output + rounds[r].first + filled, size_t(hi - filled));
		filled = std::max(filled, hi);
	}
}

// Reference-exact path for one frame: the unlz4ada loop
// (tool_unlz4ada/unlz4ada.adb:84-103) over the streaming engine, from the
// frame start or from `resume`.
static void exact_frame(const uint8_t* f, int64_t len, Sink& out, int64_t& consumed_total,
                        const Resume* resume = nullptr)
{
	int64_t consumed = 0, mbs = 0;
	lz4ada_decompressor* raw = nullptr;
	int st = lz4ada_init_with_header(f, len, LZ4ADA_SINGLE_FRAME, &consumed, &mbs, &raw);
	if (st)
		raise(st, g_thread_error);
	std::unique_ptr<lz4ada_decompressor> ctx(raw);
	std::vector<uint8_t> buf(size_t(mbs), 0);
	int eof = LZ4ADA_EOF_NO;
	int64_t pos = consumed;
	if (resume) {
		ctx->output_pos = resume->output_pos;
		ctx->output_pos_history = resume->output_pos_history;
		if (ctx->m.has_content_size)
			ctx->m.size_remaining -= resume->committed;
		ctx->hash_all = resume->hash;
		ctx->checksum_first = resume->checksum_first;
		pos = resume->at;
		if (resume->lens && !resume->lens->empty()) {
			// the history the resume block may read: Buffer and its mirror
			buffer_image(*resume, buf.data(), int64_t(buf.size()));
			ctx->ensure_device();
			if (ctx->d_buf_len < int64_t(buf.size()))
				ctx->grow_mirror(int64_t(buf.size()));
			HIP_OK(hipMemcpy(ctx->d_buf.p, buf.data(), buf.size(), hipMemcpyHostToDevice));
		}
	}
	while (pos < len) {
		int64_t c = 0, first = 1, last = 0;
		ctx->update(f + pos, len - pos, c, buf.data(), mbs, first, last);
		if (last >= first) {
			const int64_t nout = last - first + 1;
			memcpy(out.room(nout), buf.data() + first, size_t(nout));
			out.commit(nout);
		}
		pos += c;
		eof = ctx->is_end_of_frame();
		if (eof == LZ4ADA_EOF_YES)
			break;
		if (c == 0 && last < first)
			raise(LZ4ADA_CONSTRAINT_ERROR, "decoder made no progress");
	}
	if (eof == LZ4ADA_EOF_NO)
		raise(LZ4ADA_CONSTRAINT_ERROR, "End not signalled by library. Unable to process all data");
	consumed_total = pos;
}

// A device allocation that may fail without raising (the bulk path then
// shrinks its batch or hands the frame to the exact path).
template <class T>
static bool try_reserve(DevBuf<T>& b, size_t count)
{
	if (count <= b.n && b.p)
		return true;
	b.release();
	const size_t bytes = std::max<size_t>(count, 1) * sizeof(T) + 64;
	if (hipMalloc(reinterpret_cast<void**>(&b.p), bytes) != hipSuccess) {
		(void)hipGetLastError();
		b.p = nullptr;
		return false;
	}
	b.n = count;
	b.bytes = bytes;  // not a pool size class: freed, never pooled
	return true;
}

// Device scratch of the bulk path, kept per thread between calls: the
// large buffers (slots, decode copies, resolution words) cost a hipMalloc
// and a first-touch each time otherwise -- more than the decode itself on a
// 1 GiB linked frame.  lz4ada_release_device_cache() frees them.  The
// cache is never destroyed at thread exit (the HIP runtime may be gone).
enum ScratchRole { SC_FRAME, SC_OUT, SC_COMPACT, SC_X, SC_Y, SC_H, SC_TAB, SC_P, SC_F, SC_LONE, SC_U, SC_N };
struct ScratchCache {
	DevBuf<uint8_t> b[SC_N];
};
static ScratchCache& scratch_cache()
{
	static thread_local ScratchCache* c = new ScratchCache;
	return *c;
}
static void scratch_release()
{
	for (auto& x : scratch_cache().b)
		x.release();
}
// bytes of scratch `role`, or nullptr when the device has no room (the
// caller then shrinks its batch or takes the exact path; other roles may be
// in use, so they are kept)
static uint8_t* scratch(int role, size_t bytes)
{
	DevBuf<uint8_t>& d = scratch_cache().b[role];
	return try_reserve(d, bytes) ? d.p : nullptr;
}

static int64_t env_bytes(const char* name, int64_t dflt)
{
	const char* e = getenv(name);
	if (!e || !*e)
		return dflt;
	const long long v = atoll(e);
	return v > 0 ? int64_t(v) : dflt;
}

// decode_lone_blocks: every block of d (host descriptors, offsets into d_in
// and d_out) through the lone-block decoder, stored ones as a copy, while
// host threads hash the blocks' host bytes for their checksums
// (lz4ada.adb:698-707).  st gets code, out_len and cksum as the bulk
// decoder's statuses carry them; false when a block was declined (the
// caller then runs the bulk decoder, which produces the exact status).
static bool decode_lone_blocks(const uint8_t* host_in, const uint8_t* d_in,
                               const std::vector<lz4ada_block_desc>& d, uint8_t* d_out,
                               lz4ada_block_status* d_st, std::vector<lz4ada_block_status>& st,
                               DevBuf<uint8_t>& scr, hipStream_t stream)
{
	const size_t nb = d.size();
	int64_t sb = 0;
	for (const auto& x : d) {
		if (x.flags & LZ4ADA_BLOCK_STORED) {
			if (x.in_len > x.out_cap)
				return false;
		} else {
			if (x.in_len == 0)
				return false;
			sb = std::max(sb, lone_scratch_bytes(x.in_len, x.out_cap));
		}
	}
	if (sb && !try_reserve(scr, size_t(sb)))
		return false;
	HIP_OK(hipMemsetAsync(d_st, 0, nb * sizeof(lz4ada_block_status), stream));
	for (size_t i = 0; i < nb; ++i) {
		const auto& x = d[i];
		if (x.flags & LZ4ADA_BLOCK_STORED) {
			if (x.in_len)
				HIP_OK(hipMemcpyAsync(d_out + x.out_off, d_in + x.in_off, x.in_len,
				                      hipMemcpyDeviceToDevice, stream));
		} else {
			HIP_OK(launch_decode_lone(d_in + x.in_off, x.in_len, d_out + x.out_off, x.out_cap,
			                          d_st + i, scr.p, sb, stream));
		}
	}
	std::vector<std::future<uint32_t>> ck(nb);
	for (size_t i = 0; i < nb; ++i)
		if (d[i].flags & LZ4ADA_BLOCK_HAS_CKSUM) {
			const uint8_t* p = host_in + d[i].in_off;
			const size_t n = d[i].in_len;
			ck[i] = std::async(std::launch::async, [p, n] {
				lz4ada_xxh32_state h;
				lz4ada_xxh32_reset(&h, 0);
				host_xxh32_update(h, p, n);
				return host_xxh32_final(h);
			});
		}
	st.assign(nb, lz4ada_block_status{});
	HIP_OK(hipMemcpyAsync(st.data(), d_st, nb * sizeof(lz4ada_block_status), hipMemcpyDeviceToHost,
	                      stream));
	HIP_OK(hipStreamSynchronize(stream));
	bool ok = true;
	for (size_t i = 0; i < nb; ++i) {
		if (d[i].flags & LZ4ADA_BLOCK_STORED) {
			st[i].code = DS_OK;
			st[i].out_len = d[i].in_len;
		}
		if (ck[i].valid())
			st[i].cksum = ck[i].get();
		if (st[i].code != DS_OK)
			ok = false;
	}
	if (ok)  // the statuses also on the device, as the bulk decoder leaves them
		HIP_OK(hipMemcpy(d_st, st.data(), nb * sizeof(lz4ada_block_status), hipMemcpyHostToDevice));
	return ok;
}

// Output slot capacity of one block: a stored block is its payload; a
// compressed one decodes to at most 255 bytes per payload byte (a length
// extension byte adds <= 255 to a match; everything else expands less), so
// a frame of many small flushed blocks does not reserve block_max each.
static uint32_t slot_cap(const lz4ada_block_desc& d, int64_t bmax)
{
	if (d.flags & LZ4ADA_BLOCK_STORED)
		return d.in_len;
	return uint32_t(std::min<uint64_t>(uint64_t(bmax), 255ull * d.in_len + 64));
}

static uint64_t round256(uint64_t v) { return (v + 255) & ~uint64_t(255); }

// Contiguous runs of blocks [lo, hi) whose slot bytes (plus `extra` per
// block) stay within `budget` (at least one block each).
static std::vector<std::pair<uint32_t, uint32_t>> batches_of(const std::vector<lz4ada_block_desc>& descs,
                                                             int64_t bmax, uint64_t extra,
                                                             uint64_t budget)
{
	std::vector<std::pair<uint32_t, uint32_t>> v;
	uint32_t lo = 0;
	uint64_t acc = 0;
	for (uint32_t i = 0; i < descs.size(); ++i) {
		const uint64_t need = round256(slot_cap(descs[i], bmax)) + extra;
		if (i > lo && acc + need > budget) {
			v.emplace_back(lo, i);
			lo = i;
			acc = 0;
		}
		acc += need;
	}
	if (lo < descs.size())
		v.emplace_back(lo, uint32_t(descs.size()));
	return v;
}

// Independent blocks, batch by batch: block checksums + the bulk decoder
// over slots, then the batch's bytes (compacted if a block is short) to the
// sink, hashed on the way when the frame has a content checksum.
// BULK_FAIL_AT: block `fail` has a bad status or checksum; the blocks before
// it are committed (their lengths in `lens`), so the exact path can resume
// there instead of redoing the frame.
static BulkResult bulk_independent(const uint8_t* d_frame, const uint8_t* host_frame,
                                   const lz4ada_frame_info& info,
                                   const std::vector<lz4ada_block_desc>& descs, Sink& out,
                                   lz4ada_xxh32_state* h, uint64_t& total,
                                   std::vector<uint32_t>& lens, int64_t& fail)
{
	lens.clear();
	fail = -1;
	hipStream_t stream = nullptr;
	uint64_t budget = uint64_t(env_bytes("LZ4ADA_BATCH_BYTES", int64_t(4) << 30));
	uint32_t lo = 0;
	total = 0;
	while (lo < descs.size()) {
		const auto bt = batches_of(std::vector<lz4ada_block_desc>(descs.begin() + lo, descs.end()),
		                           info.block_max, 0, budget);
		const uint32_t hi = lo + bt[0].second;
		uint32_t nb = hi - lo;
		std::vector<lz4ada_block_desc> d(descs.begin() + lo, descs.begin() + hi);
		uint64_t slots = 0;
		for (auto& x : d) {
			x.out_cap = slot_cap(x, info.block_max);
			x.out_off = slots;
			slots += round256(x.out_cap);
		}
		DevBuf<lz4ada_block_desc> d_desc;
		DevBuf<lz4ada_block_status> d_st;
		uint8_t* const d_out = scratch(SC_OUT, size_t(slots));
		if (!d_out) {
			if (budget > (uint64_t(64) << 20) && nb > 1) {
				budget /= 2;  // retry this batch smaller
				continue;
			}
			return BULK_EXACT;
		}
		d_desc.reserve(nb);
		d_st.reserve(nb);
		HIP_OK(hipMemcpy(d_desc.p, d.data(), nb * sizeof(lz4ada_block_desc), hipMemcpyHostToDevice));
		std::vector<lz4ada_block_status> st(nb);
		if (!(host_frame && few_large_blocks(d) &&
		      decode_lone_blocks(host_frame, d_frame, d, d_out, d_st.p, st,
		                         scratch_cache().b[SC_LONE], stream))) {
			HIP_OK(hipMemset(d_st.p, 0, nb * sizeof(lz4ada_block_status)));
			HIP_OK(launch_decode_checked(d_frame, uint64_t(info.frame_len), d_desc.p, nb, d_out,
			                             d_st.p, stream));
			HIP_OK(hipMemcpy(st.data(), d_st.p, nb * sizeof(lz4ada_block_status),
			                 hipMemcpyDeviceToHost));
		}
		uint64_t bt_total = 0;
		bool contiguous = true;
		std::vector<uint64_t> dst_off(nb);
		uint32_t ok_n = nb;  // the blocks before the first failing one
		for (uint32_t i = 0; i < nb; ++i) {
			// the block checksum is checked before decoding (lz4ada.adb:672-676)
			if ((d[i].flags & LZ4ADA_BLOCK_HAS_CKSUM) && st[i].cksum != d[i].cksum) {
				ok_n = i;
				break;
			}
			if (st[i].code == DS_PRE_BLOCK_REF)
				return BULK_PRE_REF;  // B.Indep set, but the block reads earlier blocks (D2)
			if (st[i].code != DS_OK) {
				ok_n = i;
				break;
			}
			dst_off[i] = bt_total;
			if (bt_total != d[i].out_off)
				contiguous = false;
			bt_total += st[i].out_len;
		}
		const uint32_t nb_all = nb;
		nb = ok_n;
		const uint8_t* d_res = d_out;
		if (!contiguous) {
			DevBuf<uint64_t> d_off;
			uint8_t* const d_compact = scratch(SC_COMPACT, size_t(std::max<uint64_t>(bt_total, 1)));
			if (!d_compact)
				return BULK_EXACT;
			d_off.reserve(nb);
			HIP_OK(hipMemcpy(d_off.p, dst_off.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice));
			HIP_OK(launch_compact(d_out, d_desc.p, d_off.p, d_st.p, nb, d_compact, stream));
			HIP_OK(hipDeviceSynchronize());
			d_res = d_compact;
		}
		uint8_t* dst = out.room(int64_t(bt_total));
		if (h)  // D2H overlapped with the host XXH32 chain (content_xxh32_d2h)
			content_xxh32_d2h(*h, d_res, int64_t(bt_total), dst, stream);
		else if (bt_total)
			HIP_OK(hipMemcpy(dst, d_res, size_t(bt_total), hipMemcpyDeviceToHost));
		out.commit(int64_t(bt_total));
		total += bt_total;
		for (uint32_t i = 0; i < nb; ++i)
			lens.push_back(st[i].out_len);
		if (nb < nb_all) {
			fail = int64_t(lo) + nb;
			return BULK_FAIL_AT;
		}
		lo = hi;
	}
	return BULK_OK;
}


static void d2h(void* dst, const void* src, size_t n, hipStream_t stream)
{
	HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, stream));
	HIP_OK(hipStreamSynchronize(stream));
}

// Linked frames (and independent ones whose blocks read earlier blocks,
// D2): every block at once with synthetic history, resolved on the GPU
// (lz4ada_linked.hip), batch by batch with the previous batch's last
// 64 KiB carried as real history.  BULK_EXACT: the frame needs the exact
// path (a block error or checksum mismatch, quirk D1, a reference before
// the frame start, no device memory).
static BulkResult bulk_linked(const uint8_t* d_frame, uint64_t frame_len, int64_t block_max,
                              const std::vector<lz4ada_block_desc>& descs, LinkedSink& sink,
                              uint64_t& total, std::vector<uint32_t>& lens, int64_t& fail,
                              hipStream_t stream, const LinkedHist* hist)
{
	lens.clear();
	fail = -1;
	// a batch holds 3 decode buffers (slots + 64 KiB regions) and one 4-byte
	// word per output byte: ~7x its slot bytes
	uint64_t budget = uint64_t(env_bytes("LZ4ADA_LINKED_BATCH_BYTES", int64_t(2) << 30));
	// LZ4ADA_TRACE_LINKED=1: phase times (synchronised) to stderr
	static const bool trace = getenv("LZ4ADA_TRACE_LINKED") != nullptr;
	auto t0 = std::chrono::steady_clock::now();
	auto phase = [&](const char* name) {
		if (!trace)
			return;
		HIP_OK(hipStreamSynchronize(stream));
		const auto t1 = std::chrono::steady_clock::now();
		fprintf(stderr, "[linked] %-10s %8.3f ms\n", name,
		        std::chrono::duration<double, std::milli>(t1 - t0).count());
		t0 = t1;
	};
	DevBuf<uint8_t> d_tail[2];
	d_tail[0].reserve(size_t(HISTORY_SIZE));
	d_tail[1].reserve(size_t(HISTORY_SIZE));
	HIP_OK(hipMemsetAsync(d_tail[0].p, 0, size_t(HISTORY_SIZE), stream));
	int cur = 0;
	// the reference's Output_Pos / Output_Pos_History (lz4ada.adb:678-690,
	// 785-787), for quirk D1
	int64_t opos = 0, oph = 0;
	int64_t hist0 = 0;  // history bytes before the first block (mid-frame batch)
	if (hist) {
		hist0 = std::min<int64_t>(hist->n0 + hist->n1, HISTORY_SIZE);
		if (hist->n1 > 0)
			HIP_OK(hipMemcpyAsync(d_tail[0].p + HISTORY_SIZE - hist->n1, hist->h1, size_t(hist->n1),
			                      hipMemcpyDeviceToDevice, stream));
		if (hist->n0 > 0)
			HIP_OK(hipMemcpyAsync(d_tail[0].p + HISTORY_SIZE - hist->n1 - hist->n0, hist->h0,
			                      size_t(hist->n0), hipMemcpyDeviceToDevice, stream));
		opos = hist->output_pos;
		oph = hist->output_pos_history;
	}
	uint32_t lo = 0;
	total = 0;
	while (lo < descs.size()) {
		const auto bt = batches_of(std::vector<lz4ada_block_desc>(descs.begin() + lo, descs.end()),
		                           block_max, uint64_t(HISTORY_SIZE), budget);
		const uint32_t hi = lo + bt[0].second;
		uint32_t nb = hi - lo;
		std::vector<lz4ada_block_desc> d(descs.begin() + lo, descs.begin() + hi);
		uint64_t bytes = 0;
		for (auto& x : d) {
			x.out_cap = slot_cap(x, block_max);
			x.out_off = bytes + uint64_t(HISTORY_SIZE);
			bytes += uint64_t(HISTORY_SIZE) + round256(x.out_cap);
		}
		struct {
			uint8_t* p;
		} bx{ scratch(SC_X, size_t(bytes)) }, by{ bx.p ? scratch(SC_Y, size_t(bytes)) : nullptr },
		    bh{ by.p ? scratch(SC_H, size_t(bytes)) : nullptr },
		    tab{ bh.p ? scratch(SC_TAB, index_table_bytes(frame_len, nb)) : nullptr };
		if (!tab.p) {
			if (budget > (uint64_t(64) << 20) && nb > 1) {
				budget /= 2;
				continue;
			}
			return BULK_EXACT;
		}
		DevBuf<lz4ada_block_desc> d_desc;
		DevBuf<lz4ada_block_status> sx, sy, sh;
		d_desc.reserve(nb);
		sx.reserve(nb);
		sy.reserve(nb);
		sh.reserve(nb);
		const size_t sb = nb * sizeof(lz4ada_block_status);
		phase("alloc");
		HIP_OK(hipMemcpyAsync(d_desc.p, d.data(), nb * sizeof(lz4ada_block_desc),
		                      hipMemcpyHostToDevice, stream));
		HIP_OK(hipMemsetAsync(sx.p, 0, sb, stream));
		HIP_OK(launch_link_fill(bx.p, by.p, bh.p, d_desc.p, nb, stream));
		HIP_OK(launch_block_checksums(d_frame, d_desc.p, nb, sx.p, stream));
		HIP_OK(launch_index(d_frame, frame_len, d_desc.p, nb, tab.p, sx.p, stream));
		HIP_OK(hipMemcpyAsync(sy.p, sx.p, sb, hipMemcpyDeviceToDevice, stream));
		HIP_OK(hipMemcpyAsync(sh.p, sx.p, sb, hipMemcpyDeviceToDevice, stream));
		uint8_t* bufs[3] = { bx.p, by.p, bh.p };
		lz4ada_block_status* sts[3] = { sx.p, sy.p, sh.p };
		for (int k = 0; k < 3; ++k) {
			HIP_OK(launch_decode_idx_tab(d_frame, frame_len, d_desc.p, nb, tab.p, bufs[k], sts[k], 2,
			                             stream));
			HIP_OK(launch_decode_pc(d_frame, frame_len, d_desc.p, nb, bufs[k], sts[k], 1, LINK_HIST,
			                        stream));
		}
		phase("decodes");
		std::vector<lz4ada_block_status> st(nb);
		d2h(st.data(), sx.p, sb, stream);
		std::vector<int64_t> A(nb);
		int64_t n = 0;
		const int64_t opos0 = opos, oph0 = oph;  // this batch's start (a smaller retry rescans)
		// the first block the exact path has to take: a block error, a
		// checksum mismatch, or quirk D1 (a match reaching
		// >= D1_OFF back into the history right after a block that ended at
		// 65536..65542).  The blocks before it only point backwards, so they
		// resolve on their own and the exact path resumes at it.
		uint32_t ok_n = nb;
		for (uint32_t i = 0; i < nb; ++i) {
			if (opos >= HISTORY_SIZE)
				opos = 0;
			if (st[i].code != DS_OK ||
			    ((d[i].flags & LZ4ADA_BLOCK_HAS_CKSUM) && st[i].cksum != d[i].cksum) ||
			    ((st[i].aux & AUX_D1_RISK) && oph >= HISTORY_SIZE && oph <= HISTORY_SIZE + 6)) {
				ok_n = i;
				break;
			}
			opos += st[i].out_len;
			if (opos >= HISTORY_SIZE)
				oph = opos;
			A[i] = n;
			n += st[i].out_len;
		}
		if (ok_n < nb) {
			fail = int64_t(lo) + ok_n;
			nb = ok_n;
			if (nb == 0)
				return BULK_FAIL_AT;
		}
		if (n >= (int64_t(1) << 31) - HISTORY_SIZE) {  // words hold positions + 65536 in 31 bits
			if (nb > 1) {
				// the smaller batch rescans from this batch's start: its own
				// first failing block (if any) and the replayed positions
				budget /= 2;
				fail = -1;
				opos = opos0;
				oph = oph0;
				continue;
			}
			return BULK_EXACT;
		}
		DevBuf<int64_t> d_A;
		DevBuf<uint32_t> d_ctr;
		struct {
			uint32_t* p;
		} d_P{ reinterpret_cast<uint32_t*>(scratch(SC_P, size_t(std::max<int64_t>(n, 1)) * 4)) };
		if (!d_P.p)
			return BULK_EXACT;
		d_A.reserve(nb);
		d_ctr.reserve(2);
		HIP_OK(hipMemcpyAsync(d_A.p, A.data(), nb * sizeof(int64_t), hipMemcpyHostToDevice, stream));
		HIP_OK(hipMemsetAsync(d_ctr.p, 0, 2 * sizeof(uint32_t), stream));
		const int64_t tail_valid = std::min<int64_t>(int64_t(total) + hist0, HISTORY_SIZE);
		uint32_t ctr[2] = { 0, 0 };
		uint8_t* F = nullptr;
		// a word per output byte (resolving only the history-derived bytes,
		// round 4's sparse form, measured slower -- three gathers per target
		// instead of one word -- DESIGN §7)
		{
			// the constant bytes go to F with the words, each round writes the
			// bytes it resolves: the last round leaves the output
			F = sink.dst(n);
			if (!F)
				return BULK_EXACT;
			// span activity flags, double-buffered across rounds (an init that
			// also stepped every history-derived byte one pointer forward was
			// measured and dropped: mixed 10.32 vs 10.35 ms, chain 13.5 vs
			// 15.4, dense 31.0 vs 23.7 -- its byte gathers cost what the round
			// saves)
			const int64_t ns = link_spans(n);
			uint8_t* act = scratch(SC_U, size_t(2 * ns + 64));
			if (!act)
				return BULK_EXACT;
			// init flags the spans that hold a history-derived byte: the
			// first round reads only those
			HIP_OK(hipMemsetAsync(act + ns, 0, size_t(ns), stream));
			HIP_OK(launch_link_init(bx.p, by.p, bh.p, d_desc.p, sx.p, d_A.p, nb, block_max, d_P.p, F,
			                        act + ns, d_ctr.p, stream));
			d2h(ctr, d_ctr.p, sizeof ctr, stream);
			phase("init");
			for (int round = 0; ctr[0] > 0; ++round) {
				if (round > 64)
					return BULK_EXACT;  // never expected: every pointer goes strictly back
				HIP_OK(hipMemsetAsync(d_ctr.p, 0, 2 * sizeof(uint32_t), stream));
				uint8_t* a_out = act + (round & 1) * ns;
				const uint8_t* a_in = act + ((round + 1) & 1) * ns;
				HIP_OK(launch_link_jump(d_P.p, n, d_tail[cur].p, tail_valid, F, a_in, a_out, d_ctr.p,
				                        stream));
				d2h(ctr, d_ctr.p, sizeof ctr, stream);
				if (ctr[1])
					return BULK_EXACT;  // a reference before the frame start: the exact error
			}
			phase("jumps");
		}
		HIP_OK(launch_link_tail(F, n, d_tail[cur].p, d_tail[cur ^ 1].p, stream));
		cur ^= 1;
		phase("emit");
		sink.done(F, n);
		phase("sink");
		total += uint64_t(n);
		for (uint32_t i = 0; i < nb; ++i)
			lens.push_back(st[i].out_len);
		if (fail >= 0)
			return BULK_FAIL_AT;
		lo = hi;
	}
	return BULK_OK;
}

// Which paths the last lz4ada_decode_* call on this thread took
// (LZ4ADA_PATH_* bits; tests and diagnostics).
static thread_local int g_last_path = 0;

// for lz4ada_multi.cpp (lz4ada_internal.h)
void set_thread_error(const std::string& msg) { g_thread_error = msg; }
void set_last_path(int bits) { g_last_path = bits; }

// The stream state before block `fail`, the first one the bulk path could
// not take (its predecessors are committed): Output_Pos and
// Output_Pos_History as lz4ada.adb:678-690 and 785-787 leave them.
static void resume_state(const std::vector<uint32_t>& lens, Resume& rs)
{
	int64_t pos = 0, oph = 0;
	for (uint32_t n : lens) {
		if (pos >= HISTORY_SIZE)  // :678-680
			pos = 0;
		pos += n;
		if (pos >= HISTORY_SIZE)  // :688-690, 785-787
			oph = pos;
	}
	rs.output_pos = pos;
	rs.output_pos_history = oph;
}

// One frame from host memory (Single_Frame semantics): the bulk path when
// the frame indexes cleanly, else -- or when the bulk path finds anything
// the reference would report or treat differently -- the exact path, which
// raises the reference's exception in the reference's order.
static void decode_one_frame(const uint8_t* f, int64_t len, Sink& out, int64_t& consumed)
{
	lz4ada_frame_info info;
	std::vector<lz4ada_block_desc> descs;
	bool indexed = true;
	try {
		index_frame(f, len, info, &descs);
	} catch (const Error&) {
		indexed = false;  // the exact path raises the reference's error in order
	}
	if (indexed && info.format == LZ4ADA_FORMAT_SKIPPABLE && info.frame_len <= len) {
		consumed = info.frame_len;  // Skip (lz4ada.adb:420-433): nothing to decode
		return;
	}
	const int64_t base = out.len;
	// LZ4ADA_TRACE_FRAME=1: phase times (synchronised) to stderr
	static const bool trace = getenv("LZ4ADA_TRACE_FRAME") != nullptr;
	auto t0 = std::chrono::steady_clock::now();
	auto phase = [&](const char* name) {
		if (!trace)
			return;
		HIP_OK(hipDeviceSynchronize());
		const auto t1 = std::chrono::steady_clock::now();
		fprintf(stderr, "[frame] %-10s %8.3f ms\n", name,
		        std::chrono::duration<double, std::milli>(t1 - t0).count());
		t0 = t1;
	};
	if (indexed && info.frame_len <= len && info.format != LZ4ADA_FORMAT_SKIPPABLE &&
	    !getenv("LZ4ADA_EXACT_ONLY")) {
		device_check_or_raise();
		struct {
			uint8_t* p;
		} d_frame{ scratch(SC_FRAME, size_t(info.frame_len)) };
		phase("index");
		if (d_frame.p) {
			HIP_OK(hipMemcpy(d_frame.p, f, size_t(info.frame_len), hipMemcpyHostToDevice));
			phase("h2d");
			lz4ada_xxh32_state hs;
			lz4ada_xxh32_reset(&hs, 0);
			lz4ada_xxh32_state* h = info.content_checksum ? &hs : nullptr;
			uint64_t total = 0;
			// the reference decodes every frame as linked (B.Indep is never
			// read, lz4ada.adb:267-275); independent blocks are the fast case
			BulkResult r = BULK_PRE_REF;
			std::vector<uint32_t> lens;
			int64_t fail = -1;
			if (info.independent && !getenv("LZ4ADA_FORCE_LINKED"))
				r = bulk_independent(d_frame.p, f, info, descs, out, h, total, lens, fail);
			phase("bulk");
			const bool linked = r == BULK_PRE_REF;
			if (linked) {
				out.len = base;
				lz4ada_xxh32_reset(&hs, 0);
				LinkedSink ls;
				ls.dst = [&](int64_t n) -> uint8_t* {
					return scratch(SC_F, size_t(std::max<int64_t>(n, 1)));
				};
				ls.done = [&](const uint8_t* F, int64_t n) {
					uint8_t* dst = out.room(n);
					if (h)
						content_xxh32_d2h(*h, F, n, dst, nullptr);
					else if (n)
						HIP_OK(hipMemcpy(dst, F, size_t(n), hipMemcpyDeviceToHost));
					out.commit(n);
				};
				r = bulk_linked(d_frame.p, uint64_t(info.frame_len), info.block_max, descs, ls, total,
				                lens, fail, nullptr);
			}
			// blocks before `fail` that already decode past the declared content
			// size: the reference raises inside the first block that overruns
			// (lz4ada.adb:830-835), which a resume at `fail` would skip -- the
			// whole frame goes to the exact path instead
			const bool overrun = info.has_content_size && total > info.content_size;
			if (r == BULK_FAIL_AT && !overrun && !getenv("LZ4ADA_NO_RESUME")) {
				// the reference outputs blocks 0 .. fail-1 and then raises in
				// block `fail` (lz4ada.adb:672-676: each block is checked when it
				// is reached): the exact path resumes at that block, over the
				// Buffer the committed blocks leave, not at byte 0
				Resume rs;
				resume_state(lens, rs);
				rs.committed = total;
				rs.hash = hs;  // the blocks before `fail`, hashed on their way out
				rs.output = out.p + base;
				rs.lens = &lens;
				rs.at = int64_t(descs[size_t(fail)].in_off) - BLOCK_SIZE_BYTES;
				rs.checksum_first = info.block_checksum != 0;
				g_last_path |= LZ4ADA_PATH_EXACT |
				               (linked ? LZ4ADA_PATH_LINKED : LZ4ADA_PATH_INDEPENDENT);
				phase("state");
				try {
					exact_frame(f, len, out, consumed, &rs);
				} catch (...) {
					phase("resume");
					throw;
				}
				phase("resume");
				return;
			}
			if (r == BULK_OK && (!info.has_content_size || total == info.content_size) &&
			    (!h || (total == 0 ? 0x02cc5d05u : hs.hash) == info.content_checksum_declared)) {
				consumed = info.frame_len;
				g_last_path |= linked ? LZ4ADA_PATH_LINKED : LZ4ADA_PATH_INDEPENDENT;
				return;
			}
			out.len = base;
		}
	}
	// A legacy frame has no end mark: it ends where the next magic starts
	// (what tool_unlz4ada's per-frame re-init achieves), so hand the exact
	// path only this frame's bytes.
	const int64_t flen = (indexed && info.format == LZ4ADA_FORMAT_LEGACY) ? info.frame_len : len;
	g_last_path |= LZ4ADA_PATH_EXACT;
	exact_frame(f, flen, out, consumed);
}
}  // namespace lz4ada

extern "C" {

int lz4ada_frame_index(const uint8_t* frame, int64_t len, lz4ada_frame_info* info,
                       lz4ada_block_desc* descs, int64_t desc_cap)
{
	return guarded(nullptr, [&] {
		std::vector<lz4ada_block_desc> v;
		index_frame(frame, len, *info, descs ? &v : nullptr);
		if (descs) {
			if (int64_t(v.size()) > desc_cap)
				raise(LZ4ADA_CONSTRAINT_ERROR, "descriptor capacity exceeded");
			memcpy(descs, v.data(), v.size() * sizeof(lz4ada_block_desc));
		}
	});
}

int lz4ada_launch_decode(const void* d_frame, uint64_t frame_len, const lz4ada_block_desc* d_descs,
                         int64_t nblocks, void* d_out, lz4ada_block_status* d_status, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_decode_blocks(static_cast<const uint8_t*>(d_frame), frame_len, d_descs,
		                            uint32_t(nblocks), static_cast<uint8_t*>(d_out), d_status,
		                            static_cast<hipStream_t>(stream)));
	});
}

int lz4ada_launch_decode_variant(const void* d_frame, uint64_t frame_len,
                                 const lz4ada_block_desc* d_descs, int64_t nblocks, void* d_out,
                                 lz4ada_block_status* d_status, int variant, void* stream)
{
	return guarded(nullptr, [&] {
		if (variant < 0 || variant > 8)
			raise(LZ4ADA_ASSERTION_ERROR, "unknown decoder variant");
		HIP_OK(launch_decode_variant(static_cast<const uint8_t*>(d_frame), frame_len, d_descs,
		                             uint32_t(nblocks), static_cast<uint8_t*>(d_out), d_status,
		                             variant, static_cast<hipStream_t>(stream)));
	});
}


int64_t lz4ada_lone_scratch_bytes(int64_t n, int64_t cap) { return lone_scratch_bytes(n, cap); }

int lz4ada_launch_decode_lone(const void* d_blk, int64_t n, void* d_out, int64_t cap,
                              lz4ada_block_status* d_status, void* d_scratch,
                              int64_t scratch_bytes, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_decode_lone(static_cast<const uint8_t*>(d_blk), n, static_cast<uint8_t*>(d_out),
		                          cap, d_status, d_scratch, scratch_bytes,
		                          static_cast<hipStream_t>(stream)));
	});
}

int lz4ada_launch_block_checksums(const void* d_frame, const lz4ada_block_desc* d_descs,
                                  int64_t nblocks, lz4ada_block_status* d_status, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_block_checksums(static_cast<const uint8_t*>(d_frame), d_descs,
		                              uint32_t(nblocks), d_status,
		                              static_cast<hipStream_t>(stream)));
	});
}

int lz4ada_decode_blocks_device(const void* d_frame, uint64_t frame_len,
                                const lz4ada_block_desc* d_descs, int64_t nblocks, void* d_out,
                                lz4ada_block_status* d_status, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_decode_checked(static_cast<const uint8_t*>(d_frame), frame_len, d_descs,
		                             uint32_t(nblocks), static_cast<uint8_t*>(d_out), d_status,
		                             static_cast<hipStream_t>(stream)));
	});
}

int lz4ada_output_checksums_device(const void* d_out, const lz4ada_block_desc* d_descs,
                                   const lz4ada_block_status* d_status, int64_t nblocks,
                                   uint32_t* d_hash, void* stream)
{
	return guarded(nullptr, [&] {
		HIP_OK(launch_output_checksums(static_cast<const uint8_t*>(d_out), d_descs,
		                               uint32_t(nblocks), d_status, d_hash,
		                               static_cast<hipStream_t>(stream)));
	});
}

// A stream's next frame starts with fewer than 7 bytes left: what the
// reference CLI raises there (tool_unlz4ada/unlz4ada.adb:65-76), before
// Init_With_Header's precondition (lz4ada.ads:243) would.
static void partial_frame_check(int64_t left)
{
	if (left < 7)
		raise(LZ4ADA_CONSTRAINT_ERROR, "Partial frame detected. Unable to process all data");
}

int lz4ada_decode_frame(const uint8_t* frame, int64_t len, uint8_t* out, int64_t out_cap,
                        int64_t* out_len, int64_t* frame_consumed)
{
	*out_len = 0;
	*frame_consumed = 0;
	g_last_path = 0;
	return guarded(nullptr, [&] {
		Sink s;
		s.p = out;
		s.cap = out_cap;
		decode_one_frame(frame, len, s, *frame_consumed);
		*out_len = s.len;
	});
}

int lz4ada_decode_stream(const uint8_t* input, int64_t len, uint8_t* out, int64_t out_cap,
                         int64_t* out_len)
{
	*out_len = 0;
	g_last_path = 0;
	return guarded(nullptr, [&] {
		Sink s;
		s.p = out;
		s.cap = out_cap;
		int64_t pos = 0;
		while (pos < len) {
			int64_t c = 0;
			partial_frame_check(len - pos);
			decode_one_frame(input + pos, len - pos, s, c);
			*out_len = s.len;
			if (c <= 0)
				raise(LZ4ADA_CONSTRAINT_ERROR, "decoder made no progress");
			pos += c;
		}
	});
}

// The same into a buffer the library allocates and grows (no bound needed
// up front); release it with lz4ada_buffer_free.  On failure *out is NULL.
static int decode_alloc(const uint8_t* input, int64_t len, bool stream, uint8_t** out,
                        int64_t* out_len, int64_t* consumed, bool keep_partial = false)
{
	*out = nullptr;
	*out_len = 0;
	if (consumed)
		*consumed = 0;
	Sink s;
	s.growable = true;
	g_last_path = 0;
	const int st = guarded(nullptr, [&] {
		int64_t pos = 0;
		do {
			int64_t c = 0;
			if (stream)
				partial_frame_check(len - pos);
			decode_one_frame(input + pos, len - pos, s, c);
			if (c <= 0)
				raise(LZ4ADA_CONSTRAINT_ERROR, "decoder made no progress");
			pos += c;
		} while (stream && pos < len);
		if (consumed)
			*consumed = pos;
	});
	if (st != LZ4ADA_OK) {
		if (keep_partial) {  // what the reference had output before it raised
			*out = s.p ? s.p : static_cast<uint8_t*>(malloc(1));
			*out_len = s.len;
			return st;
		}
		free(s.p);
		return st;
	}
	*out = s.p ? s.p : static_cast<uint8_t*>(malloc(1));
	*out_len = s.len;
	return LZ4ADA_OK;
}

int lz4ada_decode_frame_alloc(const uint8_t* frame, int64_t len, uint8_t** out, int64_t* out_len,
                              int64_t* frame_consumed)
{
	return decode_alloc(frame, len, false, out, out_len, frame_consumed);
}

int lz4ada_decode_stream_alloc(const uint8_t* input, int64_t len, uint8_t** out, int64_t* out_len)
{
	return decode_alloc(input, len, true, out, out_len, nullptr);
}

int lz4ada_decode_frame_partial(const uint8_t* frame, int64_t len, uint8_t** out, int64_t* out_len,
                                int64_t* frame_consumed)
{
	return decode_alloc(frame, len, false, out, out_len, frame_consumed, true);
}

void lz4ada_buffer_free(uint8_t* p) { free(p); }

int lz4ada_decode_linked_device(const void* d_frame, uint64_t frame_len,
                                const lz4ada_block_desc* descs, int64_t nblocks, int64_t block_max,
                                void* d_out, int64_t out_cap, int64_t* out_len, void* stream)
{
	*out_len = 0;
	return guarded(nullptr, [&] {
		device_check_or_raise();
		std::vector<lz4ada_block_desc> v(descs, descs + nblocks);
		hipStream_t s = static_cast<hipStream_t>(stream);
		int64_t pos = 0;
		LinkedSink ls;
		ls.dst = [&](int64_t n) -> uint8_t* {
			return pos + n <= out_cap ? static_cast<uint8_t*>(d_out) + pos : nullptr;
		};
		ls.done = [&](const uint8_t*, int64_t n) { pos += n; };
		uint64_t total = 0;
		std::vector<uint32_t> lens;
		int64_t fail = -1;
		if (bulk_linked(static_cast<const uint8_t*>(d_frame), frame_len, block_max, v, ls, total,
		                lens, fail, s) != BULK_OK)
			raise(LZ4ADA_EXACT_PATH,
			      "the frame needs the reference-exact path (lz4ada_decode_frame): a block "
			      "error or checksum mismatch, quirk D1, or too little output room");
		HIP_OK(hipStreamSynchronize(s));
		*out_len = pos;
	});
}

int lz4ada_last_path(void) { return g_last_path; }

const char* lz4ada_bulk_decoder_kernel(int64_t nblocks)
{
	return idx_fused_kernel_name(uint32_t(std::max<int64_t>(nblocks, 0)));
}

void lz4ada_release_device_cache(void)
{
	scratch_release();
	dev_pool().release_all();
	pin_pool().release_all();
	// the facade's pooled streams and events too
	std::vector<StreamSet> sets;
	{
		std::lock_guard<std::mutex> l(g_stream_mu);
		sets.swap(stream_pool());
	}
	int cur = 0;
	(void)hipGetDevice(&cur);
	for (auto& x : sets) {
		(void)hipSetDevice(x.device);
		(void)hipStreamDestroy(x.side);
		(void)hipEventDestroy(x.ev);
		(void)hipStreamDestroy(x.stream);
	}
	(void)hipSetDevice(cur);
}

int64_t lz4ada_decoded_bound(const uint8_t* input, int64_t len)
{
	int64_t pos = 0, bound = 0;
	while (pos < len) {
		lz4ada_frame_info info;
		if (lz4ada_frame_index(input + pos, len - pos, &info, nullptr, 0) != LZ4ADA_OK)
			return -1;
		if (info.frame_len <= 0)
			return -1;
		bound += info.nblocks * info.block_max;
		pos += info.frame_len;
	}
	return bound;
}

}  // extern "C"
