// lz4ada_host_common.h -- what the host units of the MI355X LZ4Ada
// decompressor share: the reference's exceptions and 'Image texts, the
// process-wide device / pinned memory pools and stream pool, the frame
// header parser (lib/lz4ada.adb:155-375), the host XXH32 chain and the
// device-status -> exception map.  Units: lz4ada_facade.cpp (the streaming
// Update facade and the XXHash32 C-ABI), lz4ada_bulk.cpp (the bulk frame
// paths and their C-ABI), lz4ada_multi.cpp (the multi-GPU entry).
//
// The host only parses framing.  Every block byte is produced on the GPU;
// there is no CPU decoder: without a GPU, decoding calls fail with
// LZ4ADA_DEVICE_ERROR.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
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

[[noreturn]] inline void raise(int code, std::string msg) { throw Error{ code, std::move(msg) }; }

// Ada 'Image: leading blank for non-negative numbers.
inline std::string img(int64_t v)
{
	return v >= 0 ? " " + std::to_string(v) : std::to_string(v);
}
inline std::string img_u(uint64_t v) { return " " + std::to_string(v); }
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

inline const char* const RES_IMAGE[] = { "SZ_64_KIB", "SZ_256_KIB", "SZ_1_MIB",    "SZ_4_MIB",
	                                 "SZ_8_MIB",  "USE_FIRST",  "SINGLE_FRAME" };

inline thread_local std::string g_thread_error;

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

inline void device_check_or_raise()
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

// Per-block arrays (descriptors, statuses) between a host vector and device
// memory, sized from the vector itself -- never from a block count captured
// earlier (round 5: a status copy sized before a quirk-D1 stop shrank the
// batch overran its vector) -- and checked against the device buffer's
// capacity.
template <class T>
inline void vec_h2d(DevBuf<T>& d, const std::vector<T>& v, hipStream_t stream)
{
	if (v.size() > d.n)
		raise(LZ4ADA_DEVICE_ERROR, "host array larger than its device buffer");
	HIP_OK(hipMemcpyAsync(d.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, stream));
}
template <class T>
inline void vec_d2h(std::vector<T>& v, const DevBuf<T>& d, hipStream_t stream)
{
	if (v.size() > d.n)
		raise(LZ4ADA_DEVICE_ERROR, "host array larger than its device buffer");
	HIP_OK(hipMemcpyAsync(v.data(), d.p, v.size() * sizeof(T), hipMemcpyDeviceToHost, stream));
	HIP_OK(hipStreamSynchronize(stream));
}

// Pinned host memory, grow-only (the facade's output staging).
struct PinBuf {
	uint8_t* p = nullptr;
	size_t n = 0, bytes = 0;
	int dev = 0;  // the device current when it was taken (synced on release)
	PinBuf() = default;
	PinBuf(const PinBuf&) = delete;
	PinBuf& operator=(const PinBuf&) = delete;
	~PinBuf() { release(); }
	void release()
	{
		pin_pool().put(p, bytes, dev);
		p = nullptr;
		n = bytes = 0;
	}
	void reserve(size_t count)
	{
		if (count <= n && p)
			return;
		release();
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
inline std::mutex g_stream_mu;
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

inline bool concrete(int r) { return r >= LZ4ADA_SZ_64_KIB && r <= LZ4ADA_SZ_8_MIB; }

static int64_t block_size_of(int r)  // Get_Block_Size, lz4ada.adb:65-77
{
	static const int64_t lut[] = { 64 << 10, 256 << 10, 1 << 20, 4 << 20, 8 << 20 };
	return lut[r];
}

inline void check_reservation(int requested, int& effective)  // lz4ada.adb:241-260
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

inline void legacy_end_of_header(Meta& m)  // lz4ada.adb:225-239
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

inline void header_magic(Meta& m, uint32_t magic)  // lz4ada.adb:199-223
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

inline void header_flags(Meta& m, const uint8_t* hb)  // lz4ada.adb:262-328
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

inline void header_modern_end(Meta& m, const uint8_t* hb)  // lz4ada.adb:330-361
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

inline bool is_any_magic(uint32_t v)
{
	return v == MAGIC_MODERN || v == MAGIC_LEGACY || (v >= MAGIC_SKIP_LO && v <= MAGIC_SKIP_HI);
}

// XXHash32.Update / Final (lz4ada.adb:942-1017) on host bytes the GPU
// decoded (content checksums: the facade's Hash_All_Data and the bulk
// path's pipeline).  The state layout is the one the GPU kernel
// k_xxh32_update advances, so the two can continue each other.
inline uint32_t rotl32h(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t xxh_round(uint32_t acc, uint32_t w) { return rotl32h(acc + w * P2, 13) * P1; }

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
[[noreturn]] inline void raise_device_status(const SerialState& s)
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

// ---------------------------------------------- shared by the host units

// A few large blocks: one block at a time through the lone-block decoder
// (lz4ada_lone.hip, the whole GPU per block: ~0.4 ms per 4 MiB mixed block)
// beats the bulk decoder's one wave per block (~13 ms per 4 MiB block, at
// any count up to the chip's 2,048 resident waves) below ~30 blocks.
inline bool few_large_blocks(const std::vector<lz4ada_block_desc>& d)
{
	static const bool off = getenv("LZ4ADA_NO_LONE") != nullptr;
	if (off || d.empty() || d.size() > 24)
		return false;
	uint32_t mx = 0;
	for (const auto& x : d)
		mx = std::max(mx, x.in_len);
	return mx >= (512u << 10) && int64_t(mx) <= LONE_MAX_IN;
}
bool decode_lone_blocks(const uint8_t* host_in, const uint8_t* d_in,
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
BulkResult bulk_linked(const uint8_t* d_frame, uint64_t frame_len, int64_t block_max,
                              const std::vector<lz4ada_block_desc>& descs, LinkedSink& sink,
                              uint64_t& total, std::vector<uint32_t>& lens, int64_t& fail,
                              hipStream_t stream, const LinkedHist* hist = nullptr);

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

// ------------------------------------------------ bulk-path device helpers

// A device allocation that may fail without raising (the bulk path then
// shrinks its batch or hands the frame to the exact path).
template <class T>
inline bool try_reserve(DevBuf<T>& b, size_t count)
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
enum ScratchRole { SC_FRAME, SC_OUT, SC_COMPACT, SC_X, SC_Y, SC_H, SC_Z, SC_TAB, SC_P, SC_F, SC_LONE, SC_U,
	           SC_LINK, SC_M, SC_N };
struct ScratchCache {
	DevBuf<uint8_t> b[SC_N];
	PinBuf pin;  // the linked path's small host transfers (pinned: no staging copy)
};
inline ScratchCache& scratch_cache()
{
	static thread_local ScratchCache* c = new ScratchCache;
	return *c;
}
inline void scratch_release()
{
	for (auto& x : scratch_cache().b)
		x.release();
	scratch_cache().pin.release();
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
inline bool decode_lone_blocks(const uint8_t* host_in, const uint8_t* d_in,
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
inline std::vector<std::pair<uint32_t, uint32_t>> batches_of(const std::vector<lz4ada_block_desc>& descs,
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

inline void d2h(void* dst, const void* src, size_t n, hipStream_t stream)
{
	HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, stream));
	HIP_OK(hipStreamSynchronize(stream));
}


// Reference-exact path for one frame: the unlz4ada loop
// (tool_unlz4ada/unlz4ada.adb:84-103) over the streaming engine, from the
// frame start or from `resume` (lz4ada_facade.cpp).
void exact_frame(const uint8_t* f, int64_t len, Sink& out, int64_t& consumed_total,
                 const Resume* resume = nullptr);

// The content hash of device-resident output through the D2H pipeline
// (lz4ada_facade.cpp); host_out gets the bytes on the way (may be null).
void content_xxh32_d2h(lz4ada_xxh32_state& h, const uint8_t* d_data, int64_t len, uint8_t* host_out,
                       hipStream_t stream);

// A C-ABI call: the reference's exception as the status code, its text in
// *err (the context's) and in the thread's last error.
template <class F>
inline int guarded(std::string* err, F&& f)
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

}  // namespace lz4ada

