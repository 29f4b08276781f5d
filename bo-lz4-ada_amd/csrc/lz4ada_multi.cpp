// lz4ada_multi.cpp -- one frame over several GPUs from ONE process (SURVEY
// §8b "a bulk entry ... n_gpus", §8e): the C-ABI twin of bo-lz4-ada_amd/shard.py
// for callers that are not torch.distributed jobs (the Ada CLI).
//
// A frame whose blocks are independent (FLG.B.Indep) is split into
// contiguous block ranges balanced by compressed bytes (lz4ada_plan_shards,
// the rule of shard.py plan_shards).  One host worker thread per device
// copies only its range of the compressed frame to its GPU and runs the bulk
// decoder on it (lz4ada_decode_blocks_device) -- no data-path collective.
// RCCL (one communicator per device, ncclCommInitAll) carries:
//   * ONE all-reduce(MAX) of an (n+1)-word record: word 0 the rank's block
//     status, word 1+r rank r's decoded byte count (every other rank writes
//     0 there), so each rank learns the verdict and its output offset;
//   * the optional gather of every rank's bytes into one buffer on the first
//     device (ncclSend / ncclRecv), for device-resident consumers.
// Each rank copies its bytes straight to the caller's host buffer at its
// offset; the calling thread runs the frame's content checksum as ONE XXH32
// chain in frame order (lz4ada.adb:709-714, 493-501), rank r's bytes as soon
// as they have landed.
//
// Anything the bulk path would not take -- a block error or checksum
// mismatch, a block reading an earlier one (D2), a failed frame-level check,
// a linked or legacy frame -- goes to the single-GPU lz4ada_decode_frame on
// the first device, which gives the reference's output or exception (errors
// at the failing block, lz4ada.adb:672-676).
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "lz4ada_internal.h"

namespace lz4ada {
namespace {

// shard.py plan_shards: rank r takes the blocks whose compressed-prefix
// midpoint lies in [r, r+1) * total / n (in exact integers: 2 * midpoint).
void plan(const lz4ada_block_desc* d, int64_t nb, int n, int64_t* bounds)
{
	uint64_t total = 0;
	for (int64_t i = 0; i < nb; ++i)
		total += d[i].in_len;
	bounds[0] = 0;
	bounds[n] = nb;
	int r = 1;
	uint64_t acc = 0;
	for (int64_t i = 0; i < nb; ++i) {
		const uint64_t mid2 = 2 * acc + d[i].in_len;
		while (r < n && mid2 * uint64_t(n) >= 2 * uint64_t(r) * total)
			bounds[r++] = i;
		acc += d[i].in_len;
	}
	while (r < n)
		bounds[r++] = nb;
}

// A device buffer that only grows: the worker keeps one per role across
// calls, so a repeated call allocates nothing.
struct DevMem {
	void* p = nullptr;
	size_t cap = 0;
	~DevMem()
	{
		if (p)
			(void)hipFree(p);
	}
	hipError_t alloc(size_t n)
	{
		n = std::max<size_t>(n, 1);
		if (p && n <= cap)
			return hipSuccess;
		reset();
		const hipError_t e = hipMalloc(&p, n);
		if (e != hipSuccess) {
			p = nullptr;
			return e;
		}
		cap = n;
		return hipSuccess;
	}
	void reset()
	{
		if (p)
			(void)hipFree(p);
		p = nullptr;
		cap = 0;
	}
	uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};

// Per-device state kept by its worker between calls (used only on the
// worker's thread): the rank's buffers, two pinned staging chunks for the
// H2D, a copy stream and a few decode streams, so that a group of blocks
// decodes while the next one is still crossing PCIe.
constexpr int NDEC = 4;
constexpr size_t STAGE_BYTES = size_t(64) << 20;
struct DevCache {
	DevMem in, desc, st, out, comp, off, meta;
	uint8_t* pinned[2] = { nullptr, nullptr };
	hipStream_t copy = nullptr;
	hipStream_t dec[NDEC] = {};
	hipEvent_t landed[2] = { nullptr, nullptr };
	hipEvent_t done[NDEC] = {};
	int allocs = 0;  // device allocations made so far (lz4ada_multi_device_allocs)
};

// One long-lived host thread per device ordinal: its HIP stream, and the
// per-thread side streams of the bulk decoder, live as long as the process
// (a thread per call would leave streams behind at every call).
class Worker {
public:
	Worker() : th_([this] { loop(); }) { th_.detach(); }
	std::future<void> run(std::function<void()> f)
	{
		auto t = std::make_shared<std::packaged_task<void()>>(std::move(f));
		std::future<void> fut = t->get_future();
		{
			std::lock_guard<std::mutex> g(m_);
			q_.push_back([t] { (*t)(); });
		}
		cv_.notify_one();
		return fut;
	}
	hipStream_t stream = nullptr;  // created by the first job, on this thread
	DevCache cache;                // buffers and staging kept across calls

private:
	void loop()
	{
		for (;;) {
			std::function<void()> f;
			{
				std::unique_lock<std::mutex> l(m_);
				cv_.wait(l, [&] { return !q_.empty(); });
				f = std::move(q_.front());
				q_.pop_front();
			}
			f();
		}
	}
	std::mutex m_;
	std::condition_variable cv_;
	std::deque<std::function<void()>> q_;
	std::thread th_;  // last: starts once the members above exist
};

std::mutex g_multi;  // one multi-GPU call at a time (the communicators are shared)

// The worker of a device ordinal, created on first use.  The pool is looked
// up from the calling thread and from the workers' own threads, so it is
// guarded (a find racing an insert on the first multi-GPU call).
std::mutex pool_mutex;
std::map<int, Worker*>* pool = new std::map<int, Worker*>;  // never freed: detached threads use it

Worker& worker(int dev)
{
	std::lock_guard<std::mutex> g(pool_mutex);
	auto it = pool->find(dev);
	if (it == pool->end())
		it = pool->emplace(dev, new Worker).first;
	return *it->second;
}

bool has_worker(int dev)
{
	std::lock_guard<std::mutex> g(pool_mutex);
	return pool->count(dev) != 0;
}

// RCCL communicators per device list, created once (ncclCommInitAll costs
// far more than a decode of a small frame).
ncclResult_t comms_for(const std::vector<int>& devs, std::vector<ncclComm_t>*& out)
{
	static auto* cache = new std::map<std::vector<int>, std::vector<ncclComm_t>>;
	auto it = cache->find(devs);
	if (it == cache->end()) {
		std::vector<ncclComm_t> c(devs.size());
		const ncclResult_t r = ncclCommInitAll(c.data(), int(devs.size()), devs.data());
		if (r != ncclSuccess)
			return r;
		it = cache->emplace(devs, std::move(c)).first;
	}
	out = &it->second;
	return ncclSuccess;
}

// rank status words (all-reduced with MAX: the worst one wins)
enum : int64_t { RS_OK = 0, RS_BLOCK_ERROR = 1, RS_PRE_REF = 2, RS_DEVICE = 3 };

struct Rank {
	int dev = 0;
	int64_t lo = 0, hi = 0;
	ncclComm_t comm = nullptr;
	// after the all-reduce
	std::vector<int64_t> words;
	std::string err;  // HIP / RCCL failure on this rank
	std::promise<bool> landed;  // host bytes in place (the checksum chain may read them)
};

#define TRY_HIP(expr, what)                                                                  \
	do {                                                                                     \
		const hipError_t e_ = (expr);                                                        \
		if (e_ != hipSuccess)                                                                \
			throw std::string(what) + ": " + hipGetErrorString(e_);                          \
	} while (0)
#define TRY_NCCL(expr, what)                                                                 \
	do {                                                                                     \
		const ncclResult_t e_ = (expr);                                                      \
		if (e_ != ncclSuccess)                                                               \
			throw std::string(what) + ": " + ncclGetErrorString(e_);                         \
	} while (0)

static void grow(DevCache& c, DevMem& m, size_t n)
{
	const bool fresh = !m.p || std::max<size_t>(n, 1) > m.cap;
	TRY_HIP(m.alloc(n), "hipMalloc");
	if (fresh)
		++c.allocs;
}

// Phase 1 (before any collective): device, stream and the status record.
// A rank that cannot get this far would leave the others waiting in the
// all-reduce, so the call stops here if any rank fails.
void prepare(Rank& rk, int n)
{
	Worker& w = worker(rk.dev);
	TRY_HIP(hipSetDevice(rk.dev), "hipSetDevice");
	if (!w.stream)
		TRY_HIP(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking), "hipStreamCreate");
	DevCache& c = w.cache;
	if (!c.copy) {
		TRY_HIP(hipStreamCreateWithFlags(&c.copy, hipStreamNonBlocking), "hipStreamCreate");
		for (int i = 0; i < NDEC; ++i) {
			TRY_HIP(hipStreamCreateWithFlags(&c.dec[i], hipStreamNonBlocking), "hipStreamCreate");
			TRY_HIP(hipEventCreateWithFlags(&c.done[i], hipEventDisableTiming), "hipEventCreate");
		}
		for (int i = 0; i < 2; ++i) {
			TRY_HIP(hipEventCreateWithFlags(&c.landed[i], hipEventDisableTiming), "hipEventCreate");
			TRY_HIP(hipHostMalloc(reinterpret_cast<void**>(&c.pinned[i]), STAGE_BYTES, hipHostMallocDefault),
			        "hipHostMalloc");
		}
	}
	grow(c, c.meta, size_t(n + 1) * sizeof(int64_t));
}

// Phase 2: this rank's blocks, the all-reduce, the host copy, the gather.
void run_rank(Rank& rk, int r, int n, const uint8_t* frame, uint64_t frame_len,
              const lz4ada_block_desc* descs, int64_t block_max, uint8_t* out, int64_t out_cap, uint8_t* d_gather,
              int64_t gather_cap)
{
	Worker& w = worker(rk.dev);
	hipStream_t s = w.stream;
	DevCache& c = w.cache;
	const int64_t k = rk.hi - rk.lo;
	int64_t status = RS_OK, total = 0;
	const uint8_t* d_res = nullptr;
	try {
		TRY_HIP(hipSetDevice(rk.dev), "hipSetDevice");
		if (k > 0) {
			const lz4ada_block_desc* g = descs + rk.lo;
			const uint64_t b0 = g[0].in_off;
			uint64_t b1 = b0;
			std::vector<lz4ada_block_desc> loc(size_t(k), lz4ada_block_desc{});
			for (int64_t j = 0; j < k; ++j) {
				loc[size_t(j)] = g[j];
				loc[size_t(j)].in_off = g[j].in_off - b0;
				loc[size_t(j)].out_off = uint64_t(j) * uint64_t(block_max);
				loc[size_t(j)].out_cap = uint32_t(block_max);
				b1 = std::max<uint64_t>(b1, g[j].in_off + g[j].in_len + 4);
			}
			b1 = std::min<uint64_t>(b1, frame_len);
			const uint64_t out_bytes = uint64_t(k) * uint64_t(block_max);
			grow(c, c.in, b1 - b0);
			grow(c, c.desc, size_t(k) * sizeof(lz4ada_block_desc));
			grow(c, c.st, size_t(k) * sizeof(lz4ada_block_status));
			grow(c, c.out, out_bytes);
			auto* d_desc = static_cast<lz4ada_block_desc*>(c.desc.p);
			auto* d_st = static_cast<lz4ada_block_status*>(c.st.p);
			TRY_HIP(hipMemcpyAsync(d_desc, loc.data(), size_t(k) * sizeof(lz4ada_block_desc),
			                       hipMemcpyHostToDevice, c.copy),
			        "H2D");
			TRY_HIP(hipMemsetAsync(d_st, 0, size_t(k) * sizeof(lz4ada_block_status), c.copy), "memset");
			// Groups of whole blocks of at most STAGE_BYTES of input: the host
			// copies group i into pinned chunk i & 1 while the DMA of group
			// i - 1 runs, and group i decodes on its own stream as soon as its
			// bytes have landed, beside the later copies.
			int64_t j0 = 0;
			int grp = 0;
			while (j0 < k) {
				int64_t j1 = j0 + 1;
				const uint64_t g0 = loc[size_t(j0)].in_off;
				while (j1 < k && loc[size_t(j1)].in_off + loc[size_t(j1)].in_len + 4 - g0 <= STAGE_BYTES)
					++j1;
				const uint64_t g1 = j1 < k ? loc[size_t(j1)].in_off - 4 : b1 - b0;  // up to the next size word
				const int slot = grp & 1;
				if (grp >= 2)  // the DMA that last read this chunk
					TRY_HIP(hipEventSynchronize(c.landed[slot]), "staging");
				for (uint64_t x = g0; x < g1;) {  // (a block over STAGE_BYTES: in pieces)
					const uint64_t nx = std::min<uint64_t>(g1 - x, STAGE_BYTES);
					if (x > g0)
						TRY_HIP(hipEventSynchronize(c.landed[slot]), "staging");
					memcpy(c.pinned[slot], frame + b0 + x, size_t(nx));
					TRY_HIP(hipMemcpyAsync(c.in.u8() + x, c.pinned[slot], size_t(nx),
					                       hipMemcpyHostToDevice, c.copy),
					        "H2D");
					TRY_HIP(hipEventRecord(c.landed[slot], c.copy), "event");
					x += nx;
				}
				hipStream_t ds = c.dec[grp % NDEC];
				TRY_HIP(hipStreamWaitEvent(ds, c.landed[slot], 0), "event wait");
				if (lz4ada_decode_blocks_device(c.in.p, b1 - b0, d_desc + j0, j1 - j0, c.out.p,
				                                d_st + j0, ds) != LZ4ADA_OK)
					throw std::string(lz4ada_thread_last_error());
				j0 = j1;
				++grp;
			}
			for (int i = 0; i < NDEC && i < grp; ++i) {
				TRY_HIP(hipEventRecord(c.done[i], c.dec[i]), "event");
				TRY_HIP(hipStreamWaitEvent(s, c.done[i], 0), "event wait");
			}
			std::vector<lz4ada_block_status> st(static_cast<size_t>(k));
			TRY_HIP(hipMemcpyAsync(st.data(), d_st, size_t(k) * sizeof(lz4ada_block_status),
			                       hipMemcpyDeviceToHost, s),
			        "D2H");
			TRY_HIP(hipStreamSynchronize(s), "decode");
			bool contiguous = true;
			std::vector<uint64_t> dst(static_cast<size_t>(k));
			for (int64_t j = 0; j < k && status == RS_OK; ++j) {
				const auto& b = st[size_t(j)];
				if ((loc[size_t(j)].flags & LZ4ADA_BLOCK_HAS_CKSUM) && b.cksum != loc[size_t(j)].cksum)
					status = RS_BLOCK_ERROR;
				else if (b.code == DS_PRE_BLOCK_REF)
					status = RS_PRE_REF;
				else if (b.code != DS_OK)
					status = RS_BLOCK_ERROR;
				dst[size_t(j)] = uint64_t(total);
				if (uint64_t(total) != loc[size_t(j)].out_off)
					contiguous = false;
				total += b.out_len;
			}
			d_res = c.out.u8();
			if (status == RS_OK && !contiguous) {  // a short block before the last one
				grow(c, c.comp, size_t(total));
				grow(c, c.off, size_t(k) * sizeof(uint64_t));
				TRY_HIP(hipMemcpyAsync(c.off.p, dst.data(), size_t(k) * sizeof(uint64_t),
				                       hipMemcpyHostToDevice, s),
				        "H2D");
				TRY_HIP(launch_compact(c.out.u8(), d_desc, static_cast<const uint64_t*>(c.off.p), d_st,
				                       uint32_t(k), c.comp.u8(), s),
				        "compact");
				d_res = c.comp.u8();
			}
		}
	} catch (const std::string& e) {
		status = RS_DEVICE;
		total = 0;
		rk.err = e;
	}
	// the one verdict collective; every rank reaches it
	try {
		std::vector<int64_t> words(static_cast<size_t>(n + 1), 0);
		words[0] = status;
		words[size_t(1 + r)] = total;
		TRY_HIP(hipMemcpyAsync(c.meta.p, words.data(), words.size() * sizeof(int64_t),
		                       hipMemcpyHostToDevice, s),
		        "H2D");
		TRY_NCCL(ncclAllReduce(c.meta.p, c.meta.p, words.size(), ncclInt64, ncclMax, rk.comm, s),
		         "ncclAllReduce");
		TRY_HIP(hipMemcpyAsync(words.data(), c.meta.p, words.size() * sizeof(int64_t),
		                       hipMemcpyDeviceToHost, s),
		        "D2H");
		TRY_HIP(hipStreamSynchronize(s), "all-reduce");
		rk.words = words;
		if (words[0] != RS_OK)
			throw std::string();  // the verdict: nothing to copy (not an error of this rank)
		int64_t prefix = 0, sum = 0;
		for (int q = 0; q < n; ++q) {
			if (q < r)
				prefix += words[size_t(1 + q)];
			sum += words[size_t(1 + q)];
		}
		// the same decisions on every rank (they all hold the same words)
		if (d_gather && sum <= gather_cap) {
			if (r == 0) {
				TRY_NCCL(ncclGroupStart(), "ncclGroupStart");
				int64_t off = words[1];
				for (int q = 1; q < n; ++q) {
					const int64_t nq = words[size_t(1 + q)];
					if (nq > 0)
						TRY_NCCL(ncclRecv(d_gather + off, size_t(nq), ncclUint8, q, rk.comm, s),
						         "ncclRecv");
					off += nq;
				}
				TRY_NCCL(ncclGroupEnd(), "ncclGroupEnd");
				if (total > 0)
					TRY_HIP(hipMemcpyAsync(d_gather, d_res, size_t(total), hipMemcpyDeviceToDevice, s),
					        "D2D");
			} else if (total > 0) {
				TRY_NCCL(ncclSend(d_res, size_t(total), ncclUint8, 0, rk.comm, s), "ncclSend");
			}
		}
		if (out && sum <= out_cap && total > 0)
			TRY_HIP(hipMemcpyAsync(out + prefix, d_res, size_t(total), hipMemcpyDeviceToHost, s),
			        "D2H");
		TRY_HIP(hipStreamSynchronize(s), "output");
		rk.landed.set_value(true);
	} catch (const std::string& e) {
		rk.err = e;
		rk.landed.set_value(false);
	}
}

// The single-GPU product path on the first device: the reference's result
// for anything the sharded bulk path does not take.
int single_gpu(int dev, const uint8_t* frame, int64_t len, uint8_t* out, int64_t out_cap,
               uint8_t* d_gather, int64_t gather_cap, int64_t* out_len, int64_t* consumed)
{
	int prev = 0;
	(void)hipGetDevice(&prev);
	if (hipSetDevice(dev) != hipSuccess) {
		set_thread_error("hipSetDevice failed");
		return LZ4ADA_DEVICE_ERROR;
	}
	int st;
	if (out) {
		st = lz4ada_decode_frame(frame, len, out, out_cap, out_len, consumed);
		if (st == LZ4ADA_OK && d_gather && *out_len <= gather_cap &&
		    hipMemcpy(d_gather, out, size_t(*out_len), hipMemcpyHostToDevice) != hipSuccess) {
			set_thread_error("hipMemcpy to the gather buffer failed");
			st = LZ4ADA_DEVICE_ERROR;
		}
	} else {
		uint8_t* tmp = nullptr;
		st = lz4ada_decode_frame_alloc(frame, len, &tmp, out_len, consumed);
		if (st == LZ4ADA_OK) {
			if (*out_len > gather_cap) {
				set_thread_error("output capacity exceeded");
				st = LZ4ADA_CONSTRAINT_ERROR;
			} else if (*out_len &&
			           hipMemcpy(d_gather, tmp, size_t(*out_len), hipMemcpyHostToDevice) != hipSuccess) {
				set_thread_error("hipMemcpy to the gather buffer failed");
				st = LZ4ADA_DEVICE_ERROR;
			}
		}
		lz4ada_buffer_free(tmp);
	}
	(void)hipSetDevice(prev);
	return st;
}

int decode_multi(const uint8_t* frame, int64_t len, int n, const int* devices, uint8_t* out,
                 int64_t out_cap, uint8_t* d_gather, int64_t gather_cap, int64_t* out_len,
                 int64_t* consumed)
{
	*out_len = 0;
	*consumed = 0;
	set_last_path(0);
	if (n < 1 || (!out && !d_gather) || len < 0 || (!frame && len > 0)) {
		set_thread_error("lz4ada_decode_frame_multi: n_gpus >= 1 and an output are required");
		return LZ4ADA_ASSERTION_ERROR;
	}
	std::vector<int> devs(static_cast<size_t>(n));
	for (int r = 0; r < n; ++r)
		devs[size_t(r)] = devices ? devices[r] : r;
	int count = 0;
	if (hipGetDeviceCount(&count) != hipSuccess || count < 1) {
		set_thread_error("no usable HIP device");
		return LZ4ADA_DEVICE_ERROR;
	}
	for (int d : devs)
		if (d < 0 || d >= count) {
			set_thread_error("device ordinal " + std::to_string(d) + " out of range (" +
			                 std::to_string(count) + " devices)");
			return LZ4ADA_DEVICE_ERROR;
		}
	std::lock_guard<std::mutex> one(g_multi);
	lz4ada_frame_info info{};
	std::vector<lz4ada_block_desc> descs;
	bool shard = lz4ada_frame_index(frame, len, &info, nullptr, 0) == LZ4ADA_OK &&
	             info.format == LZ4ADA_FORMAT_MODERN && info.independent && info.frame_len <= len;
	if (shard) {
		descs.resize(size_t(std::max<int64_t>(info.nblocks, 1)));
		shard = lz4ada_frame_index(frame, len, &info, descs.data(), info.nblocks) == LZ4ADA_OK;
	}
	if (!shard)  // linked, legacy or skippable frames, or ones that do not index
		return single_gpu(devs[0], frame, len, out, out_cap, d_gather, gather_cap, out_len,
		                  consumed);
	std::vector<int64_t> bounds(static_cast<size_t>(n + 1));
	plan(descs.data(), info.nblocks, n, bounds.data());
	std::vector<ncclComm_t>* comms = nullptr;
	const ncclResult_t cr = comms_for(devs, comms);
	if (cr != ncclSuccess) {
		set_thread_error(std::string("ncclCommInitAll: ") + ncclGetErrorString(cr));
		return LZ4ADA_DEVICE_ERROR;
	}
	std::vector<Rank> ranks(static_cast<size_t>(n));
	std::vector<std::string> perr(static_cast<size_t>(n));
	std::vector<std::future<void>> fut;
	for (int r = 0; r < n; ++r) {
		Rank& rk = ranks[size_t(r)];
		rk.dev = devs[size_t(r)];
		rk.lo = bounds[size_t(r)];
		rk.hi = bounds[size_t(r + 1)];
		rk.comm = (*comms)[size_t(r)];
		fut.push_back(worker(rk.dev).run([&rk, &perr, r, n] {
			try {
				prepare(rk, n);
			} catch (const std::string& e) {
				perr[size_t(r)] = e;
			}
		}));
	}
	for (auto& f : fut)
		f.get();
	for (int r = 0; r < n; ++r)
		if (!perr[size_t(r)].empty()) {
			set_thread_error("device " + std::to_string(devs[size_t(r)]) + ": " + perr[size_t(r)]);
			return LZ4ADA_DEVICE_ERROR;
		}
	std::vector<std::future<bool>> landed;
	for (auto& rk : ranks)
		landed.push_back(rk.landed.get_future());
	fut.clear();
	for (int r = 0; r < n; ++r)
		fut.push_back(worker(devs[size_t(r)]).run([&, r] {
			run_rank(ranks[size_t(r)], r, n, frame, uint64_t(info.frame_len), descs.data(), info.block_max, out, out_cap,
			         d_gather, gather_cap);
		}));
	// the content checksum: one chain in frame order over the host bytes,
	// rank r's as soon as they have landed
	lz4ada_xxh32_state h;
	lz4ada_xxh32_reset(&h, 0);
	bool ok = true;
	int64_t pos = 0;
	for (int r = 0; r < n; ++r) {
		if (!landed[size_t(r)].get()) {
			ok = false;
			continue;  // every future is still collected
		}
		const int64_t nr = ranks[size_t(r)].words[size_t(1 + r)];
		if (ok && out && info.content_checksum && nr > 0 && pos + nr <= out_cap)
			lz4ada_xxh32_update(&h, out + pos, nr);
		pos += nr;
	}
	for (auto& f : fut)
		f.get();
	for (int r = 0; r < n; ++r)
		if (!ranks[size_t(r)].err.empty()) {
			set_thread_error("device " + std::to_string(devs[size_t(r)]) + ": " +
			                 ranks[size_t(r)].err);
			return LZ4ADA_DEVICE_ERROR;
		}
	const int64_t verdict = ranks[0].words.empty() ? RS_DEVICE : ranks[0].words[0];
	if (verdict == RS_DEVICE) {
		set_thread_error("a device failed during the sharded decode");
		return LZ4ADA_DEVICE_ERROR;
	}
	if (ok && verdict == RS_OK) {
		const int64_t total = pos;
		if ((out && total > out_cap) || (!out && total > gather_cap)) {
			set_thread_error("output capacity exceeded");
			return LZ4ADA_CONSTRAINT_ERROR;
		}
		bool good = !info.has_content_size || uint64_t(total) == info.content_size;
		if (good && info.content_checksum) {
			if (!out) {  // only the gathered copy: its bytes through the D2H chain
				int prev = 0;
				(void)hipGetDevice(&prev);
				good = hipSetDevice(devs[0]) == hipSuccess &&
				       lz4ada_content_xxh32_d2h(&h, d_gather, total, nullptr, nullptr) == LZ4ADA_OK;
				(void)hipSetDevice(prev);
			}
			const uint32_t got = total == 0 ? 0x02cc5d05u : lz4ada_xxh32_final(&h);
			good = good && got == info.content_checksum_declared;
		}
		if (good) {
			*out_len = total;
			*consumed = info.frame_len;
			set_last_path(LZ4ADA_PATH_INDEPENDENT | LZ4ADA_PATH_MULTI);
			return LZ4ADA_OK;
		}
	}
	// a bad block, a block reading an earlier one (D2) or a failed frame
	// check: the single-GPU path decides, as the reference would
	const int st = single_gpu(devs[0], frame, len, out, out_cap, d_gather, gather_cap, out_len,
	                          consumed);
	set_last_path(lz4ada_last_path() | LZ4ADA_PATH_MULTI);
	return st;
}

}  // namespace
}  // namespace lz4ada

extern "C" {

int lz4ada_plan_shards(const lz4ada_block_desc* descs, int64_t nblocks, int n_gpus,
                       int64_t* bounds)
{
	if (n_gpus < 1 || nblocks < 0 || (!descs && nblocks > 0) || !bounds) {
		lz4ada::set_thread_error("lz4ada_plan_shards: n_gpus >= 1 and bounds[n_gpus + 1] required");
		return LZ4ADA_ASSERTION_ERROR;
	}
	lz4ada::plan(descs, nblocks, n_gpus, bounds);
	return LZ4ADA_OK;
}

int lz4ada_decode_frame_multi(const uint8_t* frame, int64_t len, int n_gpus, const int* devices,
                              uint8_t* out, int64_t out_cap, int64_t* out_len,
                              int64_t* frame_consumed)
{
	if (!out) {
		lz4ada::set_thread_error("lz4ada_decode_frame_multi: out is required");
		return LZ4ADA_ASSERTION_ERROR;
	}
	return lz4ada::decode_multi(frame, len, n_gpus, devices, out, out_cap, nullptr, 0, out_len,
	                            frame_consumed);
}

int lz4ada_decode_frame_multi_gather(const uint8_t* frame, int64_t len, int n_gpus,
                                     const int* devices, void* d_out, int64_t out_cap,
                                     int64_t* out_len, int64_t* frame_consumed)
{
	if (!d_out) {
		lz4ada::set_thread_error("lz4ada_decode_frame_multi_gather: d_out is required");
		return LZ4ADA_ASSERTION_ERROR;
	}
	return lz4ada::decode_multi(frame, len, n_gpus, devices, nullptr, 0,
	                            static_cast<uint8_t*>(d_out), out_cap, out_len, frame_consumed);
}

}  // extern "C"

extern "C" {

int64_t lz4ada_multi_device_allocs(int device)
{
	std::lock_guard<std::mutex> one(lz4ada::g_multi);
	if (!lz4ada::has_worker(device))
		return -1;
	return lz4ada::worker(device).cache.allocs;
}

int lz4ada_rccl_version(void)
{
	int v = 0;
	return ncclGetVersion(&v) == ncclSuccess ? v : -1;
}

}  // extern "C"
