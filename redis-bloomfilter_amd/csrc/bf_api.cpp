// bf_api.cpp — the C ABI declared in include/bfhip.h.
//
// Owns the device bitset (one HIP device per handle), a HIP stream, and two
// staging slots (pinned host + device) used by the host-pointer calls so that
// packing chunk c+1 on the host overlaps the device work of chunk c.
#include "bfhip.h"
#include "bf_internal.h"
#include "bf_multi.h"
#include "bf_device.h"   // bfdev::key_ok: bf_check_offsets applies the kernels' rule

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#define BFHIP_VERSION_STR "bfhip 0.1.0 (gfx950; redis-bloomfilter 1.1.2 ruby-driver layout)"

namespace {

thread_local std::string g_create_error;

// A fork-join pool for the host side of the host-pointer calls: the offsets scan and the
// staging copies into pinned memory are memory-bandwidth work that one core cannot feed
// to PCIe (r01: 4-5e8 keys/s behind a single memcpy thread).  Workers start on first use;
// the calling thread takes parts too.
class HostPool {
public:
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : th_) t.join();
    }
    unsigned size() const { return (unsigned)th_.size() + 1; }
    void start(unsigned n) {
        if (!th_.empty() || n <= 1) return;
        for (unsigned i = 1; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    // fn(p) for every p < parts; returns when all are done.
    void run(unsigned parts, const std::function<void(unsigned)>& fn) {
        if (parts <= 1 || th_.empty()) {
            for (unsigned p = 0; p < parts; ++p) fn(p);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            parts_ = parts;
            next_.store(0);
            active_ = (unsigned)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return active_ == 0; });
        fn_ = nullptr;
    }

private:
    void work() {
        for (unsigned p; (p = next_.fetch_add(1)) < parts_;) (*fn_)(p);
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            lk.unlock();
            work();
            lk.lock();
            if (--active_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(unsigned)>* fn_ = nullptr;
    unsigned parts_ = 0, active_ = 0;
    std::atomic<unsigned> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// Host threads for the staging work: BFHIP_HOST_THREADS, else the CPUs this process may run
// on (its affinity mask, capped by the cgroup CPU quota), at most 16 — past that the copies
// saturate host memory bandwidth.
unsigned host_threads() {
    if (const char* v = getenv("BFHIP_HOST_THREADS"))
        if (*v) return std::max(1u, (unsigned)strtoul(v, nullptr, 10));
    cpu_set_t set;
    unsigned n = 1;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = (unsigned)CPU_COUNT(&set);
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long long period = 0;
        if (fscanf(f, "%31s %llu", q, &period) == 2 && strcmp(q, "max") != 0 && period)
            n = std::min<unsigned>(n, (unsigned)std::max(1ull, (strtoull(q, nullptr, 10) + period - 1) / period));
        fclose(f);
    }
    return std::max(1u, std::min(16u, n));
}

// One staging slot of the host-pointer pipeline: pinned host + device buffers for a chunk's
// key bytes, its uint32 relative offsets (widened on the device) and its per-key results.
struct Slot {
    uint8_t*  h_keys = nullptr;    // pinned, cap_bytes + 16
    uint32_t* h_off = nullptr;     // pinned, cap_keys + 1
    uint8_t*  h_out = nullptr;     // pinned, out_cap
    uint8_t*  d_keys = nullptr;
    uint32_t* d_off32 = nullptr;
    uint64_t* d_off = nullptr;
    uint8_t*  d_out = nullptr;
    uint64_t  cap_bytes = 0, cap_keys = 0, out_cap = 0;
    hipEvent_t h2d = nullptr;      // the chunk's inputs are on the device (copy stream)
    hipEvent_t done = nullptr;     // the chunk's kernels and result copy are done
    hipEvent_t op = nullptr;       // the chunk's kernels are done (compute stream; its D2H waits for it)
    // pending result copy-out
    bool      busy = false;
    uint8_t*  user_out = nullptr;
    uint64_t  out_bytes = 0;
};
constexpr int kSlots = 3;   // host staging of chunk c+2 || H2D of c+1 || kernels of c

}  // namespace

struct bf_handle {
    std::mutex mu;
    int device = 0;
    hipStream_t stream = nullptr;
    BfGeom g{};
    uint64_t m = 0, reach = 0, dev_bytes = 0;
    uint32_t k = 0;
    // partitioned filters: this handle holds shard `shard_index` of `shards`
    uint32_t shards = 1, shard_index = 0, block_log2 = 20;
    uint32_t mem_kind = 0;   // bitset allocation: 0 coarse-grained, 1 uncached, 2 fine-grained
    bool route32 = false;    // BF_FLAG_ROUTE32
    uint32_t engine = BF_ENGINE_RUBY;   // BF_FLAG_ENGINE_*: the RubyTest hash engines
    uint64_t local_bits = 0;
    // routing scratch (grown on demand)
    uint64_t* d_tmp_local = nullptr;
    uint8_t*  d_tmp_owner = nullptr;
    uint64_t  tmp_cap = 0;
    unsigned long long* d_cursor = nullptr;
    // binned-insert scratch (grown on demand) and policy: 0 never, 1 always, 2 auto
    uint32_t binned_mode = 2;
    uint32_t include_binned_mode = 2;   // the same policy for include?
    uint32_t shard_test_binned_mode = 2;   // ... and for the owner-side test of routed probes
    uint32_t bin_region_log2 = 19;   // preferred region (LDS image) size of the apply pass
    // chunked windows.  The owner's include? takes the superbin-major L2-local sweep
    // (chunk_test_l2_kernel) when the route's buckets can make superbins of <= 4 MiB (512 buckets:
    // the north-star shards at P = 2..8): 0.89 ms against 1.08 for sort + region test, 3.22 vs
    // 3.38 ms per P = 8 rank step.  Otherwise (8 MiB+ superbins, e.g. 200B x 8: 3.44 vs 3.11 ms)
    // it sorts, with 256 buckets (longer runs for the owner's mid).  profiles/r03_sim_chunks_P8.jsonl.
    // BFHIP_CHUNK_BUCKETS forces the bucket count, BFHIP_CHUNK_TEST_L2=0/1 the test (A/B only).
    uint32_t chunk_buckets = 0;   // 0: auto
    uint32_t chunk_test_l2 = 2;   // 2: auto
    void* d_bin_scratch = nullptr;   // digests, probe arrays and histograms of one binned launch
    uint64_t bin_scratch_cap = 0;
    uint64_t cap_keys = 0, cap_bytes = 0;   // chunk limits of the host-pointer calls (bf_config)
    Slot slot[kSlots];
    bool staging_ready = false;
    hipStream_t copy_stream = nullptr;      // H2D of the host-pointer pipeline
    hipStream_t d2h_stream = nullptr;       // ... and its result copies (PCIe is full duplex)
    HostPool pool;
    uint32_t* d_flag = nullptr;
    unsigned long long* d_scan = nullptr;
    uint32_t* h_flag = nullptr;   // pinned
    uint32_t* h_key_status = nullptr;   // pinned, written by the hashing kernels (take_key_status)
    // bf_shard_test_chunks_packed_dev's answer bytes and segment table (forms that pack afterwards)
    uint8_t* d_ans8 = nullptr;
    uint64_t ans8_cap = 0;
    uint64_t* d_seg = nullptr;
    uint64_t seg_cap = 0;
    uint32_t seg_nsrc = 0, seg_nh = 0;   // the geometry d_seg holds
    uint64_t seg_wcap = 0;
    // latency path of small host-pointer calls (run_small): one pinned and one device arena
    uint8_t* h_small = nullptr;
    uint8_t* d_small = nullptr;
    uint64_t small_cap = 0;
    // incremental Redis sync (bf_track_dirty): one byte per BF_DIRTY_BLOCK_BYTES of the string
    uint8_t* d_dirty = nullptr;
    uint64_t dirty_blocks = 0;
    // per-kernel timing (bf_profile): event sets awaiting harvest, recycled sets, totals
    bool profile = false;
    std::vector<BfMarks> prof_pending, prof_free;
    struct ProfAcc { std::string name; double ms; uint64_t launches; };
    std::vector<ProfAcc> prof_acc;
    // cross-stream ordering (StreamOrder): the event after the handle's last device work
    hipEvent_t order_ev = nullptr;
    hipStream_t order_stream = nullptr;
    bool order_valid = false;
    BfMulti* multi = nullptr;   // a multi-device handle (bf_config.device_count > 0): bf_multi.cpp
    std::string err;
};

namespace {

// Orders one handle's device work across streams.  Every entry point that touches the
// bitset or the handle's scratch (the binned / sequential arenas, staging, routing
// scratch) holds one of these around its launches: work arriving on a different stream
// than the previous call's first waits for that call's last launch (hipStreamWaitEvent,
// no host sync), so *_dev calls on two streams never race on the shared scratch or on
// bin_apply's plain region stores.  Calls on one stream pay only an event record.
// The key-status word (BfGeom::key_status, pinned host memory the kernels write): a hashing
// kernel of an earlier call met a key whose offsets were inconsistent (offsets not
// non-decreasing, or a key of 2 GiB or more) and hashed it as the empty key instead of running
// off the key buffer or looping over a wrapped length (bfdev::key_ok).  The kernels run
// asynchronously, so the error is reported once, as BF_EINVAL, by the next call on the handle
// (bf_sync after the call at the latest), as the region-set status is checked lazily.
int take_key_status(bf_handle* h);
// Every op's entry check (after its StreamOrder): take_key_status, and a handle created with
// BF_FLAG_ENCODER (no bitset) refused unless the op needs no bitset (the region-set encodes).
int op_check(bf_handle* h, bool needs_bits = true);

struct StreamOrder {
    bf_handle* h;
    hipStream_t s;
    StreamOrder(bf_handle* h_, hipStream_t s_) : h(h_), s(s_) {
        if (h->order_valid && h->order_stream != s) (void)hipStreamWaitEvent(s, h->order_ev, 0);
    }
    ~StreamOrder() {
        if (h->order_ev && hipEventRecord(h->order_ev, s) == hipSuccess) {
            h->order_valid = true;
            h->order_stream = s;
        }
    }
    StreamOrder(const StreamOrder&) = delete;
    StreamOrder& operator=(const StreamOrder&) = delete;
};

int set_err(bf_handle* h, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (h) h->err = buf; else g_create_error = buf;
    return code;
}

int op_check(bf_handle* h, bool needs_bits) {
    if (needs_bits && !h->g.bits)
        return set_err(h, BF_EINVAL, "an encoder handle (BF_FLAG_ENCODER) holds no bitset: region-set encodes only");
    return take_key_status(h);
}

int take_key_status(bf_handle* h) {
    if (!h->h_key_status || __atomic_load_n(h->h_key_status, __ATOMIC_ACQUIRE) == 0u) return BF_OK;
    __atomic_store_n(h->h_key_status, 0u, __ATOMIC_RELEASE);
    return set_err(h, BF_EINVAL, "an earlier call's key offsets were inconsistent (offsets must be non-decreasing "
                                 "and every key below 2 GiB): those keys were hashed as empty strings");
}

#define HIPCHK(h, expr)                                                                      \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err((h), (e_ == hipErrorOutOfMemory ? BF_ENOMEM : BF_EDEVICE),        \
                           "%s failed: %s", #expr, hipGetErrorString(e_));                   \
    } while (0)

// Makes the handle's device current for the duration of a call.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = (prev == dev) || hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// Probe-policy defaults, measured on MI355X with tools/ab_policies.py (profiles/
// ab_policies_r01.jsonl): include? loads ceil(k/4) probes before its first
// early-exit check (1B@1%: 1.82 -> 1.39 ms per 2^24 keys), insert loads the k
// words and atomics only the unset bits (5.13 -> 3.30 ms).  The environment
// overrides exist for A/B runs and never change results.
// include? probe rounds.  A bitset beyond the caches: one word at a time, stopping at the first
// 0 bit (ruby.rb:23's early exit at every probe), so a non-member costs ~2 line fills instead of
// ceil(k/4) + a round of the rest — 1B@1 % (k = 6) 1.45 -> 1.32 ms, 100M@0.1 % (k = 10)
// 2.32 -> 2.01 ms per 2^24 keys (profiles/r01d_ab_rounds_*.json).  A cache-resident bitset is
// latency-, not fill-bound: ceil(k/4) probes, then the rest at once (1M@1 %: 0.045 vs 0.049 ms).
constexpr uint64_t kSequentialProbeBytes = 64ull << 20;
uint32_t default_first_round(uint32_t k, uint64_t bytes) { return bytes > kSequentialProbeBytes ? 1 : (k + 3) / 4; }
uint32_t default_next_round(uint64_t bytes) { return bytes > kSequentialProbeBytes ? 1 : 0; }
constexpr uint32_t kDefaultInsertTest = 1;
constexpr uint32_t kDefaultMemKind = 0;
constexpr uint32_t kDefaultBinnedMode = 2;     // auto
// include? stays on the direct kernel by default: at 1B@1% (2^24 keys) the binned
// include? measured 1.92 ms against 1.48 ms direct (hash 0.76 + partition 0.43 +
// region test 0.69); BFHIP_INCLUDE_BINNED=1/2 turns it on.
constexpr uint32_t kDefaultIncludeBinnedMode = 0;
constexpr uint32_t kDefaultBinRegionLog2 = 19; // 64 KiB LDS image per apply workgroup
constexpr double kBinnedCostRatio = 3.0;       // random line-fill bytes vs bitset bytes

uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* v = getenv(name);
    if (!v || !*v) return dflt;
    return (uint32_t)strtoul(v, nullptr, 10);
}

// A/B knobs (bf_internal.h): the environment only in -DBFHIP_AB_KNOBS builds
#ifdef BFHIP_AB_KNOBS
#define ab_u32(name, dflt) env_u32(name, dflt)
#else
#define ab_u32(name, dflt) (dflt)
#endif

int free_staging(bf_handle* h) {
    for (Slot& s : h->slot) {
        if (s.done) (void)hipEventSynchronize(s.done);
        if (s.h2d) (void)hipEventSynchronize(s.h2d);
        if (s.h_keys) (void)hipHostFree(s.h_keys);
        if (s.h_off) (void)hipHostFree(s.h_off);
        if (s.h_out) (void)hipHostFree(s.h_out);
        if (s.d_keys) (void)hipFree(s.d_keys);
        if (s.d_off32) (void)hipFree(s.d_off32);
        if (s.d_off) (void)hipFree(s.d_off);
        if (s.d_out) (void)hipFree(s.d_out);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.h2d) (void)hipEventDestroy(s.h2d);
        if (s.op) (void)hipEventDestroy(s.op);
        s = Slot{};
    }
    h->staging_ready = false;
    return BF_OK;
}

uint64_t pow2_at_least(uint64_t x, uint64_t lo) {
    uint64_t p = lo;
    while (p < x) p <<= 1;
    return p;
}

// Staging sized to the call (powers of two, grown on demand, never past the bf_config chunk
// limits except for one key longer than batch_bytes): a one-key Ruby `insert` pins kilobytes,
// not the full chunk size.
int ensure_staging(bf_handle* h, uint64_t keys, uint64_t bytes, uint64_t out_bytes) {
    const uint64_t want_keys = pow2_at_least(std::min(keys, h->cap_keys), 1024);
    const uint64_t want_bytes = pow2_at_least(bytes, 1ull << 16);
    const uint64_t want_out = pow2_at_least(out_bytes, 1024);
    const Slot& cur = h->slot[0];
    if (h->staging_ready && cur.cap_keys >= want_keys && cur.cap_bytes >= want_bytes && cur.out_cap >= want_out)
        return BF_OK;
    const uint64_t ck = std::max(want_keys, cur.cap_keys), cb = std::max(want_bytes, cur.cap_bytes),
                   co = std::max(want_out, cur.out_cap);
    free_staging(h);
    if (!h->copy_stream) HIPCHK(h, hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking));
    if (!h->d2h_stream) HIPCHK(h, hipStreamCreateWithFlags(&h->d2h_stream, hipStreamNonBlocking));
    for (Slot& s : h->slot) {
        HIPCHK(h, hipHostMalloc((void**)&s.h_keys, cb + 16, hipHostMallocDefault));
        HIPCHK(h, hipHostMalloc((void**)&s.h_off, (ck + 1) * sizeof(uint32_t), hipHostMallocDefault));
        HIPCHK(h, hipHostMalloc((void**)&s.h_out, co, hipHostMallocDefault));
        HIPCHK(h, hipMalloc((void**)&s.d_keys, cb + 16));
        HIPCHK(h, hipMalloc((void**)&s.d_off32, (ck + 1) * sizeof(uint32_t)));
        HIPCHK(h, hipMalloc((void**)&s.d_off, (ck + 1) * sizeof(uint64_t)));
        HIPCHK(h, hipMalloc((void**)&s.d_out, co));
        HIPCHK(h, hipEventCreateWithFlags(&s.h2d, hipEventDisableTiming));
        HIPCHK(h, hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        HIPCHK(h, hipEventCreateWithFlags(&s.op, hipEventDisableTiming));
        s.cap_keys = ck;
        s.cap_bytes = cb;
        s.out_cap = co;
    }
    h->staging_ready = true;
    return BF_OK;
}

// Waits for a slot's previous chunk and copies its results to the caller.
int retire_slot(bf_handle* h, Slot& s) {
    if (!s.busy) return BF_OK;
    HIPCHK(h, hipEventSynchronize(s.done));
    if (s.user_out && s.out_bytes) memcpy(s.user_out, s.h_out, s.out_bytes);
    s.busy = false;
    s.user_out = nullptr;
    s.out_bytes = 0;
    return BF_OK;
}

constexpr uint64_t kParallelKeys = 1ull << 15;   // smaller calls stay on the calling thread

// Splits [0, n) into `parts` near-equal ranges.
inline uint64_t part_lo(uint64_t n, unsigned parts, unsigned p) { return n * p / parts; }

int check_keys_args(bf_handle* h, const void* keys, const uint64_t* offsets, uint64_t n) {
    if (!h) return BF_EINVAL;
    if (n == 0) return BF_OK;
    if (!offsets) return set_err(h, BF_EINVAL, "offsets is NULL");
    if (!keys && offsets[n] != offsets[0]) return set_err(h, BF_EINVAL, "key_bytes is NULL");
    return BF_OK;
}

// Binned insert / include?: worth it when the batch's random line fills (~128 B
// per probe) clearly exceed one streaming pass over a bitset that lives beyond L2.
bool use_binned(const bf_handle* h, uint64_t n, bool include, BfBinPlan* plan) {
    const uint32_t mode = include ? h->include_binned_mode : h->binned_mode;
    if (mode == 0 || h->shards > 1 || h->engine != BF_ENGINE_RUBY) return false;
    if (!bf_binned_plan(h->dev_bytes, n, h->k, h->bin_region_log2, include, plan)) return false;
    if (mode == 1) return true;
    return h->dev_bytes >= (64ull << 20) &&
           (double)n * (double)h->k * 128.0 > kBinnedCostRatio * (double)h->dev_bytes;
}

// Device scratch shared by the binned and the sequential insert paths (grown on demand).
int ensure_scratch(bf_handle* h, uint64_t bytes) {
    if (bytes <= h->bin_scratch_cap) return BF_OK;
    (void)hipDeviceSynchronize();   // earlier launches may still use the old buffer
    if (h->d_bin_scratch) (void)hipFree(h->d_bin_scratch);
    h->d_bin_scratch = nullptr;
    h->bin_scratch_cap = 0;
    const uint64_t cap = round_up(bytes, 16ull << 20);
    HIPCHK(h, hipMalloc(&h->d_bin_scratch, cap));
    h->bin_scratch_cap = cap;
    return BF_OK;
}

// bf_profile: an event set per keyed launch, harvested by bf_profile_read.
BfMarks* prof_begin(bf_handle* h, hipStream_t s) {
    if (!h->profile) return nullptr;
    BfMarks mk{};
    if (!h->prof_free.empty()) {
        mk = h->prof_free.back();
        h->prof_free.pop_back();
    } else {
        for (hipEvent_t& e : mk.ev)
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
    }
    mk.used = 0;
    if (hipEventRecord(mk.ev[0], s) != hipSuccess) {
        h->prof_free.push_back(mk);
        return nullptr;
    }
    h->prof_pending.push_back(mk);
    return &h->prof_pending.back();
}

int prof_harvest(bf_handle* h) {
    for (BfMarks& mk : h->prof_pending) {
        if (mk.used > 0) HIPCHK(h, hipEventSynchronize(mk.ev[mk.used]));
        for (int i = 0; i < mk.used; ++i) {
            float ms = 0.f;
            HIPCHK(h, hipEventElapsedTime(&ms, mk.ev[i], mk.ev[i + 1]));
            auto it = std::find_if(h->prof_acc.begin(), h->prof_acc.end(),
                                   [&](const bf_handle::ProfAcc& a) { return a.name == mk.names[i]; });
            if (it == h->prof_acc.end()) h->prof_acc.push_back({mk.names[i], (double)ms, 1});
            else { it->ms += ms; it->launches += 1; }
        }
        h->prof_free.push_back(mk);
    }
    h->prof_pending.clear();
    return BF_OK;
}

const char* op_kernel_name(BfOp op) {
    switch (op) {
        case BF_OP_INDEXES: return "bf_keys_kernel<INDEXES>";
        case BF_OP_INCLUDE: return "bf_keys_kernel<INCLUDE>";
        case BF_OP_INSERT: return "bf_keys_kernel<INSERT>";
        case BF_OP_INSERT_FLAGS: return "bf_keys_kernel<INSERT_FLAGS>";
        default: return "bf_keys_kernel<ROUTE>";
    }
}

// Every keyed launch goes through here: inserts take the binned path when it pays.
int launch_op(bf_handle* h, BfOp op, const uint8_t* k16, const uint64_t* offs, uint64_t bias, uint64_t n,
              uint8_t* out8, uint64_t* out64, uint32_t* flag, hipStream_t s) {
    if (h->engine != BF_ENGINE_RUBY) {   // RubyTest engines: one fused direct kernel per op
        if (op == BF_OP_INSERT_FLAGS && out8)
            return set_err(h, BF_EINVAL, "per_key_new is not available with a RubyTest hash engine");
        if (op == BF_OP_INSERT_FLAGS) op = BF_OP_INSERT;
        BfMarks* mk = prof_begin(h, s);
        HIPCHK(h, bf_launch_engine(h->engine, op, h->g, k16, offs, bias, n, out8, out64, flag, s));
        bf_mark(mk, s, h->engine == BF_ENGINE_MD5 ? "engine_kernel<MD5>" : "engine_kernel<SHA1>");
        return BF_OK;
    }
    if (op == BF_OP_INSERT_FLAGS && out8) {
        // Per-key flags: exact sequential semantics (bf_seq.hip), chunk after chunk in stream order.
        const uint64_t chunk = bf_seq_chunk_keys(h->k);
        int rc = ensure_scratch(h, bf_seq_scratch_bytes(std::min(n, chunk), h->k, h->g.m));
        if (rc) return rc;
        for (uint64_t c0 = 0; c0 < n; c0 += chunk) {
            const uint64_t cn = std::min(chunk, n - c0);
            BfMarks* mk = prof_begin(h, s);
            HIPCHK(h, bf_launch_insert_seq(h->g, k16, offs + c0, bias, cn, h->d_bin_scratch, out8 + c0, flag, s, mk));
        }
        return BF_OK;
    }
    // Binned insert / include?, in sub-batches of at most bf_binned_max_keys keys.
    const bool is_insert = op == BF_OP_INSERT || op == BF_OP_INSERT_FLAGS;
    BfBinPlan plan;
    const uint64_t sub = std::max<uint64_t>(1, bf_binned_max_keys(h->k, h->dev_bytes, h->bin_region_log2));
    if ((is_insert || op == BF_OP_INCLUDE) && use_binned(h, std::min(n, sub), !is_insert, &plan)) {
        for (uint64_t c0 = 0; c0 < n; c0 += sub) {
            const uint64_t cn = std::min(sub, n - c0);
            if (cn != std::min(n, sub) && !bf_binned_plan(h->dev_bytes, cn, h->k, h->bin_region_log2, !is_insert, &plan))
                return set_err(h, BF_EINVAL, "binned plan failed for a tail of %llu keys", (unsigned long long)cn);
            int rc = ensure_scratch(h, plan.scratch_bytes);
            if (rc) return rc;
            BfMarks* mk = prof_begin(h, s);
            if (is_insert)
                HIPCHK(h, bf_launch_insert_binned(h->g, plan, h->dev_bytes, k16, offs + c0, bias, cn, h->d_bin_scratch,
                                                  op == BF_OP_INSERT_FLAGS ? flag : nullptr, s, mk));
            else
                HIPCHK(h, bf_launch_include_binned(h->g, plan, h->dev_bytes, k16, offs + c0, bias, cn,
                                                   h->d_bin_scratch, out8 + c0, s, mk));
        }
        return BF_OK;
    }
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_keys(op, h->g, k16, offs, bias, n, out8, out64, flag, s));
    bf_mark(mk, s, op_kernel_name(op));
    return BF_OK;
}

// Latency path for small host-pointer calls (a Ruby per-key insert / include?): flag word,
// result bytes, uint64 offsets and key bytes share ONE pinned staging block and ONE device
// block, so a call is one H2D copy (which also zeroes the flag), the op's kernel, one D2H
// copy of [flag | results] and one stream sync — no copy stream, no offset widening, no
// event hand-offs.  Layout: [0, 16) flag, [16, 16 + R) results, then n + 1 offsets, then the
// key bytes + 16 B of slack (the key stager's whole-vector reads).
constexpr uint64_t kSmallKeys = 2048;
constexpr uint64_t kSmallBytes = 64ull << 10;

bool small_call(BfOp op, uint64_t n, uint64_t total) {
    return (op == BF_OP_INSERT || op == BF_OP_INSERT_FLAGS || op == BF_OP_INCLUDE) && n <= kSmallKeys &&
           total <= kSmallBytes;
}

// flips (bf_insert_many_changes): the direct flagging kernel also lists every bit it flipped,
// after the results, at most kSmallFlips of them; the flip count rides at [8, 16).
constexpr uint64_t kSmallFlips = 4096;

int run_small(bf_handle* h, BfOp op, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* out8,
              uint8_t* any_new, uint64_t* flips = nullptr, uint64_t* flip_count = nullptr) {
    const uint64_t total = offsets[n] - offsets[0];
    const uint64_t res = round_up(n, 16);
    const uint64_t flip_at = 16 + res, nflip = flips ? (uint64_t)n * h->k : 0;
    const uint64_t off_at = flip_at + nflip * 8, key_at = off_at + round_up((n + 1) * 8, 16);
    const uint64_t end = key_at + round_up(total + 16, 16);
    if (h->small_cap < end) {
        const uint64_t cap = 16 + round_up(kSmallKeys, 16) + kSmallFlips * 8 + round_up((kSmallKeys + 1) * 8, 16) +
                             kSmallBytes + 16;
        if (!h->h_small) HIPCHK(h, hipHostMalloc((void**)&h->h_small, cap, hipHostMallocDefault));
        if (!h->d_small) HIPCHK(h, hipMalloc((void**)&h->d_small, cap));
        h->small_cap = cap;
    }
    uint8_t* hb = h->h_small;
    memset(hb, 0, 16);
    uint64_t* ho = reinterpret_cast<uint64_t*>(hb + off_at);
    const uint64_t base = offsets[0];
    for (uint64_t j = 0; j <= n; ++j) ho[j] = offsets[j] - base;
    memcpy(hb + key_at, keys + base, total);
    memset(hb + key_at + total, 0, 16);
    HIPCHK(h, hipMemcpyAsync(h->d_small, hb, end, hipMemcpyHostToDevice, h->stream));
    const bool want_flag = op == BF_OP_INSERT_FLAGS && any_new;
    uint8_t* d_out8 = (op == BF_OP_INCLUDE || (op == BF_OP_INSERT_FLAGS && out8)) ? h->d_small + 16 : nullptr;
    const uint8_t* d_keys = h->d_small + key_at;
    const uint64_t* d_off = reinterpret_cast<const uint64_t*>(h->d_small + off_at);
    uint32_t* d_flag = want_flag ? reinterpret_cast<uint32_t*>(h->d_small) : nullptr;
    if (flips) {   // the direct flagging kernel (never binned or sequential), dirty map untouched
        BfGeom g = h->g;
        g.dirty = nullptr;
        g.flips = reinterpret_cast<unsigned long long*>(h->d_small + flip_at);
        g.flip_count = reinterpret_cast<unsigned long long*>(h->d_small + 8);
        g.flip_cap = nflip;
        BfMarks* mk = prof_begin(h, h->stream);
        if (h->engine != BF_ENGINE_RUBY) {   // RubyTest engines: their one-lane-per-probe insert
            HIPCHK(h, bf_launch_engine(h->engine, BF_OP_INSERT, g, d_keys, d_off, 0, n, nullptr, nullptr, d_flag,
                                       h->stream));
            bf_mark(mk, h->stream, h->engine == BF_ENGINE_MD5 ? "engine_kernel<MD5>" : "engine_kernel<SHA1>");
        } else {
            HIPCHK(h, bf_launch_keys(BF_OP_INSERT_FLAGS, g, d_keys, d_off, 0, n, nullptr, nullptr, d_flag, h->stream));
            bf_mark(mk, h->stream, op_kernel_name(BF_OP_INSERT_FLAGS));
        }
    } else {
        int rc = launch_op(h, op, d_keys, d_off, 0, n, d_out8, nullptr, d_flag, h->stream);
        if (rc) return rc;
    }
    const uint64_t back = flips ? flip_at + nflip * 8 : d_out8 ? 16 + n : (want_flag ? 4 : 0);
    if (back) HIPCHK(h, hipMemcpyAsync(hb, h->d_small, back, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (d_out8 && out8) memcpy(out8, hb + 16, n);
    if (want_flag) *any_new = *reinterpret_cast<const uint32_t*>(hb) ? 1 : 0;
    if (flips) {
        const uint64_t c = std::min<uint64_t>(*reinterpret_cast<const uint64_t*>(hb + 8), nflip);
        memcpy(flips, hb + flip_at, c * 8);
        *flip_count = c;
    }
    return BF_OK;
}

// Host-pointer driver: chunk, stage, launch, copy results back, as a 3-slot pipeline over
// two streams.  For chunk c: the host (a thread pool) copies its key bytes and its offsets,
// as uint32 relative to the chunk's first key, into the slot's pinned buffers; the copy
// stream moves them to the device; the compute stream waits for that (event), widens the
// offsets and runs the op, then copies the per-key results back.  So the host staging of
// chunk c+2, the H2D of chunk c+1 and the kernels of chunk c overlap, and every key costs
// L + 4 bytes over PCIe.  The offsets are scanned once up front (non-decreasing, and the
// longest key, which sizes the staging), in parallel.
int run_host(bf_handle* h, BfOp op, const uint8_t* keys, const uint64_t* offsets, uint64_t n,
             uint8_t* out8, uint64_t* out64, uint8_t* any_new) {
    int rc = check_keys_args(h, keys, offsets, n);
    if (rc) return rc;
    if (op != BF_OP_INDEXES && h->shards > 1)
        return set_err(h, BF_EINVAL, "handle holds one shard of a partitioned filter: use bf_route_dev");
    if (any_new) *any_new = 0;
    if (n == 0) return BF_OK;

    const bool par = n >= kParallelKeys;
    if (par) h->pool.start(host_threads());
    const unsigned parts = par ? h->pool.size() * 4 : 1;
    std::vector<uint64_t> part_max(parts, 0), part_bad(parts, UINT64_MAX);
    h->pool.run(parts, [&](unsigned p) {
        const uint64_t lo = part_lo(n, parts, p), hi = part_lo(n, parts, p + 1);
        uint64_t mx = 0;
        for (uint64_t j = lo; j < hi; ++j) {
            const uint64_t a = offsets[j], b = offsets[j + 1];
            if (b < a) {
                part_bad[p] = j;
                return;
            }
            mx = std::max(mx, b - a);
        }
        part_max[p] = mx;
    });
    uint64_t maxkey = 0;
    for (unsigned p = 0; p < parts; ++p) {
        if (part_bad[p] != UINT64_MAX)
            return set_err(h, BF_EINVAL, "offsets must be non-decreasing (j=%llu)", (unsigned long long)part_bad[p]);
        maxkey = std::max(maxkey, part_max[p]);
    }
    if (maxkey >= (1ull << 31))
        return set_err(h, BF_EINVAL, "a key of %llu bytes: host-pointer calls take keys below 2 GiB",
                       (unsigned long long)maxkey);
    if (small_call(op, n, offsets[n] - offsets[0])) return run_small(h, op, keys, offsets, n, out8, any_new);

    const uint64_t out_per_key = op == BF_OP_INDEXES ? (uint64_t)h->k * 8 : 1;
    // Chunks of n/8 keys (at least 2^20, at most batch_keys): enough chunks that the
    // pipeline's fill and drain (one chunk's staging, one chunk's kernels) stay small.
    const uint64_t cap_keys = op == BF_OP_INDEXES ? std::max<uint64_t>(1, h->cap_keys / (h->k * 8)) : h->cap_keys;
    const uint64_t chunk_keys = std::min(n, std::min(cap_keys, std::max<uint64_t>(n / 8, 1ull << 20)));
    const uint64_t total = offsets[n] - offsets[0];
    // A slot holds one chunk's key bytes: the mean key length x chunk_keys + 12.5 %, not the
    // whole call's bytes.  Sizing by the call made a 4M-key call after a 1M-key one re-pin
    // 3 x 64 MiB of staging inside the call (20-37 ms of a 100M@0.1 % insert, VERDICT r03
    // item 5); a chunk whose keys run longer than the mean is cut shorter below.
    const uint64_t chunk_est = std::min<uint64_t>(
        total, (uint64_t)((double)total / (double)n * (double)chunk_keys * 1.125) + 4096);
    rc = ensure_staging(h, chunk_keys, std::max(std::min(chunk_est, h->cap_bytes), maxkey), chunk_keys * out_per_key);
    if (rc) return rc;

    const bool want_flag = (op == BF_OP_INSERT_FLAGS) && any_new;
    if (want_flag) HIPCHK(h, hipMemsetAsync(h->d_flag, 0, sizeof(uint32_t), h->stream));

    uint64_t i = 0;
    int c = 0;
    while (i < n) {
        Slot& s = h->slot[c % kSlots];
        rc = retire_slot(h, s);
        if (rc) return rc;
        // chunk [i, j): at most chunk_keys keys and s.cap_bytes bytes
        const uint64_t jmax = std::min(n, i + std::min(chunk_keys, s.cap_keys));
        const uint64_t base = offsets[i];
        uint64_t j;
        if (offsets[jmax] - base <= s.cap_bytes) {
            j = jmax;
        } else {   // binary search the last j with offsets[j] - base <= cap (maxkey <= cap: j > i)
            uint64_t lo = i + 1, hi = jmax;
            while (lo < hi) {
                const uint64_t mid = (lo + hi + 1) / 2;
                if (offsets[mid] - base <= s.cap_bytes) lo = mid; else hi = mid - 1;
            }
            j = lo;
        }
        const uint64_t cn = j - i;
        const uint64_t nbytes = offsets[j] - base;
        const unsigned cparts = (par && cn >= kParallelKeys) ? h->pool.size() * 2 : 1;
        h->pool.run(cparts, [&](unsigned p) {
            const uint64_t blo = part_lo(nbytes, cparts, p), bhi = part_lo(nbytes, cparts, p + 1);
            if (bhi > blo) memcpy(s.h_keys + blo, keys + base + blo, bhi - blo);
            const uint64_t tlo = part_lo(cn + 1, cparts, p), thi = part_lo(cn + 1, cparts, p + 1);
            for (uint64_t t = tlo; t < thi; ++t) s.h_off[t] = (uint32_t)(offsets[i + t] - base);
        });
        memset(s.h_keys + nbytes, 0, 16);
        HIPCHK(h, hipMemcpyAsync(s.d_keys, s.h_keys, round_up(nbytes + 1, 16), hipMemcpyHostToDevice, h->copy_stream));
        HIPCHK(h, hipMemcpyAsync(s.d_off32, s.h_off, (cn + 1) * sizeof(uint32_t), hipMemcpyHostToDevice,
                                 h->copy_stream));
        HIPCHK(h, hipEventRecord(s.h2d, h->copy_stream));
        HIPCHK(h, hipStreamWaitEvent(h->stream, s.h2d, 0));
        HIPCHK(h, bf_launch_widen_offsets(s.d_off32, s.d_off, cn + 1, h->stream));
        uint8_t* d_out8 = (op == BF_OP_INCLUDE || (op == BF_OP_INSERT_FLAGS && out8)) ? s.d_out : nullptr;
        uint64_t* d_out64 = (op == BF_OP_INDEXES) ? reinterpret_cast<uint64_t*>(s.d_out) : nullptr;
        rc = launch_op(h, op, s.d_keys, s.d_off, 0, cn, d_out8, d_out64, want_flag ? h->d_flag : nullptr, h->stream);
        if (rc) return rc;
        s.out_bytes = 0;
        s.user_out = nullptr;
        if (d_out8 && out8) {
            s.out_bytes = cn;
            s.user_out = out8 + i;
        } else if (d_out64 && out64) {
            s.out_bytes = cn * h->k * sizeof(uint64_t);
            s.user_out = reinterpret_cast<uint8_t*>(out64 + i * h->k);
        }
        if (s.out_bytes) {
            // the result copy runs on its own stream, so chunk c + 1's kernels do not queue
            // behind chunk c's D2H (include?: 1 B per key back while the next keys go in)
            HIPCHK(h, hipEventRecord(s.op, h->stream));
            HIPCHK(h, hipStreamWaitEvent(h->d2h_stream, s.op, 0));
            HIPCHK(h, hipMemcpyAsync(s.h_out, s.d_out, s.out_bytes, hipMemcpyDeviceToHost, h->d2h_stream));
            HIPCHK(h, hipEventRecord(s.done, h->d2h_stream));
        } else {
            HIPCHK(h, hipEventRecord(s.done, h->stream));
        }
        s.busy = true;
        i = j;
        ++c;
    }
    for (Slot& s : h->slot) {
        rc = retire_slot(h, s);
        if (rc) return rc;
    }
    if (want_flag) {
        HIPCHK(h, hipMemcpyAsync(h->h_flag, h->d_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        *any_new = *h->h_flag ? 1 : 0;
    }
    return BF_OK;
}

hipStream_t pick_stream(bf_handle*, void* stream) {
    return reinterpret_cast<hipStream_t>(stream);   // verbatim: NULL is the null stream
}

// Device pointer + 16-byte alignment bias for the kernels.
const uint8_t* align_keys(const uint8_t* p, uint64_t* bias) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    *bias = a & 15u;
    return reinterpret_cast<const uint8_t*>(a & ~(uintptr_t)15);
}

int run_dev(bf_handle* h, BfOp op, const uint8_t* d_keys, const uint64_t* d_offsets, uint64_t n,
            uint8_t* d_out8, uint64_t* d_out64, uint32_t* d_flag, void* stream) {
    if (!h) return BF_EINVAL;
    if (n == 0) return BF_OK;
    if (!d_offsets || !d_keys) return set_err(h, BF_EINVAL, "NULL device pointer");
    if (op == BF_OP_INCLUDE && !d_out8) return set_err(h, BF_EINVAL, "d_out is NULL");
    if (op == BF_OP_INDEXES && !d_out64) return set_err(h, BF_EINVAL, "d_out is NULL");
    if (op != BF_OP_INDEXES && h->shards > 1)
        return set_err(h, BF_EINVAL, "handle holds one shard of a partitioned filter: use bf_route_dev");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    uint64_t bias = 0;
    const uint8_t* k16 = align_keys(d_keys, &bias);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    return launch_op(h, op, k16, d_offsets, bias, n, d_out8, d_out64, d_flag, so.s);
}

}  // namespace

// ===================================================================== ABI ==
extern "C" {

const char* bf_version(void) { return BFHIP_VERSION_STR; }

const char* bf_last_error(const bf_handle* h) {
    if (h && h->multi) return bfm_last_error(h->multi);
    return h ? h->err.c_str() : g_create_error.c_str();
}

int bf_indexes(const uint8_t* key, uint64_t len, uint64_t m_bits, uint32_t k, uint64_t* out) {
    if (m_bits == 0 || k == 0) return set_err(nullptr, BF_EINVAL, "m and k must be positive (ruby.rb:51 divides by m)");
    if (k > BF_MAX_K) return set_err(nullptr, BF_EINVAL, "k must be in [1, %u], got %u", BF_MAX_K, k);
    if (!out || (len && !key)) return set_err(nullptr, BF_EINVAL, "NULL pointer");
    BfGeom g{};
    g.m = m_bits;
    g.inv_m = 1.0 / (double)m_bits;
    g.k = k;
    g.nomod = (m_bits > (uint64_t)k * 0xFFFFFFFFull) ? 1u : 0u;
    g.mod_f32 = (m_bits >= (1ull << 17)) ? 1u : 0u;
    g.inv_m_f = (float)(1.0 / (double)m_bits);
    g.mod_sub = bf_mod_sub(m_bits, (uint64_t)k * 0xFFFFFFFFull);
    g.shards = 1;
    g.inv_shards = 1.0;
    const uint64_t kb = round_up(len + 16, 16);
    uint8_t* d = nullptr;   // key bytes (16-B slack), offsets[2], k offsets
    if (hipMalloc(&d, kb + 16 + 8ull * k) != hipSuccess) return set_err(nullptr, BF_ENOMEM, "hipMalloc failed");
    std::vector<uint8_t> host(kb + 16, 0);
    if (len) memcpy(host.data(), key, len);
    const uint64_t offs[2] = {0, len};
    memcpy(host.data() + kb, offs, 16);
    uint64_t* d_out = reinterpret_cast<uint64_t*>(d + kb + 16);
    hipError_t e = hipMemcpy(d, host.data(), kb + 16, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = bf_launch_keys(BF_OP_INDEXES, g, d, reinterpret_cast<const uint64_t*>(d + kb), 0, 1, nullptr, d_out, nullptr,
                           nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d_out, 8ull * k, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return set_err(nullptr, BF_EDEVICE, "bf_indexes: %s", hipGetErrorString(e));
    return BF_OK;
}

int bf_check_offsets(const uint64_t* offsets, uint64_t n, uint64_t* bad_key) {
    // the rule every hashing kernel applies per key (bfdev::key_ok over the whole batch: the
    // first and last offsets bound every key, each key's end is not before its start, and every
    // key is below 2 GiB, the host path's cap)
    if (bad_key) *bad_key = 0;
    if (!offsets) return set_err(nullptr, BF_EINVAL, "offsets is NULL");
    const uint64_t lo = offsets[0], hi = offsets[n];
    for (uint64_t j = 0; j < n; ++j) {
        if (!bfdev::key_ok(lo, offsets[j], offsets[j + 1], hi, nullptr)) {
            if (bad_key) *bad_key = j;
            return set_err(nullptr, BF_EINVAL, "key %llu: offsets must be non-decreasing and every key below 2 GiB",
                           (unsigned long long)j);
        }
    }
    return BF_OK;
}

int64_t bf_optimal_m(double n, double p) {
    // lib/redis/bloomfilter.rb:50-52 — left-to-right IEEE double, Float#round (half away from zero).
    // A non-finite or out-of-range result (error_rate 0 gives Infinity, where the reference
    // raises FloatDomainError) returns BF_OPTIMAL_M_INVALID instead of an undefined cast.
    const double v = std::round((-1.0 * n) * std::log(p) / std::pow(std::log(2.0), 2.0));
    if (!std::isfinite(v) || v >= 9223372036854775808.0 || v < -9223372036854775808.0) return BF_OPTIMAL_M_INVALID;
    return (int64_t)v;
}

int64_t bf_optimal_k(int64_t n, int64_t m) {
    // lib/redis/bloomfilter.rb:54-58 — Integer floor division, bumped to 1 when 0.
    if (n == 0) return 0;
    int64_t q = m / n;
    if ((m % n != 0) && ((m < 0) != (n < 0))) --q;
    int64_t h = (int64_t)std::round(std::log(2.0) * (double)q);
    if (h == 0) h += 1;
    return h;
}

int bf_create(uint64_t m_bits, uint32_t k, const bf_config* cfg, bf_handle** out) {
    g_create_error.clear();
    if (!out) return set_err(nullptr, BF_EINVAL, "out is NULL");
    *out = nullptr;
    if (m_bits == 0) return set_err(nullptr, BF_EINVAL, "m_bits == 0 (the ruby driver would raise ZeroDivisionError, ruby.rb:51)");
    if (k == 0 || k > BF_MAX_K) return set_err(nullptr, BF_EINVAL, "k must be in [1, %u], got %u", BF_MAX_K, k);
    bf_config c{};
    if (cfg && cfg->struct_size) {
        memcpy(&c, cfg, std::min<size_t>(sizeof c, cfg->struct_size));
    } else {
        c.device = -1;
    }
    if (c.device_count > 0) {   // one handle over several devices (bf_multi.cpp)
        BfMulti* mh = nullptr;
        std::string err;
        const int rc = bfm_create(m_bits, k, c, &mh, &err);
        if (rc) return set_err(nullptr, rc, "%s", err.c_str());
        bf_handle* h = new (std::nothrow) bf_handle();
        if (!h) {
            bfm_destroy(mh);
            return set_err(nullptr, BF_ENOMEM, "host allocation failed");
        }
        h->multi = mh;
        h->m = m_bits;
        h->k = k;
        *out = h;
        return BF_OK;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_err(nullptr, BF_EDEVICE, "no HIP device available");
    int dev = c.device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (dev >= ndev) return set_err(nullptr, BF_EINVAL, "device %d out of range (%d devices)", dev, ndev);

    bf_handle* h = new (std::nothrow) bf_handle();
    if (!h) return set_err(nullptr, BF_ENOMEM, "host allocation failed");
    h->device = dev;
    h->m = m_bits;
    h->k = k;
    const uint64_t maxval = (uint64_t)k * 0xFFFFFFFFull;      // largest offset ruby.rb:51 can produce
    const uint32_t eng = c.flags & (BF_FLAG_ENGINE_MD5 | BF_FLAG_ENGINE_SHA1);
    if ((c.flags & BF_FLAG_ENCODER) && (eng || c.shard_count > 1)) {
        delete h;
        return set_err(nullptr, BF_EINVAL, "BF_FLAG_ENCODER: a whole-filter ruby-derivation handle only");
    }
    if (eng == (BF_FLAG_ENGINE_MD5 | BF_FLAG_ENGINE_SHA1) || (eng && c.shard_count > 1)) {
        delete h;
        return set_err(nullptr, BF_EINVAL, "one hash engine per filter, whole-filter handles only");
    }
    h->engine = eng == BF_FLAG_ENGINE_MD5 ? BF_ENGINE_MD5 : (eng ? BF_ENGINE_SHA1 : BF_ENGINE_RUBY);
    h->reach = h->engine != BF_ENGINE_RUBY ? m_bits : std::min<uint64_t>(m_bits, maxval + 1);
    h->shards = c.shard_count > 1 ? c.shard_count : 1;
    h->shard_index = h->shards > 1 ? c.shard_index : 0;
    h->block_log2 = c.shard_block_log2 ? c.shard_block_log2 : 20;
    if (h->shards > 255 || h->shard_index >= h->shards || h->block_log2 < 3 || h->block_log2 > 40) {
        delete h;
        return set_err(nullptr, BF_EINVAL, "bad shard config (count %u, index %u, block_log2 %u)",
                       c.shard_count, c.shard_index, c.shard_block_log2);
    }
    if (h->shards == 1) {
        h->local_bits = h->reach;
    } else {   // blocks g = s, s + P, s + 2P, ... below ceil(reach / 2^b)
        const uint64_t nblocks = (h->reach + (1ull << h->block_log2) - 1) >> h->block_log2;
        const uint64_t mine = nblocks > h->shard_index ? (nblocks - 1 - h->shard_index) / h->shards + 1 : 0;
        h->local_bits = mine << h->block_log2;
    }
    h->dev_bytes = round_up(std::max<uint64_t>((h->local_bits + 7) / 8, 1), 256);
    h->route32 = (c.flags & BF_FLAG_ROUTE32) != 0;
    if (h->route32) {   // the largest shard (index 0) must address its bits in 32 bits
        const uint64_t nblocks = (h->reach + (1ull << h->block_log2) - 1) >> h->block_log2;
        const uint64_t biggest = h->shards == 1 ? h->reach : (((nblocks - 1) / h->shards + 1) << h->block_log2);
        if (biggest > (1ull << 32)) {
            delete h;
            return set_err(nullptr, BF_EINVAL, "BF_FLAG_ROUTE32 needs shards of <= 2^32 bits (largest: %llu)",
                           (unsigned long long)biggest);
        }
    }
    h->cap_keys = c.batch_keys ? c.batch_keys : (1ull << 22);
    h->cap_bytes = c.batch_bytes ? c.batch_bytes : (64ull << 20);
    if (h->cap_bytes > (1ull << 31) || h->cap_keys > (1ull << 31)) {   // uint32 relative offsets per chunk
        delete h;
        return set_err(nullptr, BF_EINVAL, "batch_keys and batch_bytes must be <= 2^31");
    }

    DeviceGuard dg(dev);
    auto fail = [&](int code, const char* what, hipError_t e) {
        set_err(nullptr, code, "%s: %s", what, hipGetErrorString(e));
        if (h->g.bits) (void)hipFree(h->g.bits);
        if (h->d_flag) (void)hipFree(h->d_flag);
        if (h->d_scan) (void)hipFree(h->d_scan);
        if (h->h_flag) (void)hipHostFree(h->h_flag);
        if (h->h_key_status) (void)hipHostFree(h->h_key_status);
        if (h->order_ev) (void)hipEventDestroy(h->order_ev);
        if (h->stream) (void)hipStreamDestroy(h->stream);
        delete h;
        return code;
    };
    if (!dg.ok) return fail(BF_EDEVICE, "hipSetDevice", hipErrorInvalidDevice);
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) != hipSuccess) return fail(BF_EDEVICE, "hipStreamCreate", e);
    if ((e = hipEventCreateWithFlags(&h->order_ev, hipEventDisableTiming)) != hipSuccess) return fail(BF_EDEVICE, "hipEventCreate", e);
    // Bitset memory kind (A/B knob): 0 coarse-grained hipMalloc, 1 uncached (MTYPE UC),
    // 2 fine-grained.
    h->mem_kind = ab_u32("BFHIP_BITS_MEM", kDefaultMemKind);
    // BF_FLAG_ENCODER: the filter's geometry without its bitset (a second handle that encodes a
    // replicated filter's next batch beside its apply: bf_encode_region_sets*_dev only)
    const bool encoder = (c.flags & BF_FLAG_ENCODER) != 0;
    if (encoder) e = hipSuccess;
    else if (h->mem_kind == 1) e = hipExtMallocWithFlags((void**)&h->g.bits, h->dev_bytes, hipDeviceMallocUncached);
    else if (h->mem_kind == 2) e = hipExtMallocWithFlags((void**)&h->g.bits, h->dev_bytes, hipDeviceMallocFinegrained);
    else e = hipMalloc((void**)&h->g.bits, h->dev_bytes);
    if (e != hipSuccess) return fail(BF_ENOMEM, "hipMalloc(bitset)", e);
    if ((e = hipMalloc((void**)&h->d_flag, 256)) != hipSuccess) return fail(BF_ENOMEM, "hipMalloc(flag)", e);
    if ((e = hipMalloc((void**)&h->d_scan, 256)) != hipSuccess) return fail(BF_ENOMEM, "hipMalloc(scan)", e);
    if ((e = hipHostMalloc((void**)&h->h_flag, 64, hipHostMallocDefault)) != hipSuccess) return fail(BF_ENOMEM, "hipHostMalloc", e);
    if ((e = hipHostMalloc((void**)&h->h_key_status, 64, hipHostMallocDefault)) != hipSuccess)
        return fail(BF_ENOMEM, "hipHostMalloc(key status)", e);
    *h->h_key_status = 0u;
    if ((e = hipHostGetDevicePointer((void**)&h->g.key_status, h->h_key_status, 0)) != hipSuccess)
        return fail(BF_EDEVICE, "hipHostGetDevicePointer(key status)", e);
    if (!encoder && (e = hipMemsetAsync(h->g.bits, 0, h->dev_bytes, h->stream)) != hipSuccess)
        return fail(BF_EDEVICE, "hipMemset", e);
    if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return fail(BF_EDEVICE, "hipStreamSynchronize", e);
    h->g.m = m_bits;
    h->g.inv_m = 1.0 / (double)m_bits;
    h->g.k = k;
    h->g.nomod = (m_bits > maxval) ? 1u : 0u;
    h->g.mod_f32 = (m_bits >= (1ull << 17)) ? 1u : 0u;
    h->g.inv_m_f = (float)(1.0 / (double)m_bits);
    // BFHIP_MOD_SUB=0: the float-estimate modulo everywhere (A/B)
    h->g.mod_sub = ab_u32("BFHIP_MOD_SUB", 1) ? bf_mod_sub(m_bits, (uint64_t)k * 0xFFFFFFFFull) : 0u;
    h->g.shards = h->shards;
    h->g.block_log2 = h->block_log2;
    h->g.inv_shards = 1.0 / (double)h->shards;
    h->g.shards_pow2 = (h->shards & (h->shards - 1u)) == 0 ? 1u : 0u;
    h->g.shard_log2 = (uint32_t)__builtin_ctz(h->shards);
    h->g.route32 = h->route32 ? 1u : 0u;
    h->g.limit = h->local_bits;
    h->g.first_round = ab_u32("BFHIP_INCLUDE_FIRST_ROUND", default_first_round(k, h->dev_bytes));
    h->g.next_round = ab_u32("BFHIP_INCLUDE_NEXT_ROUND", default_next_round(h->dev_bytes));
    h->g.route_agg = env_u32("BFHIP_ROUTE_AGG", 1);   // P = 1 only: at P = 8 the per-owner loop costs more than the LDS atomics (sim_rank A/B)
    h->g.insert_test = ab_u32("BFHIP_INSERT_TEST", kDefaultInsertTest);
    h->binned_mode = env_u32("BFHIP_INSERT_BINNED", kDefaultBinnedMode);
    h->bin_region_log2 = env_u32("BFHIP_BIN_REGION_LOG2", kDefaultBinRegionLog2);
    h->chunk_buckets = ab_u32("BFHIP_CHUNK_BUCKETS", 0);
    h->chunk_test_l2 = env_u32("BFHIP_CHUNK_TEST_L2", 2);
    h->include_binned_mode = env_u32("BFHIP_INCLUDE_BINNED", kDefaultIncludeBinnedMode);
    h->shard_test_binned_mode = env_u32("BFHIP_SHARD_TEST_BINNED", 2);
    *out = h;
    return BF_OK;
}

int bf_destroy(bf_handle* h) {
    if (!h) return BF_OK;
    if (h->multi) {
        bfm_destroy(h->multi);
        delete h;
        return BF_OK;
    }
    {
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceGuard dg(h->device);
        if (h->order_valid) (void)hipEventSynchronize(h->order_ev);
        if (h->stream) (void)hipStreamSynchronize(h->stream);
        free_staging(h);
        if (h->h_small) (void)hipHostFree(h->h_small);
        if (h->d_small) (void)hipFree(h->d_small);
        if (h->g.bits) (void)hipFree(h->g.bits);
        if (h->d_flag) (void)hipFree(h->d_flag);
        if (h->d_scan) (void)hipFree(h->d_scan);
        if (h->h_flag) (void)hipHostFree(h->h_flag);
        if (h->h_key_status) (void)hipHostFree(h->h_key_status);
        if (h->d_tmp_local) (void)hipFree(h->d_tmp_local);
        if (h->d_tmp_owner) (void)hipFree(h->d_tmp_owner);
        if (h->d_cursor) (void)hipFree(h->d_cursor);
        if (h->d_bin_scratch) (void)hipFree(h->d_bin_scratch);
        if (h->d_ans8) (void)hipFree(h->d_ans8);
        if (h->d_seg) (void)hipFree(h->d_seg);
        if (h->d_dirty) (void)hipFree(h->d_dirty);
        (void)prof_harvest(h);   // waits for marks recorded on caller streams
        for (BfMarks& mk : h->prof_free)
            for (hipEvent_t e : mk.ev) (void)hipEventDestroy(e);
        if (h->order_ev) (void)hipEventDestroy(h->order_ev);
        if (h->copy_stream) (void)hipStreamDestroy(h->copy_stream);
        if (h->d2h_stream) (void)hipStreamDestroy(h->d2h_stream);
        if (h->stream) (void)hipStreamDestroy(h->stream);
    }
    delete h;
    return BF_OK;
}

int bf_info(const bf_handle* h, uint64_t* m_bits, uint32_t* k, uint64_t* reach_bits, uint64_t* device_bytes) {
    if (h && h->multi) return bfm_info(h->multi, m_bits, k, reach_bits, device_bytes);
    if (!h) return BF_EINVAL;
    if (m_bits) *m_bits = h->m;
    if (k) *k = h->k;
    if (reach_bits) *reach_bits = h->reach;
    if (device_bytes) *device_bytes = h->dev_bytes;
    return BF_OK;
}

int bf_insert_many(bf_handle* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n,
                   uint8_t* any_new, uint8_t* per_key_new) {
    if (h && h->multi) return bfm_insert_many(h->multi, key_bytes, offsets, n, any_new, per_key_new);
    if (!h) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    const BfOp op = (any_new || per_key_new) ? BF_OP_INSERT_FLAGS : BF_OP_INSERT;
    StreamOrder so(h, h->stream);
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    int rc = run_host(h, op, key_bytes, offsets, n, per_key_new, nullptr, any_new);
    if (rc) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return BF_OK;
}

int bf_insert_many_changes(bf_handle* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n,
                           uint64_t* out_bits, uint64_t cap, uint64_t* count) {
    if (!h) return BF_EINVAL;
    if (!count) return set_err(h, BF_EINVAL, "count is NULL");
    *count = 0;
    if (h->multi) return set_err(h, BF_EINVAL, "bf_insert_many_changes: a multi-device handle (use bf_dirty_ranges)");
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = check_keys_args(h, key_bytes, offsets, n);
    if (rc) return rc;
    if (n == 0) return BF_OK;
    if (h->shards > 1) return set_err(h, BF_EINVAL, "bf_insert_many_changes: a partitioned shard");
    if (n * h->k > kSmallFlips || offsets[n] < offsets[0] || offsets[n] - offsets[0] > kSmallBytes)
        return set_err(h, BF_EINVAL, "bf_insert_many_changes takes at most %llu probes and %llu key bytes",
                       (unsigned long long)kSmallFlips, (unsigned long long)kSmallBytes);
    if (!out_bits || cap < n * h->k) return set_err(h, BF_EINVAL, "out_bits must hold n * k offsets");
    for (uint64_t j = 0; j < n; ++j)
        if (offsets[j + 1] < offsets[j]) return set_err(h, BF_EINVAL, "offsets must be non-decreasing");
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, h->stream);
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    return run_small(h, BF_OP_INSERT_FLAGS, key_bytes, offsets, n, nullptr, nullptr, out_bits, count);
}

int bf_include_many(bf_handle* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n, uint8_t* out) {
    if (h && h->multi) return bfm_include_many(h->multi, key_bytes, offsets, n, out);
    if (!h) return BF_EINVAL;
    if (n && !out) return set_err(h, BF_EINVAL, "out is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, h->stream);
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    return run_host(h, BF_OP_INCLUDE, key_bytes, offsets, n, out, nullptr, nullptr);
}

int bf_indexes_many(bf_handle* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n, uint64_t* out) {
    if (h && h->multi) return bfm_indexes_many(h->multi, key_bytes, offsets, n, out);
    if (!h) return BF_EINVAL;
    if (n && !out) return set_err(h, BF_EINVAL, "out is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, h->stream);
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    return run_host(h, BF_OP_INDEXES, key_bytes, offsets, n, nullptr, out, nullptr);
}

int bf_clear(bf_handle* h) {
    if (h && h->multi) return bfm_clear(h->multi);
    if (!h) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, h->stream);
    if (!h->g.bits) return set_err(h, BF_EINVAL, "an encoder handle (BF_FLAG_ENCODER) holds no bitset");
    HIPCHK(h, hipMemsetAsync(h->g.bits, 0, h->dev_bytes, h->stream));
    if (h->d_dirty) HIPCHK(h, hipMemsetAsync(h->d_dirty, 0, h->dirty_blocks, h->stream));   // the driver DELs the key
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return BF_OK;
}

int bf_sync(bf_handle* h) {
    if (h && h->multi) return bfm_sync(h->multi);
    if (!h) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->order_valid) HIPCHK(h, hipEventSynchronize(h->order_ev));   // the last call, on whatever stream
    return take_key_status(h);
}

}  // extern "C"

namespace {

// Trimmed length of the first `max_bytes` bytes of the device bitset (Redis STRLEN after SETBITs).
int device_trimmed_len(bf_handle* h, uint64_t* len_out) {
    StreamOrder so(h, h->stream);
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    HIPCHK(h, hipMemsetAsync(h->d_scan, 0, sizeof(unsigned long long), h->stream));
    HIPCHK(h, bf_launch_last_nonzero(h->g.bits, h->dev_bytes / 4, h->d_scan, h->stream));
    unsigned long long last = 0;
    HIPCHK(h, hipMemcpyAsync(h->h_flag, h->d_scan, sizeof last, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    memcpy(&last, h->h_flag, sizeof last);
    uint64_t len = 0;
    if (last) {
        const uint64_t w = last - 1;   // index of the last nonzero 32-bit word
        uint32_t word = 0;
        HIPCHK(h, hipMemcpy(&word, h->g.bits + w, 4, hipMemcpyDeviceToHost));
        int top = 3;
        while (top > 0 && ((word >> (8 * top)) & 0xFFu) == 0) --top;
        len = w * 4 + (uint64_t)top + 1;
    }
    *len_out = len;
    return BF_OK;
}

// Load `len` bytes (device layout) into the bitset; bits at offsets >= max_bits are refused.
int import_bytes(bf_handle* h, const uint8_t* buf, uint64_t len, uint32_t mode, uint64_t max_bits) {
    if (mode != BF_IMPORT_REPLACE && mode != BF_IMPORT_OR) return set_err(h, BF_EINVAL, "bad import mode %u", mode);
    if (len && !buf) return set_err(h, BF_EINVAL, "buf is NULL");
    const uint64_t max_bytes = (max_bits + 7) / 8;
    if (len > max_bytes)
        return set_err(h, BF_ERANGE, "string of %llu bytes exceeds the filter's %llu reachable bytes",
                       (unsigned long long)len, (unsigned long long)max_bytes);
    if (len == max_bytes && (max_bits & 7)) {
        const uint8_t beyond = (uint8_t)(0xFFu >> (max_bits & 7));
        if (buf[len - 1] & beyond)
            return set_err(h, BF_ERANGE, "string sets bits at offsets >= %llu", (unsigned long long)max_bits);
    }
    StreamOrder so(h, h->stream);
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    if (h->d_dirty) HIPCHK(h, hipMemsetAsync(h->d_dirty, 1, h->dirty_blocks, h->stream));
    if (mode == BF_IMPORT_REPLACE) {
        HIPCHK(h, hipMemsetAsync(h->g.bits, 0, h->dev_bytes, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        if (len) HIPCHK(h, hipMemcpy(h->g.bits, buf, len, hipMemcpyHostToDevice));
        return BF_OK;
    }
    if (!len) return BF_OK;
    const uint64_t tb = round_up(len, 256);
    uint32_t* tmp = nullptr;
    HIPCHK(h, hipMalloc((void**)&tmp, tb));
    hipError_t e = hipMemsetAsync(tmp, 0, tb, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) e = hipMemcpy(tmp, buf, len, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = bf_launch_or(h->g.bits, tmp, tb / 4, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    (void)hipFree(tmp);
    if (e != hipSuccess) return set_err(h, BF_EDEVICE, "import OR failed: %s", hipGetErrorString(e));
    return BF_OK;
}

int ensure_route_scratch(bf_handle* h, uint64_t probes) {
    if (!h->d_cursor) HIPCHK(h, hipMalloc((void**)&h->d_cursor, 256 * sizeof(unsigned long long)));
    if (probes <= h->tmp_cap) return BF_OK;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->d_tmp_local) (void)hipFree(h->d_tmp_local);
    if (h->d_tmp_owner) (void)hipFree(h->d_tmp_owner);
    h->d_tmp_local = nullptr;
    h->d_tmp_owner = nullptr;
    h->tmp_cap = 0;
    const uint64_t cap = round_up(probes, 1ull << 16);
    HIPCHK(h, hipMalloc((void**)&h->d_tmp_local, cap * sizeof(uint64_t)));
    HIPCHK(h, hipMalloc((void**)&h->d_tmp_owner, cap));
    h->tmp_cap = cap;
    return BF_OK;
}

}  // namespace

extern "C" {

int bf_export_redis(bf_handle* h, uint8_t* buf, uint64_t cap, uint64_t* len_out) {
    if (h && h->multi) return len_out ? bfm_export_redis(h->multi, buf, cap, len_out) : BF_EINVAL;
    if (!h || !len_out) return BF_EINVAL;
    if (h->shards > 1) return set_err(h, BF_EINVAL, "partitioned shard: use bf_shard_export and interleave blocks");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    uint64_t len = 0;
    int rc = device_trimmed_len(h, &len);
    if (rc) return rc;
    *len_out = len;
    if (!buf) return BF_OK;
    if (cap < len) return set_err(h, BF_ERANGE, "export buffer too small: need %llu bytes", (unsigned long long)len);
    if (len) HIPCHK(h, hipMemcpy(buf, h->g.bits, len, hipMemcpyDeviceToHost));
    return BF_OK;
}

int bf_import_redis(bf_handle* h, const uint8_t* buf, uint64_t len, uint32_t mode) {
    if (h && h->multi) return bfm_import_redis(h->multi, buf, len, mode);
    if (!h) return BF_EINVAL;
    if (h->shards > 1) return set_err(h, BF_EINVAL, "partitioned shard: use bf_shard_import");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    return import_bytes(h, buf, len, mode, h->reach);
}

int bf_shard_info(const bf_handle* h, uint32_t* shard_count, uint32_t* shard_index, uint32_t* block_log2,
                  uint64_t* local_bits) {
    if (h && h->multi) return bfm_shard_info(h->multi, shard_count, shard_index, block_log2, local_bits);
    if (!h) return BF_EINVAL;
    if (shard_count) *shard_count = h->shards;
    if (shard_index) *shard_index = h->shard_index;
    if (block_log2) *block_log2 = h->block_log2;
    if (local_bits) *local_bits = h->local_bits;
    return BF_OK;
}

int bf_shard_export(bf_handle* h, uint8_t* buf, uint64_t cap, uint64_t* len_out) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h || !len_out) return BF_EINVAL;
    const uint64_t len = (h->local_bits + 7) / 8;
    *len_out = len;
    if (!buf) return BF_OK;
    if (cap < len) return set_err(h, BF_ERANGE, "export buffer too small: need %llu bytes", (unsigned long long)len);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    if (h->order_valid) HIPCHK(h, hipEventSynchronize(h->order_ev));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (len) HIPCHK(h, hipMemcpy(buf, h->g.bits, len, hipMemcpyDeviceToHost));
    return BF_OK;
}

int bf_shard_import(bf_handle* h, const uint8_t* buf, uint64_t len, uint32_t mode) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    return import_bytes(h, buf, len, mode, h->local_bits);
}

int bf_route_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                 void* d_send, uint32_t* d_slot, uint64_t* d_counts, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (!d_counts) return set_err(h, BF_EINVAL, "d_counts is NULL");
    if (n && (!d_key_bytes || !d_offsets || !d_send)) return set_err(h, BF_EINVAL, "NULL device pointer");
    const uint64_t probes = n * h->k;
    if (n && probes / n != h->k) return set_err(h, BF_EINVAL, "n*k overflows");
    if (probes >= (1ull << 32)) return set_err(h, BF_EINVAL, "n*k must be < 2^32 per call (slot indices are 32-bit)");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    auto* counts = reinterpret_cast<unsigned long long*>(d_counts);
    BfBinPlan plan;
    if (h->binned_mode != 0 && bf_route_plan(n, h->k, h->shards, !h->route32, d_slot != nullptr, &plan)) {
        // fused: hash + per-tile LDS sort by owner, then one owner-major gather
        int rc = ensure_scratch(h, plan.scratch_bytes);
        if (rc) return rc;
        uint64_t bias = 0;
        const uint8_t* k16 = align_keys(d_key_bytes, &bias);
        BfMarks* mk = prof_begin(h, s);
        HIPCHK(h, bf_launch_route_fused(h->g, plan, !h->route32, k16, d_offsets, bias, n, h->d_bin_scratch, d_send,
                                        d_slot, counts, s, mk));
        return BF_OK;
    }
    int rc = ensure_route_scratch(h, std::max<uint64_t>(probes, 1));
    if (rc) return rc;
    HIPCHK(h, hipMemsetAsync(counts, 0, h->shards * sizeof(unsigned long long), s));
    BfMarks* mk = prof_begin(h, s);
    if (n) {
        uint64_t bias = 0;
        const uint8_t* k16 = align_keys(d_key_bytes, &bias);
        HIPCHK(h, bf_launch_keys(BF_OP_ROUTE, h->g, k16, d_offsets, bias, n, h->d_tmp_owner, h->d_tmp_local,
                                 nullptr, s, counts));
        bf_mark(mk, s, op_kernel_name(BF_OP_ROUTE));
    }
    HIPCHK(h, bf_launch_route_scatter(h->d_tmp_local, h->d_tmp_owner, probes, h->shards, h->k, counts,
                                      h->d_cursor, d_send, d_slot, h->route32, s));
    bf_mark(mk, s, "route_scatter");
    return BF_OK;
}

int bf_route_window_split(const bf_handle* h, uint32_t* nh) {
    if (h && h->multi) return BF_EINVAL;
    if (!h || !nh) return BF_EINVAL;
    // the largest shard (index 0) holds ceil(nblocks / P) blocks
    const uint64_t nblocks = (h->reach + (1ull << h->block_log2) - 1) >> h->block_log2;
    const uint64_t bits0 = h->shards == 1 ? h->reach : ((nblocks + h->shards - 1) / h->shards) << h->block_log2;
    *nh = (uint32_t)((bits0 + 0xFFFFFFFFull) >> 32);
    if (*nh == 0) *nh = 1;
    return BF_OK;
}

int bf_route_windows_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                         uint32_t* d_send, uint32_t* d_slot, uint64_t window_cap, uint64_t* d_counts, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (!d_counts) return set_err(h, BF_EINVAL, "d_counts is NULL");
    if (n && (!d_key_bytes || !d_offsets || !d_send)) return set_err(h, BF_EINVAL, "NULL device pointer");
    const uint64_t probes = n * h->k;
    if (n && probes / n != h->k) return set_err(h, BF_EINVAL, "n*k overflows");
    if (probes >= (1ull << 32)) return set_err(h, BF_EINVAL, "n*k must be < 2^32 per call (slot indices are 32-bit)");
    uint32_t nh = 1;
    bf_route_window_split(h, &nh);
    const uint32_t nwin = h->shards * nh;
    if (nwin > 256) return set_err(h, BF_EINVAL, "%u shards x %u sub-ranges exceed 256 windows", h->shards, nh);
    if (window_cap && (uint64_t)nwin > ~0ull / window_cap) return set_err(h, BF_EINVAL, "window_cap overflows");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    BfBinPlan plan;
    if (n && !bf_route_plan(n, h->k, nwin, false, d_slot != nullptr, &plan))
        return set_err(h, BF_EINVAL, "batch of %llu keys at k=%u over %u windows exceeds one window-route pass",
                       (unsigned long long)n, h->k, nwin);
    if (!n) plan.nsup = nwin;
    uint64_t bias = 0;
    const uint8_t* k16 = n ? align_keys(d_key_bytes, &bias) : nullptr;
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_route_windows(h->g, plan, nh, k16, d_offsets, bias, n, d_send, d_slot, window_cap,
                                      reinterpret_cast<unsigned long long*>(d_counts), s, mk));
    return BF_OK;
}

namespace {
// The chunked-window geometry of a shard handle's filter (the same on every rank: it depends
// on the largest shard's size and the window count only).
constexpr uint32_t kL2SweepMaxSupLog2 = 25;   // 4 MiB superbins: what one XCD's L2 keeps

// l2 (nullable): whether the owner's include? takes the L2-local sweep with this geometry.
static bool handle_chunks(const bf_handle* h, BfChunks* cg, uint32_t* nh_out, bool* l2 = nullptr) {
    uint32_t nh = 1;
    bf_route_window_split(h, &nh);
    const uint64_t nblocks = (h->reach + (1ull << h->block_log2) - 1) >> h->block_log2;
    const uint64_t bits0 = h->shards == 1 ? h->reach : ((nblocks + h->shards - 1) / h->shards) << h->block_log2;
    if (nh_out) *nh_out = nh;
    const uint32_t nwin = h->shards * nh;
    bool sweep = false;
    if (h->chunk_buckets) {   // forced
        if (!bf_chunk_geometry(bits0, nwin, h->bin_region_log2, cg, h->chunk_buckets)) return false;
        sweep = h->chunk_test_l2 == 1 || (h->chunk_test_l2 == 2 && cg->sup_log2 <= kL2SweepMaxSupLog2);
    } else if (h->chunk_test_l2 != 0 && bf_chunk_geometry(bits0, nwin, h->bin_region_log2, cg, 512) &&
               (h->chunk_test_l2 == 1 || cg->sup_log2 <= kL2SweepMaxSupLog2)) {
        sweep = true;
    } else if (!bf_chunk_geometry(bits0, nwin, h->bin_region_log2, cg, 256)) {
        return false;   // (shard counts whose windows take no geometry keep the plain windows)
    } else {
        // the sorted owner: 512 buckets where 256 fit, twice the superbins, so a region's runs in
        // each sorted block are twice as long for the owner's apply / test (200B x 8: apply_test
        // 1.78 -> 1.23 ms, the mids +0.32, per rank 6.96 -> 6.72 ms:
        // profiles/r06h_ab_chunk_buckets.jsonl)
        BfChunks c512;
        if (bf_chunk_geometry(bits0, nwin, h->bin_region_log2, &c512, 512)) *cg = c512;
    }
    if (l2) *l2 = sweep;
    return true;
}

static uint64_t route_tile_keys(uint32_t k) { return k <= 6 ? 2048 : 1024; }   // bf_route_plan's tiles

static int check_chunk_args(bf_handle* h, const BfChunks& cg, uint64_t dir_bytes, uint64_t tiles) {
    if (!tiles) return set_err(h, BF_EINVAL, "tiles is 0");
    if (dir_bytes < bf_chunk_dir_bytes(cg, tiles) || (dir_bytes & 15))
        return set_err(h, BF_EINVAL, "dir_bytes %llu does not hold %llu tiles (bf_route_chunk_info)",
                       (unsigned long long)dir_bytes, (unsigned long long)tiles);
    return BF_OK;
}
}  // namespace

int bf_route_chunk_info(const bf_handle* h, uint64_t n_bound, uint64_t* tiles, uint64_t* dir_bytes,
                        uint32_t* superbins) {
    if (!h || h->multi || !tiles || !dir_bytes) return BF_EINVAL;
    BfChunks cg;
    if (!handle_chunks(h, &cg, nullptr)) return BF_EINVAL;
    const uint64_t tk = route_tile_keys(h->k);
    *tiles = std::max<uint64_t>(1, (n_bound + tk - 1) / tk);
    *dir_bytes = bf_chunk_dir_bytes(cg, *tiles);
    if (superbins) *superbins = cg.S;
    return BF_OK;
}

namespace {
// dig: d_key_bytes holds n SHA-1 word quadruples (d_offsets unused).
int route_chunks_impl(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n, bool dig,
                      uint32_t* d_send, uint16_t* d_slot16, uint64_t window_cap, uint64_t* d_counts, uint8_t* d_dir,
                      uint64_t dir_bytes, uint64_t tiles, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (!d_counts || !d_dir) return set_err(h, BF_EINVAL, "d_counts / d_dir is NULL");
    if (n && (!d_key_bytes || (!dig && !d_offsets) || !d_send)) return set_err(h, BF_EINVAL, "NULL device pointer");
    if (dig && n && (reinterpret_cast<uintptr_t>(d_key_bytes) & 15u))
        return set_err(h, BF_EINVAL, "d_digests must be 16-byte aligned");
    const uint64_t probes = n * h->k;
    if (n && probes / n != h->k) return set_err(h, BF_EINVAL, "n*k overflows");
    if (probes >= (1ull << 32)) return set_err(h, BF_EINVAL, "n*k must be < 2^32 per call");
    if (window_cap >= (1ull << 32) - 1) return set_err(h, BF_EINVAL, "window_cap must be < 2^32 - 1");
    BfChunks cg;
    uint32_t nh = 1;
    if (!handle_chunks(h, &cg, &nh)) return set_err(h, BF_EINVAL, "this shard count cannot take chunked windows");
    const uint32_t nwin = h->shards * nh;
    int rc = check_chunk_args(h, cg, dir_bytes, tiles);
    if (rc) return rc;
    if ((n + route_tile_keys(h->k) - 1) / route_tile_keys(h->k) > tiles)
        return set_err(h, BF_EINVAL, "%llu keys need more than %llu route tiles", (unsigned long long)n,
                       (unsigned long long)tiles);
    if ((uint64_t)nwin > ~0ull / std::max<uint64_t>(window_cap, 1)) return set_err(h, BF_EINVAL, "window_cap overflows");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    BfBinPlan plan;
    if (n && !bf_route_plan(n, h->k, nwin, false, d_slot16 != nullptr, &plan))
        return set_err(h, BF_EINVAL, "batch of %llu keys at k=%u over %u windows exceeds one route pass",
                       (unsigned long long)n, h->k, nwin);
    if (!n) plan.nsup = nwin;
    if (n && plan.tile_keys != route_tile_keys(h->k)) return set_err(h, BF_EINVAL, "route tile size mismatch");
    cg.dir = d_dir;
    cg.dir_bytes = dir_bytes;
    cg.tiles = tiles;
    uint64_t bias = 0;
    const uint8_t* k16 = n ? (dig ? d_key_bytes : align_keys(d_key_bytes, &bias)) : nullptr;
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_route_chunks(h->g, plan, nh, cg, k16, d_offsets, bias, n, d_send, d_slot16, window_cap,
                                     reinterpret_cast<unsigned long long*>(d_counts), s, mk, dig));
    return BF_OK;
}
}  // namespace

int bf_route_chunks_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                        uint32_t* d_send, uint16_t* d_slot16, uint64_t window_cap, uint64_t* d_counts, uint8_t* d_dir,
                        uint64_t dir_bytes, uint64_t tiles, void* stream) {
    return route_chunks_impl(h, d_key_bytes, d_offsets, n, false, d_send, d_slot16, window_cap, d_counts, d_dir,
                             dir_bytes, tiles, stream);
}

int bf_route_chunks_digests_dev(bf_handle* h, const uint32_t* d_digests, uint64_t n, uint32_t* d_send,
                                uint16_t* d_slot16, uint64_t window_cap, uint64_t* d_counts, uint8_t* d_dir,
                                uint64_t dir_bytes, uint64_t tiles, void* stream) {
    return route_chunks_impl(h, reinterpret_cast<const uint8_t*>(d_digests), nullptr, n, true, d_send, d_slot16,
                             window_cap, d_counts, d_dir, dir_bytes, tiles, stream);
}

namespace {
// side (test only): a key batch [keys, offsets, n) whose SHA-1 words go to side_dig (nullable).
// d_packed (test only, instead of d_bits): the answers as packed bits in the return trip's layout
// (window (h, src) at d_packed + (src * nh + h) * ceil(window_cap / 8)).  The sorted test takes
// ordered chunks and stores them so directly; every other form (the L2 sweep, the direct owner
// ops, a geometry the ordered form does not take) writes answer bytes into the handle's own
// buffer and packs them.
static int shard_chunks_impl(bf_handle* h, const uint32_t* d_recv, uint64_t window_cap, uint32_t nsrc, const uint8_t* d_dir,
                      uint64_t dir_bytes, uint64_t tiles, const uint64_t* d_counts, uint32_t count_stride,
                      uint32_t* d_any_new, uint8_t* d_bits, bool test, void* stream,
                      const uint8_t* side_keys = nullptr, const uint64_t* side_offsets = nullptr, uint64_t side_n = 0,
                      uint32_t* side_dig = nullptr, uint8_t* d_packed = nullptr) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (side_n && (!side_keys || !side_offsets || !side_dig)) return set_err(h, BF_EINVAL, "NULL side-hash pointer");
    if (!nsrc || !window_cap)
        return side_n ? bf_hash_many_dev(h, side_keys, side_offsets, side_n, side_dig, stream) : BF_OK;
    if (!d_recv || !d_dir || !d_counts || (test && !d_bits && !d_packed)) return set_err(h, BF_EINVAL, "NULL device pointer");
    BfChunks cg;
    uint32_t nh = 1;
    bool sweep = false;
    if (!handle_chunks(h, &cg, &nh, &sweep)) return set_err(h, BF_EINVAL, "this shard count cannot take chunked windows");
    int rc = check_chunk_args(h, cg, dir_bytes, tiles);
    if (rc) return rc;
    if (count_stride < nh) return set_err(h, BF_EINVAL, "count_stride %u < %u sub-ranges", count_stride, nh);
    const uint64_t total = (uint64_t)nh * nsrc * window_cap;
    if (total / window_cap != (uint64_t)nh * nsrc || total >= (1ull << 32))
        return set_err(h, BF_EINVAL, "%u sub-ranges x %u windows x %llu entries must stay below 2^32", nh, nsrc,
                       (unsigned long long)window_cap);
    cg.tiles = tiles;
    BfChunkIn ci;
    ci.recv = d_recv;
    ci.dir = d_dir;
    ci.dir_bytes = dir_bytes;
    ci.tiles = tiles;
    ci.cap = window_cap;
    ci.limit = h->local_bits;
    ci.counts = reinterpret_cast<const unsigned long long*>(d_counts);
    ci.cstride = count_stride;
    ci.nsrc = nsrc;
    ci.nh = nh;
    ci.S = cg.S;
    ci.sup_log2 = cg.sup_log2;
    BfBinPlan plan;
    const bool binned = (test ? h->shard_test_binned_mode : h->binned_mode) != 0 &&
                        bf_chunk_plan(h->dev_bytes, cg, nh, nsrc, window_cap, test, &plan, sweep) &&
                        ((test ? h->shard_test_binned_mode : h->binned_mode) == 1 ||
                         (h->dev_bytes >= (64ull << 20) &&
                          (double)total * 128.0 > kBinnedCostRatio * (double)h->dev_bytes));
    if (d_packed && binned && !plan.l2test && !side_n &&
        bf_chunk_plan(h->dev_bytes, cg, nh, nsrc, window_cap, true, &plan, false, true)) {
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceGuard dg(h->device);
        if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
        StreamOrder so(h, pick_stream(h, stream));
        if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
        if ((rc = ensure_scratch(h, plan.scratch_bytes))) return rc;
        BfMarks* mk = prof_begin(h, so.s);
        HIPCHK(h, bf_launch_shard_test_chunks_packed(h->g, plan, h->dev_bytes, ci, h->d_bin_scratch, d_packed, so.s, mk));
        return BF_OK;
    }
    if (d_packed) {   // answer bytes into the handle's buffer, then packed per window
        const uint64_t nbytes = (uint64_t)nh * nsrc * window_cap;
        if (nbytes > h->ans8_cap) {
            std::lock_guard<std::mutex> lk(h->mu);
            DeviceGuard dg(h->device);
            if (h->order_valid) HIPCHK(h, hipEventSynchronize(h->order_ev));   // a previous call may still read it
            if (h->d_ans8) (void)hipFree(h->d_ans8);
            h->d_ans8 = nullptr;
            h->ans8_cap = 0;
            HIPCHK(h, hipMalloc((void**)&h->d_ans8, nbytes));
            h->ans8_cap = nbytes;
        }
        rc = shard_chunks_impl(h, d_recv, window_cap, nsrc, d_dir, dir_bytes, tiles, d_counts, count_stride, nullptr,
                               h->d_ans8, true, stream, side_keys, side_offsets, side_n, side_dig);
        if (rc) return rc;
        std::vector<uint64_t> seg;   // (src, count, dst): sub-range h of source src -> its packed window
        const uint64_t cap8 = (window_cap + 7) / 8;
        for (uint32_t src = 0; src < nsrc; ++src)
            for (uint32_t hh = 0; hh < nh; ++hh) {
                seg.push_back(((uint64_t)hh * nsrc + src) * window_cap);
                seg.push_back(window_cap);
                seg.push_back(((uint64_t)src * nh + hh) * cap8);
            }
        std::lock_guard<std::mutex> lk(h->mu);
        DeviceGuard dg(h->device);
        if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
        StreamOrder so(h, pick_stream(h, stream));
        const uint64_t sb = seg.size() * 8;
        // the table depends on (nsrc, nh, window_cap) only: uploaded (with one sync) when they change
        if (h->seg_nsrc != nsrc || h->seg_nh != nh || h->seg_wcap != window_cap) {
            if (h->order_valid) HIPCHK(h, hipEventSynchronize(h->order_ev));   // a previous call may still read it
            HIPCHK(h, hipStreamSynchronize(so.s));
            if (sb > h->seg_cap) {
                if (h->d_seg) (void)hipFree(h->d_seg);
                h->d_seg = nullptr;
                h->seg_cap = 0;
                HIPCHK(h, hipMalloc((void**)&h->d_seg, sb));
                h->seg_cap = sb;
            }
            HIPCHK(h, hipMemcpy(h->d_seg, seg.data(), sb, hipMemcpyHostToDevice));
            h->seg_nsrc = nsrc;
            h->seg_nh = nh;
            h->seg_wcap = window_cap;
        }
        BfMarks* mk = prof_begin(h, so.s);
        HIPCHK(h, bf_launch_pack_segments(h->d_ans8, reinterpret_cast<const unsigned long long*>(h->d_seg),
                                          nh * nsrc, window_cap, d_packed, so.s));
        bf_mark(mk, so.s, "pack_answers");
        return BF_OK;
    }
    if (!binned) {   // the direct owner ops read the same windows (the directories unused)
        for (uint32_t hi = 0; hi < nh; ++hi) {
            const uint32_t* rw = d_recv + (uint64_t)hi * nsrc * window_cap;
            const uint64_t* cw = d_counts + hi;
            rc = test ? bf_shard_test_windows_dev(h, rw, window_cap, nsrc, cw, count_stride, hi,
                                                  d_bits + (uint64_t)hi * nsrc * window_cap, stream)
                      : bf_shard_insert_windows_dev(h, rw, window_cap, nsrc, cw, count_stride, hi, d_any_new, stream);
            if (rc) return rc;
        }
        return side_n ? bf_hash_many_dev(h, side_keys, side_offsets, side_n, side_dig, stream) : BF_OK;
    }
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    if ((rc = ensure_scratch(h, plan.scratch_bytes))) return rc;
    BfMarks* mk = prof_begin(h, s);
    BfSideHash side;
    if (side_n) {
        side.keys16 = align_keys(side_keys, &side.bias);
        side.offsets = side_offsets;
        side.n = side_n;
        side.dig = reinterpret_cast<uint4*>(side_dig);
        side.key_status = h->g.key_status;
    }
    if (test)
        HIPCHK(h, bf_launch_shard_test_chunks(h->g, plan, h->dev_bytes, ci, h->d_bin_scratch, d_bits, s, mk, side));
    else
        HIPCHK(h, bf_launch_shard_insert_chunks(h->g, plan, h->dev_bytes, ci, h->d_bin_scratch, d_any_new, s, mk));
    return BF_OK;
}
}  // namespace

int bf_shard_insert_chunks_dev(bf_handle* h, const uint32_t* d_recv, uint64_t window_cap, uint32_t nsrc,
                               const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles, const uint64_t* d_counts,
                               uint32_t count_stride, uint32_t* d_any_new, void* stream) {
    return shard_chunks_impl(h, d_recv, window_cap, nsrc, d_dir, dir_bytes, tiles, d_counts, count_stride, d_any_new,
                             nullptr, false, stream);
}

int bf_shard_test_chunks_dev(bf_handle* h, const uint32_t* d_recv, uint64_t window_cap, uint32_t nsrc,
                             const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles, const uint64_t* d_counts,
                             uint32_t count_stride, uint8_t* d_bits, void* stream) {
    return shard_chunks_impl(h, d_recv, window_cap, nsrc, d_dir, dir_bytes, tiles, d_counts, count_stride, nullptr,
                             d_bits, true, stream);
}

int bf_shard_test_chunks_packed_dev(bf_handle* h, const uint32_t* d_recv, uint64_t window_cap, uint32_t nsrc,
                                    const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles, const uint64_t* d_counts,
                                    uint32_t count_stride, uint8_t* d_packed, void* stream) {
    if (h && !h->multi && !d_packed) return set_err(h, BF_EINVAL, "d_packed is NULL");
    return shard_chunks_impl(h, d_recv, window_cap, nsrc, d_dir, dir_bytes, tiles, d_counts, count_stride, nullptr,
                             nullptr, true, stream, nullptr, nullptr, 0, nullptr, d_packed);
}

int bf_shard_insert_test_chunks_packed_dev(bf_handle* h, const uint32_t* d_ins_recv, const uint8_t* d_ins_dir,
                                           const uint64_t* d_ins_counts, const uint32_t* d_tst_recv,
                                           const uint8_t* d_tst_dir, const uint64_t* d_tst_counts,
                                           uint64_t window_cap, uint32_t nsrc, uint64_t dir_bytes, uint64_t tiles,
                                           uint32_t count_stride, uint32_t* d_any_new, uint8_t* d_packed,
                                           const uint8_t* d_next_keys, const uint64_t* d_next_offsets,
                                           uint64_t n_next, uint32_t* d_next_digests, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (!d_packed) return set_err(h, BF_EINVAL, "d_packed is NULL");
    if (n_next && (!d_next_keys || !d_next_offsets || !d_next_digests))
        return set_err(h, BF_EINVAL, "NULL side-hash pointer");
    if (n_next && (reinterpret_cast<uintptr_t>(d_next_digests) & 15u))
        return set_err(h, BF_EINVAL, "d_next_digests must be 16-byte aligned");
    if (!nsrc || !window_cap)
        return n_next ? bf_hash_many_dev(h, d_next_keys, d_next_offsets, n_next, d_next_digests, stream) : BF_OK;
    if (!d_ins_recv || !d_ins_dir || !d_ins_counts || !d_tst_recv || !d_tst_dir || !d_tst_counts)
        return set_err(h, BF_EINVAL, "NULL device pointer");
    BfChunks cg;
    uint32_t nh = 1;
    bool sweep = false;
    if (!handle_chunks(h, &cg, &nh, &sweep)) return set_err(h, BF_EINVAL, "this shard count cannot take chunked windows");
    int rc = check_chunk_args(h, cg, dir_bytes, tiles);
    if (rc) return rc;
    if (count_stride < nh) return set_err(h, BF_EINVAL, "count_stride %u < %u sub-ranges", count_stride, nh);
    const uint64_t total = (uint64_t)nh * nsrc * window_cap;
    if (total / window_cap != (uint64_t)nh * nsrc || total >= (1ull << 32))
        return set_err(h, BF_EINVAL, "%u sub-ranges x %u windows x %llu entries must stay below 2^32", nh, nsrc,
                       (unsigned long long)window_cap);
    cg.tiles = tiles;
    BfBinPlan pi, pt;
    // one pass only where both owner ops would take their sorted binned forms on this shard (the
    // same rule as shard_chunks_impl) and the include? its ordered form; else the two calls
    const bool dense_enough = h->dev_bytes >= (64ull << 20) && (double)total * 128.0 > kBinnedCostRatio * (double)h->dev_bytes;
    const bool fused = h->binned_mode != 0 && h->shard_test_binned_mode != 0 && !sweep &&
                       (h->binned_mode == 1 || dense_enough) && (h->shard_test_binned_mode == 1 || dense_enough) &&
                       bf_chunk_plan(h->dev_bytes, cg, nh, nsrc, window_cap, false, &pi) &&
                       bf_chunk_plan(h->dev_bytes, cg, nh, nsrc, window_cap, true, &pt, false, true);
    if (!fused) {
        rc = bf_shard_insert_chunks_dev(h, d_ins_recv, window_cap, nsrc, d_ins_dir, dir_bytes, tiles, d_ins_counts,
                                        count_stride, d_any_new, stream);
        if (rc) return rc;
        rc = bf_shard_test_chunks_packed_dev(h, d_tst_recv, window_cap, nsrc, d_tst_dir, dir_bytes, tiles, d_tst_counts,
                                             count_stride, d_packed, stream);
        if (rc) return rc;
        return n_next ? bf_hash_many_dev(h, d_next_keys, d_next_offsets, n_next, d_next_digests, stream) : BF_OK;
    }
    BfChunkIn cii;
    cii.recv = d_ins_recv;
    cii.dir = d_ins_dir;
    cii.dir_bytes = dir_bytes;
    cii.tiles = tiles;
    cii.cap = window_cap;
    cii.limit = h->local_bits;
    cii.counts = reinterpret_cast<const unsigned long long*>(d_ins_counts);
    cii.cstride = count_stride;
    cii.nsrc = nsrc;
    cii.nh = nh;
    cii.S = cg.S;
    cii.sup_log2 = cg.sup_log2;
    BfChunkIn cit = cii;
    cit.recv = d_tst_recv;
    cit.dir = d_tst_dir;
    cit.counts = reinterpret_cast<const unsigned long long*>(d_tst_counts);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    if ((rc = ensure_scratch(h, bf_chunk_scratch_bytes(pi) + bf_chunk_scratch_bytes(pt)))) return rc;
    BfSideHash side;
    if (n_next) {
        side.keys16 = align_keys(d_next_keys, &side.bias);
        side.offsets = d_next_offsets;
        side.n = n_next;
        side.dig = reinterpret_cast<uint4*>(d_next_digests);
        side.key_status = h->g.key_status;
    }
    BfMarks* mk = prof_begin(h, so.s);
    HIPCHK(h, bf_launch_shard_insert_test_chunks_packed(h->g, pi, pt, h->dev_bytes, cii, cit, h->d_bin_scratch,
                                                        d_any_new, d_packed, so.s, mk, side));
    return BF_OK;
}

int bf_shard_test_chunks_hash_dev(bf_handle* h, const uint32_t* d_recv, uint64_t window_cap, uint32_t nsrc,
                                  const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles, const uint64_t* d_counts,
                                  uint32_t count_stride, uint8_t* d_bits, const uint8_t* d_next_keys,
                                  const uint64_t* d_next_offsets, uint64_t n_next, uint32_t* d_next_digests,
                                  void* stream) {
    return shard_chunks_impl(h, d_recv, window_cap, nsrc, d_dir, dir_bytes, tiles, d_counts, count_stride, nullptr,
                             d_bits, true, stream, d_next_keys, d_next_offsets, n_next, d_next_digests);
}

int bf_combine_chunks_packed_dev(bf_handle* h, const uint8_t* d_packed, const uint16_t* d_slot16, uint64_t window_cap,
                                 const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles, const uint64_t* d_counts,
                                 uint64_t n, uint8_t* d_out, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (n && (!d_packed || !d_slot16 || !d_dir || !d_counts || !d_out))
        return set_err(h, BF_EINVAL, "NULL device pointer");
    BfChunks cg;
    uint32_t nh = 1;
    if (!handle_chunks(h, &cg, &nh)) return set_err(h, BF_EINVAL, "this shard count cannot take chunked windows");
    int rc = check_chunk_args(h, cg, dir_bytes, tiles);
    if (rc) return rc;
    const uint64_t tk = route_tile_keys(h->k);
    if ((n + tk - 1) / tk > tiles) return set_err(h, BF_EINVAL, "n exceeds the directory's tiles");
    cg.dir = const_cast<uint8_t*>(d_dir);
    cg.dir_bytes = dir_bytes;
    cg.tiles = tiles;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_combine_chunks_packed(d_packed, d_slot16, window_cap, cg, h->shards * nh,
                                              reinterpret_cast<const unsigned long long*>(d_counts), n, (uint32_t)tk,
                                              d_out, s));
    bf_mark(mk, s, "combine_chunks");
    return BF_OK;
}

namespace {
// Owner-side OR of `count` routed local offsets: uint32 entries when u32 (+ bias), else uint64.
static int shard_insert_impl(bf_handle* h, const void* d_local, bool u32, uint64_t bias, uint64_t count, uint32_t* d_any_new,
                      void* stream, const BfWindows& win = BfWindows{}) {
    if (!h) return BF_EINVAL;
    if (count && !d_local) return set_err(h, BF_EINVAL, "d_local is NULL");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    // Binned when the routed probes' random line fills clearly exceed a streaming pass
    // over the shard (same policy and knob as the whole-filter insert).
    BfBinPlan plan;
    const uint64_t sub = std::max<uint64_t>(1, bf_binned_max_offsets(h->dev_bytes, h->bin_region_log2));
    const bool binned = h->binned_mode != 0 &&
                        bf_binned_plan_offsets(h->dev_bytes, std::min(count, sub), h->bin_region_log2, &plan) &&
                        (h->binned_mode == 1 || (h->dev_bytes >= (64ull << 20) &&
                                                 (double)count * 128.0 > kBinnedCostRatio * (double)h->dev_bytes)) &&
                        (!win.counts || (win.cap % BF_WINDOW_CAP_ALIGN == 0 && count <= sub));
    if (binned && win.counts) {   // the windows as one binned pass (entries past a window's count skipped)
        int rc = ensure_scratch(h, plan.scratch_bytes);
        if (rc) return rc;
        BfMarks* mk = prof_begin(h, s);
        HIPCHK(h, bf_launch_shard_insert_binned(h->g, plan, h->dev_bytes, d_local, u32, count, h->d_bin_scratch,
                                                d_any_new, s, mk, bias, win));
        return BF_OK;
    }
    if (binned) {
        const size_t esz = u32 ? 4 : 8;
        for (uint64_t c0 = 0; c0 < count; c0 += sub) {
            const uint64_t cn = std::min(sub, count - c0);
            if (cn != std::min(count, sub) && !bf_binned_plan_offsets(h->dev_bytes, cn, h->bin_region_log2, &plan))
                return set_err(h, BF_EINVAL, "binned plan failed for a tail of %llu offsets", (unsigned long long)cn);
            int rc = ensure_scratch(h, plan.scratch_bytes);
            if (rc) return rc;
            BfMarks* mk = prof_begin(h, s);
            HIPCHK(h, bf_launch_shard_insert_binned(h->g, plan, h->dev_bytes,
                                                    static_cast<const uint8_t*>(d_local) + c0 * esz, u32, cn,
                                                    h->d_bin_scratch, d_any_new, s, mk, bias));
        }
        return BF_OK;
    }
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_shard_insert(h->g.bits, h->local_bits, d_local, count, d_any_new, u32, s, bias, h->g.dirty, win));
    bf_mark(mk, s, "shard_insert");
    return BF_OK;
}
}  // namespace

int bf_shard_insert_dev(bf_handle* h, const void* d_local, uint64_t count, uint32_t* d_any_new, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    return shard_insert_impl(h, d_local, h->route32, 0, count, d_any_new, stream);
}

int bf_shard_insert_hi_dev(bf_handle* h, const uint32_t* d_local32, uint64_t count, uint32_t hi, uint32_t* d_any_new,
                           void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (((uint64_t)hi << 32) >= h->local_bits) return set_err(h, BF_EINVAL, "hi=%u is past the shard", hi);
    return shard_insert_impl(h, d_local32, true, (uint64_t)hi << 32, count, d_any_new, stream);
}

namespace {
static int shard_test_impl(bf_handle* h, const void* d_local, bool u32, uint64_t bias, uint64_t count, uint8_t* d_bits,
                    void* stream, const BfWindows& win = BfWindows{}) {
    if (!h) return BF_EINVAL;
    if (count && (!d_local || !d_bits)) return set_err(h, BF_EINVAL, "NULL device pointer");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    // Binned like the shard insert: routed probes carry no early exit (all k arrive), so
    // one streaming pass over the shard beats a random line fill per probe once the
    // probes outnumber the shard's lines (same cost model and knob shape as the insert).
    BfBinPlan plan;
    const uint64_t sub = std::max<uint64_t>(1, bf_binned_max_offsets(h->dev_bytes, h->bin_region_log2));
    const uint32_t mode = h->shard_test_binned_mode;
    const bool binned = mode != 0 &&
                        bf_binned_plan_offsets(h->dev_bytes, std::min(count, sub), h->bin_region_log2, &plan, true) &&
                        (mode == 1 || (h->dev_bytes >= (64ull << 20) &&
                                       (double)count * 128.0 > kBinnedCostRatio * (double)h->dev_bytes)) &&
                        (!win.counts || (win.cap % BF_WINDOW_CAP_ALIGN == 0 && count <= sub));
    if (binned && win.counts) {
        int rc = ensure_scratch(h, plan.scratch_bytes);
        if (rc) return rc;
        BfMarks* mk = prof_begin(h, s);
        HIPCHK(h, bf_launch_shard_test_binned(h->g, plan, h->dev_bytes, d_local, u32, count, h->d_bin_scratch, d_bits,
                                              s, mk, bias, win));
        return BF_OK;
    }
    if (binned) {
        const size_t esz = u32 ? 4 : 8;
        for (uint64_t c0 = 0; c0 < count; c0 += sub) {
            const uint64_t cn = std::min(sub, count - c0);
            if (cn != std::min(count, sub) &&
                !bf_binned_plan_offsets(h->dev_bytes, cn, h->bin_region_log2, &plan, true))
                return set_err(h, BF_EINVAL, "binned plan failed for a tail of %llu offsets", (unsigned long long)cn);
            int rc = ensure_scratch(h, plan.scratch_bytes);
            if (rc) return rc;
            BfMarks* mk = prof_begin(h, s);
            HIPCHK(h, bf_launch_shard_test_binned(h->g, plan, h->dev_bytes,
                                                  static_cast<const uint8_t*>(d_local) + c0 * esz, u32, cn,
                                                  h->d_bin_scratch, d_bits + c0, s, mk, bias));
        }
        return BF_OK;
    }
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_shard_test(h->g.bits, h->local_bits, d_local, count, d_bits, u32, s, bias, win));
    bf_mark(mk, s, "shard_test");
    return BF_OK;
}

}  // namespace

int bf_shard_insert_windows_dev(bf_handle* h, const uint32_t* d_local32, uint64_t window_cap, uint32_t nwin,
                                const uint64_t* d_counts, uint32_t count_stride, uint32_t hi, uint32_t* d_any_new,
                                void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (((uint64_t)hi << 32) >= h->local_bits) return set_err(h, BF_EINVAL, "hi=%u is past the shard", hi);
    if (nwin && window_cap && !d_counts) return set_err(h, BF_EINVAL, "d_counts is NULL");
    if (window_cap && (uint64_t)nwin > ~0ull / window_cap) return set_err(h, BF_EINVAL, "window sizes overflow");
    if (nwin > 65535) return set_err(h, BF_EINVAL, "at most 65535 windows");
    return shard_insert_impl(h, d_local32, true, (uint64_t)hi << 32, (uint64_t)nwin * window_cap, d_any_new, stream,
                             BfWindows(d_counts, count_stride, nwin, window_cap));
}

int bf_shard_test_windows_dev(bf_handle* h, const uint32_t* d_local32, uint64_t window_cap, uint32_t nwin,
                              const uint64_t* d_counts, uint32_t count_stride, uint32_t hi, uint8_t* d_bits,
                              void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (((uint64_t)hi << 32) >= h->local_bits) return set_err(h, BF_EINVAL, "hi=%u is past the shard", hi);
    if (nwin && window_cap && !d_counts) return set_err(h, BF_EINVAL, "d_counts is NULL");
    if (window_cap && (uint64_t)nwin > ~0ull / window_cap) return set_err(h, BF_EINVAL, "window sizes overflow");
    if (nwin > 65535) return set_err(h, BF_EINVAL, "at most 65535 windows");
    return shard_test_impl(h, d_local32, true, (uint64_t)hi << 32, (uint64_t)nwin * window_cap, d_bits, stream,
                           BfWindows(d_counts, count_stride, nwin, window_cap));
}

int bf_shard_test_dev(bf_handle* h, const void* d_local, uint64_t count, uint8_t* d_bits, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    return shard_test_impl(h, d_local, h->route32, 0, count, d_bits, stream);
}

int bf_shard_test_hi_dev(bf_handle* h, const uint32_t* d_local32, uint64_t count, uint32_t hi, uint8_t* d_bits,
                         void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (((uint64_t)hi << 32) >= h->local_bits) return set_err(h, BF_EINVAL, "hi=%u is past the shard", hi);
    return shard_test_impl(h, d_local32, true, (uint64_t)hi << 32, count, d_bits, stream);
}

int bf_combine_dev(bf_handle* h, const uint8_t* d_bits, const uint32_t* d_slot, uint64_t n, uint8_t* d_out,
                   void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (n && (!d_bits || !d_slot || !d_out)) return set_err(h, BF_EINVAL, "NULL device pointer");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_combine(d_bits, d_slot, n, h->k, d_out, s));
    bf_mark(mk, s, "combine");
    return BF_OK;
}

int bf_combine_windows_dev(bf_handle* h, const uint8_t* d_bits, const uint32_t* d_slot, uint64_t window_cap,
                           uint32_t nwin, const uint64_t* d_counts, uint64_t n, uint8_t* d_out, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (n && (!d_bits || !d_slot || !d_counts || !d_out)) return set_err(h, BF_EINVAL, "NULL device pointer");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_combine_windows(d_bits, d_slot, window_cap, reinterpret_cast<const unsigned long long*>(d_counts),
                                        nwin, n, d_out, s));
    bf_mark(mk, s, "combine");
    return BF_OK;
}

int bf_pack_segments_dev(bf_handle* h, const uint8_t* d_bits, const uint64_t* d_seg, uint32_t nseg,
                         uint64_t max_count, uint8_t* d_packed, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (nseg && (!d_bits || !d_seg || !d_packed)) return set_err(h, BF_EINVAL, "NULL device pointer");
    if (nseg > 65535) return set_err(h, BF_EINVAL, "at most 65535 segments");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_pack_segments(d_bits, reinterpret_cast<const unsigned long long*>(d_seg), nseg, max_count,
                                      d_packed, s));
    bf_mark(mk, s, "pack_answers");
    return BF_OK;
}

int bf_combine_windows_packed_dev(bf_handle* h, const uint8_t* d_packed, const uint32_t* d_slot, uint64_t window_cap,
                                  uint32_t nwin, const uint64_t* d_counts, uint64_t n, uint8_t* d_out, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (n && (!d_packed || !d_slot || !d_counts || !d_out)) return set_err(h, BF_EINVAL, "NULL device pointer");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    hipStream_t s = so.s;
    BfMarks* mk = prof_begin(h, s);
    HIPCHK(h, bf_launch_combine_windows_packed(d_packed, d_slot, window_cap,
                                               reinterpret_cast<const unsigned long long*>(d_counts), nwin, n, d_out,
                                               s));
    bf_mark(mk, s, "combine");
    return BF_OK;
}

int bf_insert_many_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                       uint32_t* d_any_new, uint8_t* d_per_key_new, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    const BfOp op = (d_any_new || d_per_key_new) ? BF_OP_INSERT_FLAGS : BF_OP_INSERT;
    return run_dev(h, op, d_key_bytes, d_offsets, n, d_per_key_new, nullptr, d_any_new, stream);
}

int bf_include_many_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                        uint8_t* d_out, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    return run_dev(h, BF_OP_INCLUDE, d_key_bytes, d_offsets, n, d_out, nullptr, nullptr, stream);
}

int bf_indexes_many_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                        uint64_t* d_out, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    return run_dev(h, BF_OP_INDEXES, d_key_bytes, d_offsets, n, nullptr, d_out, nullptr, stream);
}

namespace {
// The digest ops: binned insert when it pays (as for keys), else one direct lane per digest.
static int run_digests(bf_handle* h, BfOp op, const uint32_t* d_dig, uint64_t n, uint8_t* d_out8, uint32_t* d_flag,
                void* stream) {
    if (!h) return BF_EINVAL;
    if (h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (n == 0) return BF_OK;
    if (!d_dig) return set_err(h, BF_EINVAL, "d_digests is NULL");
    if (reinterpret_cast<uintptr_t>(d_dig) & 15u) return set_err(h, BF_EINVAL, "d_digests must be 16-byte aligned");
    if (op == BF_OP_INCLUDE && !d_out8) return set_err(h, BF_EINVAL, "d_out is NULL");
    if (h->shards > 1) return set_err(h, BF_EINVAL, "handle holds one shard of a partitioned filter");
    if (h->engine != BF_ENGINE_RUBY) return set_err(h, BF_EINVAL, "digests carry the ruby driver's derivation only");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    const uint4* dig = reinterpret_cast<const uint4*>(d_dig);
    const bool is_insert = op == BF_OP_INSERT || op == BF_OP_INSERT_FLAGS;
    BfBinPlan plan;
    const uint64_t sub = std::max<uint64_t>(1, bf_binned_max_keys(h->k, h->dev_bytes, h->bin_region_log2));
    if (is_insert && use_binned(h, std::min(n, sub), false, &plan)) {
        for (uint64_t c0 = 0; c0 < n; c0 += sub) {
            const uint64_t cn = std::min(sub, n - c0);
            if (cn != std::min(n, sub) && !bf_binned_plan(h->dev_bytes, cn, h->k, h->bin_region_log2, false, &plan))
                return set_err(h, BF_EINVAL, "binned plan failed for a tail of %llu keys", (unsigned long long)cn);
            int rc = ensure_scratch(h, plan.scratch_bytes);
            if (rc) return rc;
            BfMarks* mk = prof_begin(h, so.s);
            HIPCHK(h, bf_launch_insert_binned_digests(h->g, plan, h->dev_bytes, dig + c0, cn, h->d_bin_scratch,
                                                      op == BF_OP_INSERT_FLAGS ? d_flag : nullptr, so.s, mk));
        }
        return BF_OK;
    }
    BfMarks* mk = prof_begin(h, so.s);
    HIPCHK(h, bf_launch_digests(op, h->g, dig, n, d_out8, nullptr, d_flag, so.s));
    bf_mark(mk, so.s, op == BF_OP_INCLUDE ? "digest_kernel<INCLUDE>" : "digest_kernel<INSERT>");
    return BF_OK;
}
}  // namespace

int bf_hash_many_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                     uint32_t* d_digests, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (n && !d_digests) return set_err(h, BF_EINVAL, "d_digests is NULL");
    if (reinterpret_cast<uintptr_t>(d_digests) & 15u) return set_err(h, BF_EINVAL, "d_digests must be 16-byte aligned");
    if (n == 0) return BF_OK;
    if (!d_offsets || !d_key_bytes) return set_err(h, BF_EINVAL, "NULL device pointer");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    uint64_t bias = 0;
    const uint8_t* k16 = align_keys(d_key_bytes, &bias);
    BfMarks* mk = prof_begin(h, so.s);
    HIPCHK(h, bf_launch_keys(BF_OP_HASH, h->g, k16, d_offsets, bias, n, nullptr,
                             reinterpret_cast<uint64_t*>(d_digests), nullptr, so.s));
    bf_mark(mk, so.s, "bf_keys_kernel<HASH>");
    return BF_OK;
}

int bf_insert_digests_dev(bf_handle* h, const uint32_t* d_digests, uint64_t n, uint32_t* d_any_new,
                          uint8_t* d_per_key_new, void* stream) {
    if (h && !h->multi && d_per_key_new) return set_err(h, BF_EINVAL, "per_key_new needs the keys (bf_insert_many_dev)");
    return run_digests(h, d_any_new ? BF_OP_INSERT_FLAGS : BF_OP_INSERT, d_digests, n, nullptr, d_any_new, stream);
}

int bf_include_digests_dev(bf_handle* h, const uint32_t* d_digests, uint64_t n, uint8_t* d_out, void* stream) {
    return run_digests(h, BF_OP_INCLUDE, d_digests, n, d_out, nullptr, stream);
}

int bf_include_hash_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                        uint8_t* d_out, const uint8_t* d_next_key_bytes, const uint64_t* d_next_offsets,
                        uint64_t n_next, uint32_t* d_next_digests, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (n && (!d_key_bytes || !d_offsets || !d_out)) return set_err(h, BF_EINVAL, "NULL device pointer");
    if (n_next && (!d_next_key_bytes || !d_next_offsets || !d_next_digests))
        return set_err(h, BF_EINVAL, "NULL device pointer (next batch)");
    if (reinterpret_cast<uintptr_t>(d_next_digests) & 15u)
        return set_err(h, BF_EINVAL, "d_next_digests must be 16-byte aligned");
    if (h->shards > 1) return set_err(h, BF_EINVAL, "handle holds one shard of a partitioned filter");
    if (h->engine != BF_ENGINE_RUBY) return set_err(h, BF_EINVAL, "digests carry the ruby driver's derivation only");
    if (n + n_next == 0) return BF_OK;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    uint64_t bias = 0, nbias = 0;
    const uint8_t* k16 = n ? align_keys(d_key_bytes, &bias) : nullptr;
    const uint8_t* nk16 = n_next ? align_keys(d_next_key_bytes, &nbias) : nullptr;
    BfMarks* mk = prof_begin(h, so.s);
    HIPCHK(h, bf_launch_include_hash(h->g, k16, d_offsets, bias, n, d_out, nk16, d_next_offsets, nbias, n_next,
                                     reinterpret_cast<uint4*>(d_next_digests), so.s));
    bf_mark(mk, so.s, "include_hash_kernel");
    return BF_OK;
}

// ---- replicated inserts from region sets (include/bfhip.h) ----
namespace {
// The encode sorts a batch in one binned pass whose regions are the geometry's: the plan of
// n keys must exist and keep that region size (bf_encode_region_sets_dev refuses others).
bool sets_one_pass(const bf_handle* h, uint64_t n, uint32_t rl, BfBinPlan* plan) {
    if (n == 0) return true;
    return bf_binned_plan(h->dev_bytes, n, h->k, h->bin_region_log2, false, plan) && plan->region_log2 == rl;
}
}  // namespace

int bf_region_sets_capacity(const bf_handle* h, uint64_t n, uint64_t* bytes) {
    if (!h || h->multi || !bytes) return BF_EINVAL;
    *bytes = 0;
    uint32_t rl = 0, nbins = 0;
    BfBinPlan plan{};
    // no buffer holds a batch the encode cannot take: every rank sizes the all-gather from the
    // largest batch of all ranks, so all of them learn it here together (and fall back alike)
    if (h->engine != BF_ENGINE_RUBY || !bf_sets_geometry(h->dev_bytes, h->bin_region_log2, &rl, &nbins) ||
        !sets_one_pass(h, n, rl, &plan))
        return BF_EINVAL;
    *bytes = bf_sets_capacity_bytes(h->dev_bytes, h->bin_region_log2, n, h->k);
    return *bytes ? BF_OK : BF_EINVAL;
}

namespace {
int encode_sets(bf_handle* h, const uint8_t* d_keys, const uint64_t* d_offsets, uint64_t n, bool dig,
                uint32_t* d_sets, uint64_t sets_bytes, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (!d_sets || (reinterpret_cast<uintptr_t>(d_sets) & 15u)) return set_err(h, BF_EINVAL, "d_sets must be 16-byte aligned");
    if (n && (!d_keys || (!dig && !d_offsets))) return set_err(h, BF_EINVAL, "NULL device pointer");
    if (dig && n && (reinterpret_cast<uintptr_t>(d_keys) & 15u)) return set_err(h, BF_EINVAL, "d_digests must be 16-byte aligned");
    if (h->shards > 1) return set_err(h, BF_EINVAL, "handle holds one shard of a partitioned filter");
    if (h->engine != BF_ENGINE_RUBY) return set_err(h, BF_EINVAL, "region sets carry the ruby driver's derivation only");
    uint32_t rl = 0, nbins = 0;
    if (!bf_sets_geometry(h->dev_bytes, h->bin_region_log2, &rl, &nbins))
        return set_err(h, BF_EINVAL, "this filter's regions cannot take region sets");
    const uint64_t need = bf_sets_capacity_bytes(h->dev_bytes, h->bin_region_log2, n, h->k);
    if (sets_bytes < need)
        return set_err(h, BF_EINVAL, "sets_bytes %llu < bf_region_sets_capacity %llu", (unsigned long long)sets_bytes,
                       (unsigned long long)need);
    BfBinPlan plan{};
    plan.region_log2 = rl;
    plan.nbins = nbins;
    if (!sets_one_pass(h, n, rl, &plan))
        return set_err(h, BF_EINVAL, "a batch of %llu keys does not sort in one pass (at most %llu keys per set buffer)",
                       (unsigned long long)n,
                       (unsigned long long)bf_binned_max_keys(h->k, h->dev_bytes, h->bin_region_log2));
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h, false)) return krc;   // (an encoder handle encodes: no bitset read)
    if (n) {
        int rc = ensure_scratch(h, plan.scratch_bytes);
        if (rc) return rc;
    }
    uint64_t bias = 0;
    const uint8_t* k16 = (n && !dig) ? align_keys(d_keys, &bias) : d_keys;
    BfMarks* mk = n ? prof_begin(h, so.s) : nullptr;
    // an encoder handle encodes beside another stream's apply: a persistent encode on 3/4 of the
    // CUs (bf_binned.hip sets_encode_persistent_kernel)
    uint32_t pgrid = 0;
    if (!h->g.bits) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || cus <= 0)
            cus = 256;
        pgrid = std::max<uint32_t>(1u, (uint32_t)cus * 3u / 4u);
    }
    HIPCHK(h, bf_launch_encode_sets(h->g, plan, h->dev_bytes, k16, d_offsets, bias, n, dig, h->d_bin_scratch, d_sets,
                                    std::min<uint64_t>(sets_bytes / 4, 0xFFFFFFFFull), so.s, mk, pgrid));
    return BF_OK;
}
}  // namespace

int bf_encode_region_sets_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                              uint32_t* d_sets, uint64_t sets_bytes, void* stream) {
    return encode_sets(h, d_key_bytes, d_offsets, n, false, d_sets, sets_bytes, stream);
}

int bf_encode_region_sets_digests_dev(bf_handle* h, const uint32_t* d_digests, uint64_t n, uint32_t* d_sets,
                                      uint64_t sets_bytes, void* stream) {
    return encode_sets(h, reinterpret_cast<const uint8_t*>(d_digests), nullptr, n, true, d_sets, sets_bytes, stream);
}

int bf_insert_region_sets_dev(bf_handle* h, const uint32_t* d_sets, uint64_t stride_bytes, uint32_t nsrc,
                              uint64_t probes_hint, uint32_t* d_any_new, uint32_t* d_status, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (nsrc == 0) return BF_OK;
    if (!d_sets || (reinterpret_cast<uintptr_t>(d_sets) & 15u) || (stride_bytes & 15u))
        return set_err(h, BF_EINVAL, "d_sets and stride_bytes must be 16-byte aligned");
    if (h->shards > 1) return set_err(h, BF_EINVAL, "handle holds one shard of a partitioned filter");
    // the sets hold offsets of the ruby driver's derivation: ORing them into an engine filter of
    // the same m and k would set bits its own derivation never probes
    if (h->engine != BF_ENGINE_RUBY) return set_err(h, BF_EINVAL, "region sets carry the ruby driver's derivation only");
    uint32_t rl = 0, nbins = 0;
    if (!bf_sets_geometry(h->dev_bytes, h->bin_region_log2, &rl, &nbins))
        return set_err(h, BF_EINVAL, "this filter's regions cannot take region sets");
    if (stride_bytes < 4 * bf_sets_header_words(nbins))   // the apply reads both per-region tables
        return set_err(h, BF_EINVAL, "stride_bytes below a set buffer's header and tables");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    BfMarks* mk = prof_begin(h, so.s);
    HIPCHK(h, bf_launch_insert_sets(h->g, h->dev_bytes, rl, nbins, d_sets, stride_bytes / 4, nsrc, probes_hint,
                                    d_any_new, d_status, so.s, mk));
    return BF_OK;
}

int bf_insert_encode_region_sets_dev(bf_handle* h, const uint32_t* d_sets, uint64_t stride_bytes, uint32_t nsrc,
                                     uint64_t probes_hint, uint32_t* d_any_new, uint32_t* d_status,
                                     const uint32_t* d_next_digests, uint64_t n_next, uint32_t* d_next_sets,
                                     uint64_t next_sets_bytes, void* stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (nsrc == 0)   // nothing to apply: the encode alone
        return encode_sets(h, reinterpret_cast<const uint8_t*>(d_next_digests), nullptr, n_next, true, d_next_sets,
                           next_sets_bytes, stream);
    if (!d_sets || (reinterpret_cast<uintptr_t>(d_sets) & 15u) || (stride_bytes & 15u))
        return set_err(h, BF_EINVAL, "d_sets and stride_bytes must be 16-byte aligned");
    if (!d_next_sets || (reinterpret_cast<uintptr_t>(d_next_sets) & 15u))
        return set_err(h, BF_EINVAL, "d_next_sets must be 16-byte aligned");
    if (n_next && (!d_next_digests || (reinterpret_cast<uintptr_t>(d_next_digests) & 15u)))
        return set_err(h, BF_EINVAL, "d_next_digests must be a 16-byte aligned device pointer");
    if (h->shards > 1) return set_err(h, BF_EINVAL, "handle holds one shard of a partitioned filter");
    if (h->engine != BF_ENGINE_RUBY) return set_err(h, BF_EINVAL, "region sets carry the ruby driver's derivation only");
    uint32_t rl = 0, nbins = 0;
    if (!bf_sets_geometry(h->dev_bytes, h->bin_region_log2, &rl, &nbins))
        return set_err(h, BF_EINVAL, "this filter's regions cannot take region sets");
    if (stride_bytes < 4 * bf_sets_header_words(nbins))
        return set_err(h, BF_EINVAL, "stride_bytes below a set buffer's header and tables");
    // the next batch's buffer is written while the sets are read: it must not be one of them
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(d_sets), a1 = a0 + (uint64_t)nsrc * stride_bytes;
    const uintptr_t b0 = reinterpret_cast<uintptr_t>(d_next_sets), b1 = b0 + next_sets_bytes;
    if (b0 < a1 && a0 < b1) return set_err(h, BF_EINVAL, "d_next_sets overlaps the set buffers being inserted");
    const uint64_t need = bf_sets_capacity_bytes(h->dev_bytes, h->bin_region_log2, n_next, h->k);
    if (next_sets_bytes < need)
        return set_err(h, BF_EINVAL, "next_sets_bytes %llu < bf_region_sets_capacity %llu",
                       (unsigned long long)next_sets_bytes, (unsigned long long)need);
    BfBinPlan plan{};
    plan.region_log2 = rl;
    plan.nbins = nbins;
    if (!sets_one_pass(h, n_next, rl, &plan))
        return set_err(h, BF_EINVAL, "a batch of %llu keys does not sort in one pass", (unsigned long long)n_next);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (!dg.ok) return set_err(h, BF_EDEVICE, "hipSetDevice(%d) failed", h->device);
    StreamOrder so(h, pick_stream(h, stream));
    if (int krc = op_check(h)) return krc;   // a bitset-less handle; an earlier call's bad key offsets
    if (n_next) {
        int rc = ensure_scratch(h, plan.scratch_bytes);
        if (rc) return rc;
    }
    BfMarks* mk = prof_begin(h, so.s);
    if (n_next == 0) {   // an empty next batch: its buffer is the header alone
        HIPCHK(h, bf_launch_encode_sets(h->g, plan, h->dev_bytes, nullptr, nullptr, 0, 0, true, h->d_bin_scratch,
                                        d_next_sets, std::min<uint64_t>(next_sets_bytes / 4, 0xFFFFFFFFull), so.s,
                                        nullptr));
        HIPCHK(h, bf_launch_insert_sets(h->g, h->dev_bytes, rl, nbins, d_sets, stride_bytes / 4, nsrc, probes_hint,
                                        d_any_new, d_status, so.s, mk));
        return BF_OK;
    }
    HIPCHK(h, bf_launch_insert_encode_sets(h->g, plan, h->dev_bytes, rl, nbins, d_sets, stride_bytes / 4, nsrc,
                                           probes_hint, d_any_new, d_status,
                                           reinterpret_cast<const uint8_t*>(d_next_digests), n_next, h->d_bin_scratch,
                                           d_next_sets, std::min<uint64_t>(next_sets_bytes / 4, 0xFFFFFFFFull), so.s,
                                           mk));
    return BF_OK;
}

int bf_stream(bf_handle* h, void** stream) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h || !stream) return BF_EINVAL;
    *stream = reinterpret_cast<void*>(h->stream);
    return BF_OK;
}

int bf_device_bits(bf_handle* h, void** d_bits, uint64_t* device_bytes) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    if (!h->g.bits) return set_err(h, BF_EINVAL, "an encoder handle (BF_FLAG_ENCODER) holds no bitset");
    if (d_bits) *d_bits = h->g.bits;
    if (device_bytes) *device_bytes = h->dev_bytes;
    return BF_OK;
}

int bf_profile(bf_handle* h, uint32_t enable) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    int rc = prof_harvest(h);
    h->profile = enable != 0;
    return rc;
}

int bf_profile_read(bf_handle* h, char* names, double* total_ms, uint64_t* launches, uint32_t cap,
                    uint32_t* n_out, uint32_t reset) {
    if (h && h->multi) return bfm_fail(h->multi, BF_EINVAL, "multi-device handle: use the host-pointer API");
    if (!h || !n_out) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    int rc = prof_harvest(h);
    if (rc) return rc;
    *n_out = (uint32_t)h->prof_acc.size();
    for (uint32_t i = 0; i < cap && i < h->prof_acc.size(); ++i) {
        const bf_handle::ProfAcc& a = h->prof_acc[i];
        if (names) snprintf(names + (size_t)i * BF_PROFILE_NAME_LEN, BF_PROFILE_NAME_LEN, "%s", a.name.c_str());
        if (total_ms) total_ms[i] = a.ms;
        if (launches) launches[i] = a.launches;
    }
    if (reset) h->prof_acc.clear();
    return BF_OK;
}

int bf_track_dirty(bf_handle* h, uint32_t enable) {
    if (h && h->multi) return bfm_track_dirty(h->multi, enable);
    if (!h) return BF_EINVAL;
    if (h->shards > 1) return set_err(h, BF_EINVAL, "dirty tracking needs a whole-filter handle");
    return bfi_track_dirty(h, enable);
}

}  // extern "C"

int bfi_track_dirty(bf_handle* h, uint32_t enable) {
    if (!h->g.bits) return set_err(h, BF_EINVAL, "an encoder handle (BF_FLAG_ENCODER) holds no bitset");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    HIPCHK(h, hipDeviceSynchronize());   // no launch may still use the map
    if (!enable) {
        if (h->d_dirty) (void)hipFree(h->d_dirty);
        h->d_dirty = nullptr;
        h->dirty_blocks = 0;
        h->g.dirty = nullptr;
        return BF_OK;
    }
    if (!h->d_dirty) {
        h->dirty_blocks = (h->dev_bytes + BF_DIRTY_BLOCK_BYTES - 1) / BF_DIRTY_BLOCK_BYTES;
        HIPCHK(h, hipMalloc((void**)&h->d_dirty, h->dirty_blocks));
    }
    HIPCHK(h, hipMemset(h->d_dirty, 0, h->dirty_blocks));
    h->g.dirty = h->d_dirty;
    return BF_OK;
}

// The changed byte ranges of the handle's own bytes (whole filter: the Redis string; shard:
// its local bytes), clipped to their trimmed length; clear forgets them.
int bfi_dirty_local(bf_handle* h, std::vector<uint64_t>* out, bool clear) {
    if (!h->d_dirty) return set_err(h, BF_EINVAL, "dirty tracking is off (bf_track_dirty)");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    HIPCHK(h, hipDeviceSynchronize());   // inserts may have run on any stream
    std::vector<uint8_t> map(h->dirty_blocks);
    HIPCHK(h, hipMemcpy(map.data(), h->d_dirty, h->dirty_blocks, hipMemcpyDeviceToHost));
    uint64_t len = 0;
    int rc = device_trimmed_len(h, &len);
    if (rc) return rc;
    out->clear();
    for (uint64_t b = 0; b < h->dirty_blocks;) {
        if (!map[b]) { ++b; continue; }
        uint64_t e = b;
        while (e < h->dirty_blocks && map[e]) ++e;
        const uint64_t off = b * BF_DIRTY_BLOCK_BYTES;
        const uint64_t end = std::min<uint64_t>(e * BF_DIRTY_BLOCK_BYTES, len);
        if (end > off) { out->push_back(off); out->push_back(end - off); }
        b = e;
    }
    if (clear) HIPCHK(h, hipMemset(h->d_dirty, 0, h->dirty_blocks));
    return BF_OK;
}

int bfi_trimmed_len(bf_handle* h, uint64_t* len) {
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    return device_trimmed_len(h, len);
}

int bfi_export_local(bf_handle* h, uint64_t offset, uint64_t len, uint8_t* buf) {
    if (offset > h->dev_bytes || len > h->dev_bytes - offset)
        return set_err(h, BF_ERANGE, "range [%llu, +%llu) outside the %llu-byte bitset", (unsigned long long)offset,
                       (unsigned long long)len, (unsigned long long)h->dev_bytes);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    if (h->order_valid) HIPCHK(h, hipEventSynchronize(h->order_ev));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (len) HIPCHK(h, hipMemcpy(buf, reinterpret_cast<const uint8_t*>(h->g.bits) + offset, len, hipMemcpyDeviceToHost));
    return BF_OK;
}

extern "C" {

int bf_dirty_ranges(bf_handle* h, uint64_t* ranges, uint32_t cap, uint32_t* n_out, uint64_t* redis_len,
                    uint32_t clear) {
    if (h && h->multi) return n_out ? bfm_dirty_ranges(h->multi, ranges, cap, n_out, redis_len, clear) : BF_EINVAL;
    if (!h || !n_out) return BF_EINVAL;
    if (!h->d_dirty) return set_err(h, BF_EINVAL, "dirty tracking is off (bf_track_dirty)");
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    HIPCHK(h, hipDeviceSynchronize());   // inserts may have run on any stream
    std::vector<uint8_t> map(h->dirty_blocks);
    HIPCHK(h, hipMemcpy(map.data(), h->d_dirty, h->dirty_blocks, hipMemcpyDeviceToHost));
    uint64_t len = 0;
    int rc = device_trimmed_len(h, &len);
    if (rc) return rc;
    if (redis_len) *redis_len = len;
    // adjacent dirty blocks coalesce; everything is clipped to the string's length, so
    // SETRANGE grows the key exactly as the SETBITs would have
    std::vector<uint64_t> out;
    for (uint64_t b = 0; b < h->dirty_blocks;) {
        if (!map[b]) { ++b; continue; }
        uint64_t e = b;
        while (e < h->dirty_blocks && map[e]) ++e;
        const uint64_t off = b * BF_DIRTY_BLOCK_BYTES;
        const uint64_t end = std::min<uint64_t>(e * BF_DIRTY_BLOCK_BYTES, len);
        if (end > off) { out.push_back(off); out.push_back(end - off); }
        b = e;
    }
    *n_out = (uint32_t)(out.size() / 2);
    if (ranges) {
        if (*n_out > cap) return set_err(h, BF_ERANGE, "%u dirty ranges, room for %u", *n_out, cap);
        memcpy(ranges, out.data(), out.size() * sizeof(uint64_t));
    }
    if (clear && (ranges || *n_out == 0)) HIPCHK(h, hipMemset(h->d_dirty, 0, h->dirty_blocks));
    return BF_OK;
}

int bf_export_range(bf_handle* h, uint64_t offset, uint64_t len, uint8_t* buf) {
    if (h && h->multi) return (len && !buf) ? BF_EINVAL : bfm_export_range(h->multi, offset, len, buf);
    if (!h || (len && !buf)) return BF_EINVAL;
    if (h->shards > 1) return set_err(h, BF_EINVAL, "partitioned shard: use bf_shard_export");
    if (!h->g.bits) return set_err(h, BF_EINVAL, "an encoder handle (BF_FLAG_ENCODER) holds no bitset");
    if (offset > h->dev_bytes || len > h->dev_bytes - offset)
        return set_err(h, BF_ERANGE, "range [%llu, +%llu) outside the %llu-byte bitset", (unsigned long long)offset,
                       (unsigned long long)len, (unsigned long long)h->dev_bytes);
    std::lock_guard<std::mutex> lk(h->mu);
    DeviceGuard dg(h->device);
    HIPCHK(h, hipDeviceSynchronize());
    if (len) HIPCHK(h, hipMemcpy(buf, reinterpret_cast<const uint8_t*>(h->g.bits) + offset, len,
                                 hipMemcpyDeviceToHost));
    return BF_OK;
}

int bf_insert_plan(const bf_handle* h, uint64_t n, uint32_t* binned, uint64_t* scratch_bytes) {
    if (h && h->multi) return bfm_insert_plan(h->multi, n, binned, scratch_bytes);
    if (!h) return BF_EINVAL;
    BfBinPlan plan{};
    const bool b = n > 0 && use_binned(h, n, false, &plan);
    if (binned) *binned = b ? 1u : 0u;
    if (scratch_bytes) *scratch_bytes = b ? plan.scratch_bytes : 0;
    return BF_OK;
}

}  // extern "C"
