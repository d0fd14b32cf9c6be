// bf_multi.cpp — multi-device handles: one process, several GPUs behind one bf_handle
// (bf_config.device_count / devices / mode; include/bfhip.h).  This is what the Ruby
// driver's `devices:` option reaches (Redis::Bloomfilter.new(driver: 'hip', devices: 8),
// lib/redis/bloomfilter.rb:43-45), so one Ruby process drives a whole node.
//
// A multi-device handle owns one per-device bf_handle per slot and composes them through
// the ABI's own entry points:
//   BF_MODE_REPLICATED   whole-filter handles; inserts go to every device (one host thread
//                        per device), include? batches are split over the devices.
//   BF_MODE_PARTITIONED  shard handles (shard_count = devices, block-cyclic ownership):
//                        each device routes its part of a batch into per-owner windows
//                        (bf_route_windows_dev), the owners pull their windows with peer
//                        copies over xGMI (hipMemcpyPeerAsync on the owner's stream), OR
//                        them in (bf_shard_insert_hi_dev) or test them
//                        (bf_shard_test_hi_dev), and include? answers go back by peer copy
//                        into the requester's window layout for bf_combine_windows_dev.
// Everything runs within one process, so the exchange needs no collective library: a
// device-to-device copy over xGMI is the all-to-all's send/recv.
#include "bf_multi.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>

namespace {

constexpr uint64_t kPartKeys = 1ull << 22;   // keys per device per round of a partitioned call

struct DevScratch {
    hipStream_t s = nullptr;
    uint8_t* keys = nullptr;
    uint64_t keys_cap = 0;
    uint64_t* offs = nullptr;
    uint64_t offs_cap = 0;
    uint32_t* send = nullptr;
    uint32_t* slot = nullptr;
    uint64_t send_cap = 0;   // entries of send and slot
    uint64_t* counts = nullptr;
    uint32_t* recv = nullptr;
    uint64_t recv_cap = 0;   // entries
    uint8_t* bits = nullptr;   // owner answers, receive layout
    uint64_t bits_cap = 0;
    uint8_t* back = nullptr;   // requester answers, window layout
    uint64_t back_cap = 0;
    uint8_t* out = nullptr;
    uint64_t out_cap = 0;
    uint32_t* flag = nullptr;
    hipEvent_t ev = nullptr;
    // per round (host)
    uint64_t a = 0, n = 0, cap = 0;
    std::vector<uint64_t> rel;   // relative offsets (kept alive until the copies finish)
    std::vector<uint64_t> cnt;   // window counts
};

}  // namespace

struct BfMulti {
    uint32_t mode = BF_MODE_REPLICATED;
    uint32_t D = 0;
    std::vector<int> dev;
    std::vector<bf_handle*> sub;
    std::vector<DevScratch> ds;
    uint64_t m = 0, reach = 0, local_max = 0;
    uint32_t k = 0, block_log2 = 20, nh = 1;
    bool tracking = false;
    std::mutex mu;
    std::string err;
};

namespace {

int fail(BfMulti* mh, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(BfMulti* mh, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    mh->err = buf;
    return code;
}

// A sub-handle's failure, with its message, as the multi-device handle's.
int sub_rc(BfMulti* mh, uint32_t d, int rc) {
    if (rc != BF_OK) fail(mh, rc, "device slot %u (HIP device %d): %s", d, mh->dev[d], bf_last_error(mh->sub[d]));
    return rc;
}

#define MCHK(mh, expr)                                                                          \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail((mh), e_ == hipErrorOutOfMemory ? BF_ENOMEM : BF_EDEVICE, "%s failed: %s", #expr, \
                        hipGetErrorString(e_));                                                 \
    } while (0)

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <typename T>
int grow(BfMulti* mh, T** p, uint64_t* cap, uint64_t need) {
    if (need <= *cap) return BF_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const uint64_t c = std::max<uint64_t>(need + need / 4, 1024);
    MCHK(mh, hipMalloc((void**)p, c * sizeof(T)));
    *cap = c;
    return BF_OK;
}

// Runs f(d) for every device slot on its own host thread; the first failure wins.
template <typename F>
int each_device(BfMulti* mh, F&& f) {
    std::vector<int> rc(mh->D, BF_OK);
    std::vector<std::thread> th;
    for (uint32_t d = 1; d < mh->D; ++d) th.emplace_back([&, d] { rc[d] = f(d); });
    rc[0] = f(0);
    for (std::thread& t : th) t.join();
    for (uint32_t d = 0; d < mh->D; ++d)
        if (rc[d] != BF_OK) return sub_rc(mh, d, rc[d]);
    return BF_OK;
}

uint64_t bb_of(const BfMulti* mh) { return (1ull << mh->block_log2) / 8; }

// Local byte lb of shard s -> its byte in the Redis string.
uint64_t global_byte(const BfMulti* mh, uint32_t s, uint64_t lb) {
    const uint64_t bb = bb_of(mh);
    return ((lb / bb) * mh->D + s) * bb + lb % bb;
}

// Trimmed Redis length of a partitioned filter: the largest global position of any shard's
// last nonzero byte, + 1.
int partitioned_len(BfMulti* mh, uint64_t* len) {
    uint64_t best = 0;
    for (uint32_t s = 0; s < mh->D; ++s) {
        uint64_t ll = 0;
        int rc = bfi_trimmed_len(mh->sub[s], &ll);
        if (rc) return sub_rc(mh, s, rc);
        if (ll) best = std::max(best, global_byte(mh, s, ll - 1) + 1);
    }
    *len = best;
    return BF_OK;
}

// ---- partitioned batches ------------------------------------------------------------

// Window capacity for a device's part of nd keys: 1/D of its probes + 12.5 % + slack per
// window (the block-cyclic map spreads them evenly); a skewed part overflows and is routed
// again with nd*k, which always fits.
uint64_t window_cap(const BfMulti* mh, uint64_t nd) {
    const uint64_t probes = nd * mh->k;
    return std::max<uint64_t>(1, std::min<uint64_t>(probes, probes / mh->D + probes / (8ull * mh->D) + 4096));
}

}  // namespace

// The per-slot words every round may touch whatever its part's size: the window counts and
// the owner's any_new flag.  Allocated on the slot's own device, for every slot — an owner
// whose own part is empty still ORs other devices' windows and reports any_new.
static int ensure_small(BfMulti* mh, uint32_t d) {
    DevScratch& x = mh->ds[d];
    if (x.counts && x.flag) return BF_OK;
    DevGuard g(mh->dev[d]);
    if (!x.counts) MCHK(mh, hipMalloc((void**)&x.counts, 256 * sizeof(uint64_t)));
    if (!x.flag) MCHK(mh, hipMalloc((void**)&x.flag, 256));
    return BF_OK;
}

// Allocations of one device's round (keys, offsets, windows).
static int prepare_round(BfMulti* mh, uint32_t d, const uint8_t* keys, const uint64_t* offsets, bool want_slot) {
    DevScratch& x = mh->ds[d];
    DevGuard g(mh->dev[d]);
    const uint32_t nwin = mh->D * mh->nh;
    const uint64_t base = offsets[x.a];
    const uint64_t bytes = offsets[x.a + x.n] - base;
    int rc;
    if ((rc = grow(mh, &x.keys, &x.keys_cap, bytes + 16))) return rc;
    if ((rc = grow(mh, &x.offs, &x.offs_cap, x.n + 1))) return rc;
    uint64_t scap = x.send_cap;
    if (nwin * x.cap > scap) {
        if (x.slot) (void)hipFree(x.slot);
        x.slot = nullptr;
        if ((rc = grow(mh, &x.send, &x.send_cap, nwin * x.cap))) return rc;
        MCHK(mh, hipMalloc((void**)&x.slot, x.send_cap * sizeof(uint32_t)));
    }
    x.rel.resize(x.n + 1);
    for (uint64_t j = 0; j <= x.n; ++j) x.rel[j] = offsets[x.a + j] - base;
    x.cnt.assign(nwin, 0);
    if (bytes) MCHK(mh, hipMemcpyAsync(x.keys, keys + base, bytes, hipMemcpyHostToDevice, x.s));
    MCHK(mh, hipMemsetAsync(x.keys + bytes, 0, 16, x.s));
    MCHK(mh, hipMemcpyAsync(x.offs, x.rel.data(), (x.n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, x.s));
    (void)want_slot;
    return BF_OK;
}

// Enqueue the hash + route of device d's part into its windows and the window counts' trip
// to the host (route_wait collects them), so every device routes at the same time.
static int route_enqueue(BfMulti* mh, uint32_t d, bool want_slot) {
    DevScratch& x = mh->ds[d];
    DevGuard g(mh->dev[d]);
    const uint32_t nwin = mh->D * mh->nh;
    int rc = bf_route_windows_dev(mh->sub[d], x.keys, x.offs, x.n, x.send, want_slot ? x.slot : nullptr, x.cap,
                                  x.counts, x.s);
    if (rc) return sub_rc(mh, d, rc);
    MCHK(mh, hipMemcpyAsync(x.cnt.data(), x.counts, nwin * sizeof(uint64_t), hipMemcpyDeviceToHost, x.s));
    return BF_OK;
}

static int route_wait(BfMulti* mh, uint32_t d) {
    DevGuard g(mh->dev[d]);
    MCHK(mh, hipStreamSynchronize(mh->ds[d].s));
    return BF_OK;
}

// One round of a partitioned insert (want_bits = false) or include? over the device parts
// set up in mh->ds[*].{a, n}.
static int partitioned_round(BfMulti* mh, const uint8_t* keys, const uint64_t* offsets, bool include, uint8_t* out,
                             bool* any_new) {
    const uint32_t D = mh->D, nh = mh->nh, nwin = D * nh;
    int rc;
    for (uint32_t d = 0; d < D; ++d)
        if ((rc = ensure_small(mh, d))) return rc;
    for (uint32_t d = 0; d < D; ++d) {   // every device's route in flight at once
        DevScratch& x = mh->ds[d];
        x.cap = window_cap(mh, x.n);
        if (x.n == 0) {
            x.cnt.assign(nwin, 0);
            continue;
        }
        if ((rc = prepare_round(mh, d, keys, offsets, include))) return rc;
        if ((rc = route_enqueue(mh, d, include))) return rc;
    }
    for (uint32_t d = 0; d < D; ++d) {
        DevScratch& x = mh->ds[d];
        if (x.n == 0) continue;
        if ((rc = route_wait(mh, d))) return rc;
        const uint64_t mx = *std::max_element(x.cnt.begin(), x.cnt.end());
        if (mx > x.cap) {   // a skewed part: windows that always fit
            x.cap = std::max<uint64_t>(x.n * mh->k, 1);
            if ((rc = prepare_round(mh, d, keys, offsets, include))) return rc;
            if ((rc = route_enqueue(mh, d, include))) return rc;
            if ((rc = route_wait(mh, d))) return rc;
        }
    }
    // each requester's answer windows, on the requester's own device, before any owner
    // pushes into them (a grow inside the owner loop would allocate on the owner's device)
    if (include)
        for (uint32_t d = 0; d < D; ++d) {
            DevScratch& x = mh->ds[d];
            if (!x.n) continue;
            DevGuard g(mh->dev[d]);
            if ((rc = grow(mh, &x.back, &x.back_cap, (uint64_t)nwin * x.cap))) return rc;
        }
    // owners pull their windows (sub-range major, then source), apply or test them, and
    // (include?) push the answers back into each requester's window layout
    for (uint32_t o = 0; o < D; ++o) {
        DevScratch& y = mh->ds[o];
        DevGuard g(mh->dev[o]);
        uint64_t total = 0;
        for (uint32_t d = 0; d < D; ++d)
            for (uint32_t h = 0; h < nh; ++h) total += mh->ds[d].cnt[o * nh + h];
        if ((rc = grow(mh, &y.recv, &y.recv_cap, std::max<uint64_t>(total, 1)))) return rc;
        if (include && (rc = grow(mh, &y.bits, &y.bits_cap, std::max<uint64_t>(total, 1)))) return rc;
        if (!include && any_new) MCHK(mh, hipMemsetAsync(y.flag, 0, sizeof(uint32_t), y.s));
        uint64_t at = 0;
        for (uint32_t h = 0; h < nh; ++h) {
            const uint64_t h0 = at;
            for (uint32_t d = 0; d < D; ++d) {
                const DevScratch& x = mh->ds[d];
                const uint64_t c = x.cnt[o * nh + h];
                if (!c) continue;
                MCHK(mh, hipMemcpyPeerAsync(y.recv + at, mh->dev[o], x.send + (uint64_t)(o * nh + h) * x.cap,
                                            mh->dev[d], c * sizeof(uint32_t), y.s));
                at += c;
            }
            if (at == h0) continue;
            if (!include) {
                rc = bf_shard_insert_hi_dev(mh->sub[o], y.recv + h0, at - h0, h, any_new ? y.flag : nullptr, y.s);
                if (rc) return sub_rc(mh, o, rc);
            } else {
                rc = bf_shard_test_hi_dev(mh->sub[o], y.recv + h0, at - h0, h, y.bits + h0, y.s);
                if (rc) return sub_rc(mh, o, rc);
                uint64_t bt = h0;
                for (uint32_t d = 0; d < D; ++d) {
                    DevScratch& x = mh->ds[d];
                    const uint64_t c = x.cnt[o * nh + h];
                    if (!c) continue;
                    MCHK(mh, hipMemcpyPeerAsync(x.back + (uint64_t)(o * nh + h) * x.cap, mh->dev[d], y.bits + bt,
                                                mh->dev[o], c, y.s));
                    bt += c;
                }
            }
        }
        MCHK(mh, hipEventRecord(y.ev, y.s));
    }
    if (!include) {
        for (uint32_t o = 0; o < D; ++o) {
            DevGuard g(mh->dev[o]);
            MCHK(mh, hipStreamSynchronize(mh->ds[o].s));
            if (any_new) {
                uint32_t f = 0;
                MCHK(mh, hipMemcpy(&f, mh->ds[o].flag, sizeof f, hipMemcpyDeviceToHost));
                if (f) *any_new = true;
            }
        }
        return BF_OK;
    }
    // requesters: wait for every owner's answers, AND them per key, copy out
    for (uint32_t d = 0; d < D; ++d) {
        DevScratch& x = mh->ds[d];
        if (!x.n) continue;
        DevGuard g(mh->dev[d]);
        for (uint32_t o = 0; o < D; ++o) MCHK(mh, hipStreamWaitEvent(x.s, mh->ds[o].ev, 0));
        if ((rc = grow(mh, &x.out, &x.out_cap, x.n))) return rc;
        rc = bf_combine_windows_dev(mh->sub[d], x.back, x.slot, x.cap, nwin, x.counts, x.n, x.out, x.s);
        if (rc) return sub_rc(mh, d, rc);
        MCHK(mh, hipMemcpyAsync(out + x.a, x.out, x.n, hipMemcpyDeviceToHost, x.s));
    }
    for (uint32_t d = 0; d < D; ++d) {
        DevGuard g(mh->dev[d]);
        MCHK(mh, hipStreamSynchronize(mh->ds[d].s));
    }
    return BF_OK;
}

static int partitioned_batch(BfMulti* mh, const uint8_t* keys, const uint64_t* offsets, uint64_t n, bool include,
                             uint8_t* out, bool* any_new) {
    for (uint64_t j = 0; j < n; ++j)
        if (offsets[j + 1] < offsets[j])
            return fail(mh, BF_EINVAL, "offsets must be non-decreasing (j=%llu)", (unsigned long long)j);
    const uint64_t per_round = kPartKeys * mh->D;
    for (uint64_t r0 = 0; r0 < n; r0 += per_round) {
        const uint64_t rn = std::min(per_round, n - r0);
        for (uint32_t d = 0; d < mh->D; ++d) {   // contiguous, near-equal parts
            mh->ds[d].a = r0 + rn * d / mh->D;
            mh->ds[d].n = r0 + rn * (d + 1) / mh->D - mh->ds[d].a;
        }
        int rc = partitioned_round(mh, keys, offsets, include, out, any_new);
        if (rc) return rc;
    }
    return BF_OK;
}

// ---- lifecycle ------------------------------------------------------------------------

int bfm_create(uint64_t m_bits, uint32_t k, const bf_config& cfg, BfMulti** out, std::string* err) {
    *out = nullptr;
    if (cfg.device_count == 0 || cfg.device_count > BF_MAX_DEVICES) {
        *err = "device_count must be in [1, BF_MAX_DEVICES]";
        return BF_EINVAL;
    }
    if (cfg.mode != BF_MODE_REPLICATED && cfg.mode != BF_MODE_PARTITIONED) {
        *err = "mode must be BF_MODE_REPLICATED or BF_MODE_PARTITIONED";
        return BF_EINVAL;
    }
    if (cfg.shard_count > 1) {
        *err = "a multi-device handle holds the whole filter (shard_count must be 0 or 1)";
        return BF_EINVAL;
    }
    if (cfg.mode == BF_MODE_PARTITIONED && (cfg.flags & (BF_FLAG_ENGINE_MD5 | BF_FLAG_ENGINE_SHA1))) {
        *err = "the RubyTest hash engines need a replicated (whole-filter) layout";
        return BF_EINVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        *err = "no HIP device available";
        return BF_EDEVICE;
    }
    BfMulti* mh = new (std::nothrow) BfMulti();
    if (!mh) {
        *err = "host allocation failed";
        return BF_ENOMEM;
    }
    mh->mode = cfg.mode;
    mh->D = cfg.device_count;
    mh->m = m_bits;
    mh->k = k;
    mh->block_log2 = cfg.shard_block_log2 ? cfg.shard_block_log2 : 20;
    mh->dev.assign(cfg.devices, cfg.devices + mh->D);
    auto bail = [&](int code, const std::string& msg) {
        *err = msg;
        bfm_destroy(mh);
        return code;
    };
    // validate every ordinal before any HIP call names one (hipSetDevice on a bad ordinal
    // would leave a sticky error on this thread)
    for (uint32_t d = 0; d < mh->D; ++d)
        if (mh->dev[d] < 0 || mh->dev[d] >= ndev)
            return bail(BF_EINVAL, "devices[" + std::to_string(d) + "] = " + std::to_string(mh->dev[d]) +
                                       " out of range (" + std::to_string(ndev) + " devices)");
    mh->ds.resize(mh->D);
    // peer access between distinct devices (xGMI); a repeated device needs none
    for (uint32_t a = 0; a < mh->D; ++a)
        for (uint32_t b = 0; b < mh->D; ++b) {
            if (mh->dev[a] == mh->dev[b]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, mh->dev[a], mh->dev[b]) == hipSuccess && can) {
                DevGuard g(mh->dev[a]);
                const hipError_t e = hipDeviceEnablePeerAccess(mh->dev[b], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
            }
        }
    for (uint32_t d = 0; d < mh->D; ++d) {
        bf_config c = cfg;
        c.struct_size = sizeof(bf_config);
        c.device = mh->dev[d];
        c.device_count = 0;
        if (mh->mode == BF_MODE_PARTITIONED && mh->D > 1) {
            c.shard_count = mh->D;
            c.shard_index = d;
            c.shard_block_log2 = mh->block_log2;
            c.flags &= ~BF_FLAG_ROUTE32;   // the window route carries uint32 entries anyway
        } else {
            c.shard_count = 0;
            c.shard_index = 0;
        }
        bf_handle* h = nullptr;
        const int rc = bf_create(m_bits, k, &c, &h);
        if (rc) return bail(rc, std::string("device slot ") + std::to_string(d) + ": " + bf_last_error(nullptr));
        mh->sub.push_back(h);
        DevGuard g(mh->dev[d]);
        if (hipStreamCreateWithFlags(&mh->ds[d].s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&mh->ds[d].ev, hipEventDisableTiming) != hipSuccess)
            return bail(BF_EDEVICE, "stream / event creation failed");
    }
    uint64_t reach = 0;
    (void)bf_info(mh->sub[0], nullptr, nullptr, &reach, nullptr);
    mh->reach = mh->mode == BF_MODE_PARTITIONED ? std::min<uint64_t>(m_bits, (uint64_t)k * 0xFFFFFFFFull + 1) : reach;
    if (mh->mode == BF_MODE_PARTITIONED && mh->D > 1) {
        uint32_t nh = 1;
        (void)bf_route_window_split(mh->sub[0], &nh);
        mh->nh = nh;
        if (mh->D * nh > 256) return bail(BF_EINVAL, "devices x 2^32-bit sub-ranges exceed 256 route windows");
    }
    *out = mh;
    return BF_OK;
}

void bfm_destroy(BfMulti* mh) {
    if (!mh) return;
    for (uint32_t d = 0; d < mh->ds.size(); ++d) {
        DevScratch& x = mh->ds[d];
        if (!x.s) continue;   // nothing was created on this slot
        DevGuard g(mh->dev[d]);
        if (x.s) (void)hipStreamSynchronize(x.s);
        for (void* p : {(void*)x.keys, (void*)x.offs, (void*)x.send, (void*)x.slot, (void*)x.counts, (void*)x.recv,
                        (void*)x.bits, (void*)x.back, (void*)x.out, (void*)x.flag})
            if (p) (void)hipFree(p);
        if (x.ev) (void)hipEventDestroy(x.ev);
        if (x.s) (void)hipStreamDestroy(x.s);
    }
    for (bf_handle* h : mh->sub) bf_destroy(h);
    delete mh;
}

const char* bfm_last_error(const BfMulti* mh) { return mh->err.c_str(); }

int bfm_fail(BfMulti* mh, int code, const char* msg) { return fail(mh, code, "%s", msg); }

int bfm_info(const BfMulti* mh, uint64_t* m_bits, uint32_t* k, uint64_t* reach_bits, uint64_t* device_bytes) {
    if (m_bits) *m_bits = mh->m;
    if (k) *k = mh->k;
    if (reach_bits) *reach_bits = mh->reach;
    if (device_bytes) {   // summed over the devices
        uint64_t tot = 0;
        for (bf_handle* h : mh->sub) {
            uint64_t b = 0;
            (void)bf_info(h, nullptr, nullptr, nullptr, &b);
            tot += b;
        }
        *device_bytes = tot;
    }
    return BF_OK;
}

int bfm_shard_info(const BfMulti* mh, uint32_t* shard_count, uint32_t* shard_index, uint32_t* block_log2,
                   uint64_t* local_bits) {
    const bool part = mh->mode == BF_MODE_PARTITIONED && mh->D > 1;
    if (shard_count) *shard_count = part ? mh->D : 1;
    if (shard_index) *shard_index = 0;
    if (block_log2) *block_log2 = mh->block_log2;
    if (local_bits) *local_bits = mh->reach;
    return BF_OK;
}

// ---- batches --------------------------------------------------------------------------

int bfm_insert_many(BfMulti* mh, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* any_new,
                    uint8_t* per_key_new) {
    std::lock_guard<std::mutex> lk(mh->mu);
    if (any_new) *any_new = 0;
    if (n && !offsets) return fail(mh, BF_EINVAL, "offsets is NULL");
    if (mh->mode == BF_MODE_REPLICATED || mh->D == 1) {
        // every replica takes the whole batch; the flags are identical across replicas
        std::vector<uint8_t> flags(mh->D, 0);
        int rc = each_device(mh, [&](uint32_t d) {
            return bf_insert_many(mh->sub[d], keys, offsets, n, any_new ? &flags[d] : nullptr,
                                  d == 0 ? per_key_new : nullptr);
        });
        if (rc) return rc;
        if (any_new) *any_new = flags[0];
        return BF_OK;
    }
    if (per_key_new) return fail(mh, BF_EINVAL, "per_key_new needs a single-device or BF_MODE_REPLICATED handle");
    if (n == 0) return BF_OK;
    bool anyn = false;
    int rc = partitioned_batch(mh, keys, offsets, n, false, nullptr, any_new ? &anyn : nullptr);
    if (rc) return rc;
    if (any_new) *any_new = anyn ? 1 : 0;
    return BF_OK;
}

int bfm_include_many(BfMulti* mh, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* out) {
    std::lock_guard<std::mutex> lk(mh->mu);
    if (n && (!offsets || !out)) return fail(mh, BF_EINVAL, "NULL pointer");
    if (n == 0) return BF_OK;
    if (mh->mode == BF_MODE_REPLICATED || mh->D == 1) {
        // include? is read-only: each replica answers a contiguous part of the batch
        return each_device(mh, [&](uint32_t d) {
            const uint64_t a = n * d / mh->D, b = n * (d + 1) / mh->D;
            return b > a ? bf_include_many(mh->sub[d], keys, offsets + a, b - a, out + a) : BF_OK;
        });
    }
    return partitioned_batch(mh, keys, offsets, n, true, out, nullptr);
}

int bfm_indexes_many(BfMulti* mh, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint64_t* out) {
    std::lock_guard<std::mutex> lk(mh->mu);
    return sub_rc(mh, 0, bf_indexes_many(mh->sub[0], keys, offsets, n, out));
}

int bfm_clear(BfMulti* mh) {
    std::lock_guard<std::mutex> lk(mh->mu);
    return each_device(mh, [&](uint32_t d) { return bf_clear(mh->sub[d]); });
}

int bfm_sync(BfMulti* mh) {
    std::lock_guard<std::mutex> lk(mh->mu);
    return each_device(mh, [&](uint32_t d) { return bf_sync(mh->sub[d]); });
}

int bfm_insert_plan(const BfMulti* mh, uint64_t n, uint32_t* binned, uint64_t* scratch_bytes) {
    return bf_insert_plan(mh->sub[0], n, binned, scratch_bytes);
}

// ---- Redis string -----------------------------------------------------------------------

int bfm_export_redis(BfMulti* mh, uint8_t* buf, uint64_t cap, uint64_t* len_out) {
    std::lock_guard<std::mutex> lk(mh->mu);
    if (mh->mode == BF_MODE_REPLICATED || mh->D == 1)
        return sub_rc(mh, 0, bf_export_redis(mh->sub[0], buf, cap, len_out));
    uint64_t len = 0;
    int rc = partitioned_len(mh, &len);
    if (rc) return rc;
    *len_out = len;
    if (!buf) return BF_OK;
    if (cap < len) return fail(mh, BF_ERANGE, "export buffer too small: need %llu bytes", (unsigned long long)len);
    // each shard's local bytes in chunks of whole ownership blocks, scattered into place
    const uint64_t bb = bb_of(mh);
    const uint64_t chunk_blocks = std::max<uint64_t>(1, (256ull << 20) / bb);
    std::vector<uint8_t> tmp(chunk_blocks * bb);
    for (uint32_t s = 0; s < mh->D; ++s) {
        uint64_t local_bits = 0;
        (void)bf_shard_info(mh->sub[s], nullptr, nullptr, nullptr, &local_bits);
        const uint64_t lbytes = (local_bits + 7) / 8;
        for (uint64_t j0 = 0; j0 * bb < lbytes; j0 += chunk_blocks) {
            const uint64_t first = (j0 * mh->D + s) * bb;
            if (first >= len) break;
            const uint64_t lo = j0 * bb, ln = std::min(chunk_blocks * bb, lbytes - lo);
            if ((rc = bfi_export_local(mh->sub[s], lo, ln, tmp.data()))) return sub_rc(mh, s, rc);
            for (uint64_t j = 0; j * bb < ln; ++j) {
                const uint64_t off = ((j0 + j) * mh->D + s) * bb;
                if (off >= len) break;
                memcpy(buf + off, tmp.data() + j * bb, std::min({bb, len - off, ln - j * bb}));
            }
        }
    }
    return BF_OK;
}

int bfm_import_redis(BfMulti* mh, const uint8_t* buf, uint64_t len, uint32_t mode) {
    std::lock_guard<std::mutex> lk(mh->mu);
    if (mh->mode == BF_MODE_REPLICATED || mh->D == 1)
        return each_device(mh, [&](uint32_t d) { return bf_import_redis(mh->sub[d], buf, len, mode); });
    if (len && !buf) return fail(mh, BF_EINVAL, "buf is NULL");
    const uint64_t max_bytes = (mh->reach + 7) / 8;
    if (len > max_bytes)
        return fail(mh, BF_ERANGE, "string of %llu bytes exceeds the filter's %llu reachable bytes",
                    (unsigned long long)len, (unsigned long long)max_bytes);
    if (len == max_bytes && (mh->reach & 7) && (buf[len - 1] & (uint8_t)(0xFFu >> (mh->reach & 7))))
        return fail(mh, BF_ERANGE, "string sets bits at offsets >= %llu", (unsigned long long)mh->reach);
    const uint64_t bb = bb_of(mh);
    return each_device(mh, [&](uint32_t s) {
        uint64_t local_bits = 0;
        (void)bf_shard_info(mh->sub[s], nullptr, nullptr, nullptr, &local_bits);
        std::vector<uint8_t> loc((local_bits + 7) / 8, 0);
        for (uint64_t j = 0; j * bb < loc.size(); ++j) {
            const uint64_t off = (j * mh->D + s) * bb;
            if (off >= len) break;
            memcpy(loc.data() + j * bb, buf + off, std::min({bb, len - off, (uint64_t)loc.size() - j * bb}));
        }
        return bf_shard_import(mh->sub[s], loc.data(), loc.size(), mode);
    });
}

int bfm_track_dirty(BfMulti* mh, uint32_t enable) {
    std::lock_guard<std::mutex> lk(mh->mu);
    mh->tracking = enable != 0;
    if (mh->mode == BF_MODE_REPLICATED || mh->D == 1)   // every replica takes the same inserts
        return sub_rc(mh, 0, bf_track_dirty(mh->sub[0], enable));
    for (uint32_t s = 0; s < mh->D; ++s) {
        const int rc = bfi_track_dirty(mh->sub[s], enable);
        if (rc) return sub_rc(mh, s, rc);
    }
    return BF_OK;
}

int bfm_dirty_ranges(BfMulti* mh, uint64_t* ranges, uint32_t cap, uint32_t* n_out, uint64_t* redis_len,
                     uint32_t clear) {
    std::lock_guard<std::mutex> lk(mh->mu);
    if (mh->mode == BF_MODE_REPLICATED || mh->D == 1)
        return sub_rc(mh, 0, bf_dirty_ranges(mh->sub[0], ranges, cap, n_out, redis_len, clear));
    if (!mh->tracking) return fail(mh, BF_EINVAL, "dirty tracking is off (bf_track_dirty)");
    uint64_t len = 0;
    int rc = partitioned_len(mh, &len);
    if (rc) return rc;
    if (redis_len) *redis_len = len;
    // local ranges of every shard -> string ranges (split at ownership blocks), merged
    const uint64_t bb = bb_of(mh);
    std::vector<std::pair<uint64_t, uint64_t>> g;   // [start, end)
    const bool forget = clear && ranges;
    for (uint32_t s = 0; s < mh->D; ++s) {
        std::vector<uint64_t> loc;
        if ((rc = bfi_dirty_local(mh->sub[s], &loc, false))) return sub_rc(mh, s, rc);
        for (size_t i = 0; i + 1 < loc.size(); i += 2)
            for (uint64_t lo = loc[i], end = loc[i] + loc[i + 1]; lo < end;) {
                const uint64_t stop = std::min(end, (lo / bb + 1) * bb);
                const uint64_t a = global_byte(mh, s, lo);
                const uint64_t b = std::min(a + (stop - lo), len);
                if (b > a) g.emplace_back(a, b);
                lo = stop;
            }
    }
    std::sort(g.begin(), g.end());
    std::vector<uint64_t> outv;
    for (const auto& r : g) {
        if (!outv.empty() && outv[outv.size() - 2] + outv.back() >= r.first) {
            const uint64_t st = outv[outv.size() - 2];
            outv.back() = std::max(outv.back(), r.second - st);
        } else {
            outv.push_back(r.first);
            outv.push_back(r.second - r.first);
        }
    }
    *n_out = (uint32_t)(outv.size() / 2);
    if (ranges) {
        if (*n_out > cap) return fail(mh, BF_ERANGE, "%u dirty ranges, room for %u", *n_out, cap);
        memcpy(ranges, outv.data(), outv.size() * sizeof(uint64_t));
    }
    if (forget || (clear && *n_out == 0))
        for (uint32_t s = 0; s < mh->D; ++s) {
            std::vector<uint64_t> drop;
            if ((rc = bfi_dirty_local(mh->sub[s], &drop, true))) return sub_rc(mh, s, rc);
        }
    return BF_OK;
}

int bfm_export_range(BfMulti* mh, uint64_t offset, uint64_t len, uint8_t* buf) {
    std::lock_guard<std::mutex> lk(mh->mu);
    if (mh->mode == BF_MODE_REPLICATED || mh->D == 1) return sub_rc(mh, 0, bf_export_range(mh->sub[0], offset, len, buf));
    const uint64_t bb = bb_of(mh);
    for (uint64_t at = offset, end = offset + len; at < end;) {
        const uint64_t gblk = at / bb;
        const uint32_t s = (uint32_t)(gblk % mh->D);
        const uint64_t lo = (gblk / mh->D) * bb + at % bb;
        const uint64_t n = std::min(end, (gblk + 1) * bb) - at;
        const int rc = bfi_export_local(mh->sub[s], lo, n, buf + (at - offset));
        if (rc) return sub_rc(mh, s, rc);
        at += n;
    }
    return BF_OK;
}
