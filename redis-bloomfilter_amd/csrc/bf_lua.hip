// bf_lua.hip — the Lua driver's scalable filter on the device
// (lib/bloomfilter_driver/lua.rb, vendor/assets/lua/add.lua, check.lua).
//
// State, as in Redis: a count (KEYS[1]:count) and layers KEYS[1]:1 .. :N, each a
// SETBIT-layout bitstring of bits_n bits.  Layer n has scale 2^(n-1) * entries,
// bits_n = floor(-(scale * log(precision * 0.5^n)) / 0.4804530139182) and
// k_n = floor(0.69314718055995 * bits_n / scale) (add.lua:16-25, check.lua:41-47);
// probe i = 1 .. k_n is (h[i % 2] + i * h[2 + ((i + i % 2) % 4) / 2]) % bits_n over
// the same SHA-1 words as the ruby driver (add.lua:30-41) — probe_offset with a
// 1-based index.  An item goes to layer ceil(log(ceil((entries + count + 1) /
// entries)) / 0.69314718055995) and bumps the count only if it set a new bit
// (add.lua:6-17, 43-54); include? checks layers 1 .. index(count) (check.lua).
//
// insert_many keeps add.lua's sequential semantics exactly: per layer, the
// sequential-flag kernels (bf_seq.hip) tell which keys would set a new bit, the
// batch is cut where the count reaches the layer's capacity, the keys before the
// cut are applied, and the rest continue on the next layer.
#include "bfhip.h"
#include "bf_device.h"

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

using namespace bfdev;

namespace {

constexpr uint32_t kLuaMaxLayers = 64;
constexpr int kLuaTile = 256;
constexpr int kLuaStageVec = 16384 / 16;

thread_local std::string g_lua_create_error;

__global__ __launch_bounds__(kLuaTile) void lua_check_kernel(const BfGeom* __restrict__ layers, uint32_t nlayers,
                                                             const uint8_t* __restrict__ keys16,
                                                             const uint64_t* __restrict__ offsets, uint64_t bias,
                                                             uint64_t n, uint8_t* __restrict__ out,
                                                             uint32_t* __restrict__ key_status) {
    __shared__ uint64_t s_off[kLuaTile + 1];
    __shared__ uint4 s_stage[kLuaStageVec + kStageSlackVec];
    const uint64_t tile0 = (uint64_t)blockIdx.x * kLuaTile;
    const uint32_t cnt = (uint32_t)((n - tile0) < (uint64_t)kLuaTile ? (n - tile0) : kLuaTile);
    for_key_tile<kLuaTile, kLuaStageVec>(keys16, offsets, bias, tile0, cnt, s_off, s_stage, key_status,
        [&](auto staged, uint32_t lane, const uint32_t* src, uint32_t s, uint32_t L) {
            uint32_t H[5];
            sha1_any<decltype(staged)::value>(src, s, L, H);
            uint32_t found = 0;
            for (uint32_t li = 0; li < nlayers && !found; ++li) {   // check.lua:38-59
                const BfGeom g = layers[li];
                uint32_t ok = 1;
                for (uint32_t i = 1; i <= g.k && ok; ++i) {
                    const uint64_t o = probe_offset(g, H[0], H[1], H[2], H[3], i);
                    ok = (g.bits[o >> 5] >> ((uint32_t)(o ^ 7u) & 31u)) & 1u;
                }
                found = ok;
            }
            out[tile0 + lane] = (uint8_t)found;
        });
}

// Keys that set a new bit (per-key flags 0/1) summed into *count: the layer count's INCR
// (add.lua:48-50) without reading the flags back to the host.
// 16 bytes per lane and step, one atomic per workgroup (atomics on one word serialise).
__global__ __launch_bounds__(256) void lua_count_kernel(const uint8_t* __restrict__ flags, uint64_t n,
                                                        unsigned long long* __restrict__ count) {
    __shared__ uint32_t s_part[4];
    uint32_t c = 0;
    // an unaligned head and the tail byte by byte (workgroup 0), the rest as 16-B vectors
    const uint64_t head = min<uint64_t>(n, (16u - (reinterpret_cast<uintptr_t>(flags) & 15u)) & 15u);
    const uint64_t nv = (n - head) / 16;
    const uint4* fv = reinterpret_cast<const uint4*>(flags + head);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = fv[i];   // bytes are 0 / 1: a byte-wise sum of each word fits 8 bits
        const uint32_t w = v.x + v.y + v.z + v.w;
        c += (w & 0xFFu) + ((w >> 8) & 0xFFu) + ((w >> 16) & 0xFFu) + (w >> 24);
    }
    if (blockIdx.x == 0) {
        if (threadIdx.x < head) c += flags[threadIdx.x];
        for (uint64_t i = head + nv * 16 + threadIdx.x; i < n; i += 256) c += flags[i];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t tot = s_part[0] + s_part[1] + s_part[2] + s_part[3];
        if (tot) atomicAdd(count, (unsigned long long)tot);
    }
}

// The cut of a chunk that may fill its layer (add.lua:48-50), on the device so the host reads
// it back once, after the apply: cnt[0] holds the chunk's new keys (lua_count_kernel).  Below
// `room` the whole chunk stays (cnt[1] = n); else cnt[1] = the index after the key whose INCR
// brings the count to `room`, and cnt[0] = room.  One workgroup: a contiguous byte segment per
// lane, a scan of the segment sums, then the lane whose segment holds the crossing walks it.
__global__ __launch_bounds__(1024) void lua_cut_kernel(const uint8_t* __restrict__ flags, uint64_t n, uint64_t room,
                                                       unsigned long long* __restrict__ cnt) {
    __shared__ uint32_t s_sum[1024];
    if (cnt[0] < room) {   // workgroup-uniform
        if (threadIdx.x == 0) cnt[1] = n;
        return;
    }
    const uint32_t t = threadIdx.x;
    const uint64_t per = (n + 1023) / 1024;
    const uint64_t a = min<uint64_t>((uint64_t)t * per, n), b = min<uint64_t>(a + per, n);
    uint32_t loc = 0;
    for (uint64_t i = a; i < b; ++i) loc += flags[i];
    s_sum[t] = loc;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {   // inclusive scan
        const uint32_t v = t >= d ? s_sum[t - d] : 0u;
        __syncthreads();
        s_sum[t] += v;
        __syncthreads();
    }
    uint64_t c = s_sum[t] - loc;   // new keys before this segment
    if (c >= room || c + loc < room) return;
    for (uint64_t i = a; i < b; ++i) {
        c += flags[i];
        if (c == room) {
            cnt[0] = room;
            cnt[1] = i + 1;
            return;
        }
    }
}

}  // namespace

struct bf_lua {
    std::mutex mu;
    int device = 0;
    hipStream_t stream = nullptr;
    double entries = 0, precision = 0;
    uint64_t count = 0;
    std::vector<BfGeom> layers;   // layers[n - 1]: bitset of layer n (allocated on first use)
    std::vector<uint64_t> layer_bytes;
    // layer bitsets a clear dropped, kept for the next filter's layers of the same size (layer n
    // always has the same bits for one handle): a cleared filter refills without hipMalloc
    std::vector<std::pair<uint64_t, uint32_t*>> pool;
    BfGeom* d_layers = nullptr;   // device copy of the layer table for lua_check_kernel
    uint32_t d_layers_n = 0;      // layers of that copy (layers never change once made; clear resets)
    void* scratch = nullptr;
    uint64_t scratch_cap = 0;
    uint8_t *d_keys = nullptr, *d_out = nullptr, *h_out = nullptr;
    uint64_t* d_off = nullptr;
    uint64_t keys_cap = 0, n_cap = 0;
    unsigned long long* d_last = nullptr;
    unsigned long long* d_flips = nullptr;   // bf_lua_insert_many_changes: [count | entries]
    unsigned long long* h_flips = nullptr;   // pinned mirror of d_flips (small calls read it back at once)
    uint64_t flips_cap = 0;
    uint8_t* h_stage = nullptr;              // pinned [offsets | keys] of small calls (one H2D)
    unsigned long long* d_cnt = nullptr;     // lua_count_kernel's sum (device calls)
    unsigned long long* h_cnt = nullptr;     // ... read back through pinned memory
    uint32_t* h_key_status = nullptr;        // pinned, written by the hashing kernels (bf_api.cpp take_key_status)
    uint32_t* d_key_status = nullptr;        // ... its device address (every layer's BfGeom::key_status)
    // calls on different streams (the _dev entry points take the caller's) are ordered: each
    // waits for the event the previous call recorded, as bf_handle's calls are
    hipEvent_t order_ev = nullptr;
    hipStream_t order_stream = nullptr;
    bool order_valid = false;
    // bf_lua_profile: HIP events around every kernel, accumulated per name (per layer)
    bool profile = false;
    std::vector<BfMarks> prof_pending, prof_free;
    struct ProfAcc { std::string name; double ms; uint64_t launches; };
    std::vector<ProfAcc> prof_acc;
    std::vector<std::string> prof_names;     // "<kernel>[L<layer>]", fixed at create (stable c_str())
    std::string err;
};

namespace {

int lua_err(bf_lua* h, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (h) h->err = buf; else g_lua_create_error = buf;
    return code;
}

#define LUACHK(h, expr)                                                                            \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return lua_err((h), (e_ == hipErrorOutOfMemory ? BF_ENOMEM : BF_EDEVICE), "%s failed: %s", \
                           #expr, hipGetErrorString(e_));                                          \
    } while (0)

struct LuaDeviceGuard {
    int prev = -1;
    explicit LuaDeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~LuaDeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// add.lua:13-15 / check.lua:9-11, in IEEE double like Lua 5.1's numbers.
uint32_t lua_index(double entries, double count) {
    const double factor = std::ceil((entries + count) / entries);
    return (uint32_t)std::ceil(std::log(factor) / 0.69314718055995);
}

// add.lua:16-25 (check.lua:41-47 computes the same values).
void lua_layer(double entries, double precision, uint32_t n, uint64_t* bits, uint32_t* k) {
    const double scale = std::pow(2.0, (double)n - 1.0) * entries;
    const double b = std::floor(-(scale * std::log(precision * std::pow(0.5, (double)n))) / 0.4804530139182);
    const double kk = std::floor(0.69314718055995 * b / scale);
    *bits = b > 0 ? (uint64_t)b : 0;
    *k = kk > 0 ? (uint32_t)kk : 0;
}

// Largest count whose insert still lands in `layer` (counts c with index(c) == layer).
uint64_t lua_layer_capacity(double entries, uint32_t layer, uint64_t from) {
    uint64_t lo = from, step = 1;
    while (lua_index(entries, (double)(lo + step)) <= layer) {
        lo += step;
        step <<= 1;
    }
    uint64_t hi = lo + step;   // index(hi) > layer >= index(lo)
    while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (lua_index(entries, (double)mid) <= layer) lo = mid; else hi = mid;
    }
    return lo;
}

// New layers are cleared on stream s (the call's stream: no cross-stream wait needed).
int ensure_layer(bf_lua* h, uint32_t n, hipStream_t s) {
    if (n == 0 || n > kLuaMaxLayers) return lua_err(h, BF_EINVAL, "layer %u outside 1..%u", n, kLuaMaxLayers);
    while (h->layers.size() < n) {
        const uint32_t li = (uint32_t)h->layers.size() + 1;
        uint64_t m;
        uint32_t k;
        lua_layer(h->entries, h->precision, li, &m, &k);
        if (m == 0 || k == 0 || k > BF_MAX_K)
            return lua_err(h, BF_EINVAL, "layer %u: %llu bits, %u hashes (entries %g, precision %g)", li,
                           (unsigned long long)m, k, h->entries, h->precision);
        BfGeom g{};
        const uint64_t bytes = ((m + 7) / 8 + 255) / 256 * 256;
        auto it = std::find_if(h->pool.begin(), h->pool.end(), [&](const std::pair<uint64_t, uint32_t*>& x) {
            return x.first == bytes;
        });
        if (it != h->pool.end()) {
            g.bits = it->second;
            h->pool.erase(it);
        } else {
            LUACHK(h, hipMalloc((void**)&g.bits, bytes));
        }
        LUACHK(h, hipMemsetAsync(g.bits, 0, bytes, s));
        g.m = m;
        g.inv_m = 1.0 / (double)m;
        g.k = k;
        g.nomod = m > (uint64_t)(k + 1) * 0xFFFFFFFFull ? 1u : 0u;   // probes i = 1..k: v <= (k+1)(2^32-1)
        g.mod_f32 = m >= (1ull << 17) ? 1u : 0u;
        g.inv_m_f = (float)(1.0 / (double)m);
        g.mod_sub = bf_mod_sub(m, (uint64_t)(k + 1) * 0xFFFFFFFFull);
        g.shards = 1;
        g.inv_shards = 1.0;
        g.block_log2 = 20;
        g.key_status = h->d_key_status;
        h->layers.push_back(g);
        h->layer_bytes.push_back(bytes);
    }
    return BF_OK;
}

int ensure_io(bf_lua* h, uint64_t key_bytes, uint64_t n) {
    if (key_bytes + 16 > h->keys_cap) {
        if (h->d_keys) (void)hipFree(h->d_keys);
        h->d_keys = nullptr;
        h->keys_cap = std::max<uint64_t>(key_bytes + 16, 1 << 16) * 2;
        LUACHK(h, hipMalloc((void**)&h->d_keys, h->keys_cap));
    }
    if (n + 1 > h->n_cap) {
        if (h->d_off) (void)hipFree(h->d_off);
        if (h->d_out) (void)hipFree(h->d_out);
        if (h->h_out) (void)hipHostFree(h->h_out);
        h->d_off = nullptr;
        h->d_out = nullptr;
        h->h_out = nullptr;
        h->n_cap = std::max<uint64_t>(n + 1, 1 << 12) * 2;
        LUACHK(h, hipMalloc((void**)&h->d_off, h->n_cap * 8));
        LUACHK(h, hipMalloc((void**)&h->d_out, h->n_cap));
        LUACHK(h, hipHostMalloc((void**)&h->h_out, h->n_cap, hipHostMallocDefault));
    }
    return BF_OK;
}

// The key-status word the hashing kernels write (bfdev::key_ok): reported once, as BF_EINVAL,
// by the next call on the handle (bf_api.cpp take_key_status).
int lua_take_key_status(bf_lua* h) {
    if (!h->h_key_status || __atomic_load_n(h->h_key_status, __ATOMIC_ACQUIRE) == 0u) return BF_OK;
    __atomic_store_n(h->h_key_status, 0u, __ATOMIC_RELEASE);
    return lua_err(h, BF_EINVAL, "an earlier call's key offsets were inconsistent (offsets must be non-decreasing "
                                 "and every key below 2 GiB): those keys were hashed as empty strings");
}

// Stream order across calls (bf_api.cpp's StreamOrder): wait for the previous call's event,
// record this call's at the end.
struct LuaOrder {
    bf_lua* h;
    hipStream_t s;
    LuaOrder(bf_lua* h_, hipStream_t s_) : h(h_), s(s_) {
        if (h->order_valid && h->order_stream != s) (void)hipStreamWaitEvent(s, h->order_ev, 0);
    }
    ~LuaOrder() {
        if (h->order_ev && hipEventRecord(h->order_ev, s) == hipSuccess) {
            h->order_valid = true;
            h->order_stream = s;
        }
    }
};

enum LuaKern { kLuaCand = 0, kLuaMark = 1, kLuaCheck = 2, kLuaCount = 3, kLuaKerns = 4 };
const char* const kLuaKernName[kLuaKerns] = {"lua_seq_candidates", "lua_seq_mark", "lua_check", "lua_count"};

const char* lua_prof_name(const bf_lua* h, LuaKern kind, uint32_t layer) {
    return h->prof_names[(size_t)kind * kLuaMaxLayers + (layer ? layer - 1 : 0)].c_str();
}

BfMarks* lua_prof_begin(bf_lua* h, hipStream_t s) {
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

int lua_prof_harvest(bf_lua* h) {
    for (BfMarks& mk : h->prof_pending) {
        if (mk.used > 0) LUACHK(h, hipEventSynchronize(mk.ev[mk.used]));
        for (int i = 0; i < mk.used; ++i) {
            float ms = 0.f;
            LUACHK(h, hipEventElapsedTime(&ms, mk.ev[i], mk.ev[i + 1]));
            auto it = std::find_if(h->prof_acc.begin(), h->prof_acc.end(),
                                   [&](const bf_lua::ProfAcc& a) { return a.name == mk.names[i]; });
            if (it == h->prof_acc.end()) h->prof_acc.push_back({mk.names[i], (double)ms, 1});
            else { it->ms += ms; it->launches += 1; }
        }
        h->prof_free.push_back(mk);
    }
    h->prof_pending.clear();
    return BF_OK;
}

int ensure_lua_scratch(bf_lua* h, uint64_t bytes) {
    if (bytes <= h->scratch_cap) return BF_OK;
    LUACHK(h, hipStreamSynchronize(h->stream));
    if (h->scratch) (void)hipFree(h->scratch);
    h->scratch = nullptr;
    h->scratch_cap = 0;
    LUACHK(h, hipMalloc(&h->scratch, bytes));
    h->scratch_cap = bytes;
    return BF_OK;
}

// Small calls (a per-key insert / include?): offsets and key bytes go through one pinned block
// and one H2D copy, with no host sync (every call ends with one, so the block is free again).
constexpr uint64_t kLuaSmallKeys = 2048;
constexpr uint64_t kLuaSmallBytes = 64ull << 10;

// Keys to the device (offsets rebased to 0), 16-byte aligned with slack.
int stage_keys(bf_lua* h, const uint8_t* keys, const uint64_t* offsets, uint64_t n) {
    for (uint64_t j = 0; j < n; ++j)
        if (offsets[j + 1] < offsets[j]) return lua_err(h, BF_EINVAL, "offsets must be non-decreasing (j=%llu)",
                                                        (unsigned long long)j);
    const uint64_t base = offsets[0], nbytes = offsets[n] - offsets[0];
    int rc = ensure_io(h, nbytes, n);
    if (rc) return rc;
    if (n <= kLuaSmallKeys && nbytes <= kLuaSmallBytes) {
        const uint64_t off_bytes = (kLuaSmallKeys + 1) * 8;
        if (!h->h_stage) LUACHK(h, hipHostMalloc((void**)&h->h_stage, off_bytes + kLuaSmallBytes + 16,
                                                 hipHostMallocDefault));
        uint64_t* ho = reinterpret_cast<uint64_t*>(h->h_stage);
        for (uint64_t j = 0; j <= n; ++j) ho[j] = offsets[j] - base;
        uint8_t* hk = h->h_stage + off_bytes;
        if (nbytes) memcpy(hk, keys + base, nbytes);
        memset(hk + nbytes, 0, 16);
        LUACHK(h, hipMemcpyAsync(h->d_off, ho, (n + 1) * 8, hipMemcpyHostToDevice, h->stream));
        LUACHK(h, hipMemcpyAsync(h->d_keys, hk, nbytes + 16, hipMemcpyHostToDevice, h->stream));
        return BF_OK;
    }
    std::vector<uint64_t> rebased(n + 1);
    for (uint64_t j = 0; j <= n; ++j) rebased[j] = offsets[j] - base;
    if (nbytes) LUACHK(h, hipMemcpyAsync(h->d_keys, keys + base, nbytes, hipMemcpyHostToDevice, h->stream));
    LUACHK(h, hipMemsetAsync(h->d_keys + nbytes, 0, 16, h->stream));
    LUACHK(h, hipMemcpyAsync(h->d_off, rebased.data(), (n + 1) * 8, hipMemcpyHostToDevice, h->stream));
    LUACHK(h, hipStreamSynchronize(h->stream));   // `rebased` is freed on return
    return BF_OK;
}

}  // namespace

extern "C" {

int bf_lua_layer_params(double entries, double precision, uint32_t layer, uint64_t* bits, uint32_t* k) {
    if (!(entries > 0) || !(precision > 0) || layer == 0) return BF_EINVAL;
    uint64_t b;
    uint32_t kk;
    lua_layer(entries, precision, layer, &b, &kk);
    if (bits) *bits = b;
    if (k) *k = kk;
    return BF_OK;
}

int bf_lua_index(double entries, uint64_t count, uint32_t* layer) {
    if (!(entries > 0) || !layer) return BF_EINVAL;
    *layer = lua_index(entries, (double)count);
    return BF_OK;
}

int bf_lua_create(double entries, double precision, const bf_config* cfg, bf_lua** out) {
    if (!out) return lua_err(nullptr, BF_EINVAL, "out is NULL");
    *out = nullptr;
    if (!(entries > 0) || !(precision > 0) || !(precision < 1))
        return lua_err(nullptr, BF_EINVAL, "entries must be > 0 and precision in (0, 1) (got %g, %g)", entries,
                       precision);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return lua_err(nullptr, BF_EDEVICE, "no HIP device available");
    int dev = (cfg && cfg->struct_size >= 8) ? cfg->device : -1;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
    if (dev >= ndev) return lua_err(nullptr, BF_EINVAL, "device %d out of range (%d devices)", dev, ndev);
    bf_lua* h = new (std::nothrow) bf_lua();
    if (!h) return lua_err(nullptr, BF_ENOMEM, "host allocation failed");
    h->device = dev;
    h->entries = entries;
    h->precision = precision;
    LuaDeviceGuard dg(dev);
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&h->order_ev, hipEventDisableTiming) != hipSuccess ||
        hipMalloc((void**)&h->d_layers, kLuaMaxLayers * sizeof(BfGeom)) != hipSuccess ||
        hipMalloc((void**)&h->d_last, 64) != hipSuccess || hipMalloc((void**)&h->d_cnt, 64) != hipSuccess ||
        hipHostMalloc((void**)&h->h_cnt, 64, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&h->h_key_status, 64, hipHostMallocDefault) != hipSuccess ||
        (*h->h_key_status = 0u, hipHostGetDevicePointer((void**)&h->d_key_status, h->h_key_status, 0)) != hipSuccess) {
        if (h->stream) (void)hipStreamDestroy(h->stream);
        if (h->h_cnt) (void)hipHostFree(h->h_cnt);
        if (h->h_key_status) (void)hipHostFree(h->h_key_status);
        if (h->order_ev) (void)hipEventDestroy(h->order_ev);
        if (h->d_layers) (void)hipFree(h->d_layers);
        if (h->d_last) (void)hipFree(h->d_last);
        if (h->d_cnt) (void)hipFree(h->d_cnt);
        delete h;
        return lua_err(nullptr, BF_EDEVICE, "stream / table allocation failed");
    }
    h->prof_names.reserve((size_t)kLuaKerns * kLuaMaxLayers);
    for (int kd = 0; kd < kLuaKerns; ++kd)
        for (uint32_t l = 1; l <= kLuaMaxLayers; ++l)
            h->prof_names.push_back(std::string(kLuaKernName[kd]) + (kd == kLuaCheck ? "" : "[L" + std::to_string(l) + "]"));
    *out = h;
    return BF_OK;
}

int bf_lua_destroy(bf_lua* h) {
    if (!h) return BF_OK;
    {
        std::lock_guard<std::mutex> lk(h->mu);
        LuaDeviceGuard dg(h->device);
        (void)hipStreamSynchronize(h->stream);
        for (BfGeom& g : h->layers) (void)hipFree(g.bits);
        for (auto& x : h->pool) (void)hipFree(x.second);
        for (void* p : {(void*)h->d_layers, (void*)h->scratch, (void*)h->d_keys, (void*)h->d_out, (void*)h->d_off,
                        (void*)h->d_last, (void*)h->d_flips, (void*)h->d_cnt})
            if (p) (void)hipFree(p);
        for (std::vector<BfMarks>* v : {&h->prof_pending, &h->prof_free})
            for (BfMarks& mk : *v)
                for (hipEvent_t e : mk.ev)
                    if (e) (void)hipEventDestroy(e);
        if (h->order_ev) (void)hipEventDestroy(h->order_ev);
        if (h->h_cnt) (void)hipHostFree(h->h_cnt);
        if (h->h_out) (void)hipHostFree(h->h_out);
        if (h->h_flips) (void)hipHostFree(h->h_flips);
        if (h->h_stage) (void)hipHostFree(h->h_stage);
        if (h->h_key_status) (void)hipHostFree(h->h_key_status);
        (void)hipStreamDestroy(h->stream);
    }
    delete h;
    return BF_OK;
}

const char* bf_lua_last_error(const bf_lua* h) { return h ? h->err.c_str() : g_lua_create_error.c_str(); }

int bf_lua_get_count(const bf_lua* h, uint64_t* count) {
    if (!h || !count) return BF_EINVAL;
    *count = h->count;
    return BF_OK;
}

int bf_lua_set_count(bf_lua* h, uint64_t count) {
    if (!h) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    h->count = count;
    return BF_OK;
}

int bf_lua_layers(const bf_lua* h, uint32_t* nlayers) {
    if (!h || !nlayers) return BF_EINVAL;
    *nlayers = (uint32_t)h->layers.size();
    return BF_OK;
}

int bf_lua_clear(bf_lua* h) {
    if (!h) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    LuaDeviceGuard dg(h->device);
    LUACHK(h, hipStreamSynchronize(h->stream));
    if (h->order_valid) LUACHK(h, hipEventSynchronize(h->order_ev));   // a _dev call's stream
    for (size_t i = 0; i < h->layers.size(); ++i) h->pool.push_back({h->layer_bytes[i], h->layers[i].bits});
    h->layers.clear();
    h->layer_bytes.clear();
    h->d_layers_n = 0;
    h->count = 0;
    return BF_OK;
}

}  // extern "C"

namespace {

// flips (bf_lua_insert_many_changes): every bit the batch flips, (layer << 58) | offset, into
// a device list of `cap` entries that is copied to `flips` at the end; *flip_count = all of them.
int lua_insert(bf_lua* h, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* per_key_new,
               uint64_t* new_layers, uint64_t* flips, uint64_t cap, uint64_t* flip_count) {
    if (!h) return BF_EINVAL;
    if (new_layers) *new_layers = 0;
    if (flip_count) *flip_count = 0;
    if (n == 0) return BF_OK;
    if (!offsets || (!keys && offsets[n] != offsets[0])) return lua_err(h, BF_EINVAL, "NULL keys / offsets");
    std::lock_guard<std::mutex> lk(h->mu);
    LuaDeviceGuard dg(h->device);
    LuaOrder lo(h, h->stream);
    if (int krc = lua_take_key_status(h)) return krc;   // an earlier call's bad key offsets
    int rc = stage_keys(h, keys, offsets, n);
    if (rc) return rc;
    unsigned long long* d_flips = nullptr;
    constexpr uint64_t kSmallFlips = 4096;   // lists up to this long come back with the flags
    const bool small_flips = flips && cap <= kSmallFlips;
    bool last_read = false;   // the last chunk's flags D2H also carried the flip list
    if (flips) {   // [count | cap entries], kept on the handle
        if (h->flips_cap < cap) {
            LUACHK(h, hipStreamSynchronize(h->stream));
            if (h->d_flips) (void)hipFree(h->d_flips);
            h->d_flips = nullptr;
            h->flips_cap = 0;
            const uint64_t c = std::max<uint64_t>(cap, kSmallFlips);
            LUACHK(h, hipMalloc((void**)&h->d_flips, (c + 1) * 8));
            h->flips_cap = c;
        }
        if (!h->h_flips) LUACHK(h, hipHostMalloc((void**)&h->h_flips, (kSmallFlips + 1) * 8, hipHostMallocDefault));
        d_flips = h->d_flips;
        LUACHK(h, hipMemsetAsync(d_flips, 0, 8, h->stream));
    }
    uint64_t s = 0;
    while (s < n) {
        const uint32_t layer = lua_index(h->entries, (double)(h->count + 1));   // add.lua:6-15
        if ((rc = ensure_layer(h, layer, h->stream))) return rc;
        const BfGeom& g = h->layers[layer - 1];
        const uint64_t room = lua_layer_capacity(h->entries, layer, h->count + 1) - h->count;   // >= 1
        const uint64_t cn = std::min<uint64_t>(n - s, bf_seq_chunk_keys(g.k));
        if ((rc = ensure_lua_scratch(h, bf_seq_scratch_bytes(cn, g.k, g.m)))) return rc;
        // which keys would set a new bit of this layer, in order (nothing applied yet)
        BfMarks* mk = lua_prof_begin(h, h->stream);
        LUACHK(h, bf_launch_seq_candidates(g, 1, h->d_keys, h->d_off + s, 0, cn, h->scratch, h->stream));
        bf_mark(mk, h->stream, lua_prof_name(h, kLuaCand, layer));
        BfGeom ga = g;
        if (d_flips) {
            ga.flips = d_flips + 1;
            ga.flip_count = d_flips;
            ga.flip_cap = cap;
            ga.flip_tag = (uint64_t)layer << 58;
        }
        uint64_t take = cn, fresh = 0;
        bool read_now = false;
        if (room >= cn) {
            // no key of the chunk can fill the layer before the last one: flags and apply in ONE
            // mark pass, one sync (the per-key insert's case)
            LUACHK(h, bf_launch_seq_mark(ga, 1, cn, cn, h->scratch, h->d_out, nullptr, h->stream));
            bf_mark(mk, h->stream, lua_prof_name(h, kLuaMark, layer));
            LUACHK(h, hipMemcpyAsync(h->h_out, h->d_out, cn, hipMemcpyDeviceToHost, h->stream));
            if (d_flips && small_flips)
                LUACHK(h, hipMemcpyAsync(h->h_flips, d_flips, (cap + 1) * 8, hipMemcpyDeviceToHost, h->stream));
            LUACHK(h, hipStreamSynchronize(h->stream));
            read_now = d_flips && small_flips;
            for (uint64_t j = 0; j < cn; ++j) fresh += h->h_out[j];
        } else {
            LUACHK(h, bf_launch_seq_mark(g, 1, cn, 0, h->scratch, h->d_out, nullptr, h->stream));
            bf_mark(mk, h->stream, lua_prof_name(h, kLuaMark, layer));
            LUACHK(h, hipMemcpyAsync(h->h_out, h->d_out, cn, hipMemcpyDeviceToHost, h->stream));
            LUACHK(h, hipStreamSynchronize(h->stream));
            // cut after the key whose INCR fills the layer (add.lua:48-50); later keys go up a layer
            for (uint64_t j = 0; j < cn; ++j) {
                fresh += h->h_out[j];
                if (fresh == room) {
                    take = j + 1;
                    break;
                }
            }
            mk = lua_prof_begin(h, h->stream);
            LUACHK(h, bf_launch_seq_mark(ga, 1, cn, take, h->scratch, nullptr, nullptr, h->stream));
            bf_mark(mk, h->stream, lua_prof_name(h, kLuaMark, layer));
        }
        if (per_key_new) memcpy(per_key_new + s, h->h_out, take);
        if (fresh && new_layers && layer <= 64) *new_layers |= 1ull << (layer - 1);
        h->count += fresh;
        s += take;
        last_read = read_now;
    }
    if (d_flips) {
        unsigned long long c = 0;
        if (small_flips && last_read) {   // read back with the last chunk's flags
            c = h->h_flips[0];
            if (c <= cap && c) memcpy(flips, h->h_flips + 1, c * 8);
        } else {
            LUACHK(h, hipMemcpyAsync(&c, d_flips, 8, hipMemcpyDeviceToHost, h->stream));
            LUACHK(h, hipStreamSynchronize(h->stream));
            if (c <= cap && c) LUACHK(h, hipMemcpy(flips, d_flips + 1, c * 8, hipMemcpyDeviceToHost));
        }
        *flip_count = c;
        if (c > cap) return lua_err(h, BF_ERANGE, "%llu bits flipped, out_bits holds %llu (the insert is applied)",
                                    c, (unsigned long long)cap);
    }
    LUACHK(h, hipStreamSynchronize(h->stream));
    return BF_OK;
}

// Layers up to n exist, cleared on the caller's stream (no host sync: VERDICT r05 item 5).
int ensure_layer_on(bf_lua* h, uint32_t n, hipStream_t s) { return ensure_layer(h, n, s); }

// bf_lua_insert_many on device-resident keys (the caller's stream): add.lua's sequential
// semantics exactly as lua_insert, with the per-key flags left on the device and the count's
// INCRs summed there (lua_count_kernel) and a layer's cut found there (lua_cut_kernel); the
// host reads 16 bytes per chunk, after its apply, to pick the next layer.
int lua_insert_dev(bf_lua* h, const uint8_t* d_keys, const uint64_t* d_offsets, uint64_t n, uint8_t* d_per_key_new,
                   uint64_t* new_layers, hipStream_t s) {
    if (new_layers) *new_layers = 0;
    if (n == 0) return BF_OK;
    if (!d_keys || !d_offsets) return lua_err(h, BF_EINVAL, "NULL device pointer");
    std::lock_guard<std::mutex> lk(h->mu);
    LuaDeviceGuard dg(h->device);
    LuaOrder lo(h, s);
    if (int krc = lua_take_key_status(h)) return krc;   // an earlier call's bad key offsets
    uint64_t bias = 0;
    const uintptr_t a = reinterpret_cast<uintptr_t>(d_keys);
    bias = a & 15u;
    const uint8_t* k16 = reinterpret_cast<const uint8_t*>(a & ~(uintptr_t)15);
    int rc = ensure_io(h, 0, std::min<uint64_t>(n, bf_seq_chunk_keys(1)));   // d_out / h_out for one chunk
    if (rc) return rc;
    uint64_t done = 0;
    while (done < n) {
        const uint32_t layer = lua_index(h->entries, (double)(h->count + 1));   // add.lua:6-15
        if ((rc = ensure_layer_on(h, layer, s))) return rc;
        const BfGeom& g = h->layers[layer - 1];
        const uint64_t room = lua_layer_capacity(h->entries, layer, h->count + 1) - h->count;   // >= 1
        const uint64_t cn = std::min<uint64_t>(n - done, bf_seq_chunk_keys(g.k));
        if ((rc = ensure_io(h, 0, cn))) return rc;
        if ((rc = ensure_lua_scratch(h, bf_seq_scratch_bytes(cn, g.k, g.m)))) return rc;
        uint8_t* flags = d_per_key_new ? d_per_key_new + done : h->d_out;
        BfMarks* mk = lua_prof_begin(h, s);
        LUACHK(h, bf_launch_seq_candidates(g, 1, k16, d_offsets + done, bias, cn, h->scratch, s));
        bf_mark(mk, s, lua_prof_name(h, kLuaCand, layer));
        const uint32_t grid = (uint32_t)std::min<uint64_t>((cn / 16 + 255) / 256 + 1, 256);
        LUACHK(h, hipMemsetAsync(h->d_cnt, 0, 16, s));
        if (room >= cn) {   // the whole chunk lands in this layer: flags and apply in one pass
            LUACHK(h, bf_launch_seq_mark(g, 1, cn, cn, h->scratch, flags, nullptr, s));
            bf_mark(mk, s, lua_prof_name(h, kLuaMark, layer));
            hipLaunchKernelGGL(lua_count_kernel, dim3(grid), dim3(256), 0, s, flags, cn, h->d_cnt);
            LUACHK(h, hipGetLastError());
            bf_mark(mk, s, lua_prof_name(h, kLuaCount, layer));
            LUACHK(h, hipMemcpyAsync(h->h_cnt, h->d_cnt, 8, hipMemcpyDeviceToHost, s));
            h->h_cnt[1] = cn;
        } else {   // the chunk may fill the layer: cut after the key whose INCR fills it (add.lua:48-50)
            // flags first; the INCRs summed and the cut found on the device (lua_cut_kernel),
            // then the keys before the cut applied with that limit — one read-back, at the end
            LUACHK(h, bf_launch_seq_mark(g, 1, cn, 0, h->scratch, flags, nullptr, s));
            bf_mark(mk, s, lua_prof_name(h, kLuaMark, layer));
            hipLaunchKernelGGL(lua_count_kernel, dim3(grid), dim3(256), 0, s, flags, cn, h->d_cnt);
            hipLaunchKernelGGL(lua_cut_kernel, dim3(1), dim3(1024), 0, s, flags, cn, room, h->d_cnt);
            LUACHK(h, hipGetLastError());
            bf_mark(mk, s, lua_prof_name(h, kLuaCount, layer));
            LUACHK(h, bf_launch_seq_mark(g, 1, cn, cn, h->scratch, nullptr, nullptr, s, h->d_cnt + 1));
            bf_mark(mk, s, lua_prof_name(h, kLuaMark, layer));
            LUACHK(h, hipMemcpyAsync(h->h_cnt, h->d_cnt, 16, hipMemcpyDeviceToHost, s));
        }
        LUACHK(h, hipStreamSynchronize(s));
        const uint64_t fresh = h->h_cnt[0], take = h->h_cnt[1];
        if (take == 0 || take > cn) return lua_err(h, BF_EDEVICE, "layer %u: cut at %llu of %llu keys", layer,
                                                   (unsigned long long)take, (unsigned long long)cn);
        if (fresh && new_layers && layer <= 64) *new_layers |= 1ull << (layer - 1);
        h->count += fresh;
        done += take;
    }
    return BF_OK;
}

}  // namespace

extern "C" {

int bf_lua_insert_many_dev(bf_lua* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                           uint8_t* d_per_key_new, uint64_t* new_layers, void* stream) {
    if (!h) return BF_EINVAL;
    return lua_insert_dev(h, d_key_bytes, d_offsets, n, d_per_key_new, new_layers,
                          reinterpret_cast<hipStream_t>(stream));
}

int bf_lua_include_many_dev(bf_lua* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                            uint8_t* d_out, void* stream) {
    if (!h) return BF_EINVAL;
    if (n == 0) return BF_OK;
    if (!d_key_bytes || !d_offsets || !d_out) return lua_err(h, BF_EINVAL, "NULL device pointer");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lk(h->mu);
    LuaDeviceGuard dg(h->device);
    LuaOrder lo(h, s);
    if (int krc = lua_take_key_status(h)) return krc;   // an earlier call's bad key offsets
    if (h->count == 0) {   // check.lua:3-7
        LUACHK(h, hipMemsetAsync(d_out, 0, n, s));
        return BF_OK;
    }
    const uint32_t index = lua_index(h->entries, (double)h->count);   // check.lua:9-11
    int rc = ensure_layer_on(h, index, s);
    if (rc) return rc;
    if (h->d_layers_n < index) {   // the table is pageable host memory: the copy completes on return
        LUACHK(h, hipMemcpyAsync(h->d_layers, h->layers.data(), index * sizeof(BfGeom), hipMemcpyHostToDevice, s));
        LUACHK(h, hipStreamSynchronize(s));
        h->d_layers_n = index;
    }
    const uintptr_t a = reinterpret_cast<uintptr_t>(d_key_bytes);
    BfMarks* mk = lua_prof_begin(h, s);
    hipLaunchKernelGGL(lua_check_kernel, dim3((uint32_t)((n + kLuaTile - 1) / kLuaTile)), dim3(kLuaTile), 0, s,
                       h->d_layers, index, reinterpret_cast<const uint8_t*>(a & ~(uintptr_t)15), d_offsets,
                       (uint64_t)(a & 15u), n, d_out, h->d_key_status);
    LUACHK(h, hipGetLastError());
    bf_mark(mk, s, lua_prof_name(h, kLuaCheck, index));
    return BF_OK;
}

int bf_lua_profile(bf_lua* h, uint32_t enable) {
    if (!h) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    LuaDeviceGuard dg(h->device);
    int rc = lua_prof_harvest(h);
    h->profile = enable != 0;
    return rc;
}

int bf_lua_profile_read(bf_lua* h, char* names, double* total_ms, uint64_t* launches, uint32_t cap,
                        uint32_t* n_out, uint32_t reset) {
    if (!h || !n_out) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    LuaDeviceGuard dg(h->device);
    int rc = lua_prof_harvest(h);
    if (rc) return rc;
    *n_out = (uint32_t)h->prof_acc.size();
    for (uint32_t i = 0; i < cap && i < h->prof_acc.size(); ++i) {
        const bf_lua::ProfAcc& acc = h->prof_acc[i];
        if (names) snprintf(names + (size_t)i * BF_PROFILE_NAME_LEN, BF_PROFILE_NAME_LEN, "%s", acc.name.c_str());
        if (total_ms) total_ms[i] = acc.ms;
        if (launches) launches[i] = acc.launches;
    }
    if (reset) h->prof_acc.clear();
    return BF_OK;
}

int bf_lua_insert_many(bf_lua* h, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* per_key_new,
                       uint64_t* new_layers) {
    return lua_insert(h, keys, offsets, n, per_key_new, new_layers, nullptr, 0, nullptr);
}

int bf_lua_insert_many_changes(bf_lua* h, const uint8_t* keys, const uint64_t* offsets, uint64_t n,
                               uint8_t* per_key_new, uint64_t* new_layers, uint64_t* out_bits, uint64_t cap,
                               uint64_t* count) {
    if (!h) return BF_EINVAL;
    if (!count || (cap && !out_bits)) return lua_err(h, BF_EINVAL, "NULL out_bits / count");
    return lua_insert(h, keys, offsets, n, per_key_new, new_layers, out_bits, cap, count);
}

int bf_lua_include_many(bf_lua* h, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* out) {
    if (!h) return BF_EINVAL;
    if (n == 0) return BF_OK;
    if (!offsets || !out || (!keys && offsets[n] != offsets[0])) return lua_err(h, BF_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->count == 0) {   // check.lua:3-7
        memset(out, 0, n);
        return BF_OK;
    }
    LuaDeviceGuard dg(h->device);
    LuaOrder lo(h, h->stream);
    if (int krc = lua_take_key_status(h)) return krc;   // an earlier call's bad key offsets
    const uint32_t index = lua_index(h->entries, (double)h->count);   // check.lua:9-11
    int rc = ensure_layer(h, index, h->stream);
    if (rc) return rc;
    if ((rc = stage_keys(h, keys, offsets, n))) return rc;
    if (h->d_layers_n < index) {   // upload the table only when a layer was added
        LUACHK(h, hipMemcpyAsync(h->d_layers, h->layers.data(), index * sizeof(BfGeom), hipMemcpyHostToDevice,
                                 h->stream));
        h->d_layers_n = index;
    }
    BfMarks* mk = lua_prof_begin(h, h->stream);
    hipLaunchKernelGGL(lua_check_kernel, dim3((uint32_t)((n + kLuaTile - 1) / kLuaTile)), dim3(kLuaTile), 0,
                       h->stream, h->d_layers, index, h->d_keys, h->d_off, (uint64_t)0, n, h->d_out,
                       h->d_key_status);
    LUACHK(h, hipGetLastError());
    bf_mark(mk, h->stream, lua_prof_name(h, kLuaCheck, index));
    LUACHK(h, hipMemcpyAsync(out, h->d_out, n, hipMemcpyDeviceToHost, h->stream));
    LUACHK(h, hipStreamSynchronize(h->stream));
    return BF_OK;
}

int bf_lua_export_layer(bf_lua* h, uint32_t layer, uint8_t* buf, uint64_t cap, uint64_t* len_out) {
    if (!h || !len_out) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    *len_out = 0;
    if (layer == 0 || layer > h->layers.size()) return BF_OK;   // a layer never written: absent key
    LuaDeviceGuard dg(h->device);
    LuaOrder lo(h, h->stream);
    if (int krc = lua_take_key_status(h)) return krc;   // an earlier call's bad key offsets
    const BfGeom& g = h->layers[layer - 1];
    LUACHK(h, hipMemsetAsync(h->d_last, 0, 8, h->stream));
    LUACHK(h, bf_launch_last_nonzero(g.bits, h->layer_bytes[layer - 1] / 4, h->d_last, h->stream));
    unsigned long long last = 0;
    LUACHK(h, hipMemcpyAsync(&last, h->d_last, 8, hipMemcpyDeviceToHost, h->stream));
    LUACHK(h, hipStreamSynchronize(h->stream));
    uint64_t len = 0;
    if (last) {   // trim inside the last nonzero word
        uint8_t w[4];
        LUACHK(h, hipMemcpy(w, reinterpret_cast<const uint8_t*>(g.bits) + (last - 1) * 4, 4, hipMemcpyDeviceToHost));
        len = (last - 1) * 4 + 4;
        while (len > (last - 1) * 4 && w[len - (last - 1) * 4 - 1] == 0) --len;
    }
    *len_out = len;
    if (!buf) return BF_OK;
    if (cap < len) return lua_err(h, BF_ERANGE, "buffer of %llu bytes, layer string is %llu", (unsigned long long)cap,
                                  (unsigned long long)len);
    if (len) LUACHK(h, hipMemcpy(buf, g.bits, len, hipMemcpyDeviceToHost));
    return BF_OK;
}

int bf_lua_import_layer(bf_lua* h, uint32_t layer, const uint8_t* buf, uint64_t len) {
    if (!h || (len && !buf)) return BF_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    LuaDeviceGuard dg(h->device);
    LuaOrder lo(h, h->stream);
    if (int krc = lua_take_key_status(h)) return krc;   // an earlier call's bad key offsets
    int rc = ensure_layer(h, layer, h->stream);
    if (rc) return rc;
    const BfGeom& g = h->layers[layer - 1];
    const uint64_t full = (g.m + 7) / 8;
    if (len > full) return lua_err(h, BF_EINVAL, "layer %u string of %llu bytes exceeds %llu", layer,
                                   (unsigned long long)len, (unsigned long long)full);
    if (len == full && (g.m & 7) && (buf[len - 1] & (0xFF >> (g.m & 7))))
        return lua_err(h, BF_EINVAL, "layer %u string sets bits at or beyond %llu", layer, (unsigned long long)g.m);
    LUACHK(h, hipMemsetAsync(g.bits, 0, h->layer_bytes[layer - 1], h->stream));
    if (len) LUACHK(h, hipMemcpyAsync(g.bits, buf, len, hipMemcpyHostToDevice, h->stream));
    LUACHK(h, hipStreamSynchronize(h->stream));
    return BF_OK;
}

}  // extern "C"
