// bf_seq.hip — exact sequential per-key results for a batch insert.
//
// The ruby driver inserts one key per call: SETBIT k times, found = every old
// bit was 1 (ruby.rb:57-61).  Run over a batch in order, key j is "new" iff one
// of its bits was 0 before the batch AND no earlier key of the batch set it.
// With first(b) = the smallest batch index whose probes include bit b:
//
//     new(j)  <=>  exists probe b of j:  prebit(b) == 0  and  first(b) == j
//
// (first(b) <= j always holds for j's own probes).  Two kernels per chunk:
//   1. seq_candidates: hash (shared SHA-1 / ruby.rb:41-55 derivation), test every
//      probe against the pre-batch bitset; for each 0 bit record the min index j —
//      DIRECT: in a table of one uint32 per bit of the filter (one atomicMin at the
//      offset), for filters whose table is not much larger than the hash table below
//      (seq_direct: the Lua layout's 1M-scale layers, 44 MB at 11M bits); else in a
//      global open-addressing table keyed by bit offset (atomicCAS claim + atomicMin);
//      keep the digest and the key's mask of 0-probes;
//   2. seq_mark: new(j) from the table, then OR the 0-probes of keys j < limit in.
// Filters of up to 2^27 bits and batches of 4096+ keys take the binned form below instead
// (the table per region of the filter, in LDS; launched behind the same two entry points).
// Chunks run in stream order, so chunk c+1 tests against chunk c's bits: the
// result is that of inserting every key one by one.  "Found before its own
// insert" — what bf_10_000.rb and the spec's test_error_rate compare include?
// against — is !new(j).  The probe indices are i0 .. i0+k-1: 0-based for the
// ruby driver (ruby.rb:50), 1-based for the Lua scripts (add.lua:37).
#include "bf_device.h"

using namespace bfdev;

namespace {

constexpr int kSeqTile = 256;
constexpr int kSeqStageVec = 16384 / 16;

__device__ __forceinline__ uint64_t mix64(uint64_t x) {   // SplitMix64 finalizer
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

template <bool DIRECT>
__global__ __launch_bounds__(kSeqTile) void seq_candidates_kernel(BfGeom g, uint32_t i0,
                                                                  const uint8_t* __restrict__ keys16,
                                                                  const uint64_t* __restrict__ offsets, uint64_t bias,
                                                                  uint64_t n, unsigned long long* __restrict__ tkeys,
                                                                  uint32_t* __restrict__ tvals, uint64_t tmask,
                                                                  uint4* __restrict__ digests,
                                                                  unsigned long long* __restrict__ cand) {
    __shared__ uint64_t s_off[kSeqTile + 1];
    __shared__ uint4 s_stage[kSeqStageVec + kStageSlackVec];
    const uint64_t tile0 = (uint64_t)blockIdx.x * kSeqTile;
    const uint32_t cnt = (uint32_t)((n - tile0) < (uint64_t)kSeqTile ? (n - tile0) : kSeqTile);
    for_key_tile<kSeqTile, kSeqStageVec>(keys16, offsets, bias, tile0, cnt, s_off, s_stage, g.key_status,
        [&](auto staged, uint32_t lane, const uint32_t* src, uint32_t s, uint32_t L) {
            uint32_t H[5];
            sha1_any<decltype(staged)::value>(src, s, L, H);
            const uint32_t j = (uint32_t)(tile0 + lane);
            digests[j] = make_uint4(H[0], H[1], H[2], H[3]);
            unsigned long long cm = 0;
            for (uint32_t i = 0; i < g.k; ++i) {
                const uint64_t o = probe_offset(g, H[0], H[1], H[2], H[3], i0 + i);
                if ((g.bits[o >> 5] >> ((uint32_t)(o ^ 7u) & 31u)) & 1u) continue;
                cm |= 1ull << i;
                if constexpr (DIRECT) {   // one word per bit (o < m): no claim, no probing
                    atomicMin(tvals + o, j);
                    continue;
                }
                const unsigned long long key = o + 1;   // 0 marks an empty slot
                uint64_t slot = mix64(o) & tmask;
                for (;;) {   // the table holds <= half its slots: a free or matching slot exists
                    const unsigned long long cur = atomicCAS(tkeys + slot, 0ull, key);
                    if (cur == 0ull || cur == key) {
                        atomicMin(tvals + slot, j);
                        break;
                    }
                    slot = (slot + 1) & tmask;
                }
            }
            cand[j] = cm;
        });
}

// out8 / any_flag (nullable) get new(j) for j < n; the 0-probes of keys j < limit are ORed in.
template <bool DIRECT>
__global__ __launch_bounds__(256) void seq_mark_kernel(BfGeom g, uint32_t i0, uint64_t n, uint64_t limit,
                                                       const unsigned long long* __restrict__ d_limit,
                                                       const unsigned long long* __restrict__ tkeys,
                                                       const uint32_t* __restrict__ tvals, uint64_t tmask,
                                                       const uint4* __restrict__ digests,
                                                       const unsigned long long* __restrict__ cand,
                                                       uint8_t* __restrict__ out8, uint32_t* __restrict__ any_flag) {
    if (d_limit) limit = min<uint64_t>(limit, *d_limit);
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t isnew = 0;
    if (j < n) {
        unsigned long long cm = cand[j];
        if (cm) {
            const uint4 H = digests[j];
            while (cm) {
                const uint32_t i = (uint32_t)__builtin_ctzll(cm);
                cm &= cm - 1;
                const uint64_t o = probe_offset(g, H.x, H.y, H.z, H.w, i0 + i);
                uint64_t slot = o;
                if constexpr (!DIRECT) {
                    const unsigned long long key = o + 1;
                    slot = mix64(o) & tmask;
                    while (tkeys[slot] != key) slot = (slot + 1) & tmask;   // inserted by seq_candidates
                }
                isnew |= tvals[slot] == (uint32_t)j ? 1u : 0u;
                if (j < limit) {
                    const uint32_t bit = 1u << ((uint32_t)(o ^ 7u) & 31u);
                    if (g.dirty) g.dirty[o >> kDirtyShiftBits] = 1;
                    if (g.flips) {   // the bit flips once: reported by the one OR that set it (a key
                                     // may probe one bit twice, and later keys probe it too)
                        const uint32_t old = __hip_atomic_fetch_or(g.bits + (o >> 5), bit, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT);
                        if (!(old & bit)) {
                            const unsigned long long at = atomicAdd(g.flip_count, 1ull);
                            if (at < g.flip_cap) g.flips[at] = o | g.flip_tag;
                        }
                    } else {
                        __hip_atomic_fetch_or(g.bits + (o >> 5), bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
        }
        if (out8) out8[j] = (uint8_t)isnew;
    }
    if (any_flag) report_any_new(any_flag, isnew != 0 && j < limit);
}

// ---- Binned form: the first-index table in LDS, one workgroup per region of the filter ----
// The direct form's table (one uint32 per filter bit) is 44 MB for the 1M-entry Lua layer, and
// every 0-probe is a random device atomicMin into it (0.99 GB of fills for
// 7.3M probes).  For filters of at most kSeqMaxRegions regions of 2^14 bits the batch's
// 0-probes are binned by region instead, and each region builds its part of the table in LDS
// (2^14 uint32 = 64 KB):
//   seq_bin_count  hash; digest + 0-probe mask per key; per-region counts (LDS, then one device
//                  atomic per workgroup and region);
//   seq_bin_scan   region bases (one workgroup);
//   seq_bin_place  every 0-probe as (j << 14 | bit within the region) at its region's next slot;
//   seq_region     (the mark) first[] by LDS atomicMin, then new(j) = (first[b] == j), and bit
//                  b ORed into the region's LDS image when first[b] == j < limit (a bit whose
//                  first key is at or past the limit is set by no key before it).
// Within a region the order of the entries is free: min and OR commute.
constexpr uint32_t kSeqRegionLog2 = 14;
constexpr uint32_t kSeqRegionBits = 1u << kSeqRegionLog2;
constexpr uint32_t kSeqRegionWords = kSeqRegionBits / 32;
constexpr uint32_t kSeqMaxRegions = 8192;       // filters of up to 2^27 bits
constexpr uint32_t kSeqBinSub = 4;              // 256-key tiles per binning workgroup
constexpr uint64_t kSeqBinnedMinKeys = 4096;    // smaller batches: the direct / hash forms (fewer launches)
constexpr uint32_t kSeqRegionLanes = 1024;

bool seq_binned(uint64_t n, uint64_t m) {
    return n >= kSeqBinnedMinKeys && m <= ((uint64_t)kSeqMaxRegions << kSeqRegionLog2);
}

uint32_t seq_regions(uint64_t m) { return (uint32_t)((m + kSeqRegionBits - 1) >> kSeqRegionLog2); }

__global__ __launch_bounds__(kSeqTile) void seq_bin_count_kernel(BfGeom g, uint32_t i0,
                                                                 const uint8_t* __restrict__ keys16,
                                                                 const uint64_t* __restrict__ offsets, uint64_t bias,
                                                                 uint64_t n, uint32_t nreg,
                                                                 uint4* __restrict__ digests,
                                                                 unsigned long long* __restrict__ cand,
                                                                 uint32_t* __restrict__ counts) {
    __shared__ uint64_t s_off[kSeqTile + 1];
    __shared__ uint4 s_stage[kSeqStageVec + kStageSlackVec];
    extern __shared__ uint32_t s_cnt[];   // nreg
    for (uint32_t r = threadIdx.x; r < nreg; r += kSeqTile) s_cnt[r] = 0;   // ordered by for_key_tile's barrier
    for (uint32_t sub = 0; sub < kSeqBinSub; ++sub) {
        const uint64_t tile0 = ((uint64_t)blockIdx.x * kSeqBinSub + sub) * kSeqTile;
        if (tile0 >= n) break;   // workgroup-uniform
        const uint32_t cnt = (uint32_t)((n - tile0) < (uint64_t)kSeqTile ? (n - tile0) : kSeqTile);
        for_key_tile<kSeqTile, kSeqStageVec>(keys16, offsets, bias, tile0, cnt, s_off, s_stage, g.key_status,
            [&](auto staged, uint32_t lane, const uint32_t* src, uint32_t s, uint32_t L) {
                uint32_t H[5];
                sha1_any<decltype(staged)::value>(src, s, L, H);
                const uint32_t j = (uint32_t)(tile0 + lane);
                digests[j] = make_uint4(H[0], H[1], H[2], H[3]);
                unsigned long long cm = 0;
                for (uint32_t i = 0; i < g.k; ++i) {
                    const uint64_t o = probe_offset(g, H[0], H[1], H[2], H[3], i0 + i);
                    if ((g.bits[o >> 5] >> ((uint32_t)(o ^ 7u) & 31u)) & 1u) continue;
                    cm |= 1ull << i;
                    atomicAdd(&s_cnt[(uint32_t)(o >> kSeqRegionLog2)], 1u);
                }
                cand[j] = cm;
            });
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < nreg; r += kSeqTile)
        if (s_cnt[r]) atomicAdd(counts + r, s_cnt[r]);
}

// base[r] = cursor[r] = the exclusive prefix sum of counts (nreg <= 8192: 8 per lane).
__global__ __launch_bounds__(1024) void seq_bin_scan_kernel(const uint32_t* __restrict__ counts, uint32_t nreg,
                                                            uint32_t* __restrict__ base,
                                                            uint32_t* __restrict__ cursor) {
    __shared__ uint32_t s_sum[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nreg + 1023) / 1024;
    const uint32_t r0 = min(t * per, nreg), r1 = min(r0 + per, nreg);
    uint32_t loc = 0;
    for (uint32_t r = r0; r < r1; ++r) loc += counts[r];
    s_sum[t] = loc;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {   // inclusive Hillis-Steele scan
        const uint32_t v = t >= d ? s_sum[t - d] : 0u;
        __syncthreads();
        s_sum[t] += v;
        __syncthreads();
    }
    uint32_t run = s_sum[t] - loc;
    for (uint32_t r = r0; r < r1; ++r) {
        base[r] = run;
        cursor[r] = run;
        run += counts[r];
    }
}

__global__ __launch_bounds__(kSeqTile) void seq_bin_place_kernel(BfGeom g, uint32_t i0, uint64_t n, uint32_t nreg,
                                                                 const uint4* __restrict__ digests,
                                                                 const unsigned long long* __restrict__ cand,
                                                                 uint32_t* __restrict__ cursor,
                                                                 unsigned long long* __restrict__ entries) {
    extern __shared__ uint32_t s_at[];   // nreg: counts, then the workgroup's next slot per region
    for (uint32_t r = threadIdx.x; r < nreg; r += kSeqTile) s_at[r] = 0;
    uint4 Hq[kSeqBinSub];
    unsigned long long cq[kSeqBinSub];
    const uint64_t j0 = (uint64_t)blockIdx.x * kSeqBinSub * kSeqTile + threadIdx.x;
#pragma unroll
    for (uint32_t q = 0; q < kSeqBinSub; ++q) {
        const uint64_t j = j0 + (uint64_t)q * kSeqTile;
        cq[q] = j < n ? cand[j] : 0ull;
        Hq[q] = cq[q] ? digests[j] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kSeqBinSub; ++q)
        for (unsigned long long cm = cq[q]; cm; cm &= cm - 1) {
            const uint64_t o = probe_offset(g, Hq[q].x, Hq[q].y, Hq[q].z, Hq[q].w, i0 + (uint32_t)__builtin_ctzll(cm));
            atomicAdd(&s_at[(uint32_t)(o >> kSeqRegionLog2)], 1u);
        }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < nreg; r += kSeqTile)
        if (s_at[r]) s_at[r] = atomicAdd(cursor + r, s_at[r]);
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kSeqBinSub; ++q) {
        const unsigned long long j = j0 + (uint64_t)q * kSeqTile;
        for (unsigned long long cm = cq[q]; cm; cm &= cm - 1) {
            const uint64_t o = probe_offset(g, Hq[q].x, Hq[q].y, Hq[q].z, Hq[q].w, i0 + (uint32_t)__builtin_ctzll(cm));
            const uint32_t slot = atomicAdd(&s_at[(uint32_t)(o >> kSeqRegionLog2)], 1u);
            entries[slot] = (j << kSeqRegionLog2) | (o & (kSeqRegionBits - 1));
        }
    }
}

__global__ __launch_bounds__(kSeqRegionLanes) void seq_region_kernel(BfGeom g, uint64_t limit,
                                                                     const unsigned long long* __restrict__ d_limit,
                                                                     const uint32_t* __restrict__ base,
                                                                     const uint32_t* __restrict__ counts,
                                                                     const unsigned long long* __restrict__ entries,
                                                                     uint8_t* __restrict__ out8,
                                                                     uint32_t* __restrict__ any_flag) {
    __shared__ uint32_t s_first[kSeqRegionBits];
    __shared__ uint32_t s_img[kSeqRegionWords];
    if (d_limit) limit = min<uint64_t>(limit, *d_limit);
    const uint32_t r = blockIdx.x, t = threadIdx.x;
    const uint64_t w0 = (uint64_t)r * kSeqRegionWords;
    const uint32_t nw = (uint32_t)min<uint64_t>(kSeqRegionWords, (g.m + 31) / 32 - w0);
    const bool apply = limit > 0;   // launch-uniform
    uint4* f4 = reinterpret_cast<uint4*>(s_first);
    for (uint32_t v = t; v < kSeqRegionBits / 4; v += kSeqRegionLanes) f4[v] = make_uint4(~0u, ~0u, ~0u, ~0u);
    if (apply && t < nw) s_img[t] = g.bits[w0 + t];
    __syncthreads();
    const uint32_t beg = base[r], cnt = counts[r];
    for (uint32_t e = t; e < cnt; e += kSeqRegionLanes) {
        const unsigned long long x = entries[beg + e];
        atomicMin(&s_first[(uint32_t)x & (kSeqRegionBits - 1)], (uint32_t)(x >> kSeqRegionLog2));
    }
    __syncthreads();
    bool fresh = false;
    for (uint32_t e = t; e < cnt; e += kSeqRegionLanes) {
        const unsigned long long x = entries[beg + e];
        const uint32_t b = (uint32_t)x & (kSeqRegionBits - 1), j = (uint32_t)(x >> kSeqRegionLog2);
        if (s_first[b] != j) continue;
        if (out8) out8[j] = 1;
        if (j >= limit) continue;
        fresh = true;
        const uint32_t bit = 1u << ((b ^ 7u) & 31u);
        const uint32_t old = atomicOr(&s_img[b >> 5], bit);
        if (old & bit) continue;   // key j probes bit b twice: the other entry reports it
        const uint64_t o = ((uint64_t)r << kSeqRegionLog2) | b;
        if (g.dirty) g.dirty[o >> kDirtyShiftBits] = 1;
        if (g.flips) {   // the bit flips once, reported by its first key
            const unsigned long long at = atomicAdd(g.flip_count, 1ull);
            if (at < g.flip_cap) g.flips[at] = o | g.flip_tag;
        }
    }
    if (any_flag) report_any_new(any_flag, fresh);
    if (!apply) return;
    __syncthreads();
    if (t < nw) g.bits[w0 + t] = s_img[t];
}

uint64_t align256(uint64_t x) { return (x + 255) & ~(uint64_t)255; }

struct SeqBinCarve {
    uint32_t *counts, *base, *cursor;
    uint4* digests;
    unsigned long long *cand, *entries;
    uint32_t nreg;
};

SeqBinCarve seq_bin_carve(void* scratch, uint64_t n, uint32_t k, uint64_t m) {
    SeqBinCarve c{};
    c.nreg = seq_regions(m);
    uint8_t* at = static_cast<uint8_t*>(scratch);
    c.counts = reinterpret_cast<uint32_t*>(at);
    at += align256(c.nreg * 4ull);
    c.base = reinterpret_cast<uint32_t*>(at);
    at += align256(c.nreg * 4ull);
    c.cursor = reinterpret_cast<uint32_t*>(at);
    at += align256(c.nreg * 4ull);
    c.digests = reinterpret_cast<uint4*>(at);
    at += align256(n * 16);
    c.cand = reinterpret_cast<unsigned long long*>(at);
    at += align256(n * 8);
    c.entries = reinterpret_cast<unsigned long long*>(at);
    (void)k;
    return c;
}

uint64_t seq_bin_scratch_bytes(uint64_t n, uint32_t k, uint64_t m) {
    return 3 * align256(seq_regions(m) * 4ull) + align256(n * 16) + align256(n * 8) + align256(n * k * 8);
}

struct SeqCarve {
    unsigned long long* tkeys;
    uint32_t* tvals;
    uint4* digests;
    unsigned long long* cand;
    uint64_t slots;
};

// The hash table's slots for n keys of k probes (at most half full).
uint64_t seq_slots(uint64_t n, uint32_t k) {
    uint64_t s = 1024;
    while (s < 2 * n * (uint64_t)k) s <<= 1;
    return s;
}

// One uint32 per filter bit when that table is no bigger than the hash table (12 B per slot),
// so neither its clear nor the scratch grows, and at most 1 GiB: the Lua layout's 1M-scale
// layers (11M bits = 44 MB against a 16M-slot, 192 MB table for a 2^20-key chunk), small
// filters under big batches.  Probe updates are then one atomicMin each, with no claim loop.
// (the old bound let the direct table reach twice the hash table's bytes.)
bool seq_direct(uint64_t n, uint32_t k, uint64_t m) {
    return m <= (1ull << 28) && 4 * m <= 12 * seq_slots(n, k);
}

SeqCarve seq_carve(void* scratch, uint64_t n, uint32_t k, uint64_t m) {
    SeqCarve c{};
    uint8_t* at = static_cast<uint8_t*>(scratch);
    if (seq_direct(n, k, m)) {
        c.slots = m;
        c.tkeys = nullptr;
        c.tvals = reinterpret_cast<uint32_t*>(at);
        at += align256(m * 4);
    } else {
        c.slots = seq_slots(n, k);
        c.tkeys = reinterpret_cast<unsigned long long*>(at);
        at += align256(c.slots * 8);
        c.tvals = reinterpret_cast<uint32_t*>(at);
        at += align256(c.slots * 4);
    }
    c.digests = reinterpret_cast<uint4*>(at);
    at += align256(n * 16);
    c.cand = reinterpret_cast<unsigned long long*>(at);
    return c;
}

}  // namespace

uint64_t bf_seq_chunk_keys(uint32_t k) {
    const uint64_t c = (1ull << 25) / (k ? k : 1);   // table <= 2^26 slots (768 MiB)
    return c < (1ull << 22) ? (c ? c : 1) : (1ull << 22);
}

uint64_t bf_seq_scratch_bytes(uint64_t n, uint32_t k, uint64_t m) {
    if (seq_binned(n, m)) return seq_bin_scratch_bytes(n, k, m);
    const uint64_t tab = seq_direct(n, k, m) ? align256(m * 4) : align256(seq_slots(n, k) * 8) + align256(seq_slots(n, k) * 4);
    return tab + align256(n * 16) + align256(n * 8);
}

hipError_t bf_launch_seq_candidates(const BfGeom& g, uint32_t i0, const uint8_t* keys16, const uint64_t* offsets,
                                    uint64_t bias, uint64_t n, void* scratch, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipError_t e;
    if (seq_binned(n, g.m)) {
        const SeqBinCarve c = seq_bin_carve(scratch, n, g.k, g.m);
        if ((e = hipMemsetAsync(c.counts, 0, c.nreg * 4ull, s)) != hipSuccess) return e;
        const uint32_t wgs = (uint32_t)((n + kSeqBinSub * kSeqTile - 1) / (kSeqBinSub * kSeqTile));
        const size_t lds = c.nreg * sizeof(uint32_t);
        hipLaunchKernelGGL(seq_bin_count_kernel, dim3(wgs), dim3(kSeqTile), lds, s, g, i0, keys16, offsets, bias, n,
                           c.nreg, c.digests, c.cand, c.counts);
        hipLaunchKernelGGL(seq_bin_scan_kernel, dim3(1), dim3(1024), 0, s, c.counts, c.nreg, c.base, c.cursor);
        hipLaunchKernelGGL(seq_bin_place_kernel, dim3(wgs), dim3(kSeqTile), lds, s, g, i0, n, c.nreg, c.digests,
                           c.cand, c.cursor, c.entries);
        return hipGetLastError();
    }
    const SeqCarve c = seq_carve(scratch, n, g.k, g.m);
    if (c.tkeys && (e = hipMemsetAsync(c.tkeys, 0, c.slots * 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(c.tvals, 0xFF, c.slots * 4, s)) != hipSuccess) return e;
    const uint32_t blocks = (uint32_t)((n + kSeqTile - 1) / kSeqTile);
    if (c.tkeys)
        hipLaunchKernelGGL(seq_candidates_kernel<false>, dim3(blocks), dim3(kSeqTile), 0, s, g, i0, keys16, offsets,
                           bias, n, c.tkeys, c.tvals, c.slots - 1, c.digests, c.cand);
    else
        hipLaunchKernelGGL(seq_candidates_kernel<true>, dim3(blocks), dim3(kSeqTile), 0, s, g, i0, keys16, offsets,
                           bias, n, c.tkeys, c.tvals, 0, c.digests, c.cand);
    return hipGetLastError();
}

hipError_t bf_launch_seq_mark(const BfGeom& g, uint32_t i0, uint64_t n, uint64_t limit, void* scratch, uint8_t* out8,
                              uint32_t* any_flag, hipStream_t s, const unsigned long long* d_limit) {
    if (n == 0) return hipSuccess;
    if (seq_binned(n, g.m)) {   // the region kernel writes only the 1s of out8
        const SeqBinCarve c = seq_bin_carve(scratch, n, g.k, g.m);
        hipError_t e;
        if (out8 && (e = hipMemsetAsync(out8, 0, n, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(seq_region_kernel, dim3(c.nreg), dim3(kSeqRegionLanes), 0, s, g, limit, d_limit, c.base,
                           c.counts, c.entries, out8, any_flag);
        return hipGetLastError();
    }
    const SeqCarve c = seq_carve(scratch, n, g.k, g.m);
    if (c.tkeys)
        hipLaunchKernelGGL(seq_mark_kernel<false>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, g, i0, n, limit,
                           d_limit, c.tkeys, c.tvals, c.slots - 1, c.digests, c.cand, out8, any_flag);
    else
        hipLaunchKernelGGL(seq_mark_kernel<true>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, g, i0, n, limit,
                           d_limit, c.tkeys, c.tvals, 0, c.digests, c.cand, out8, any_flag);
    return hipGetLastError();
}

hipError_t bf_launch_insert_seq(const BfGeom& g, const uint8_t* keys16, const uint64_t* offsets, uint64_t bias,
                                uint64_t n, void* scratch, uint8_t* out8, uint32_t* any_flag, hipStream_t s,
                                BfMarks* mk) {
    hipError_t e = bf_launch_seq_candidates(g, 0, keys16, offsets, bias, n, scratch, s);
    if (e != hipSuccess) return e;
    bf_mark(mk, s, "seq_candidates");
    e = bf_launch_seq_mark(g, 0, n, n, scratch, out8, any_flag, s);
    bf_mark(mk, s, "seq_mark");
    return e;
}
