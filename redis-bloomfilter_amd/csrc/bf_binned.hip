// bf_binned.hip — binned ("sweep") insert and include? for filters far larger than L2.
//
// The direct kernels (bf_kernels.hip) cost every probe a random 128-B DRAM
// line fill (plus, for insert, a memory-side atomic per bit still 0).  When a
// batch carries many probes per filter line, streaming the filter once is far
// cheaper.  This path sorts the batch's probes by filter region and then walks
// the filter region by region, each region held in LDS:
//
//   1. bin_front    hashes every key (ruby.rb:41-55 derivation, shared with the
//                   direct kernels) and, per tile of 1024-2048 keys, counting-
//                   sorts the tile's probes by superbin (2^rel consecutive
//                   regions) in LDS.  The sorted tile is written contiguously at
//                   its fixed place (tile * keys * k), with a table of its
//                   superbin run boundaries; each workgroup also totals its
//                   probes per superbin.  include? carries each probe's key
//                   index and presets the answers to 1.
//   2. bin_group_sum / bin_group_scan: superbin totals per group of 64
//                   front workgroups; the exclusive prefix over (superbin,
//                   group) gives each group's window in the level-2 array, cut
//                   into chunk blocks of 8192 probes.
//   3. bin_mid      one workgroup per chunk block gathers its probes from the
//                   superbin's runs in the group's tiles, counting-sorts them by
//                   region in LDS and writes the block contiguously (region-local
//                   offsets) with its table of region boundaries.
//   4. bin_apply    (insert) one workgroup per region gathers the region's run
//                   from every chunk block of its superbin, ORs the probes into
//                   an LDS image of the region, then read-OR-writes the touched
//                   16-B vectors of the bitset — plain stores: no other
//                   workgroup owns the region.
//      bin_test     (include?) loads the region into LDS and clears the answer
//                   of every key with a probe on a 0 bit.
// The insert result equals atomic OR (idempotent, commutative); the include?
// answer is the AND of the key's k bits (ruby.rb:20-30) without the early exit.
#include "bf_device.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

using namespace bfdev;

namespace {
// Level-1 (bin_front) and level-2 (bin_mid) staging stores are non-temporal: each array is
// read back once by the next pass, and nt stores keep the filter's lines in the caches
// (measured: bin_front 0.59 -> 0.575 ms, bin_apply 0.53 -> 0.50 ms).
__device__ __forceinline__ void stage_store(uint32_t* p, uint32_t v) { __builtin_nontemporal_store(v, p); }
}  // namespace

namespace {

constexpr int kTile = 1024;                   // lanes per workgroup of the front / mid passes
constexpr int kStageVec = 16384 / 16;         // 16 KiB LDS key stage per 1024-key sub-tile
// superbins of the front pass (LDS counters; a sort tag is (superbin << 16) | rank).  512 with
// run lengths balanced between the front and bin_mid (416 superbins at 10B) measured slower:
// 10B step 6.85 vs 6.55 ms
constexpr uint32_t kMaxSup = 256;
constexpr uint32_t kMaxOwners = 256;          // route buckets / windows (owner x sub-range)
constexpr uint32_t kChunkBuckets = 512;       // route sort buckets of chunked windows (window x superbin x 2^sub2)
// <= 512 regions per superbin: the reach-capped 10B / 200B bitsets (55.8e9 bits) then take
// 2^19-bit regions (64 KiB of LDS, two apply workgroups per CU) instead of 2^20 (one):
// bin_apply 2.65 -> 2.48 ms per 2^24 x 13 probes (r02)
constexpr uint32_t kMaxRel = 9;
constexpr uint32_t kMaxBlocks = 512;          // front workgroups before tiles per workgroup grow
// front workgroups once they hold kMaxTilesPerBlock tiles each: 16384 x 16 tiles takes a
// merged replicated insert (8 ranks x 2^24 keys at k = 13, 10B@0.01 %) in ONE pass, so the
// bitset is streamed by one apply instead of one per sub-batch
constexpr uint32_t kMaxFrontBlocks = 16384;
constexpr uint32_t kGroupBlocks = 64;         // front workgroups per group (one wave in bin_group_sum)
constexpr uint32_t kTileProbes = 12288;       // probes per front tile (LDS sort buffer)
constexpr int kSlots = 12;                    // probes per lane per tile (k <= 12)
constexpr int kWideSlots = 16;                // ... for 12 < k <= 16 (one key per lane, 1 workgroup per CU)
constexpr uint32_t kTwoKeys = 6;              // k <= 6: two keys per lane per tile
constexpr uint32_t kMaxTilesPerBlock = 16;    // <= 1024 tiles per group: one run-table pass in bin_mid
constexpr uint32_t kBlockProbes = 8192;       // probes per level-2 chunk block (one bin_mid workgroup)
constexpr int kChunkPerLane = kBlockProbes / kTile;
constexpr uint32_t kRunsPerPass = 1024;       // run-table entries per gather pass (one lane each)
constexpr uint32_t kMidBuckets = 128;         // bin_mid sort buckets per block (>= regions per superbin)
constexpr uint32_t kMidParts = 2;             // bin_mid workgroups per level-2 window (1 and 4: same time)
constexpr uint32_t kApplyLanes = 1024;
constexpr uint32_t kPipeLanes = 1024;         // bin_apply_pipe_kernel: one workgroup per CU

// Exclusive prefix sum of v over the workgroup (blockDim.x a multiple of 64,
// at most 1024 lanes); *total gets the workgroup sum.  s_w: 16 words of LDS.
// Contains barriers: every lane must call it.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t x = wave_incl_scan(v);
    if (lane == 63u) s_w[wid] = x;
    __syncthreads();
    if (wid == 0) {
        const uint32_t s = wave_incl_scan(lane < nw ? s_w[lane] : 0u);
        if (lane < nw) s_w[lane] = s;   // inclusive wave totals
    }
    __syncthreads();
    const uint32_t r = (wid ? s_w[wid - 1] : 0u) + x - v;
    if (total) *total = s_w[nw - 1];
    __syncthreads();   // s_w may be reused right after
    return r;
}

// DIG: the keys arrive as their SHA-1 words (keys16 is then a uint4 array, 16 B per key,
// offsets unused): no staging, no hashing — the front pass is a partition pass.
template <bool KEYS, int SLOTS, bool DIG = false>
__device__ __forceinline__ void bin_front_body(BfGeom g, const uint8_t* __restrict__ keys16,
                                                          const uint64_t* __restrict__ offsets, uint64_t bias,
                                                          uint64_t n, uint32_t tile_keys, uint32_t tiles_per_block,
                                                          uint32_t sup_log2, uint32_t nsup,
                                                          uint32_t* __restrict__ level1,
                                                          uint32_t* __restrict__ level1_key,
                                                          uint16_t* __restrict__ stab, uint32_t* __restrict__ gcnt,
                                                          uint8_t* __restrict__ out8) {
    __shared__ uint64_t s_off[kTile + 1];
    __shared__ uint4 s_stage[kStageVec + kStageSlackVec];
    __shared__ uint32_t s_cnt[kMaxSup], s_lbase[kMaxSup], s_gcnt[kMaxSup];
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_sorted[kTile * SLOTS];
    __shared__ uint32_t s_key[KEYS ? kTile * SLOTS : 1];
    const uint32_t t = threadIdx.x;
    if (t < kMaxSup) {
        s_cnt[t] = 0;
        s_gcnt[t] = 0;
    }
    __syncthreads();
    const uint32_t k = g.k;
    const uint32_t kpl = tile_keys / kTile;   // 1 or 2 keys per lane
    const uint64_t smask = (1ull << sup_log2) - 1ull;
    const uint64_t ntiles = (n + tile_keys - 1) / tile_keys;
    const uint64_t tb0 = (uint64_t)blockIdx.x * tiles_per_block;
    const uint64_t tb1 = (tb0 + tiles_per_block < ntiles) ? tb0 + tiles_per_block : ntiles;
    for (uint64_t tile = tb0; tile < tb1; ++tile) {
        const uint64_t key0 = tile * tile_keys;
        const uint32_t tk = (uint32_t)((n - key0) < (uint64_t)tile_keys ? (n - key0) : tile_keys);
        uint4 H0 = make_uint4(0, 0, 0, 0), H1 = make_uint4(0, 0, 0, 0);
        if constexpr (DIG) {
            const uint4* dig = reinterpret_cast<const uint4*>(keys16);
            if (t < tk) H0 = dig[key0 + t];
            if (kTile + t < tk) H1 = dig[key0 + kTile + t];
        } else {
            for_key_tile<kTile, kStageVec>(keys16, offsets, bias, key0, tk < (uint32_t)kTile ? tk : kTile, s_off,
                                           s_stage, g.key_status, [&](auto staged, uint32_t, const uint32_t* src, uint32_t s, uint32_t L) {
                uint32_t H[5];
                sha1_any<decltype(staged)::value>(src, s, L, H);
                H0 = make_uint4(H[0], H[1], H[2], H[3]);
            });
            if (tk > (uint32_t)kTile) {   // workgroup-uniform: the second key of each lane
                for_key_tile<kTile, kStageVec>(keys16, offsets, bias, key0 + kTile, tk - kTile, s_off, s_stage,
                    g.key_status, [&](auto staged, uint32_t, const uint32_t* src, uint32_t s, uint32_t L) {
                        uint32_t H[5];
                        sha1_any<decltype(staged)::value>(src, s, L, H);
                        H1 = make_uint4(H[0], H[1], H[2], H[3]);
                    });
            }
        }
        const bool live0 = t < tk;
        const bool live1 = kpl == 2 && kTile + t < tk;
        if constexpr (KEYS) {   // include?: every answer starts true; bin_test clears it
            if (live0) out8[key0 + t] = 1;
            if (live1) out8[key0 + kTile + t] = 1;
        }
        // A: each probe -> (superbin, rank inside the tile's superbin run)
        uint32_t tag[SLOTS], loc[SLOTS];
#pragma unroll
        for (int q = 0; q < SLOTS; ++q) {
            const bool second = kpl == 2 && q >= (int)kTwoKeys;
            const uint32_t i = second ? (uint32_t)q - kTwoKeys : (uint32_t)q;
            const bool live = i < k && (second ? live1 : live0);
            tag[q] = 0xFFFFFFFFu;
            loc[q] = 0;
            if (live) {
                const uint4 H = second ? H1 : H0;
                const uint64_t o = probe_offset(g, H.x, H.y, H.z, H.w, i);
                const uint32_t sb = (uint32_t)(o >> sup_log2);
                tag[q] = (sb << 16) | atomicAdd(s_cnt + sb, 1u);
                loc[q] = (uint32_t)(o & smask);
            }
        }
        __syncthreads();
        // B: run boundaries of the tile (lane nsup writes the tile's probe count)
        const uint32_t c = t < kMaxSup ? s_cnt[t] : 0u;
        const uint32_t ex = block_excl_scan(c, s_w, nullptr);
        if (t <= nsup) stab[(uint64_t)t * ntiles + tile] = (uint16_t)ex;   // [superbin][tile]
        if (t < kMaxSup) {
            s_lbase[t] = ex;
            s_gcnt[t] += c;
            s_cnt[t] = 0;
        }
        __syncthreads();
        // C: counting sort in LDS
#pragma unroll
        for (int q = 0; q < SLOTS; ++q) {
            if (tag[q] != 0xFFFFFFFFu) {
                const uint32_t d = s_lbase[tag[q] >> 16] + (tag[q] & 0xFFFFu);
                s_sorted[d] = loc[q];
                if constexpr (KEYS) {
                    const bool second = kpl == 2 && q >= (int)kTwoKeys;
                    s_key[d] = (uint32_t)(key0 + (second ? kTile + t : t));
                }
            }
        }
        __syncthreads();
        // D: the sorted tile, contiguous at its fixed place
        const uint64_t seg = key0 * k;
        const uint32_t tp = tk * k;
        for (uint32_t j = t; j < tp; j += kTile) {
            stage_store(level1 + seg + j, s_sorted[j]);
            if constexpr (KEYS) level1_key[seg + j] = s_key[j];
        }
        // the next tile's first LDS writes (staging, then s_sorted) follow barriers
    }
    if (t < nsup) gcnt[(uint64_t)blockIdx.x * nsup + t] = s_gcnt[t];
}

// insert: 8 waves per SIMD (2 workgroups per CU: 77 KiB of LDS, <= 64 VGPRs)
template <bool DIG>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8)))
void bin_front_kernel(BfGeom g, const uint8_t* __restrict__ keys16, const uint64_t* __restrict__ offsets,
                      uint64_t bias, uint64_t n, uint32_t tile_keys, uint32_t tiles_per_block, uint32_t sup_log2,
                      uint32_t nsup, uint32_t* __restrict__ level1, uint32_t* __restrict__ level1_key,
                      uint16_t* __restrict__ stab, uint32_t* __restrict__ gcnt, uint8_t* __restrict__ out8) {
    bin_front_body<false, kSlots, DIG>(g, keys16, offsets, bias, n, tile_keys, tiles_per_block, sup_log2, nsup,
                                       level1, level1_key, stab, gcnt, out8);
}

// 12 < k <= 16: 16 probe slots per lane (64 KiB sort buffer, one workgroup per CU)
template <bool KEYS, bool DIG = false>
__global__ __launch_bounds__(kTile) void bin_front_wide_kernel(BfGeom g, const uint8_t* __restrict__ keys16,
                                                               const uint64_t* __restrict__ offsets, uint64_t bias,
                                                               uint64_t n, uint32_t tile_keys,
                                                               uint32_t tiles_per_block, uint32_t sup_log2,
                                                               uint32_t nsup, uint32_t* __restrict__ level1,
                                                               uint32_t* __restrict__ level1_key,
                                                               uint16_t* __restrict__ stab, uint32_t* __restrict__ gcnt,
                                                               uint8_t* __restrict__ out8) {
    bin_front_body<KEYS, kWideSlots, DIG>(g, keys16, offsets, bias, n, tile_keys, tiles_per_block, sup_log2, nsup,
                                          level1, level1_key, stab, gcnt, out8);
}

// ... from SHA-1 words (the pipelined insert at k > 12: 10B / 200B): no key stage, so 67 KiB
// of LDS, and capped at 64 VGPRs for two workgroups per CU
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8)))
void bin_front_wide_dig_kernel(BfGeom g, const uint8_t* __restrict__ keys16, const uint64_t* __restrict__ offsets,
                               uint64_t bias, uint64_t n, uint32_t tile_keys, uint32_t tiles_per_block,
                               uint32_t sup_log2, uint32_t nsup, uint32_t* __restrict__ level1,
                               uint32_t* __restrict__ level1_key, uint16_t* __restrict__ stab,
                               uint32_t* __restrict__ gcnt, uint8_t* __restrict__ out8) {
    bin_front_body<false, kWideSlots, true>(g, keys16, offsets, bias, n, tile_keys, tiles_per_block, sup_log2, nsup,
                                            level1, level1_key, stab, gcnt, out8);
}

// include?: key indices ride along (123 KiB of LDS: one workgroup per CU)
__global__ __launch_bounds__(kTile)
void bin_front_keys_kernel(BfGeom g, const uint8_t* __restrict__ keys16, const uint64_t* __restrict__ offsets,
                           uint64_t bias, uint64_t n, uint32_t tile_keys, uint32_t tiles_per_block, uint32_t sup_log2,
                           uint32_t nsup, uint32_t* __restrict__ level1, uint32_t* __restrict__ level1_key,
                           uint16_t* __restrict__ stab, uint32_t* __restrict__ gcnt, uint8_t* __restrict__ out8) {
    bin_front_body<true, kSlots>(g, keys16, offsets, bias, n, tile_keys, tiles_per_block, sup_log2, nsup, level1,
                                 level1_key, stab, gcnt, out8);
}

// Owner side of a partitioned filter: the probes arrive as shard-local offsets
// (already hashed and routed), so the front pass only sorts them by superbin,
// 12288 per tile, into the same level-1 layout bin_mid reads.
// KEYS (the binned shard test): each offset carries its input position, so the test pass
// can write the offset's answer byte.
// Window layout (wcounts != NULL, wcap a multiple of kTileProbes): tile t lies in window
// (t * kTileProbes) / wcap, whose entries past its live count min(wcounts[w * wstride], wcap)
// are skipped like the tail of a short last tile.
template <typename Off, bool KEYS>
__device__ __forceinline__ void bin_front_offsets_body(const Off* __restrict__ local, uint64_t count,
                                                       uint32_t tiles_per_block, uint32_t sup_log2, uint32_t nsup,
                                                       uint32_t* __restrict__ level1,
                                                       uint32_t* __restrict__ level1_key,
                                                       uint16_t* __restrict__ stab, uint32_t* __restrict__ gcnt,
                                                       uint64_t bias, const unsigned long long* __restrict__ wcounts,
                                                       uint32_t wstride, uint64_t wcap, uint64_t limit,
                                                       uint8_t* __restrict__ oob_out) {
    __shared__ uint32_t s_cnt[kMaxSup], s_lbase[kMaxSup], s_gcnt[kMaxSup];
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_sorted[kTileProbes];
    __shared__ uint16_t s_key[KEYS ? kTileProbes : 1];   // tile-relative input positions (< 2^14)
    const uint32_t t = threadIdx.x;
    if (t < kMaxSup) {
        s_cnt[t] = 0;
        s_gcnt[t] = 0;
    }
    __syncthreads();
    const uint64_t smask = (1ull << sup_log2) - 1ull;
    const uint64_t ntiles = (count + kTileProbes - 1) / kTileProbes;
    const bool vec_ok = (reinterpret_cast<uintptr_t>(local) & 15u) == 0;   // uniform
    static_assert(kTileProbes == kTile * kSlots, "a tile is kSlots entries per lane");
    const uint64_t tb0 = (uint64_t)blockIdx.x * tiles_per_block;
    const uint64_t tb1 = (tb0 + tiles_per_block < ntiles) ? tb0 + tiles_per_block : ntiles;
    for (uint64_t tile = tb0; tile < tb1; ++tile) {
        const uint64_t p0 = tile * kTileProbes;
        uint32_t tp = (uint32_t)((count - p0) < (uint64_t)kTileProbes ? (count - p0) : kTileProbes);
        if (wcounts) {
            const uint64_t w = p0 / wcap, i0 = p0 - w * wcap;
            uint64_t live = wcounts[w * wstride];
            if (live > wcap) live = 0;   // an overflowed window holds unwritten entries: skip it whole
            tp = live > i0 ? (uint32_t)(live - i0 < (uint64_t)tp ? live - i0 : tp) : 0u;
        }
        // Lane t takes entries [12t, 12t + 12): 48 (96) contiguous bytes, read as 16-B vectors
        // when the tile's buffer is aligned and the lane's entries are all live (the tail lane
        // and a misaligned caller buffer read entry by entry).
        uint32_t tag[kSlots], loc[kSlots];
        Off ent[kSlots];
        const uint32_t j0 = t * (uint32_t)kSlots;
        if (vec_ok && j0 + kSlots <= tp) {
            constexpr int kNV = kSlots * (int)sizeof(Off) / 16;
            const uint4* src = reinterpret_cast<const uint4*>(local + p0 + j0);
            uint4 vb[kNV];
#pragma unroll
            for (int v = 0; v < kNV; ++v) vb[v] = src[v];
            __builtin_memcpy(ent, vb, sizeof(ent));
        } else {
#pragma unroll
            for (int q = 0; q < kSlots; ++q) ent[q] = j0 + q < tp ? local[p0 + j0 + q] : (Off)0;
        }
#pragma unroll
        for (int q = 0; q < kSlots; ++q) {
            const uint32_t j = j0 + (uint32_t)q;
            tag[q] = 0xFFFFFFFFu;
            loc[q] = 0;
            if (j < tp) {
                const uint64_t o = (uint64_t)ent[q] + bias;
                if (o < limit) {
                    const uint32_t sb = (uint32_t)(o >> sup_log2);
                    tag[q] = (sb << 16) | atomicAdd(s_cnt + sb, 1u);
                    loc[q] = (uint32_t)(o & smask);
                } else if (oob_out) {   // an offset past the shard: dropped (insert), answered 0 (test)
                    oob_out[p0 + j] = 0;
                }
            }
        }
        __syncthreads();
        const uint32_t c = t < kMaxSup ? s_cnt[t] : 0u;
        const uint32_t ex = block_excl_scan(c, s_w, nullptr);
        if (t <= nsup) stab[(uint64_t)t * ntiles + tile] = (uint16_t)ex;   // [superbin][tile]
        if (t < kMaxSup) {
            s_lbase[t] = ex;
            s_gcnt[t] += c;
            s_cnt[t] = 0;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kSlots; ++q)
            if (tag[q] != 0xFFFFFFFFu) {
                const uint32_t d = s_lbase[tag[q] >> 16] + (tag[q] & 0xFFFFu);
                s_sorted[d] = loc[q];
                if constexpr (KEYS) s_key[d] = (uint16_t)(t * (uint32_t)kSlots + (uint32_t)q);
            }
        __syncthreads();
        for (uint32_t j = t; j < tp; j += kTile) {
            level1[p0 + j] = s_sorted[j];
            if constexpr (KEYS) level1_key[p0 + j] = (uint32_t)p0 + s_key[j];
        }
    }
    if (t < nsup) gcnt[(uint64_t)blockIdx.x * nsup + t] = s_gcnt[t];
}

template <typename Off>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8)))
void bin_front_offsets_kernel(const Off* __restrict__ local, uint64_t count, uint32_t tiles_per_block,
                              uint32_t sup_log2, uint32_t nsup, uint32_t* __restrict__ level1,
                              uint16_t* __restrict__ stab, uint32_t* __restrict__ gcnt, uint64_t bias,
                              const unsigned long long* __restrict__ wcounts, uint32_t wstride, uint64_t wcap,
                              uint64_t limit) {
    bin_front_offsets_body<Off, false>(local, count, tiles_per_block, sup_log2, nsup, level1, nullptr, stab, gcnt,
                                       bias, wcounts, wstride, wcap, limit, nullptr);
}

// 76 KiB of LDS (u16 positions): two workgroups per CU at 8 waves per SIMD, as the plain pass
template <typename Off>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8)))
void bin_front_offsets_keys_kernel(const Off* __restrict__ local, uint64_t count,
                                                                       uint32_t tiles_per_block, uint32_t sup_log2,
                                                                       uint32_t nsup, uint32_t* __restrict__ level1,
                                                                       uint32_t* __restrict__ level1_key,
                                                                       uint16_t* __restrict__ stab,
                                                                       uint32_t* __restrict__ gcnt, uint64_t bias,
                                                                       const unsigned long long* __restrict__ wcounts,
                                                                       uint32_t wstride, uint64_t wcap, uint64_t limit,
                                                                       uint8_t* __restrict__ out8) {
    bin_front_offsets_body<Off, true>(local, count, tiles_per_block, sup_log2, nsup, level1, level1_key, stab, gcnt,
                                      bias, wcounts, wstride, wcap, limit, out8);
}

// gsum[sb][q] = probes of superbin sb in the tiles of front workgroups [64q, 64q + 64).
// One workgroup per superbin, one wave per group (kMaxBlocks front workgroups per pass).
__global__ __launch_bounds__(kMaxBlocks) void bin_group_sum_kernel(const uint32_t* __restrict__ gcnt,
                                                                   uint32_t nblocks, uint32_t nsup, uint32_t nq,
                                                                   uint32_t* __restrict__ gsum) {
    const uint32_t sb = blockIdx.x;
    for (uint32_t w = threadIdx.x; w < nq * kGroupBlocks; w += kMaxBlocks) {   // wave-uniform bound
        uint32_t v = w < nblocks ? gcnt[(uint64_t)w * nsup + sb] : 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
        if ((w & 63u) == 0) gsum[sb * nq + w / kGroupBlocks] = v;
    }
}

// base[i]: exclusive prefix of gsum over windows i = (superbin, group); base[N] =
// all probes.  cb_base[i]: first chunk block of window i (ceil(size / kBlockProbes)
// blocks each), cb_base[N] = all blocks; cb_window[b] / cb_start[b]: the window
// and level-2 position of chunk block b.  One workgroup, kScanPer windows per lane, for
// N <= kScanWindows; larger N take the hierarchical scan below (launch_scan).
constexpr uint32_t kScanPer = 4;
constexpr uint32_t kScanWindows = 1024 * kScanPer;
constexpr uint32_t kLocalScanPer = 4;                 // groups per lane of bin_scan_local_kernel
constexpr uint32_t kMaxGroups = 1024 * kLocalScanPer; // groups per superbin
constexpr uint32_t kMaxWindows = kMaxSup * kMaxGroups;
__global__ __launch_bounds__(1024) void bin_group_scan_kernel(const uint32_t* __restrict__ gsum, uint32_t N,
                                                              uint32_t* __restrict__ base,
                                                              uint32_t* __restrict__ cb_base,
                                                              uint32_t* __restrict__ cb_window,
                                                              uint32_t* __restrict__ cb_start, uint32_t nq,
                                                              unsigned long long* __restrict__ totals) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_cb[kScanWindows + 1];
    const uint32_t t = threadIdx.x;
    uint32_t v[kScanPer], cv[kScanPer], sum = 0, csum = 0;
#pragma unroll
    for (uint32_t e = 0; e < kScanPer; ++e) {   // lane t owns windows [kScanPer t, kScanPer t + kScanPer)
        const uint32_t w = kScanPer * t + e;
        v[e] = w < N ? gsum[w] : 0u;
        cv[e] = (v[e] + kBlockProbes - 1) / kBlockProbes;
        sum += v[e];
        csum += cv[e];
    }
    uint32_t total, ctotal;
    uint32_t ex = block_excl_scan(sum, s_w, &total);
    uint32_t cex = block_excl_scan(csum, s_w, &ctotal);
#pragma unroll
    for (uint32_t e = 0; e < kScanPer; ++e) {
        const uint32_t w = kScanPer * t + e;
        if (w < N) {
            base[w] = ex;
            cb_base[w] = cex;
            s_cb[w] = cex;
            if (totals && v[e]) atomicAdd(totals + w / nq, (unsigned long long)v[e]);   // per-bucket totals
        }
        ex += v[e];
        cex += cv[e];
    }
    if (t == 0) {
        base[N] = total;
        cb_base[N] = ctotal;
        s_cb[N] = ctotal;
    }
    __syncthreads();
    // every block's window and level-2 start, all lanes over all blocks (a window
    // may hold thousands of blocks): the window is the last one starting at or
    // before the block
    for (uint32_t blk = t; blk < ctotal; blk += 1024) {
        uint32_t lo = 0, hi = N - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (s_cb[mid] <= blk) lo = mid; else hi = mid - 1;
        }
        cb_window[blk] = lo;
        cb_start[blk] = base[lo] + (blk - s_cb[lo]) * kBlockProbes;   // base: this workgroup's own stores
    }
}

// The same scan for N > kScanWindows windows, in three steps: per superbin over its groups
// (bin_scan_local), over the superbins (bin_scan_top), then every window's offsets and chunk
// blocks (bin_scan_fill).  stot: 2 words per superbin (its probes, its chunk blocks).
__global__ __launch_bounds__(1024) void bin_scan_local_kernel(const uint32_t* __restrict__ gsum, uint32_t nq,
                                                              uint32_t* __restrict__ base,
                                                              uint32_t* __restrict__ cb_base,
                                                              uint32_t* __restrict__ stot) {
    __shared__ uint32_t s_w[16];
    const uint32_t sb = blockIdx.x, t = threadIdx.x;
    uint32_t v[kLocalScanPer], cv[kLocalScanPer], sum = 0, csum = 0;
#pragma unroll
    for (uint32_t e = 0; e < kLocalScanPer; ++e) {
        const uint32_t q = kLocalScanPer * t + e;
        v[e] = q < nq ? gsum[(uint64_t)sb * nq + q] : 0u;
        cv[e] = (v[e] + kBlockProbes - 1) / kBlockProbes;
        sum += v[e];
        csum += cv[e];
    }
    uint32_t total, ctotal;
    uint32_t ex = block_excl_scan(sum, s_w, &total);
    uint32_t cex = block_excl_scan(csum, s_w, &ctotal);
#pragma unroll
    for (uint32_t e = 0; e < kLocalScanPer; ++e) {
        const uint32_t q = kLocalScanPer * t + e;
        if (q < nq) {
            base[(uint64_t)sb * nq + q] = ex;   // superbin-relative until bin_scan_fill
            cb_base[(uint64_t)sb * nq + q] = cex;
        }
        ex += v[e];
        cex += cv[e];
    }
    if (t == 0) {
        stot[2 * sb] = total;
        stot[2 * sb + 1] = ctotal;
    }
}

__global__ __launch_bounds__(1024) void bin_scan_top_kernel(uint32_t* __restrict__ stot, uint32_t nsup, uint32_t N,
                                                            uint32_t* __restrict__ base,
                                                            uint32_t* __restrict__ cb_base) {
    __shared__ uint32_t s_w[16];
    const uint32_t t = threadIdx.x;
    const uint32_t v = t < nsup ? stot[2 * t] : 0u, cv = t < nsup ? stot[2 * t + 1] : 0u;
    uint32_t total, ctotal;
    const uint32_t ex = block_excl_scan(v, s_w, &total);
    const uint32_t cex = block_excl_scan(cv, s_w, &ctotal);
    if (t < nsup) {
        stot[2 * t] = ex;
        stot[2 * t + 1] = cex;
    }
    if (t == 0) {
        base[N] = total;
        cb_base[N] = ctotal;
    }
}

__global__ __launch_bounds__(256) void bin_scan_fill_kernel(const uint32_t* __restrict__ gsum, uint32_t N, uint32_t nq,
                                                            const uint32_t* __restrict__ stot,
                                                            uint32_t* __restrict__ base,
                                                            uint32_t* __restrict__ cb_base,
                                                            uint32_t* __restrict__ cb_window,
                                                            uint32_t* __restrict__ cb_start) {
    const uint32_t w = blockIdx.x * 256 + threadIdx.x;
    if (w >= N) return;
    const uint32_t sb = w / nq;
    const uint32_t b = base[w] + stot[2 * sb], cb = cb_base[w] + stot[2 * sb + 1];
    base[w] = b;
    cb_base[w] = cb;
    const uint32_t nb = (gsum[w] + kBlockProbes - 1) / kBlockProbes;
    for (uint32_t j = 0; j < nb; ++j) {
        cb_window[cb + j] = w;
        cb_start[cb + j] = b + j * kBlockProbes;
    }
}

// Last run whose start is <= f in an LDS run table of nt >= 1 ascending starts.
__device__ __forceinline__ uint32_t run_of(const uint32_t* s_pre, uint32_t nt, uint32_t f) {
    uint32_t lo = 0, hi = nt - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_pre[mid] <= f) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Rank of this lane's probe among the tile's probes to `owner`, taken with ONE LDS atomic
// per (wave, owner) instead of one per probe: with few owners (P <= g.route_agg) every lane
// of a wave would otherwise hit the same few LDS words (P = 1: all of them).  Loops over the
// distinct owners present in the wave.  Every lane of the wave must call it.
__device__ __forceinline__ uint32_t wave_agg_rank(bool live, uint32_t owner, uint32_t* s_cnt) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = (1ull << lane) - 1ull;
    uint64_t pending = __ballot(live);
    uint32_t rank = 0;
    while (pending) {   // wave-uniform
        const int leader = __builtin_ctzll(pending);
        const uint32_t o = (uint32_t)__shfl((int)owner, leader);
        const bool mine = live && owner == o;
        const uint64_t grp = __ballot(mine);
        uint32_t base = 0;
        if ((int)lane == leader) base = atomicAdd(s_cnt + o, (uint32_t)__popcll(grp));
        base = (uint32_t)__shfl((int)base, leader);
        if (mine) rank = base + (uint32_t)__popcll(grp & below);
        pending &= ~grp;
    }
    return rank;
}

// Requester side of a partitioned filter (bf_route_dev): hash, then per tile an
// LDS counting sort of the tile's probes by owner shard (block-cyclic map of
// include/bfhip.h), written contiguously at the tile's fixed place with the
// tile's owner run table [owner][tile]; per-workgroup owner totals.  WIDE: the
// owner-local offsets need more than 32 bits (their high byte is kept apart);
// SLOT: each probe carries its key index.
//
// WIN (bf_route_windows_dev): no tile-major level 1, group scan or gather pass.  Each tile
// claims room for its owner-s run in owner s's fixed window of the send buffer with one
// global atomic per (tile, owner) on wcounts[s], and writes the run straight there
// (entries [s*wcap, s*wcap + wcounts[s]) in an unspecified order; slots ride along).  A run
// that would pass wcap is dropped; wcounts[s] still ends at the owner's full total, so
// the caller sees the overflow and re-routes through the contiguous path.
//
// CHUNK (bf_route_chunks_dev): as WIN, but each tile's run for a window is itself sorted by
// the owner's superbin (superbin = sub-range-local offset >> cg.sup_log2, cg.S per window),
// and the tile records its chunk in the window's directory: the run's place in the window
// and its superbin run table (BfChunks).  The owner then reads the received windows as a
// level-1 array of chunks and skips its own front (sort) pass; slots are u16, tile-relative.
template <bool WIDE, bool SLOT, int SLOTS, bool WIN, bool CHUNK = false, bool DIG = false>
__device__ __forceinline__ void route_front_body(BfGeom g, const uint8_t* __restrict__ keys16,
                                                 const uint64_t* __restrict__ offsets, uint64_t bias,
                                                 uint64_t n, uint32_t tile_keys, uint32_t tiles_per_block,
                                                 uint32_t P, uint32_t* __restrict__ lo1,
                                                 uint8_t* __restrict__ hi1, uint32_t* __restrict__ key1,
                                                 uint16_t* __restrict__ stab,
                                                 uint32_t* __restrict__ gcnt, uint64_t wcap,
                                                 unsigned long long* __restrict__ wcounts,
                                                 void* __restrict__ wsend, uint32_t* __restrict__ wslot,
                                                 uint32_t nh, BfChunks cg = BfChunks{}) {
    // The key stage (offsets + bytes) is dead once the tile is hashed, so the sorted
    // tile-relative key indices (u16) reuse it: 76 KiB in all without WIDE, two
    // workgroups per CU.
    constexpr uint32_t kOffVec = (8 * (kTile + 1) + 15) / 16;
    constexpr uint32_t kStageRaw = kOffVec + kStageVec + kStageSlackVec;
    constexpr uint32_t kKeyRaw = (kTile * SLOTS * 2 + 15) / 16;
    constexpr uint32_t kRawVec = SLOT && kKeyRaw > kStageRaw ? kKeyRaw : kStageRaw;
    __shared__ uint4 s_raw[kRawVec];
    uint64_t* s_off = reinterpret_cast<uint64_t*>(s_raw);
    uint4* s_stage = s_raw + kOffVec;
    uint16_t* s_key = reinterpret_cast<uint16_t*>(s_raw);
    // CHUNK: up to kChunkBuckets (window, superbin, low bits) buckets; the window route keeps
    // no per-workgroup totals (s_gcnt), which keeps the LDS within two workgroups per CU
    constexpr uint32_t NB = CHUNK ? kChunkBuckets : kMaxOwners;
    __shared__ uint32_t s_cnt[NB], s_lbase[NB], s_gcnt[WIN ? 1 : kMaxOwners];
    __shared__ uint32_t s_w[16];
    __shared__ unsigned long long s_gbase[WIN ? kMaxOwners : 1];
    __shared__ uint32_t s_obase[WIN ? kMaxOwners : 1];
    // WIN: ~128 sort buckets however few the owners, so that the LDS rank atomics do not
    // all land on P words (the owner's buckets stay consecutive: one run per owner)
    uint32_t sub_log2 = 0;
    if constexpr (CHUNK)
        sub_log2 = cg.sub2;   // buckets (window, superbin, low offset bits): P * S << sub2 <= kMaxSup
    else if constexpr (WIN)
        while ((P << (sub_log2 + 1)) <= 128u) ++sub_log2;
    const uint32_t wS = CHUNK ? cg.S : 1u;   // a window's first bucket: (w * wS) << sub_log2
    __shared__ uint32_t s_lo[kTile * SLOTS];
    __shared__ uint8_t s_hi[WIDE ? kTile * SLOTS : 1];
    const uint32_t t = threadIdx.x;
    if (t < NB) s_cnt[t] = 0;
    if constexpr (!WIN)
        if (t < kMaxOwners) s_gcnt[t] = 0;
    __syncthreads();
    const uint32_t k = g.k;
    const uint32_t kpl = tile_keys / kTile;
    const uint64_t ntiles = (n + tile_keys - 1) / tile_keys;
    const uint64_t tb0 = (uint64_t)blockIdx.x * tiles_per_block;
    const uint64_t tb1 = (tb0 + tiles_per_block < ntiles) ? tb0 + tiles_per_block : ntiles;
    for (uint64_t tile = tb0; tile < tb1; ++tile) {
        const uint64_t key0 = tile * tile_keys;
        const uint32_t tk = (uint32_t)((n - key0) < (uint64_t)tile_keys ? (n - key0) : tile_keys);
        uint4 H0 = make_uint4(0, 0, 0, 0), H1 = make_uint4(0, 0, 0, 0);
        if constexpr (DIG) {   // the keys' SHA-1 words, hashed earlier (bf_route_chunks_digests_dev)
            const uint4* dg = reinterpret_cast<const uint4*>(keys16);
            if (t < tk) H0 = dg[key0 + t];
            if (kTile + t < tk) H1 = dg[key0 + kTile + t];
        } else {
        for_key_tile<kTile, kStageVec>(keys16, offsets, bias, key0, tk < (uint32_t)kTile ? tk : kTile, s_off, s_stage,
            g.key_status, [&](auto staged, uint32_t, const uint32_t* src, uint32_t s, uint32_t L) {
                uint32_t H[5];
                sha1_any<decltype(staged)::value>(src, s, L, H);
                H0 = make_uint4(H[0], H[1], H[2], H[3]);
            });
        if (tk > (uint32_t)kTile) {
            for_key_tile<kTile, kStageVec>(keys16, offsets, bias, key0 + kTile, tk - kTile, s_off, s_stage,
                g.key_status, [&](auto staged, uint32_t, const uint32_t* src, uint32_t s, uint32_t L) {
                    uint32_t H[5];
                    sha1_any<decltype(staged)::value>(src, s, L, H);
                    H1 = make_uint4(H[0], H[1], H[2], H[3]);
                });
        }
        }
        const bool live0 = t < tk;
        const bool live1 = kpl == 2 && kTile + t < tk;
        uint32_t tag[SLOTS], lo[SLOTS];
        uint8_t hi[SLOTS];
        // keys per lane as a compile-time constant (as bin_front_body): each slot's i is one
        auto probes = [&](auto kplc) {
        constexpr uint32_t KPL = decltype(kplc)::value;
#pragma unroll
        for (int q = 0; q < SLOTS; ++q) {
            const bool second = KPL == 2 && q >= (int)kTwoKeys;
            const uint32_t i = second ? (uint32_t)q - kTwoKeys : (uint32_t)q;
            const bool live = i < k && (second ? live1 : live0);
            tag[q] = 0xFFFFFFFFu;
            lo[q] = 0;
            hi[q] = 0;
            uint32_t owner = 0;
            if (live) {
                const uint4 H = second ? H1 : H0;
                uint64_t local;
                owner_local(g, probe_offset(g, H.x, H.y, H.z, H.w, i), owner, local);
                lo[q] = (uint32_t)local;
                hi[q] = (uint8_t)(local >> 32);
            }
            if constexpr (WIN) {   // bucket = (window, low offset bits): 2^sub_log2 LDS counters per window
                if (live) {
                    const uint32_t win = owner * nh + hi[q];   // window = (owner, 2^32-bit sub-range)
                    uint32_t wb = win;
                    if constexpr (CHUNK) {   // ... (window, owner superbin, low offset bits)
                        uint32_t sb = lo[q] >> cg.sup_log2;
                        if (sb >= cg.S) sb = cg.S - 1u;   // never for a valid offset (the geometry covers the shard)
                        wb = win * cg.S + sb;
                    }
                    const uint32_t bkt = (wb << sub_log2) | (lo[q] & ((1u << sub_log2) - 1u));
                    tag[q] = (bkt << 16) | atomicAdd(s_cnt + bkt, 1u);
                }
            } else if (P <= g.route_agg) {   // workgroup-uniform
                const uint32_t r = wave_agg_rank(live, owner, s_cnt);
                if (live) tag[q] = (owner << 16) | r;
            } else if (live) {
                tag[q] = (owner << 16) | atomicAdd(s_cnt + owner, 1u);
            }
        }
        };
        if (kpl == 2) probes(std::integral_constant<uint32_t, 2>{});
        else probes(std::integral_constant<uint32_t, 1>{});
        __syncthreads();
        const uint32_t c = t < NB ? s_cnt[t] : 0u;
        const uint32_t ex = block_excl_scan(c, s_w, nullptr);
        if constexpr (!WIN)
            if (t <= P) stab[(uint64_t)t * ntiles + tile] = (uint16_t)ex;   // [owner][tile]
        if (t < NB) {
            s_lbase[t] = ex;
            if constexpr (!WIN) s_gcnt[t] += c;
            s_cnt[t] = 0;
        }
        __syncthreads();
        if constexpr (WIN) {
            if (t < P) {   // claim this tile's owner-t run (its buckets, consecutive) in owner t's window
                const uint32_t lo_b = (t * wS) << sub_log2, hi_b = ((t + 1) * wS) << sub_log2;
                const uint32_t ob = s_lbase[lo_b], oc = (hi_b < NB ? s_lbase[hi_b] : tk * k) - ob;
                unsigned long long gb = 0;
                if constexpr (CHUNK) {
                    // one 64-bit atomic gives the run's place AND its rank among the window's runs
                    // (claims counted in the high bits): the owner then walks the runs in window
                    // order through the directory's rank table, with no sort (BfChunkIn::ranked)
                    if (oc) {
                        uint8_t* dw = cg.dir + (uint64_t)t * cg.dir_bytes;
                        const unsigned long long x = atomicAdd(
                            reinterpret_cast<unsigned long long*>(dw + bf_chunk_dir_claim_offset(cg, cg.tiles)),
                            (1ull << kClaimRankShift) | (unsigned long long)oc);
                        gb = x & ((1ull << kClaimRankShift) - 1ull);
                        reinterpret_cast<uint16_t*>(dw + bf_chunk_dir_rank_offset(cg, cg.tiles))
                            [x >> kClaimRankShift] = (uint16_t)(tile + 1u);   // 0: no run at that rank
                        atomicAdd(wcounts + t, (unsigned long long)oc);   // the window's live count
                    }
                } else if (oc) {
                    gb = atomicAdd(wcounts + t, (unsigned long long)oc);
                }
                s_gbase[t] = (gb + oc <= wcap) ? (unsigned long long)t * wcap + gb : ~0ull;   // ~0: overflow
                s_obase[t] = ob;
                if constexpr (CHUNK)   // the chunk's place in window t (0xFFFFFFFF: dropped, the window overflows)
                    reinterpret_cast<uint32_t*>(cg.dir + (uint64_t)t * cg.dir_bytes)[tile] =
                        (gb + oc <= wcap) ? (uint32_t)gb : 0xFFFFFFFFu;
            }
            if constexpr (CHUNK) {   // the chunk's superbin run table in every window: [sb][tile], [S] = length
                const uint32_t S1 = cg.S + 1u;
                for (uint32_t e = t; e < P * S1; e += kTile) {
                    const uint32_t w = e / S1, sb = e - w * S1;
                    const uint32_t b0 = (w * cg.S) << sub_log2, b1 = (w * cg.S + sb) << sub_log2;
                    const uint32_t v = (b1 < NB ? s_lbase[b1] : tk * k) - s_lbase[b0];
                    reinterpret_cast<uint16_t*>(cg.dir + (uint64_t)w * cg.dir_bytes + 4 * cg.tiles)
                        [(uint64_t)sb * cg.tiles + tile] = (uint16_t)v;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < SLOTS; ++q) {
            if (tag[q] != 0xFFFFFFFFu) {
                const uint32_t d = s_lbase[tag[q] >> 16] + (tag[q] & 0xFFFFu);
                s_lo[d] = lo[q];
                if constexpr (WIDE) s_hi[d] = hi[q];
                if constexpr (SLOT) {
                    const bool second = kpl == 2 && q >= (int)kTwoKeys;
                    s_key[d] = (uint16_t)(second ? kTile + t : t);
                }
            }
        }
        __syncthreads();
        const uint64_t seg = key0 * k;
        const uint32_t tp = tk * k;
        if constexpr (WIN) {
            // the window of sorted entry j: one search for the lane's first entry, then forward
            // steps (its entries are kTile apart, a window holds ~tp / P of them)
            uint32_t o = run_of(s_obase, P, t < tp ? t : 0u);
            for (uint32_t j = t; j < tp; j += kTile) {
                while (o + 1u < P && s_obase[o + 1u] <= j) ++o;
                const unsigned long long gb = s_gbase[o];   // the run's place in owner o's window
                if (gb != ~0ull) {
                    const uint64_t d = gb + (j - s_obase[o]);
                    static_cast<uint32_t*>(wsend)[d] = s_lo[j];   // the window implies the high bits
                    if constexpr (SLOT) {
                        if constexpr (CHUNK) reinterpret_cast<uint16_t*>(wslot)[d] = s_key[j];   // tile-relative
                        else wslot[d] = (uint32_t)key0 + s_key[j];
                    }
                }
            }
            __syncthreads();   // s_gbase and the staged keys are rewritten by the next tile
        } else {
            for (uint32_t j = t; j < tp; j += kTile) {
                lo1[seg + j] = s_lo[j];
                if constexpr (WIDE) hi1[seg + j] = s_hi[j];
                if constexpr (SLOT) key1[seg + j] = (uint32_t)key0 + s_key[j];
            }
            if constexpr (SLOT) __syncthreads();   // the next tile's staging overwrites s_key
        }
    }
    if constexpr (!WIN)
        if (t < P) gcnt[(uint64_t)blockIdx.x * P + t] = s_gcnt[t];
}

#define BF_ROUTE_FRONT_ARGS                                                                                     \
    BfGeom g, const uint8_t* __restrict__ keys16, const uint64_t* __restrict__ offsets, uint64_t bias, uint64_t n, \
        uint32_t tile_keys, uint32_t tiles_per_block, uint32_t P, uint32_t* __restrict__ lo1,                   \
        uint8_t* __restrict__ hi1, uint32_t* __restrict__ key1, uint16_t* __restrict__ stab,                     \
        uint32_t* __restrict__ gcnt, uint64_t wcap, unsigned long long* __restrict__ wcounts,                 \
        void* __restrict__ wsend, uint32_t* __restrict__ wslot, uint32_t nh
#define BF_ROUTE_FRONT_PASS \
    g, keys16, offsets, bias, n, tile_keys, tiles_per_block, P, lo1, hi1, key1, stab, gcnt, wcap, wcounts, wsend, wslot, nh
template <bool WIDE, bool SLOT, int SLOTS, bool WIN, bool CHUNK = false, bool DIG = false>
__global__ __launch_bounds__(kTile) void route_front_kernel(BF_ROUTE_FRONT_ARGS, BfChunks cg) {
    route_front_body<WIDE, SLOT, SLOTS, WIN, CHUNK, DIG>(BF_ROUTE_FRONT_PASS, cg);
}
// 32-bit offsets (shards of <= 2^32 bits): 76 KiB of LDS with or without slots, so two
// workgroups per CU at 8 waves per SIMD, as bin_front
template <bool SLOT, bool WIN, bool CHUNK = false, bool DIG = false>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8)))
void route_front32_kernel(BF_ROUTE_FRONT_ARGS, BfChunks cg) {
    route_front_body<false, SLOT, kSlots, WIN, CHUNK, DIG>(BF_ROUTE_FRONT_PASS, cg);
}
#undef BF_ROUTE_FRONT_PASS
#undef BF_ROUTE_FRONT_ARGS

// The chunked route from SHA-1 words (bf_route_chunks_digests_dev) in sorted-index form: the
// tile's LDS sort moves one u16 per probe — (key within the tile) << 4 | probe index — instead
// of its 32-bit offset and u16 slot, and the write loop derives the offset again from the key's
// words, which stay in LDS.  Same buckets, claims, directory and window contents as
// route_front_body<.., WIN, CHUNK, DIG>, whose sort buffers (72.8 KiB without slots, 105.5 KiB
// with, 92-102 VGPRs at k = 13) hold one workgroup per CU: here 56-72 KiB and <= 64 VGPRs make
// two, so one workgroup's claims and barriers hide behind the other's work.
// HASH (bf_route_chunks_dev, k > 12): the keys are hashed here, one per lane, their bytes staged
// in the index buffer (dead until the tile's scan).
template <bool SLOT, int SLOTS, bool HASH = false>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8)))
void route_chunks_idx_kernel(BfGeom g, const uint8_t* __restrict__ keys16, const uint64_t* __restrict__ offsets,
                             uint64_t bias, uint64_t n, uint32_t tile_keys,
                             uint32_t tiles_per_block, uint32_t P, uint64_t wcap,
                             unsigned long long* __restrict__ wcounts, uint32_t* __restrict__ wsend,
                             uint16_t* __restrict__ wslot, uint32_t nh, BfChunks cg) {
    static_assert(SLOTS <= 16 && kTile * SLOTS <= 65536, "a probe index is 4 bits, a sort slot 16");
    constexpr uint32_t NB = kChunkBuckets;
    constexpr uint32_t kOffVec = (8 * (kTile + 1) + 15) / 16;
    static_assert(!HASH || (SLOTS > kSlots && (kOffVec + kStageVec + kStageSlackVec) * 16 <= kTile * SLOTS * 2),
                  "the key stage fits the index buffer (one key per lane)");
    __shared__ uint4 s_idx4[kTile * SLOTS * 2 / 16];
    uint16_t* s_idx = reinterpret_cast<uint16_t*>(s_idx4);
    __shared__ uint4 s_dig[SLOTS > kSlots ? kTile : 2 * kTile];   // k > 12: one key per lane
    const uint4* dig = reinterpret_cast<const uint4*>(keys16);
    __shared__ uint32_t s_cnt[NB], s_lbase[NB];
    __shared__ uint32_t s_w[16];
    __shared__ unsigned long long s_gbase[kMaxOwners];
    __shared__ uint32_t s_obase[kMaxOwners];
    const uint32_t sub_log2 = cg.sub2, wS = cg.S;
    const uint32_t t = threadIdx.x;
    if (t < NB) s_cnt[t] = 0;
    __syncthreads();
    const uint32_t k = g.k;
    const uint32_t kpl = tile_keys / kTile;
    const uint64_t ntiles = (n + tile_keys - 1) / tile_keys;
    const uint64_t tb0 = (uint64_t)blockIdx.x * tiles_per_block;
    const uint64_t tb1 = (tb0 + tiles_per_block < ntiles) ? tb0 + tiles_per_block : ntiles;
    for (uint64_t tile = tb0; tile < tb1; ++tile) {
        const uint64_t key0 = tile * tile_keys;
        const uint32_t tk = (uint32_t)((n - key0) < (uint64_t)tile_keys ? (n - key0) : tile_keys);
        const bool live0 = t < tk;
        const bool live1 = kpl == 2 && kTile + t < tk;
        uint4 H0 = make_uint4(0, 0, 0, 0), H1 = make_uint4(0, 0, 0, 0);
        if constexpr (HASH) {   // kpl == 1
            for_key_tile<kTile, kStageVec>(keys16, offsets, bias, key0, tk, reinterpret_cast<uint64_t*>(s_idx4),
                                           s_idx4 + kOffVec, g.key_status,
                [&](auto staged, uint32_t, const uint32_t* src, uint32_t s0, uint32_t L) {
                    uint32_t H[5];
                    sha1_any<decltype(staged)::value>(src, s0, L, H);
                    H0 = make_uint4(H[0], H[1], H[2], H[3]);
                });
        } else {
            if (live0) H0 = dig[key0 + t];
            if (live1) H1 = dig[key0 + kTile + t];
        }
        s_dig[t] = H0;
        if (kpl == 2) s_dig[kTile + t] = H1;
        uint32_t tag[SLOTS];
        auto probes = [&](auto kplc) {
            constexpr uint32_t KPL = decltype(kplc)::value;
#pragma unroll
            for (int q = 0; q < SLOTS; ++q) {
                const bool second = KPL == 2 && q >= (int)kTwoKeys;
                const uint32_t i = second ? (uint32_t)q - kTwoKeys : (uint32_t)q;
                tag[q] = 0xFFFFFFFFu;
                if (i < k && (second ? live1 : live0)) {
                    const uint4 H = second ? H1 : H0;
                    uint32_t owner;
                    uint64_t local;
                    owner_local(g, probe_offset(g, H.x, H.y, H.z, H.w, i), owner, local);
                    const uint32_t lo = (uint32_t)local;
                    uint32_t sb = lo >> cg.sup_log2;
                    if (sb >= cg.S) sb = cg.S - 1u;   // never for a valid offset (the geometry covers the shard)
                    const uint32_t wb = (owner * nh + (uint32_t)(local >> 32)) * cg.S + sb;
                    const uint32_t bkt = (wb << sub_log2) | (lo & ((1u << sub_log2) - 1u));
                    tag[q] = (bkt << 16) | atomicAdd(s_cnt + bkt, 1u);
                }
            }
        };
        if (kpl == 2) probes(std::integral_constant<uint32_t, 2>{});
        else probes(std::integral_constant<uint32_t, 1>{});
        __syncthreads();
        const uint32_t c = t < NB ? s_cnt[t] : 0u;
        const uint32_t ex = block_excl_scan(c, s_w, nullptr);
        if (t < NB) {
            s_lbase[t] = ex;
            s_cnt[t] = 0;
        }
        __syncthreads();
        if (t < P) {   // claim this tile's window-t run: its place and its rank among the window's runs
            const uint32_t lo_b = (t * wS) << sub_log2, hi_b = ((t + 1) * wS) << sub_log2;
            const uint32_t ob = s_lbase[lo_b], oc = (hi_b < NB ? s_lbase[hi_b] : tk * k) - ob;
            unsigned long long gb = 0;
            if (oc) {
                uint8_t* dw = cg.dir + (uint64_t)t * cg.dir_bytes;
                const unsigned long long x = atomicAdd(
                    reinterpret_cast<unsigned long long*>(dw + bf_chunk_dir_claim_offset(cg, cg.tiles)),
                    (1ull << kClaimRankShift) | (unsigned long long)oc);
                gb = x & ((1ull << kClaimRankShift) - 1ull);
                reinterpret_cast<uint16_t*>(dw + bf_chunk_dir_rank_offset(cg, cg.tiles))[x >> kClaimRankShift] =
                    (uint16_t)(tile + 1u);
                atomicAdd(wcounts + t, (unsigned long long)oc);
            }
            s_gbase[t] = (gb + oc <= wcap) ? (unsigned long long)t * wcap + gb : ~0ull;
            s_obase[t] = ob;
            reinterpret_cast<uint32_t*>(cg.dir + (uint64_t)t * cg.dir_bytes)[tile] =
                (gb + oc <= wcap) ? (uint32_t)gb : 0xFFFFFFFFu;
        }
        {   // the chunk's superbin run table in every window: [sb][tile], [S] = length
            const uint32_t S1 = cg.S + 1u;
            for (uint32_t e = t; e < P * S1; e += kTile) {
                const uint32_t w = e / S1, sb = e - w * S1;
                const uint32_t b0 = (w * cg.S) << sub_log2, b1 = (w * cg.S + sb) << sub_log2;
                const uint32_t v = (b1 < NB ? s_lbase[b1] : tk * k) - s_lbase[b0];
                reinterpret_cast<uint16_t*>(cg.dir + (uint64_t)w * cg.dir_bytes + 4 * cg.tiles)
                    [(uint64_t)sb * cg.tiles + tile] = (uint16_t)v;
            }
        }
        auto place = [&](auto kplc) {
            constexpr uint32_t KPL = decltype(kplc)::value;
#pragma unroll
            for (int q = 0; q < SLOTS; ++q)
                if (tag[q] != 0xFFFFFFFFu) {
                    const bool second = KPL == 2 && q >= (int)kTwoKeys;
                    const uint32_t i = second ? (uint32_t)q - kTwoKeys : (uint32_t)q;
                    s_idx[s_lbase[tag[q] >> 16] + (tag[q] & 0xFFFFu)] = (uint16_t)(((second ? kTile + t : t) << 4) | i);
                }
        };
        if (kpl == 2) place(std::integral_constant<uint32_t, 2>{});
        else place(std::integral_constant<uint32_t, 1>{});
        __syncthreads();
        const uint32_t tp = tk * k;
        uint32_t o = run_of(s_obase, P, t < tp ? t : 0u);
        for (uint32_t j = t; j < tp; j += kTile) {
            while (o + 1u < P && s_obase[o + 1u] <= j) ++o;
            const unsigned long long gb = s_gbase[o];
            if (gb == ~0ull) continue;   // the window overflows: the run is dropped
            const uint32_t x = s_idx[j], key = x >> 4;
            const uint4 H = s_dig[key];
            uint32_t owner;
            uint64_t local;
            owner_local(g, probe_offset(g, H.x, H.y, H.z, H.w, x & 15u), owner, local);
            const uint64_t d = gb + (j - s_obase[o]);
            wsend[d] = (uint32_t)local;   // the window implies the high bits
            if constexpr (SLOT) wslot[d] = (uint16_t)key;   // tile-relative
        }
        __syncthreads();   // s_gbase, s_dig and s_idx are rewritten by the next tile
    }
}

// One workgroup per 8192-probe block of an (owner, group) window (the grid is an
// upper bound; spare workgroups exit): the owner's runs from the group's tiles
// are copied, in order, to the window's place in the send buffer (owner-major,
// so owner s's probes are one contiguous all-to-all segment).  Block-granular
// so that the parallelism does not depend on the number of owners.
template <bool WIDE, bool SLOT>
__global__ __launch_bounds__(kTile) void route_gather_kernel(const uint32_t* __restrict__ lo1,
                                                             const uint8_t* __restrict__ hi1,
                                                             const uint32_t* __restrict__ key1,
                                                             const uint16_t* __restrict__ stab, uint64_t ntiles,
                                                             uint32_t tile_probes, uint32_t tiles_per_group,
                                                             uint32_t nowners, uint32_t nq,
                                                             const uint32_t* __restrict__ base,
                                                             const uint32_t* __restrict__ cb_base,
                                                             const uint32_t* __restrict__ cb_window,
                                                             void* __restrict__ send, uint32_t* __restrict__ slot) {
    __shared__ uint32_t s_pre[kRunsPerPass], s_gst[kRunsPerPass];
    __shared__ uint32_t s_w[16];
    const uint32_t t = threadIdx.x, b = blockIdx.x;
    if (b >= cb_base[nowners * nq]) return;   // workgroup-uniform
    const uint32_t w = cb_window[b];
    const uint32_t owner = w / nq, q = w - owner * nq;
    const uint32_t wbase = base[w];
    const uint32_t E = base[w + 1] - wbase;
    const uint32_t f0 = (b - cb_base[w]) * kBlockProbes;
    const uint32_t f_end = (E - f0 < kBlockProbes) ? E : f0 + kBlockProbes;
    const uint64_t tlo = (uint64_t)q * tiles_per_group;
    const uint64_t thi = (tlo + tiles_per_group < ntiles) ? tlo + tiles_per_group : ntiles;
    const uint32_t nt = (uint32_t)(thi - tlo);
    uint32_t len = 0, st = 0;
    if (t < nt) {
        const uint32_t a = stab[(uint64_t)owner * ntiles + tlo + t];
        len = stab[(uint64_t)(owner + 1) * ntiles + tlo + t] - a;
        st = (uint32_t)((tlo + t) * tile_probes) + a;
    }
    const uint32_t ex = block_excl_scan(len, s_w, nullptr);
    if (t < nt) {
        s_pre[t] = ex;
        s_gst[t] = st;
    }
    __syncthreads();
    const uint32_t fw = f0 + (t >> 6) * (64u * kChunkPerLane);
    uint32_t i = run_of(s_pre, nt, fw < f_end ? fw : f_end - 1);
#pragma unroll
    for (int u = 0; u < kChunkPerLane; ++u) {
        const uint32_t f = fw + u * 64 + (t & 63u);
        if (f < f_end) {
            while (i + 1 < nt && s_pre[i + 1] <= f) ++i;
            const uint32_t idx = s_gst[i] + (f - s_pre[i]);
            if constexpr (WIDE)
                static_cast<uint64_t*>(send)[wbase + f] = ((uint64_t)hi1[idx] << 32) | lo1[idx];
            else
                static_cast<uint32_t*>(send)[wbase + f] = lo1[idx];
            if constexpr (SLOT) slot[wbase + f] = key1[idx];
        }
    }
}

// bin_mid's workgroup order.  grouped: workgroup b runs on XCD x = b % 8, and superbin sb's
// nq * kMidParts workgroups all run on XCD sb % 8 in (group, part) order, so the partial-line
// stores of its region run table rows (tabs[region][block], one u16 per block) merge in one L2
// instead of eight (10B: 26.9M -> 16.3M write requests, bin_mid 0.656 -> 0.633 ms).  (Each XCD
// on one contiguous eighth of the superbins instead: 1.14 ms — the XCDs must sweep the same
// address neighbourhood, as in bin_apply)  Otherwise b = w * kMidParts + part.
// Returns sb (>= nsup: a spare workgroup of mid_grid).
__device__ __forceinline__ uint32_t mid_superbin(uint32_t nsup, uint32_t nq, bool grouped, uint32_t* q,
                                                 uint32_t* part) {
    if (!grouped) {
        const uint32_t w = blockIdx.x / kMidParts;
        *part = blockIdx.x - w * kMidParts;
        *q = w % nq;
        return w / nq;
    }
    const uint32_t wpsb = nq * kMidParts, xi = blockIdx.x >> 3;
    const uint32_t i = xi / wpsb, wq = xi - i * wpsb;
    *q = wq / kMidParts;
    *part = wq - *q * kMidParts;
    return (blockIdx.x & 7u) + 8u * i;
}
__host__ __device__ inline bool mid_grouped(uint32_t nsup) { return nsup >= 64; }
uint32_t mid_grid(uint32_t nsup, uint32_t nq) {
    return mid_grouped(nsup) ? 8u * ((nsup + 7u) / 8u) * nq * kMidParts : nsup * nq * kMidParts;
}

// One workgroup per (window, part): window w = (superbin sb, group q)
// concatenates superbin sb's runs from the group's tiles in tile order; it is
// cut into chunk blocks of kBlockProbes, and part p of kMidParts takes an equal
// share of them.  The run table is built once; each block's loads are issued
// while the previous block is sorted and written.
template <bool KEYS>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8))) void bin_mid_kernel(const uint32_t* __restrict__ level1,
                                                        const uint32_t* __restrict__ level1_key,
                                                        const uint16_t* __restrict__ stab, uint64_t ntiles,
                                                        uint32_t tile_probes, uint32_t tiles_per_group,
                                                        uint32_t nsup, uint32_t nq, uint32_t region_log2,
                                                        uint32_t rel_log2, const uint32_t* __restrict__ base,
                                                        const uint32_t* __restrict__ cb_base, uint64_t max_chunks,
                                                        uint16_t* __restrict__ tabs, uint32_t* __restrict__ level2,
                                                        uint32_t* __restrict__ level2_key) {
    __shared__ uint32_t s_pre[kRunsPerPass], s_gst[kRunsPerPass];
    __shared__ uint32_t s_cnt[1u << kMaxRel];
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_sorted[kBlockProbes];
    __shared__ uint32_t s_key[KEYS ? kBlockProbes : 1];
    const uint32_t t = threadIdx.x;
    uint32_t w_q, w_part;
    const uint32_t sb = mid_superbin(nsup, nq, mid_grouped(nsup), &w_q, &w_part);   // XCD-grouped
    if (sb >= nsup) return;   // workgroup-uniform: the grid is rounded up to whole XCD rows
    const uint32_t q = w_q, part = w_part;
    const uint32_t w = sb * nq + q;
    const uint32_t wbase = base[w];
    const uint32_t E = base[w + 1] - wbase;
    const uint32_t nblk = (E + kBlockProbes - 1) / kBlockProbes;
    const uint32_t c_lo = (uint32_t)((uint64_t)nblk * part / kMidParts);
    const uint32_t c_hi = (uint32_t)((uint64_t)nblk * (part + 1) / kMidParts);
    if (c_lo >= c_hi) return;   // workgroup-uniform
    const uint32_t b0 = cb_base[w];
    const uint32_t R = 1u << rel_log2;
    const uint32_t rmask = (1u << region_log2) - 1u;
    // Sort buckets = (region, low offset bits): at least kMidBuckets LDS counters however few
    // the regions per superbin, so that the rank atomics do not pile onto R words (a 150 MB
    // shard has R = 16); a region's sub-buckets are consecutive, so its probes stay one run.
    uint32_t sub = 0;
    while ((R << sub) < kMidBuckets) ++sub;
    const uint32_t NB = R << sub, smask_b = (1u << sub) - 1u;
    // run table of the group's tiles (consecutive lanes, consecutive tiles: coalesced)
    const uint64_t tlo = (uint64_t)q * tiles_per_group;
    const uint64_t thi = (tlo + tiles_per_group < ntiles) ? tlo + tiles_per_group : ntiles;
    const uint32_t nt = (uint32_t)(thi - tlo);   // <= kRunsPerPass (plan)
    uint32_t len = 0, st = 0;
    if (t < nt) {
        const uint32_t a = stab[(uint64_t)sb * ntiles + tlo + t];
        len = stab[(uint64_t)(sb + 1) * ntiles + tlo + t] - a;
        st = (uint32_t)((tlo + t) * tile_probes) + a;
    }
    const uint32_t ex = block_excl_scan(len, s_w, nullptr);
    if (t < nt) {
        s_pre[t] = ex;
        s_gst[t] = st;
    }
    __syncthreads();
    // Wave v of the block takes entries [f0 + 512v, f0 + 512v + 512): one binary
    // search per wave, then each lane walks the run table forward (runs are
    // ~tile probes / superbins long, so a step of 64 entries crosses at most a few).
    auto load = [&](uint32_t f0, uint32_t* lv, uint32_t* kv) {
        const uint32_t fw = f0 + (t >> 6) * (64u * kChunkPerLane);
        uint32_t i = run_of(s_pre, nt, fw < E ? fw : E - 1);
#pragma unroll
        for (int u = 0; u < kChunkPerLane; ++u) {
            const uint32_t f = fw + u * 64 + (t & 63u);
            lv[u] = 0xFFFFFFFFu;   // never a superbin-local offset (< 2^28)
            kv[u] = 0;
            if (f < E) {
                while (i + 1 < nt && s_pre[i + 1] <= f) ++i;
                const uint32_t idx = s_gst[i] + (f - s_pre[i]);
                lv[u] = level1[idx];
                if constexpr (KEYS) kv[u] = level1_key[idx];
            }
        }
    };
    uint32_t lv[kChunkPerLane], kv[kChunkPerLane];
    load(c_lo * kBlockProbes, lv, kv);
    for (uint32_t c = c_lo; c < c_hi; ++c) {
        const uint32_t f0 = c * kBlockProbes;
        const uint32_t f1 = (E - f0 < kBlockProbes) ? E : f0 + kBlockProbes;
        if (t < NB) s_cnt[t] = 0;
        __syncthreads();   // also orders the previous block's reads of s_sorted / s_cnt
        uint32_t tag[kChunkPerLane];
#pragma unroll
        for (int u = 0; u < kChunkPerLane; ++u) {
            tag[u] = 0xFFFFFFFFu;
            if (lv[u] != 0xFFFFFFFFu) {
                const uint32_t bk = ((lv[u] >> region_log2) << sub) | (lv[u] & smask_b);
                tag[u] = (bk << 16) | atomicAdd(s_cnt + bk, 1u);
            }
        }
        uint32_t nlv[kChunkPerLane], nkv[kChunkPerLane];
        if (c + 1 < c_hi) load(f0 + kBlockProbes, nlv, nkv);   // next block in flight
        __syncthreads();
        const uint32_t cn = t < NB ? s_cnt[t] : 0u;
        const uint32_t cex = block_excl_scan(cn, s_w, nullptr);   // its barriers order the s_cnt reads first
        if (!(t & smask_b) && (t >> sub) <= R)
            tabs[(uint64_t)(t >> sub) * max_chunks + b0 + c] = (uint16_t)cex;   // [region][block]
        if (t < NB) s_cnt[t] = cex;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kChunkPerLane; ++u) {
            if (tag[u] != 0xFFFFFFFFu) {
                const uint32_t d = s_cnt[tag[u] >> 16] + (tag[u] & 0xFFFFu);
                s_sorted[d] = lv[u] & rmask;
                if constexpr (KEYS) s_key[d] = kv[u];
            }
        }
        __syncthreads();
        const uint32_t out0 = wbase + f0;
        for (uint32_t j = t; j < f1 - f0; j += kTile) {
            stage_store(level2 + out0 + j, s_sorted[j]);
            if constexpr (KEYS) level2_key[out0 + j] = s_key[j];
        }
        if (c + 1 < c_hi) {
#pragma unroll
            for (int u = 0; u < kChunkPerLane; ++u) {
                lv[u] = nlv[u];
                kv[u] = nkv[u];
            }
        }
    }
}

// Region r's probes: one run in each chunk block of its superbin.  Calls
// visit(idx) for every level-2 index of the region (kLoads per lane in flight
// through the caller's batching); run tables in LDS, passes of kRunsPerPass
// blocks.  Contains barriers: every lane must call it.
template <int kLoads, typename Visit>
__device__ __forceinline__ void for_region_probes(const uint32_t* __restrict__ cb_base,
                                                  const uint32_t* __restrict__ cb_start,
                                                  const uint16_t* __restrict__ tabs, uint64_t max_chunks, uint32_t r,
                                                  uint32_t nq, uint32_t rel_log2, uint32_t* s_pre, uint32_t* s_gst,
                                                  uint32_t* s_w, Visit&& visit) {
    const uint32_t R = 1u << rel_log2;
    const uint32_t sb = r >> rel_log2, rl = r & (R - 1u);
    const uint32_t t = threadIdx.x, lanes = blockDim.x;
    const uint32_t bb0 = cb_base[sb * nq], bb1 = cb_base[(sb + 1) * nq];
    const uint32_t pass = lanes < kRunsPerPass ? lanes : kRunsPerPass;   // one run-table entry per lane
    for (uint32_t p0 = bb0; p0 < bb1; p0 += pass) {
        const uint32_t nt = (bb1 - p0 < pass) ? bb1 - p0 : pass;
        uint32_t len = 0, st = 0;
        if (t < nt) {   // consecutive lanes, consecutive blocks: coalesced
            const uint32_t a = tabs[(uint64_t)rl * max_chunks + p0 + t];
            len = tabs[(uint64_t)(rl + 1) * max_chunks + p0 + t] - a;
            st = cb_start[p0 + t] + a;
        }
        uint32_t E;
        const uint32_t ex = block_excl_scan(len, s_w, &E);
        if (t < nt) {
            s_pre[t] = ex;
            s_gst[t] = st;
        }
        __syncthreads();
        // wave v takes kLoads * 64 consecutive entries per step.  Its first entry's run: the
        // count of run starts <= fw, one ballot per 64 table entries (the starts ascend, so
        // they are a prefix); then every run start inside the wave's span moves the lanes
        // past it one run on (a wave-uniform loop over the few starts there, ~2 at 10B).
        // (Was a binary search per wave and a per-lane walk: ~100 VALU per wave and step.)
        const uint32_t span = kLoads * 64u, lane = t & 63u;
        for (uint32_t fb = 0; fb < E; fb += span * (lanes >> 6)) {
            const uint32_t fw = fb + (t >> 6) * span;
            uint32_t idx[kLoads];
#pragma unroll
            for (int c = 0; c < kLoads; ++c) idx[c] = 0xFFFFFFFFu;
            if (fw < E) {   // wave-uniform
                uint32_t i0 = 0;
                for (uint32_t b = 0; b < nt; b += 64u) {
                    const uint32_t j = b + lane;
                    const uint32_t c = (uint32_t)__popcll(__ballot(j < nt && s_pre[j] <= fw));
                    if (c) i0 = b + c - 1u;
                    if (c < 64u) break;
                }
                const uint32_t fend = E - fw < span ? E : fw + span;
                uint32_t ic[kLoads];
#pragma unroll
                for (int c = 0; c < kLoads; ++c) ic[c] = i0;
                for (uint32_t i = i0 + 1u; i < nt; ++i) {
                    const uint32_t B = __builtin_amdgcn_readfirstlane(s_pre[i]);
                    if (B >= fend) break;
#pragma unroll
                    for (int c = 0; c < kLoads; ++c) ic[c] += (fw + c * 64u + lane >= B) ? 1u : 0u;
                }
#pragma unroll
                for (int c = 0; c < kLoads; ++c) {
                    const uint32_t f = fw + c * 64u + lane;
                    if (f < E) idx[c] = s_gst[ic[c]] + (f - s_pre[ic[c]]);
                }
            }
            visit(idx);
        }
        __syncthreads();   // the next pass rewrites the run table
    }
}

// bin_apply reads a region with plain loads and writes it back with non-temporal stores: the
// region has one owner, and the written lines then do not evict include?'s cached lines
// (measured against nt loads, nt loads + stores and plain stores).
typedef uint32_t apply_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 apply_load(const uint4* p) { return *p; }
__device__ __forceinline__ void apply_store(uint4* p, uint4 v) {
    const apply_u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<apply_u32x4*>(p));
}

// Workgroup b's region.  xg > 1: xg consecutive regions on one XCD (workgroups b, b + 8, ...
// b + 8 (xg - 1) run on XCD b % 8 at about the same time), so the level-2 lines two
// neighbouring regions' runs share are fetched into one L2 once instead of into two; every XCD
// still sweeps the same 8 xg-region neighbourhood (a contiguous eighth per XCD measured
// slower).  A tail of fewer than 8 xg regions keeps the identity map.
__device__ __forceinline__ uint32_t apply_region(uint32_t b, uint32_t nb, uint32_t xg) {
    if (xg <= 1) return b;
    const uint32_t span = 8u * xg, full = nb - nb % span;
    if (b >= full) return b;
    const uint32_t w = b % span;
    return b - w + (w & 7u) * xg + (w >> 3);
}

template <uint32_t RLOG2, uint32_t LANES, int LOADS = 8>
__global__ __launch_bounds__(LANES) void bin_apply_kernel(uint32_t* __restrict__ bits, uint64_t nwords,
                                                          const uint32_t* __restrict__ level2,
                                                          const uint32_t* __restrict__ cb_base,
                                                          const uint32_t* __restrict__ cb_start,
                                                          const uint16_t* __restrict__ tabs, uint64_t max_chunks,
                                                          uint32_t nq, uint32_t rel_log2, uint32_t dense,
                                                          uint32_t* __restrict__ any_flag,
                                                          uint8_t* __restrict__ dirty, uint32_t store_fresh,
                                                          uint32_t xg) {
    constexpr uint32_t kVec = 1u << (RLOG2 - 7);   // 16-B vectors per region
    constexpr uint32_t kPer = kVec / LANES;
    constexpr int kLoads = LOADS;   // level-2 loads per lane and gather step (BFHIP_APPLY_LOADS)
    static_assert(kPer * LANES == kVec, "region must tile the workgroup");
    __shared__ uint4 s_mask4[kVec];
    __shared__ uint32_t s_pre[kRunsPerPass], s_gst[kRunsPerPass], s_w[16];
    uint32_t* s_mask = reinterpret_cast<uint32_t*>(s_mask4);
    const uint32_t t = threadIdx.x;
    const uint32_t r = apply_region(blockIdx.x, gridDim.x, xg);
    const uint64_t v0 = (uint64_t)r * kVec;
    const uint64_t nvec = nwords / 4;
    uint4* gv = reinterpret_cast<uint4*>(bits);
    // Dense batch (dense >= 1: at least one probe per 128-B line on average, so nearly every
    // line is touched): the region's vectors are loaded first, so that read overlaps the probe
    // pass; dense == 2 (a probe per 16-B vector) also writes the region back whole, in full
    // lines.  Sparse batch: only the touched vectors are read, after it.
    uint4 old[kPer];
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {
        const uint32_t v = c * LANES + t;
        old[c] = make_uint4(0, 0, 0, 0);
        if (dense && v0 + v < nvec) old[c] = apply_load(gv + v0 + v);
    }
    for (uint32_t v = t; v < kVec; v += LANES) s_mask4[v] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for_region_probes<kLoads>(cb_base, cb_start, tabs, max_chunks, r, nq, rel_log2, s_pre, s_gst, s_w,
        [&](const uint32_t* idx) {
            uint32_t l[kLoads];
#pragma unroll
            for (int c = 0; c < kLoads; ++c) l[c] = idx[c] != 0xFFFFFFFFu ? level2[idx[c]] : 0xFFFFFFFFu;
#pragma unroll
            for (int c = 0; c < kLoads; ++c)
                if (l[c] != 0xFFFFFFFFu) atomicOr(s_mask + (l[c] >> 5), 1u << ((l[c] ^ 7u) & 31u));
        });
    uint4 msk[kPer];
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {   // sparse: every touched vector's load issues before any store
        const uint32_t v = c * LANES + t;
        msk[c] = s_mask4[v];
        if (!dense && v0 + v < nvec && (msk[c].x | msk[c].y | msk[c].z | msk[c].w)) old[c] = apply_load(gv + v0 + v);
    }
    uint32_t fresh = 0;
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {
        const uint32_t v = c * LANES + t;
        // fr: the bits this vector gains (0 for an untouched one: its mask is 0)
        const uint32_t fr = (msk[c].x & ~old[c].x) | (msk[c].y & ~old[c].y) | (msk[c].z & ~old[c].z) |
                            (msk[c].w & ~old[c].w);
        fresh |= fr;
        if (v0 + v >= nvec) continue;
        // (writing whole 64-B sectors when any of their vectors gains a bit, instead of 32-B
        // partial writes, measured 2.459 vs 2.448 ms at 10B: profiles/r03t_apply_ab.jsonl)
        bool st;
        if (dense == 2) st = true;
        else if (store_fresh) st = fr != 0u;   // every probe hit a set bit: nothing to store
        else st = (msk[c].x | msk[c].y | msk[c].z | msk[c].w) != 0u;
        if (st)
            apply_store(gv + v0 + v, make_uint4(old[c].x | msk[c].x, old[c].y | msk[c].y, old[c].z | msk[c].z, old[c].w | msk[c].w));
        if (dirty && fr) dirty[((v0 + v) * 128) >> kDirtyShiftBits] = 1;
    }
    if (any_flag) report_any_new(any_flag, fresh != 0);
}

// bin_apply for dense batches (every region read whole), persistent and software-pipelined.
// bin_apply's workgroup waits out three dependent memory round trips per region (its vectors
// and run table, then the level-2 probes, then its stores) with two regions per CU in flight
// (the LDS image), so the 10B / 200B apply streamed at ~3.9 TB/s.  Here each workgroup walks
// regions r = blockIdx.x + i * G and keeps a three-stage pipeline in registers: while it ORs
// region r's probes into the LDS image and writes r back, the vectors and the first level-2
// step of r + G and the run table of r + 2G are already in flight.  An iteration then waits
// only for loads issued one iteration earlier.  The prefetch loads are unconditional (clamped
// addresses; past the last region a workgroup reloads its last one), so the compiler's
// in-order vmcnt waits for older values leave the younger prefetches outstanding.  Two LDS
// run-table buffers alternate between r and r + G, the register buffers by unrolling the
// region loop twice (a register copy would wait for the stores just issued).
constexpr int kWaitVm0 = 0x0F70;   // s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15) (gfx9 encoding)
template <uint32_t RLOG2, uint32_t LANES, int LOADS = 8>
__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(4, 4))) void bin_apply_pipe_kernel(uint32_t* __restrict__ bits, uint64_t nwords,
                                                               uint32_t nbins, const uint32_t* __restrict__ level2,
                                                               const uint32_t* __restrict__ cb_base,
                                                               const uint32_t* __restrict__ cb_start,
                                                               const uint16_t* __restrict__ tabs, uint64_t max_chunks,
                                                               uint32_t nq, uint32_t rel_log2, uint32_t dense,
                                                               uint32_t* __restrict__ any_flag,
                                                               uint8_t* __restrict__ dirty, uint32_t store_fresh) {
    constexpr uint32_t kVec = 1u << (RLOG2 - 7);   // 16-B vectors per region
    constexpr uint32_t kPer = kVec / LANES;
    constexpr int kLoads = LOADS;   // (BFHIP_APPLY_PIPE_LOADS A/B)
    constexpr uint32_t kPass = LANES < kRunsPerPass ? LANES : kRunsPerPass;   // run-table entries per pass
    static_assert(kPer * LANES == kVec, "region must tile the workgroup");
    __shared__ uint4 s_mask4[kVec];
    __shared__ uint32_t s_pre[2][kPass], s_gst[2][kPass], s_w[16];
    uint32_t* s_mask = reinterpret_cast<uint32_t*>(s_mask4);
    const uint32_t t = threadIdx.x;
    const uint32_t R = 1u << rel_log2;
    const uint64_t nvec = nwords / 4;
    uint4* gv = reinterpret_cast<uint4*>(bits);
    const uint32_t G = gridDim.x;
    const uint32_t span = kLoads * 64u, step = span * (LANES >> 6);
    if (blockIdx.x >= nbins) return;   // workgroup-uniform
    const uint32_t last = blockIdx.x + (nbins - 1 - blockIdx.x) / G * G;   // this workgroup's last region
    auto clampr = [&](uint32_t q) { return q < last ? q : last; };

    // The run-table row of region q for its first pass (lane t: chunk block bb0 + t).
    struct Tab { uint32_t a, b, cs; };
    auto load_tab = [&](uint32_t q) {
        const uint32_t sb = q >> rel_log2, rl = q & (R - 1u);
        const uint32_t bb0 = cb_base[sb * nq], bb1 = cb_base[(sb + 1) * nq];
        const uint32_t nt = bb1 - bb0;
        const uint64_t j = nt ? bb0 + (t < nt ? t : nt - 1u) : 0u;
        Tab x;
        x.a = tabs[(uint64_t)rl * max_chunks + j];
        x.b = tabs[(uint64_t)(rl + 1) * max_chunks + j];
        x.cs = cb_start[j];
        return x;
    };
    // Scans a run-table pass into LDS buffer bi; returns the pass's probe count (uniform).
    // Contains barriers.
    auto scan = [&](uint32_t nt, uint32_t len, uint32_t st, uint32_t bi) {
        uint32_t E;
        const uint32_t ex = block_excl_scan(t < nt ? len : 0u, s_w, &E);
        if (t < nt) {
            s_pre[bi][t] = ex;
            s_gst[bi][t] = st;
        }
        __syncthreads();
        return E;
    };
    auto pass_nt = [&](uint32_t q) {
        const uint32_t sb = q >> rel_log2;
        const uint32_t n = cb_base[(sb + 1) * nq] - cb_base[sb * nq];
        return n < kPass ? n : kPass;
    };
    // Level-2 values of step fb of the pass in buffer bi.  Every load issues (entry 0 stands in
    // past the pass's E probes), so the number of loads in flight is static; mark() skips them.
    auto load_l2 = [&](uint32_t bi, uint32_t nt, uint32_t E, uint32_t fb, uint32_t* l) {
        const uint32_t fw = fb + (t >> 6) * span;
        uint32_t i = (nt && fw < E) ? run_of(s_pre[bi], nt, fw) : 0u;
#pragma unroll
        for (int c = 0; c < kLoads; ++c) {
            const uint32_t f = fw + c * 64 + (t & 63u);
            uint32_t idx = 0;
            if (f < E) {
                while (i + 1 < nt && s_pre[bi][i + 1] <= f) ++i;
                idx = s_gst[bi][i] + (f - s_pre[bi][i]);
            }
            l[c] = level2[idx];
        }
    };
    auto mark = [&](const uint32_t* l, uint32_t E, uint32_t fb) {
        const uint32_t fw = fb + (t >> 6) * span;
#pragma unroll
        for (int c = 0; c < kLoads; ++c)
            if (fw + c * 64 + (t & 63u) < E) atomicOr(s_mask + (l[c] >> 5), 1u << ((l[c] ^ 7u) & 31u));
    };
    auto load_vecs = [&](uint32_t q, uint4* vo) {
        const uint64_t v0 = (uint64_t)q * kVec;
#pragma unroll
        for (uint32_t c = 0; c < kPer; ++c) {
            const uint64_t v = v0 + c * LANES + t;
            vo[c] = apply_load(gv + (v < nvec ? v : nvec - 1));
        }
    };

    uint32_t fresh = 0;
    // Region r: its vectors (cur), first level-2 step (lv), first-pass table (LDS buffer bi,
    // E probes over nt blocks) are in flight or ready; r + G's run-table row (tn) is in flight.
    // Issues r + G's step / vectors into (nlv, nxt), r + 2G's row into tnn, and returns r + G's E.
    auto region = [&](uint32_t r, uint32_t bi, uint32_t nt, uint32_t E, const uint4* cur, const uint32_t* lv,
                      const Tab& tn, uint4* nxt, uint32_t* nlv, Tab& tnn, uint32_t& ntn) {
        const uint32_t rn = clampr(r + G);
        // stage 1: r + G's table -> LDS buffer bi ^ 1 (its row was issued an iteration ago)
        ntn = pass_nt(rn);
        const uint32_t En = scan(ntn, tn.b - tn.a, tn.cs + tn.a, bi ^ 1u);
        // stage 2: issue r + 2G's row, r + G's first level-2 step and its vectors
        tnn = load_tab(clampr(r + 2 * G));
        load_l2(bi ^ 1u, ntn, En, 0, nlv);
        load_vecs(rn, nxt);
        // stage 3: r's probes into the image (lv waited: issued before everything above)
        mark(lv, E, 0);
        // The rare paths below end each trip with vmcnt(0) (they wait for their loads anyway), so
        // at their exits the compiler's wait state is the main path's: no full wait joins it.
        for (uint32_t fb = step; fb < E; fb += step) {   // regions of more than one step
            uint32_t l[kLoads];
            load_l2(bi, nt, E, fb, l);
            mark(l, E, fb);
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
        }
        const uint32_t sb = r >> rel_log2, rl = r & (R - 1u);
        const uint32_t bb0 = cb_base[sb * nq], bb1 = cb_base[(sb + 1) * nq];
        for (uint32_t p0 = bb0 + kPass; p0 < bb1; p0 += kPass) {   // superbins of more than kPass blocks
            const uint32_t pn = (bb1 - p0 < kPass) ? bb1 - p0 : kPass;
            uint32_t len = 0, st = 0;
            if (t < pn) {
                const uint32_t a = tabs[(uint64_t)rl * max_chunks + p0 + t];
                len = tabs[(uint64_t)(rl + 1) * max_chunks + p0 + t] - a;
                st = cb_start[p0 + t] + a;
            }
            __syncthreads();   // every lane is past its reads of buffer bi
            const uint32_t Ep = scan(pn, len, st, bi);
            for (uint32_t fb = 0; fb < Ep; fb += step) {
                uint32_t l[kLoads];
                load_l2(bi, pn, Ep, fb, l);
                mark(l, Ep, fb);
            }
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
        }
        __syncthreads();   // the image is complete
        // OR the image into the region; each lane then zeroes the mask vectors it read
        const uint64_t v0 = (uint64_t)r * kVec;
#pragma unroll
        for (uint32_t c = 0; c < kPer; ++c) {
            const uint32_t v = c * LANES + t;
            const uint4 m = s_mask4[v];
            s_mask4[v] = make_uint4(0, 0, 0, 0);
            if (v0 + v < nvec && (dense == 2 || (m.x | m.y | m.z | m.w))) {
                const uint32_t fr = (m.x & ~cur[c].x) | (m.y & ~cur[c].y) | (m.z & ~cur[c].z) | (m.w & ~cur[c].w);
                fresh |= fr;
                if (store_fresh && dense != 2 && !fr) continue;   // every probe hit a set bit: nothing to store
                apply_store(gv + v0 + v, make_uint4(cur[c].x | m.x, cur[c].y | m.y, cur[c].z | m.z, cur[c].w | m.w));
                if (dirty && fr) dirty[((v0 + v) * 128) >> kDirtyShiftBits] = 1;
            }
        }
        return En;
    };

    // prologue: region blockIdx.x's table, first step and vectors; the next region's row
    uint32_t r = blockIdx.x;
    for (uint32_t v = t; v < kVec; v += LANES) s_mask4[v] = make_uint4(0, 0, 0, 0);
    uint4 bufA[kPer], bufB[kPer];
    uint32_t lA[kLoads], lB[kLoads];
    Tab tA, tB;
    uint32_t ntA, ntB, EA, EB;
    {
        const Tab t0 = load_tab(r);
        ntA = pass_nt(r);
        EA = scan(ntA, t0.b - t0.a, t0.cs + t0.a, 0u);
        tA = load_tab(clampr(r + G));
        load_l2(0u, ntA, EA, 0, lA);
        load_vecs(r, bufA);
    }
    for (;; r += 2 * G) {
        EB = region(r, 0u, ntA, EA, bufA, lA, tA, bufB, lB, tB, ntB);
        if (r + G >= nbins) break;
        EA = region(r + G, 1u, ntB, EB, bufB, lB, tB, bufA, lA, tA, ntA);
        if (r + 2 * G >= nbins) break;
    }
    if (any_flag) report_any_new(any_flag, fresh != 0);
}

// include?: the region in LDS; a probe on a 0 bit clears its key's answer.  The probe
// streams and the region are read non-temporally, so that the scattered answer bytes keep
// their lines in the caches (0.745 -> 0.691 ms at P = 8).
// L2ORDER (the chunked owner's packed answers): each probe's answer byte (0/1) is stored at its
// level-2 index instead — runs of consecutive bytes, no scatter, no key array read — and
// chunk_unsort_kernel moves them to receive order (200B x 8: 1.74 -> ~0.5 ms).
template <uint32_t RLOG2, uint32_t LANES, bool L2ORDER = false>
__global__ __launch_bounds__(LANES) void bin_test_kernel(const uint32_t* __restrict__ bits, uint64_t nwords,
                                                         const uint32_t* __restrict__ level2,
                                                         const uint32_t* __restrict__ level2_key,
                                                         const uint32_t* __restrict__ cb_base,
                                                         const uint32_t* __restrict__ cb_start,
                                                         const uint16_t* __restrict__ tabs, uint64_t max_chunks,
                                                         uint32_t nq, uint32_t rel_log2, uint8_t* __restrict__ out8) {
    constexpr uint32_t kVec = 1u << (RLOG2 - 7);
    constexpr int kLoads = 8;
    __shared__ uint4 s_bits4[kVec];
    __shared__ uint32_t s_pre[kRunsPerPass], s_gst[kRunsPerPass], s_w[16];
    const uint32_t* s_bits = reinterpret_cast<const uint32_t*>(s_bits4);
    const uint32_t t = threadIdx.x;
    const uint32_t r = blockIdx.x;
    const uint64_t v0 = (uint64_t)r * kVec;
    const uint64_t nvec = nwords / 4;
    typedef uint32_t nt_u32x4 __attribute__((ext_vector_type(4)));
    const nt_u32x4* gn = reinterpret_cast<const nt_u32x4*>(bits);
    for (uint32_t v = t; v < kVec; v += LANES) {
        nt_u32x4 x = {0u, 0u, 0u, 0u};
        if (v0 + v < nvec) x = __builtin_nontemporal_load(gn + v0 + v);
        s_bits4[v] = make_uint4(x.x, x.y, x.z, x.w);
    }
    __syncthreads();
    for_region_probes<kLoads>(cb_base, cb_start, tabs, max_chunks, r, nq, rel_log2, s_pre, s_gst, s_w,
        [&](const uint32_t* idx) {
            uint32_t l[kLoads], key[kLoads];
#pragma unroll
            for (int c = 0; c < kLoads; ++c) {
                l[c] = 0xFFFFFFFFu;
                key[c] = 0;
                if (idx[c] != 0xFFFFFFFFu) {
                    l[c] = __builtin_nontemporal_load(level2 + idx[c]);
                    if constexpr (!L2ORDER) key[c] = __builtin_nontemporal_load(level2_key + idx[c]);
                }
            }
#pragma unroll
            for (int c = 0; c < kLoads; ++c) {
                if constexpr (L2ORDER) {
                    if (l[c] != 0xFFFFFFFFu) out8[idx[c]] = (uint8_t)((s_bits[l[c] >> 5] >> ((l[c] ^ 7u) & 31u)) & 1u);
                } else if (l[c] != 0xFFFFFFFFu && !((s_bits[l[c] >> 5] >> ((l[c] ^ 7u) & 31u)) & 1u)) {
                    out8[key[c]] = 0;
                }
            }
        });
}

// The owner's insert and include? of one partitioned step in ONE pass over the shard: region r
// is read once, its insert probes (level-2 arrays of the insert plan) ORed into the LDS image and
// the region written back as bin_apply does, then its include? probes (the test plan's level
// 2) tested against the updated image, each answer stored at its level-2 index (bin_test
// <L2ORDER>).  The answers see every insert of the step, as insert-then-test does: a test probe
// in region r reads only region r.  One read of the shard and one run-table walk set-up fewer
// than bin_apply + bin_test.
struct BfL2 {   // one plan's level-2 arrays and run tables
    const uint32_t* level2;
    const uint32_t* cb_base;
    const uint32_t* cb_start;
    const uint16_t* tabs;
    uint64_t max_chunks;
    uint32_t nq;
};
// SIDE: the workgroups also hash another key batch (the requester's next include? batch: sh),
// an equal share each, staged through the LDS image before it is cleared, while the region's
// vectors are in flight; the next step then routes that batch from its words.
template <uint32_t RLOG2, uint32_t LANES, int ILOADS, bool SIDE = false>
// (8 waves per SIMD = two 2^19-bit workgroups per CU: the SIDE form stays within 64 VGPRs)
__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(RLOG2 == 19 ? 8 : 4, 8))) void bin_apply_test_kernel(uint32_t* __restrict__ bits, uint64_t nwords, BfL2 ins,
                                                               BfL2 tst, uint32_t rel_log2, uint32_t dense,
                                                               uint32_t* __restrict__ any_flag,
                                                               uint8_t* __restrict__ dirty, uint32_t store_fresh,
                                                               uint8_t* __restrict__ ans2, BfSideHash sh) {
    constexpr uint32_t kVec = 1u << (RLOG2 - 7);
    constexpr uint32_t kPer = kVec / LANES;
    constexpr int kTLoads = 8;
    static_assert(kPer * LANES == kVec, "region must tile the workgroup");
    __shared__ uint4 s_img4[kVec];
    __shared__ uint32_t s_pre[kRunsPerPass], s_gst[kRunsPerPass], s_w[16];
    uint32_t* s_img = reinterpret_cast<uint32_t*>(s_img4);
    const uint32_t t = threadIdx.x;
    const uint32_t r = apply_region(blockIdx.x, gridDim.x, 2u);
    const uint64_t v0 = (uint64_t)r * kVec;
    const uint64_t nvec = nwords / 4;
    uint4* gv = reinterpret_cast<uint4*>(bits);
    // every region is read: the test needs all of it (dense or not)
    uint4 old[kPer];
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {
        const uint32_t v = c * LANES + t;
        old[c] = v0 + v < nvec ? apply_load(gv + v0 + v) : make_uint4(0, 0, 0, 0);
    }
    if constexpr (SIDE) {   // this workgroup's share of the side batch, LANES keys per tile
        static_assert(8 * (LANES + 1) + 16 * (kStageVec + kStageSlackVec) <= 16 * kVec, "side stage fits the image");
        const uint64_t per = (sh.n + gridDim.x - 1) / gridDim.x;
        const uint64_t k0 = (uint64_t)blockIdx.x * per, k1 = k0 + per < sh.n ? k0 + per : sh.n;
        uint64_t* s_off = reinterpret_cast<uint64_t*>(s_img4);
        uint4* s_stage = s_img4 + (8 * (LANES + 1) + 15) / 16;
        for (uint64_t j0 = k0; j0 < k1; j0 += LANES) {   // workgroup-uniform
            const uint32_t cnt = (uint32_t)(k1 - j0 < LANES ? k1 - j0 : LANES);
            for_key_tile<LANES, kStageVec>(sh.keys16, sh.offsets, sh.bias, j0, cnt, s_off, s_stage, sh.key_status,
                [&](auto staged, uint32_t lane, const uint32_t* src, uint32_t s0, uint32_t L) {
                    uint32_t H[5];
                    sha1_any<decltype(staged)::value>(src, s0, L, H);
                    sh.dig[j0 + lane] = make_uint4(H[0], H[1], H[2], H[3]);
                });
        }
    }
    for (uint32_t v = t; v < kVec; v += LANES) s_img4[v] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for_region_probes<ILOADS>(ins.cb_base, ins.cb_start, ins.tabs, ins.max_chunks, r, ins.nq, rel_log2, s_pre, s_gst,
                              s_w, [&](const uint32_t* idx) {
        uint32_t l[ILOADS];
#pragma unroll
        for (int c = 0; c < ILOADS; ++c) l[c] = idx[c] != 0xFFFFFFFFu ? ins.level2[idx[c]] : 0xFFFFFFFFu;
#pragma unroll
        for (int c = 0; c < ILOADS; ++c)
            if (l[c] != 0xFFFFFFFFu) atomicOr(s_img + (l[c] >> 5), 1u << ((l[c] ^ 7u) & 31u));
    });
    // (for_region_probes ends with a barrier: the insert image is complete)
    uint32_t fresh = 0;
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {
        const uint32_t v = c * LANES + t;
        const uint4 m = s_img4[v];
        const uint4 nw = make_uint4(old[c].x | m.x, old[c].y | m.y, old[c].z | m.z, old[c].w | m.w);
        s_img4[v] = nw;   // the image becomes the region after the step's inserts
        const uint32_t fr = (m.x & ~old[c].x) | (m.y & ~old[c].y) | (m.z & ~old[c].z) | (m.w & ~old[c].w);
        fresh |= fr;
        if (v0 + v >= nvec) continue;
        bool st;
        if (dense == 2) st = true;
        else if (store_fresh) st = fr != 0u;
        else st = (m.x | m.y | m.z | m.w) != 0u;
        if (st) apply_store(gv + v0 + v, nw);
        if (dirty && fr) dirty[((v0 + v) * 128) >> kDirtyShiftBits] = 1;
    }
    if (any_flag) report_any_new(any_flag, fresh != 0);
    __syncthreads();
    for_region_probes<kTLoads>(tst.cb_base, tst.cb_start, tst.tabs, tst.max_chunks, r, tst.nq, rel_log2, s_pre, s_gst,
                               s_w, [&](const uint32_t* idx) {
        uint32_t l[kTLoads];
#pragma unroll
        for (int c = 0; c < kTLoads; ++c)
            l[c] = idx[c] != 0xFFFFFFFFu ? __builtin_nontemporal_load(tst.level2 + idx[c]) : 0xFFFFFFFFu;
#pragma unroll
        for (int c = 0; c < kTLoads; ++c)
            if (l[c] != 0xFFFFFFFFu) ans2[idx[c]] = (uint8_t)((s_img[l[c] >> 5] >> ((l[c] ^ 7u) & 31u)) & 1u);
    });
}

// ---- chunked windows, owner side (bf_route_chunks_dev's windows as level 1) ----------------

// The run of superbin lsb (window-local) in chunk c of sub-range h: c = src * tiles + tile.
// An overflowed window (live count past cap) or a dropped chunk has none.
__device__ __forceinline__ uint64_t chunks_per_src(const BfChunkIn& ci) { return ci.ranked ? ci.cps : ci.tiles; }
// The tile holding rank r's run in window j (ranked chunks), or ~0 when no run has that rank.
__device__ __forceinline__ uint64_t ranked_tile(const BfChunkIn& ci, uint32_t j, uint64_t r) {
    const uint8_t* d = ci.dir + (uint64_t)j * ci.dir_bytes;
    const uint32_t v = reinterpret_cast<const uint16_t*>(d + 4 * ci.tiles + 2 * (uint64_t)(ci.S + 1) * ci.tiles)[r];
    return v && v <= ci.tiles ? (uint64_t)v - 1u : ~0ull;
}
__device__ __forceinline__ void chunk_run(const BfChunkIn& ci, uint32_t h, uint32_t lsb, uint64_t c, uint32_t* len,
                                          uint32_t* st) {
    const uint64_t cps = chunks_per_src(ci);
    const uint32_t src = (uint32_t)(c / cps);
    uint64_t tile = c - (uint64_t)src * cps;
    const uint32_t j = h * ci.nsrc + src;
    *len = 0;
    *st = 0;
    if (tile >= ci.tiles || ci.counts[(uint64_t)src * ci.cstride + h] > ci.cap) return;
    if (ci.ranked && (tile = ranked_tile(ci, j, tile)) == ~0ull) return;   // rank -> tile
    const uint8_t* d = ci.dir + (uint64_t)j * ci.dir_bytes;
    const uint32_t start = reinterpret_cast<const uint32_t*>(d)[tile];
    if (start == 0xFFFFFFFFu) return;
    const uint16_t* tab = reinterpret_cast<const uint16_t*>(d + 4 * ci.tiles);
    const uint32_t a = tab[(uint64_t)lsb * ci.tiles + tile], b = tab[(uint64_t)(lsb + 1) * ci.tiles + tile];
    if (b > a && (uint64_t)start + b <= ci.cap) {   // a directory never points past its window
        *len = b - a;
        *st = (uint32_t)((uint64_t)j * ci.cap + start + a);
    }
}

// gsum[sb][q] = probes of (global) superbin sb in chunk group q (kRunsPerPass chunks of its
// sub-range).  One workgroup per (superbin, group), one lane per chunk: coalesced table reads.
// runs (nullable): window w = sb * nq + q's run table, (exclusive prefix of the run lengths,
// the run's first receive index) for kRunsPerPass chunks, for chunk_test_l2_kernel.
// istart (with runs): istart[w * parts + p] = the run holding the first probe of part p of
// window w (the L2 sweep's items), so an item loads only its own runs.
__global__ __launch_bounds__(kRunsPerPass) void chunk_group_sum_kernel(BfChunkIn ci, uint32_t nq,
                                                                       uint32_t* __restrict__ gsum,
                                                                       uint2* __restrict__ runs, uint32_t parts,
                                                                       uint16_t* __restrict__ istart) {
    __shared__ uint32_t s_w[16];
    const uint32_t sb = blockIdx.x, q = blockIdx.y, t = threadIdx.x;
    const uint32_t h = sb / ci.S, lsb = sb - h * ci.S;
    const uint64_t c = (uint64_t)q * kRunsPerPass + t;
    uint32_t len = 0, st = 0;
    if (c < (uint64_t)ci.nsrc * chunks_per_src(ci)) chunk_run(ci, h, lsb, c, &len, &st);
    uint32_t total;
    const uint32_t ex = block_excl_scan(len, s_w, &total);
    if (t == 0) gsum[sb * nq + q] = total;
    if (runs) {
        const uint64_t w = (uint64_t)sb * nq + q;
        runs[w * kRunsPerPass + t] = make_uint2(ex, st);
        if (len)
            for (uint32_t p = 0; p < parts; ++p) {
                const uint32_t f0 = (uint32_t)((uint64_t)total * p / parts);
                if (f0 >= ex && f0 < ex + len) istart[w * parts + p] = (uint16_t)t;
            }
    }
}

// Owner side of a chunked include? without sorting: the probes of superbin sb stay in their
// receive order (runs of each chunk), and every workgroup sweeps the superbins in the same
// order — item i = (sb, group q, part) goes to workgroup i % gridDim, and a superbin has at
// least gridDim items — so at any time the chip probes about one superbin (a few MiB): its
// lines stay in every XCD's L2 and the random probes hit there (tools/probe_xcd.hip: 4 MiB
// windows per XCD take ~178 G probes/s against ~55 G/s beyond the caches).  Answers are
// stored in receive order, so a run's byte stores are contiguous (no scatter); an entry
// outside its superbin or past the shard answers 0.  Every live entry gets an answer.
constexpr uint32_t kL2Lanes = 256;
constexpr int kL2Loads = 8;
// 256 CUs x 6 workgroups of 4 waves.  With the per-wave run search, grid A/B (P = 8): 1024 /
// 1280 / 1536 / 1792 / 2048 -> test_l2 0.81 / 1.02 / 0.74 / 0.95 / 0.97 ms; P = 4: 0.78 at 1024,
// 0.72 at 1536 (profiles/r04o8_ab_l2_grid.jsonl, r04n_ab_l2_grid.jsonl, r04p_ab_l2_grid_P4.jsonl)
constexpr uint32_t kL2Grid = 1536;
constexpr uint32_t kL2MaxParts = 256;
template <bool SIDE, bool WALK = true, int LOADS = kL2Loads>
__global__ __launch_bounds__(kL2Lanes) void chunk_test_l2_kernel(BfChunkIn ci, const uint32_t* __restrict__ bits,
                                                                 uint32_t nsup, uint32_t nq, uint32_t parts,
                                                                 const uint32_t* __restrict__ gsum,
                                                                 const uint2* __restrict__ runs,
                                                                 const uint16_t* __restrict__ istart,
                                                                 uint8_t* __restrict__ out8, BfSideHash sh) {
    __shared__ uint32_t s_pre[kRunsPerPass], s_gst[kRunsPerPass];
    constexpr uint32_t kSideVec = 256;   // 4 KiB key stage: a tile of 256 keys of <= ~16 B each
    __shared__ uint64_t s_soff[kL2Lanes + 1];
    __shared__ uint4 s_sstage[kSideVec + kStageSlackVec];
    const uint32_t t = threadIdx.x;
    // Side job (sh.n > 0): SHA-1 words of another batch, one key per lane in tiles of kL2Lanes
    // keys; tile T belongs to workgroup T % gridDim and is hashed at the top of one of its items
    // (spread evenly), so hashing waves overlap other waves' probe latency, as the single-GPU
    // include? kernel hashes the next insert batch (bf_include_hash_kernel).  A tile's key bytes
    // are staged into LDS with one coalesced pass (a tile past the stage reads from global).
    const uint64_t sh_tiles = (sh.n + kL2Lanes - 1) / kL2Lanes;
    const uint64_t sh_mine = sh_tiles > blockIdx.x ? (sh_tiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
    uint64_t sh_done = 0;
    auto side_hash = [&](uint64_t upto) {   // this workgroup's tiles [sh_done, upto); has barriers
        for (; sh_done < upto; ++sh_done) {
            const uint64_t j0 = (blockIdx.x + sh_done * gridDim.x) * kL2Lanes;
            const uint32_t cnt = (uint32_t)(sh.n - j0 < kL2Lanes ? sh.n - j0 : kL2Lanes);
            __syncthreads();   // the previous tile's readers of the stage are done
            if (t < cnt) s_soff[t] = sh.offsets[j0 + t] + sh.bias;
            if (t == 0) s_soff[cnt] = sh.offsets[j0 + cnt] + sh.bias;
            __syncthreads();
            const uint64_t abase = s_soff[0] & ~(uint64_t)15;
            const uint64_t nvec = s_soff[cnt] >= s_soff[0] ? (s_soff[cnt] - abase + 15) >> 4 : ~0ull;
            const bool staged = nvec <= kSideVec;   // workgroup-uniform
            if (staged) {
                const uint4* gv = reinterpret_cast<const uint4*>(sh.keys16 + abase);
                for (uint32_t v = t; v < (uint32_t)nvec; v += kL2Lanes) s_sstage[v] = gv[v];
            }
            __syncthreads();
            if (t < cnt) {
                const bool ok = key_ok(s_soff[0], s_soff[t], s_soff[t + 1], s_soff[cnt], sh.key_status);
                const uint64_t ks = ok ? s_soff[t] : (staged ? abase : 0), L = ok ? s_soff[t + 1] - ks : 0;
                uint32_t H[5];
                if (staged) {
                    sha1_key_staged(reinterpret_cast<const uint32_t*>(s_sstage), (uint32_t)(ks - abase), (uint32_t)L, H);
                } else {
                    const uint64_t kbase = ks & ~(uint64_t)3;
                    sha1_key(reinterpret_cast<const uint32_t*>(sh.keys16 + kbase), (uint32_t)(ks - kbase), (uint32_t)L, H);
                }
                sh.dig[j0 + t] = make_uint4(H[0], H[1], H[2], H[3]);
            }
        }
    };
    const uint64_t nch = (uint64_t)ci.nsrc * chunks_per_src(ci);
    // XCD-local sweep: workgroup b runs on XCD b % 8 (round-robin dispatch; the grid is a
    // multiple of 8), and XCD x sweeps superbins x, x + 8, ..., its gridDim / 8 workgroups
    // sharing each superbin's items.  So each XCD's L2 holds one superbin, where a sweep of the
    // whole grid over one superbin made every XCD fetch the same lines (tools/probe_xcd.hip is
    // this layout: 178 G probes/s at 4 MiB per XCD).
    const uint32_t xcd = blockIdx.x & 7u, g8 = gridDim.x >> 3;
    const uint64_t per_sb = (uint64_t)nq * parts;
    const uint64_t items = (uint64_t)((nsup + 7u - xcd) >> 3) * per_sb;   // this XCD's superbins
    const uint64_t k0 = blockIdx.x >> 3;
    const uint64_t my_items = items > k0 ? (items - 1 - k0) / g8 + 1 : 0;
    uint64_t ii = 0;
    for (uint64_t k = k0; k < items; k += g8, ++ii) {
        if constexpr (SIDE) side_hash((ii + 1) * sh_mine / my_items);
        const uint32_t sb = xcd + 8u * (uint32_t)(k / per_sb);
        const uint64_t kk = k - (uint64_t)(k / per_sb) * per_sb;
        const uint32_t q = (uint32_t)(kk / parts), part = (uint32_t)(kk - (uint64_t)q * parts);
        const uint32_t w = sb * nq + q;
        const uint32_t E = gsum[w];
        const uint32_t f0 = (uint32_t)((uint64_t)E * part / parts), f1 = (uint32_t)((uint64_t)E * (part + 1) / parts);
        if (f0 >= f1) continue;   // workgroup-uniform
        const uint64_t c0 = (uint64_t)q * kRunsPerPass;
        const uint32_t ntw = (uint32_t)(nch - c0 < kRunsPerPass ? nch - c0 : kRunsPerPass);
        // only this item's runs: from the run holding f0 to the one holding the next part's f0
        const uint32_t i0 = istart[(uint64_t)w * parts + part];
        const uint32_t i1 = part + 1 < parts ? istart[(uint64_t)w * parts + part + 1] : ntw - 1;
        const uint32_t nt = i1 - i0 + 1;
        __syncthreads();   // the previous item's readers of s_pre / s_gst are done
        for (uint32_t j = t; j < nt; j += kL2Lanes) {
            const uint2 r = runs[(uint64_t)w * kRunsPerPass + i0 + j];
            s_pre[j] = r.x;
            s_gst[j] = r.y;
        }
        __syncthreads();
        const uint32_t h = sb / ci.S, lsb = sb - h * ci.S;
        const uint64_t hoff = (uint64_t)h << 32;
        for (uint32_t fb = f0; fb < f1; fb += kL2Lanes * LOADS) {
            uint32_t idx[LOADS], o[LOADS];
            // WALK: wave v takes LOADS x 64 consecutive entries, one run search for the
            // wave's first entry, then each lane walks the run table forward (runs of ~40
            // entries: a step of 64 crosses one or two), instead of a search per entry
            const uint32_t fw = fb + (t >> 6) * (64u * LOADS);
            uint32_t i = 0;
            if constexpr (WALK) i = run_of(s_pre, nt, fw < f1 ? fw : f1 - 1);
#pragma unroll
            for (int u = 0; u < LOADS; ++u) {
                const uint32_t f = WALK ? fw + u * 64u + (t & 63u) : fb + u * kL2Lanes + t;
                idx[u] = 0xFFFFFFFFu;
                o[u] = 0;
                if (f < f1) {
                    if constexpr (WALK) {
                        while (i + 1 < nt && s_pre[i + 1] <= f) ++i;
                    } else {
                        i = run_of(s_pre, nt, f);
                    }
                    idx[u] = s_gst[i] + (f - s_pre[i]);
                    o[u] = ci.recv[idx[u]];
                }
            }
            uint32_t v[LOADS];
#pragma unroll
            for (int u = 0; u < LOADS; ++u) {
                v[u] = 0;
                if (idx[u] != 0xFFFFFFFFu && (o[u] >> ci.sup_log2) == lsb && hoff + o[u] < ci.limit)
                    v[u] = bits[(hoff + o[u]) >> 5];
            }
#pragma unroll
            for (int u = 0; u < LOADS; ++u)
                if (idx[u] != 0xFFFFFFFFu) {
                    const bool ok = (o[u] >> ci.sup_log2) == lsb && hoff + o[u] < ci.limit;
                    out8[idx[u]] = ok ? (uint8_t)((v[u] >> ((o[u] ^ 7u) & 31u)) & 1u) : (uint8_t)0;
                }
        }
    }
    if constexpr (SIDE) side_hash(sh_mine);
}

// bin_mid over chunked windows: window w = (superbin sb, chunk group q) concatenates sb's runs
// from the group's chunks; each 8192-probe block is sorted by region in LDS as in bin_mid.
// The received entries are window-local offsets: an entry outside its superbin or past the
// shard is dropped (KEYS: answered 0), so peer data never addresses outside the bitset.  KEYS:
// each probe's position is its index in the receive buffer (no level-1 key array).
// CONTIG: lane t takes entries t * kChunkPerLane .. + kChunkPerLane - 1 of a block (its run walk
// rarely steps: runs average ~26 entries at 200B x 8), instead of entries 64 apart (a wave's
// loads 64 consecutive entries, and each lane's walk crosses ~2.5 runs per load).
template <bool KEYS, bool CONTIG = false>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8, 8)))
void bin_mid_chunks_kernel(BfChunkIn ci, uint32_t nsup, uint32_t nq, uint32_t region_log2, uint32_t rel_log2,
                           const uint32_t* __restrict__ base, const uint32_t* __restrict__ cb_base,
                           uint64_t max_chunks, uint16_t* __restrict__ tabs, uint32_t* __restrict__ level2,
                           uint32_t* __restrict__ level2_key, uint8_t* __restrict__ out8,
                           const uint2* __restrict__ runs) {
    __shared__ uint32_t s_pre[kRunsPerPass], s_gst[kRunsPerPass];
    __shared__ uint32_t s_cnt[1u << kMaxRel];
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_sorted[kBlockProbes];
    __shared__ uint32_t s_key[KEYS ? kBlockProbes : 1];
    const uint32_t t = threadIdx.x;
    uint32_t w_q, w_part;
    // linear order: the owner's few superbins (36 at P = 8) would leave XCDs unevenly loaded
    // grouped (0.405 vs 0.381 ms)
    const uint32_t sb = mid_superbin(nsup, nq, false, &w_q, &w_part);
    const uint32_t q = w_q, part = w_part;
    const uint32_t w = sb * nq + q;
    const uint32_t wbase = base[w];
    const uint32_t E = base[w + 1] - wbase;
    const uint32_t nblk = (E + kBlockProbes - 1) / kBlockProbes;
    const uint32_t c_lo = (uint32_t)((uint64_t)nblk * part / kMidParts);
    const uint32_t c_hi = (uint32_t)((uint64_t)nblk * (part + 1) / kMidParts);
    if (c_lo >= c_hi) return;   // workgroup-uniform
    const uint32_t b0 = cb_base[w];
    const uint32_t R = 1u << rel_log2;
    const uint32_t rmask = (1u << region_log2) - 1u;
    uint32_t sub = 0;
    while ((R << sub) < kMidBuckets) ++sub;
    const uint32_t NB = R << sub, smask_b = (1u << sub) - 1u;
    const uint32_t h = sb / ci.S, lsb = sb - h * ci.S;
    const uint64_t hoff = (uint64_t)h << 32;
    const uint32_t smask = (1u << ci.sup_log2) - 1u;
    // run table of the group's chunks: chunk_group_sum_kernel's (one coalesced load), or built
    // here from the directories (dependent reads: rank table, start, run table)
    const uint64_t nch = (uint64_t)ci.nsrc * chunks_per_src(ci), c0 = (uint64_t)q * kRunsPerPass;
    const uint32_t nt = (uint32_t)(nch - c0 < kRunsPerPass ? nch - c0 : kRunsPerPass);
    if (runs) {
        if (t < nt) {
            const uint2 r = runs[(uint64_t)w * kRunsPerPass + t];
            s_pre[t] = r.x;
            s_gst[t] = r.y;
        }
    } else {
        uint32_t len = 0, st = 0;
        if (t < nt) chunk_run(ci, h, lsb, c0 + t, &len, &st);
        const uint32_t ex = block_excl_scan(len, s_w, nullptr);
        if (t < nt) {
            s_pre[t] = ex;
            s_gst[t] = st;
        }
    }
    __syncthreads();
    auto load = [&](uint32_t f0, uint32_t* lv, uint32_t* kv) {
        const uint32_t fw = CONTIG ? f0 + t * (uint32_t)kChunkPerLane : f0 + (t >> 6) * (64u * kChunkPerLane);
        uint32_t i = run_of(s_pre, nt, fw < E ? fw : E - 1);
#pragma unroll
        for (int u = 0; u < kChunkPerLane; ++u) {
            const uint32_t f = CONTIG ? fw + u : fw + u * 64 + (t & 63u);
            lv[u] = 0xFFFFFFFFu;
            kv[u] = 0;
            if (f < E) {
                while (i + 1 < nt && s_pre[i + 1] <= f) ++i;
                const uint32_t idx = s_gst[i] + (f - s_pre[i]);
                const uint32_t o = ci.recv[idx];
                if ((o >> ci.sup_log2) == lsb && hoff + o < ci.limit) {
                    lv[u] = o & smask;
                    kv[u] = idx;
                } else if constexpr (KEYS) {
                    if (out8) out8[idx] = 0;   // an offset past the shard answers 0 (packed answers: never set)
                }
            }
        }
    };
    uint32_t lv[kChunkPerLane], kv[kChunkPerLane];
    load(c_lo * kBlockProbes, lv, kv);
    for (uint32_t c = c_lo; c < c_hi; ++c) {
        const uint32_t f0 = c * kBlockProbes;
        const uint32_t f1 = (E - f0 < kBlockProbes) ? E : f0 + kBlockProbes;
        if (t < NB) s_cnt[t] = 0;
        __syncthreads();
        uint32_t tag[kChunkPerLane];
#pragma unroll
        for (int u = 0; u < kChunkPerLane; ++u) {
            tag[u] = 0xFFFFFFFFu;
            if (lv[u] != 0xFFFFFFFFu) {
                const uint32_t bk = ((lv[u] >> region_log2) << sub) | (lv[u] & smask_b);
                tag[u] = (bk << 16) | atomicAdd(s_cnt + bk, 1u);
            }
        }
        uint32_t nlv[kChunkPerLane], nkv[kChunkPerLane];
        if (c + 1 < c_hi) load(f0 + kBlockProbes, nlv, nkv);   // next block in flight
        __syncthreads();
        const uint32_t cn = t < NB ? s_cnt[t] : 0u;
        const uint32_t cex = block_excl_scan(cn, s_w, nullptr);
        if (!(t & smask_b) && (t >> sub) <= R)
            tabs[(uint64_t)(t >> sub) * max_chunks + b0 + c] = (uint16_t)cex;   // [region][block]
        if (t < NB) s_cnt[t] = cex;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kChunkPerLane; ++u) {
            if (tag[u] != 0xFFFFFFFFu) {
                const uint32_t d = s_cnt[tag[u] >> 16] + (tag[u] & 0xFFFFu);
                s_sorted[d] = lv[u] & rmask;
                if constexpr (KEYS) s_key[d] = kv[u];
            }
        }
        __syncthreads();
        const uint32_t out0 = wbase + f0;
        for (uint32_t j = t; j < f1 - f0; j += kTile) {
            stage_store(level2 + out0 + j, s_sorted[j]);
            if constexpr (KEYS) level2_key[out0 + j] = s_key[j];
        }
        if (c + 1 < c_hi) {
#pragma unroll
            for (int u = 0; u < kChunkPerLane; ++u) {
                lv[u] = nlv[u];
                kv[u] = nkv[u];
            }
        }
    }
}

// Requester side of a chunked include?: one workgroup per route tile; the tile's chunk in
// every window (its place and length from the directory the route wrote) gives each entry's
// tile-relative key (slot16) and its answer bit; a 0 clears that key's answer in LDS, and the
// tile's answers leave as one coalesced store.
constexpr uint32_t kCombineLanes = 256;
__global__ __launch_bounds__(kCombineLanes) void combine_chunks_packed_kernel(
        const uint8_t* __restrict__ packed, const uint16_t* __restrict__ slot16, uint64_t wcap, uint64_t wcap8,
        BfChunks cg, uint32_t nwin, const unsigned long long* __restrict__ counts, uint64_t n, uint32_t tile_keys,
        uint8_t* __restrict__ out) {
    __shared__ uint8_t s_ans[2 * kTile];
    __shared__ uint32_t s_pre[kMaxOwners], s_st[kMaxOwners], s_w[16];
    const uint32_t t = threadIdx.x;
    const uint64_t tile = blockIdx.x, key0 = tile * tile_keys;
    const uint32_t tk = (uint32_t)(n - key0 < tile_keys ? n - key0 : tile_keys);
    for (uint32_t j = t; j < tile_keys; j += kCombineLanes) s_ans[j] = 1;
    uint32_t len = 0, st = 0;
    if (t < nwin && counts[t] <= wcap) {
        const uint8_t* d = cg.dir + (uint64_t)t * cg.dir_bytes;
        const uint32_t start = reinterpret_cast<const uint32_t*>(d)[tile];
        const uint32_t l = reinterpret_cast<const uint16_t*>(d + 4 * cg.tiles)[(uint64_t)cg.S * cg.tiles + tile];
        if (start != 0xFFFFFFFFu && (uint64_t)start + l <= wcap) {
            len = l;
            st = start;
        }
    }
    uint32_t E;
    const uint32_t ex = block_excl_scan(len, s_w, &E);
    if (t < nwin) {
        s_pre[t] = ex;
        s_st[t] = st;
    }
    __syncthreads();
    constexpr int U = 8;   // entries per lane in flight
    for (uint32_t fb = 0; fb < E; fb += U * kCombineLanes) {
        uint32_t key[U], byte[U], sh[U];
        // wave v takes U x 64 consecutive entries: one window search, then a forward walk
        const uint32_t fw = fb + (t >> 6) * (64u * U);
        uint32_t w = run_of(s_pre, nwin, fw < E ? fw : E - 1);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t f = fw + u * 64u + (t & 63u);
            key[u] = 0xFFFFFFFFu;
            byte[u] = 0xFFu;
            sh[u] = 0;
            if (f < E) {
                while (w + 1 < nwin && s_pre[w + 1] <= f) ++w;
                const uint64_t e = (uint64_t)s_st[w] + (f - s_pre[w]);
                key[u] = slot16[(uint64_t)w * wcap + e];
                byte[u] = packed[(uint64_t)w * wcap8 + (e >> 3)];
                sh[u] = (uint32_t)(e & 7u);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (key[u] < tk && !((byte[u] >> sh[u]) & 1u)) s_ans[key[u]] = 0;   // every writer stores the same 0
    }
    __syncthreads();
    for (uint32_t j = t; j < tk; j += kCombineLanes) out[key0 + j] = s_ans[j];
}

// ---- the sorted owner test's answers as packed bits, without a scatter -------------------
//
// bin_test writes each probe's answer at its receive position: at 200B x 8 that is ~10^8
// scattered byte stores per step (1.74 ms of bin_test's time, against ~0.5 ms for the same
// kernel storing the answers at their level-2 index: profiles/r06d_ab_test_order.jsonl).  The
// route claims window space tile by tile in arbitrary order, so a group of chunks spans its
// whole window.  Ranked chunks fix that: the route records the order it claimed each window's
// runs in (the directory's rank table), the owner's mid groups chunks by rank, and then group q's runs in
// sub-range h are ONE contiguous range of one window.  The test stores answers in level-2
// order (bin_test<L2ORDER>); chunk_unsort_kernel, one workgroup per (h, q), reads the group's
// level-2 entries (receive index + answer), sets the answer bits of that range in an LDS
// bitmap and stores them as the window's packed bits — the return trip's layout, so no
// separate pack pass either.
constexpr uint32_t kUnsortWords = 38912;       // LDS bitmap of one group's range per pass: 1,245,184 entries

// One workgroup per (group q, sub-range h): the answers of group q's level-2 entries in the
// superbins of h (ans2[l] at level-2 index l, its receive index level2_key[l]) as bits of the
// window's packed answers (window (h, src) at packed + (src * nh + h) * cap8, bit e = entry e,
// LSB first: combine_chunks_packed_kernel's layout).  packed must be zeroed: a live entry with no
// level-2 entry (its offset was past the shard) answers 0, and the range's two edge words, which
// it may share with the neighbouring groups, are ORed in.  A range wider than the LDS bitmap
// takes several passes over the group's entries (the 200B x 8 shard's first 2^32-bit sub-range:
// ~1.04M entries per group, one pass).
__global__ __launch_bounds__(1024) void chunk_unsort_kernel(BfChunkIn ci, uint32_t nq, uint32_t nsup,
                                                            const uint32_t* __restrict__ base,
                                                            const uint32_t* __restrict__ level2_key,
                                                            const uint8_t* __restrict__ ans2,
                                                            uint8_t* __restrict__ packed, uint64_t cap8) {
    __shared__ uint32_t s_bits[kUnsortWords];
    __shared__ uint32_t s_lo[16], s_hi[16];
    const uint32_t t = threadIdx.x, q = blockIdx.x, h = blockIdx.y;
    const uint64_t c0 = (uint64_t)q * kRunsPerPass;
    const uint32_t src = (uint32_t)(c0 / ci.cps);
    const uint64_t r0 = c0 - (uint64_t)src * ci.cps;
    if (src >= ci.nsrc || ci.counts[(uint64_t)src * ci.cstride + h] > ci.cap) return;   // overflowed: replayed
    const uint32_t j = h * ci.nsrc + src;
    // the group's range [lo, hi) of window j: its chunks' runs, consecutive by rank
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    const uint64_t tile = r0 + t < ci.tiles ? ranked_tile(ci, j, r0 + t) : ~0ull;
    if (tile != ~0ull) {
        const uint8_t* d = ci.dir + (uint64_t)j * ci.dir_bytes;
        const uint32_t st = reinterpret_cast<const uint32_t*>(d)[tile];
        const uint32_t ln = reinterpret_cast<const uint16_t*>(d + 4 * ci.tiles)[(uint64_t)ci.S * ci.tiles + tile];
        if (st != 0xFFFFFFFFu && ln && st < ci.cap) {   // chunk_run reads runs inside [st, min(st + ln, cap))
            lo = st;
            hi = (uint64_t)st + ln < ci.cap ? st + ln : (uint32_t)ci.cap;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {   // every lane of the workgroup is active here
        const uint32_t a = (uint32_t)__shfl_xor((int)lo, off), b = (uint32_t)__shfl_xor((int)hi, off);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    if ((t & 63u) == 0) {
        s_lo[t >> 6] = lo;
        s_hi[t >> 6] = hi;
    }
    __syncthreads();
    uint32_t LO = 0xFFFFFFFFu, HI = 0;
    for (uint32_t i = 0; i < 16; ++i) {
        LO = s_lo[i] < LO ? s_lo[i] : LO;
        HI = s_hi[i] > HI ? s_hi[i] : HI;
    }
    if (LO >= HI) return;   // workgroup-uniform: no probe of this group reached sub-range h
    const uint32_t a0 = LO & ~31u, nw = (HI - a0 + 31u) >> 5;
    uint32_t* out = reinterpret_cast<uint32_t*>(packed + ((uint64_t)src * ci.nh + h) * cap8) + (a0 >> 5);
    const uint64_t jbase = (uint64_t)j * ci.cap;
    const uint32_t sb1 = (h + 1) * ci.S < nsup ? (h + 1) * ci.S : nsup;
    constexpr uint32_t kU = 4;   // loads in flight per lane: 4 entries each (16 B of receive indices, 4 answers)
    for (uint32_t w0 = 0; w0 < nw; w0 += kUnsortWords) {   // passes of kUnsortWords words
        const uint32_t pw = nw - w0 < kUnsortWords ? nw - w0 : kUnsortWords;
        for (uint32_t i = t; i < pw; i += 1024) s_bits[i] = 0;
        __syncthreads();
        const uint32_t b0 = w0 << 5, b1 = (w0 + pw) << 5;   // this pass's entries, relative to a0
        for (uint32_t sb = h * ci.S; sb < sb1; ++sb) {
            const uint32_t w = sb * nq + q, l0 = base[w], l1 = base[w + 1];
            for (uint32_t q0 = (l0 & ~3u) + 4u * t; q0 < l1; q0 += 4u * 1024u * kU) {
                uint4 kv[kU];
                uint32_t av[kU];
#pragma unroll
                for (uint32_t u = 0; u < kU; ++u) {
                    const uint32_t qa = q0 + u * 4u * 1024u;
                    kv[u] = make_uint4(0, 0, 0, 0);
                    av[u] = 0;
                    if (qa < l1) {
                        kv[u] = *reinterpret_cast<const uint4*>(level2_key + qa);
                        av[u] = *reinterpret_cast<const uint32_t*>(ans2 + qa);
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < kU; ++u) {
                    const uint32_t qa = q0 + u * 4u * 1024u;
                    const uint32_t k4[4] = {kv[u].x, kv[u].y, kv[u].z, kv[u].w};
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        // e < cap (chunk_run's runs end inside the window); ri in [b0, b1): this pass
                        const uint32_t ri = (uint32_t)(k4[i] - jbase) - a0;
                        if (((av[u] >> (8 * i)) & 0xFFu) && qa + i >= l0 && qa + i < l1 && ri >= b0 && ri < b1)
                            atomicOr(s_bits + ((ri - b0) >> 5), 1u << (ri & 31u));
                    }
                }
            }
        }
        __syncthreads();
        for (uint32_t i = t; i < pw; i += 1024) {
            const bool edge = (w0 + i == 0) || (w0 + i == nw - 1);   // shared with the neighbouring groups
            if (edge) atomicOr(out + w0 + i, s_bits[i]);
            else out[w0 + i] = s_bits[i];
        }
        __syncthreads();   // the next pass clears the bitmap
    }
}

uint64_t align256(uint64_t x) { return (x + 255) & ~(uint64_t)255; }

struct Carve {
    uint32_t *level1, *level1_key, *level2, *level2_key, *gcnt, *gsum, *base, *cb_base, *cb_window, *cb_start;
    uint16_t *stab, *tabs;
    uint8_t* ans2;   // ranked chunked test: the answers in level-2 order
    uint2* runs;   // the chunked L2-local test's window run tables
    uint16_t* istart;   // ... and the first run of each of its items
    uint32_t* stot;   // hierarchical scan: per-superbin totals
    uint64_t bytes;
};

Carve carve(const BfBinPlan& p, void* at0) {
    Carve c{};
    uint8_t* at = static_cast<uint8_t*>(at0);
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) { uint8_t* q = at ? at + off : nullptr; off += align256(bytes); return q; };
    const uint64_t N = (uint64_t)p.nsup * p.ngroups;
    const bool l1 = !p.chunked;   // a chunked plan's level 1 is the received windows themselves
    c.level1 = l1 ? reinterpret_cast<uint32_t*>(take(p.probes * 4)) : nullptr;
    c.level2 = p.l2test ? nullptr : reinterpret_cast<uint32_t*>(take(p.probes * 4));
    c.level1_key = l1 && p.with_keys ? reinterpret_cast<uint32_t*>(take(p.probes * 4)) : nullptr;
    c.level2_key = p.with_keys && !p.l2test ? reinterpret_cast<uint32_t*>(take(p.probes * 4)) : nullptr;
    c.stab = l1 ? reinterpret_cast<uint16_t*>(take(p.ntiles * (p.nsup + 1) * 2)) : nullptr;   // [superbin][tile]
    c.gcnt = l1 ? reinterpret_cast<uint32_t*>(take((uint64_t)p.nblocks * p.nsup * 4)) : nullptr;
    c.gsum = reinterpret_cast<uint32_t*>(take(N * 4));
    c.base = reinterpret_cast<uint32_t*>(take((N + 1) * 4));
    c.cb_base = reinterpret_cast<uint32_t*>(take((N + 1) * 4));
    c.cb_window = reinterpret_cast<uint32_t*>(take(p.max_chunks * 4));
    c.cb_start = reinterpret_cast<uint32_t*>(take(p.max_chunks * 4));
    c.stot = reinterpret_cast<uint32_t*>(take(2 * kMaxSup * 4));
    if (p.l2test) {   // sorts nothing: the window run tables only
        c.runs = reinterpret_cast<uint2*>(take(N * kRunsPerPass * sizeof(uint2)));
        c.istart = reinterpret_cast<uint16_t*>(take(N * kL2MaxParts * sizeof(uint16_t)));
        c.bytes = off;
        return c;
    }
    if (p.chunked)   // the window run tables chunk_group_sum_kernel writes for bin_mid_chunks_kernel
        c.runs = reinterpret_cast<uint2*>(take(N * kRunsPerPass * sizeof(uint2)));
    c.tabs = reinterpret_cast<uint16_t*>(take(p.max_chunks * ((1ull << p.rel_log2) + 1) * 2));   // [region][block]
    if (p.ordered) c.ans2 = take(p.probes + 16);   // the unsort reads whole 4-byte quads
    c.bytes = off;
    return c;
}

// Window offsets and chunk blocks from gsum: one workgroup up to kScanWindows windows, the
// hierarchical scan beyond.
void launch_scan(const BfBinPlan& p, const Carve& c, hipStream_t s) {
    const uint32_t N = p.nsup * p.ngroups;
    if (N <= kScanWindows) {
        hipLaunchKernelGGL(bin_group_scan_kernel, dim3(1), dim3(1024), 0, s, c.gsum, N, c.base, c.cb_base,
                           c.cb_window, c.cb_start, p.ngroups, (unsigned long long*)nullptr);
        return;
    }
    hipLaunchKernelGGL(bin_scan_local_kernel, dim3(p.nsup), dim3(1024), 0, s, c.gsum, p.ngroups, c.base, c.cb_base,
                       c.stot);
    hipLaunchKernelGGL(bin_scan_top_kernel, dim3(1), dim3(1024), 0, s, c.stot, p.nsup, N, c.base, c.cb_base);
    hipLaunchKernelGGL(bin_scan_fill_kernel, dim3((N + 255) / 256), dim3(256), 0, s, c.gsum, N, p.ngroups, c.stot,
                       c.base, c.cb_base, c.cb_window, c.cb_start);
}

// bin_group_sum .. bin_mid over the level-1 array a front pass wrote.
hipError_t launch_groups_mid(const BfGeom& g, const BfBinPlan& p, const Carve& c, hipStream_t s, BfMarks* mk) {
    hipLaunchKernelGGL(bin_group_sum_kernel, dim3(p.nsup), dim3(kMaxBlocks), 0, s, c.gcnt, p.nblocks, p.nsup,
                       p.ngroups, c.gsum);
    launch_scan(p, c, s);
    bf_mark(mk, s, "bin_group");
    const uint32_t tiles_per_group = kGroupBlocks * p.tiles_per_block;
    if (p.with_keys)
        hipLaunchKernelGGL(bin_mid_kernel<true>, dim3(mid_grid(p.nsup, p.ngroups)), dim3(kTile), 0, s, c.level1,
                           c.level1_key, c.stab, p.ntiles, p.tile_probes, tiles_per_group, p.nsup, p.ngroups,
                           p.region_log2, p.rel_log2, c.base, c.cb_base, p.max_chunks, c.tabs, c.level2,
                           c.level2_key);
    else
        hipLaunchKernelGGL(bin_mid_kernel<false>, dim3(mid_grid(p.nsup, p.ngroups)), dim3(kTile), 0, s, c.level1,
                           c.level1_key, c.stab, p.ntiles, p.tile_probes, tiles_per_group, p.nsup, p.ngroups,
                           p.region_log2, p.rel_log2, c.base, c.cb_base, p.max_chunks, c.tabs, c.level2,
                           c.level2_key);
    bf_mark(mk, s, p.with_keys ? "bin_mid_keys" : "bin_mid");
    return hipGetLastError();
}

// bin_front .. bin_mid: the batch's probes in region-sorted chunk blocks.
// dig: keys16 holds the keys' SHA-1 words (uint4 per key) instead of key bytes (inserts only).
hipError_t launch_partition(const BfGeom& g, const BfBinPlan& p, const Carve& c, const uint8_t* keys16,
                            const uint64_t* offsets, uint64_t bias, uint64_t n, uint8_t* out8, hipStream_t s,
                            BfMarks* mk, bool dig = false) {
    const uint32_t sup_log2 = p.region_log2 + p.rel_log2;
    if (dig) {
        if (p.with_keys) return hipErrorInvalidValue;
        static const bool wide2 = [] {   // A/B: BFHIP_FRONT_WIDE2=0 takes one workgroup per CU
            const char* e = BF_AB_GETENV("BFHIP_FRONT_WIDE2");
            return !(e && e[0] == '0');
        }();
        if (g.k > (uint32_t)kSlots && wide2)
            hipLaunchKernelGGL(bin_front_wide_dig_kernel, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, bias,
                               n, p.tile_keys, p.tiles_per_block, sup_log2, p.nsup, c.level1, c.level1_key, c.stab,
                               c.gcnt, out8);
        else if (g.k > (uint32_t)kSlots)
            hipLaunchKernelGGL((bin_front_wide_kernel<false, true>), dim3(p.nblocks), dim3(kTile), 0, s, g, keys16,
                               offsets, bias, n, p.tile_keys, p.tiles_per_block, sup_log2, p.nsup, c.level1,
                               c.level1_key, c.stab, c.gcnt, out8);
        else
            hipLaunchKernelGGL(bin_front_kernel<true>, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, bias, n,
                               p.tile_keys, p.tiles_per_block, sup_log2, p.nsup, c.level1, c.level1_key, c.stab,
                               c.gcnt, out8);
        bf_mark(mk, s, "bin_front_digest");
        return launch_groups_mid(g, p, c, s, mk);
    }
    if (g.k > (uint32_t)kSlots) {
        if (p.with_keys)
            hipLaunchKernelGGL(bin_front_wide_kernel<true>, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets,
                               bias, n, p.tile_keys, p.tiles_per_block, sup_log2, p.nsup, c.level1, c.level1_key,
                               c.stab, c.gcnt, out8);
        else
            hipLaunchKernelGGL(bin_front_wide_kernel<false>, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets,
                               bias, n, p.tile_keys, p.tiles_per_block, sup_log2, p.nsup, c.level1, c.level1_key,
                               c.stab, c.gcnt, out8);
    } else if (p.with_keys)
        hipLaunchKernelGGL(bin_front_keys_kernel, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, bias, n,
                           p.tile_keys, p.tiles_per_block, sup_log2, p.nsup, c.level1, c.level1_key, c.stab, c.gcnt,
                           out8);
    else
        hipLaunchKernelGGL(bin_front_kernel<false>, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, bias, n,
                           p.tile_keys, p.tiles_per_block, sup_log2, p.nsup, c.level1, c.level1_key, c.stab, c.gcnt,
                           out8);
    bf_mark(mk, s, p.with_keys ? "bin_front_keys" : "bin_front");
    return launch_groups_mid(g, p, c, s, mk);
}

}  // namespace

namespace {

// Superbins of a bitset in the region size plan_common picks (0: no plan).
uint32_t superbins(uint64_t bitset_bytes, uint32_t pref_region_log2);

// Front tiles one pass can take: kMaxTilesPerBlock per workgroup, at most kMaxFrontBlocks
// workgroups, and (superbin, group) windows within the scan's kMaxWindows.
uint64_t max_tiles(uint64_t bitset_bytes, uint32_t pref_region_log2) {
    const uint32_t nsup = superbins(bitset_bytes, pref_region_log2);
    if (nsup == 0) return 0;
    const uint64_t groups = std::min<uint64_t>(kMaxWindows / nsup, kMaxGroups);
    const uint64_t blocks = std::min<uint64_t>(kMaxFrontBlocks, groups * kGroupBlocks);
    return blocks * kMaxTilesPerBlock;
}

}  // namespace

uint64_t bf_binned_max_keys(uint32_t k, uint64_t bitset_bytes, uint32_t pref_region_log2) {
    if (k == 0) return 0;
    const uint64_t tile_keys = k <= kTwoKeys ? 2 * kTile : kTile;
    const uint64_t n = max_tiles(bitset_bytes, pref_region_log2) * tile_keys;
    return std::min<uint64_t>(n, ((1ull << 32) - 1) / k);
}

uint64_t bf_binned_max_offsets(uint64_t bitset_bytes, uint32_t pref_region_log2) {
    return std::min<uint64_t>(max_tiles(bitset_bytes, pref_region_log2) * kTileProbes, (1ull << 32) - 1);
}

namespace {

// n units of k probes each, tile_units per front tile.
bool plan_common(uint64_t bitset_bytes, uint64_t n, uint32_t k, uint32_t tile_units, uint32_t pref_region_log2,
                 bool with_keys, BfBinPlan* plan) {
    const uint64_t probes = n * k;
    if (probes >= (1ull << 32)) return false;
    const uint64_t bits = bitset_bytes * 8;
    // region (LDS image) sizes tried, the preferred one first: 2^18 (32 KiB, 512 lanes), 2^19, 2^20
    const uint32_t order[3] = {pref_region_log2 == 20 ? 20u : (pref_region_log2 == 18 ? 18u : 19u),
                               pref_region_log2 == 20 ? 19u : (pref_region_log2 == 18 ? 19u : 20u),
                               pref_region_log2 == 18 ? 20u : 0u};
    for (uint32_t rl : order) {
        if (rl == 0) break;
        const uint64_t nbins = (bits + (1ull << rl) - 1) >> rl;
        uint32_t rel = 0;
        while (((nbins + (1ull << rel) - 1) >> rel) > kMaxSup) ++rel;
        if (rel > kMaxRel) continue;
        BfBinPlan p{};
        p.region_log2 = rl;
        p.nbins = (uint32_t)nbins;
        p.rel_log2 = rel;
        p.nsup = (uint32_t)((nbins + (1ull << rel) - 1) >> rel);
        p.with_keys = with_keys;
        p.tile_keys = tile_units;
        p.tile_probes = tile_units * k;
        p.ntiles = (n + tile_units - 1) / tile_units;
        p.tiles_per_block = (uint32_t)std::min<uint64_t>((p.ntiles + kMaxBlocks - 1) / kMaxBlocks, kMaxTilesPerBlock);
        if (p.ntiles > (uint64_t)kMaxFrontBlocks * p.tiles_per_block) continue;
        p.nblocks = (uint32_t)((p.ntiles + p.tiles_per_block - 1) / p.tiles_per_block);
        p.ngroups = (p.nblocks + kGroupBlocks - 1) / kGroupBlocks;
        if ((uint64_t)p.nsup * p.ngroups > kMaxWindows || p.ngroups > kMaxGroups) continue;
        p.probes = probes;
        p.max_chunks = (probes + kBlockProbes - 1) / kBlockProbes + (uint64_t)p.nsup * p.ngroups;
        p.scratch_bytes = carve(p, nullptr).bytes;
        *plan = p;
        return true;
    }
    return false;
}

uint32_t superbins(uint64_t bitset_bytes, uint32_t pref_region_log2) {
    BfBinPlan p{};
    return plan_common(bitset_bytes, 1, 1, 1, pref_region_log2, false, &p) ? p.nsup : 0;
}

}  // namespace

bool bf_binned_plan(uint64_t bitset_bytes, uint64_t n, uint32_t k, uint32_t pref_region_log2, bool with_keys,
                    BfBinPlan* plan) {
    if (k == 0 || k > (uint32_t)kWideSlots || n == 0) return false;
    return plan_common(bitset_bytes, n, k, k <= kTwoKeys ? 2 * kTile : kTile, pref_region_log2, with_keys, plan);
}

bool bf_binned_plan_offsets(uint64_t bitset_bytes, uint64_t count, uint32_t pref_region_log2, BfBinPlan* plan,
                            bool with_keys) {
    if (count == 0) return false;
    return plan_common(bitset_bytes, count, 1, kTileProbes, pref_region_log2, with_keys, plan);
}

namespace {

// Below the whole-region density, store only the vectors that gain a bit instead of every
// touched one: 10B@0.01 % step 6.27 ms against 6.43 (profiles/r03m_apply_fresh.jsonl).
// BFHIP_APPLY_FRESH=0 stores every touched vector (A/B only)
uint32_t apply_store_fresh() {
    static const uint32_t v = [] {
        const char* e = BF_AB_GETENV("BFHIP_APPLY_FRESH");
        return (uint32_t)!(e && e[0] == '0');
    }();
    return v;
}

// bin_apply's regions per XCD group (apply_region): 2 measured 2.394 / 2.395 ms against 2.423 /
// 2.431 (1) and 2.409 / 2.401 (4) at 10B (profiles/r04a_ab_xg.jsonl).  BFHIP_APPLY_XG overrides.
uint32_t apply_xcd_group() {
    static const uint32_t v = [] {
        const char* e = BF_AB_GETENV("BFHIP_APPLY_XG");
        return (e && e[0]) ? (uint32_t)std::strtoul(e, nullptr, 10) : 2u;
    }();
    return v;
}

// Workgroups of the persistent dense apply (bin_apply_pipe_kernel): one per CU (an LDS image
// plus two run-table buffers; 4 waves per SIMD for its register pipeline).  BFHIP_APPLY_PIPE_GRID=n overrides it; 0 takes bin_apply_kernel (A/B).
uint32_t apply_pipe_grid() {
    static const uint32_t v = [] {
        const char* e = BF_AB_GETENV("BFHIP_APPLY_PIPE_GRID");
        if (e && e[0]) return (uint32_t)std::strtoul(e, nullptr, 10);
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return (uint32_t)cus;
    }();
    return v;
}

// Dense apply form: 1 bin_apply_pipe_kernel, 0 bin_apply_kernel (BFHIP_APPLY_FORM, A/B).  By default a batch dense enough to rewrite whole regions (dense 2,
// the north-star step: 0.52 -> 0.474 ms) takes the pipelined form; a line-dense one (the 10B
// step, ~4 probes per line) keeps bin_apply (2.40 ms against 2.97 pipelined at one workgroup
// per CU: profiles/r03p_apply_pipe.jsonl; a two-workgroup-per-CU form with only the run table
// prefetched measured 2.44: the 10B apply is not bound by its dependent round trips).
uint32_t apply_form(uint32_t dense) {
    static const uint32_t v = [] {
        const char* e = BF_AB_GETENV("BFHIP_APPLY_FORM");
        return (e && e[0]) ? (uint32_t)std::strtoul(e, nullptr, 10) : 255u;
    }();
    return v != 255u ? v : (dense == 2 ? 1u : 0u);
}

hipError_t launch_apply(const BfGeom& g, const BfBinPlan& p, const Carve& c, uint64_t bitset_bytes,
                        uint32_t* any_flag, hipStream_t s, BfMarks* mk) {
    const uint64_t nwords = bitset_bytes / 4;
    // dense = 2: at least one probe per 16-B vector on average (the region is read before the
    // probe pass and written back whole); 1: at least one per 128-B line (read first, touched
    // vectors written); 0: sparse.  Measured at 1B@1 % (13 probes / line, 2: 0.503 -> 0.492
    // ms) and 10B@0.01 % (4 / line, 1: 2.81 -> 2.65 ms; writing whole lines there: 2.81)
    const uint64_t vecs = (uint64_t)p.nbins << (p.region_log2 - 7);
    const uint32_t dense = p.probes >= vecs ? 2u : (p.probes >= vecs / 8 ? 1u : 0u);
    const uint32_t pg = apply_pipe_grid();
    const uint32_t form = apply_form(dense);
    // the pipeline pays off over many regions per workgroup: a 150 MB shard (2288 regions, 9
    // per workgroup) measured 0.206 pipelined against 0.164 ms (P = 8 owner insert)
    if (dense && pg && p.region_log2 == 19 && form == 1 && p.nbins >= 16 * pg) {   // 2^20-bit regions: not pipelined
        [[maybe_unused]] static const int pl = [] {
            const char* e = BF_AB_GETENV("BFHIP_APPLY_PIPE_LOADS");
            return e && *e && std::atoi(e) == 4 ? 4 : 8;
        }();
#define BF_APPLY_PIPE(LD)                                                                                         \
    hipLaunchKernelGGL((bin_apply_pipe_kernel<19, kPipeLanes, LD>), dim3(std::min<uint32_t>(p.nbins, pg)),         \
                       dim3(kPipeLanes), 0, s, g.bits, nwords, p.nbins, c.level2, c.cb_base, c.cb_start, c.tabs,   \
                       p.max_chunks, p.ngroups, p.rel_log2, dense, any_flag, g.dirty, apply_store_fresh())
#ifdef BFHIP_AB_KNOBS
        if (pl == 4) BF_APPLY_PIPE(4);
        else
#endif
        BF_APPLY_PIPE(8);
#undef BF_APPLY_PIPE
    } else if (p.region_log2 == 18)
        hipLaunchKernelGGL((bin_apply_kernel<18, kApplyLanes / 2>), dim3(p.nbins), dim3(kApplyLanes / 2), 0, s,
                           g.bits, nwords, c.level2, c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups,
                           p.rel_log2, dense, any_flag, g.dirty, apply_store_fresh(), apply_xcd_group());
    else if (p.region_log2 == 19) {
        // level-2 loads per lane and gather step: a region's probes over all 16 waves (2) when
        // it has at most 16 x 64 x 4 of them, else fewer waves with more loads in flight each
        // (8).  10B@0.01 % (~2k probes per region): 2.37 -> 2.25 ms; a P = 8 owner's insert
        // (~44k per region): 0.16 ms at 8 against 0.23 at 2 (profiles/r04i_ab_apply_loads.jsonl)
        static const int forced = [] {
            const char* e = BF_AB_GETENV("BFHIP_APPLY_LOADS");
            const int v = e && *e ? std::atoi(e) : 0;
            return v == 1 || v == 2 || v == 4 || v == 8 ? v : 0;
        }();
        const int loads = forced ? forced : (p.probes <= (uint64_t)p.nbins * 4096u ? 2 : 8);
#define BF_APPLY19(LD)                                                                                          \
    hipLaunchKernelGGL((bin_apply_kernel<19, kApplyLanes, LD>), dim3(p.nbins), dim3(kApplyLanes), 0, s, g.bits, \
                       nwords, c.level2, c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups, p.rel_log2, dense, \
                       any_flag, g.dirty, apply_store_fresh(), apply_xcd_group())
        if (loads == 2) BF_APPLY19(2);
#ifdef BFHIP_AB_KNOBS
        else if (loads == 1) BF_APPLY19(1);
        else if (loads == 4) BF_APPLY19(4);
#endif
        else BF_APPLY19(8);
#undef BF_APPLY19
    }
    else
        hipLaunchKernelGGL((bin_apply_kernel<20, kApplyLanes>), dim3(p.nbins), dim3(kApplyLanes), 0, s, g.bits,
                           nwords, c.level2, c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups, p.rel_log2, dense,
                           any_flag, g.dirty, apply_store_fresh(), apply_xcd_group());
    bf_mark(mk, s, "bin_apply");
    return hipGetLastError();
}

}  // namespace

hipError_t bf_launch_insert_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                   const uint8_t* keys16, const uint64_t* offsets, uint64_t bias, uint64_t n,
                                   void* scratch, uint32_t* any_flag, hipStream_t s, BfMarks* mk) {
    if (n == 0) return hipSuccess;
    if (p.with_keys) return hipErrorInvalidValue;
    const Carve c = carve(p, scratch);
    hipError_t e = launch_partition(g, p, c, keys16, offsets, bias, n, nullptr, s, mk);
    if (e != hipSuccess) return e;
    return launch_apply(g, p, c, bitset_bytes, any_flag, s, mk);
}

hipError_t bf_launch_insert_binned_digests(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                           const uint4* dig, uint64_t n, void* scratch, uint32_t* any_flag,
                                           hipStream_t s, BfMarks* mk) {
    if (n == 0) return hipSuccess;
    if (p.with_keys) return hipErrorInvalidValue;
    const Carve c = carve(p, scratch);
    hipError_t e = launch_partition(g, p, c, reinterpret_cast<const uint8_t*>(dig), nullptr, 0, n, nullptr, s, mk, true);
    if (e != hipSuccess) return e;
    return launch_apply(g, p, c, bitset_bytes, any_flag, s, mk);
}

hipError_t bf_launch_shard_insert_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                         const void* local, bool route32, uint64_t count, void* scratch,
                                         uint32_t* any_flag, hipStream_t s, BfMarks* mk, uint64_t bias,
                                         const BfWindows& w) {
    if (count == 0) return hipSuccess;
    if (w.counts && (w.cap == 0 || w.cap % kTileProbes)) return hipErrorInvalidValue;
    const Carve c = carve(p, scratch);
    const uint32_t sup_log2 = p.region_log2 + p.rel_log2;
    if (route32)
        hipLaunchKernelGGL(bin_front_offsets_kernel<uint32_t>, dim3(p.nblocks), dim3(kTile), 0, s,
                           static_cast<const uint32_t*>(local), count, p.tiles_per_block, sup_log2, p.nsup, c.level1,
                           c.stab, c.gcnt, bias, w.counts, w.stride, w.cap, g.limit);
    else
        hipLaunchKernelGGL(bin_front_offsets_kernel<uint64_t>, dim3(p.nblocks), dim3(kTile), 0, s,
                           static_cast<const uint64_t*>(local), count, p.tiles_per_block, sup_log2, p.nsup, c.level1,
                           c.stab, c.gcnt, bias, w.counts, w.stride, w.cap, g.limit);
    bf_mark(mk, s, "bin_front_offsets");
    hipError_t e = launch_groups_mid(g, p, c, s, mk);
    if (e != hipSuccess) return e;
    return launch_apply(g, p, c, bitset_bytes, any_flag, s, mk);
}

namespace {

hipError_t launch_test(const BfGeom& g, const BfBinPlan& p, const Carve& c, uint64_t bitset_bytes, uint8_t* out8,
                       hipStream_t s, BfMarks* mk) {
    const uint64_t nwords = bitset_bytes / 4;
    if (p.region_log2 == 18)
        hipLaunchKernelGGL((bin_test_kernel<18, kApplyLanes / 2>), dim3(p.nbins), dim3(kApplyLanes / 2), 0, s,
                           g.bits, nwords, c.level2, c.level2_key, c.cb_base, c.cb_start, c.tabs, p.max_chunks,
                           p.ngroups, p.rel_log2, out8);
    else if (p.region_log2 == 19)
        hipLaunchKernelGGL((bin_test_kernel<19, kApplyLanes>), dim3(p.nbins), dim3(kApplyLanes), 0, s, g.bits,
                           nwords, c.level2, c.level2_key, c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups,
                           p.rel_log2, out8);
    else
        hipLaunchKernelGGL((bin_test_kernel<20, kApplyLanes>), dim3(p.nbins), dim3(kApplyLanes), 0, s, g.bits,
                           nwords, c.level2, c.level2_key, c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups,
                           p.rel_log2, out8);
    bf_mark(mk, s, "bin_test");
    return hipGetLastError();
}

}  // namespace

// Owner side of a partitioned include?: the received offsets sorted by region (their input
// positions riding along), each region of the shard loaded once into LDS, and every
// offset's answer byte written (preset to 1, cleared on a 0 bit).
hipError_t bf_launch_shard_test_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                       const void* local, bool route32, uint64_t count, void* scratch, uint8_t* out8,
                                       hipStream_t s, BfMarks* mk, uint64_t bias, const BfWindows& w) {
    if (count == 0) return hipSuccess;
    if (!p.with_keys || !out8) return hipErrorInvalidValue;
    if (w.counts && (w.cap == 0 || w.cap % kTileProbes)) return hipErrorInvalidValue;
    const Carve c = carve(p, scratch);
    const uint32_t sup_log2 = p.region_log2 + p.rel_log2;
    hipError_t e = hipMemsetAsync(out8, 1, count, s);
    if (e != hipSuccess) return e;
    if (route32)
        hipLaunchKernelGGL(bin_front_offsets_keys_kernel<uint32_t>, dim3(p.nblocks), dim3(kTile), 0, s,
                           static_cast<const uint32_t*>(local), count, p.tiles_per_block, sup_log2, p.nsup, c.level1,
                           c.level1_key, c.stab, c.gcnt, bias, w.counts, w.stride, w.cap, g.limit, out8);
    else
        hipLaunchKernelGGL(bin_front_offsets_keys_kernel<uint64_t>, dim3(p.nblocks), dim3(kTile), 0, s,
                           static_cast<const uint64_t*>(local), count, p.tiles_per_block, sup_log2, p.nsup, c.level1,
                           c.level1_key, c.stab, c.gcnt, bias, w.counts, w.stride, w.cap, g.limit, out8);
    bf_mark(mk, s, "bin_front_offsets_keys");
    if ((e = launch_groups_mid(g, p, c, s, mk)) != hipSuccess) return e;
    return launch_test(g, p, c, bitset_bytes, out8, s, mk);
}

hipError_t bf_launch_include_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                    const uint8_t* keys16, const uint64_t* offsets, uint64_t bias, uint64_t n,
                                    void* scratch, uint8_t* out8, hipStream_t s, BfMarks* mk) {
    if (n == 0) return hipSuccess;
    if (!p.with_keys || !out8) return hipErrorInvalidValue;
    const Carve c = carve(p, scratch);
    hipError_t e = launch_partition(g, p, c, keys16, offsets, bias, n, out8, s, mk);
    if (e != hipSuccess) return e;
    return launch_test(g, p, c, bitset_bytes, out8, s, mk);
}

// ---- partitioned filters, requester side ---------------------------------

namespace {

struct RouteCarve {
    uint32_t *lo1, *key1, *gcnt, *gsum, *base, *cb_base, *cb_window, *cb_start;
    uint8_t* hi1;
    uint16_t* stab;
    uint64_t bytes;
};

RouteCarve route_carve(const BfBinPlan& p, bool wide, bool with_slot, void* at0) {
    RouteCarve c{};
    uint8_t* at = static_cast<uint8_t*>(at0);
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) { uint8_t* q = at ? at + off : nullptr; off += align256(bytes); return q; };
    const uint64_t N = (uint64_t)p.nsup * p.ngroups;
    c.lo1 = reinterpret_cast<uint32_t*>(take(p.probes * 4));
    c.hi1 = wide ? take(p.probes) : nullptr;
    c.key1 = with_slot ? reinterpret_cast<uint32_t*>(take(p.probes * 4)) : nullptr;
    c.stab = reinterpret_cast<uint16_t*>(take(p.ntiles * (p.nsup + 1) * 2));
    c.gcnt = reinterpret_cast<uint32_t*>(take((uint64_t)p.nblocks * p.nsup * 4));
    c.gsum = reinterpret_cast<uint32_t*>(take(N * 4));
    c.base = reinterpret_cast<uint32_t*>(take((N + 1) * 4));
    c.cb_base = reinterpret_cast<uint32_t*>(take((N + 1) * 4));
    c.cb_window = reinterpret_cast<uint32_t*>(take(p.max_chunks * 4));
    c.cb_start = reinterpret_cast<uint32_t*>(take(p.max_chunks * 4));
    c.bytes = off;
    return c;
}

}  // namespace

// The route runs one batch in one pass (its send buffer is owner-major over the whole batch),
// so past kMaxBlocks x kMaxTilesPerBlock tiles it takes more front workgroups, as long as the
// (owner, group) windows fit the one-workgroup scan.

bool bf_route_plan(uint64_t n, uint32_t k, uint32_t shards, bool wide, bool with_slot, BfBinPlan* plan) {
    if (k == 0 || k > (uint32_t)kWideSlots || n == 0 || shards == 0 || shards > kMaxOwners) return false;
    const uint64_t probes = n * k;
    if (probes >= (1ull << 32)) return false;
    BfBinPlan p{};
    p.nsup = shards;   // buckets = owner shards
    p.tile_keys = k <= kTwoKeys ? 2 * kTile : kTile;
    p.tile_probes = p.tile_keys * k;
    p.ntiles = (n + p.tile_keys - 1) / p.tile_keys;
    p.tiles_per_block = (uint32_t)((p.ntiles + kMaxBlocks - 1) / kMaxBlocks);
    if (p.tiles_per_block > kMaxTilesPerBlock) p.tiles_per_block = kMaxTilesPerBlock;
    if (p.ntiles > (uint64_t)kMaxFrontBlocks * p.tiles_per_block) return false;
    p.nblocks = (uint32_t)((p.ntiles + p.tiles_per_block - 1) / p.tiles_per_block);
    p.ngroups = (p.nblocks + kGroupBlocks - 1) / kGroupBlocks;
    if ((uint64_t)p.nsup * p.ngroups > kScanWindows) return false;   // one-workgroup scan (per-owner totals)
    p.probes = probes;
    p.max_chunks = (probes + kBlockProbes - 1) / kBlockProbes + (uint64_t)p.nsup * p.ngroups;
    p.scratch_bytes = route_carve(p, wide, with_slot, nullptr).bytes;
    *plan = p;
    return true;
}

hipError_t bf_launch_route_fused(const BfGeom& g, const BfBinPlan& p, bool wide, const uint8_t* keys16,
                                 const uint64_t* offsets, uint64_t bias, uint64_t n, void* scratch, void* send,
                                 uint32_t* slot, unsigned long long* counts, hipStream_t s, BfMarks* mk) {
    const RouteCarve c = route_carve(p, wide, slot != nullptr, scratch);
    hipError_t e;
    if ((e = hipMemsetAsync(counts, 0, (uint64_t)p.nsup * sizeof(unsigned long long), s)) != hipSuccess) return e;
    if (n == 0) return hipSuccess;
#define BF_ROUTE_FRONT(W, S, SL)                                                                                  \
    hipLaunchKernelGGL((route_front_kernel<W, S, SL, false>), dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, \
                       bias, n, p.tile_keys, p.tiles_per_block, p.nsup, c.lo1, c.hi1, c.key1, c.stab, c.gcnt,       \
                       (uint64_t)0, nullptr, nullptr, nullptr, 1u, BfChunks{})
    if (g.k > (uint32_t)kSlots) {
        if (wide) { if (slot) BF_ROUTE_FRONT(true, true, kWideSlots); else BF_ROUTE_FRONT(true, false, kWideSlots); }
        else { if (slot) BF_ROUTE_FRONT(false, true, kWideSlots); else BF_ROUTE_FRONT(false, false, kWideSlots); }
    }
    else if (wide) { if (slot) BF_ROUTE_FRONT(true, true, kSlots); else BF_ROUTE_FRONT(true, false, kSlots); }
    else if (slot)
        hipLaunchKernelGGL((route_front32_kernel<true, false>), dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets,
                           bias, n, p.tile_keys, p.tiles_per_block, p.nsup, c.lo1, c.hi1, c.key1, c.stab, c.gcnt,
                           (uint64_t)0, nullptr, nullptr, nullptr, 1u, BfChunks{});
    else
        hipLaunchKernelGGL((route_front32_kernel<false, false>), dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets,
                           bias, n, p.tile_keys, p.tiles_per_block, p.nsup, c.lo1, c.hi1, c.key1, c.stab, c.gcnt,
                           (uint64_t)0, nullptr, nullptr, nullptr, 1u, BfChunks{});
#undef BF_ROUTE_FRONT
    bf_mark(mk, s, slot ? "route_front_slot" : "route_front");
    hipLaunchKernelGGL(bin_group_sum_kernel, dim3(p.nsup), dim3(kMaxBlocks), 0, s, c.gcnt, p.nblocks, p.nsup,
                       p.ngroups, c.gsum);
    hipLaunchKernelGGL(bin_group_scan_kernel, dim3(1), dim3(1024), 0, s, c.gsum, p.nsup * p.ngroups, c.base,
                       c.cb_base, c.cb_window, c.cb_start, p.ngroups, counts);
    bf_mark(mk, s, "route_group");
    const uint32_t tiles_per_group = kGroupBlocks * p.tiles_per_block;
    const dim3 grid((uint32_t)p.max_chunks);
#define BF_ROUTE_GATHER(W, S)                                                                                    \
    hipLaunchKernelGGL((route_gather_kernel<W, S>), grid, dim3(kTile), 0, s, c.lo1, c.hi1, c.key1, c.stab,       \
                       p.ntiles, p.tile_probes, tiles_per_group, p.nsup, p.ngroups, c.base, c.cb_base,          \
                       c.cb_window, send, slot)
    if (wide) { if (slot) BF_ROUTE_GATHER(true, true); else BF_ROUTE_GATHER(true, false); }
    else { if (slot) BF_ROUTE_GATHER(false, true); else BF_ROUTE_GATHER(false, false); }
#undef BF_ROUTE_GATHER
    bf_mark(mk, s, slot ? "route_gather_slot" : "route_gather");
    return hipGetLastError();
}

// Window route (bf_route_windows_dev): the front pass alone, each tile's runs written
// straight into fixed windows of wcap uint32 entries, window = owner * nh + (local >> 32)
// (nh = 1 when every shard fits 2^32 bits), with no level 1, group scan or gather.
// p comes from bf_route_plan over shards * nh buckets.
hipError_t bf_launch_route_windows(const BfGeom& g, const BfBinPlan& p, uint32_t nh, const uint8_t* keys16,
                                   const uint64_t* offsets, uint64_t bias, uint64_t n, void* send, uint32_t* slot,
                                   uint64_t wcap, unsigned long long* counts, hipStream_t s, BfMarks* mk) {
    hipError_t e;
    if ((e = hipMemsetAsync(counts, 0, (uint64_t)p.nsup * sizeof(unsigned long long), s)) != hipSuccess) return e;
    if (n == 0) return hipSuccess;
#define BF_ROUTE_WIN(KERNEL)                                                                                      \
    hipLaunchKernelGGL(KERNEL, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, bias, n, p.tile_keys,      \
                       p.tiles_per_block, p.nsup, nullptr, nullptr, nullptr, nullptr, nullptr, wcap, counts, send, \
                       slot, nh, BfChunks{})
    if (g.k > (uint32_t)kSlots) {
        if (slot) BF_ROUTE_WIN((route_front_kernel<false, true, kWideSlots, true>));
        else BF_ROUTE_WIN((route_front_kernel<false, false, kWideSlots, true>));
    }
    else if (slot) BF_ROUTE_WIN((route_front32_kernel<true, true>));
    else BF_ROUTE_WIN((route_front32_kernel<false, true>));
#undef BF_ROUTE_WIN
    bf_mark(mk, s, slot ? "route_win_slot" : "route_win");
    return hipGetLastError();
}

// ---- chunked windows: geometry, plans, launches ----------------------------------------------

bool bf_chunk_geometry(uint64_t shard0_bits, uint32_t nwin, uint32_t pref_region_log2, BfChunks* cg,
                       uint32_t max_buckets) {
    if (max_buckets == 0 || max_buckets > kChunkBuckets) max_buckets = kChunkBuckets;
    if (nwin == 0 || nwin > kMaxOwners) return false;
    const uint32_t rl = (pref_region_log2 >= 18 && pref_region_log2 <= 20) ? pref_region_log2 : 19u;
    uint64_t nbins0 = (shard0_bits + (1ull << rl) - 1) >> rl;
    if (nbins0 == 0) nbins0 = 1;
    for (uint32_t rel = 0; rel <= kMaxRel; ++rel) {
        const uint32_t sup_log2 = rl + rel;
        const uint64_t per_sub = 1ull << (32 - sup_log2);   // superbins per 2^32-bit sub-range window
        const uint64_t S = std::min<uint64_t>((nbins0 + (1ull << rel) - 1) >> rel, per_sub);
        if ((uint64_t)nwin * S > max_buckets) continue;
        BfChunks c{};
        c.S = (uint32_t)S;
        c.sup_log2 = sup_log2;
        c.region_log2 = rl;
        c.rel_log2 = rel;
        c.sub2 = 0;
        while (((uint64_t)nwin * S << (c.sub2 + 1)) <= max_buckets) ++c.sub2;
        *cg = c;
        return true;
    }
    return false;
}

uint64_t bf_chunk_dir_bytes(const BfChunks& cg, uint64_t tiles) {
    return (bf_chunk_dir_claim_offset(cg, tiles) + 8 + 15) & ~(uint64_t)15;
}

bool bf_chunk_ordered_ok(uint64_t tiles, uint64_t cap) {
    return tiles >= 1 && tiles < 0xFFFFu && ((cap + 7) / 8) % 4 == 0;
}

bool bf_chunk_plan(uint64_t bitset_bytes, const BfChunks& cg, uint32_t nh, uint32_t nsrc, uint64_t cap,
                   bool with_keys, BfBinPlan* plan, bool l2test, bool ordered) {
    if (nh == 0 || nsrc == 0 || cap == 0 || cg.tiles == 0) return false;
    const uint64_t probes = (uint64_t)nh * nsrc * cap;
    if (probes >= (1ull << 32)) return false;
    BfBinPlan p{};
    p.chunked = true;
    p.with_keys = with_keys;
    p.l2test = l2test && with_keys;
    p.ordered = ordered && with_keys && !p.l2test;
    if (p.ordered && !bf_chunk_ordered_ok(cg.tiles, cap)) return false;
    p.tiles = cg.tiles;
    p.nwin = nh * nsrc;
    p.cps = p.ordered ? (cg.tiles + kRunsPerPass - 1) / kRunsPerPass * kRunsPerPass : cg.tiles;
    p.region_log2 = cg.region_log2;
    p.rel_log2 = cg.rel_log2;
    const uint64_t bits = bitset_bytes * 8;
    const uint64_t nbins = (bits + (1ull << p.region_log2) - 1) >> p.region_log2;
    p.nbins = (uint32_t)nbins;
    p.nsup = (uint32_t)((nbins + (1ull << p.rel_log2) - 1) >> p.rel_log2);
    if (p.nsup == 0 || p.nsup > (uint64_t)nh * cg.S) return false;
    p.ngroups = (uint32_t)(((uint64_t)nsrc * p.cps + kRunsPerPass - 1) / kRunsPerPass);
    if ((uint64_t)p.nsup * p.ngroups > kMaxWindows || p.ngroups > kMaxGroups) return false;
    p.probes = probes;
    p.max_chunks = (probes + kBlockProbes - 1) / kBlockProbes + (uint64_t)p.nsup * p.ngroups;
    p.scratch_bytes = carve(p, nullptr).bytes;
    *plan = p;
    return true;
}

namespace {
hipError_t launch_chunk_mid(const BfBinPlan& p, const Carve& c, const BfChunkIn& ci, uint8_t* out8, hipStream_t s,
                            BfMarks* mk) {
    // the group sums also write each window's run table, which the mid's workgroups then read
    // in one coalesced load instead of walking the directories themselves
    uint2* runs = c.runs;
#ifdef BFHIP_AB_KNOBS
    if (const char* v = BF_AB_GETENV("BFHIP_MID_RUNS")) runs = atoi(v) ? runs : nullptr;   // (A/B)
#endif
    hipLaunchKernelGGL(chunk_group_sum_kernel, dim3(p.nsup, p.ngroups), dim3(kRunsPerPass), 0, s, ci, p.ngroups,
                       c.gsum, runs, 0u, (uint16_t*)nullptr);
    launch_scan(p, c, s);
    bf_mark(mk, s, "chunk_group");
#define BF_MID_CHUNKS(K, C)                                                                                     \
    hipLaunchKernelGGL((bin_mid_chunks_kernel<K, C>), dim3(p.nsup * p.ngroups * kMidParts), dim3(kTile), 0, s, ci,   \
                       p.nsup, p.ngroups, p.region_log2, p.rel_log2, c.base, c.cb_base, p.max_chunks, c.tabs, c.level2, \
                       c.level2_key, out8, runs)
    // lane-contiguous entries where the shard spans several 2^32-bit sub-ranges: 200B x 8, mids
    // 1.00 / 1.19 -> 0.93 / 1.12 ms; the north star x 8 (one sub-range) keeps the strided form,
    // 0.371 vs 0.393 ms (profiles/r06t_ab_mid_contig.jsonl)
    bool contig = ci.nh > 1;
#ifdef BFHIP_AB_KNOBS
    if (const char* e = BF_AB_GETENV("BFHIP_MID_CONTIG")) contig = e[0] == '1';   // (A/B)
#endif
    if (contig) {
        if (p.with_keys) BF_MID_CHUNKS(true, true);
        else BF_MID_CHUNKS(false, true);
    } else if (p.with_keys) {
        BF_MID_CHUNKS(true, false);
    } else {
        BF_MID_CHUNKS(false, false);
    }
#undef BF_MID_CHUNKS
    bf_mark(mk, s, p.with_keys ? "mid_chunks_keys" : "mid_chunks");
    return hipGetLastError();
}
}  // namespace

hipError_t bf_launch_shard_insert_chunks(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                         const BfChunkIn& ci, void* scratch, uint32_t* any_flag, hipStream_t s,
                                         BfMarks* mk) {
    if (!p.chunked || p.with_keys) return hipErrorInvalidValue;
    const Carve c = carve(p, scratch);
    hipError_t e = launch_chunk_mid(p, c, ci, nullptr, s, mk);
    if (e != hipSuccess) return e;
    return launch_apply(g, p, c, bitset_bytes, any_flag, s, mk);
}

hipError_t bf_launch_shard_insert_test_chunks_packed(const BfGeom& g, const BfBinPlan& pi, const BfBinPlan& pt,
                                                     uint64_t bitset_bytes, const BfChunkIn& cii, BfChunkIn cit,
                                                     void* scratch, uint32_t* any_flag, uint8_t* packed, hipStream_t s,
                                                     BfMarks* mk, const BfSideHash& side) {
    if (!pi.chunked || pi.with_keys || !pt.chunked || !pt.with_keys || !pt.ordered || !packed ||
        pi.region_log2 != pt.region_log2 || pi.rel_log2 != pt.rel_log2 || pi.nbins != pt.nbins ||
        pt.tiles != cit.tiles || pt.nwin != cit.nh * cit.nsrc)
        return hipErrorInvalidValue;
    const Carve ci_ = carve(pi, scratch);
    const Carve ct = carve(pt, static_cast<uint8_t*>(scratch) + carve(pi, nullptr).bytes);
    hipError_t e = launch_chunk_mid(pi, ci_, cii, nullptr, s, mk);   // the inserts' level 2
    if (e != hipSuccess) return e;
    cit.ranked = true;
    cit.cps = pt.cps;
    const uint64_t cap8 = (cit.cap + 7) / 8;
    if ((e = hipMemsetAsync(packed, 0, (uint64_t)pt.nwin * cap8, s)) != hipSuccess) return e;
    if ((e = launch_chunk_mid(pt, ct, cit, nullptr, s, mk)) != hipSuccess) return e;   // the tests' level 2 + keys
    const uint64_t nwords = bitset_bytes / 4;
    const BfL2 li{ci_.level2, ci_.cb_base, ci_.cb_start, ci_.tabs, pi.max_chunks, pi.ngroups};
    const BfL2 lt{ct.level2, ct.cb_base, ct.cb_start, ct.tabs, pt.max_chunks, pt.ngroups};
    const uint64_t vecs = (uint64_t)pi.nbins << (pi.region_log2 - 7);
    const uint32_t dense = pi.probes >= vecs ? 2u : (pi.probes >= vecs / 8 ? 1u : 0u);
    const int iloads = pi.probes <= (uint64_t)pi.nbins * 4096u ? 2 : 8;   // as launch_apply
#define BF_APPLY_TEST(RL, LANES, LD, SD)                                                                          \
    hipLaunchKernelGGL((bin_apply_test_kernel<RL, LANES, LD, SD>), dim3(pi.nbins), dim3(LANES), 0, s, g.bits, nwords, \
                       li, lt, pi.rel_log2, dense, any_flag, g.dirty, apply_store_fresh(), ct.ans2, side)
    const bool sd = side.n != 0;
    if (pi.region_log2 == 18) {   // (a 2^18-bit image cannot hold the side stage: hashed in a pass of its own)
        if (sd) {
            hipError_t he = bf_launch_keys(BF_OP_HASH, g, side.keys16, side.offsets, side.bias, side.n, nullptr,
                                           reinterpret_cast<uint64_t*>(side.dig), nullptr, s);
            if (he != hipSuccess) return he;
        }
        if (iloads == 2) BF_APPLY_TEST(18, kApplyLanes / 2, 2, false);
        else BF_APPLY_TEST(18, kApplyLanes / 2, 8, false);
    } else if (pi.region_log2 == 19) {
        if (iloads == 2) {
            if (sd) BF_APPLY_TEST(19, kApplyLanes, 2, true);
            else BF_APPLY_TEST(19, kApplyLanes, 2, false);
        } else {
            if (sd) BF_APPLY_TEST(19, kApplyLanes, 8, true);
            else BF_APPLY_TEST(19, kApplyLanes, 8, false);
        }
    } else {
        if (iloads == 2) {
            if (sd) BF_APPLY_TEST(20, kApplyLanes, 2, true);
            else BF_APPLY_TEST(20, kApplyLanes, 2, false);
        } else {
            if (sd) BF_APPLY_TEST(20, kApplyLanes, 8, true);
            else BF_APPLY_TEST(20, kApplyLanes, 8, false);
        }
    }
#undef BF_APPLY_TEST
    bf_mark(mk, s, sd ? "apply_test_hash" : "apply_test");
    hipLaunchKernelGGL(chunk_unsort_kernel, dim3(pt.ngroups, cit.nh), dim3(1024), 0, s, cit, pt.ngroups, pt.nsup,
                       ct.base, ct.level2_key, ct.ans2, packed, cap8);
    bf_mark(mk, s, "unsort_packed");
    return hipGetLastError();
}

uint64_t bf_chunk_scratch_bytes(const BfBinPlan& p) { return carve(p, nullptr).bytes; }

hipError_t bf_launch_shard_test_chunks(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                       const BfChunkIn& ci, void* scratch, uint8_t* out8, hipStream_t s,
                                       BfMarks* mk, const BfSideHash& side) {
    if (!p.chunked || !p.with_keys || !out8) return hipErrorInvalidValue;
    const Carve c = carve(p, scratch);
    if (p.l2test) {   // no sort: a superbin-major sweep, probes in receive order, answers stored in place
        // each XCD sweeps its own superbins, >= grid / 8 items each (chunk_test_l2_kernel)
        static const uint32_t grid = [] {
            const char* e = BF_AB_GETENV("BFHIP_L2_GRID");   // A/B: resident workgroups of the sweep
            const int v = e ? std::atoi(e) : (int)kL2Grid;
            return (uint32_t)(v >= 64 && v <= 8192 ? v : (int)kL2Grid) & ~7u;   // whole XCD groups
        }();
        // each XCD's grid / 8 workgroups share a superbin's items: at least one item each
        const uint32_t parts = std::min<uint32_t>((grid / 8 + p.ngroups - 1) / p.ngroups, kL2MaxParts);
        hipLaunchKernelGGL(chunk_group_sum_kernel, dim3(p.nsup, p.ngroups), dim3(kRunsPerPass), 0, s, ci, p.ngroups,
                           c.gsum, c.runs, parts, c.istart);
        bf_mark(mk, s, "chunk_group");
        // entries' runs: one search per wave and a forward walk (1), or a search per entry (0; A/B)
        [[maybe_unused]] static const bool walk = [] {
            const char* e = BF_AB_GETENV("BFHIP_L2_WALK");
            return !(e && *e == '0');
        }();
        [[maybe_unused]] static const int l2_loads = [] {
            const char* e = BF_AB_GETENV("BFHIP_L2_LOADS");
            return e && *e ? std::atoi(e) : kL2Loads;
        }();
        if (side.n)
            hipLaunchKernelGGL(chunk_test_l2_kernel<true>, dim3(grid), dim3(kL2Lanes), 0, s, ci, g.bits, p.nsup,
                               p.ngroups, parts, c.gsum, c.runs, c.istart, out8, side);
#ifdef BFHIP_AB_KNOBS
        else if (walk && l2_loads == 16)   // (A/B: BFHIP_L2_LOADS, entries per lane in flight)
            hipLaunchKernelGGL((chunk_test_l2_kernel<false, true, 16>), dim3(grid), dim3(kL2Lanes), 0, s, ci,
                               g.bits, p.nsup, p.ngroups, parts, c.gsum, c.runs, c.istart, out8, side);
        else if (walk && l2_loads == 4)
            hipLaunchKernelGGL((chunk_test_l2_kernel<false, true, 4>), dim3(grid), dim3(kL2Lanes), 0, s, ci,
                               g.bits, p.nsup, p.ngroups, parts, c.gsum, c.runs, c.istart, out8, side);
        else if (!walk)
            hipLaunchKernelGGL((chunk_test_l2_kernel<false, false>), dim3(grid), dim3(kL2Lanes), 0, s, ci, g.bits,
                               p.nsup, p.ngroups, parts, c.gsum, c.runs, c.istart, out8, side);
#endif
        else
            hipLaunchKernelGGL((chunk_test_l2_kernel<false, true>), dim3(grid), dim3(kL2Lanes), 0, s, ci, g.bits,
                               p.nsup, p.ngroups, parts, c.gsum, c.runs, c.istart, out8, side);
        bf_mark(mk, s, side.n ? "test_l2_hash" : "test_l2");
        return hipGetLastError();
    }
    if (side.n) {   // the sorted test has no latency to hide: hash in a pass of its own
        hipError_t e = bf_launch_keys(BF_OP_HASH, g, side.keys16, side.offsets, side.bias, side.n, nullptr,
                                      reinterpret_cast<uint64_t*>(side.dig), nullptr, s);
        if (e != hipSuccess) return e;
    }
    hipError_t e = hipMemsetAsync(out8, 1, p.probes, s);   // every entry's answer starts true
    if (e != hipSuccess) return e;
    if ((e = launch_chunk_mid(p, c, ci, out8, s, mk)) != hipSuccess) return e;
    return launch_test(g, p, c, bitset_bytes, out8, s, mk);
}

hipError_t bf_launch_shard_test_chunks_packed(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                              BfChunkIn ci, void* scratch, uint8_t* packed, hipStream_t s,
                                              BfMarks* mk) {
    if (!p.chunked || !p.with_keys || !p.ordered || !packed || p.tiles != ci.tiles || p.nwin != ci.nh * ci.nsrc)
        return hipErrorInvalidValue;
    const Carve c = carve(p, scratch);
    ci.ranked = true;
    ci.cps = p.cps;
    const uint64_t cap8 = (ci.cap + 7) / 8;
    hipError_t e = hipMemsetAsync(packed, 0, (uint64_t)p.nwin * cap8, s);   // entries with no level-2 entry answer 0
    if (e != hipSuccess) return e;
    if ((e = launch_chunk_mid(p, c, ci, nullptr, s, mk)) != hipSuccess) return e;
    const uint64_t nwords = bitset_bytes / 4;
    if (p.region_log2 == 18)
        hipLaunchKernelGGL((bin_test_kernel<18, kApplyLanes / 2, true>), dim3(p.nbins), dim3(kApplyLanes / 2), 0, s,
                           g.bits, nwords, c.level2, c.level2_key, c.cb_base, c.cb_start, c.tabs, p.max_chunks,
                           p.ngroups, p.rel_log2, c.ans2);
    else if (p.region_log2 == 19)
        hipLaunchKernelGGL((bin_test_kernel<19, kApplyLanes, true>), dim3(p.nbins), dim3(kApplyLanes), 0, s, g.bits,
                           nwords, c.level2, c.level2_key, c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups,
                           p.rel_log2, c.ans2);
    else
        hipLaunchKernelGGL((bin_test_kernel<20, kApplyLanes, true>), dim3(p.nbins), dim3(kApplyLanes), 0, s, g.bits,
                           nwords, c.level2, c.level2_key, c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups,
                           p.rel_log2, c.ans2);
    bf_mark(mk, s, "bin_test_l2order");
    hipLaunchKernelGGL(chunk_unsort_kernel, dim3(p.ngroups, ci.nh), dim3(1024), 0, s, ci, p.ngroups, p.nsup, c.base,
                       c.level2_key, c.ans2, packed, cap8);
    bf_mark(mk, s, "unsort_packed");
    return hipGetLastError();
}

hipError_t bf_launch_route_chunks(const BfGeom& g, const BfBinPlan& p, uint32_t nh, const BfChunks& cg,
                                  const uint8_t* keys16, const uint64_t* offsets, uint64_t bias, uint64_t n,
                                  void* send, uint16_t* slot16, uint64_t wcap, unsigned long long* counts,
                                  hipStream_t s, BfMarks* mk, bool dig) {
    hipError_t e;
    if ((e = hipMemsetAsync(counts, 0, (uint64_t)p.nsup * sizeof(unsigned long long), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(cg.dir, 0, (uint64_t)p.nsup * cg.dir_bytes, s)) != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    uint32_t* slot = reinterpret_cast<uint32_t*>(slot16);   // the CHUNK body stores u16 through it
#define BF_ROUTE_CH(KERNEL)                                                                                       \
    hipLaunchKernelGGL(KERNEL, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, bias, n, p.tile_keys,      \
                       p.tiles_per_block, p.nsup, nullptr, nullptr, nullptr, nullptr, nullptr, wcap, counts, send, \
                       slot, nh, cg)
    // the sorted-index form (route_chunks_idx_kernel) where the offset form holds one workgroup
    // per CU: k > 12 (200B x 8: 0.72 / 0.80 -> 0.62 / 0.66 ms insert / include? route); at k <= 12
    // route_front32's form already runs two and measured the same or 8 % faster (nstar x 8:
    // 0.331 vs 0.357 ms insert route), profiles/r06j_sim_P8.jsonl
    bool idx = g.k > (uint32_t)kSlots;
#ifdef BFHIP_AB_KNOBS
    if (const char* v = BF_AB_GETENV("BFHIP_ROUTE_IDX")) idx = atoi(v) != 0 && (g.k > (uint32_t)kSlots || dig);
#endif
    if (idx) {
        uint32_t* ws = static_cast<uint32_t*>(send);
#define BF_ROUTE_IDX(KERNEL)                                                                                       \
    hipLaunchKernelGGL(KERNEL, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, bias, n, p.tile_keys,          \
                       p.tiles_per_block, p.nsup, wcap, counts, ws, slot16, nh, cg)
        if (g.k > (uint32_t)kSlots) {
            if (dig) {
                if (slot16) BF_ROUTE_IDX((route_chunks_idx_kernel<true, kWideSlots>));
                else BF_ROUTE_IDX((route_chunks_idx_kernel<false, kWideSlots>));
            } else if (slot16) BF_ROUTE_IDX((route_chunks_idx_kernel<true, kWideSlots, true>));
            else BF_ROUTE_IDX((route_chunks_idx_kernel<false, kWideSlots, true>));
        }
#ifdef BFHIP_AB_KNOBS
        else if (slot16) BF_ROUTE_IDX((route_chunks_idx_kernel<true, kSlots>));
        else BF_ROUTE_IDX((route_chunks_idx_kernel<false, kSlots>));
#endif
#undef BF_ROUTE_IDX
    } else if (dig) {
        if (g.k > (uint32_t)kSlots) {
            if (slot16) BF_ROUTE_CH((route_front_kernel<false, true, kWideSlots, true, true, true>));
            else BF_ROUTE_CH((route_front_kernel<false, false, kWideSlots, true, true, true>));
        }
        else if (slot16) BF_ROUTE_CH((route_front32_kernel<true, true, true, true>));
        else BF_ROUTE_CH((route_front32_kernel<false, true, true, true>));
    } else if (g.k > (uint32_t)kSlots) {
        if (slot16) BF_ROUTE_CH((route_front_kernel<false, true, kWideSlots, true, true>));
        else BF_ROUTE_CH((route_front_kernel<false, false, kWideSlots, true, true>));
    }
    else if (slot16) BF_ROUTE_CH((route_front32_kernel<true, true, true>));
    else BF_ROUTE_CH((route_front32_kernel<false, true, true>));
#undef BF_ROUTE_CH
    bf_mark(mk, s, slot16 ? (dig ? "route_chunks_slot_dig" : "route_chunks_slot") : (dig ? "route_chunks_dig" : "route_chunks"));
    return hipGetLastError();
}

hipError_t bf_launch_combine_chunks_packed(const uint8_t* packed, const uint16_t* slot16, uint64_t wcap,
                                           const BfChunks& cg, uint32_t nwin, const unsigned long long* counts,
                                           uint64_t n, uint32_t tile_keys, uint8_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (nwin > kMaxOwners || tile_keys > 2 * kTile || tile_keys == 0) return hipErrorInvalidValue;
    const uint64_t grid = (n + tile_keys - 1) / tile_keys;
    hipLaunchKernelGGL(combine_chunks_packed_kernel, dim3((uint32_t)grid), dim3(kCombineLanes), 0, s, packed, slot16,
                       wcap, (wcap + 7) / 8, cg, nwin, counts, n, tile_keys, out);
    return hipGetLastError();
}

// ---- replicated inserts from region sets (BASELINE configs[3]'s layout) --------
//
// A replicated filter must OR every rank's batch into every replica.  Shipping SHA-1 words
// (16 B per key, 9.8 bits per probe at k = 13) is compact, but then every replica sorts all
// P batches' probes by region (the 8 x 2^24-key merged insert at 10B spends 8.8 of its 16.5 ms
// in bin_front + bin_mid, identical on every replica).  Here each rank sorts ITS OWN batch
// once (bin_front .. bin_mid) and encodes, per region, the set of distinct region-local offsets
// its probes hit as an Elias-Fano set: with n offsets in a region of U bits, l = floor(log2(U /
// n)) low bits of each offset in a packed array, then the high parts in unary (offset i sets
// bit (x_i >> l) + i of the upper bitmap): n (l + 1) + U / 2^l bits, ~ log2(U / n) + 2 bits per
// offset, about the SHA-1 words' size (sorted offsets carry no more entropy than that).  A
// region whose set would exceed U bits is written as its bitmap.  Every replica then ORs all
// ranks' sets in ONE pass over the bitset (sets_apply_kernel), with no sort at all.
//
// A set buffer (uint32 words): [0] magic "BFRS", [1] region_log2, [2] regions R, [3] words
// reserved, [4 + r] region r's first word (0: no offsets), [4 + R + r] its set's header word,
// sets from sets_first_word(R) in region order.  Region r's place is reserved before the encode (sets_size_kernel +
// sets_place_kernel): its probe count E_r from the level-2 run tables bounds its set at
// sets_region_words(E_r) words, so the encode needs no allocator and the layout is a function
// of the batch alone.  A set: word 0 = n | (l << 24) (l = 31: bitmap), then ceil(n l / 32)
// words of low bits (offset i's at bit i l, LSB first), then ceil((n + (U >> l)) / 32) words of
// the upper bitmap; a bitmap set is the region's U / 32 words in the bitset's own word layout.
namespace {
constexpr uint32_t kSetsMagic = 0x53524642u;   // "BFRS"
constexpr uint32_t kSetsHdr = 4;
constexpr uint32_t kSetsBitmap = 31u;
constexpr uint32_t kMaxSetSrc = 16;            // sources per sets_apply launch
constexpr uint32_t kLowsStage = 3840;           // low-bit words sets_apply stages in LDS (15 KB: two 2^19-bit workgroups per CU)
// [4, 4 + R): each region's first word; [4 + R, 4 + 2R): each region's set header (so a
// reader gets both in one round trip); the sets from sets_first_word(R)
__host__ __device__ inline uint64_t sets_first_word(uint32_t nbins) {
    return ((uint64_t)kSetsHdr + 2ull * nbins + 63) & ~(uint64_t)63;
}
// bit j of the result <-> region offset 32 w + j (the bitset's word w holds offset 32 w + j at
// bit j ^ 7: Redis byte order); an involution
__device__ __forceinline__ uint32_t offset_order(uint32_t w) { return __builtin_bswap32(__builtin_bitreverse32(w)); }

// An empty batch's buffer: the header and every region absent.
__global__ void sets_header_kernel(uint32_t* __restrict__ out, uint32_t rl, uint32_t nbins) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        out[0] = kSetsMagic;
        out[1] = rl;
        out[2] = nbins;
        out[3] = (uint32_t)sets_first_word(nbins);
    }
    if (i < nbins) {
        out[kSetsHdr + i] = 0;
        out[kSetsHdr + nbins + i] = 0;
    }
}

// A bound on the words of the set of a region its batch probes E times: the set has n <= E
// offsets and takes < n (log2(U / n) + 3) bits (l <= log2(U / n), U >> l < 2 n), increasing in
// n, or U bits as a bitmap (only when that is smaller); + a header word and two words of
// padding.  bf_sets_capacity_bytes bounds the sum over the regions (concave in E).
__device__ __forceinline__ uint32_t sets_region_words(uint32_t E, uint32_t U) {
    if (E == 0) return 0;
    const double e = (double)min(E, U), bits = e * (__log2f((float)((double)U / e)) + 3.01);
    return 4u + (uint32_t)((bits < (double)U ? bits : (double)U) / 32.0);
}

// Per superbin: region r's probe count E_r = sum over the superbin's level-2 blocks of its run
// length (a telescoping sum of the [region][block] run-start rows) -> its set's reserved words,
// their exclusive prefix inside the superbin into out[4 + r] (bit 31: the region has probes),
// and the superbin's total into sb_tot[sb] (sets_place_kernel scans those).
__global__ __launch_bounds__(1024) void sets_size_kernel(const uint16_t* __restrict__ tabs,
                                                         const uint32_t* __restrict__ cb_base, uint64_t max_chunks,
                                                         uint32_t nq, uint32_t rel_log2, uint32_t nbins, uint32_t U,
                                                         uint32_t* __restrict__ out, uint32_t* __restrict__ sb_tot) {
    __shared__ uint32_t s_row[(1u << kMaxRel) + 1];
    __shared__ uint32_t s_w[16];
    const uint32_t sb = blockIdx.x, t = threadIdx.x, R = 1u << rel_log2;
    const uint32_t bb0 = cb_base[sb * nq], bb1 = cb_base[(sb + 1) * nq];
    if (t <= R) {
        uint32_t sum = 0;
        const uint16_t* row = tabs + (uint64_t)t * max_chunks;
        for (uint32_t b = bb0; b < bb1; ++b) sum += row[b];
        s_row[t] = sum;
    }
    __syncthreads();
    const uint32_t r = sb * R + t;
    const uint32_t w = (t < R && r < nbins) ? sets_region_words(s_row[t + 1] - s_row[t], U) : 0u;
    uint32_t total;
    const uint32_t lp = block_excl_scan(w, s_w, &total);
    if (t < R && r < nbins) {
        out[kSetsHdr + r] = w ? (lp | 0x80000000u) : 0u;
        if (!w) out[kSetsHdr + nbins + r] = 0u;   // the encode writes the others
    }
    if (t == 0) sb_tot[sb] = total;
}

// One workgroup: each superbin's first word (sets from sets_first_word(R), superbins in order)
// into sb_tot, and the header; [3] = the words reserved in all (> the capacity cannot happen;
// the encode then writes no region past cap_words).
__global__ __launch_bounds__(1024) void sets_place_kernel(uint32_t* __restrict__ out, uint32_t* __restrict__ sb_tot,
                                                          uint32_t nsup, uint32_t rl, uint32_t nbins) {
    __shared__ uint32_t s_w[16];
    const uint32_t t = threadIdx.x;
    const uint32_t v = t < nsup ? sb_tot[t] : 0u;
    uint32_t total;
    const uint32_t ex = block_excl_scan(v, s_w, &total);
    const uint32_t first = (uint32_t)sets_first_word(nbins);
    if (t < nsup) sb_tot[t] = first + ex;
    if (t == 0) {
        out[0] = kSetsMagic;
        out[1] = rl;
        out[2] = nbins;
        out[3] = first + total;
    }
}

// One workgroup per region: the region's probes (level 2, as bin_apply gathers them) into an
// LDS bitmap, then each lane's WPL consecutive words -> its offsets in ascending order (their
// ranks from one workgroup scan of the lanes' counts), and the set written from them.
//   l >= 5 (at most U / 32 offsets, the sparse sets of every bench layout): each lane walks its
//   offsets once, in one loop over all its words — the next non-zero word re-read from the
//   bitmap, which stays intact — ORing every offset's low bits and upper-bitmap bit into a small
//   LDS image of the set (at most 14 KB, in the dead run table), copied out whole.  The loop's
//   trip count is the wave's largest per-lane offset count (~6 at the 10B layout), not the sum
//   over the lane's words of the wave's largest per-word count (~22: the r04 form, where every
//   word of every lane took at least one trip; VALU-bound).
//   l < 5 (dense) and bitmap sets: assembled in the bitmap's own LDS after every lane has taken
//   its words into registers.
// 78 KiB of LDS at 2^19-bit regions: two workgroups per CU.
// the LDS words the encode's run table / sparse-set image takes beside its bitmap
template <uint32_t RLOG2>
constexpr uint32_t sets_encode_run_lds() {
    constexpr uint32_t NW = (1u << RLOG2) / 32;
    // the gather's run table, then a sparse set's image: at l >= 5 (n <= U / 2^l) the low bits
    // take at most 5 NW / 32 words (l = 5) and the upper bitmap 2 NW / 32
    constexpr uint32_t kSetLds = 5u * NW / 32u + 2u * NW / 32u + 2u;
    return 2 * kRunsPerPass > kSetLds ? 2 * kRunsPerPass : kSetLds;
}

// Region r's set (nbins regions): the body of sets_encode_kernel, also run by
// sets_apply_encode_kernel after its apply of the same region, in the same LDS.
template <uint32_t RLOG2, uint32_t LANES, int LOADS>
__device__ __forceinline__ void sets_encode_region(uint32_t r, uint32_t nbins, const uint32_t* __restrict__ level2,
                                                   const uint32_t* __restrict__ cb_base,
                                                   const uint32_t* __restrict__ cb_start,
                                                   const uint16_t* __restrict__ tabs, uint64_t max_chunks,
                                                   uint32_t nq, uint32_t rel_log2, uint32_t* __restrict__ out,
                                                   const uint32_t* __restrict__ sb_first, uint32_t cap_words,
                                                   uint32_t stop, uint4* s_m4, uint32_t* s_runs, uint32_t* s_w) {
    constexpr uint32_t U = 1u << RLOG2, NW = U / 32, WPL = NW / LANES;
    static_assert(WPL * LANES == NW && WPL % 4 == 0 && WPL <= 32, "region words must tile the lanes in vectors");
    constexpr uint32_t kSetLds = 5u * NW / 32u + 2u * NW / 32u + 2u;
    uint32_t* s_m = reinterpret_cast<uint32_t*>(s_m4);
    uint32_t* s_pre = s_runs;
    uint32_t* s_gst = s_runs + kRunsPerPass;
    uint32_t* s_set = s_runs;
    const uint32_t t = threadIdx.x;
    // the region's reserved place: its superbin's first word + its prefix in the superbin
    // (sets_size_kernel / sets_place_kernel); loaded while the LDS image is cleared
    const uint32_t rv = out[kSetsHdr + r], sbf = sb_first[r >> rel_log2];
    for (uint32_t v = t; v < NW / 4; v += LANES) s_m4[v] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (!(rv & 0x80000000u)) return;   // workgroup-uniform: no probes (out[4 + r] is already 0)
#ifdef BFHIP_AB_KNOBS
    if (stop == 3) {   // (A/B: where the time goes; BFHIP_SETS_STOP) the region left absent
        if (t == 0) out[kSetsHdr + r] = out[kSetsHdr + nbins + r] = 0;   // every lane read rv before the barrier
        return;
    }
#endif
    const uint32_t st = sbf + (rv & 0x7FFFFFFFu);
    // LOADS level-2 loads per lane and step: a region's ~2k probes over all 16 waves (2), or
    // over 4 of them with more loads in flight each (8)
    for_region_probes<LOADS>(cb_base, cb_start, tabs, max_chunks, r, nq, rel_log2, s_pre, s_gst, s_w,
        [&](const uint32_t* idx) {
            uint32_t l[LOADS];
#pragma unroll
            for (int c = 0; c < LOADS; ++c) l[c] = idx[c] != 0xFFFFFFFFu ? level2[idx[c]] : 0xFFFFFFFFu;
#pragma unroll
            for (int c = 0; c < LOADS; ++c)
                if (l[c] != 0xFFFFFFFFu) atomicOr(s_m + (l[c] >> 5), 1u << ((l[c] ^ 7u) & 31u));
        });
#ifdef BFHIP_AB_KNOBS
    if (stop == 2) {   // (A/B)
        if (t == 0) out[kSetsHdr + r] = out[kSetsHdr + nbins + r] = 0;
        return;
    }
#endif
    // the run table is dead (for_region_probes ends on a barrier): a sparse set's image is
    // cleared; the scan's barriers below order these stores before its first atomic
    for (uint32_t v = t; v < kSetLds; v += LANES) s_set[v] = 0;
    // the lane's offset count and which of its words hold any (popcounts do not depend on the
    // bit order inside a word)
    uint32_t cnt = 0, nz = 0;
#pragma unroll
    for (uint32_t q = 0; q < WPL / 4; ++q) {
        const uint4 v = s_m4[t * (WPL / 4) + q];
        cnt += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
        nz |= (v.x ? 1u : 0u) << (4 * q) | (v.y ? 2u : 0u) << (4 * q) | (v.z ? 4u : 0u) << (4 * q) |
              (v.w ? 8u : 0u) << (4 * q);
    }
    uint32_t n;
    const uint32_t base = block_excl_scan(cnt, s_w, &n);
    uint32_t l = 0, lw = 0, uw = 0, words = 0;
    bool bitmap = false;
    if (n) {
        l = 31u - __clz(U / n);
        bitmap = (uint64_t)n * l + n + (U >> l) > U;
        lw = (n * l + 31u) / 32u;
        uw = (n + (U >> l) + 31u) / 32u;
        words = 1u + (bitmap ? NW : lw + uw);
    }
    // past the capacity (bf_sets_capacity_bytes bounds every batch, so never): not written,
    // and out[3] > capacity tells the reader
    const bool fits = (uint64_t)st + words <= cap_words;
    if (t == 0) {   // every lane read rv before the barriers above
        out[kSetsHdr + r] = fits ? st : 0u;
        out[kSetsHdr + nbins + r] = fits ? n | ((bitmap ? kSetsBitmap : l) << 24) : 0u;
    }
    if (!fits) return;   // workgroup-uniform
    uint32_t* o = out + st;
#ifdef BFHIP_AB_KNOBS
    if (stop == 1) {   // (A/B) the region left absent, so no reader decodes the unwritten set
        if (t == 0) out[kSetsHdr + r] = out[kSetsHdr + nbins + r] = 0;
        return;
    }
#else
    (void)stop;
#endif
    if (bitmap) {   // the LDS bitmap is still intact
        if (t == 0) o[0] = n | (kSetsBitmap << 24);
        for (uint32_t v = t; v < NW; v += LANES) o[1 + v] = s_m[v];
        return;
    }
    const uint32_t lmask = (1u << l) - 1u;   // l <= RLOG2 < 32
    if (t == 0) o[0] = n | (l << 24);
    // each lane's offsets in ascending order, low bits and upper-bitmap bit ORed into the set's
    // words at lo / up (one loop over all the lane's words, see above)
    auto walk = [&](uint32_t* lo_w, uint32_t* up_w) {
        uint32_t i = base, bp = base * l, w = 0, xb = 0;
        for (;;) {
            if (!w) {   // the lane's next non-zero word, from the bitmap
                if (!nz) break;
                const uint32_t j = (uint32_t)__builtin_ctz(nz);
                nz &= nz - 1u;
                w = offset_order(s_m[t * WPL + j]);
                xb = (t * WPL + j) * 32u;
            }
            const uint32_t x = xb | (uint32_t)__builtin_ctz(w);
            w &= w - 1u;
            if (l) {
                const uint32_t lo = x & lmask, sh = bp & 31u, wi = bp >> 5;
                atomicOr(lo_w + wi, lo << sh);
                if (sh + l > 32u) atomicOr(lo_w + wi + 1, lo >> (32u - sh));
            }
            const uint32_t u = (x >> l) + i;
            atomicOr(up_w + (u >> 5), 1u << (u & 31u));
            ++i;
            bp += l;
        }
    };
    if (l >= 5u) {   // workgroup-uniform: a sparse set (lw + uw <= kSetLds), built in LDS
        walk(s_set, s_set + lw);
        __syncthreads();
        for (uint32_t v = t; v < lw + uw; v += LANES) o[1 + v] = s_set[v];
        return;
    }
    // dense (more than U / 32 offsets, no bench layout): built in place in global memory, so
    // that the bitmap stays readable
    for (uint32_t v = t; v < lw + uw; v += LANES) o[1 + v] = 0;
    __threadfence();   // every lane's zeros are complete in memory (the barrier alone does not
    __syncthreads();   // wait for global stores) before any lane's atomics reach those words
    walk(o + 1, o + 1 + lw);
}


template <uint32_t RLOG2, uint32_t LANES, int LOADS>
__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(2 * LANES / 256))) void sets_encode_kernel(const uint32_t* __restrict__ level2,
                                                            const uint32_t* __restrict__ cb_base,
                                                            const uint32_t* __restrict__ cb_start,
                                                            const uint16_t* __restrict__ tabs, uint64_t max_chunks,
                                                            uint32_t nq, uint32_t rel_log2, uint32_t* __restrict__ out,
                                                            const uint32_t* __restrict__ sb_first, uint32_t cap_words,
                                                            uint32_t stop) {
    __shared__ uint4 s_m4[(1u << RLOG2) / 128];
    __shared__ uint32_t s_runs[sets_encode_run_lds<RLOG2>()], s_w[16];
    sets_encode_region<RLOG2, LANES, LOADS>(blockIdx.x, gridDim.x, level2, cb_base, cb_start, tabs, max_chunks, nq,
                                            rel_log2, out, sb_first, cap_words, stop, s_m4, s_runs, s_w);
}

// One workgroup per region: every source's set for the region ORed into an LDS image (bitmap
// sets word by word; Elias-Fano sets decoded one pass of LANES upper-bitmap words at a time
// across all sources: an offset's rank in its set is its rank among all sources' upper bits
// minus the offsets of the sources before it), then bin_apply's read-OR-write of the region.
// A source whose header does not match (magic, region geometry, capacity) is skipped and
// flagged in *status.
// sets_encode_kernel as a persistent grid: workgroup b encodes regions b, b + G, ... (G =
// gridDim.x).  An encoder handle's encode runs beside another stream's apply: with G = 3/4 of
// the CUs it holds one of the two workgroup slots of those CUs for the whole encode, and the
// apply keeps the rest, instead of the two kernels taking turns on whole CUs (the replicated
// 10B x 8 replica step 9.78 / 9.83 -> 9.54 / 9.59 ms; G = 224 / 256 / 320: 9.64 / 9.70 / 9.77,
// profiles/r06y_ab_sets_enc_grid.jsonl).
template <uint32_t RLOG2, uint32_t LANES, int LOADS>
__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(2 * LANES / 256)))
void sets_encode_persistent_kernel(const uint32_t* __restrict__ level2, const uint32_t* __restrict__ cb_base,
                                   const uint32_t* __restrict__ cb_start, const uint16_t* __restrict__ tabs,
                                   uint64_t max_chunks, uint32_t nq, uint32_t rel_log2, uint32_t* __restrict__ out,
                                   const uint32_t* __restrict__ sb_first, uint32_t cap_words, uint32_t nbins) {
    __shared__ uint4 s_m4[(1u << RLOG2) / 128];
    __shared__ uint32_t s_runs[sets_encode_run_lds<RLOG2>()], s_w[16];
    for (uint32_t r = blockIdx.x; r < nbins; r += gridDim.x) {
        sets_encode_region<RLOG2, LANES, LOADS>(r, nbins, level2, cb_base, cb_start, tabs, max_chunks, nq, rel_log2,
                                                out, sb_first, cap_words, 0u, s_m4, s_runs, s_w);
        __syncthreads();   // every lane is past the region's LDS before the next one clears it
    }
}

// sets_apply_kernel's LDS tables beside the region image and the low-bit stage
struct SetsApplyTabs {
    uint32_t w[16];
    uint32_t st[kMaxSetSrc], hdr[kMaxSetSrc], uw0[kMaxSetSrc + 1], np[kMaxSetSrc + 1], lw0[kMaxSetSrc + 1];
};

// Region r: the body of sets_apply_kernel, also run by sets_apply_encode_kernel.  Ends with every
// lane past its last LDS access of the image but without a barrier.
template <uint32_t RLOG2, uint32_t LANES, uint32_t STAGE>
__device__ __forceinline__ void sets_apply_region(uint32_t r, uint32_t* __restrict__ bits, uint64_t nwords,
                                                  const uint32_t* __restrict__ sets, uint64_t stride_words,
                                                  uint32_t nsrc, uint32_t nbins, uint32_t dense,
                                                  uint32_t* __restrict__ any_flag, uint8_t* __restrict__ dirty,
                                                  uint32_t store_fresh, uint32_t* __restrict__ status,
                                                  uint4* s_mask4, uint32_t* s_lows, SetsApplyTabs& T) {
    constexpr uint32_t kVec = 1u << (RLOG2 - 7);
    constexpr uint32_t kPer = kVec / LANES;
    constexpr uint32_t U = 1u << RLOG2, NW = U / 32;
    static_assert(kPer * LANES == kVec, "region must tile the workgroup");
    uint32_t* s_w = T.w;
    uint32_t* s_st = T.st;
    uint32_t* s_hdr = T.hdr;
    uint32_t* s_uw0 = T.uw0;
    uint32_t* s_np = T.np;
    uint32_t* s_lw0 = T.lw0;
    uint32_t* s_mask = reinterpret_cast<uint32_t*>(s_mask4);
    const uint32_t t = threadIdx.x;
    const uint64_t v0 = (uint64_t)r * kVec;
    const uint64_t nvec = nwords / 4;
    uint4* gv = reinterpret_cast<uint4*>(bits);
    uint4 old[kPer];
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {
        const uint32_t v = c * LANES + t;
        old[c] = make_uint4(0, 0, 0, 0);
        if (dense && v0 + v < nvec) old[c] = apply_load(gv + v0 + v);
    }
    for (uint32_t v = t; v < kVec; v += LANES) s_mask4[v] = make_uint4(0, 0, 0, 0);
    uint32_t st = 0, hdr = 0;
    if (t < nsrc) {   // source t's set for this region
        const uint32_t* S = sets + (uint64_t)t * stride_words;
        // (the host checked stride_words >= sets_first_word(nbins): the tables read below are
        // inside every buffer; [3] must cover them too and stay inside the stride)
        bool ok = S[0] == kSetsMagic && S[1] == RLOG2 && S[2] == nbins && S[3] >= sets_first_word(nbins) &&
                  S[3] <= stride_words;
        if (ok) {
            st = S[kSetsHdr + r];
            hdr = S[kSetsHdr + nbins + r];   // beside the place: one round trip
            if (st) {   // the set must lie inside the buffer: a damaged entry is skipped, not read
                const uint32_t n = hdr & 0xFFFFFFu, l = hdr >> 24;
                const bool shape = n && n <= U && (l == kSetsBitmap || (l >= 1u && l <= RLOG2));   // (EF: l >= 1)
                const uint64_t need = !shape ? 0 : 1ull + (l == kSetsBitmap ? NW : (n * l + 31u) / 32u + (n + (U >> l) + 31u) / 32u);
                if (!shape || (uint64_t)st + need > stride_words) {
                    ok = false;
                    st = hdr = 0;
                }
            }
        }
        if (!ok && status) atomicOr(status, 1u);
        s_st[t] = st;
        s_hdr[t] = hdr;
    }
    if (t < 64) {   // wave 0 (nsrc <= 16): upper-bitmap words, offsets and low-bit words of the
                    // Elias-Fano sources before each source, as three wave scans
        const uint32_t n = hdr & 0xFFFFFFu, l = hdr >> 24;
        const bool ef = st && l != kSetsBitmap;   // (st = 0 past nsrc)
        const uint32_t ua = ef ? (n + (U >> l) + 31u) / 32u : 0u, nn = ef ? n : 0u, ll = ef ? (n * l + 31u) / 32u : 0u;
        const uint32_t ia = wave_incl_scan(ua), in = wave_incl_scan(nn), il = wave_incl_scan(ll);
        if (t <= nsrc) {
            s_uw0[t] = ia - ua;
            s_np[t] = in - nn;
            s_lw0[t] = il - ll;
        }
    }
    __syncthreads();
    // the source of word q of a table of per-source starts (sources with no words are skipped)
    // (a binary search: the last source whose start is <= q; four dependent LDS reads)
    static_assert(kMaxSetSrc == 16, "source_of searches 16 sources");
    auto source_of = [&](const uint32_t* starts, uint32_t q) {
        uint32_t s = 0;
#pragma unroll
        for (uint32_t step = kMaxSetSrc / 2; step; step >>= 1)
            if (s + step < nsrc && starts[s + step] <= q) s += step;
        return s;
    };
    // The low bits are read in offset order, a word or two per offset: staged once into LDS,
    // coalesced, instead of a dependent global load per offset.  Sets too big for the stage
    // (dense regions, many sources) read them from global memory.
    const uint32_t TL = s_lw0[nsrc];
    const bool staged = STAGE && TL <= STAGE;   // workgroup-uniform
    if (staged) {
        for (uint32_t q = t; q < TL; q += LANES) {
            const uint32_t s = source_of(s_lw0, q);
            s_lows[q] = sets[(uint64_t)s * stride_words + s_st[s] + 1 + (q - s_lw0[s])];
        }
        if (t == 0) s_lows[TL] = 0;   // the word past the last source's lows: read, masked off
    }
    for (uint32_t s = 0; s < nsrc; ++s) {   // bitmap sets
        if (!s_st[s] || (s_hdr[s] >> 24) != kSetsBitmap) continue;   // workgroup-uniform
        const uint32_t* B = sets + (uint64_t)s * stride_words + s_st[s] + 1;
        for (uint32_t v = t; v < NW; v += LANES) {
            const uint32_t x = B[v];
            if (x) atomicOr(s_mask + v, x);
        }
    }
    const uint32_t TW = s_uw0[nsrc];
    uint32_t carry = 0;
    for (uint32_t g0 = 0; g0 < TW; g0 += LANES) {   // Elias-Fano sets
        const uint32_t g = g0 + t;
        uint32_t word = 0, s = 0;
        if (g < TW) {
            s = source_of(s_uw0, g);
            const uint32_t n = s_hdr[s] & 0xFFFFFFu, l = s_hdr[s] >> 24;
            word = sets[(uint64_t)s * stride_words + s_st[s] + 1 + (n * l + 31u) / 32u + (g - s_uw0[s])];
        }
        uint32_t tot;
        const uint32_t pre = block_excl_scan(__popc(word), s_w, &tot);   // (its barriers also order the staging)
        if (word) {   // ~16 offsets: their low bits are consecutive
            const uint32_t n = s_hdr[s] & 0xFFFFFFu, l = s_hdr[s] >> 24;
            const uint32_t lmask = (1u << l) - 1u;
            const uint32_t i = carry + pre - s_np[s];   // rank of this word's first offset in its set
            const uint32_t lim = (n * l + 31u) / 32u - 1u;   // last low-bits word (l >= 1)
            // offset i + e: high part p0 + (its bit in the word) - (i + e), low bits at (i + e) l.
            // The two loops differ only in where the low bits are read (LDS stage or the set in
            // global memory): one copy each, so neither reads through a flat (either-space) load.
            // Two offsets per trip: both low-bit reads are in flight together.
            auto decode = [&](const uint32_t* lw) {
                uint32_t d = (g - s_uw0[s]) * 32u - i, bp = i * l;
                while (word) {
                    // (l >= 1 by the header check; a damaged set's ranks can pass n: reads stay
                    // inside its lows)
                    const uint32_t b0 = (uint32_t)__builtin_ctz(word);
                    word &= word - 1u;
                    const bool two = word != 0u;
                    const uint32_t b1 = two ? (uint32_t)__builtin_ctz(word) : 0u;
                    word &= two ? word - 1u : word;
                    const uint32_t bq = bp + l;
                    const uint32_t w0 = min(bp >> 5, lim), w1 = min(bq >> 5, lim);
                    const uint32_t lo0 = __builtin_amdgcn_alignbit(lw[w0 + 1u], lw[w0], bp & 31u) & lmask;
                    const uint32_t lo1 = __builtin_amdgcn_alignbit(lw[w1 + 1u], lw[w1], bq & 31u) & lmask;
                    const uint32_t x0 = ((d + b0) << l) | lo0;
                    const uint32_t x1 = ((d - 1u + b1) << l) | lo1;
                    if (x0 < U) atomicOr(s_mask + (x0 >> 5), 1u << ((x0 ^ 7u) & 31u));
                    if (two && x1 < U) atomicOr(s_mask + (x1 >> 5), 1u << ((x1 ^ 7u) & 31u));
                    d -= two ? 2u : 1u;
                    bp += two ? 2u * l : l;
                }
            };
            if (staged) decode(s_lows + s_lw0[s]);   // workgroup-uniform; s_lows[TL] is a readable 0
            else decode(sets + (uint64_t)s * stride_words + s_st[s] + 1);
        }
        carry += tot;
    }
    __syncthreads();
    uint4 msk[kPer];
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {
        const uint32_t v = c * LANES + t;
        msk[c] = s_mask4[v];
        if (!dense && v0 + v < nvec && (msk[c].x | msk[c].y | msk[c].z | msk[c].w)) old[c] = apply_load(gv + v0 + v);
    }
    uint32_t fresh = 0;
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {
        const uint32_t v = c * LANES + t;
        const uint32_t fr = (msk[c].x & ~old[c].x) | (msk[c].y & ~old[c].y) | (msk[c].z & ~old[c].z) |
                            (msk[c].w & ~old[c].w);
        fresh |= fr;
        if (v0 + v >= nvec) continue;
        bool stv;
        if (dense == 2) stv = true;
        else if (store_fresh) stv = fr != 0u;
        else stv = (msk[c].x | msk[c].y | msk[c].z | msk[c].w) != 0u;
        if (stv)
            apply_store(gv + v0 + v, make_uint4(old[c].x | msk[c].x, old[c].y | msk[c].y, old[c].z | msk[c].z,
                                                old[c].w | msk[c].w));
        if (dirty && fr) dirty[((v0 + v) * 128) >> kDirtyShiftBits] = 1;
    }
    if (any_flag) report_any_new(any_flag, fresh != 0);
}

template <uint32_t RLOG2, uint32_t LANES, uint32_t STAGE>
__global__ __launch_bounds__(LANES) void sets_apply_kernel(uint32_t* __restrict__ bits, uint64_t nwords,
                                                           const uint32_t* __restrict__ sets, uint64_t stride_words,
                                                           uint32_t nsrc, uint32_t nbins, uint32_t dense,
                                                           uint32_t* __restrict__ any_flag, uint8_t* __restrict__ dirty,
                                                           uint32_t store_fresh, uint32_t* __restrict__ status,
                                                           uint32_t xg) {
    __shared__ uint4 s_mask4[1u << (RLOG2 - 7)];
    __shared__ SetsApplyTabs s_tabs;
    __shared__ uint32_t s_lows[STAGE + 1];   // every Elias-Fano source's low-bit words, back to back
    sets_apply_region<RLOG2, LANES, STAGE>(apply_region(blockIdx.x, gridDim.x, xg), bits, nwords, sets, stride_words,
                                           nsrc, nbins, dense, any_flag, dirty, store_fresh, status, s_mask4, s_lows,
                                           s_tabs);
}

// One step's two region passes in one launch (bf_insert_encode_region_sets_dev): region r's
// sets from every source ORed into the bitset (sets_apply_region), then, in the same LDS, region
// r's set of the NEXT batch encoded (sets_encode_region).  The two passes wait on different
// things — the apply on the bitset stream, the encode on LDS atomics and its VALU walk — and
// the two workgroups of a CU are at different points of their regions, so each hides the
// other's stalls; as two kernels on two streams they take turns on whole CUs instead (DESIGN
// §6b).  79.5 KiB of LDS at 2^19-bit regions: two workgroups per CU.
template <uint32_t RLOG2, uint32_t LANES, uint32_t STAGE, int LOADS>
__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(2 * LANES / 256)))
void sets_apply_encode_kernel(uint32_t* __restrict__ bits, uint64_t nwords, const uint32_t* __restrict__ sets,
                              uint64_t stride_words, uint32_t nsrc, uint32_t nbins, uint32_t dense,
                              uint32_t* __restrict__ any_flag, uint8_t* __restrict__ dirty, uint32_t store_fresh,
                              uint32_t* __restrict__ status, uint32_t xg, const uint32_t* __restrict__ level2,
                              const uint32_t* __restrict__ cb_base, const uint32_t* __restrict__ cb_start,
                              const uint16_t* __restrict__ tabs, uint64_t max_chunks, uint32_t nq, uint32_t rel_log2,
                              uint32_t* __restrict__ out, const uint32_t* __restrict__ sb_first, uint32_t cap_words) {
    constexpr uint32_t kRun = sets_encode_run_lds<RLOG2>();
    __shared__ uint4 s_mask4[1u << (RLOG2 - 7)];
    __shared__ SetsApplyTabs s_tabs;
    __shared__ uint32_t s_lows[(STAGE + 1) > kRun ? STAGE + 1 : kRun];
    const uint32_t r = apply_region(blockIdx.x, gridDim.x, xg);
    sets_apply_region<RLOG2, LANES, STAGE>(r, bits, nwords, sets, stride_words, nsrc, nbins, dense, any_flag, dirty,
                                           store_fresh, status, s_mask4, s_lows, s_tabs);
    __syncthreads();   // the image and the stage are reused by the encode
    sets_encode_region<RLOG2, LANES, LOADS>(r, nbins, level2, cb_base, cb_start, tabs, max_chunks, nq, rel_log2, out,
                                            sb_first, cap_words, 0u, s_mask4, s_lows, s_tabs.w);
}

#ifdef BFHIP_AB_KNOBS
// (A/B only, BFHIP_SETS_PIPE=1; measured slower, DESIGN §6f: 5.06 vs 4.58 ms at 10B x 8, 0.61
// vs 0.53 ms at the north star x 2 — one region per CU at a time loses to two one-shot
// workgroups per CU, whose decodes overlap each other's barrier and scan latency.)
// sets_apply_kernel, persistent and software-pipelined (one 1024-lane workgroup per CU walking
// regions r, r + G, ...), for batches dense enough to rewrite every region (VERDICT r04 item
// 4).  The one-shot kernel pays, per region, two dependent round trips (the per-source headers,
// then the sets' words) before it can decode, and at the 10B filter decodes every offset's low
// bits with a dependent global load (16 KB of them do not fit its 15 KB stage at two workgroups
// per CU).  Here, while region r is decoded from LDS, region r + G's set words (the first UPL
// upper-bitmap words and up to LPL low-bit words per lane) and its 64 KB of bitset vectors are
// already in flight in registers, and r + 2G's headers too; r's low bits were staged into LDS
// (LPL x LANES words, 24 KB) at the top of its iteration.  Region r + G's source tables (place,
// header, the three per-source prefixes) are built into the second of two LDS table buffers.
// The prefetch loads are unconditional (a clamped stand-in address past the data), so the
// compiler's in-order vmcnt waits leave them outstanding while r decodes.  Words beyond the
// prefetch (more than UPL x LANES upper words, or low bits past the stage) and bitmap sets are
// read on the spot, as the one-shot kernel does.  Results are the one-shot kernel's, bit for
// bit (tests/test_gpu_region_sets.py runs both).
template <uint32_t RLOG2, uint32_t LANES, uint32_t UPL, uint32_t LPL>
__global__ __launch_bounds__(LANES) __attribute__((amdgpu_waves_per_eu(4, 4))) void sets_apply_pipe_kernel(
    uint32_t* __restrict__ bits, uint64_t nwords, const uint32_t* __restrict__ sets, uint64_t stride_words,
    uint32_t nsrc, uint32_t nbins, uint32_t dense, uint32_t* __restrict__ any_flag, uint8_t* __restrict__ dirty,
    uint32_t store_fresh, uint32_t* __restrict__ status) {
    constexpr uint32_t kVec = 1u << (RLOG2 - 7);
    constexpr uint32_t kPer = kVec / LANES;
    constexpr uint32_t U = 1u << RLOG2, NW = U / 32;
    constexpr uint32_t kStage = LPL * LANES;
    static_assert(kPer * LANES == kVec, "region must tile the workgroup");
    __shared__ uint4 s_mask4[kVec];
    __shared__ uint32_t s_lows[kStage + 1];
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_st[2][kMaxSetSrc], s_hdr[2][kMaxSetSrc];
    __shared__ uint32_t s_uw0[2][kMaxSetSrc + 1], s_np[2][kMaxSetSrc + 1], s_lw0[2][kMaxSetSrc + 1];
    __shared__ uint32_t s_ok;
    uint32_t* s_mask = reinterpret_cast<uint32_t*>(s_mask4);
    const uint32_t t = threadIdx.x;
    const uint32_t G = gridDim.x;
    const uint64_t nvec = nwords / 4;
    uint4* gv = reinterpret_cast<uint4*>(bits);
    if (blockIdx.x >= nbins) return;   // workgroup-uniform
    const uint32_t last = blockIdx.x + (nbins - 1 - blockIdx.x) / G * G;
    auto clampr = [&](uint32_t q) { return q < last ? q : last; };

    // which sources' buffers match this filter (one header check per workgroup)
    if (t == 0) s_ok = 0;
    for (uint32_t v = t; v < kVec; v += LANES) s_mask4[v] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (t < nsrc) {
        const uint32_t* S = sets + (uint64_t)t * stride_words;
        const bool ok = S[0] == kSetsMagic && S[1] == RLOG2 && S[2] == nbins && S[3] >= sets_first_word(nbins) &&
                        S[3] <= stride_words;
        if (ok) atomicOr(&s_ok, 1u << t);
        else if (status) atomicOr(status, 1u);
    }
    __syncthreads();
    const uint32_t okmask = s_ok;
    const bool my_ok = t < nsrc && ((okmask >> t) & 1u);
    const uint32_t* mine = sets + (uint64_t)(t < nsrc ? t : 0) * stride_words;

    // region q's place and header of source t (lanes t < nsrc)
    auto load_hdr = [&](uint32_t q, uint32_t& st, uint32_t& hdr) {
        st = hdr = 0;
        if (my_ok) {
            st = mine[kSetsHdr + q];
            hdr = mine[kSetsHdr + nbins + q];
        }
    };
    // the tables of a region into buffer bi: damaged entries dropped (and flagged), the
    // per-source prefixes of upper words, offsets and low-bit words.  Contains a barrier.
    auto tables = [&](uint32_t bi, uint32_t st, uint32_t hdr) {
        if (t < 64) {
            if (t < nsrc && st) {
                const uint32_t n = hdr & 0xFFFFFFu, l = hdr >> 24;
                const bool shape = n && n <= U && (l == kSetsBitmap || (l >= 1u && l <= RLOG2));   // (EF: l >= 1)
                const uint64_t need = !shape ? 0 : 1ull + (l == kSetsBitmap ? NW : (n * l + 31u) / 32u +
                                                                                 (n + (U >> l) + 31u) / 32u);
                if (!shape || (uint64_t)st + need > stride_words) {
                    st = hdr = 0;
                    if (status) atomicOr(status, 1u);
                }
            }
            if (t >= nsrc) st = hdr = 0;
            const uint32_t n = hdr & 0xFFFFFFu, l = hdr >> 24;
            const bool ef = st && l != kSetsBitmap;
            const uint32_t ua = ef ? (n + (U >> l) + 31u) / 32u : 0u, nn = ef ? n : 0u,
                           ll = ef ? (n * l + 31u) / 32u : 0u;
            const uint32_t ia = wave_incl_scan(ua), in = wave_incl_scan(nn), il = wave_incl_scan(ll);
            if (t < nsrc) {
                s_st[bi][t] = st;
                s_hdr[bi][t] = hdr;
            }
            if (t <= nsrc) {
                s_uw0[bi][t] = ia - ua;
                s_np[bi][t] = in - nn;
                s_lw0[bi][t] = il - ll;
            }
        }
        __syncthreads();
    };
    // the last source whose start in table `starts` is <= q (four dependent LDS reads)
    auto source_of = [&](const uint32_t* starts, uint32_t q) {
        uint32_t s = 0;
#pragma unroll
        for (uint32_t stp = kMaxSetSrc / 2; stp; stp >>= 1)
            if (s + stp < nsrc && starts[s + stp] <= q) s += stp;
        return s;
    };
    // address of upper-bitmap word g / low-bit word q of the region in table bi (a stand-in,
    // the buffer's first word, past the region's words: every prefetch issues)
    auto upper_addr = [&](uint32_t bi, uint32_t g) -> const uint32_t* {
        if (g >= s_uw0[bi][nsrc]) return sets;
        const uint32_t s = source_of(s_uw0[bi], g);
        const uint32_t n = s_hdr[bi][s] & 0xFFFFFFu, l = s_hdr[bi][s] >> 24;
        return sets + (uint64_t)s * stride_words + s_st[bi][s] + 1 + (n * l + 31u) / 32u + (g - s_uw0[bi][s]);
    };
    auto lows_addr = [&](uint32_t bi, uint32_t q) -> const uint32_t* {
        if (q >= s_lw0[bi][nsrc]) return sets;
        const uint32_t s = source_of(s_lw0[bi], q);
        return sets + (uint64_t)s * stride_words + s_st[bi][s] + 1 + (q - s_lw0[bi][s]);
    };
    auto load_words = [&](uint32_t bi, uint32_t* uw, uint32_t* lo) {
#pragma unroll
        for (uint32_t p = 0; p < UPL; ++p) uw[p] = *upper_addr(bi, p * LANES + t);
#pragma unroll
        for (uint32_t j = 0; j < LPL; ++j) lo[j] = *lows_addr(bi, j * LANES + t);
    };
    auto load_vecs = [&](uint32_t q, uint4* vo) {
        const uint64_t v0 = (uint64_t)q * kVec;
#pragma unroll
        for (uint32_t c = 0; c < kPer; ++c) {
            const uint64_t v = v0 + c * LANES + t;
            vo[c] = apply_load(gv + (v < nvec ? v : nvec - 1));
        }
    };

    uint32_t fresh = 0;
    // Region r (tables in buffer bi, its vectors cur, words uw / lo in registers), r + G's
    // headers (hst, hhd) loaded.  Issues r + G's words / vectors into (nuw, nlo, nxt) and r + 2G's
    // headers into (nst, nhd).
    auto region = [&](uint32_t r, uint32_t bi, const uint4* cur, const uint32_t* uw, const uint32_t* lo,
                      uint32_t hst, uint32_t hhd, uint4* nxt, uint32_t* nuw, uint32_t* nlo, uint32_t& nst,
                      uint32_t& nhd) {
        // r's low bits into the stage (the previous region's decode ended on a barrier).  The
        // workgroup-uniform values read from LDS go through readfirstlane, so that their branches
        // are scalar: a wait inside a branch the compiler must treat as divergent runs on every
        // path, and a vmcnt(0) there would wait for r + G's prefetch
        const uint32_t TL = __builtin_amdgcn_readfirstlane(s_lw0[bi][nsrc]);
        const bool staged = TL <= kStage;   // workgroup-uniform
        if (staged) {
#pragma unroll
            for (uint32_t j = 0; j < LPL; ++j) s_lows[j * LANES + t] = lo[j];
            if (t == 0) s_lows[TL] = 0;   // read past the last source's lows, masked off
        }
        // r + G's tables (their barrier also publishes the stage), then its prefetches
        const uint32_t rn = clampr(r + G);
        tables(bi ^ 1u, hst, hhd);
        load_hdr(clampr(r + 2 * G), nst, nhd);
        load_words(bi ^ 1u, nuw, nlo);
        load_vecs(rn, nxt);
        // decode r: bitmap sets word by word (rare: read on the spot)
        for (uint32_t s = 0; s < nsrc; ++s) {
            const uint32_t sst = __builtin_amdgcn_readfirstlane(s_st[bi][s]);
            const uint32_t shd = __builtin_amdgcn_readfirstlane(s_hdr[bi][s]);
            if (!sst || (shd >> 24) != kSetsBitmap) continue;   // workgroup-uniform
            const uint32_t* B = sets + (uint64_t)s * stride_words + sst + 1;
            for (uint32_t v = t; v < NW; v += LANES) {
                const uint32_t x = B[v];
                if (x) atomicOr(s_mask + v, x);
            }
            __builtin_amdgcn_s_waitcnt(kWaitVm0);
        }
        // Elias-Fano sets: one pass of LANES upper words at a time over all sources.  The first
        // UPL passes use the prefetched words, as straight-line code: in a loop the compiler's
        // wait for those registers becomes vmcnt(0), which would also wait for r + G's prefetch.
        const uint32_t TW = __builtin_amdgcn_readfirstlane(s_uw0[bi][nsrc]);
        uint32_t carry = 0;
        // (staged is a compile-time branch: a run-time select between the LDS stage and global
        // memory would be a flat load, whose wait is vmcnt(0) as well)
        auto pass = [&](auto stg, uint32_t g, uint32_t word) {   // contains barriers (the scan)
            constexpr bool kStaged = decltype(stg)::value;
            uint32_t tot;
            const uint32_t pre = block_excl_scan(__popc(word), s_w, &tot);
            if (word) {
                const uint32_t s = source_of(s_uw0[bi], g);
                const uint32_t n = s_hdr[bi][s] & 0xFFFFFFu, l = s_hdr[bi][s] >> 24;
                const uint32_t* lows = sets + (uint64_t)s * stride_words + s_st[bi][s] + 1;
                const uint32_t* slows = s_lows + s_lw0[bi][s];
                const uint32_t lmask = (1u << l) - 1u;
                uint32_t i = carry + pre - s_np[bi][s];   // rank of this word's first offset in its set
                const uint32_t p0 = (g - s_uw0[bi][s]) * 32u;
                const uint32_t lim = l ? (n * l + 31u) / 32u - 1u : 0u;   // last low-bits word
                while (word) {
                    const uint32_t pp = p0 + (uint32_t)__builtin_ctz(word);
                    word &= word - 1u;
                    uint32_t lo_ = 0;
                    if (l) {
                        const uint32_t bp = i * l, wi = bp >> 5;
                        uint32_t a, b;
                        if constexpr (kStaged) {   // (a damaged set's ranks can pass n: reads stay inside its lows)
                            a = slows[min(wi, lim)];
                            b = slows[min(wi, lim) + 1u];
                        } else {
                            a = lows[min(wi, lim)];
                            b = lows[min(wi + 1u, lim)];
                        }
                        lo_ = (uint32_t)(((uint64_t)b << 32 | a) >> (bp & 31u)) & lmask;
                    }
                    const uint32_t x = ((pp - i) << l) | lo_;
                    if (x < U) atomicOr(s_mask + (x >> 5), 1u << ((x ^ 7u) & 31u));
                    ++i;
                }
            }
            carry += tot;
        };
        if (staged) {
#pragma unroll
            for (uint32_t p = 0; p < UPL; ++p)   // workgroup-uniform tests
                if (p * LANES < TW) pass(std::true_type{}, p * LANES + t, p * LANES + t < TW ? uw[p] : 0u);
        } else {   // (low bits past the stage: read on the spot, each read waited out)
#pragma unroll
            for (uint32_t p = 0; p < UPL; ++p)
                if (p * LANES < TW) pass(std::false_type{}, p * LANES + t, p * LANES + t < TW ? uw[p] : 0u);
        }
        for (uint32_t g0 = UPL * LANES; g0 < TW; g0 += LANES) {   // more upper words: read on the spot
            const uint32_t g = g0 + t;
            const uint32_t word = g < TW ? *upper_addr(bi, g) : 0u;
            if (staged) pass(std::true_type{}, g, word);
            else pass(std::false_type{}, g, word);
            __builtin_amdgcn_s_waitcnt(kWaitVm0);   // (the rare path ends on a full wait, as the main path may assume)
        }
        __syncthreads();   // the image is complete
        const uint64_t v0 = (uint64_t)r * kVec;
#pragma unroll
        for (uint32_t c = 0; c < kPer; ++c) {
            const uint32_t v = c * LANES + t;
            const uint4 m = s_mask4[v];
            s_mask4[v] = make_uint4(0, 0, 0, 0);
            if (v0 + v < nvec && (dense == 2 || (m.x | m.y | m.z | m.w))) {
                const uint32_t fr = (m.x & ~cur[c].x) | (m.y & ~cur[c].y) | (m.z & ~cur[c].z) | (m.w & ~cur[c].w);
                fresh |= fr;
                if (store_fresh && dense != 2 && !fr) continue;
                apply_store(gv + v0 + v, make_uint4(cur[c].x | m.x, cur[c].y | m.y, cur[c].z | m.z, cur[c].w | m.w));
                if (dirty && fr) dirty[((v0 + v) * 128) >> kDirtyShiftBits] = 1;
            }
        }
        __syncthreads();   // every lane is past its reads of the stage and of table bi
    };

    // prologue: region blockIdx.x's tables, words and vectors; the next region's headers
    uint32_t r = blockIdx.x;
    uint4 bufA[kPer], bufB[kPer];
    uint32_t uwA[UPL], uwB[UPL], loA[LPL], loB[LPL];
    uint32_t stA, hdA, stB, hdB;
    {
        uint32_t st0, hd0;
        load_hdr(r, st0, hd0);
        tables(0u, st0, hd0);
        load_hdr(clampr(r + G), stA, hdA);
        load_words(0u, uwA, loA);
        load_vecs(r, bufA);
    }
    for (;; r += 2 * G) {
        region(r, 0u, bufA, uwA, loA, stA, hdA, bufB, uwB, loB, stB, hdB);
        if (r + G >= nbins) break;
        region(r + G, 1u, bufB, uwB, loB, stB, hdB, bufA, uwA, loA, stA, hdA);
        if (r + 2 * G >= nbins) break;
    }
    if (any_flag) report_any_new(any_flag, fresh != 0);
}
#endif  // BFHIP_AB_KNOBS
}  // namespace

namespace {
// A/B only (BFHIP_SETS_STOP, -DBFHIP_AB_KNOBS builds): the encode stops after its probe pass
// (2), before writing the set (1), or at once (3); the output is then incomplete.  0: the whole
// encode (the shipped library has no stop points at all).
uint32_t sets_stop() {
    static const uint32_t v = [] {
        const char* e = BF_AB_GETENV("BFHIP_SETS_STOP");
        return (e && e[0]) ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
    }();
    return v;
}
}  // namespace

uint64_t bf_sets_header_words(uint32_t nbins) { return sets_first_word(nbins); }

bool bf_sets_geometry(uint64_t bitset_bytes, uint32_t pref_region_log2, uint32_t* region_log2, uint32_t* nbins) {
    BfBinPlan p{};
    if (!plan_common(bitset_bytes, 1, 1, 1, pref_region_log2, false, &p)) return false;
    if (p.region_log2 != 18 && p.region_log2 != 19) return false;   // the encode's LDS holds <= 2^19 bits
    *region_log2 = p.region_log2;
    *nbins = p.nbins;
    return true;
}

uint64_t bf_sets_capacity_bytes(uint64_t bitset_bytes, uint32_t pref_region_log2, uint64_t n, uint32_t k) {
    uint32_t rl = 0, R = 0;
    if (!bf_sets_geometry(bitset_bytes, pref_region_log2, &rl, &R)) return 0;
    // n k probes hit at most N = n k distinct offsets.  A set of n_r offsets takes < n_r
    // (log2(U / n_r) + 3) bits (l <= log2(U / n_r), U >> l < 2 n_r), concave in n_r, so over R
    // regions the total peaks at an even split: N (log2(U R / N) + 3); a bitmap set (U bits)
    // is taken only below its Elias-Fano size.  Plus 4 words of header and padding per region
    // (sets_region_words: the places reserved per region before the encode).
    const double U = (double)(1ull << rl), N = std::min((double)n * (double)k, U * R);
    double bitsum = 0.0;
    if (N > 0) bitsum = std::min(N * (std::log2(U * R / N) + 3.01), U * R) * 1.01 + 4096.0;
    const uint64_t words = sets_first_word(R) + 4ull * R + (uint64_t)(bitsum / 32.0) + 64;   // (first word: 2R tables)
    return ((words + 63) & ~63ull) * 4;   // whole 256-B units: buffers laid end to end stay aligned
}

hipError_t bf_launch_encode_sets(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes, const uint8_t* keys16,
                                 const uint64_t* offsets, uint64_t bias, uint64_t n, bool dig, void* scratch,
                                 uint32_t* out, uint64_t cap_words, hipStream_t s, BfMarks* mk,
                                 uint32_t persistent_grid) {
    (void)bitset_bytes;
    if (cap_words >= (1ull << 32)) return hipErrorInvalidValue;
    if (n == 0) {
        hipLaunchKernelGGL(sets_header_kernel, dim3((p.nbins + 255) / 256), dim3(256), 0, s, out, p.region_log2, p.nbins);
        return hipGetLastError();
    }
    if (p.with_keys) return hipErrorInvalidValue;
    const Carve c = carve(p, scratch);
    hipError_t e = launch_partition(g, p, c, keys16, offsets, bias, n, nullptr, s, mk, dig);
    if (e != hipSuccess) return e;
    // c.stot (the hierarchical scan's superbin totals) is free once bin_mid has run
    hipLaunchKernelGGL(sets_size_kernel, dim3(p.nsup), dim3(1024), 0, s, c.tabs, c.cb_base, p.max_chunks, p.ngroups,
                       p.rel_log2, p.nbins, 1u << p.region_log2, out, c.stot);
    hipLaunchKernelGGL(sets_place_kernel, dim3(1), dim3(1024), 0, s, out, c.stot, p.nsup, p.region_log2, p.nbins);
    // level-2 loads per lane and gather step, as bin_apply chooses them: 2 (a region's probes
    // over all 16 waves) up to 4096 probes per region on average, else 8.  10B (~2k per region):
    // 2.85 (2) / 2.94 (4) / 3.26 (8) ms, r04 encode; north star x 2 (~5.5k): 0.552 / 0.546 (2),
    // 0.532 / 0.517 (4), 0.520 / 0.520 (8) ms (profiles/r04h_ab_sets_enc_loads.jsonl,
    // r05w_ab_sets_enc_loads_nstar.jsonl).  BFHIP_SETS_ENC_LOADS (A/B) forces 1, 2, 4 or 8.
    static const int forced = [] {
        const char* e = BF_AB_GETENV("BFHIP_SETS_ENC_LOADS");
        const int v = e && *e ? std::atoi(e) : 0;
        return v == 8 || v == 4 || v == 2 || v == 1 ? v : 0;
    }();
    const int loads = forced ? forced : (n * g.k <= (uint64_t)p.nbins * 4096u ? 2 : 8);
    uint32_t enc_grid = persistent_grid;
#ifdef BFHIP_AB_KNOBS
    if (const char* e = BF_AB_GETENV("BFHIP_SETS_ENC_GRID")) enc_grid = (uint32_t)std::strtoul(e, nullptr, 10);   // (A/B)
#endif
    if (enc_grid && p.region_log2 == 19) {
        if (loads == 8)
            hipLaunchKernelGGL((sets_encode_persistent_kernel<19, kApplyLanes, 8>), dim3(enc_grid), dim3(kApplyLanes),
                               0, s, c.level2, c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups, p.rel_log2, out,
                               c.stot, (uint32_t)cap_words, p.nbins);
        else
            hipLaunchKernelGGL((sets_encode_persistent_kernel<19, kApplyLanes, 2>), dim3(enc_grid), dim3(kApplyLanes),
                               0, s, c.level2, c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups, p.rel_log2, out,
                               c.stot, (uint32_t)cap_words, p.nbins);
        bf_mark(mk, s, "sets_encode");
        return hipGetLastError();
    }
#define BF_SETS_ENCODE(RL, LN, LD)                                                                              \
    hipLaunchKernelGGL((sets_encode_kernel<RL, LN, LD>), dim3(p.nbins), dim3(LN), 0, s, c.level2, c.cb_base,    \
                       c.cb_start, c.tabs, p.max_chunks, p.ngroups, p.rel_log2, out, c.stot, (uint32_t)cap_words, \
                       sets_stop())
    if (p.region_log2 == 19) {
        if (loads == 8) BF_SETS_ENCODE(19, kApplyLanes, 8);
#ifdef BFHIP_AB_KNOBS
        else if (loads == 4) BF_SETS_ENCODE(19, kApplyLanes, 4);
        else if (loads == 1) BF_SETS_ENCODE(19, kApplyLanes, 1);
#endif
        else BF_SETS_ENCODE(19, kApplyLanes, 2);
    } else if (p.region_log2 == 18) {
        if (loads == 8) BF_SETS_ENCODE(18, kApplyLanes / 2, 8);
#ifdef BFHIP_AB_KNOBS
        else if (loads == 4) BF_SETS_ENCODE(18, kApplyLanes / 2, 4);
#endif
        else BF_SETS_ENCODE(18, kApplyLanes / 2, 2);
    } else {
        return hipErrorInvalidValue;
    }
#undef BF_SETS_ENCODE
    bf_mark(mk, s, "sets_encode");
    return hipGetLastError();
}

hipError_t bf_launch_insert_sets(const BfGeom& g, uint64_t bitset_bytes, uint32_t region_log2, uint32_t nbins,
                                 const uint32_t* sets, uint64_t stride_words, uint32_t nsrc, uint64_t probes_hint,
                                 uint32_t* any_flag, uint32_t* status, hipStream_t s, BfMarks* mk) {
    if (nsrc == 0) return hipSuccess;
    const uint64_t nwords = bitset_bytes / 4;
    const uint64_t vecs = (uint64_t)nbins << (region_log2 - 7);
    const uint32_t dense = probes_hint >= vecs ? 2u : (probes_hint >= vecs / 8 ? 1u : 0u);
    // low-bit stage: 1 (default) 15 KB at 2^19-bit regions (two workgroups per CU), 7.5 KB at
    // 2^18; 0: none (A/B; a 48-KB stage at one workgroup per CU measured 7.07 against 4.72 ms
    // at 10B, profiles/r04g_ab_sets_stage.jsonl)
    [[maybe_unused]] static const uint32_t stage = [] {
        const char* e = BF_AB_GETENV("BFHIP_SETS_STAGE");
        return e && *e ? (uint32_t)std::strtoul(e, nullptr, 10) : 1u;
    }();
    // regions per XCD group (apply_region, as bin_apply): 2 measured 4.061 / 4.021 ms against
    // 4.115 / 4.128 (1) at 10B x 8 (profiles/r05w_ab_sets_xg.jsonl).  BFHIP_SETS_XG (A/B) overrides.
    static const uint32_t sets_xg = [] {
        const char* e = BF_AB_GETENV("BFHIP_SETS_XG");
        return e && *e ? (uint32_t)std::strtoul(e, nullptr, 10) : 2u;
    }();
#ifdef BFHIP_AB_KNOBS
    // (A/B: BFHIP_SETS_PIPE=1 takes the persistent pipelined form for dense batches at 2^19-bit
    // regions with many regions per workgroup; measured slower, kept for the record)
    static const uint32_t pg = apply_pipe_grid();
    static const bool pipe_on = [] {
        const char* e = BF_AB_GETENV("BFHIP_SETS_PIPE");
        return e && e[0] == '1';
    }();
    const bool pipe = pipe_on && dense && region_log2 == 19 && pg && nbins >= 16 * pg;
#endif
    for (uint32_t s0 = 0; s0 < nsrc; s0 += kMaxSetSrc) {
        const uint32_t ns = std::min<uint32_t>(kMaxSetSrc, nsrc - s0);
        const uint32_t* src = sets + (uint64_t)s0 * stride_words;
#ifdef BFHIP_AB_KNOBS
        if (pipe) {
            hipLaunchKernelGGL((sets_apply_pipe_kernel<19, kPipeLanes, 2, 5>), dim3(std::min<uint32_t>(nbins, pg)),
                               dim3(kPipeLanes), 0, s, g.bits, nwords, src, stride_words, ns, nbins, dense, any_flag,
                               g.dirty, apply_store_fresh(), status);
            continue;
        }
#endif
#define BF_SETS_APPLY(RL, LN, ST)                                                                              \
    hipLaunchKernelGGL((sets_apply_kernel<RL, LN, ST>), dim3(nbins), dim3(LN), 0, s, g.bits, nwords, src,       \
                       stride_words, ns, nbins, dense, any_flag, g.dirty, apply_store_fresh(), status, sets_xg)
        if (region_log2 == 19) {
#ifdef BFHIP_AB_KNOBS
            if (stage == 0) BF_SETS_APPLY(19, kApplyLanes, 0);
            else
#endif
            BF_SETS_APPLY(19, kApplyLanes, kLowsStage);
        } else if (region_log2 == 18) {
#ifdef BFHIP_AB_KNOBS
            if (stage == 0) BF_SETS_APPLY(18, kApplyLanes / 2, 0);
            else
#endif
            BF_SETS_APPLY(18, kApplyLanes / 2, kLowsStage / 2);
        } else {
            return hipErrorInvalidValue;
        }
#undef BF_SETS_APPLY
    }
    bf_mark(mk, s, "sets_apply");
    return hipGetLastError();
}

hipError_t bf_launch_insert_encode_sets(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                        uint32_t region_log2, uint32_t nbins, const uint32_t* sets,
                                        uint64_t stride_words, uint32_t nsrc, uint64_t probes_hint, uint32_t* any_flag,
                                        uint32_t* status, const uint8_t* next_dig, uint64_t n_next, void* scratch,
                                        uint32_t* next_out, uint64_t cap_words, hipStream_t s, BfMarks* mk) {
    if (cap_words >= (1ull << 32)) return hipErrorInvalidValue;
    bool fuse = n_next && nsrc && nsrc <= kMaxSetSrc && !p.with_keys && p.region_log2 == region_log2 &&
                p.nbins == nbins && (region_log2 == 19 || region_log2 == 18);
#ifdef BFHIP_AB_KNOBS
    if (const char* v = BF_AB_GETENV("BFHIP_SETS_FUSE")) fuse = fuse && atoi(v) != 0;   // (A/B: 0 = two kernels)
#endif
    if (!fuse) {   // the next batch's encode (no bitset read), then the apply: the two calls in order
        hipError_t e = bf_launch_encode_sets(g, p, bitset_bytes, next_dig, nullptr, 0, n_next, true, scratch, next_out,
                                             cap_words, s, mk);
        if (e != hipSuccess) return e;
        return bf_launch_insert_sets(g, bitset_bytes, region_log2, nbins, sets, stride_words, nsrc, probes_hint, any_flag,
                                     status, s, mk);
    }
    const Carve c = carve(p, scratch);
    hipError_t e = launch_partition(g, p, c, next_dig, nullptr, 0, n_next, nullptr, s, mk, true);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sets_size_kernel, dim3(p.nsup), dim3(1024), 0, s, c.tabs, c.cb_base, p.max_chunks, p.ngroups,
                       p.rel_log2, p.nbins, 1u << p.region_log2, next_out, c.stot);
    hipLaunchKernelGGL(sets_place_kernel, dim3(1), dim3(1024), 0, s, next_out, c.stot, p.nsup, p.region_log2, p.nbins);
    const int loads = n_next * g.k <= (uint64_t)p.nbins * 4096u ? 2 : 8;   // as bf_launch_encode_sets
    const uint64_t nwords = bitset_bytes / 4;
    const uint64_t vecs = (uint64_t)nbins << (region_log2 - 7);
    const uint32_t dense = probes_hint >= vecs ? 2u : (probes_hint >= vecs / 8 ? 1u : 0u);
    const uint32_t xg = 2u;   // as bf_launch_insert_sets
#define BF_SETS_APPLY_ENCODE(RL, LN, ST, LD)                                                                     \
    hipLaunchKernelGGL((sets_apply_encode_kernel<RL, LN, ST, LD>), dim3(nbins), dim3(LN), 0, s, g.bits, nwords, sets, \
                       stride_words, nsrc, nbins, dense, any_flag, g.dirty, apply_store_fresh(), status, xg, c.level2,  \
                       c.cb_base, c.cb_start, c.tabs, p.max_chunks, p.ngroups, p.rel_log2, next_out, c.stot,           \
                       (uint32_t)cap_words)
    if (region_log2 == 19) {
        if (loads == 8) BF_SETS_APPLY_ENCODE(19, kApplyLanes, kLowsStage, 8);
        else BF_SETS_APPLY_ENCODE(19, kApplyLanes, kLowsStage, 2);
    } else {
        if (loads == 8) BF_SETS_APPLY_ENCODE(18, kApplyLanes / 2, kLowsStage / 2, 8);
        else BF_SETS_APPLY_ENCODE(18, kApplyLanes / 2, kLowsStage / 2, 2);
    }
#undef BF_SETS_APPLY_ENCODE
    bf_mark(mk, s, "sets_apply_encode");
    return hipGetLastError();
}
