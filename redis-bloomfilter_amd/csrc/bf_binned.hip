// bf_binned.hip — binned ("sweep") insert for filters far larger than L2.
//
// The direct insert (bf_kernels.hip) costs every probe a random 128-B DRAM
// line fill (test) and, for bits still 0, a memory-side atomic.  When a batch
// carries many probes per filter line that is far more traffic than streaming
// the filter once.  This path sorts the batch's probes by filter region with
// two LDS-sorted partition passes whose global writes are coalesced runs, then
// ORs each region in LDS and streams it once:
//
//   1. bin_count    hashes every key (ruby.rb:41-55 derivation, shared with the
//                   direct kernels), stores its 4 digest words (16 B/key) and
//                   histograms its probes by 2^rl-bit region in LDS.  Workgroup
//                   w owns a fixed key range; it writes its region counts and
//                   its superbin counts (superbin = 2^rel consecutive regions).
//   2. bin_colsum   region totals (column sums over the workgroups);
//      bin_supscan  per superbin, the exclusive prefix over workgroups (each
//                   workgroup's exact write window inside the superbin);
//      bin_scan     region bases (exclusive prefix of the totals) + cursors.
//   3. bin_part1    re-derives the probes from the digests, tile by tile; per
//                   tile an LDS counting sort by superbin, then each superbin's
//                   run is written contiguously (level-1 array, superbin-local
//                   u32 offsets).
//   4. bin_part2    per 8192-probe chunk of the level-1 array: LDS counting sort
//                   by region, one returning atomic per (chunk, region) reserves
//                   the run, coalesced writes (level-2 array, region-local u32).
//   5. bin_apply    one workgroup per region ORs its probes into an LDS image of
//                   the region (LDS atomics), then read-OR-writes the region's
//                   touched 16-B vectors of the bitset — plain stores, since no
//                   other workgroup owns that region.
// Result: the same bitset as atomic OR (OR is idempotent and commutative).
#include "bf_device.h"

using namespace bfdev;

namespace {

constexpr int kTile = 1024;                   // lanes of the count / partition workgroups
constexpr int kTileStageVec = 32768 / 16;     // 32 KiB LDS key stage (count pass)
constexpr uint32_t kMaxBins = 24576;          // region histogram capacity (96 KiB)
constexpr uint32_t kMaxSup = 256;             // superbins (u8 tags in part1)
constexpr uint32_t kMaxBlocks = 512;          // count / part1 workgroups (two per CU)
constexpr uint32_t kP1Probes = 12288;         // probes per part1 tile (64 KiB of LDS: two workgroups per CU)
constexpr int kP1Slots = 12;                  // probes per lane per part1 tile (k <= 12)
constexpr uint32_t kP1TwoKeys = 6;            // k <= 6: two keys per lane per tile
constexpr uint32_t kP2Probes = 8192;          // probes per part2 workgroup
constexpr int kP2PerLane = kP2Probes / kTile;
constexpr uint32_t kP2Bins = 512;             // local region bins per part2 workgroup (52 KiB: three per CU)
constexpr uint32_t kApplyLanes = 1024;

// Exclusive prefix sum of v over the workgroup (blockDim.x a multiple of 64,
// at most 1024 lanes); *total gets the workgroup sum.  s_w: 16 words of LDS.
// Contains barriers: every lane must call it.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= (uint32_t)off) x += y;
    }
    if (lane == 63u) s_w[wid] = x;
    __syncthreads();
    if (wid == 0) {
        uint32_t s = lane < nw ? s_w[lane] : 0u;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const uint32_t y = __shfl_up(s, off);
            if (lane >= (uint32_t)off) s += y;
        }
        if (lane < nw) s_w[lane] = s;   // inclusive wave totals
    }
    __syncthreads();
    const uint32_t r = (wid ? s_w[wid - 1] : 0u) + x - v;
    if (total) *total = s_w[nw - 1];
    __syncthreads();   // s_w may be reused right after
    return r;
}

__global__ __launch_bounds__(kTile) void bin_count_kernel(BfGeom g, const uint8_t* __restrict__ keys16,
                                                          const uint64_t* __restrict__ offsets, uint64_t bias,
                                                          uint64_t n, uint64_t chunk, uint32_t region_log2,
                                                          uint32_t nbins, uint32_t rel_log2, uint32_t nsup,
                                                          uint32_t* __restrict__ counts, uint32_t* __restrict__ scnt,
                                                          uint4* __restrict__ digests) {
    __shared__ uint32_t s_hist[kMaxBins];
    __shared__ uint64_t s_off[kTile + 1];
    __shared__ uint4 s_stage[kTileStageVec + kStageSlackVec];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < nbins; i += kTile) s_hist[i] = 0;
    __syncthreads();
    const uint64_t k0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t k1 = (k0 + chunk < n) ? k0 + chunk : n;
    for (uint64_t tile0 = k0; tile0 < k1; tile0 += kTile) {
        const uint32_t cnt = (uint32_t)((k1 - tile0) < (uint64_t)kTile ? (k1 - tile0) : kTile);
        for_key_tile<kTile, kTileStageVec>(keys16, offsets, bias, tile0, cnt, s_off, s_stage,
            [&](auto staged, uint32_t lane, const uint32_t* src, uint32_t s, uint32_t L) {
                uint32_t H[5];
                sha1_any<decltype(staged)::value>(src, s, L, H);
                digests[tile0 + lane] = make_uint4(H[0], H[1], H[2], H[3]);   // for the partition pass
                for (uint32_t i = 0; i < g.k; ++i)
                    atomicAdd(s_hist + (uint32_t)(probe_offset(g, H[0], H[1], H[2], H[3], i) >> region_log2), 1u);
            });
    }
    uint32_t* row = counts + (uint64_t)blockIdx.x * nbins;
    for (uint32_t i = t; i < nbins; i += kTile) row[i] = s_hist[i];
    for (uint32_t sb = t; sb < nsup; sb += kTile) {
        const uint32_t r0 = sb << rel_log2;
        const uint32_t r1 = (r0 + (1u << rel_log2) < nbins) ? r0 + (1u << rel_log2) : nbins;
        uint32_t sum = 0;
        for (uint32_t r = r0; r < r1; ++r) sum += s_hist[r];
        scnt[(uint64_t)blockIdx.x * nsup + sb] = sum;
    }
}

// totals[r] = sum over workgroups b of counts[b][r].  64 regions x 16 row groups per workgroup.
__global__ __launch_bounds__(1024) void bin_colsum_kernel(const uint32_t* __restrict__ counts, uint32_t nblocks,
                                                          uint32_t nbins, uint32_t* __restrict__ totals) {
    __shared__ uint32_t s_part[16][64];
    const uint32_t x = threadIdx.x & 63u, y = threadIdx.x >> 6;
    const uint32_t r = blockIdx.x * 64 + x;
    uint32_t sum = 0;
    if (r < nbins) {
#pragma unroll 8
        for (uint32_t b = y; b < nblocks; b += 16) sum += counts[(uint64_t)b * nbins + r];
    }
    s_part[y][x] = sum;
    __syncthreads();
    if (y == 0 && r < nbins) {
        uint32_t tot = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) tot += s_part[j][x];
        totals[r] = tot;
    }
}

// scnt[b][sb] -> exclusive prefix over b, in place.  One workgroup (kMaxBlocks lanes) per superbin.
__global__ __launch_bounds__(kMaxBlocks) void bin_supscan_kernel(uint32_t* __restrict__ scnt, uint32_t nblocks,
                                                          uint32_t nsup) {
    __shared__ uint32_t s_w[16];
    const uint32_t t = threadIdx.x, sb = blockIdx.x;
    const uint32_t v = t < nblocks ? scnt[(uint64_t)t * nsup + sb] : 0u;
    const uint32_t ex = block_excl_scan(v, s_w, nullptr);
    if (t < nblocks) scnt[(uint64_t)t * nsup + sb] = ex;
}

// bases[r] = exclusive prefix of totals, bases[nbins] = total probes, cursor[r] = bases[r].
// One workgroup; the totals pass through LDS so every global access is coalesced.
__global__ __launch_bounds__(1024) void bin_scan_kernel(const uint32_t* __restrict__ totals, uint32_t nbins,
                                                        uint32_t* __restrict__ bases, uint32_t* __restrict__ cursor) {
    __shared__ uint32_t s_v[kMaxBins];
    __shared__ uint32_t s_w[16];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < nbins; i += 1024) s_v[i] = totals[i];
    __syncthreads();
    const uint32_t per = (nbins + 1023) / 1024;
    const uint32_t b0 = t * per;
    uint32_t sum = 0;
    for (uint32_t i = 0; i < per; ++i)
        if (b0 + i < nbins) sum += s_v[b0 + i];
    uint32_t total;
    uint32_t run = block_excl_scan(sum, s_w, &total);
    for (uint32_t i = 0; i < per; ++i)
        if (b0 + i < nbins) { const uint32_t c = s_v[b0 + i]; s_v[b0 + i] = run; run += c; }
    __syncthreads();
    for (uint32_t i = t; i < nbins; i += 1024) { bases[i] = s_v[i]; cursor[i] = s_v[i]; }
    if (t == 0) bases[nbins] = total;
}

// Level 1: probes grouped by superbin.  Workgroup w walks the key range of the
// count pass's workgroup w; its run inside superbin sb starts at
// bases[sb << rel] + scnt[w][sb] and grows tile by tile.
__global__ __launch_bounds__(kTile) void bin_part1_kernel(BfGeom g, const uint4* __restrict__ digests, uint64_t n,
                                                          uint64_t chunk, uint32_t sup_log2, uint32_t rel_log2,
                                                          uint32_t nsup, uint32_t nbins,
                                                          const uint32_t* __restrict__ scnt,
                                                          const uint32_t* __restrict__ bases,
                                                          uint32_t* __restrict__ level1) {
    __shared__ uint32_t s_cur[kMaxSup], s_cnt[kMaxSup], s_lbase[kMaxSup], s_gdst[kMaxSup];
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_sorted[kP1Probes];
    __shared__ uint8_t s_sb[kP1Probes];
    const uint32_t t = threadIdx.x;
    if (t < nsup) {
        const uint32_t r = t << rel_log2;
        s_cur[t] = bases[r < nbins ? r : nbins] + scnt[(uint64_t)blockIdx.x * nsup + t];
    }
    if (t < kMaxSup) s_cnt[t] = 0;
    __syncthreads();
    const uint32_t k = g.k;
    const uint32_t kpl = k <= kP1TwoKeys ? 2u : 1u;   // keys per lane per tile
    const uint32_t tile_keys = kTile * kpl;
    const uint64_t smask = (1ull << sup_log2) - 1ull;
    const uint64_t k0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t k1 = (k0 + chunk < n) ? k0 + chunk : n;
    // digests of the next tile are loaded while the current one is sorted and written
    uint4 N0 = make_uint4(0, 0, 0, 0), N1 = make_uint4(0, 0, 0, 0);
    if (k0 + t < k1) N0 = digests[k0 + t];
    if (kpl == 2 && k0 + kTile + t < k1) N1 = digests[k0 + kTile + t];
    for (uint64_t tile0 = k0; tile0 < k1; tile0 += tile_keys) {
        const uint32_t tk = (uint32_t)((k1 - tile0) < (uint64_t)tile_keys ? (k1 - tile0) : tile_keys);
        // A: probes of this lane's keys -> (superbin, rank in the tile's superbin run)
        const bool live0 = t < tk;
        const bool live1 = kpl == 2 && kTile + t < tk;
        const uint4 H0 = N0, H1 = N1;
        uint32_t tag[kP1Slots], loc[kP1Slots];
#pragma unroll
        for (int q = 0; q < kP1Slots; ++q) {
            const bool second = kpl == 2 && q >= (int)kP1TwoKeys;
            const uint32_t i = kpl == 2 ? (second ? (uint32_t)q - kP1TwoKeys : (uint32_t)q) : (uint32_t)q;
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
        const uint64_t nx = tile0 + tile_keys;
        if (nx + t < k1) N0 = digests[nx + t];
        if (kpl == 2 && nx + kTile + t < k1) N1 = digests[nx + kTile + t];
        // B: tile-local run bases, global run bases; cursors advance past this tile
        const uint32_t c = t < kMaxSup ? s_cnt[t] : 0u;
        const uint32_t ex = block_excl_scan(c, s_w, nullptr);
        if (t < kMaxSup) {
            s_lbase[t] = ex;
            if (c) { s_gdst[t] = s_cur[t]; s_cur[t] += c; }
            s_cnt[t] = 0;
        }
        __syncthreads();
        // C: counting-sort the tile in LDS
#pragma unroll
        for (int q = 0; q < kP1Slots; ++q) {
            if (tag[q] != 0xFFFFFFFFu) {
                const uint32_t sb = tag[q] >> 16;
                const uint32_t d = s_lbase[sb] + (tag[q] & 0xFFFFu);
                s_sorted[d] = loc[q];
                s_sb[d] = (uint8_t)sb;
            }
        }
        __syncthreads();
        // D: consecutive lanes write consecutive slots of each superbin run
        const uint32_t tp = tk * k;
        for (uint32_t j = t; j < tp; j += kTile) {
            const uint32_t sb = s_sb[j];
            level1[s_gdst[sb] + (j - s_lbase[sb])] = s_sorted[j];
        }
    }
}

// Level 2: one chunk of the level-1 array, grouped by region.  The chunk's
// superbins are found from the superbin bases; each (chunk, region) run is
// reserved with one atomic on the region's cursor.
__global__ __launch_bounds__(kTile) void bin_part2_kernel(const uint32_t* __restrict__ level1, uint32_t P,
                                                          const uint32_t* __restrict__ bases, uint32_t nbins,
                                                          uint32_t nsup, uint32_t region_log2, uint32_t rel_log2,
                                                          uint32_t* __restrict__ cursor,
                                                          uint32_t* __restrict__ level2) {
    __shared__ uint32_t s_sbb[kMaxSup + 1];
    __shared__ uint32_t s_cnt[kP2Bins], s_gdst[kP2Bins];   // s_cnt becomes the local run bases
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_first, s_last;
    __shared__ uint32_t s_sorted[kP2Probes];
    __shared__ uint16_t s_lr[kP2Probes];
    const uint32_t t = threadIdx.x;
    const uint32_t p0 = blockIdx.x * kP2Probes;
    const uint32_t p1 = (P - p0 < kP2Probes) ? P : p0 + kP2Probes;
    if (t <= nsup) {
        const uint32_t r = t << rel_log2;
        s_sbb[t] = bases[r < nbins ? r : nbins];
    }
    if (t < kP2Bins) s_cnt[t] = 0;
    __syncthreads();
    if (t < 2) {   // superbin of p0 (lane 0) / of p1 - 1 (lane 1): last sb with s_sbb[sb] <= p
        const uint32_t p = t ? p1 - 1 : p0;
        uint32_t lo = 0, hi = nsup - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (s_sbb[mid] <= p) lo = mid; else hi = mid - 1;
        }
        if (t) s_last = lo; else s_first = lo;
    }
    __syncthreads();
    const uint32_t sb_first = s_first, sb_last = s_last;
    const uint32_t rfirst = sb_first << rel_log2;
    const uint32_t range = (sb_last - sb_first + 1) << rel_log2;
    const uint32_t rmask = (1u << region_log2) - 1u;
    uint32_t loc[kP2PerLane];
#pragma unroll
    for (int c = 0; c < kP2PerLane; ++c) {
        const uint32_t p = p0 + c * kTile + t;
        loc[c] = p < p1 ? level1[p] : 0u;
    }
    if (range > kP2Bins) {   // workgroup-uniform: many sparse superbins in one chunk
#pragma unroll
        for (int c = 0; c < kP2PerLane; ++c) {
            const uint32_t p = p0 + c * kTile + t;
            if (p < p1) {
                uint32_t sb = sb_first;
                while (p >= s_sbb[sb + 1]) ++sb;
                const uint32_t r = (sb << rel_log2) + (loc[c] >> region_log2);
                level2[atomicAdd(cursor + r, 1u)] = loc[c] & rmask;
            }
        }
        return;
    }
    uint32_t tag[kP2PerLane];
#pragma unroll
    for (int c = 0; c < kP2PerLane; ++c) {
        const uint32_t p = p0 + c * kTile + t;
        tag[c] = 0xFFFFFFFFu;
        if (p < p1) {
            uint32_t sb = sb_first;
            while (p >= s_sbb[sb + 1]) ++sb;
            const uint32_t lr = ((sb - sb_first) << rel_log2) + (loc[c] >> region_log2);
            tag[c] = (lr << 16) | atomicAdd(s_cnt + lr, 1u);
        }
    }
    __syncthreads();
    const uint32_t cnt = t < range ? s_cnt[t] : 0u;
    const uint32_t ex = block_excl_scan(cnt, s_w, nullptr);   // its barriers order the s_cnt reads first
    if (t < kP2Bins) s_cnt[t] = ex;
    if (cnt) s_gdst[t] = atomicAdd(cursor + rfirst + t, cnt);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kP2PerLane; ++c) {
        if (tag[c] != 0xFFFFFFFFu) {
            const uint32_t lr = tag[c] >> 16;
            const uint32_t d = s_cnt[lr] + (tag[c] & 0xFFFFu);
            s_sorted[d] = loc[c] & rmask;
            s_lr[d] = (uint16_t)lr;
        }
    }
    __syncthreads();
    for (uint32_t j = t; j < p1 - p0; j += kTile) {
        const uint32_t lr = s_lr[j];
        level2[s_gdst[lr] + (j - s_cnt[lr])] = s_sorted[j];
    }
}

template <uint32_t RLOG2, uint32_t LANES>
__global__ __launch_bounds__(LANES) void bin_apply_kernel(uint32_t* __restrict__ bits, uint64_t nwords,
                                                          const uint32_t* __restrict__ binned,
                                                          const uint32_t* __restrict__ bases,
                                                          uint32_t* __restrict__ any_flag) {
    constexpr uint32_t kVec = 1u << (RLOG2 - 7);   // 16-B vectors per region
    constexpr uint32_t kPer = kVec / LANES;
    constexpr int kLoads = 8;
    static_assert(kPer * LANES == kVec, "region must tile the workgroup");
    __shared__ uint4 s_mask4[kVec];
    uint32_t* s_mask = reinterpret_cast<uint32_t*>(s_mask4);
    const uint32_t t = threadIdx.x;
    const uint32_t r = blockIdx.x;
    const uint64_t v0 = (uint64_t)r * kVec;
    const uint64_t nvec = nwords / 4;
    uint4* gv = reinterpret_cast<uint4*>(bits);
    const uint32_t pb = bases[r], p1 = bases[r + 1];
    // Dense region (at least one probe per 16-B vector on average; most vectors are
    // touched): its bitset vectors are loaded first, so that read overlaps the probe
    // pass.  Sparse region: only the touched vectors are read, after the probe pass.
    const bool dense = p1 - pb >= kVec;   // workgroup-uniform
    uint4 old[kPer];
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {
        const uint32_t v = c * LANES + t;
        old[c] = make_uint4(0, 0, 0, 0);
        if (dense && v0 + v < nvec) old[c] = gv[v0 + v];
    }
    for (uint32_t v = t; v < kVec; v += LANES) s_mask4[v] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    for (uint32_t p = pb + t; p < p1; p += kLoads * LANES) {   // kLoads loads in flight per lane
        uint32_t l[kLoads];
#pragma unroll
        for (int c = 0; c < kLoads; ++c) l[c] = (p + c * LANES < p1) ? binned[p + c * LANES] : 0xFFFFFFFFu;
#pragma unroll
        for (int c = 0; c < kLoads; ++c)
            if (l[c] != 0xFFFFFFFFu) atomicOr(s_mask + (l[c] >> 5), 1u << ((l[c] ^ 7u) & 31u));
    }
    __syncthreads();
    uint4 msk[kPer];
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {   // sparse: every touched vector's load issues before any store
        const uint32_t v = c * LANES + t;
        msk[c] = s_mask4[v];
        if (!dense && v0 + v < nvec && (msk[c].x | msk[c].y | msk[c].z | msk[c].w)) old[c] = gv[v0 + v];
    }
    uint32_t fresh = 0;
#pragma unroll
    for (uint32_t c = 0; c < kPer; ++c) {
        const uint32_t v = c * LANES + t;
        if (v0 + v < nvec && (msk[c].x | msk[c].y | msk[c].z | msk[c].w)) {
            fresh |= (msk[c].x & ~old[c].x) | (msk[c].y & ~old[c].y) | (msk[c].z & ~old[c].z) | (msk[c].w & ~old[c].w);
            gv[v0 + v] = make_uint4(old[c].x | msk[c].x, old[c].y | msk[c].y, old[c].z | msk[c].z, old[c].w | msk[c].w);
        }
    }
    if (any_flag) {
        const unsigned long long b = __ballot(fresh != 0);
        if (b != 0ull && (t & 63u) == (uint32_t)__builtin_ctzll(b))
            __hip_atomic_fetch_or(any_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

uint64_t align256(uint64_t x) { return (x + 255) & ~(uint64_t)255; }

struct Carve {
    uint32_t *counts, *scnt, *totals, *bases, *cursor, *level1, *level2;
    uint4* digests;
    uint64_t bytes;
};

Carve carve(const BfBinPlan& p, uint64_t n, void* base) {
    Carve c{};
    uint8_t* at = static_cast<uint8_t*>(base);
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) { uint8_t* q = at ? at + off : nullptr; off += align256(bytes); return q; };
    c.digests = reinterpret_cast<uint4*>(take(n * 16));
    c.level1 = reinterpret_cast<uint32_t*>(take(p.probes * 4));
    c.level2 = reinterpret_cast<uint32_t*>(take(p.probes * 4));
    c.counts = reinterpret_cast<uint32_t*>(take((uint64_t)p.nblocks * p.nbins * 4));
    c.scnt = reinterpret_cast<uint32_t*>(take((uint64_t)p.nblocks * p.nsup * 4));
    c.totals = reinterpret_cast<uint32_t*>(take((uint64_t)p.nbins * 4));
    c.bases = reinterpret_cast<uint32_t*>(take((uint64_t)(p.nbins + 1) * 4));
    c.cursor = reinterpret_cast<uint32_t*>(take((uint64_t)p.nbins * 4));
    c.bytes = off;
    return c;
}

}  // namespace

bool bf_binned_plan(uint64_t bitset_bytes, uint64_t n, uint32_t k, uint32_t pref_region_log2, BfBinPlan* plan) {
    if (k == 0 || k > (uint32_t)kP1Slots || n == 0) return false;   // k > 12: the direct insert
    const uint64_t bits = bitset_bytes * 8;
    const uint32_t order[2] = {pref_region_log2 == 20 ? 20u : 19u, pref_region_log2 == 20 ? 19u : 20u};
    for (uint32_t rl : order) {
        const uint64_t nbins = (bits + (1ull << rl) - 1) >> rl;
        if (nbins > kMaxBins) continue;
        uint32_t rel = 0;
        while (((nbins + (1ull << rel) - 1) >> rel) > kMaxSup) ++rel;
        plan->region_log2 = rl;
        plan->nbins = (uint32_t)nbins;
        plan->rel_log2 = rel;
        plan->nsup = (uint32_t)((nbins + (1ull << rel) - 1) >> rel);
        const uint64_t per_block = 2ull * kTile * 16;   // >= 16 tiles per workgroup
        uint64_t blocks = (n + per_block - 1) / per_block;
        if (blocks > kMaxBlocks) blocks = kMaxBlocks;
        if (blocks == 0) blocks = 1;
        plan->nblocks = (uint32_t)blocks;
        plan->chunk = ((n + blocks - 1) / blocks + kTile - 1) / kTile * kTile;
        plan->probes = n * k;
        if (plan->probes >= (1ull << 32)) return false;
        plan->scratch_bytes = carve(*plan, n, nullptr).bytes;
        return true;
    }
    return false;
}

hipError_t bf_launch_insert_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                   const uint8_t* keys16, const uint64_t* offsets, uint64_t bias, uint64_t n,
                                   void* scratch, uint32_t* any_flag, hipStream_t s, BfMarks* mk) {
    if (n == 0) return hipSuccess;
    const Carve c = carve(p, n, scratch);
    const uint32_t P = (uint32_t)p.probes;
    hipLaunchKernelGGL(bin_count_kernel, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, bias, n, p.chunk,
                       p.region_log2, p.nbins, p.rel_log2, p.nsup, c.counts, c.scnt, c.digests);
    bf_mark(mk, s, "bin_count");
    hipLaunchKernelGGL(bin_colsum_kernel, dim3((p.nbins + 63) / 64), dim3(1024), 0, s, c.counts, p.nblocks, p.nbins,
                       c.totals);
    bf_mark(mk, s, "bin_colsum");
    hipLaunchKernelGGL(bin_supscan_kernel, dim3(p.nsup), dim3(kMaxBlocks), 0, s, c.scnt, p.nblocks, p.nsup);
    bf_mark(mk, s, "bin_supscan");
    hipLaunchKernelGGL(bin_scan_kernel, dim3(1), dim3(1024), 0, s, c.totals, p.nbins, c.bases, c.cursor);
    bf_mark(mk, s, "bin_scan");
    hipLaunchKernelGGL(bin_part1_kernel, dim3(p.nblocks), dim3(kTile), 0, s, g, c.digests, n, p.chunk,
                       p.region_log2 + p.rel_log2, p.rel_log2, p.nsup, p.nbins, c.scnt, c.bases, c.level1);
    bf_mark(mk, s, "bin_part1");
    hipLaunchKernelGGL(bin_part2_kernel, dim3((P + kP2Probes - 1) / kP2Probes), dim3(kTile), 0, s, c.level1, P,
                       c.bases, p.nbins, p.nsup, p.region_log2, p.rel_log2, c.cursor, c.level2);
    bf_mark(mk, s, "bin_part2");
    const uint64_t nwords = bitset_bytes / 4;
    if (p.region_log2 == 19)
        hipLaunchKernelGGL((bin_apply_kernel<19, kApplyLanes>), dim3(p.nbins), dim3(kApplyLanes), 0, s, g.bits,
                           nwords, c.level2, c.bases, any_flag);
    else
        hipLaunchKernelGGL((bin_apply_kernel<20, kApplyLanes>), dim3(p.nbins), dim3(kApplyLanes), 0, s, g.bits,
                           nwords, c.level2, c.bases, any_flag);
    bf_mark(mk, s, "bin_apply");
    return hipGetLastError();
}
