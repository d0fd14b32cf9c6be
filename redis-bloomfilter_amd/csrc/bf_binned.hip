// bf_binned.hip — binned ("sweep") insert for filters far larger than L2.
//
// The direct insert (bf_kernels.hip) costs every probe a random 128-B DRAM
// line fill (test) and, for bits still 0, a memory-side atomic.  When a batch
// carries many probes per filter line that is far more traffic than streaming
// the filter once, so this path
//   1. bin_count:   hashes every key (ruby.rb:41-55 derivation, shared with the
//                   direct kernels), keeps its 4 digest words (16 B/key) and
//                   histograms its probes by 2^R-bit region in LDS (one
//                   histogram per workgroup, a fixed key range each);
//   2. bin_colscan / bin_scan: turns the [workgroup][region] counts into
//                   write cursors (region-major, workgroup-minor);
//   3. bin_scatter: re-derives the probes of the same key ranges from the
//                   digests and writes each probe's in-region offset (u32) to
//                   its region's bin;
//   4. bin_apply:   one workgroup per region ORs its bin into an LDS image of
//                   the region (LDS atomics), then read-OR-writes the region's
//                   touched 16-B vectors of the bitset — plain stores, since no
//                   other workgroup owns that region.
// Result: the same bitset as atomic OR (OR is idempotent and commutative).
#include "bf_device.h"

using namespace bfdev;

namespace {

constexpr int kTile = 1024;                   // keys per workgroup tile (16 waves: one workgroup per CU)
constexpr int kTileStageVec = 32768 / 16;     // 32 KiB LDS key stage
constexpr uint32_t kApply = 512;              // lanes per apply workgroup (2 per CU at 64 KiB of LDS)
constexpr uint32_t kMaxBins = 24576;          // LDS histogram / cursor capacity (96 KiB)

__global__ __launch_bounds__(kTile) void bin_count_kernel(BfGeom g, const uint8_t* __restrict__ keys16,
                                                          const uint64_t* __restrict__ offsets, uint64_t bias,
                                                          uint64_t n, uint64_t chunk, uint32_t region_log2,
                                                          uint32_t nbins, uint32_t* __restrict__ counts,
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
                digests[tile0 + lane] = make_uint4(H[0], H[1], H[2], H[3]);   // for the scatter pass
                for (uint32_t i = 0; i < g.k; ++i)
                    atomicAdd(s_hist + (uint32_t)(probe_offset(g, H[0], H[1], H[2], H[3], i) >> region_log2), 1u);
            });
    }
    uint32_t* row = counts + (uint64_t)blockIdx.x * nbins;
    for (uint32_t i = t; i < nbins; i += kTile) row[i] = s_hist[i];
}

// counts[b][r] -> exclusive prefix over b (per region r); totals[r] = column sum.
__global__ __launch_bounds__(256) void bin_colscan_kernel(uint32_t* __restrict__ counts, uint32_t nblocks,
                                                          uint32_t nbins, uint32_t* __restrict__ totals) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;
    if (r >= nbins) return;
    uint32_t run = 0;
    uint32_t b = 0;
    for (; b + 8 <= nblocks; b += 8) {       // 8 independent loads in flight
        uint32_t c[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = counts[(uint64_t)(b + j) * nbins + r];
#pragma unroll
        for (int j = 0; j < 8; ++j) { counts[(uint64_t)(b + j) * nbins + r] = run; run += c[j]; }
    }
    for (; b < nblocks; ++b) {
        const uint32_t c = counts[(uint64_t)b * nbins + r];
        counts[(uint64_t)b * nbins + r] = run;
        run += c;
    }
    totals[r] = run;
}

// bases[r] = exclusive prefix of totals, bases[nbins] = total probes.  One workgroup.
__global__ __launch_bounds__(1024) void bin_scan_kernel(const uint32_t* __restrict__ totals, uint32_t nbins,
                                                        uint32_t* __restrict__ bases) {
    __shared__ uint32_t s_part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nbins + 1023) / 1024;
    const uint32_t b0 = t * per;
    uint32_t sum = 0;
    for (uint32_t i = 0; i < per; ++i)
        if (b0 + i < nbins) sum += totals[b0 + i];
    s_part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {   // Hillis-Steele inclusive scan
        const uint32_t v = t >= off ? s_part[t - off] : 0u;
        __syncthreads();
        s_part[t] += v;
        __syncthreads();
    }
    uint32_t run = s_part[t] - sum;
    for (uint32_t i = 0; i < per; ++i)
        if (b0 + i < nbins) { bases[b0 + i] = run; run += totals[b0 + i]; }
    if (t == 1023) bases[nbins] = s_part[1023];
}

// Reads the digests the count pass stored (no re-hash); per key, all of a
// chunk's LDS cursor atomics issue before its stores.
__global__ __launch_bounds__(kTile) void bin_scatter_kernel(BfGeom g, const uint4* __restrict__ digests,
                                                            uint64_t n, uint64_t chunk, uint32_t region_log2,
                                                            uint32_t nbins, const uint32_t* __restrict__ counts,
                                                            const uint32_t* __restrict__ bases,
                                                            uint32_t* __restrict__ binned) {
    __shared__ uint32_t s_cur[kMaxBins];
    const uint32_t t = threadIdx.x;
    const uint32_t* row = counts + (uint64_t)blockIdx.x * nbins;
    for (uint32_t i = t; i < nbins; i += kTile) s_cur[i] = bases[i] + row[i];
    __syncthreads();
    const uint64_t k0 = (uint64_t)blockIdx.x * chunk;
    const uint64_t k1 = (k0 + chunk < n) ? k0 + chunk : n;
    const uint64_t rmask = (1ull << region_log2) - 1ull;
    for (uint64_t key = k0 + t; key < k1; key += kTile) {
        const uint4 H = digests[key];
        for (uint32_t i0 = 0; i0 < g.k; i0 += kChunk) {
            uint32_t pos[kChunk], loc[kChunk];
#pragma unroll
            for (int c = 0; c < kChunk; ++c) {
                if (i0 + c < g.k) {
                    const uint64_t o = probe_offset(g, H.x, H.y, H.z, H.w, i0 + c);
                    loc[c] = (uint32_t)(o & rmask);
                    pos[c] = atomicAdd(s_cur + (uint32_t)(o >> region_log2), 1u);
                }
            }
#pragma unroll
            for (int c = 0; c < kChunk; ++c)
                if (i0 + c < g.k) binned[pos[c]] = loc[c];
        }
    }
}

template <uint32_t RLOG2>
__global__ __launch_bounds__(kApply) void bin_apply_kernel(uint32_t* __restrict__ bits, uint64_t nwords,
                                                           const uint32_t* __restrict__ binned,
                                                           const uint32_t* __restrict__ bases,
                                                           uint32_t* __restrict__ any_flag) {
    constexpr uint32_t kWords = 1u << (RLOG2 - 5);
    __shared__ uint4 s_mask4[kWords / 4];
    uint32_t* s_mask = reinterpret_cast<uint32_t*>(s_mask4);
    const uint32_t t = threadIdx.x;
    const uint32_t r = blockIdx.x;
    for (uint32_t v = t; v < kWords / 4; v += kApply) s_mask4[v] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const uint32_t p1 = bases[r + 1];
    for (uint32_t p = bases[r] + t; p < p1; p += kApply) {
        const uint32_t l = binned[p];
        atomicOr(s_mask + (l >> 5), 1u << ((l ^ 7u) & 31u));
    }
    __syncthreads();
    const uint64_t w0 = (uint64_t)r * kWords;
    uint4* gv = reinterpret_cast<uint4*>(bits);
    uint32_t fresh = 0;
    for (uint32_t v = t; v < kWords / 4; v += kApply) {
        const uint64_t gw = w0 + 4ull * v;
        if (gw >= nwords) break;
        const uint4 msk = s_mask4[v];
        if (msk.x | msk.y | msk.z | msk.w) {
            uint4 old = gv[gw >> 2];
            fresh |= (msk.x & ~old.x) | (msk.y & ~old.y) | (msk.z & ~old.z) | (msk.w & ~old.w);
            old.x |= msk.x; old.y |= msk.y; old.z |= msk.z; old.w |= msk.w;
            gv[gw >> 2] = old;
        }
    }
    if (any_flag) {
        const unsigned long long b = __ballot(fresh != 0);
        if (b != 0ull && (t & 63u) == (uint32_t)__builtin_ctzll(b))
            __hip_atomic_fetch_or(any_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace

bool bf_binned_plan(uint64_t bitset_bytes, uint64_t n, uint32_t k, BfBinPlan* plan) {
    const uint64_t bits = bitset_bytes * 8;
    for (uint32_t rl : {19u, 20u}) {
        const uint64_t nbins = (bits + (1ull << rl) - 1) >> rl;
        if (nbins <= kMaxBins) {
            plan->region_log2 = rl;
            plan->nbins = (uint32_t)nbins;
            const uint64_t per_block = 2ull * kTile * 16;   // >= 16 tiles per workgroup
            uint64_t blocks = (n + per_block - 1) / per_block;
            if (blocks > 256) blocks = 256;                 // one per CU (132 KiB of LDS each)
            if (blocks == 0) blocks = 1;
            plan->nblocks = (uint32_t)blocks;
            plan->chunk = ((n + blocks - 1) / blocks + kTile - 1) / kTile * kTile;
            plan->probes = n * k;
            return plan->probes < (1ull << 32);
        }
    }
    return false;
}

hipError_t bf_launch_insert_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                   const uint8_t* keys16, const uint64_t* offsets, uint64_t bias, uint64_t n,
                                   uint32_t* counts, uint32_t* totals, uint32_t* bases, uint32_t* binned,
                                   void* digests, uint32_t* any_flag, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint4* dg = static_cast<uint4*>(digests);
    hipLaunchKernelGGL(bin_count_kernel, dim3(p.nblocks), dim3(kTile), 0, s, g, keys16, offsets, bias, n, p.chunk,
                       p.region_log2, p.nbins, counts, dg);
    hipLaunchKernelGGL(bin_colscan_kernel, dim3((p.nbins + 255) / 256), dim3(256), 0, s, counts, p.nblocks, p.nbins,
                       totals);
    hipLaunchKernelGGL(bin_scan_kernel, dim3(1), dim3(1024), 0, s, totals, p.nbins, bases);
    hipLaunchKernelGGL(bin_scatter_kernel, dim3(p.nblocks), dim3(kTile), 0, s, g, dg, n, p.chunk,
                       p.region_log2, p.nbins, counts, bases, binned);
    const uint64_t nwords = bitset_bytes / 4;
    if (p.region_log2 == 19)
        hipLaunchKernelGGL(bin_apply_kernel<19>, dim3(p.nbins), dim3(kApply), 0, s, g.bits, nwords, binned, bases, any_flag);
    else
        hipLaunchKernelGGL(bin_apply_kernel<20>, dim3(p.nbins), dim3(kApply), 0, s, g.bits, nwords, binned, bases, any_flag);
    return hipGetLastError();
}
