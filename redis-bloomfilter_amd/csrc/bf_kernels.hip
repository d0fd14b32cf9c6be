// bf_kernels.hip — CDNA4 (gfx950) kernels for the Bloom-filter hot path.
//
// One lane per key.  A 256-lane workgroup owns 256 consecutive keys:
//   1. the 257 offsets are read coalesced into LDS;
//   2. the workgroup's packed key bytes [off[0], off[256]) are staged into LDS
//      with 16-byte coalesced loads (fallback: per-lane global reads when the
//      span exceeds the 16 KiB stage);
//   3. each lane builds its big-endian SHA-1 message words from LDS with
//      v_alignbyte + v_perm (byte swap) and runs the 80-round compression
//      (single block for keys <= 55 bytes, the generic multi-block loop otherwise);
//   4. the k offsets follow ruby.rb:41-55 exactly:
//        idx_i = (h[i%2] + i*h[2 + (((i + i%2) % 4) / 2)]) mod m
//      with the modulo done by a double-precision reciprocal + one correction
//      (no integer divide on the GPU), skipped entirely when m > k*(2^32-1);
//   5. the op: gather k words and AND (include?), atomic-OR k words (insert),
//      or store the offsets (indexes_for).
//
// Bit o of the filter is bit ((o ^ 7) & 31) of little-endian word o >> 5, i.e.
// byte o >> 3 under mask 0x80 >> (o & 7) — the Redis SETBIT layout, so the
// device buffer IS the Redis string.
#include "bf_device.h"

namespace {

using namespace bfdev;

template <int OP, typename Side>
__device__ __forceinline__ void digest_op(const BfGeom& g, const uint32_t H[4], uint64_t key,
                                          uint8_t* __restrict__ out8, uint64_t* __restrict__ out64,
                                          uint32_t& newflag, uint32_t* hist, Side&& side) {
    const uint32_t k = g.k;
    if constexpr (OP == BF_OP_HASH) {
        reinterpret_cast<uint4*>(out64)[key] = make_uint4(H[0], H[1], H[2], H[3]);
    } else if constexpr (OP == BF_OP_INDEXES) {
        for (uint32_t i = 0; i < k; ++i)
            out64[key * k + i] = probe_offset(g, H[0], H[1], H[2], H[3], i);
    } else if constexpr (OP == BF_OP_ROUTE) {
        for (uint32_t i = 0; i < k; ++i) {
            uint32_t owner;
            uint64_t local;
            owner_local(g, probe_offset(g, H[0], H[1], H[2], H[3], i), owner, local);
            if (g.route32) reinterpret_cast<uint32_t*>(out64)[key * k + i] = (uint32_t)local;
            else out64[key * k + i] = local;
            out8[key * k + i] = (uint8_t)owner;
            atomicAdd(hist + owner, 1u);   // LDS histogram
        }
    } else if constexpr (OP == BF_OP_INCLUDE) {
        // Rounds of up to kChunk independent loads; after the first round (first_round
        // probes) a lane whose AND already failed stops issuing loads — ruby.rb:23's
        // early exit, which only ever saves bandwidth, never changes the answer.
        uint32_t ok = 1u;
        uint32_t i0 = 0;
        uint32_t rend = (g.first_round && g.first_round < k) ? g.first_round : k;
        bool first = true;
        while (i0 < k) {
            const uint32_t e = (i0 + kChunk < rend) ? i0 + kChunk : rend;
            uint32_t v[kChunk], sh[kChunk];
#pragma unroll
            for (int c = 0; c < kChunk; ++c) {   // issue every load of the round first
                v[c] = 0xFFFFFFFFu; sh[c] = 0;
                if (i0 + c < e) {
                    const uint64_t o = probe_offset(g, H[0], H[1], H[2], H[3], i0 + c);
                    sh[c] = (uint32_t)(o ^ 7u) & 31u;
                    v[c] = g.bits[o >> 5];
                }
            }
            if (first) {
                side();
                first = false;
            }
#pragma unroll
            for (int c = 0; c < kChunk; ++c) ok &= v[c] >> sh[c];
            i0 = e;
            rend = (g.next_round && i0 + g.next_round < k) ? i0 + g.next_round : k;
            if (!(ok & 1u)) break;
        }
        out8[key] = (uint8_t)(ok & 1u);
    } else {
        uint32_t isnew = 0;
        for (uint32_t i0 = 0; i0 < k; i0 += kChunk) {
            uint64_t w[kChunk];
            uint32_t mask[kChunk], v[kChunk];
#pragma unroll
            for (int c = 0; c < kChunk; ++c) {
                w[c] = 0; mask[c] = 0; v[c] = 0;
                if (i0 + c < k) {
                    const uint64_t o = probe_offset(g, H[0], H[1], H[2], H[3], i0 + c);
                    w[c] = o >> 5;
                    mask[c] = 1u << ((uint32_t)(o ^ 7u) & 31u);
                    // test-then-set: a 1 seen here is final (bits only go 0 -> 1 within a
                    // launch); a stale 0 just costs an atomic that then reports the truth.
                    if (g.insert_test) v[c] = g.bits[w[c]];
                }
            }
#pragma unroll
            for (int c = 0; c < kChunk; ++c) {
                if (mask[c] && !(v[c] & mask[c])) {
                    if (g.dirty) g.dirty[w[c] >> (kDirtyShiftBits - 5)] = 1;   // bf_track_dirty
                    if constexpr (OP == BF_OP_INSERT_FLAGS) {
                        const uint32_t old = __hip_atomic_fetch_or(g.bits + w[c], mask[c], __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT);
                        isnew |= (old & mask[c]) ? 0u : 1u;
                        if (g.flips && !(old & mask[c])) {   // this lane flipped it: report it once
                            const unsigned long long at = atomicAdd(g.flip_count, 1ull);
                            if (at < g.flip_cap)
                                g.flips[at] = ((w[c] << 5) | ((uint64_t)(__builtin_ctz(mask[c]) ^ 7u))) | g.flip_tag;
                        }
                    } else {
                        __hip_atomic_fetch_or(g.bits + w[c], mask[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
        }
        if constexpr (OP == BF_OP_INSERT_FLAGS) {
            if (out8) out8[key] = (uint8_t)isnew;
            newflag = isnew;
        }
    }
}

struct NoSide {
    __device__ __forceinline__ void operator()() const {}
};

template <int OP, bool STAGED>
__device__ __forceinline__ void key_op(const BfGeom& g, const uint32_t* src, uint32_t s, uint32_t L,
                                       uint64_t key, uint8_t* __restrict__ out8,
                                       uint64_t* __restrict__ out64, uint32_t& newflag,
                                       uint32_t* hist) {
    uint32_t H[5];
    sha1_any<STAGED>(src, s, L, H);
    digest_op<OP>(g, H, key, out8, out64, newflag, hist, NoSide{});
}

template <int OP>
__global__ __launch_bounds__(kBlock) void bf_keys_kernel(BfGeom g, const uint8_t* __restrict__ keys16,
                                                         const uint64_t* __restrict__ offsets,
                                                         uint64_t bias, uint64_t n,
                                                         uint8_t* __restrict__ out8,
                                                         uint64_t* __restrict__ out64,
                                                         uint32_t* __restrict__ any_flag,
                                                         unsigned long long* __restrict__ counts) {
    __shared__ uint64_t s_off[kBlock + 1];
    __shared__ uint4 s_stage[kStageVec + kStageSlackVec];   // slack: sha1_key_staged reads up to 64 B past a key
    __shared__ uint32_t s_hist[OP == BF_OP_ROUTE ? 256 : 1];

    const uint64_t blk0 = (uint64_t)blockIdx.x * kBlock;
    const uint32_t t = threadIdx.x;
    const uint64_t rem = n - blk0;
    const uint32_t cnt = rem < (uint64_t)kBlock ? (uint32_t)rem : (uint32_t)kBlock;

    if (t < cnt) s_off[t] = offsets[blk0 + t] + bias;
    if (t == 0) s_off[cnt] = offsets[blk0 + cnt] + bias;
    if constexpr (OP == BF_OP_ROUTE) s_hist[t] = 0;   // kBlock == 256 bins
    __syncthreads();

    const uint64_t start = s_off[0];
    const uint64_t end = s_off[cnt];
    const uint64_t abase = start & ~(uint64_t)15;
    const uint64_t nvec = end >= start ? (end - abase + 15) >> 4 : ~0ull;
    const bool staged = nvec <= (uint64_t)kStageVec;   // workgroup-uniform

    uint32_t newflag = 0;
    if (staged) {
        const uint4* gv = reinterpret_cast<const uint4*>(keys16 + abase);
        for (uint32_t v = t; v < (uint32_t)nvec; v += kBlock) s_stage[v] = gv[v];
        __syncthreads();
        if (t < cnt) {
            const bool ok = key_ok(start, s_off[t], s_off[t + 1], end, g.key_status);   // else the empty key
            const uint32_t s = ok ? (uint32_t)(s_off[t] - abase) : 0u;
            const uint32_t L = ok ? (uint32_t)(s_off[t + 1] - s_off[t]) : 0u;
            const uint32_t* sw = reinterpret_cast<const uint32_t*>(s_stage);
            key_op<OP, true>(g, sw, s, L, blk0 + t, out8, out64, newflag, s_hist);
        }
    } else if (t < cnt) {
        // Span too large for the stage (long keys): read each key straight from global.
        const bool ok = key_ok(start, s_off[t], s_off[t + 1], end, g.key_status);
        const uint64_t ks = ok ? s_off[t] : 0;
        const uint64_t kbase = ks & ~(uint64_t)3;
        const uint32_t* gw = reinterpret_cast<const uint32_t*>(keys16 + kbase);
        const uint64_t L64 = ok ? s_off[t + 1] - ks : 0;
        key_op<OP, false>(g, gw, (uint32_t)(ks - kbase), (uint32_t)L64, blk0 + t, out8, out64, newflag, s_hist);
    }

    if constexpr (OP == BF_OP_ROUTE) {
        __syncthreads();
        if (t < g.shards && s_hist[t]) atomicAdd(counts + t, (unsigned long long)s_hist[t]);
    }

    if constexpr (OP == BF_OP_INSERT_FLAGS) {
        if (any_flag) report_any_new(any_flag, newflag != 0);
    }
}

// The ops on precomputed SHA-1 words (bf_hash_many_dev's output, 16 B per key): one lane per
// key, no hashing.
template <int OP>
__global__ __launch_bounds__(kBlock) void bf_digest_kernel(BfGeom g, const uint4* __restrict__ dig, uint64_t n,
                                                           uint8_t* __restrict__ out8, uint64_t* __restrict__ out64,
                                                           uint32_t* __restrict__ any_flag) {
    const uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t newflag = 0;
    if (j < n) {
        const uint4 d = dig[j];
        const uint32_t H[4] = {d.x, d.y, d.z, d.w};
        digest_op<OP>(g, H, j, out8, out64, newflag, nullptr, NoSide{});
    }
    if constexpr (OP == BF_OP_INSERT_FLAGS) {
        if (any_flag) report_any_new(any_flag, newflag != 0);
    }
}

// include? of batch Q fused with the SHA-1 of another batch S (S's digests out): both key
// tiles are staged into LDS up front (8 KiB each, so the LDS per workgroup — and the 32
// waves per CU the include? needs for its memory parallelism — stay what the plain include?
// kernel has); the lane hashes its Q key, issues the first probe round, hashes its S key
// while those loads are in flight, stores the S digest, then finishes the probes.  The
// include? waits on its probes' memory latency with its VALUs mostly idle, so S's hashing
// costs little here, and S's insert then skips its own hash pass (bin_front_digest).
// A tile whose bytes exceed its 8 KiB stage hashes from global memory instead.
constexpr int kHalfStageVec = 480;   // 7.5 KiB per stage: 2 stages + offsets <= 20 KiB, 8 workgroups per CU

// Stages one tile's offsets and bytes; returns whether the bytes fit the stage (uniform).
__device__ __forceinline__ bool stage_tile(const uint8_t* __restrict__ keys16, const uint64_t* __restrict__ offsets,
                                           uint64_t bias, uint64_t key0, uint32_t cnt, uint64_t* s_off,
                                           uint4* s_stage, uint64_t* abase_out) {
    const uint32_t t = threadIdx.x;
    if (cnt == 0) return true;
    // s_off was filled (and a barrier passed) by the caller
    const uint64_t start = s_off[0];
    const uint64_t end = s_off[cnt];
    const uint64_t abase = start & ~(uint64_t)15;
    const uint64_t nvec = end >= start ? (end - abase + 15) >> 4 : ~0ull;
    *abase_out = abase;
    if (nvec > (uint64_t)kHalfStageVec) return false;
    const uint4* gv = reinterpret_cast<const uint4*>(keys16 + abase);
    for (uint32_t v = t; v < (uint32_t)nvec; v += kBlock) s_stage[v] = gv[v];
    (void)offsets; (void)bias; (void)key0;
    return true;
}

// Key t of a staged tile of cnt keys (a key bfdev::key_ok refuses: the empty key).
__device__ __forceinline__ void hash_tile_key(const uint8_t* __restrict__ keys16, const uint64_t* s_off,
                                              const uint4* s_stage, bool staged, uint64_t abase, uint32_t t,
                                              uint32_t cnt, uint32_t* key_status, uint32_t H[5]) {
    const bool ok = key_ok(s_off[0], s_off[t], s_off[t + 1], s_off[cnt], key_status);
    if (staged) {
        sha1_key_staged(reinterpret_cast<const uint32_t*>(s_stage), ok ? (uint32_t)(s_off[t] - abase) : 0u,
                        ok ? (uint32_t)(s_off[t + 1] - s_off[t]) : 0u, H);
    } else {
        const uint64_t ks = ok ? s_off[t] : 0;
        const uint64_t kbase = ks & ~(uint64_t)3;
        sha1_key(reinterpret_cast<const uint32_t*>(keys16 + kbase), (uint32_t)(ks - kbase),
                 ok ? (uint32_t)(s_off[t + 1] - ks) : 0u, H);
    }
}

__global__ __launch_bounds__(kBlock) void bf_include_hash_kernel(BfGeom g, const uint8_t* __restrict__ keys16,
                                                                 const uint64_t* __restrict__ offsets, uint64_t bias,
                                                                 uint64_t n, uint8_t* __restrict__ out8,
                                                                 const uint8_t* __restrict__ skeys16,
                                                                 const uint64_t* __restrict__ soffsets, uint64_t sbias,
                                                                 uint64_t sn, uint4* __restrict__ sdig) {
    __shared__ uint64_t s_off[kBlock + 1], s_soff[kBlock + 1];
    __shared__ uint4 s_stage[kHalfStageVec + kStageSlackVec], s_sstage[kHalfStageVec + kStageSlackVec];
    const uint64_t blk0 = (uint64_t)blockIdx.x * kBlock;
    const uint32_t t = threadIdx.x;
    const uint32_t cnt = blk0 < n ? (n - blk0 < (uint64_t)kBlock ? (uint32_t)(n - blk0) : (uint32_t)kBlock) : 0u;
    const uint32_t scnt = blk0 < sn ? (sn - blk0 < (uint64_t)kBlock ? (uint32_t)(sn - blk0) : (uint32_t)kBlock) : 0u;
    if (t < cnt) s_off[t] = offsets[blk0 + t] + bias;
    if (t == 0 && cnt) s_off[cnt] = offsets[blk0 + cnt] + bias;
    if (t < scnt) s_soff[t] = soffsets[blk0 + t] + sbias;
    if (t == 0 && scnt) s_soff[scnt] = soffsets[blk0 + scnt] + sbias;
    __syncthreads();
    uint64_t abase = 0, sabase = 0;
    const bool qstaged = stage_tile(keys16, offsets, bias, blk0, cnt, s_off, s_stage, &abase);
    const bool sstaged = stage_tile(skeys16, soffsets, sbias, blk0, scnt, s_soff, s_sstage, &sabase);
    __syncthreads();
    auto side = [&]() {
        if (t < scnt) {
            uint32_t H[5];
            hash_tile_key(skeys16, s_soff, s_sstage, sstaged, sabase, t, scnt, g.key_status, H);
            sdig[blk0 + t] = make_uint4(H[0], H[1], H[2], H[3]);
        }
    };
    if (t < cnt) {
        uint32_t H[5];
        hash_tile_key(keys16, s_off, s_stage, qstaged, abase, t, cnt, g.key_status, H);
        uint32_t newflag = 0;
        digest_op<BF_OP_INCLUDE>(g, H, blk0 + t, out8, nullptr, newflag, nullptr, side);
    } else {
        side();
    }
}

__global__ __launch_bounds__(256) void last_nonzero_kernel(const uint4* __restrict__ v, uint64_t nvec,
                                                           unsigned long long* __restrict__ d_last) {
    unsigned long long best = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
        const uint4 x = v[i];
        unsigned long long cand = 0;
        if (x.w) cand = 4 * i + 4;
        else if (x.z) cand = 4 * i + 3;
        else if (x.y) cand = 4 * i + 2;
        else if (x.x) cand = 4 * i + 1;
        best = cand > best ? cand : best;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(best, off);
        best = o > best ? o : best;
    }
    if ((threadIdx.x & 63u) == 0 && best) atomicMax(d_last, best);
}

__global__ __launch_bounds__(256) void or_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                 uint64_t nvec) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
        uint4 a = dst[i];
        const uint4 b = src[i];
        a.x |= b.x; a.y |= b.y; a.z |= b.z; a.w |= b.w;
        dst[i] = a;
    }
}

// ---- partitioned filters ---------------------------------------------------

constexpr int kScatterItems = 8;   // probes per lane in the scatter pass

// cursor[s] = exclusive prefix sum of counts (P <= 255: one wave is plenty).
__global__ void displ_kernel(const unsigned long long* __restrict__ counts, uint32_t P,
                             unsigned long long* __restrict__ cursor) {
    if (threadIdx.x == 0) {
        unsigned long long acc = 0;
        for (uint32_t s = 0; s < P; ++s) { cursor[s] = acc; acc += counts[s]; }
    }
}

// Groups probes by owner: one LDS histogram per workgroup, one global
// atomicAdd per (workgroup, owner) to reserve a contiguous range, then every
// probe lands at range base + its LDS rank.
template <typename Off>
__global__ __launch_bounds__(256) void route_scatter_kernel(const Off* __restrict__ local,
                                                            const uint8_t* __restrict__ owner,
                                                            uint64_t total, uint32_t P, uint32_t k,
                                                            unsigned long long* __restrict__ cursor,
                                                            Off* __restrict__ send,
                                                            uint32_t* __restrict__ slot) {
    __shared__ uint32_t s_cnt[256];
    __shared__ unsigned long long s_base[256];
    const uint32_t t = threadIdx.x;
    s_cnt[t] = 0;
    __syncthreads();
    const uint64_t p0 = (uint64_t)blockIdx.x * 256 * kScatterItems;
    uint32_t own[kScatterItems], rank[kScatterItems];
#pragma unroll
    for (int it = 0; it < kScatterItems; ++it) {
        const uint64_t p = p0 + (uint64_t)it * 256 + t;
        own[it] = 0xFFFFFFFFu;
        if (p < total) {
            own[it] = owner[p];
            rank[it] = atomicAdd(s_cnt + own[it], 1u);
        }
    }
    __syncthreads();
    if (t < P && s_cnt[t]) s_base[t] = atomicAdd(cursor + t, (unsigned long long)s_cnt[t]);
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kScatterItems; ++it) {
        const uint64_t p = p0 + (uint64_t)it * 256 + t;
        if (own[it] != 0xFFFFFFFFu) {
            const unsigned long long pos = s_base[own[it]] + rank[it];
            send[pos] = local[p];
            if (slot) slot[pos] = (uint32_t)(p / k);   // key index of send entry pos
        }
    }
}

// Window layout (wcounts != NULL): blockIdx.y is window w, whose entries sit at w * wcap and
// whose live count is min(wcounts[w * wstride], wcap) (the sync-free exchange's fixed
// receive windows); otherwise one run of `count` entries.
template <bool FLAGS, typename Off>
__global__ __launch_bounds__(256) void shard_insert_kernel(uint32_t* __restrict__ bits, uint64_t limit,
                                                           const Off* __restrict__ local,
                                                           uint64_t count, uint32_t* __restrict__ any_flag,
                                                           uint64_t bias, uint8_t* __restrict__ dirty,
                                                           uint64_t wcap, const unsigned long long* __restrict__ wcounts,
                                                           uint32_t wstride) {
    // Test-then-set as in the direct insert: 4 probes per lane in flight, an atomic
    // only for bits still 0 (a 1 seen here is final within the launch).
    constexpr int U = 4;
    if (wcounts) {
        local += (uint64_t)blockIdx.y * wcap;
        count = wcounts[(uint64_t)blockIdx.y * wstride];
        if (count > wcap) count = 0;   // an overflowed window holds unwritten entries: skip it whole
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t isnew = 0;
    for (uint64_t p0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p0 < count; p0 += U * stride) {
        uint64_t w[U];
        uint32_t mask[U], v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t p = p0 + u * stride;
            mask[u] = 0; v[u] = 0; w[u] = 0;
            if (p < count) {
                const uint64_t o = (uint64_t)local[p] + bias;
                if (o < limit) {   // an offset past the shard is dropped, never dereferenced
                    w[u] = o >> 5;
                    mask[u] = 1u << ((uint32_t)(o ^ 7u) & 31u);
                    v[u] = bits[w[u]];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (mask[u] && !(v[u] & mask[u])) {
                if (dirty) dirty[w[u] >> (kDirtyShiftBits - 5)] = 1;   // bf_track_dirty (shards of a multi-device handle)
                if constexpr (FLAGS) {
                    const uint32_t old = __hip_atomic_fetch_or(bits + w[u], mask[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    isnew |= (old & mask[u]) ? 0u : 1u;
                } else {
                    __hip_atomic_fetch_or(bits + w[u], mask[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
    if constexpr (FLAGS) report_any_new(any_flag, isnew != 0);
}

template <typename Off>
__global__ __launch_bounds__(256) void shard_test_kernel(const uint32_t* __restrict__ bits, uint64_t limit,
                                                         const Off* __restrict__ local, uint64_t count,
                                                         uint8_t* __restrict__ out, uint64_t bias, uint64_t wcap,
                                                         const unsigned long long* __restrict__ wcounts,
                                                         uint32_t wstride) {
    constexpr int U = 4;   // 4 independent probe loads per lane in flight
    if (wcounts) {   // window layout, as shard_insert_kernel
        local += (uint64_t)blockIdx.y * wcap;
        out += (uint64_t)blockIdx.y * wcap;
        count = wcounts[(uint64_t)blockIdx.y * wstride];
        if (count > wcap) count = 0;   // an overflowed window holds unwritten entries: skip it whole
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p0 < count; p0 += U * stride) {
        uint32_t v[U], sh[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t p = p0 + u * stride;
            v[u] = 0; sh[u] = 0;
            if (p < count) {
                const uint64_t o = (uint64_t)local[p] + bias;
                if (o < limit) {   // an offset past the shard answers 0, never dereferenced
                    sh[u] = (uint32_t)(o ^ 7u) & 31u;
                    v[u] = bits[o >> 5];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t p = p0 + u * stride;
            if (p < count) out[p] = (uint8_t)((v[u] >> sh[u]) & 1u);
        }
    }
}

// out[] preset to 1: a probe whose owner answered 0 clears its key's answer (every
// writer stores the same 0, so no atomics are needed).
__global__ __launch_bounds__(256) void combine_kernel(const uint8_t* __restrict__ bits,
                                                      const uint32_t* __restrict__ slot, uint64_t total,
                                                      uint64_t n, uint8_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total; p += stride)
        if (!bits[p] && slot[p] < n) out[slot[p]] = 0;
}

// The same over the window layout of bf_route_windows_dev: window s holds counts[s] live
// entries at s*wcap; the rest of each window is ignored.
__global__ __launch_bounds__(256) void combine_windows_kernel(const uint8_t* __restrict__ bits,
                                                              const uint32_t* __restrict__ slot, uint64_t wcap,
                                                              const unsigned long long* __restrict__ counts,
                                                              uint32_t P, uint64_t n, uint8_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t s = blockIdx.y;   // one grid row per window
    // an overflowed window (counts[s] > wcap) holds unwritten entries: it is skipped whole
    // (the synced exchange re-routes such a batch; the sync-free one replays it)
    const uint64_t live = counts[s] <= wcap ? counts[s] : 0;
    const uint8_t* wb = bits + s * wcap;
    const uint32_t* ws = slot + s * wcap;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < live; i += stride)
        if (!wb[i] && ws[i] < n) out[ws[i]] = 0;
}

// Answer bytes -> bits for the return trip of a partitioned include?: segment q =
// (src offset, count, dst byte offset) packs bits[src .. src + count) LSB-first into
// ceil(count / 8) bytes at packed[dst].  One grid row per segment.  A segment whose source is
// 16-B aligned and whose destination is 4-B aligned (every window of the sync-free exchange:
// caps are multiples of 12288) takes 32 answer bytes per lane in two 16-B loads and stores one
// u32: each 8 bytes fold to a byte by one multiply (the bytes are 0 or 1; bit 8i -> bit 56 + i).
// (The byte-per-load form ran at 0.74 TB/s: 0.33 ms per 218M answers at 200B x 8.)
__device__ __forceinline__ uint32_t pack8(uint64_t x) {
    return (uint32_t)(((x & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
}

__global__ __launch_bounds__(256) void pack_segments_kernel(const uint8_t* __restrict__ bits,
                                                            const unsigned long long* __restrict__ seg,
                                                            uint8_t* __restrict__ packed) {
    const unsigned long long src = seg[3 * blockIdx.y], cnt = seg[3 * blockIdx.y + 1], dst = seg[3 * blockIdx.y + 2];
    const uint64_t nbytes = (cnt + 7) / 8;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t b0 = 0;   // packed bytes done by the vector loop
    if (((src & 15u) | (dst & 3u)) == 0) {   // segment-uniform
        const uint64_t nw = cnt / 32;   // whole u32 words of output
        const uint4* in = reinterpret_cast<const uint4*>(bits + src);
        uint32_t* out = reinterpret_cast<uint32_t*>(packed + dst);
        for (uint64_t w = t0; w < nw; w += stride) {
            const uint4 a = in[2 * w], b = in[2 * w + 1];
            out[w] = pack8(((uint64_t)a.y << 32) | a.x) | (pack8(((uint64_t)a.w << 32) | a.z) << 8) |
                     (pack8(((uint64_t)b.y << 32) | b.x) << 16) | (pack8(((uint64_t)b.w << 32) | b.z) << 24);
        }
        b0 = nw * 4;
    }
    for (uint64_t b = b0 + t0; b < nbytes; b += stride) {   // the tail (or an unaligned segment)
        uint32_t v = 0;
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i)
            if (b * 8 + i < cnt) v |= (uint32_t)(bits[src + b * 8 + i] & 1u) << i;
        packed[dst + b] = (uint8_t)v;
    }
}

// combine_windows_kernel over packed answers: window s's entry i is bit (i & 7) of
// packed[s * wcap8 + i / 8].
__global__ __launch_bounds__(256) void combine_windows_packed_kernel(const uint8_t* __restrict__ packed,
                                                                     const uint32_t* __restrict__ slot, uint64_t wcap,
                                                                     uint64_t wcap8,
                                                                     const unsigned long long* __restrict__ counts,
                                                                     uint64_t n, uint8_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t s = blockIdx.y;
    // an overflowed window (counts[s] > wcap) holds unwritten entries: it is skipped whole
    // (the synced exchange re-routes such a batch; the sync-free one replays it)
    const uint64_t live = counts[s] <= wcap ? counts[s] : 0;
    const uint8_t* wb = packed + s * wcap8;
    const uint32_t* ws = slot + s * wcap;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < live; i += stride)
        if (!((wb[i >> 3] >> (i & 7)) & 1u) && ws[i] < n) out[ws[i]] = 0;
}

// Host-pointer calls ship each chunk's offsets as uint32 relative to the chunk's first key
// (4 B per key over PCIe instead of 8); the kernels take uint64.
__global__ __launch_bounds__(256) void widen_offsets_kernel(const uint32_t* __restrict__ in,
                                                            uint64_t* __restrict__ out, uint64_t count) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride)
        out[i] = in[i];
}

uint32_t stream_grid(uint64_t nvec) {
    uint64_t g = (nvec + 255) / 256;
    if (g > 2048) g = 2048;   // grid-stride beyond 8 blocks per CU
    return g ? (uint32_t)g : 1u;
}

}  // namespace

hipError_t bf_launch_keys(BfOp op, const BfGeom& g, const uint8_t* keys16, const uint64_t* offsets,
                          uint64_t bias, uint64_t n, uint8_t* out8, uint64_t* out64,
                          uint32_t* any_flag, hipStream_t s, unsigned long long* counts) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)blocks), block(kBlock);
#define BF_LAUNCH(OPC) \
    hipLaunchKernelGGL(bf_keys_kernel<OPC>, grid, block, 0, s, g, keys16, offsets, bias, n, out8, out64, any_flag, counts)
    switch (op) {
        case BF_OP_INDEXES: BF_LAUNCH(BF_OP_INDEXES); break;
        case BF_OP_INCLUDE: BF_LAUNCH(BF_OP_INCLUDE); break;
        case BF_OP_INSERT: BF_LAUNCH(BF_OP_INSERT); break;
        case BF_OP_INSERT_FLAGS: BF_LAUNCH(BF_OP_INSERT_FLAGS); break;
        case BF_OP_HASH: BF_LAUNCH(BF_OP_HASH); break;
        case BF_OP_ROUTE:
            if (!counts || g.shards == 0 || g.shards > 255) return hipErrorInvalidValue;
            BF_LAUNCH(BF_OP_ROUTE);
            break;
        default:
            return hipErrorInvalidValue;
    }
#undef BF_LAUNCH
    return hipGetLastError();
}

hipError_t bf_launch_route_scatter(const void* local, const uint8_t* owner, uint64_t total, uint32_t P,
                                   uint32_t k, const unsigned long long* counts, unsigned long long* cursor,
                                   void* send, uint32_t* slot, bool route32, hipStream_t s) {
    hipLaunchKernelGGL(displ_kernel, dim3(1), dim3(64), 0, s, counts, P, cursor);
    if (total == 0) return hipGetLastError();
    const uint64_t per = 256ull * kScatterItems;
    const dim3 grid((uint32_t)((total + per - 1) / per));
    if (route32)
        hipLaunchKernelGGL(route_scatter_kernel<uint32_t>, grid, dim3(256), 0, s, static_cast<const uint32_t*>(local),
                           owner, total, P, k, cursor, static_cast<uint32_t*>(send), slot);
    else
        hipLaunchKernelGGL(route_scatter_kernel<uint64_t>, grid, dim3(256), 0, s, static_cast<const uint64_t*>(local),
                           owner, total, P, k, cursor, static_cast<uint64_t*>(send), slot);
    return hipGetLastError();
}

// Grid of a windowed launch: `count` entries over nwin windows of wcap (nwin = 1: one run).
static dim3 window_grid(uint64_t count, uint32_t nwin) {
    if (nwin <= 1) return dim3(stream_grid(count));
    uint32_t gx = stream_grid(count) / nwin;
    return dim3(gx ? gx : 1u, nwin);
}

template <typename Off>
static void launch_shard_insert(uint32_t* bits, uint64_t limit, const void* local, uint64_t count, uint32_t* any_flag,
                                uint64_t bias, uint8_t* dirty, hipStream_t s, const BfWindows& w) {
    const Off* l = static_cast<const Off*>(local);
    const dim3 grid = window_grid(count, w.counts ? w.nwin : 1u);
    if (any_flag)
        hipLaunchKernelGGL((shard_insert_kernel<true, Off>), grid, dim3(256), 0, s, bits, limit, l, count, any_flag,
                           bias, dirty, w.cap, w.counts, w.stride);
    else
        hipLaunchKernelGGL((shard_insert_kernel<false, Off>), grid, dim3(256), 0, s, bits, limit, l, count, any_flag,
                           bias, dirty, w.cap, w.counts, w.stride);
}

hipError_t bf_launch_shard_insert(uint32_t* bits, uint64_t limit, const void* local, uint64_t count,
                                  uint32_t* any_flag, bool route32, hipStream_t s, uint64_t bias, uint8_t* dirty,
                                  const BfWindows& w) {
    if (count == 0) return hipSuccess;
    if (route32) launch_shard_insert<uint32_t>(bits, limit, local, count, any_flag, bias, dirty, s, w);
    else launch_shard_insert<uint64_t>(bits, limit, local, count, any_flag, bias, dirty, s, w);
    return hipGetLastError();
}

hipError_t bf_launch_shard_test(const uint32_t* bits, uint64_t limit, const void* local, uint64_t count, uint8_t* out,
                                bool route32, hipStream_t s, uint64_t bias, const BfWindows& w) {
    if (count == 0) return hipSuccess;
    const dim3 grid = window_grid(count, w.counts ? w.nwin : 1u);
    if (route32)
        hipLaunchKernelGGL(shard_test_kernel<uint32_t>, grid, dim3(256), 0, s, bits, limit,
                           static_cast<const uint32_t*>(local), count, out, bias, w.cap, w.counts, w.stride);
    else
        hipLaunchKernelGGL(shard_test_kernel<uint64_t>, grid, dim3(256), 0, s, bits, limit,
                           static_cast<const uint64_t*>(local), count, out, bias, w.cap, w.counts, w.stride);
    return hipGetLastError();
}

hipError_t bf_launch_combine(const uint8_t* bits, const uint32_t* slot, uint64_t n, uint32_t k, uint8_t* out,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(out, 1, n, s);
    if (e != hipSuccess) return e;
    const uint64_t total = n * k;
    hipLaunchKernelGGL(combine_kernel, dim3(stream_grid(total)), dim3(256), 0, s, bits, slot, total, n, out);
    return hipGetLastError();
}

hipError_t bf_launch_combine_windows(const uint8_t* bits, const uint32_t* slot, uint64_t wcap,
                                     const unsigned long long* counts, uint32_t P, uint64_t n, uint8_t* out,
                                     hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(out, 1, n, s);
    if (e != hipSuccess) return e;
    if (wcap == 0) return hipSuccess;
    uint32_t gx = stream_grid(wcap) / P;
    hipLaunchKernelGGL(combine_windows_kernel, dim3(gx ? gx : 1u, P), dim3(256), 0, s, bits, slot, wcap, counts, P,
                       n, out);
    return hipGetLastError();
}

hipError_t bf_launch_pack_segments(const uint8_t* bits, const unsigned long long* seg, uint32_t nseg,
                                   uint64_t max_count, uint8_t* packed, hipStream_t s) {
    if (nseg == 0 || max_count == 0) return hipSuccess;
    uint32_t gx = stream_grid((max_count + 31) / 32) / nseg;   // a lane per 32 answers
    hipLaunchKernelGGL(pack_segments_kernel, dim3(gx ? gx : 1u, nseg), dim3(256), 0, s, bits, seg, packed);
    return hipGetLastError();
}

hipError_t bf_launch_combine_windows_packed(const uint8_t* packed, const uint32_t* slot, uint64_t wcap,
                                            const unsigned long long* counts, uint32_t P, uint64_t n, uint8_t* out,
                                            hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(out, 1, n, s);
    if (e != hipSuccess) return e;
    if (wcap == 0) return hipSuccess;
    uint32_t gx = stream_grid(wcap) / P;
    hipLaunchKernelGGL(combine_windows_packed_kernel, dim3(gx ? gx : 1u, P), dim3(256), 0, s, packed, slot, wcap,
                       (wcap + 7) / 8, counts, n, out);
    return hipGetLastError();
}

hipError_t bf_launch_last_nonzero(const uint32_t* words, uint64_t nwords, unsigned long long* d_last,
                                  hipStream_t s) {
    const uint64_t nvec = nwords / 4;
    if (nvec == 0) return hipSuccess;
    hipLaunchKernelGGL(last_nonzero_kernel, dim3(stream_grid(nvec)), dim3(256), 0, s,
                       reinterpret_cast<const uint4*>(words), nvec, d_last);
    return hipGetLastError();
}

hipError_t bf_launch_or(uint32_t* dst, const uint32_t* src, uint64_t nwords, hipStream_t s) {
    const uint64_t nvec = nwords / 4;
    if (nvec == 0) return hipSuccess;
    hipLaunchKernelGGL(or_kernel, dim3(stream_grid(nvec)), dim3(256), 0, s,
                       reinterpret_cast<uint4*>(dst), reinterpret_cast<const uint4*>(src), nvec);
    return hipGetLastError();
}

hipError_t bf_launch_widen_offsets(const uint32_t* in, uint64_t* out, uint64_t count, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(widen_offsets_kernel, dim3(stream_grid(count)), dim3(256), 0, s, in, out, count);
    return hipGetLastError();
}

hipError_t bf_launch_digests(BfOp op, const BfGeom& g, const uint4* dig, uint64_t n, uint8_t* out8, uint64_t* out64,
                             uint32_t* any_flag, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)blocks), block(kBlock);
    switch (op) {
        case BF_OP_INDEXES: hipLaunchKernelGGL(bf_digest_kernel<BF_OP_INDEXES>, grid, block, 0, s, g, dig, n, out8, out64, any_flag); break;
        case BF_OP_INCLUDE: hipLaunchKernelGGL(bf_digest_kernel<BF_OP_INCLUDE>, grid, block, 0, s, g, dig, n, out8, out64, any_flag); break;
        case BF_OP_INSERT: hipLaunchKernelGGL(bf_digest_kernel<BF_OP_INSERT>, grid, block, 0, s, g, dig, n, out8, out64, any_flag); break;
        case BF_OP_INSERT_FLAGS: hipLaunchKernelGGL(bf_digest_kernel<BF_OP_INSERT_FLAGS>, grid, block, 0, s, g, dig, n, out8, out64, any_flag); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t bf_launch_include_hash(const BfGeom& g, const uint8_t* keys16, const uint64_t* offsets, uint64_t bias,
                                  uint64_t n, uint8_t* out8, const uint8_t* skeys16, const uint64_t* soffsets,
                                  uint64_t sbias, uint64_t sn, uint4* sdig, hipStream_t s) {
    const uint64_t m = n > sn ? n : sn;
    if (m == 0) return hipSuccess;
    const uint64_t blocks = (m + kBlock - 1) / kBlock;
    if (blocks > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bf_include_hash_kernel, dim3((uint32_t)blocks), dim3(kBlock), 0, s, g, keys16, offsets, bias, n,
                       out8, skeys16, soffsets, sbias, sn, sdig);
    return hipGetLastError();
}
