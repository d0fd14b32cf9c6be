// bf_device.h — device-side building blocks shared by the kernels: SHA-1 over
// LDS-staged packed keys, the ruby driver's offset derivation, the ownership
// map of partitioned filters, and the workgroup key-tile stager.
#pragma once
#include "bf_internal.h"

#include <type_traits>

namespace bfdev {

constexpr int kBlock = 256;             // lanes per workgroup = keys per workgroup
constexpr int kStageBytes = 16384;      // LDS key stage per workgroup
constexpr int kStageVec = kStageBytes / 16;
constexpr int kChunk = 8;               // probes issued together per key
constexpr int kStageSlackVec = 5;       // LDS slack (16-B vectors) past a key stage

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_rotateleft32(x, n); }

// a ^ b ^ c in ONE gfx950 v_bitop3_b32 (truth table 0x96).  hipcc (ROCm 7.2)
// emits two v_xor_b32 for this pattern; SHA-1 has 40 parity rounds and 64
// schedule steps that each need it.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// FIPS 180-4 SHA-1 compression of one 16-word block; w[] is consumed as the
// circular message schedule.  Fully unrolled so every w index is static.
__device__ __forceinline__ void sha1_compress(uint32_t h[5], uint32_t w[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        uint32_t f, kk;
        if (t < 20)      { f = d ^ (b & (c ^ d));           kk = 0x5A827999u; }  // Ch  -> v_bitop3 0xac
        else if (t < 40) { f = xor3(b, c, d);               kk = 0x6ED9EBA1u; }  // Parity
        else if (t < 60) { f = (b & c) | (d & (b | c));     kk = 0x8F1BBCDCu; }  // Maj
        else             { f = xor3(b, c, d);               kk = 0xCA62C1D6u; }
        const uint32_t tmp = rotl(a, 5) + f + e + kk + wt;
        e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

// Word `wi` (big-endian) of the SHA-1-padded message of a key of L bytes whose
// first byte sits at byte position s of the 32-bit word array `src`.
template <typename Src>
__device__ __forceinline__ uint32_t msg_word(Src src, uint32_t s, uint32_t L, uint32_t wi,
                                             uint32_t total_words) {
    if (wi == total_words - 1) return L << 3;   // bit length, low word
    if (wi == total_words - 2) return L >> 29;  // bit length, high word
    const int valid = (int)L - (int)(4u * wi);  // key bytes left at this word
    uint32_t x = 0;
    if (valid > 0) {
        const uint32_t a = s + 4u * wi;
        const uint32_t lo = src[a >> 2];
        const uint32_t hi = src[(a >> 2) + 1];
        x = __builtin_amdgcn_alignbyte(hi, lo, a & 3u);  // bytes a..a+3, little-endian
    }
    if (valid < 4) {
        if (valid >= 0) {
            x &= (valid == 0) ? 0u : (0xFFFFFFFFu >> (8 * (4 - valid)));
            x |= 0x80u << (8 * valid);                // the FIPS padding byte
        } else {
            x = 0u;
        }
    }
    return __builtin_bswap32(x);
}

template <typename Src>
__device__ __forceinline__ void sha1_key(Src src, uint32_t s, uint32_t L, uint32_t H[5]) {
    H[0] = 0x67452301u; H[1] = 0xEFCDAB89u; H[2] = 0x98BADCFEu; H[3] = 0x10325476u; H[4] = 0xC3D2E1F0u;
    const uint32_t nblk = (L + 8u) / 64u + 1u;
    const uint32_t total = nblk * 16u;
    for (uint32_t b = 0; b < nblk; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = msg_word(src, s, L, b * 16u + j, total);
        sha1_compress(H, w);
    }
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP moves (no LDS round trips, as
// __shfl_up's ds_bpermute takes): four row shifts inside each 16-lane row, then the row ends
// broadcast into the rows above (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and
// 3; gfx9-family DPP).  A lane whose source is shifted out or masked keeps 0.  Every lane of the
// wave must be active (block_excl_scan's contract).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t y = (uint32_t)__shfl_xor((int)x, off);
        x = x > y ? x : y;
    }
    return __builtin_amdgcn_readfirstlane(x);
}

// SHA-1 of a key staged in LDS.  Waves whose keys all fit one block (L <= 55:
// every key family the benches and the reference's tests use) build the 16
// message words branch-free: word j < L/4 is key data, word L/4 carries the
// tail bytes + the 0x80 pad, later words are zero, w15 = 8L.  The wave-uniform
// max of L/4 bounds the loop, so short keys read and build only a few words.
// Needs 64 B of readable LDS slack past the stage.  Other waves: sha1_key.
__device__ __forceinline__ void sha1_key_staged(const uint32_t* src, uint32_t s, uint32_t L, uint32_t H[5]) {
    if (__ballot(L > 55u) != 0ull) {   // wave-uniform
        sha1_key(src, s, L, H);
        return;
    }
    H[0] = 0x67452301u; H[1] = 0xEFCDAB89u; H[2] = 0x98BADCFEu; H[3] = 0x10325476u; H[4] = 0xC3D2E1F0u;
    const uint32_t pw = L >> 2;
    const uint32_t pb = (L & 3u) * 8u;
    const uint32_t keep = (1u << pb) - 1u;   // key-data bytes of the pad word
    const uint32_t pad = 0x80u << pb;
    const uint32_t lim = wave_max_u32(pw);   // words above lim are zero in every lane
    const uint32_t base = s >> 2;
    const uint32_t sh = s & 3u;
#ifndef BFHIP_SHA_SHORT
#define BFHIP_SHA_SHORT 0
#endif
    if (BFHIP_SHA_SHORT && lim <= 4u) {   // wave-uniform: every key <= 19 bytes (the bench's
        // decimal keys): w5..w14 are zero at compile time, so their adds and the early message
        // schedule's XORs fold away (a separate unrolled compression).  Off by default: the
        // north-star step 2.467 / 2.420 vs 2.481 / 2.433 ms, the P = 8 routes within noise
        // (profiles/r04r_ab_sha_short.jsonl); build with -DBFHIP_SHA_SHORT=1 to take it
        uint32_t w[16];
        uint32_t lo = src[base];
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) {
            const uint32_t hi = src[base + j + 1];
            const uint32_t d = __builtin_amdgcn_alignbyte(hi, lo, sh);
            lo = hi;
            w[j] = __builtin_bswap32(j < pw ? d : (j == pw ? ((d & keep) | pad) : 0u));
        }
#pragma unroll
        for (uint32_t j = 5; j < 15; ++j) w[j] = 0u;
        w[15] = L << 3;
        sha1_compress(H, w);
        return;
    }
    uint32_t w[16];
    uint32_t lo = src[base];
#pragma unroll
    for (uint32_t j = 0; j < 14; ++j) {
        uint32_t x = 0u;
        if (j <= lim) {
            const uint32_t hi = src[base + j + 1];
            const uint32_t d = __builtin_amdgcn_alignbyte(hi, lo, sh);
            lo = hi;
            x = __builtin_bswap32(j < pw ? d : (j == pw ? ((d & keep) | pad) : 0u));
        }
        w[j] = x;
    }
    w[14] = 0u;
    w[15] = L << 3;
    sha1_compress(H, w);
}

// Dispatch: keys staged in LDS take the branch-free path, global reads the generic one.
template <bool STAGED>
__device__ __forceinline__ void sha1_any(const uint32_t* src, uint32_t s, uint32_t L, uint32_t H[5]) {
    if constexpr (STAGED) sha1_key_staged(src, s, L, H);
    else sha1_key(src, s, L, H);
}

// ruby.rb:50-53 for probe i, reduced mod m without an integer divide.
__device__ __forceinline__ uint64_t probe_offset(const BfGeom& g, uint32_t h0, uint32_t h1,
                                                 uint32_t h2, uint32_t h3, uint32_t i) {
    const uint32_t a = (i & 1u) ? h1 : h0;
    const uint32_t b = (((i + (i & 1u)) & 3u) >> 1) ? h3 : h2;
    const uint64_t v = (uint64_t)a + (uint64_t)i * (uint64_t)b;  // < k * 2^32: exact
    if (g.nomod) return v;
    if (g.mod_sub) {   // v < (mod_sub + 1) m: conditional subtractions, no estimate
        uint64_t r = v;
#pragma unroll
        for (uint32_t j = 0; j < 3u; ++j)
            if (j < g.mod_sub) r = r >= g.m ? r - g.m : r;
        return r;
    }
    if (g.mod_f32) {
        // m >= 2^17 (set at create): q = v/m < 2^21 (v < 2^38), and a float32 estimate
        // (relative error <= 2^-22) is off by at most one after truncation; the remainder
        // is then fixed exactly in 64-bit integers.
        const float vf = __builtin_fmaf((float)(uint32_t)(v >> 32), 4294967296.0f, (float)(uint32_t)v);
        const uint32_t q = (uint32_t)(vf * g.inv_m_f);
        int64_t r = (int64_t)(v - (uint64_t)q * g.m);
        if (r < 0) r += (int64_t)g.m;
        else if ((uint64_t)r >= g.m) r -= (int64_t)g.m;
        return (uint64_t)r;
    }
    // q within +-1 of floor(v/m): v < 2^38 is exact in a double, 1/m carries 2^-53 relative error.
    const uint64_t q = (uint64_t)((double)v * g.inv_m);
    int64_t r = (int64_t)(v - q * g.m);
    if (r < 0) r += (int64_t)g.m;
    else if ((uint64_t)r >= g.m) r -= (int64_t)g.m;
    return (uint64_t)r;
}

// Block-cyclic ownership of partitioned filters (include/bfhip.h, bf_config):
// block b = o >> block_log2 lives on shard b % P at local block b / P.
__device__ __forceinline__ void owner_local(const BfGeom& g, uint64_t o, uint32_t& owner, uint64_t& local) {
    const uint64_t blk = o >> g.block_log2;
    if (g.shards_pow2) {   // 2, 4, 8 ... GPUs: mask and shift
        owner = (uint32_t)blk & (g.shards - 1u);
        local = ((blk >> g.shard_log2) << g.block_log2) | (o & ((1ull << g.block_log2) - 1ull));
        return;
    }
    // blk < 2^44 is exact in a double and 1/P carries 2^-53 relative error: the estimate
    // is within one of blk / P, fixed exactly below (no 64-bit integer divide)
    uint64_t lblk = (uint64_t)((double)blk * g.inv_shards);
    int64_t own = (int64_t)(blk - lblk * g.shards);
    if (own < 0) { --lblk; own += g.shards; }
    else if (own >= (int64_t)g.shards) { ++lblk; own -= g.shards; }
    owner = (uint32_t)own;
    local = (lblk << g.block_log2) | (o & ((1ull << g.block_log2) - 1ull));
}


// Longest key a kernel hashes: the host path's cap (bf_api.cpp run_host refuses keys of 2 GiB).
constexpr uint64_t kMaxKeyBytes = 1ull << 31;

// Whether key [a, b) of a tile whose offsets run from lo to hi may be hashed: lo <= a <= b <=
// hi and b - a < kMaxKeyBytes.  Tiles chain (one tile's last offset is the next one's first),
// so every key of a batch passing means offsets[0..n] is non-decreasing and every key lies
// inside [offsets[0], offsets[n]).  A key that fails is hashed as the empty string (no byte
// read) and *status (the handle's key-status word, nullable) gets 1: a wrapped length would
// run ~2^26 SHA-1 blocks in one lane (round 5's hang came from a wrapped length) or read past
// the key buffer.  Only failing lanes store; the comparisons cost a few VALU per key.
__host__ __device__ __forceinline__ bool key_ok(uint64_t lo, uint64_t a, uint64_t b, uint64_t hi, uint32_t* status) {
    const bool ok = lo <= a && a <= b && b <= hi && b - a < kMaxKeyBytes;
    if (!ok && status) *status = 1u;
    return ok;
}

// Stages one tile of up to TILE consecutive keys (offsets + packed bytes) into
// LDS and hands each lane its key: f(lane, src_words, start_byte, len).  When the
// tile's bytes exceed the stage (or its offsets run backwards), lanes read their key straight
// from global.  A key key_ok refuses is handed over as the empty key at byte 0.
// Ends with a barrier, so the caller may restage the same LDS right after.
template <int TILE, int STAGE_VEC, typename F>
__device__ __forceinline__ void for_key_tile(const uint8_t* __restrict__ keys16,
                                             const uint64_t* __restrict__ offsets, uint64_t bias,
                                             uint64_t tile0, uint32_t cnt, uint64_t* s_off,
                                             uint4* s_stage, uint32_t* key_status, F&& f) {
    const uint32_t t = threadIdx.x;
    if (t < cnt) s_off[t] = offsets[tile0 + t] + bias;
    if (t == 0) s_off[cnt] = offsets[tile0 + cnt] + bias;
    __syncthreads();
    const uint64_t start = s_off[0];
    const uint64_t end = s_off[cnt];
    const uint64_t abase = start & ~(uint64_t)15;
    const uint64_t nvec = end >= start ? (end - abase + 15) >> 4 : ~0ull;
    if (nvec <= (uint64_t)STAGE_VEC) {   // workgroup-uniform
        const uint4* gv = reinterpret_cast<const uint4*>(keys16 + abase);
        for (uint32_t v = t; v < (uint32_t)nvec; v += TILE) s_stage[v] = gv[v];
        __syncthreads();
        if (t < cnt) {
            const bool ok = key_ok(start, s_off[t], s_off[t + 1], end, key_status);
            f(std::true_type{}, t, reinterpret_cast<const uint32_t*>(s_stage), ok ? (uint32_t)(s_off[t] - abase) : 0u,
              ok ? (uint32_t)(s_off[t + 1] - s_off[t]) : 0u);
        }
    } else if (t < cnt) {
        const bool ok = key_ok(start, s_off[t], s_off[t + 1], end, key_status);
        const uint64_t ks = ok ? s_off[t] : 0;
        const uint64_t kbase = ks & ~(uint64_t)3;
        f(std::false_type{}, t, reinterpret_cast<const uint32_t*>(keys16 + kbase), (uint32_t)(ks - kbase),
          ok ? (uint32_t)(s_off[t + 1] - ks) : 0u);
    }
    __syncthreads();
}


// any_new (the reference's !found, ruby.rb:61-62) as one flag word for a whole launch: every
// writer stores 1, so a wave reports at most once, and not at all once it reads the flag set
// (agent-scope load: L2-served).  A stale 0 only costs an atomic.  Without the check every
// wave with a fresh bit sent a device-scope atomic to the same word — ~11 ns each at the
// memory side, serialised: 1.7M waves of the 10B bin_apply took 19 ms (r03).
__device__ __forceinline__ void report_any_new(uint32_t* any_flag, bool mine) {
    const unsigned long long b = __ballot(mine);
    if (b == 0ull || (threadIdx.x & 63u) != (uint32_t)__builtin_ctzll(b)) return;
    if (__hip_atomic_load(any_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    __hip_atomic_fetch_or(any_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace bfdev
