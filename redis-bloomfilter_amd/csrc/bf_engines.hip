// bf_engines.hip — the RubyTest driver's hash engines (lib/bloomfilter_driver/ruby_test.rb:43-61)
// on the device: probe i of a key is digest("#{i}-#{key.to_s}") read as one big-endian
// integer (`hexdigest.to_i(16)`: 128 bits for MD5, 160 for SHA-1) mod m.  Unlike the ruby
// driver's double hashing (one SHA-1 per key), every probe is its own hash, so the kernels
// run one lane per (key, probe): consecutive lanes are the probes of one key and share its
// bytes through L1.  Offsets reach all of [0, m), so an engine filter is never capped at
// k(2^32-1)+1 bits.  crc32 is broken upstream (Integer#to_i takes no radix, :52) and has no
// kernel: the host refuses it as the reference would fail at its first call.
#include "bf_device.h"

namespace {

using bfdev::rotl;
using bfdev::sha1_compress;

constexpr int kLanes = 256;

// RFC 1321 MD5 compression of one 16-word little-endian block.
__device__ __forceinline__ void md5_compress(uint32_t st[4], const uint32_t w[16]) {
    constexpr uint32_t K[64] = {
        0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
        0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
        0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
        0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
        0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
        0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
        0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
        0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};
    constexpr int S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        uint32_t f;
        int gi;
        if (t < 16)      { f = d ^ (b & (c ^ d));  gi = t; }
        else if (t < 32) { f = c ^ (d & (b ^ c));  gi = (5 * t + 1) & 15; }
        else if (t < 48) { f = b ^ c ^ d;          gi = (3 * t + 5) & 15; }
        else             { f = c ^ (b | ~d);       gi = (7 * t) & 15; }
        const uint32_t tmp = d;
        d = c;
        c = b;
        b = b + rotl(a + f + K[t] + w[gi], S[(t >> 4) * 4 + (t & 3)]);
        a = tmp;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

// Byte j of "#{i}-" + key + padding.  The prefix (<= 11 bytes) lives in three registers.
struct Msg {
    uint32_t pre0, pre1, pre2;   // prefix bytes, little-endian packed
    uint32_t P;                  // prefix length
    const uint8_t* key;
    uint32_t L;                  // key length
};

__device__ __forceinline__ uint32_t msg_byte(const Msg& m, uint32_t j) {
    if (j < m.P) {
        const uint32_t wv = j < 4 ? m.pre0 : (j < 8 ? m.pre1 : m.pre2);
        return (wv >> (8u * (j & 3u))) & 0xFFu;
    }
    j -= m.P;
    if (j < m.L) return m.key[j];
    return j == m.L ? 0x80u : 0u;
}

__device__ __forceinline__ Msg make_msg(uint32_t i, const uint8_t* key, uint32_t L) {
    // prepend digits least significant first: byte 0 ends up the leading digit, '-' last
    unsigned __int128 x = '-';
    uint32_t P = 1;
    do {
        x = (x << 8) | ('0' + i % 10u);
        i /= 10u;
        ++P;
    } while (i);
    return Msg{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64), P, key, L};
}

// (r * 2^32 + w) mod m for r < m.
__device__ __forceinline__ uint64_t mod_step(uint64_t r, uint32_t w, uint64_t m) {
    if (m <= 0xFFFFFFFFull) return ((r << 32) | w) % m;
    return (uint64_t)((((unsigned __int128)r << 32) | w) % m);
}

// ruby_test.rb:52-61: the engine's offset of probe i.
template <uint32_t ENGINE>
__device__ __forceinline__ uint64_t engine_offset(const uint8_t* key, uint32_t L, uint32_t i, uint64_t m) {
    const Msg msg = make_msg(i, key, L);
    const uint32_t T = msg.P + L;
    const uint32_t nblk = (T + 8u) / 64u + 1u;
    uint32_t st[5];
    if constexpr (ENGINE == BF_ENGINE_MD5) {
        st[0] = 0x67452301u; st[1] = 0xefcdab89u; st[2] = 0x98badcfeu; st[3] = 0x10325476u;
    } else {
        st[0] = 0x67452301u; st[1] = 0xEFCDAB89u; st[2] = 0x98BADCFEu; st[3] = 0x10325476u; st[4] = 0xC3D2E1F0u;
    }
    for (uint32_t b = 0; b < nblk; ++b) {
        uint32_t w[16];
        const bool last = b + 1 == nblk;
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) {
            const uint32_t p = b * 64u + 4u * j;
            uint32_t x = msg_byte(msg, p) | (msg_byte(msg, p + 1) << 8) | (msg_byte(msg, p + 2) << 16) |
                         (msg_byte(msg, p + 3) << 24);
            if constexpr (ENGINE == BF_ENGINE_MD5) {
                if (last && j == 14) x = T << 3;     // bit length, little-endian 64-bit
                if (last && j == 15) x = T >> 29;
            } else {
                x = __builtin_bswap32(x);
                if (last && j == 14) x = T >> 29;    // bit length, big-endian 64-bit
                if (last && j == 15) x = T << 3;
            }
            w[j] = x;
        }
        if constexpr (ENGINE == BF_ENGINE_MD5) md5_compress(st, w);
        else sha1_compress(st, w);
    }
    // hexdigest.to_i(16): the digest bytes as one big-endian integer, most significant word first
    uint64_t r = 0;
    if constexpr (ENGINE == BF_ENGINE_MD5) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r = mod_step(r, __builtin_bswap32(st[j]), m);
    } else {
#pragma unroll
        for (int j = 0; j < 5; ++j) r = mod_step(r, st[j], m);
    }
    return r;
}

// One lane per (key, probe).  INDEXES: offsets out (key-major); INCLUDE: out8 preset to 1,
// a probe on a 0 bit clears its key's answer (ruby_test.rb:22-31); INSERT: test, then
// atomicOr for a 0 bit, any_new by ballot, dirty blocks marked, flipped bits listed when
// g.flips is set (ruby_test.rb:63-68).
template <uint32_t ENGINE, BfOp OP>
__global__ __launch_bounds__(kLanes) void engine_kernel(BfGeom g, const uint8_t* __restrict__ keys16,
                                                        const uint64_t* __restrict__ offsets, uint64_t bias,
                                                        uint64_t n, uint8_t* __restrict__ out8,
                                                        uint64_t* __restrict__ out64, uint32_t* any_flag) {
    const uint64_t t = (uint64_t)blockIdx.x * kLanes + threadIdx.x;
    const uint64_t total = n * g.k;
    bool fresh = false;
    if (t < total) {
        const uint64_t key = t / g.k;
        const uint32_t i = (uint32_t)(t - key * g.k);
        // a key whose offsets are inconsistent is hashed as the empty key (bfdev::key_ok)
        const bool ok = bfdev::key_ok(offsets[0], offsets[key], offsets[key + 1], offsets[n],
                                      i == 0 ? g.key_status : nullptr);
        const uint64_t s = ok ? offsets[key] + bias : bias + offsets[0];
        const uint32_t L = ok ? (uint32_t)(offsets[key + 1] - offsets[key]) : 0u;
        const uint64_t o = engine_offset<ENGINE>(keys16 + s, L, i, g.m);
        const uint64_t w = o >> 5;
        const uint32_t mask = 1u << ((uint32_t)(o ^ 7u) & 31u);
        if constexpr (OP == BF_OP_INDEXES) {
            out64[t] = o;
        } else if constexpr (OP == BF_OP_INCLUDE) {
            if (!(g.bits[w] & mask)) out8[key] = 0;
        } else {
            if (!(g.bits[w] & mask)) {
                if (g.dirty) g.dirty[w >> (kDirtyShiftBits - 5)] = 1;
                fresh = !(atomicOr(g.bits + w, mask) & mask);
                if (fresh && g.flips) {   // bf_insert_many_changes: this lane flipped it
                    const unsigned long long at = atomicAdd(g.flip_count, 1ull);
                    if (at < g.flip_cap) g.flips[at] = o | g.flip_tag;
                }
            }
        }
    }
    if constexpr (OP == BF_OP_INSERT) {
        if (any_flag) bfdev::report_any_new(any_flag, fresh);
    }
}

template <uint32_t ENGINE>
hipError_t launch(BfOp op, const BfGeom& g, const uint8_t* k16, const uint64_t* offsets, uint64_t bias, uint64_t n,
                  uint8_t* out8, uint64_t* out64, uint32_t* flag, hipStream_t s) {
    const uint64_t blocks = (n * g.k + kLanes - 1) / kLanes;
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;   // the host chunks far below this
    switch (op) {
        case BF_OP_INDEXES:
            engine_kernel<ENGINE, BF_OP_INDEXES><<<blocks, kLanes, 0, s>>>(g, k16, offsets, bias, n, out8, out64, flag);
            break;
        case BF_OP_INCLUDE: {
            hipError_t e = hipMemsetAsync(out8, 1, n, s);
            if (e != hipSuccess) return e;
            engine_kernel<ENGINE, BF_OP_INCLUDE><<<blocks, kLanes, 0, s>>>(g, k16, offsets, bias, n, out8, out64, flag);
            break;
        }
        case BF_OP_INSERT:
            engine_kernel<ENGINE, BF_OP_INSERT><<<blocks, kLanes, 0, s>>>(g, k16, offsets, bias, n, out8, out64, flag);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t bf_launch_engine(uint32_t engine, BfOp op, const BfGeom& g, const uint8_t* k16, const uint64_t* offsets,
                            uint64_t bias, uint64_t n, uint8_t* out8, uint64_t* out64, uint32_t* flag, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (engine == BF_ENGINE_MD5) return launch<BF_ENGINE_MD5>(op, g, k16, offsets, bias, n, out8, out64, flag, s);
    if (engine == BF_ENGINE_SHA1) return launch<BF_ENGINE_SHA1>(op, g, k16, offsets, bias, n, out8, out64, flag, s);
    return hipErrorInvalidValue;
}
