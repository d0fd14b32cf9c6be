/*
 * bf_oracle.c — CPU restatement of the reference ruby driver (see bf_oracle.h).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the HIP path and the timed
 * CPU baseline ("port") of bench.py.  Never linked by the product.
 */
#include "bf_oracle.h"

#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------- SHA-1 --
 * FIPS 180-4 §6.1, written from the standard (not from any reference file:
 * the reference calls Ruby's Digest::SHA1, ruby.rb:42). */
static uint32_t rol32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void sha1_compress(uint32_t h[5], const uint8_t blk[64]) {
    uint32_t w[80];
    for (int t = 0; t < 16; ++t)
        w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) |
               ((uint32_t)blk[4 * t + 2] << 8) | (uint32_t)blk[4 * t + 3];
    for (int t = 16; t < 80; ++t) w[t] = rol32(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int t = 0; t < 80; ++t) {
        uint32_t f, kk;
        if (t < 20) { f = (b & c) | (~b & d); kk = 0x5A827999u; }
        else if (t < 40) { f = b ^ c ^ d; kk = 0x6ED9EBA1u; }
        else if (t < 60) { f = (b & c) | (b & d) | (c & d); kk = 0x8F1BBCDCu; }
        else { f = b ^ c ^ d; kk = 0xCA62C1D6u; }
        uint32_t tmp = rol32(a, 5) + f + e + kk + w[t];
        e = d; d = c; c = rol32(b, 30); b = a; a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

static void sha1_words(const uint8_t* msg, uint64_t len, uint32_t h[5]) {
    h[0] = 0x67452301u; h[1] = 0xEFCDAB89u; h[2] = 0x98BADCFEu; h[3] = 0x10325476u; h[4] = 0xC3D2E1F0u;
    uint64_t full = len / 64;
    for (uint64_t b = 0; b < full; ++b) sha1_compress(h, msg + 64 * b);
    uint8_t tail[128];
    uint64_t rem = len - 64 * full;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, msg + 64 * full, (size_t)rem);
    tail[rem] = 0x80;
    uint64_t tl = (rem + 1 + 8 <= 64) ? 64 : 128;
    uint64_t bitlen = len * 8u;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bitlen >> (8 * i));
    sha1_compress(h, tail);
    if (tl == 128) sha1_compress(h, tail + 64);
}

void bfo_sha1(const uint8_t* msg, uint64_t len, uint8_t out[20]) {
    uint32_t h[5];
    sha1_words(msg, len, h);
    for (int i = 0; i < 5; ++i) {
        out[4 * i] = (uint8_t)(h[i] >> 24); out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8); out[4 * i + 3] = (uint8_t)h[i];
    }
}

/* --------------------------------------------------------------- sizing --
 * bloomfilter.rb:50-52:  (-1 * n * Math.log(p) / (Math.log(2)**2)).round
 * Evaluated left to right in IEEE double; `**2` is pow(x, 2); Float#round is
 * round-half-away-from-zero == C round(). */
int64_t bfo_optimal_m(double n, double p) {
    double v = (-1.0 * n) * log(p) / pow(log(2.0), 2.0);
    return (int64_t)round(v);
}

/* bloomfilter.rb:54-58:  h = (Math.log(2) * (bf_size / num_of_elements)).round; h += 1 if h.zero?
 * With Integer n, bf_size / n is Integer floor division (Ruby floors toward -inf). */
static int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}
int64_t bfo_optimal_k_int(int64_t n, int64_t m) {
    int64_t h = (int64_t)round(log(2.0) * (double)floordiv(m, n));
    if (h == 0) h += 1;
    return h;
}
int64_t bfo_optimal_k_float(double n, int64_t m) {
    int64_t h = (int64_t)round(log(2.0) * ((double)m / n));
    if (h == 0) h += 1;
    return h;
}

/* ------------------------------------------------------------- indexes --
 * ruby.rb:41-55.  h[j] = sha[8j, 8].to_i(16) is the j-th big-endian digest
 * word H_j.  idx_i = (h[i % 2] + i * h[2 + (((i + (i % 2)) % 4) / 2)]) % bits.
 * The value is < k * 2^32, so uint64 arithmetic is exact. */
void bfo_indexes(const uint8_t* key, uint64_t len, uint64_t m, uint32_t k, uint64_t* out) {
    uint32_t h[5];
    sha1_words(key, len, h);
    for (uint32_t i = 0; i < k; ++i) {
        uint64_t a = h[i % 2];
        uint64_t b = h[2 + (((i + (i % 2)) % 4) / 2)];
        out[i] = (a + (uint64_t)i * b) % m;
    }
}

void bfo_indexes_many(const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint64_t m, uint32_t k,
                      uint64_t* out) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static, 1024)
#endif
    for (int64_t j = 0; j < (int64_t)n; ++j)
        bfo_indexes(keys + offsets[j], offsets[j + 1] - offsets[j], m, k, out + (uint64_t)j * k);
}

uint64_t bfo_reach_bits(uint64_t m, uint32_t k) {
    uint64_t reach = (uint64_t)k * 0xFFFFFFFFull + 1ull;
    return m < reach ? m : reach;
}

/* ------------------------------------------------------ bitset (Redis) -- */
static inline int getbit(const uint8_t* bits, uint64_t o) { return (bits[o >> 3] >> (7 - (o & 7))) & 1; }

/* ruby.rb:57-63 sequential semantics: k SETBITs per key in key order;
 * a key is "new" (found == false) iff some SETBIT returned 0. */
void bfo_insert_many(uint8_t* bits, uint64_t m, uint32_t k, const uint8_t* keys,
                     const uint64_t* offsets, uint64_t n, uint8_t* per_key_new, uint8_t* any_new) {
    uint64_t idx[256];
    uint8_t any = 0;
    for (uint64_t j = 0; j < n; ++j) {
        bfo_indexes(keys + offsets[j], offsets[j + 1] - offsets[j], m, k, idx);
        uint8_t isnew = 0;
        for (uint32_t i = 0; i < k; ++i) {
            uint64_t o = idx[i];
            uint8_t mask = (uint8_t)(0x80u >> (o & 7));
            if (!(bits[o >> 3] & mask)) isnew = 1;
            bits[o >> 3] |= mask;
        }
        if (per_key_new) per_key_new[j] = isnew;
        any |= isnew;
    }
    if (any_new) *any_new = any;
}

/* ruby.rb:20-30: true iff none of the k GETBITs is 0 (the early exit changes latency only). */
void bfo_include_many(const uint8_t* bits, uint64_t m, uint32_t k, const uint8_t* keys,
                      const uint64_t* offsets, uint64_t n, uint8_t* out) {
    uint64_t idx[256];
    for (uint64_t j = 0; j < n; ++j) {
        bfo_indexes(keys + offsets[j], offsets[j + 1] - offsets[j], m, k, idx);
        uint8_t r = 1;
        for (uint32_t i = 0; i < k && r; ++i) r = (uint8_t)getbit(bits, idx[i]);
        out[j] = r;
    }
}

void bfo_insert_many_omp(uint8_t* bits, uint64_t m, uint32_t k, const uint8_t* keys,
                         const uint64_t* offsets, uint64_t n, int threads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static, 4096) num_threads(threads)
#endif
    for (int64_t j = 0; j < (int64_t)n; ++j) {
        uint64_t idx[256];
        bfo_indexes(keys + offsets[j], offsets[j + 1] - offsets[j], m, k, idx);
        for (uint32_t i = 0; i < k; ++i) {
            uint64_t o = idx[i];
            __atomic_fetch_or(&bits[o >> 3], (uint8_t)(0x80u >> (o & 7)), __ATOMIC_RELAXED);
        }
    }
    (void)threads;
}

void bfo_include_many_omp(const uint8_t* bits, uint64_t m, uint32_t k, const uint8_t* keys,
                          const uint64_t* offsets, uint64_t n, uint8_t* out, int threads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static, 4096) num_threads(threads)
#endif
    for (int64_t j = 0; j < (int64_t)n; ++j) {
        uint64_t idx[256];
        bfo_indexes(keys + offsets[j], offsets[j + 1] - offsets[j], m, k, idx);
        uint8_t r = 1;
        for (uint32_t i = 0; i < k && r; ++i) r = (uint8_t)getbit(bits, idx[i]);
        out[j] = r;
    }
    (void)threads;
}

uint64_t bfo_redis_len(const uint8_t* bits, uint64_t nbytes) {
    while (nbytes > 0 && bits[nbytes - 1] == 0) --nbytes;
    return nbytes;
}

int bfo_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
