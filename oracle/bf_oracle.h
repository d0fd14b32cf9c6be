/*
 * bf_oracle.h — CPU restatement of the reference ruby driver's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or as the timed CPU baseline).  The product (libbfhip.so and the Python
 * package redis-bloomfilter_amd/) never links, imports or falls back to it.
 *
 * Restates (paths relative to the reference repository):
 *   lib/redis/bloomfilter.rb:50-52  optimal_m  (Ruby Float#round semantics)
 *   lib/redis/bloomfilter.rb:54-58  optimal_k  (Integer floor division, 0 -> 1)
 *   lib/bloomfilter_driver/ruby.rb:41-55  indexes_for (SHA-1, 4 BE words, double hashing)
 *   lib/bloomfilter_driver/ruby.rb:57-63  set  (k x SETBIT, found / EXPIRE decision)
 *   lib/bloomfilter_driver/ruby.rb:20-30  include? (AND of k GETBITs)
 *   Redis SETBIT/GETBIT bit order (external server): offset o -> byte o>>3,
 *   mask 0x80 >> (o & 7); string length = max set offset / 8 + 1.
 *
 * SHA-1 is FIPS 180-4 (the reference gets it from Ruby stdlib digest/sha1,
 * ruby.rb:3,42; version unpinned). Pinned here by the FIPS known answers and
 * by golden vectors from Python hashlib (tests/golden/).
 */
#ifndef BF_ORACLE_H
#define BF_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

void     bfo_sha1(const uint8_t* msg, uint64_t len, uint8_t out[20]);
int64_t  bfo_optimal_m(double n, double p);                 /* bloomfilter.rb:50-52 */
int64_t  bfo_optimal_k_int(int64_t n, int64_t m);           /* bloomfilter.rb:54-58, Integer n */
int64_t  bfo_optimal_k_float(double n, int64_t m);          /* Float n: float division */
void     bfo_indexes(const uint8_t* key, uint64_t len, uint64_t m, uint32_t k, uint64_t* out);
void     bfo_indexes_many(const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint64_t m,
                          uint32_t k, uint64_t* out);
uint64_t bfo_reach_bits(uint64_t m, uint32_t k);            /* min(m, k*(2^32-1)+1) */

/* Host bitset in Redis byte order.  `bits` must hold ceil(reach/8) bytes. */
void     bfo_insert_many(uint8_t* bits, uint64_t m, uint32_t k,
                         const uint8_t* keys, const uint64_t* offsets, uint64_t n,
                         uint8_t* per_key_new /* nullable, sequential semantics */,
                         uint8_t* any_new /* nullable */);
void     bfo_include_many(const uint8_t* bits, uint64_t m, uint32_t k,
                          const uint8_t* keys, const uint64_t* offsets, uint64_t n,
                          uint8_t* out);
/* OpenMP versions (the strong CPU baseline); insert uses atomic byte OR. */
void     bfo_insert_many_omp(uint8_t* bits, uint64_t m, uint32_t k,
                             const uint8_t* keys, const uint64_t* offsets, uint64_t n,
                             int threads);
void     bfo_include_many_omp(const uint8_t* bits, uint64_t m, uint32_t k,
                              const uint8_t* keys, const uint64_t* offsets, uint64_t n,
                              uint8_t* out, int threads);
/* Length of the Redis string holding `bits` (trailing zero bytes trimmed). */
uint64_t bfo_redis_len(const uint8_t* bits, uint64_t nbytes);
int      bfo_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif
