// bf_internal.h — shared between the kernels (bf_kernels.hip) and the C ABI (bf_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Filter geometry as the kernels see it.
struct BfGeom {
    uint32_t* bits;    // device bitset, Redis byte order viewed as LE 32-bit words
    uint64_t  m;       // modulus (options[:bits], lib/redis/bloomfilter.rb:27)
    double    inv_m;   // 1.0 / m, for the division-free modulo
    uint32_t  k;       // hashes per key (options[:hashes], bloomfilter.rb:28)
    uint32_t  nomod;   // 1 iff m > k*(2^32-1): every derived offset is already < m
};

enum BfOp : int {
    BF_OP_INDEXES      = 0,  // write the k offsets of each key (ruby.rb:41-55)
    BF_OP_INCLUDE      = 1,  // AND of the k bits (ruby.rb:20-30)
    BF_OP_INSERT       = 2,  // OR the k bits in, no per-key result (ruby.rb:57-60)
    BF_OP_INSERT_FLAGS = 3,  // ... and report which keys / whether any bit flipped (ruby.rb:61-62)
};

// Keys: byte j of the packed buffer for offset o is keys16[o + bias - 0] where
// keys16 is 16-byte aligned and readable up to the next 16-byte boundary past
// the last key byte.  (bias is added modulo 2^64.)
hipError_t bf_launch_keys(BfOp op, const BfGeom& g, const uint8_t* keys16, const uint64_t* offsets,
                          uint64_t bias, uint64_t n, uint8_t* out8, uint64_t* out64,
                          uint32_t* any_flag, hipStream_t s);

// *d_last = 1 + index of the last nonzero 32-bit word in words[0, nwords) (0 if none).
// d_last must be zeroed before the launch.  nwords must be a multiple of 4.
hipError_t bf_launch_last_nonzero(const uint32_t* words, uint64_t nwords,
                                  unsigned long long* d_last, hipStream_t s);

// dst[i] |= src[i] for i < nwords (nwords multiple of 4, both 16-byte aligned).
hipError_t bf_launch_or(uint32_t* dst, const uint32_t* src, uint64_t nwords, hipStream_t s);
