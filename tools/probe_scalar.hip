// Microbenchmark: random 4-byte probes of a 1.2 GB bitset through the SCALAR load path
// (s_load from wave-uniform addresses: the scalar cache fills its own lines from L2) against
// plain vector loads.  tools/probe_granularity.hip found that every vector-load form leaves L2
// as one 128-B request per probe (~55 G probes/s); this asks whether the scalar path's
// requests are smaller or more numerous.  Reads only: no stores of any kind through the
// scalar path.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_scalar tools/probe_scalar.hip
//   ./tools/probe_scalar
//   rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
//       --kernel-trace -d <dir> -o run -- ./tools/probe_scalar
//
// Every index is < the buffer's word count by construction (a multiply-shift of a 32-bit
// hash onto [0, words)); each lane stores one word of output with a vector store.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHK(x)                                                                                  \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t word_of(uint64_t p, uint32_t seed, uint64_t words) {
    return (uint32_t)(((uint64_t)mix32((uint32_t)p * 2654435761u + seed) * words) >> 32);
}

// Vector baseline: U independent probes per lane in flight.
__global__ __launch_bounds__(256) void probe_vec(const uint32_t* __restrict__ bits, uint64_t words, uint64_t probes,
                                                 uint32_t seed, uint32_t* __restrict__ out) {
    constexpr int U = 8;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t p0 = tid; p0 < probes; p0 += U * stride) {
        uint32_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t p = p0 + u * stride;
            v[u] = p < probes ? bits[word_of(p, seed, words)] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
    }
    out[tid] = acc;
}

// Scalar path: each wave takes its lanes' probe words one lane at a time (readlane makes the
// address wave-uniform, so the load is an s_load), B loads in flight per wave.
template <int B>
__global__ __launch_bounds__(256) void probe_scalar(const uint32_t* __restrict__ bits, uint64_t words,
                                                    uint64_t probes, uint32_t seed, uint32_t* __restrict__ out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t acc = 0;
    for (uint64_t p0 = tid - lane; p0 < probes; p0 += stride) {   // wave-uniform loop
        const uint64_t p = p0 + lane;
        const uint32_t w = p < probes ? word_of(p, seed, words) : 0u;
        uint32_t mine = 0;
#pragma unroll
        for (int j0 = 0; j0 < 64; j0 += B) {
            uint32_t s[B];
#pragma unroll
            for (int j = 0; j < B; ++j) {
                const uint32_t wj = __builtin_amdgcn_readlane(w, j0 + j);
                s[j] = bits[wj];
            }
#pragma unroll
            for (int j = 0; j < B; ++j) mine = lane == (uint32_t)(j0 + j) ? s[j] : mine;
        }
        acc ^= mine;
    }
    out[tid] = acc;
}


// Mixed: waves pull 1024-probe chunks from a global counter; wave w takes the scalar path
// when (w & 3) < S, the vector path otherwise, so the launch time reflects the two paths'
// combined throughput (are 64-B scalar fills additive to the 128-B vector fills?).
template <int S>
__global__ __launch_bounds__(256) void probe_mixed(const uint32_t* __restrict__ bits, uint64_t words,
                                                   uint64_t probes, uint32_t seed, uint32_t* __restrict__ out,
                                                   unsigned long long* __restrict__ counter) {
    constexpr uint32_t kChunk = 1024;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const bool scalar = (int)(wave & 3u) < S;
    uint32_t acc = 0;
    for (;;) {
        unsigned long long c = 0;
        if (lane == 0) c = atomicAdd(counter, 1ull);
        c = __shfl(c, 0);
        const uint64_t p0 = c * kChunk;
        if (p0 >= probes) break;
        if (scalar) {
            for (uint32_t r = 0; r < kChunk / 64; ++r) {
                const uint64_t p = p0 + r * 64 + lane;
                const uint32_t w = p < probes ? word_of(p, seed, words) : 0u;
                uint32_t mine = 0;
#pragma unroll
                for (int j0 = 0; j0 < 64; j0 += 16) {
                    uint32_t s[16];
#pragma unroll
                    for (int j = 0; j < 16; ++j) s[j] = bits[__builtin_amdgcn_readlane(w, j0 + j)];
#pragma unroll
                    for (int j = 0; j < 16; ++j) mine = lane == (uint32_t)(j0 + j) ? s[j] : mine;
                }
                acc ^= mine;
            }
        } else {
            uint32_t v[kChunk / 64];
#pragma unroll
            for (uint32_t r = 0; r < kChunk / 64; ++r) {
                const uint64_t p = p0 + r * 64 + lane;
                v[r] = p < probes ? bits[word_of(p, seed, words)] : 0u;
            }
#pragma unroll
            for (uint32_t r = 0; r < kChunk / 64; ++r) acc ^= v[r];
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <typename K>
static float run_mixed(K kern, const uint32_t* d, uint64_t words, uint64_t probes, uint32_t* out,
                       unsigned long long* counter, hipStream_t s, int reps) {
    const dim3 grid(256 * 8), block(256);
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    CHK(hipMemsetAsync(counter, 0, 8, s));
    hipLaunchKernelGGL(kern, grid, block, 0, s, d, words, probes, 1u, out, counter);
    float total = 0;
    for (int r = 0; r < reps; ++r) {
        CHK(hipMemsetAsync(counter, 0, 8, s));
        CHK(hipEventRecord(a, s));
        hipLaunchKernelGGL(kern, grid, block, 0, s, d, words, probes, 2u + r, out, counter);
        CHK(hipEventRecord(b, s));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        total += ms;
    }
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return total / reps;
}

template <typename K>
static float run(K kern, const uint32_t* d, uint64_t words, uint64_t probes, uint32_t* out, hipStream_t s, int reps) {
    const dim3 grid(2048 * 4), block(256);
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipLaunchKernelGGL(kern, grid, block, 0, s, d, words, probes, 1u, out);
    CHK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, grid, block, 0, s, d, words, probes, 2u + r, out);
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return ms / reps;
}

int main() {
    const uint64_t bytes = 1198132288ull;   // the north-star filter's bitset
    const uint64_t words = bytes / 4;
    const uint64_t probes = 1ull << 27;
    const int reps = 5;
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    uint32_t* out = nullptr;
    CHK(hipMalloc(&out, (size_t)2048 * 4 * 256 * 4));
    uint32_t* d = nullptr;
    CHK(hipMalloc(&d, bytes));
    CHK(hipMemsetAsync(d, 0x5A, bytes, s));
    CHK(hipStreamSynchronize(s));
    unsigned long long* counter = nullptr;
    CHK(hipMalloc(&counter, 8));
    struct V { const char* name; float ms; } v[] = {
        {"vector", run(probe_vec, d, words, probes, out, s, reps)},
        {"scalar_b8", run(probe_scalar<8>, d, words, probes, out, s, reps)},
        {"scalar_b16", run(probe_scalar<16>, d, words, probes, out, s, reps)},
        {"scalar_b32", run(probe_scalar<32>, d, words, probes, out, s, reps)},
        {"mixed_s0of4", run_mixed(probe_mixed<0>, d, words, probes, out, counter, s, reps)},
        {"mixed_s1of4", run_mixed(probe_mixed<1>, d, words, probes, out, counter, s, reps)},
        {"mixed_s2of4", run_mixed(probe_mixed<2>, d, words, probes, out, counter, s, reps)},
        {"mixed_s3of4", run_mixed(probe_mixed<3>, d, words, probes, out, counter, s, reps)},
        {"mixed_s4of4", run_mixed(probe_mixed<4>, d, words, probes, out, counter, s, reps)},
    };
    for (const V& x : v)
        std::printf("{\"variant\": \"%s\", \"ms\": %.4f, \"Gprobes_per_s\": %.2f}\n", x.name, x.ms,
                    probes / (x.ms * 1e6));
    CHK(hipFree(d));
    CHK(hipFree(counter));
    CHK(hipFree(out));
    CHK(hipStreamDestroy(s));
    return 0;
}
