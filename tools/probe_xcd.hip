// Microbenchmark: random 4-byte probes confined, per XCD, to one window of the bitset at a
// time (XCD-local superbins), against probes spread over the whole 1.2 GB bitset.
//
// A partitioned owner receives its probes already sorted by superbin (bf_route_chunks_dev).
// If every workgroup of one XCD probes the same superbin at once and that superbin fits the
// XCD's 4 MiB L2, the probes become L2 hits instead of fabric requests (~55 G/s).  This
// measures the rate of that access pattern for window sizes 0.5-16 MiB.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_xcd tools/probe_xcd.hip && ./tools/probe_xcd
//
// Persistent grid: 8 groups (blockIdx % 8: blocks that share an XCD) x G workgroups; group x
// walks windows x, x + 8, x + 16, ... (one window per step, all its workgroups together), each
// workgroup taking its share of the window's probes.  Every index is < the buffer's word count
// by construction; each lane stores one word of output (vector store).
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

constexpr int kLanes = 256;

// win_words == 0: every probe anywhere in [0, words) (the unsorted baseline)
__global__ __launch_bounds__(kLanes) void probe_xcd_kernel(const uint32_t* __restrict__ bits, uint64_t words,
                                                           uint64_t win_words, uint64_t per_window, uint32_t G,
                                                           uint32_t seed, uint32_t* __restrict__ out) {
    constexpr int U = 8;
    const uint32_t grp = blockIdx.x % 8u, mem = blockIdx.x / 8u;
    const uint64_t nwin = win_words ? words / win_words : 1;
    uint32_t acc = 0;
    const uint64_t share = per_window / G;   // probes of this workgroup per window
    for (uint64_t w = grp; w < nwin; w += 8) {
        const uint64_t base = win_words ? w * win_words : 0;
        const uint64_t span = win_words ? win_words : words;
        for (uint64_t p0 = threadIdx.x; p0 < share; p0 += U * kLanes) {
            uint32_t v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t p = p0 + u * kLanes;
                v[u] = 0;
                if (p < share) {
                    const uint32_t h = mix32((uint32_t)(w * 7919u + mem * 104729u + p) * 2654435761u + seed);
                    v[u] = bits[base + (((uint64_t)h * span) >> 32)];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc ^= v[u];
        }
    }
    out[(uint64_t)blockIdx.x * kLanes + threadIdx.x] = acc;
}

int main() {
    const uint64_t bytes = 1198132224ull;   // the north-star bitset (9,585,058,377 bits, 1.2 GB)
    const uint64_t words = bytes / 4;
    uint32_t *d, *out;
    CHK(hipMalloc(&d, bytes));
    CHK(hipMemset(d, 0x5A, bytes));
    const uint32_t G = 64;   // workgroups per XCD group (256 CUs x 2 per CU / 8)
    CHK(hipMalloc(&out, (uint64_t)8 * G * kLanes * 4));
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const uint64_t total = 100ull << 20;   // ~ the probes one P = 8 owner tests per step
    const uint64_t wins_kib[] = {0, 512, 1024, 2048, 4096, 8192, 16384, 65536};
    for (uint64_t kib : wins_kib) {
        const uint64_t ww = kib * 256;   // words per window
        const uint64_t nwin = ww ? words / ww : 1;
        const uint64_t per_window = (total / nwin / G) * G;
        const uint64_t probes = per_window * nwin;
        hipLaunchKernelGGL(probe_xcd_kernel, dim3(8 * G), dim3(kLanes), 0, s, d, words, ww, per_window, G, 1u, out);
        CHK(hipEventRecord(a, s));
        const int reps = 5;
        for (int r = 0; r < reps; ++r)
            hipLaunchKernelGGL(probe_xcd_kernel, dim3(8 * G), dim3(kLanes), 0, s, d, words, ww, per_window, G,
                               2u + r, out);
        CHK(hipEventRecord(b, s));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        std::printf("{\"window_kib\": %llu, \"windows\": %llu, \"probes\": %llu, \"ms\": %.4f, \"gprobes_per_s\": %.2f}\n",
                    (unsigned long long)kib, (unsigned long long)nwin, (unsigned long long)probes, ms,
                    probes / (ms * 1e6));
    }
    CHK(hipFree(d));
    CHK(hipFree(out));
    return 0;
}
