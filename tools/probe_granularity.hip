// Microbenchmark: random 4-byte probes of a 1.2 GB bitset (the north-star filter's size),
// by memory type and per-load cache policy, to see which forms leave L2 as requests smaller
// than a 128-B line fill.  The include? kernel is bound by those fills (~4.3 per key at 50 %
// members), so a smaller request per probe is the lever left on it.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_granularity tools/probe_granularity.hip
//   ./tools/probe_granularity             (prints one line per variant)
//   ./tools/probe_granularity sweep       (working-set sweep only, up to 6.98 GB)
//   rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
//       --kernel-trace -d <dir> -o run -- ./tools/probe_granularity
//
// Every index is < the buffer's word count by construction (a multiply-shift of a 32-bit
// hash onto [0, words)); each lane stores one word of output (vector store).
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

// POLICY: 0 plain global load, 1 nontemporal builtin, 2+ raw buffer load with cache-policy
// aux = POLICY - 2 (gfx950: sc0 = 1, nt = 2, sc1 = 16)
template <int POLICY>
__global__ __launch_bounds__(256) void probe_kernel(const uint32_t* __restrict__ bits, uint64_t words,
                                                    uint64_t probes, uint32_t seed, uint32_t* __restrict__ out) {
    constexpr int U = 8;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(bits), (short)0, 0x7FFFFFFF, 0x00020000);
    for (uint64_t p0 = tid; p0 < probes; p0 += U * stride) {
        uint32_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t p = p0 + u * stride;
            v[u] = 0;
            if (p < probes) {
                const uint64_t w = ((uint64_t)mix32((uint32_t)p * 2654435761u + seed) * words) >> 32;
                if constexpr (POLICY == 0) v[u] = bits[w];
                else if constexpr (POLICY == 1) v[u] = __builtin_nontemporal_load(bits + w);
                else {
                    // the 1.2 GB buffer fits the descriptor's 2^31-byte range: a 32-bit voffset
                    v[u] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (uint32_t)(w * 4u), 0, POLICY - 2);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
    }
    out[tid] = acc;
}

template <int POLICY>
static float run(const uint32_t* d, uint64_t words, uint64_t probes, uint32_t* out, hipStream_t s, int reps) {
    const dim3 grid(2048 * 4), block(256);
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipLaunchKernelGGL(probe_kernel<POLICY>, grid, block, 0, s, d, words, probes, 1u, out);
    CHK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(probe_kernel<POLICY>, grid, block, 0, s, d, words, probes, 2u + r, out);
    CHK(hipEventRecord(b, s));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char** argv) {
    // "sweep": only the working-set sweep, extended past the north-star filter to the
    // reach-capped 10B / 200B bitsets (6.98 GB)
    const bool sweep_only = argc > 1 && argv[1][0] == 's';
    const uint64_t bytes = 1198132288ull;   // 9585058377 bits rounded up to 64 B (the north-star filter)
    const uint64_t words = bytes / 4;
    const uint64_t probes = 1ull << 27;      // 134M random 4-B probes per launch
    const int reps = 5;
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    uint32_t* out = nullptr;
    CHK(hipMalloc(&out, (size_t)2048 * 4 * 256 * 4));
    struct Mem { const char* name; unsigned flags; bool ext; } mems[] = {
        {"hipMalloc", 0, false},
        {"uncached", hipDeviceMallocUncached, true},
        {"finegrained", hipDeviceMallocFinegrained, true},
    };
    for (const Mem& m : mems) {
        if (sweep_only) break;
        uint32_t* d = nullptr;
        if (m.ext) {
            if (hipExtMallocWithFlags(reinterpret_cast<void**>(&d), bytes, m.flags) != hipSuccess) {
                std::printf("{\"mem\": \"%s\", \"error\": \"alloc failed\"}\n", m.name);
                (void)hipGetLastError();
                continue;
            }
        } else {
            CHK(hipMalloc(&d, bytes));
        }
        CHK(hipMemsetAsync(d, 0x5A, bytes, s));
        CHK(hipStreamSynchronize(s));
        const char* pol[] = {"plain", "nontemporal", "buf", "buf_sc0", "buf_nt", "buf_sc0_nt",
                             "buf_sc1", "buf_sc0_sc1", "buf_sc1_nt", "buf_sc0_sc1_nt"};
        float ms[10];
        ms[0] = run<0>(d, words, probes, out, s, reps);
        ms[1] = run<1>(d, words, probes, out, s, reps);
        ms[2] = run<2 + 0>(d, words, probes, out, s, reps);
        ms[3] = run<2 + 1>(d, words, probes, out, s, reps);
        ms[4] = run<2 + 2>(d, words, probes, out, s, reps);
        ms[5] = run<2 + 3>(d, words, probes, out, s, reps);
        ms[6] = run<2 + 16>(d, words, probes, out, s, reps);
        ms[7] = run<2 + 17>(d, words, probes, out, s, reps);
        ms[8] = run<2 + 18>(d, words, probes, out, s, reps);
        ms[9] = run<2 + 19>(d, words, probes, out, s, reps);
        for (int i = 0; i < 10; ++i)
            std::printf("{\"mem\": \"%s\", \"policy\": \"%s\", \"ms\": %.4f, \"Gprobes_per_s\": %.2f, "
                        "\"TBps_if_128B\": %.3f}\n",
                        m.name, pol[i], ms[i], probes / (ms[i] * 1e6), probes * 128.0 / (ms[i] * 1e9));
        std::fflush(stdout);
        CHK(hipFree(d));
    }
    // working-set sweep (plain loads, hipMalloc): L2 (4 MiB per XCD), Infinity Cache
    // (256 MiB), past it
    for (uint64_t mb : {2ull, 16ull, 64ull, 128ull, 192ull, 256ull, 384ull, 600ull, 1143ull, 2400ull, 4800ull, 6656ull}) {
        if (!sweep_only && mb > 1143ull) break;
        const uint64_t b = mb << 20;
        uint32_t* d = nullptr;
        CHK(hipMalloc(&d, b));
        CHK(hipMemsetAsync(d, 0x5A, b, s));
        const float ms = run<0>(d, b / 4, probes, out, s, reps);
        std::printf("{\"mem\": \"hipMalloc\", \"working_set_MiB\": %llu, \"ms\": %.4f, \"Gprobes_per_s\": %.2f}\n",
                    (unsigned long long)mb, ms, probes / (ms * 1e6));
        std::fflush(stdout);
        CHK(hipFree(d));
    }
    CHK(hipFree(out));
    CHK(hipStreamDestroy(s));
    return 0;
}
