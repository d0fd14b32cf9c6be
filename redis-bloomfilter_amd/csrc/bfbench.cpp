// bfbench — the C++ bench binary of SURVEY §8(b)'s "Callers": drives libbfhip.so through its C
// ABI alone (include/bfhip.h; no Python, no torch), so the engine's numbers can be taken, and
// profiled with rocprofv3, from native code.
//
//   bfbench [--config nstar|100m|10b|200b|1m|1m_big] [--steps K] [--warmup W] [--pipeline 0|1]
//           [--host] [--version]
//
// Workload = bench.py's: the filter of BASELINE's config (bf_optimal_m / bf_optimal_k), its
// reachable prefix prefilled to 50 % random bit density (bf_import_redis), and per step one
// insert batch of `batch` fresh decimal-string keys (uniform ints in [0, n)) plus one include?
// batch of half that step's keys and half non-members (ints in [n, 2n)).  Keys are built on the
// host and copied to the device before the timed region (4 distinct batch pairs, cycled).
// Timed with HIP events around the steps on one stream; --pipeline 1 runs the digest pipeline
// (bf_insert_digests_dev + bf_include_hash_dev).  --host also times the host-pointer calls
// (PCIe included).  Prints one JSON line; exits 1 on any error or false negative.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "bfhip.h"

namespace {

#define HCHK(x)                                                                                  \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::fprintf(stderr, "bfbench: %s: %s\n", #x, hipGetErrorString(e_));                \
            std::exit(1);                                                                        \
        }                                                                                        \
    } while (0)

void bf_ok(int rc, bf_handle* h, const char* what) {
    if (rc != BF_OK) {
        std::fprintf(stderr, "bfbench: %s: status %d: %s\n", what, rc, bf_last_error(h));
        std::exit(1);
    }
}

struct Config {
    const char* name;
    double n;
    double p;
    uint64_t batch;
};

const Config kConfigs[] = {
    {"nstar", 1e9, 0.01, 1ull << 24},   {"100m", 1e8, 0.001, 1ull << 24},
    {"10b", 1e10, 0.0001, 1ull << 24},  {"200b", 2e11, 0.0001, 1ull << 24},
    {"1m", 1e6, 0.01, 1ull << 20},      {"1m_big", 1e6, 0.01, 1ull << 24},
};

uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Runs f(lo, hi) over [0, n) on the host's threads.
template <typename F>
void par_for(uint64_t n, F&& f) {
    unsigned t = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (unsigned i = 0; i < t; ++i)
        th.emplace_back([&, i] { f(n * i / t, n * (i + 1) / t); });
    for (auto& x : th) x.join();
}

// Packed decimal strings of vals[j] (the `data.to_s` of an Integer), n+1 offsets, 16 B slack.
void pack_decimal(const std::vector<uint64_t>& vals, std::vector<uint8_t>& bytes, std::vector<uint64_t>& offs) {
    const uint64_t n = vals.size();
    std::vector<uint8_t> len(n);
    par_for(n, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t j = lo; j < hi; ++j) {
            uint64_t v = vals[j];
            uint8_t l = 1;
            while (v >= 10) { v /= 10; ++l; }
            len[j] = l;
        }
    });
    offs.assign(n + 1, 0);
    for (uint64_t j = 0; j < n; ++j) offs[j + 1] = offs[j] + len[j];
    bytes.assign(offs[n] + 16, 0);
    par_for(n, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t j = lo; j < hi; ++j) {
            uint64_t v = vals[j];
            for (int i = len[j] - 1; i >= 0; --i) {
                bytes[offs[j] + i] = (uint8_t)('0' + v % 10);
                v /= 10;
            }
        }
    });
}

struct DevBatch {
    uint8_t* keys = nullptr;
    uint64_t* offs = nullptr;
    uint64_t n = 0;
    std::vector<uint8_t> hkeys;
    std::vector<uint64_t> hoffs;
};

void to_device(DevBatch& b) {
    HCHK(hipMalloc(&b.keys, b.hkeys.size()));
    HCHK(hipMalloc(&b.offs, b.hoffs.size() * 8));
    HCHK(hipMemcpy(b.keys, b.hkeys.data(), b.hkeys.size(), hipMemcpyHostToDevice));
    HCHK(hipMemcpy(b.offs, b.hoffs.data(), b.hoffs.size() * 8, hipMemcpyHostToDevice));
}

}  // namespace

int main(int argc, char** argv) {
    std::string cfg_name = "nstar";
    int steps = 10, warmup = 2, pipeline = 1;
    bool host = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { std::fprintf(stderr, "bfbench: %s needs a value\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "--config") cfg_name = next();
        else if (a == "--steps") steps = std::atoi(next());
        else if (a == "--warmup") warmup = std::atoi(next());
        else if (a == "--pipeline") pipeline = std::atoi(next());
        else if (a == "--host") host = true;
        else if (a == "--version") { std::printf("%s\n", bf_version()); return 0; }
        else { std::fprintf(stderr, "bfbench: unknown argument %s\n", a.c_str()); return 2; }
    }
    const Config* c = nullptr;
    for (const Config& x : kConfigs)
        if (cfg_name == x.name) c = &x;
    if (!c || steps < 1 || warmup < 0) { std::fprintf(stderr, "bfbench: bad --config / --steps\n"); return 2; }

    const int64_t m = bf_optimal_m(c->n, c->p);
    const int64_t k = bf_optimal_k((int64_t)c->n, m);
    bf_config cfg{};
    cfg.struct_size = sizeof(cfg);
    cfg.device = 0;
    bf_handle* h = nullptr;
    bf_ok(bf_create((uint64_t)m, (uint32_t)k, &cfg, &h), nullptr, "bf_create");
    uint64_t mm = 0, reach = 0, dev_bytes = 0;
    uint32_t kk = 0;
    bf_ok(bf_info(h, &mm, &kk, &reach, &dev_bytes), h, "bf_info");

    // 50 % random bit density over the reachable prefix (bench.py's prefill)
    {
        const uint64_t nb = (reach + 7) / 8;
        std::vector<uint8_t> pre(nb);
        par_for(nb / 8, [&](uint64_t lo, uint64_t hi) {
            uint64_t s = 0x5EEDull * 1000003ull + lo;
            for (uint64_t w = lo; w < hi; ++w) {
                const uint64_t r = splitmix(s);
                std::memcpy(pre.data() + 8 * w, &r, 8);
            }
        });
        if (reach & 7) pre[nb - 1] &= (uint8_t)(0xFF00u >> (reach & 7));   // no bit at or past reach
        bf_ok(bf_import_redis(h, pre.data(), nb, BF_IMPORT_REPLACE), h, "bf_import_redis");
    }

    const uint64_t B = c->batch;
    const int kPairs = 4;
    std::vector<DevBatch> ins(kPairs), inc(kPairs);
    const uint64_t nmax = (uint64_t)c->n;
    for (int b = 0; b < kPairs; ++b) {
        std::vector<uint64_t> iv(B), qv(B);
        uint64_t s = 0x5EEDull + 977 * (uint64_t)b;
        for (uint64_t j = 0; j < B; ++j) iv[j] = splitmix(s) % nmax;
        for (uint64_t j = 0; j < B; ++j) qv[j] = (j < B / 2) ? iv[2 * j % B] : nmax + splitmix(s) % nmax;
        pack_decimal(iv, ins[b].hkeys, ins[b].hoffs);
        pack_decimal(qv, inc[b].hkeys, inc[b].hoffs);
        ins[b].n = inc[b].n = B;
        to_device(ins[b]);
        to_device(inc[b]);
    }
    uint32_t* dig[kPairs];
    for (int b = 0; b < kPairs; ++b) HCHK(hipMalloc(&dig[b], B * 16));
    uint8_t* d_out = nullptr;
    HCHK(hipMalloc(&d_out, B));
    hipStream_t st;
    HCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

    auto plain_step = [&](int i) {
        const DevBatch& I = ins[i % kPairs];
        const DevBatch& Q = inc[i % kPairs];
        bf_ok(bf_insert_many_dev(h, I.keys, I.offs, B, nullptr, nullptr, st), h, "bf_insert_many_dev");
        bf_ok(bf_include_many_dev(h, Q.keys, Q.offs, B, d_out, st), h, "bf_include_many_dev");
    };
    auto pipe_step = [&](int i) {   // dig[i] holds I_i's SHA-1 words
        const DevBatch& Q = inc[i % kPairs];
        const DevBatch& In = ins[(i + 1) % kPairs];
        bf_ok(bf_insert_digests_dev(h, dig[i % kPairs], B, nullptr, nullptr, st), h, "bf_insert_digests_dev");
        bf_ok(bf_include_hash_dev(h, Q.keys, Q.offs, B, d_out, In.keys, In.offs, B, dig[(i + 1) % kPairs], st), h,
              "bf_include_hash_dev");
    };
    if (pipeline) bf_ok(bf_hash_many_dev(h, ins[0].keys, ins[0].offs, B, dig[0], st), h, "bf_hash_many_dev");
    for (int i = 0; i < warmup; ++i) pipeline ? pipe_step(i) : plain_step(i);
    HCHK(hipStreamSynchronize(st));
    bf_ok(bf_profile(h, 1), h, "bf_profile");
    hipEvent_t e0, e1;
    HCHK(hipEventCreate(&e0));
    HCHK(hipEventCreate(&e1));
    const auto w0 = std::chrono::steady_clock::now();
    HCHK(hipEventRecord(e0, st));
    for (int i = warmup; i < warmup + steps; ++i) pipeline ? pipe_step(i) : plain_step(i);
    HCHK(hipEventRecord(e1, st));
    HCHK(hipEventSynchronize(e1));
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
    float ms = 0.f;
    HCHK(hipEventElapsedTime(&ms, e0, e1));

    // the last step's include? answers: every member found
    std::vector<uint8_t> got(B);
    HCHK(hipMemcpy(got.data(), d_out, B, hipMemcpyDeviceToHost));
    uint64_t fn = 0, fp = 0;
    for (uint64_t j = 0; j < B; ++j) {
        if (j < B / 2) fn += got[j] ? 0 : 1;
        else fp += got[j];
    }

    const uint32_t cap = 32;
    std::vector<char> names(cap * BF_PROFILE_NAME_LEN);
    std::vector<double> tot(cap);
    std::vector<uint64_t> launches(cap);
    uint32_t nk = 0;
    bf_ok(bf_profile_read(h, names.data(), tot.data(), launches.data(), cap, &nk, 1), h, "bf_profile_read");
    bf_ok(bf_profile(h, 0), h, "bf_profile");

    std::string kern = "{";
    for (uint32_t i = 0; i < std::min(nk, cap); ++i) {
        char buf[160];
        std::snprintf(buf, sizeof buf, "%s\"%s\": %.4f", i ? ", " : "", &names[i * BF_PROFILE_NAME_LEN],
                      launches[i] ? tot[i] / (double)launches[i] : 0.0);
        kern += buf;
    }
    kern += "}";

    double host_ins = 0, host_inc = 0;
    if (host) {
        std::vector<uint8_t> hout(B);
        bf_ok(bf_insert_many(h, ins[0].hkeys.data(), ins[0].hoffs.data(), B, nullptr, nullptr), h, "bf_insert_many");
        bf_ok(bf_include_many(h, inc[0].hkeys.data(), inc[0].hoffs.data(), B, hout.data()), h, "bf_include_many");
        const int reps = 3;
        auto t = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r)
            bf_ok(bf_insert_many(h, ins[r % kPairs].hkeys.data(), ins[r % kPairs].hoffs.data(), B, nullptr, nullptr), h,
                  "bf_insert_many");
        host_ins = reps * (double)B / std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
        t = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r)
            bf_ok(bf_include_many(h, inc[r % kPairs].hkeys.data(), inc[r % kPairs].hoffs.data(), B, hout.data()), h,
                  "bf_include_many");
        host_inc = reps * (double)B / std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
    }

    std::printf("{\"tool\": \"bfbench\", \"version\": \"%s\", \"config\": \"%s\", \"m\": %" PRId64 ", \"k\": %" PRId64
                ", \"batch\": %" PRIu64 ", \"steps\": %d, \"warmup\": %d, \"pipelined\": %d, \"ms_per_step\": %.4f, "
                "\"keys_per_s\": %.6e, \"wall_s\": %.4f, \"false_negatives\": %" PRIu64 ", \"observed_fp_rate\": %.6f, "
                "\"kernels_ms\": %s, \"host_api\": %s}\n",
                bf_version(), c->name, m, k, B, steps, warmup, pipeline, ms / steps, 2.0 * B * steps / (ms / 1e3),
                wall, fn, (double)fp / (double)(B - B / 2), kern.c_str(),
                host ? ("{\"insert_keys_per_s\": " + std::to_string(host_ins) + ", \"include_keys_per_s\": " +
                        std::to_string(host_inc) + "}").c_str()
                     : "null");
    for (int b = 0; b < kPairs; ++b) {
        (void)hipFree(ins[b].keys); (void)hipFree(ins[b].offs);
        (void)hipFree(inc[b].keys); (void)hipFree(inc[b].offs);
        (void)hipFree(dig[b]);
    }
    (void)hipFree(d_out);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(st);
    bf_destroy(h);
    return fn ? 1 : 0;
}
