// bf_internal.h — shared between the kernels (bf_kernels.hip) and the C ABI (bf_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

// A/B knobs (kernel variants measured against the defaults) are read from the
// environment only in the builds tools/build_ab_libs.sh makes with -DBFHIP_AB_KNOBS.  The
// shipped library takes the measured defaults: the names are not even in its strings, so no
// inherited variable can change what it computes or how (tests/test_abi.py checks the list).
// The knobs a test uses to force a path (all of which give identical results) stay readable.
#ifdef BFHIP_AB_KNOBS
#define BF_AB_GETENV(name) std::getenv(name)
#else
#define BF_AB_GETENV(name) ((const char*)nullptr)
#endif

// Filter geometry as the kernels see it.
struct BfGeom {
    uint32_t* bits;    // device bitset, Redis byte order viewed as LE 32-bit words
    uint64_t  m;       // modulus (options[:bits], lib/redis/bloomfilter.rb:27)
    double    inv_m;   // 1.0 / m, for the division-free modulo
    uint32_t  k;       // hashes per key (options[:hashes], bloomfilter.rb:28)
    uint32_t  nomod;   // 1 iff m > k*(2^32-1): every derived offset is already < m
    uint32_t  mod_f32; // 1 iff m >= 2^17: the quotient is estimated in float32 (else float64)
    float     inv_m_f; // (float)(1.0 / m)
    uint32_t  mod_sub; // 1..3: every derived offset v <= vmax is below (mod_sub + 1) m, so v mod m
                       // is at most mod_sub conditional subtractions (the north-star m ~ 2.2 x 2^32:
                       // 2); 0: the float-estimate paths (bf_mod_sub)
    uint32_t  shards;  // partitioned filters: shard count P (1 = whole filter)
    uint32_t  block_log2;  // ownership block = 2^block_log2 bits, owner = block % P
    double    inv_shards;  // 1.0 / P, for the division-free block -> (owner, local block) map
    uint32_t  shards_pow2; // 1 iff P is a power of two: the map is a mask and a shift
    uint32_t  shard_log2;  // log2(P) when shards_pow2
    // probe policies (tuning; results are identical for every setting)
    uint32_t  first_round;  // include?: probes loaded before the first early-exit check (0 = all k)
    uint32_t  next_round;   // include?: probes per later round (0 = all the rest at once)
    uint32_t  route_agg;    // route: wave-aggregated owner ranks when P <= route_agg (else LDS atomics)
    uint32_t  insert_test;  // insert: 1 = load the k words first, atomic-OR only the unset bits
    uint32_t  route32;      // BF_FLAG_ROUTE32: routed owner-local offsets are uint32
    uint8_t*  dirty;        // nullable: one byte per 2^kDirtyShiftBits-bit block, set to 1 when an
                            // insert may have changed the block (bf_track_dirty)
    uint64_t  limit;        // the handle's local bits: owner-side kernels drop routed offsets >= limit
                            // (caller-supplied device data never addresses past the bitset)
    // nullable (BF_OP_INSERT_FLAGS direct kernel, seq_mark): every bit this launch flipped 0 -> 1
    // is appended once to flips[0 .. *flip_count) (entries past flip_cap are counted, not stored)
    unsigned long long* flips;
    unsigned long long* flip_count;
    uint64_t  flip_cap;
    uint64_t  flip_tag;     // ORed into every reported offset (the Lua layout: layer << 58)
    // nullable: the handle's key-status word (pinned host memory the device writes): a hashing
    // kernel stores 1 when a key's offsets are inconsistent (bfdev::key_ok) and hashes that key
    // as the empty string; the next call on the handle returns BF_EINVAL (bf_api.cpp)
    uint32_t* key_status;
};

// BfGeom::mod_sub for a modulus m and the largest value the derivation reaches (ruby.rb:51:
// k (2^32 - 1); the Lua scripts' i = 1..k: (k + 1) (2^32 - 1)).
inline uint32_t bf_mod_sub(uint64_t m, uint64_t vmax) {
    const uint64_t q = vmax / m;
    return q <= 3 ? (uint32_t)q : 0u;
}

constexpr uint32_t kDirtyShiftBits = 19;   // dirty-tracking block: 2^19 bits = BF_DIRTY_BLOCK_BYTES of the string

// The sync-free exchange's receive layout: nwin windows of cap entries, window w's live count
// counts[w * stride] on the device, or none when that exceeds cap (an overflowed window holds
// unwritten entries).  counts == NULL: one run of `count` entries.
struct BfWindows {
    const unsigned long long* counts = nullptr;
    uint32_t stride = 1;
    uint32_t nwin = 1;
    uint64_t cap = 0;
    BfWindows() = default;
    BfWindows(const uint64_t* c, uint32_t s, uint32_t n, uint64_t wcap)
        : counts(reinterpret_cast<const unsigned long long*>(c)), stride(s ? s : 1u), nwin(n), cap(wcap) {}
};

// Chunked windows (bf_route_chunks_dev): every route tile's run for a window is sorted by
// the owner's superbin, and the window carries a directory of those runs, so the owner's
// binned pass starts at bin_mid.  Window w's directory at dir + w * dir_bytes: uint32
// start[tiles] (the run's first entry in the window; 0xFFFFFFFF = dropped, the window
// overflowed), then uint16 tab[(S + 1) * tiles]: tab[sb * tiles + tile] = the run's first
// entry of superbin sb, relative to start, and tab[S * tiles + tile] = the run's length.
struct BfChunks {
    uint8_t* dir = nullptr;
    uint64_t dir_bytes = 0;
    uint64_t tiles = 0;        // directory capacity in route tiles (>= every sender's ntiles)
    uint32_t S = 1;            // owner superbins per window (a window-local offset >> sup_log2)
    uint32_t sup_log2 = 0;     // = region_log2 + rel_log2 of the owner's plan
    uint32_t sub2 = 0;         // route sort buckets per (window, superbin): 2^sub2 (low offset bits)
    uint32_t region_log2 = 19, rel_log2 = 0;
};
// The geometry every rank derives alike from the largest shard's size (shard 0) and the
// window count; false when nwin * S cannot fit the route's sort buckets (max_buckets <= 512).
bool bf_chunk_geometry(uint64_t shard0_bits, uint32_t nwin, uint32_t pref_region_log2, BfChunks* cg,
                       uint32_t max_buckets = 0 /* 0: the route's 512 */);
uint64_t bf_chunk_dir_bytes(const BfChunks& cg, uint64_t tiles);

// Owner side: the received windows (slot j = h * nsrc + src at recv + j * cap, its live
// count counts[src * cstride + h]) with their directories.
struct BfChunkIn {
    const uint32_t* recv = nullptr;
    const uint8_t* dir = nullptr;
    uint64_t dir_bytes = 0, tiles = 0, cap = 0, limit = 0;
    const unsigned long long* counts = nullptr;
    uint32_t cstride = 1, nsrc = 1, nh = 1, S = 1, sup_log2 = 0;
    // Ranked chunks (the sorted owner test with packed answers): chunk c = src * cps + r is the
    // tile whose run has rank r in window (h, src) — the order the route claimed the window's
    // runs in, recorded in the directory's rank table — and cps = tiles rounded up to whole
    // run-table passes, so every group of chunks lies in one window and its runs are ONE
    // contiguous range of it.  Unranked: chunk c = src * tiles + tile.
    bool ranked = false;
    uint64_t cps = 0;
};
// Directory of window w (BfChunks / bf_route_chunks_dev), after start[tiles] and tab[(S + 1) *
// tiles]: rank[tiles] (uint16: 1 + the tile whose run the route claimed r-th in the window, 0 =
// none) and an 8-byte claim counter (runs claimed << kClaimRankShift | entries claimed).
constexpr uint32_t kClaimRankShift = 40;
__host__ __device__ inline uint64_t bf_chunk_dir_rank_offset(const BfChunks& cg, uint64_t tiles) {
    return 4 * tiles + 2 * (uint64_t)(cg.S + 1) * tiles;
}
__host__ __device__ inline uint64_t bf_chunk_dir_claim_offset(const BfChunks& cg, uint64_t tiles) {
    return (bf_chunk_dir_rank_offset(cg, tiles) + 2 * tiles + 7) & ~(uint64_t)7;
}

enum BfOp : int {
    BF_OP_INDEXES      = 0,  // write the k offsets of each key (ruby.rb:41-55)
    BF_OP_INCLUDE      = 1,  // AND of the k bits (ruby.rb:20-30)
    BF_OP_INSERT       = 2,  // OR the k bits in, no per-key result (ruby.rb:57-60)
    BF_OP_INSERT_FLAGS = 3,  // ... and report which keys / whether any bit flipped (ruby.rb:61-62)
    BF_OP_ROUTE        = 4,  // owner-local offset (out64) + owner shard (out8) per probe,
                             // per-owner probe counts accumulated into counts[P]
    BF_OP_HASH         = 5,  // the key's SHA-1 words H0..H3 (16 B per key, out64 as uint4[])
};

// Keys: byte j of the packed buffer for offset o is keys16[o + bias - 0] where
// keys16 is 16-byte aligned and readable up to the next 16-byte boundary past
// the last key byte.  (bias is added modulo 2^64.)
hipError_t bf_launch_keys(BfOp op, const BfGeom& g, const uint8_t* keys16, const uint64_t* offsets,
                          uint64_t bias, uint64_t n, uint8_t* out8, uint64_t* out64,
                          uint32_t* any_flag, hipStream_t s,
                          unsigned long long* counts = nullptr /* BF_OP_ROUTE only */);

// RubyTest hash engines (bf_engines.hip, ruby_test.rb:43-61): one lane per (key, probe),
// offset = digest("#{i}-#{key}") as a big-endian integer mod m.  op: INDEXES, INCLUDE
// (out8 preset to 1 inside) or INSERT (any_flag nullable).
enum BfEngine : uint32_t { BF_ENGINE_RUBY = 0, BF_ENGINE_MD5 = 1, BF_ENGINE_SHA1 = 2 };
hipError_t bf_launch_engine(uint32_t engine, BfOp op, const BfGeom& g, const uint8_t* k16, const uint64_t* offsets,
                            uint64_t bias, uint64_t n, uint8_t* out8, uint64_t* out64, uint32_t* flag, hipStream_t s);

// Binned insert (bf_binned.hip): plan + launch.  The launch carves every
// intermediate (probe arrays, run tables, histograms) out of one device
// scratch buffer of plan.scratch_bytes.
struct BfBinPlan {
    uint32_t region_log2;   // 2^region_log2 bits per region (LDS image in the apply / test pass)
    uint32_t nbins;         // regions covering the bitset
    uint32_t rel_log2;      // superbin = 2^rel_log2 consecutive regions (level-1 partition)
    uint32_t nsup;          // superbins covering the bitset (<= 256)
    bool     with_keys;     // include?: probes carry their key index
    uint32_t tile_keys;     // keys per front tile (2048 for k <= 6, else 1024)
    uint32_t tile_probes;   // probes per full front tile (level-1 segment stride)
    uint64_t ntiles;        // front tiles
    uint32_t tiles_per_block;
    uint32_t nblocks;       // front workgroups (<= 512)
    uint32_t ngroups;       // groups of 64 front workgroups (level-2 windows per superbin)
    uint64_t probes;        // n * k (< 2^32)
    uint64_t max_chunks;    // bound on level-2 chunk blocks (bin_mid grid)
    uint64_t scratch_bytes; // device scratch the launch needs
    bool     chunked;       // level 1 = received chunked windows (no front pass, no level-1 arrays)
    bool     l2test;        // chunked include?: the superbin-major L2-local test (no mid sort, no level 2)
    bool     ordered;       // chunked include? with packed answers: chunks ranked by run start (BfChunkIn::ranked)
    uint64_t cps;           // ... chunks per source (tiles rounded up to whole groups)
    uint32_t nwin;          // ... received windows (nh * nsrc)
    uint64_t tiles;         // ... directory tiles
};
// Optional per-kernel timing: when a BfMarks is passed, a launcher records
// marks->ev[i] after its i-th kernel (ev[0] before the first), named names[i].
struct BfMarks {
    static constexpr int kMax = 12;
    hipEvent_t ev[kMax + 1];
    const char* names[kMax];
    int used;   // kernels marked
};
inline void bf_mark(BfMarks* mk, hipStream_t s, const char* name) {
    if (!mk || mk->used >= BfMarks::kMax) return;
    mk->names[mk->used] = name;
    (void)hipEventRecord(mk->ev[++mk->used], s);
}
// Largest batch one binned launch takes on this bitset (larger batches go in
// sub-batches): up to 4096 front workgroups of 16 tiles, within 4096 (superbin,
// group) windows of the one-workgroup scan.
uint64_t bf_binned_max_keys(uint32_t k, uint64_t bitset_bytes, uint32_t pref_region_log2);
// false: the batch / filter shape is outside the binned path (k > 16, more than
// bf_binned_max_keys keys, or a bitset beyond 65536 regions of 2^20 bits).
bool bf_binned_plan(uint64_t bitset_bytes, uint64_t n, uint32_t k, uint32_t pref_region_log2, bool with_keys,
                    BfBinPlan* plan);
hipError_t bf_launch_insert_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                   const uint8_t* keys16, const uint64_t* offsets, uint64_t bias, uint64_t n,
                                   void* scratch, uint32_t* any_flag, hipStream_t s, BfMarks* marks = nullptr);
// The same on keys given as their SHA-1 words (bf_hash_many_dev's output): no hash pass.
hipError_t bf_launch_insert_binned_digests(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                           const uint4* dig, uint64_t n, void* scratch, uint32_t* any_flag,
                                           hipStream_t s, BfMarks* marks = nullptr);
// Owner side of a partitioned filter: `count` routed shard-local offsets (uint32
// when route32, else uint64) ORed into the shard through the same pipeline.
uint64_t bf_binned_max_offsets(uint64_t bitset_bytes, uint32_t pref_region_log2);
bool bf_binned_plan_offsets(uint64_t bitset_bytes, uint64_t count, uint32_t pref_region_log2, BfBinPlan* plan,
                            bool with_keys = false);
// Window layout (w.counts != NULL): count = nwin * cap entries, cap a multiple of
// BF_WINDOW_CAP_ALIGN; entries past a window's live count are skipped.
hipError_t bf_launch_shard_insert_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                         const void* local, bool route32, uint64_t count, void* scratch,
                                         uint32_t* any_flag, hipStream_t s, BfMarks* marks = nullptr,
                                         uint64_t bias = 0, const BfWindows& w = BfWindows{});
// Binned shard test (owner side of a partitioned include?): out8[i] = bit of local[i].
// Plan with bf_binned_plan_offsets(..., with_keys = true).
hipError_t bf_launch_shard_test_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                       const void* local, bool route32, uint64_t count, void* scratch, uint8_t* out8,
                                       hipStream_t s, BfMarks* mk, uint64_t bias = 0,
                                       const BfWindows& w = BfWindows{});
// plan.with_keys must be set; out8 gets the n answers.
hipError_t bf_launch_include_binned(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                    const uint8_t* keys16, const uint64_t* offsets, uint64_t bias, uint64_t n,
                                    void* scratch, uint8_t* out8, hipStream_t s, BfMarks* marks = nullptr);

// Replicated inserts from region sets (bf_binned.hip): every rank encodes its own
// batch once as per-region Elias-Fano sets of the offsets it probes; every replica ORs all
// ranks' sets in with one pass over the bitset.  Geometry: the regions a bitset of this size
// takes (region_log2 18 or 19; false otherwise).  Capacity: a bound on the set buffer of any
// batch of n keys.  The encode's plan (bf_binned_plan) must have the geometry's region size.
bool bf_sets_geometry(uint64_t bitset_bytes, uint32_t pref_region_log2, uint32_t* region_log2, uint32_t* nbins);
uint64_t bf_sets_capacity_bytes(uint64_t bitset_bytes, uint32_t pref_region_log2, uint64_t n, uint32_t k);
// Words before a set buffer's first set: the header and the two per-region tables.
uint64_t bf_sets_header_words(uint32_t nbins);
// persistent_grid > 0: the encode pass as a persistent grid of that many workgroups (an encoder
// handle's, beside another stream's apply; 2^19-bit regions), 0: one workgroup per region.
hipError_t bf_launch_encode_sets(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes, const uint8_t* keys16,
                                 const uint64_t* offsets, uint64_t bias, uint64_t n, bool dig, void* scratch,
                                 uint32_t* out, uint64_t cap_words, hipStream_t s, BfMarks* marks = nullptr,
                                 uint32_t persistent_grid = 0);
// One step of a replicated filter: nsrc set buffers ORed in (as bf_launch_insert_sets) and the
// next batch (n_next SHA-1 word quadruples, plan p) encoded into next_out (as
// bf_launch_encode_sets with dig), the two region passes in one kernel when they share the
// region geometry and one launch takes every source.
hipError_t bf_launch_insert_encode_sets(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                        uint32_t region_log2, uint32_t nbins, const uint32_t* sets,
                                        uint64_t stride_words, uint32_t nsrc, uint64_t probes_hint, uint32_t* any_flag,
                                        uint32_t* status, const uint8_t* next_dig, uint64_t n_next, void* scratch,
                                        uint32_t* next_out, uint64_t cap_words, hipStream_t s, BfMarks* marks = nullptr);
hipError_t bf_launch_insert_sets(const BfGeom& g, uint64_t bitset_bytes, uint32_t region_log2, uint32_t nbins,
                                 const uint32_t* sets, uint64_t stride_words, uint32_t nsrc, uint64_t probes_hint,
                                 uint32_t* any_flag, uint32_t* status, hipStream_t s, BfMarks* marks = nullptr);

// Exact sequential per-key results (bf_seq.hip): batches of at most
// bf_seq_chunk_keys(k) keys, scratch of bf_seq_scratch_bytes(n, k, m) (m: the filter's bits).  Probe
// indices i0 .. i0+k-1 (0 for the ruby driver, 1 for the Lua scripts).
uint64_t bf_seq_chunk_keys(uint32_t k);
uint64_t bf_seq_scratch_bytes(uint64_t n, uint32_t k, uint64_t m);
hipError_t bf_launch_seq_candidates(const BfGeom& g, uint32_t i0, const uint8_t* keys16, const uint64_t* offsets,
                                    uint64_t bias, uint64_t n, void* scratch, hipStream_t s);
// new(j) -> out8 / any_flag (nullable) for j < n; ORs the 0-probes of keys j < limit into g.bits
// (limit = min(limit, *d_limit) when d_limit is given: a cut the device computed).
hipError_t bf_launch_seq_mark(const BfGeom& g, uint32_t i0, uint64_t n, uint64_t limit, void* scratch,
                              uint8_t* out8, uint32_t* any_flag, hipStream_t s,
                              const unsigned long long* d_limit = nullptr);
hipError_t bf_launch_insert_seq(const BfGeom& g, const uint8_t* keys16, const uint64_t* offsets, uint64_t bias,
                                uint64_t n, void* scratch, uint8_t* out8, uint32_t* any_flag, hipStream_t s,
                                BfMarks* marks = nullptr);

// Chunked windows, owner side (bf_binned.hip): plan over the shard for nh sub-ranges x nsrc
// windows of cap entries and `tiles` chunks each; insert (any_flag nullable) or test (out8[i]
// = bit of recv entry i, for every live entry; plan with_keys).
bool bf_chunk_plan(uint64_t bitset_bytes, const BfChunks& cg, uint32_t nh, uint32_t nsrc, uint64_t cap,
                   bool with_keys, BfBinPlan* plan, bool l2test = false, bool ordered = false);
// Whether the ranked (packed-answer) test takes this geometry: a tile index fits the directory's
// uint16 rank table and each window's packed answers start on a 4-byte word.
bool bf_chunk_ordered_ok(uint64_t tiles, uint64_t cap);
hipError_t bf_launch_shard_insert_chunks(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                         const BfChunkIn& ci, void* scratch, uint32_t* any_flag, hipStream_t s,
                                         BfMarks* marks = nullptr);
// A side job for the owner test: the SHA-1 words of another key batch (a requester's next
// include? batch), hashed by the L2 sweep's workgroups between their items (keys16 aligned
// down to 16 B, bias = the dropped bytes; n = 0: none).
struct BfSideHash {
    const uint8_t* keys16 = nullptr;
    const uint64_t* offsets = nullptr;
    uint64_t bias = 0, n = 0;
    uint4* dig = nullptr;
    uint32_t* key_status = nullptr;   // BfGeom::key_status of the handle
};
hipError_t bf_launch_shard_test_chunks(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                       const BfChunkIn& ci, void* scratch, uint8_t* out8, hipStream_t s,
                                       BfMarks* marks = nullptr, const BfSideHash& side = BfSideHash{});
// The same test with the answers as packed bits in the return trip's layout (window (h, src) at
// packed + (src * nh + h) * ceil(cap / 8), LSB first): ordered chunks, answers stored in level-2
// order and moved to receive order per group in LDS (plan: bf_chunk_plan(..., ordered = true)).
hipError_t bf_launch_shard_test_chunks_packed(const BfGeom& g, const BfBinPlan& p, uint64_t bitset_bytes,
                                              BfChunkIn ci, void* scratch, uint8_t* packed, hipStream_t s,
                                              BfMarks* marks = nullptr);
// One step's owner work in one pass over the shard: the insert windows (plan pi, as
// bf_launch_shard_insert_chunks) ORed in and the include? windows (plan pt, ordered, as
// bf_launch_shard_test_chunks_packed) tested against the result, region by region.  Scratch:
// bf_chunk_scratch_bytes(pi) + bf_chunk_scratch_bytes(pt).
uint64_t bf_chunk_scratch_bytes(const BfBinPlan& p);
hipError_t bf_launch_shard_insert_test_chunks_packed(const BfGeom& g, const BfBinPlan& pi, const BfBinPlan& pt,
                                                     uint64_t bitset_bytes, const BfChunkIn& cii, BfChunkIn cit,
                                                     void* scratch, uint32_t* any_flag, uint8_t* packed, hipStream_t s,
                                                     BfMarks* marks, const BfSideHash& side);
// Requester side: the window route with directories (cg.dir zeroed here first; slot16
// nullable: tile-relative key indices).
// dig: keys16 holds the keys' SHA-1 words (uint4 per key; offsets unused) instead of key bytes.
hipError_t bf_launch_route_chunks(const BfGeom& g, const BfBinPlan& p, uint32_t nh, const BfChunks& cg,
                                  const uint8_t* keys16, const uint64_t* offsets, uint64_t bias, uint64_t n,
                                  void* send, uint16_t* slot16, uint64_t wcap, unsigned long long* counts,
                                  hipStream_t s, BfMarks* marks = nullptr, bool dig = false);
// out[j] = AND over every window's chunk of j's tile of the packed answer bits (window w at
// packed + w * ceil(wcap / 8)); one workgroup per route tile, answers gathered in LDS.
hipError_t bf_launch_combine_chunks_packed(const uint8_t* packed, const uint16_t* slot16, uint64_t wcap,
                                           const BfChunks& cg, uint32_t nwin, const unsigned long long* counts,
                                           uint64_t n, uint32_t tile_keys, uint8_t* out, hipStream_t s);

// Partitioned filters, requester side, fused (bf_binned.hip): hash + per-tile
// LDS sort by owner, then an owner-major gather into send[] (uint64 entries when
// wide, else uint32) and slot[] (key index of each send entry, nullable);
// counts[s] = probes for owner s.  Needs k <= 16 and P x groups <= 4096 windows.
bool bf_route_plan(uint64_t n, uint32_t k, uint32_t shards, bool wide, bool with_slot, BfBinPlan* plan);
hipError_t bf_launch_route_fused(const BfGeom& g, const BfBinPlan& p, bool wide, const uint8_t* keys16,
                                 const uint64_t* offsets, uint64_t bias, uint64_t n, void* scratch, void* send,
                                 uint32_t* slot, unsigned long long* counts, hipStream_t s,
                                 BfMarks* marks = nullptr);

// Window route (bf_binned.hip): the fused route's front pass writing each tile's owner
// runs straight into send[s*wcap ..] (and slot[s*wcap ..]) at places claimed with
// atomics on counts[s]; a run past wcap is dropped (counts[s] > wcap tells the caller).
hipError_t bf_launch_route_windows(const BfGeom& g, const BfBinPlan& p, uint32_t nh, const uint8_t* keys16,
                                   const uint64_t* offsets, uint64_t bias, uint64_t n, void* send, uint32_t* slot,
                                   uint64_t wcap, unsigned long long* counts, hipStream_t s,
                                   BfMarks* marks = nullptr);
// out[j] = AND of bits[p] over the window entries p = s*wcap + i, i < counts[s], s < P,
// with slot[p] == j.
hipError_t bf_launch_combine_windows(const uint8_t* bits, const uint32_t* slot, uint64_t wcap,
                                     const unsigned long long* counts, uint32_t P, uint64_t n, uint8_t* out,
                                     hipStream_t s);

// Answer bytes -> LSB-first bits per segment (seg: nseg triples src, count, dst byte);
// max_count bounds the counts (grid size).  And the windowed combine over such bits
// (window s at packed + s * ceil(wcap / 8)).
hipError_t bf_launch_pack_segments(const uint8_t* bits, const unsigned long long* seg, uint32_t nseg,
                                   uint64_t max_count, uint8_t* packed, hipStream_t s);
hipError_t bf_launch_combine_windows_packed(const uint8_t* packed, const uint32_t* slot, uint64_t wcap,
                                            const unsigned long long* counts, uint32_t P, uint64_t n, uint8_t* out,
                                            hipStream_t s);

// Partitioned filters.  cursor[P]: scratch.  Groups `total` (owner, local) probe
// pairs by owner into send[]; slot[pos] (nullable) = key index (probe / k) of send entry pos.
// counts[P] must hold the per-owner totals (from BF_OP_ROUTE).
// `local` (tmp, from BF_OP_ROUTE) and `send` hold uint64, or uint32 when route32.
hipError_t bf_launch_route_scatter(const void* local, const uint8_t* owner, uint64_t total,
                                   uint32_t P, uint32_t k, const unsigned long long* counts,
                                   unsigned long long* cursor, void* send, uint32_t* slot,
                                   bool route32, hipStream_t s);
// bias: added to every local offset (the 2^32-bit sub-range of a split window route)
// dirty (nullable): the shard's bf_track_dirty map
hipError_t bf_launch_shard_insert(uint32_t* bits, uint64_t limit, const void* local, uint64_t count,
                                  uint32_t* any_flag, bool route32, hipStream_t s, uint64_t bias = 0,
                                  uint8_t* dirty = nullptr, const BfWindows& w = BfWindows{});
hipError_t bf_launch_shard_test(const uint32_t* bits, uint64_t limit, const void* local, uint64_t count,
                                uint8_t* out, bool route32, hipStream_t s, uint64_t bias = 0,
                                const BfWindows& w = BfWindows{});
// out[j] = AND of bits[p] over the n*k send entries p with slot[p] == j.
hipError_t bf_launch_combine(const uint8_t* bits, const uint32_t* slot, uint64_t n, uint32_t k,
                             uint8_t* out, hipStream_t s);

// *d_last = 1 + index of the last nonzero 32-bit word in words[0, nwords) (0 if none).
// d_last must be zeroed before the launch.  nwords must be a multiple of 4.
hipError_t bf_launch_last_nonzero(const uint32_t* words, uint64_t nwords,
                                  unsigned long long* d_last, hipStream_t s);

// dst[i] |= src[i] for i < nwords (nwords multiple of 4, both 16-byte aligned).
hipError_t bf_launch_or(uint32_t* dst, const uint32_t* src, uint64_t nwords, hipStream_t s);

// out[i] = in[i] (uint32 -> uint64), i < count: the host-pointer calls' relative offsets.
hipError_t bf_launch_widen_offsets(const uint32_t* in, uint64_t* out, uint64_t count, hipStream_t s);

// The ops (INDEXES, INCLUDE, INSERT, INSERT_FLAGS) on precomputed SHA-1 words (16 B per key).
hipError_t bf_launch_digests(BfOp op, const BfGeom& g, const uint4* dig, uint64_t n, uint8_t* out8, uint64_t* out64,
                             uint32_t* any_flag, hipStream_t s);
// include? of (keys16, offsets, n) -> out8, fused with the SHA-1 of (skeys16, soffsets, sn) -> sdig.
hipError_t bf_launch_include_hash(const BfGeom& g, const uint8_t* keys16, const uint64_t* offsets, uint64_t bias,
                                  uint64_t n, uint8_t* out8, const uint8_t* skeys16, const uint64_t* soffsets,
                                  uint64_t sbias, uint64_t sn, uint4* sdig, hipStream_t s);
