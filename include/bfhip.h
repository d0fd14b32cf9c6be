/*
 * bfhip.h — C ABI of libbfhip.so, the MI355X Bloom-filter engine behind
 * `Redis::Bloomfilter.new(..., driver: 'hip')`.
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes, and
 * returns an int status (BF_OK = 0).  No exceptions cross the ABI.  The
 * library owns device memory and streams; the caller owns every buffer it
 * passes (read/written during the call only).  Calls on one handle are
 * serialised by an internal mutex, and so is their device work, across
 * streams too: a call whose launches go to a different stream than the
 * previous call's waits (on the device, hipStreamWaitEvent) for that call's
 * last launch, because the launches share the bitset and the handle's
 * scratch.  Different handles are independent.
 *
 * Reference interface each entry point replaces (paths relative to the
 * reference repository kontera-technologies/redis-bloomfilter @ 1.1.2):
 *
 *   bf_create          Redis::BloomfilterDriver::Ruby#initialize  lib/bloomfilter_driver/ruby.rb:10-12
 *                      (m = options[:bits], k = options[:hashes] from
 *                       lib/redis/bloomfilter.rb:27-28)
 *   bf_destroy         (driver object going out of scope)
 *   bf_insert_many     Ruby#insert / #set, one key per call          ruby.rb:15-17, 57-63
 *                      (k pipelined SETBIT; `any_new` = !found, which drives EXPIRE at ruby.rb:62)
 *   bf_insert_many_changes  Ruby#insert, with the bits it set          ruby.rb:57-63
 *                      (the SETBITs that changed something: what write-through replays)
 *   bf_include_many    Ruby#include?                                  ruby.rb:20-30
 *   bf_indexes_many    Ruby#indexes_for (protected)                   ruby.rb:41-55
 *   bf_check_offsets   `data.to_s` of every key (a packed batch's offsets are consistent) ruby.rb:42
 *   bf_clear          Ruby#clear (DEL key_name)                      ruby.rb:33-35
 *   bf_export_redis    GET key_name — the Redis string SETBIT builds  ruby.rb:59 (SETBIT layout)
 *   bf_import_redis    SET key_name — load a string written by the ruby driver
 *   bf_optimal_m/_k    Redis::Bloomfilter.optimal_m / optimal_k       lib/redis/bloomfilter.rb:50-58
 *   bf_version         Redis::Bloomfilter.version                     lib/redis/bloomfilter/version.rb:6-8
 *
 * Device-resident variants (`*_dev`) take device pointers and a hipStream_t
 * (as void*, used verbatim: NULL is HIP's null stream, bf_stream() gives the
 * handle's own) and do not synchronise; they are what bench.py times and what
 * the multi-GPU layer composes.
 *
 * Bit layout (identical to the Redis string written by SETBIT): bit offset o
 * lives in byte o >> 3 under mask 0x80 >> (o & 7).  On the device the bytes
 * are viewed as little-endian 32-bit words: word o >> 5, mask
 * 1u << ((o ^ 7) & 31).  Export is therefore a memcpy of the trimmed prefix.
 */
#ifndef BFHIP_H
#define BFHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes */
#define BF_OK       0
#define BF_EINVAL   1   /* bad argument: m == 0 (the ref raises ZeroDivisionError at ruby.rb:51), k == 0, NULL */
#define BF_ENOMEM   2   /* device or host allocation failed */
#define BF_EDEVICE  3   /* HIP runtime error / no device */
#define BF_ERCCL    4   /* reserved: collective failure (multi-GPU layer) */
#define BF_ERANGE   5   /* output buffer too small (bf_export_redis) / string outside the reachable range */

#define BF_MAX_K    64u /* hashes supported per key */
#define BF_MAX_DEVICES 16 /* devices of one multi-device handle */

/* ---- multi-device handles (bf_config.mode) */
#define BF_MODE_REPLICATED  0u  /* every device holds the whole filter; include? batches split over them */
#define BF_MODE_PARTITIONED 1u  /* the reachable prefix block-cyclically split; probes routed to owners */

/* ---- import modes */
#define BF_IMPORT_REPLACE 0u  /* like SET key value            */
#define BF_IMPORT_OR      1u  /* union with the current filter */

typedef struct bf_handle bf_handle;

typedef struct bf_config {
    uint32_t struct_size;      /* sizeof(bf_config); 0 => defaults for every field        */
    int32_t  device;           /* HIP device ordinal; -1 => current device                 */
    uint64_t batch_keys;       /* keys per internal chunk of host-pointer calls (0 = 1<<22) */
    uint64_t batch_bytes;      /* key bytes per internal chunk (0 = 64 MiB)                 */
    /* Partitioned filters (one handle per GPU, one shard each).  Bit offset o of the
     * reachable prefix belongs to block g = o >> shard_block_log2, owned by shard
     * g % shard_count; inside the owner it sits at local offset
     * ((g / shard_count) << shard_block_log2) | (o & (2^shard_block_log2 - 1)).
     * Block-cyclic, so the probe-dense first 2^32 bits (h0 < 2^32, ruby.rb:51)
     * spread over every shard. */
    uint32_t shard_count;      /* 0 or 1 => the handle holds the whole filter; max 255     */
    uint32_t shard_index;      /* this handle's shard, < shard_count                       */
    uint32_t shard_block_log2; /* ownership block size, 3..40 (0 => 20: 128 KiB blocks)    */
    uint32_t flags;            /* BF_FLAG_* */
    /* Multi-device handles (one process, several GPUs; the Ruby driver's `devices:` and
     * `mode:` options, SURVEY §8 b).  device_count > 0 makes a handle over
     * devices[0 .. device_count) (`device` is then ignored; a device may repeat):
     *   BF_MODE_REPLICATED   every device holds the whole filter.  Inserts go to every
     *                        device (in parallel, one host thread each), include? batches
     *                        are split over the devices.  Export reads device 0.
     *   BF_MODE_PARTITIONED  the reachable prefix is split block-cyclically over the devices
     *                        (shard_block_log2, as for one-handle-per-GPU shards).  Each
     *                        device hashes its part of a batch into per-owner windows
     *                        (bf_route_windows_dev), the windows travel to their owners by
     *                        peer copies over xGMI (hipMemcpyPeerAsync), the owners apply
     *                        or test them, and include? answers travel back the same way.
     * The host-pointer API, export / import (the owner shards' blocks interleaved), clear,
     * dirty tracking and bf_export_range work on both; per_key_new needs BF_MODE_REPLICATED;
     * the device-resident (*_dev, bf_device_bits, bf_stream) and shard entry points return
     * BF_EINVAL on a multi-device handle.  shard_count / shard_index must be 0 / 1. */
    uint32_t device_count;
    uint32_t mode;             /* BF_MODE_* */
    int32_t  devices[BF_MAX_DEVICES];
} bf_config;

/* bf_config.flags */
#define BF_FLAG_ROUTE32 1u     /* routed owner-local offsets (d_send / d_local) are uint32, halving the
                                  all-to-all bytes; needs every shard's local_bits <= 2^32 (else BF_EINVAL) */
/* The RubyTest driver's hash engines (lib/bloomfilter_driver/ruby_test.rb:43-61), instead of
 * the ruby driver's derivation: offset of probe i = MD5 / SHA-1 hexdigest of "#{i}-#{key}"
 * read as one 128 / 160-bit integer, mod m.  Offsets cover all of [0, m) (no reach cap).
 * Whole-filter handles only; per_key_new is refused (BF_EINVAL).  crc32 has no flag: the
 * reference's engine_crc32 raises at its first call (Integer#to_i takes no radix, :52). */
#define BF_FLAG_ENGINE_MD5  2u
#define BF_FLAG_ENGINE_SHA1 4u
/* An encoder handle: the filter's geometry (m, k, its regions) and binned scratch but NO bitset
 * in device memory.  Only bf_encode_region_sets_dev / _digests_dev run on it (every other op
 * returns BF_EINVAL): a replicated filter encodes its next batch on a second stream through it,
 * beside its own handle's apply, since one handle orders all of its calls (the set buffers are
 * the same as its filter handle's). */
#define BF_FLAG_ENCODER     8u

/* ---- lifecycle */
int  bf_create(uint64_t m_bits, uint32_t k, const bf_config* cfg, bf_handle** out);
int  bf_destroy(bf_handle* h);
const char* bf_last_error(const bf_handle* h);   /* h == NULL: last error of bf_create on this thread */
const char* bf_version(void);

/* ---- filter geometry: m, k, and the reachable prefix min(m, k*(2^32-1)+1)
 *      (ruby.rb:44-51 only ever produces offsets below k*(2^32-1)+1). */
int  bf_info(const bf_handle* h, uint64_t* m_bits, uint32_t* k, uint64_t* reach_bits,
             uint64_t* device_bytes);

/* ---- host-pointer batch API.  keys: packed key bytes (`data.to_s`);
 *      offsets: n+1 byte offsets into key_bytes, key j = [offsets[j], offsets[j+1]).
 *      offsets[0] need not be 0. */
int  bf_insert_many(bf_handle* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n,
                    uint8_t* any_new /* nullable: 1 iff some bit flipped 0->1 (drives EXPIRE) */,
                    uint8_t* per_key_new /* nullable, n bytes: 1 iff, inserting the keys one by one in
                                            batch order (ruby.rb:57-61), this key flipped a bit; its
                                            complement is include?-before-insert (bf_10_000.rb:37) */);
int  bf_include_many(bf_handle* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n,
                     uint8_t* out /* n bytes, 0/1 */);
int  bf_indexes_many(bf_handle* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n,
                     uint64_t* out /* n*k offsets, key-major */);
int  bf_clear(bf_handle* h);

/* ---- Redis-string sync.  Export writes the trimmed Redis string (length =
 *      last nonzero byte + 1, exactly what k SETBITs would have grown the key
 *      to).  buf == NULL => only *len_out is set.  cap < len => BF_ERANGE. */
int  bf_export_redis(bf_handle* h, uint8_t* buf, uint64_t cap, uint64_t* len_out);
int  bf_import_redis(bf_handle* h, const uint8_t* buf, uint64_t len, uint32_t mode);

/* ---- device-resident API (device pointers; async on `stream`).
 *      Key bytes: the kernels read d_key_bytes in aligned 16-byte vectors, so the buffer
 *      must stay readable up to 16 bytes past d_key_bytes + d_offsets[n] (pad the
 *      allocation by 16 bytes; the host-pointer API does this in its staging copy).
 *      Key offsets: d_offsets[0..n] must be non-decreasing and every key shorter than 2 GiB
 *      (ruby.rb:42 hashes `data.to_s`: every key has a finite length).  The host-pointer API
 *      checks this before any copy; the device entry points cannot read the offsets without a
 *      sync, so every hashing kernel checks each key against its tile's first and last
 *      offsets (the rule bf_check_offsets applies) and hashes a key that fails as the empty
 *      string — it never loops over a wrapped length or reads outside [d_offsets[0],
 *      d_offsets[n]) — and the NEXT call on the handle (bf_sync at the latest) returns
 *      BF_EINVAL once; the results of the call that met it are not meaningful. */
int  bf_check_offsets(const uint64_t* offsets /* n+1 */, uint64_t n,
                      uint64_t* bad_key /* nullable: the first key j the rule refuses */);
int  bf_insert_many_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets,
                        uint64_t n, uint32_t* d_any_new /* nullable: OR-ed with 1 when a bit flips */,
                        uint8_t* d_per_key_new /* nullable */, void* stream);
int  bf_include_many_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets,
                         uint64_t n, uint8_t* d_out, void* stream);
int  bf_indexes_many_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets,
                         uint64_t n, uint64_t* d_out, void* stream);
/* ---- SHA-1 words as a reusable intermediate.  A key's k offsets depend only on the first
 *      four big-endian words H0..H3 of its SHA-1 (ruby.rb:42-47's h[0..3]), so a batch hashed
 *      once can be inserted and tested without hashing again (the reference's check-then-add
 *      loop, bf_10_000.rb:34-43, hashes every key twice).  Digests: 4 uint32 per key, H0..H3,
 *      16-byte aligned.
 *   bf_hash_many_dev        keys -> digests
 *   bf_insert_digests_dev   bf_insert_many_dev on digests (d_per_key_new must be NULL)
 *   bf_include_digests_dev  bf_include_many_dev on digests
 *   bf_include_hash_dev     include? of one key batch fused with hashing another batch into
 *                           digests: the include? is bound by its probes' memory latency and
 *                           its VALUs mostly idle, so the other batch's SHA-1 runs there
 *                           nearly free — e.g. the next insert batch of a stream of
 *                           insert + include? steps, which then goes in with
 *                           bf_insert_digests_dev and skips its own hash pass.  The include?
 *                           answers are those of the filter as it stands (the hashing touches
 *                           no filter state). */
int  bf_hash_many_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                      uint32_t* d_digests, void* stream);
int  bf_insert_digests_dev(bf_handle* h, const uint32_t* d_digests, uint64_t n, uint32_t* d_any_new,
                           uint8_t* d_per_key_new, void* stream);
int  bf_include_digests_dev(bf_handle* h, const uint32_t* d_digests, uint64_t n, uint8_t* d_out, void* stream);
int  bf_include_hash_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                         uint8_t* d_out, const uint8_t* d_next_key_bytes, const uint64_t* d_next_offsets,
                         uint64_t n_next, uint32_t* d_next_digests, void* stream);
/* ---- Replicated inserts from region sets (ruby.rb:57-63 on every replica of a replicated
 *      filter; BASELINE configs[3]'s "replicated on 8 GPUs, key batches sharded").  Each rank
 *      sorts ITS OWN batch by filter region once and encodes it; the encoded batches of all
 *      ranks travel (an all-gather of fixed-size buffers); every replica ORs all of them in
 *      with one pass over its bitset and no sort.  Per region the encoding is the set of
 *      distinct region-local offsets the batch probes, as an Elias-Fano set (~log2(region bits
 *      / offsets) + 2 bits per offset: about the size of the keys' SHA-1 words).  The bitset
 *      after bf_insert_region_sets_dev of every rank's sets equals the one after inserting
 *      every rank's keys (OR is idempotent and commutative).
 *   bf_region_sets_capacity  bytes a set buffer needs for any batch of <= n keys (a bound,
 *                            the same on every handle of this m and k: size the all-gather).
 *                            BF_EINVAL when one encode cannot take n keys (more than one
 *                            binned pass) or the handle is not the ruby derivation: sized from
 *                            the largest batch of all ranks, every rank learns it together
 *   bf_encode_region_sets_dev / _digests_dev   keys (or their SHA-1 words) -> d_sets
 *                            (sets_bytes >= the capacity; 16-byte aligned; the filter is not
 *                            modified).  n = 0 writes an empty set buffer.
 *   bf_insert_region_sets_dev  nsrc set buffers at d_sets + s * stride_bytes (each written by
 *                            an encode on a handle of the same m and k) ORed into the filter;
 *                            probes_hint = the probes they hold (sum of n * k: picks the apply's
 *                            density form, never the result); d_any_new as bf_insert_many_dev;
 *                            BF_EINVAL for an engine handle (BF_FLAG_ENGINE_*), or a stride
 *                            below a buffer's header and per-region tables;
 *                            d_status (nullable) gets 1 ORed in when a buffer's header does not
 *                            match this filter (that buffer is skipped), or a region's entry
 *                            would reach past its buffer (that region of that buffer is
 *                            skipped).  A set body is read only inside its own bounds.
 *   bf_insert_encode_region_sets_dev  one replica step's two region passes in one call:
 *                            bf_insert_region_sets_dev of the nsrc buffers, and
 *                            bf_encode_region_sets_digests_dev of the NEXT batch (n_next SHA-1
 *                            word quadruples) into d_next_sets, which must not overlap the
 *                            buffers being inserted.  Region r is applied and then r's next
 *                            set encoded by the same workgroup in the same LDS, so the apply's
 *                            bitset stream and the encode's LDS / VALU work overlap inside each
 *                            CU.  Results equal the two calls'. */
int  bf_region_sets_capacity(const bf_handle* h, uint64_t n, uint64_t* bytes);
int  bf_encode_region_sets_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                               uint32_t* d_sets, uint64_t sets_bytes, void* stream);
int  bf_encode_region_sets_digests_dev(bf_handle* h, const uint32_t* d_digests, uint64_t n, uint32_t* d_sets,
                                       uint64_t sets_bytes, void* stream);
int  bf_insert_region_sets_dev(bf_handle* h, const uint32_t* d_sets, uint64_t stride_bytes, uint32_t nsrc,
                               uint64_t probes_hint, uint32_t* d_any_new /* nullable */,
                               uint32_t* d_status /* nullable */, void* stream);
int  bf_insert_encode_region_sets_dev(bf_handle* h, const uint32_t* d_sets, uint64_t stride_bytes, uint32_t nsrc,
                                      uint64_t probes_hint, uint32_t* d_any_new /* nullable */,
                                      uint32_t* d_status /* nullable */, const uint32_t* d_next_digests,
                                      uint64_t n_next, uint32_t* d_next_sets, uint64_t next_sets_bytes, void* stream);
/* The device bitset (Redis byte order, device_bytes long, zero past the reachable prefix). */
int  bf_device_bits(bf_handle* h, void** d_bits, uint64_t* device_bytes);
/* How an insert batch of n keys will run (no launch): *binned = 1 for the binned
 * (hash, partition, per-region LDS apply) pipeline, 0 for the direct test-then-atomic
 * kernel; *scratch_bytes = device scratch the binned pipeline allocates for it.
 * The choice never changes results; BFHIP_INSERT_BINNED=0/1 forces it. */
int  bf_insert_plan(const bf_handle* h, uint64_t n, uint32_t* binned, uint64_t* scratch_bytes);

/* ---- incremental Redis sync.  With tracking on, every insert
 *      (direct, binned and sequential paths) marks the BF_DIRTY_BLOCK_BYTES blocks
 *      of the Redis string it may have changed; imports mark everything; bf_clear
 *      forgets it all (the driver DELs the key).  bf_dirty_ranges returns the
 *      changed byte ranges (offset, length pairs; adjacent blocks coalesced, clipped
 *      to the string's trimmed length *redis_len, so SETRANGE of each range grows the
 *      key exactly as the SETBITs would have) and, with clear != 0, forgets them;
 *      ranges == NULL only counts.  Whole-filter handles only. */
#define BF_DIRTY_BLOCK_BYTES 65536
int  bf_track_dirty(bf_handle* h, uint32_t enable);
int  bf_dirty_ranges(bf_handle* h, uint64_t* ranges /* 2*cap */, uint32_t cap, uint32_t* n_out,
                     uint64_t* redis_len /* nullable */, uint32_t clear);
int  bf_export_range(bf_handle* h, uint64_t offset, uint64_t len, uint8_t* buf);
/* Per-key write-through (ruby.rb:57-63 issues k SETBITs per insert): inserts a small batch
 * (n * k <= 4096 probes, <= 64 KiB of key bytes) and lists every bit offset it flipped from
 * 0 to 1, each once, in out_bits[0 .. *count) (cap >= n * k).  SETBIT of exactly those
 * offsets brings a Redis copy of the filter to the device's state — the same string the
 * ruby driver's k SETBITs per key build, since a SETBIT that changes nothing neither
 * changes nor grows the string — and *count > 0 is the ref's `!found` (EXPIRE).  Leaves
 * the dirty-block map untouched.  Whole-filter handles only (every hash engine; a
 * multi-device handle or a shard: BF_EINVAL, use bf_dirty_ranges). */
int  bf_insert_many_changes(bf_handle* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n,
                            uint64_t* out_bits, uint64_t cap, uint64_t* count);

/* ---- per-kernel timing.  While enabled, every keyed launch (insert / include? /
 *      indexes, host or device API) records HIP events on its stream between its
 *      kernels; bf_profile_read waits for them and returns, per kernel name, the
 *      summed duration and launch count (names in BF_PROFILE_NAME_LEN-byte slots).
 *      *n_out = kernels known (may exceed cap).  reset != 0 clears the totals. */
#define BF_PROFILE_NAME_LEN 64
int  bf_profile(bf_handle* h, uint32_t enable);
int  bf_profile_read(bf_handle* h, char* names, double* total_ms, uint64_t* launches, uint32_t cap,
                     uint32_t* n_out, uint32_t reset);
int  bf_stream(bf_handle* h, void** stream);   /* the handle's own (non-blocking) hipStream_t */
int  bf_sync(bf_handle* h);                    /* synchronise the handle's own stream and the stream of its
                                                  last call; BF_EINVAL if a kernel met inconsistent key
                                                  offsets since the last call (see the *_dev API) */

/* ---- partitioned filters (multi-GPU; the collective between the steps is the
 *      caller's, e.g. RCCL all-to-all through torch.distributed).
 *
 *  requester:  bf_route_dev     hash n keys; every probe (j, i) becomes an owner-local
 *                               offset in d_send, grouped by owner shard: owner s's probes
 *                               are d_send[displ[s] .. displ[s] + d_counts[s]), displ the
 *                               exclusive prefix sum of d_counts; d_slot[p] (nullable: an
 *                               insert does not need it) is the index j of the key that
 *                               send entry p belongs to.  Needs n*k < 2^32.
 *  owner:      bf_shard_insert_dev   OR the received local offsets into this shard
 *              bf_shard_test_dev     one byte (0/1) per received local offset
 *  requester:  bf_combine_dev   d_bits[p] = the owner's answer for send entry p (returned in
 *                               send order); d_out[j] = AND of d_bits[p] over the k entries
 *                               with d_slot[p] == j (include? answer)
 *
 *  Works on any handle: on a whole-filter handle shard_count = 1 routes everything to 0.
 *  d_counts must hold shard_count uint64 and is written, not accumulated.
 *  The owner ops take device data from the caller (or from a peer): a local offset at or past
 *  the shard's local_bits is dropped by the inserts and answers 0 in the tests, and a combine
 *  slot >= n is ignored, so no entry ever addresses memory outside the bitset or the answers. */
int  bf_shard_info(const bf_handle* h, uint32_t* shard_count, uint32_t* shard_index,
                   uint32_t* block_log2, uint64_t* local_bits);
int  bf_route_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                  void* d_send /* uint64[n*k], or uint32 with BF_FLAG_ROUTE32 */,
                  uint32_t* d_slot /* nullable, n*k */,
                  uint64_t* d_counts, void* stream);
/* bf_route_window_split  nh = the 2^32-bit sub-ranges of the largest shard (1 when every
 *                        shard fits 2^32 bits): the window route keeps nwin = shard_count*nh
 *                        windows, window w = s*nh + hi holding owner s's probes whose local
 *                        offset is (hi << 32) | entry.
 * bf_route_windows_dev   bf_route_dev without its owner-major gather pass: window w's
 *                        probes land in d_send[w*window_cap .. w*window_cap + d_counts[w])
 *                        as uint32, in an unspecified order, with d_slot (nullable)
 *                        alongside; each window feeds one send of a grouped send/recv
 *                        exchange.  d_counts holds nwin uint64.  If some d_counts[w] >
 *                        window_cap (a skewed batch), that window's contents are undefined
 *                        (the windowed owner ops and combines skip it): route again with
 *                        window_cap = n*k, which always fits.
 * bf_shard_insert_hi_dev / bf_shard_test_hi_dev   the owner ops on the uint32 entries of
 *                        sub-range hi (local offset = (hi << 32) | entry).
 * bf_combine_windows_dev bf_combine_dev over that layout: d_bits and d_slot indexed by window
 *                        entry, the live entries of window w being the first d_counts[w]. */
int  bf_route_window_split(const bf_handle* h, uint32_t* nh);
int  bf_route_windows_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                          uint32_t* d_send /* nwin*window_cap entries */, uint32_t* d_slot /* nullable */,
                          uint64_t window_cap, uint64_t* d_counts /* nwin */, void* stream);
int  bf_shard_insert_hi_dev(bf_handle* h, const uint32_t* d_local32, uint64_t count, uint32_t hi,
                            uint32_t* d_any_new /* nullable */, void* stream);
int  bf_shard_test_hi_dev(bf_handle* h, const uint32_t* d_local32, uint64_t count, uint32_t hi, uint8_t* d_bits,
                          void* stream);
int  bf_combine_windows_dev(bf_handle* h, const uint8_t* d_bits, const uint32_t* d_slot, uint64_t window_cap,
                            uint32_t nwin, const uint64_t* d_counts /* device, nwin */, uint64_t n,
                            uint8_t* d_out, void* stream);
/* The return trip of a window-routed include? at one bit per probe:
 * bf_pack_segments_dev           owner: segment q of d_seg (device, nseg triples of uint64:
 *                                source offset, count, destination byte offset) packs the answer
 *                                bytes d_bits[src .. src + count) LSB-first into ceil(count/8)
 *                                bytes at d_packed[dst]; max_count >= every count.
 * bf_combine_windows_packed_dev  requester: bf_combine_windows_dev with window w's answers
 *                                as bits at d_packed + w*ceil(window_cap/8). */
int  bf_pack_segments_dev(bf_handle* h, const uint8_t* d_bits, const uint64_t* d_seg, uint32_t nseg,
                          uint64_t max_count, uint8_t* d_packed, void* stream);
int  bf_combine_windows_packed_dev(bf_handle* h, const uint8_t* d_packed, const uint32_t* d_slot,
                                   uint64_t window_cap, uint32_t nwin, const uint64_t* d_counts, uint64_t n,
                                   uint8_t* d_out, void* stream);
/* The sync-free exchange (no host wait for counts): every source sends its whole windows,
 * window_cap entries each, so the receive layout is fixed and the live counts stay on the
 * device.  The owner ops then run over nwin received windows of sub-range hi: window w holds
 * d_local32[w*window_cap ..], of which the first min(d_counts[w*count_stride], window_cap)
 * entries are live (local offset (hi << 32) | entry); the test writes one byte per window
 * entry to d_bits (entries past a count: unspecified).  A window whose count exceeds
 * window_cap overflowed in the route (runs past the cap were dropped, leaving unwritten
 * entries below it) and is skipped whole, here and by the windowed combines: the caller
 * learns of it from the counts and re-does the batch (PartitionedFilter replays it through
 * the synced exchange).  A window_cap that is a multiple of
 * BF_WINDOW_CAP_ALIGN lets the owner take the binned (sort by region) path. */
#define BF_WINDOW_CAP_ALIGN 12288
int  bf_shard_insert_windows_dev(bf_handle* h, const uint32_t* d_local32, uint64_t window_cap, uint32_t nwin,
                                 const uint64_t* d_counts, uint32_t count_stride, uint32_t hi, uint32_t* d_any_new,
                                 void* stream);
int  bf_shard_test_windows_dev(bf_handle* h, const uint32_t* d_local32, uint64_t window_cap, uint32_t nwin,
                               const uint64_t* d_counts, uint32_t count_stride, uint32_t hi, uint8_t* d_bits,
                               void* stream);
/* Chunked windows: the sync-free exchange without the owner's sort pass.  Replaces the
 * owner-side half of SETBIT / GETBIT routing for ruby.rb:57-60 / :20-30 (the same offsets
 * as bf_route_windows_dev reach the same bits; only their order inside a window and a
 * directory beside it differ).
 * bf_route_chunk_info       tiles = ceil(n_bound / keys per route tile), the directory
 *                           capacity every rank must use for batches of <= n_bound keys, and
 *                           dir_bytes = one window's directory; BF_EINVAL if this shard
 *                           count cannot take chunked windows (the caller keeps the windows
 *                           above).  Every rank gets the same values for the same n_bound.
 *                           A directory is uint32 start[tiles] then uint16 tab[(superbins +
 *                           1) * tiles] ([sb][tile] run starts, row superbins = run lengths).
 * bf_route_chunks_dev       bf_route_windows_dev whose per-tile runs are sorted by the
 *                           owner's superbin, plus window w's directory at d_dir +
 *                           w*dir_bytes (tiles entries; route tile t's run: its place in the
 *                           window and its superbin run table).  d_slot16 (nullable) holds
 *                           each entry's key index relative to its route tile (uint16).
 *                           n must be <= tiles * keys per tile.
 * bf_shard_insert_chunks_dev / bf_shard_test_chunks_dev   owner: nsrc sources' received
 *                           windows of every sub-range hi < nh, window (hi, src) at d_recv +
 *                           (hi*nsrc + src)*window_cap with its directory at d_dir +
 *                           (hi*nsrc + src)*dir_bytes and live count d_counts[src*count_stride
 *                           + hi] (a window past window_cap is skipped whole); one call for
 *                           every sub-range.  The test writes d_bits[(hi*nsrc + src)*window_cap
 *                           + i] for the live entries i.
 * bf_shard_test_chunks_packed_dev  the test with its answers as packed bits in the return
 *                           trip's layout: window (hi, src) at d_packed + (src*nh + hi) *
 *                           ceil(window_cap/8), bit i (LSB first) = live entry i (1 = its bit
 *                           is set; an offset past the shard answers 0) — what
 *                           bf_combine_chunks_packed_dev reads, with no pack pass between.  The
 *                           sorted owner test ranks each window's route tiles by their run's
 *                           start so that a group of chunks is one contiguous range of its
 *                           window, stores the answers in sorted order and moves each group's
 *                           back to receive order in LDS (no scattered answer stores).
 * bf_shard_insert_test_chunks_packed_dev  one step's owner work: the insert windows (as
 *                           bf_shard_insert_chunks_dev) then the include? windows (as
 *                           bf_shard_test_chunks_packed_dev), in ONE pass over the shard where
 *                           both take their sorted forms (each region read once, its inserts
 *                           ORed in and written back, its include? probes tested against the
 *                           result); every answer sees every insert, as the two calls in order.
 *                           d_next_keys / d_next_offsets / n_next (n_next = 0: none): another key
 *                           batch whose SHA-1 words go to d_next_digests (16-byte aligned), hashed
 *                           by the same pass while it streams the shard — this rank's next include?
 *                           batch, which bf_route_chunks_digests_dev then routes without hashing.
 * bf_combine_chunks_packed_dev  requester: the include? answers from window w's answer bits
 *                           at d_packed + w*ceil(window_cap/8), through this rank's own
 *                           route directory and slots.  A window whose count exceeds
 *                           window_cap (overflowed: its entries were never all written, so the
 *                           owner skipped it) contributes no answers, and the keys routed
 *                           there answer 1: after ANY overflow on ANY rank the combined answers
 *                           are false positives the caller must discard and recompute through
 *                           a re-route (distributed.py replays the step through the synced
 *                           exchange).  The same holds for bf_combine_windows[_packed]_dev.
 * bf_route_chunks_digests_dev   bf_route_chunks_dev from the keys' SHA-1 words (16-byte
 *                           aligned uint32[4] per key, as bf_hash_many_dev writes them).
 * bf_shard_test_chunks_hash_dev bf_shard_test_chunks_dev that also writes the SHA-1 words of
 *                           another key batch (this rank's next include? batch) to
 *                           d_next_digests: the owner test is latency-bound, so its waves hash
 *                           between their probe rounds (ruby.rb:41-47 per key, as
 *                           bf_hash_many_dev; the next step then routes from the words). */
int  bf_route_chunk_info(const bf_handle* h, uint64_t n_bound, uint64_t* tiles, uint64_t* dir_bytes,
                         uint32_t* superbins /* nullable: the owner superbins per window */);
int  bf_route_chunks_dev(bf_handle* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                         uint32_t* d_send /* nwin*window_cap */, uint16_t* d_slot16 /* nullable */,
                         uint64_t window_cap, uint64_t* d_counts /* nwin */, uint8_t* d_dir /* nwin*dir_bytes */,
                         uint64_t dir_bytes, uint64_t tiles, void* stream);
int  bf_shard_insert_chunks_dev(bf_handle* h, const uint32_t* d_recv, uint64_t window_cap, uint32_t nsrc,
                                const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles, const uint64_t* d_counts,
                                uint32_t count_stride, uint32_t* d_any_new /* nullable */, void* stream);
int  bf_shard_test_chunks_dev(bf_handle* h, const uint32_t* d_recv, uint64_t window_cap, uint32_t nsrc,
                              const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles, const uint64_t* d_counts,
                              uint32_t count_stride, uint8_t* d_bits, void* stream);
int  bf_shard_test_chunks_packed_dev(bf_handle* h, const uint32_t* d_recv, uint64_t window_cap, uint32_t nsrc,
                                     const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles,
                                     const uint64_t* d_counts, uint32_t count_stride,
                                     uint8_t* d_packed /* nsrc*nh*ceil(window_cap/8) */, void* stream);
int  bf_shard_insert_test_chunks_packed_dev(bf_handle* h, const uint32_t* d_ins_recv, const uint8_t* d_ins_dir,
                                            const uint64_t* d_ins_counts, const uint32_t* d_tst_recv,
                                            const uint8_t* d_tst_dir, const uint64_t* d_tst_counts,
                                            uint64_t window_cap, uint32_t nsrc, uint64_t dir_bytes, uint64_t tiles,
                                            uint32_t count_stride, uint32_t* d_any_new /* nullable */,
                                            uint8_t* d_packed, const uint8_t* d_next_keys,
                                            const uint64_t* d_next_offsets, uint64_t n_next,
                                            uint32_t* d_next_digests, void* stream);
int  bf_combine_chunks_packed_dev(bf_handle* h, const uint8_t* d_packed, const uint16_t* d_slot16,
                                  uint64_t window_cap, const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles,
                                  const uint64_t* d_counts /* nwin */, uint64_t n, uint8_t* d_out, void* stream);
int  bf_route_chunks_digests_dev(bf_handle* h, const uint32_t* d_digests, uint64_t n,
                                 uint32_t* d_send, uint16_t* d_slot16 /* nullable */, uint64_t window_cap,
                                 uint64_t* d_counts, uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles,
                                 void* stream);
int  bf_shard_test_chunks_hash_dev(bf_handle* h, const uint32_t* d_recv, uint64_t window_cap, uint32_t nsrc,
                                   const uint8_t* d_dir, uint64_t dir_bytes, uint64_t tiles,
                                   const uint64_t* d_counts, uint32_t count_stride, uint8_t* d_bits,
                                   const uint8_t* d_next_keys, const uint64_t* d_next_offsets, uint64_t n_next,
                                   uint32_t* d_next_digests, void* stream);
int  bf_shard_insert_dev(bf_handle* h, const void* d_local /* uint64 or uint32 (ROUTE32) */, uint64_t count,
                         uint32_t* d_any_new /* nullable */, void* stream);
int  bf_shard_test_dev(bf_handle* h, const void* d_local, uint64_t count, uint8_t* d_bits,
                       void* stream);
int  bf_combine_dev(bf_handle* h, const uint8_t* d_bits, const uint32_t* d_slot, uint64_t n,
                    uint8_t* d_out, void* stream);
/* The shard's bytes in local layout (local_bits/8 bytes, untrimmed); the caller
 * interleaves shards block by block to rebuild the Redis string. */
int  bf_shard_export(bf_handle* h, uint8_t* buf, uint64_t cap, uint64_t* len_out);
int  bf_shard_import(bf_handle* h, const uint8_t* buf, uint64_t len, uint32_t mode);

/* ---- the Lua driver's scalable layout (lib/bloomfilter_driver/lua.rb,
 *      vendor/assets/lua/add.lua + check.lua), device-resident.
 *
 *   bf_lua_create        Lua#initialize (lua.rb:14-17): entries = options[:size],
 *                        precision = options[:error_rate]; no layer exists yet
 *   bf_lua_insert_many   add.lua, one EVALSHA per key, in batch order: the item goes to
 *                        layer index(count + 1) and INCRs the count iff it set a new bit
 *                        (add.lua:6-54); per_key_new[j] = that INCR; *new_layers bit n-1
 *                        = layer n got a new item (the keys add.lua:52 EXPIREs)
 *   bf_lua_insert_many_changes  the same, plus every bit the batch flipped 0 -> 1 (each once)
 *                        as (layer << 58) | offset in out_bits[0 .. *count): the SETBITs
 *                        add.lua:43-47 issued that changed a layer string, which write-through
 *                        replays; *count > cap: BF_ERANGE after the insert is applied
 *   bf_lua_include_many  check.lua: 0 without a count, else any of layers 1..index(count)
 *                        holding all of its k_n bits (check.lua:1-61)
 *   bf_lua_clear         lua.rb:28-30 (KEYS name:* + DEL): layers and count dropped
 *   bf_lua_get/set_count KEYS[1]:count;  bf_lua_export/import_layer  KEYS[1]:n (SETBIT layout)
 *   bf_lua_layer_params  add.lua:16-25: bits and k of layer n (host only, no device)
 *   bf_lua_index         add.lua:13-15 / check.lua:9-11: the layer of a count (host only)
 *   bf_lua_insert_many_dev / bf_lua_include_many_dev   the same two ops on device-resident
 *                        keys (bf_insert_many_dev's layout: 16 B readable past offsets[n]) on
 *                        the caller's stream (NULL: the null stream), per-key flags and answers
 *                        in device memory.  The insert returns with the count updated (the host
 *                        picks each chunk's layer from it: one 8-byte read per chunk); include?
 *                        returns once enqueued.  Calls on different streams are ordered.
 *   bf_lua_profile / bf_lua_profile_read   per-kernel HIP-event timing as bf_profile, names
 *                        "lua_seq_candidates[L<n>]", "lua_seq_mark[L<n>]", "lua_count[L<n>]"
 *                        (per layer n) and "lua_check" */
typedef struct bf_lua bf_lua;
int  bf_lua_create(double entries, double precision, const bf_config* cfg /* device only */, bf_lua** out);
int  bf_lua_destroy(bf_lua* h);
const char* bf_lua_last_error(const bf_lua* h);   /* h == NULL: last error of bf_lua_create */
int  bf_lua_insert_many(bf_lua* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n,
                        uint8_t* per_key_new /* nullable */, uint64_t* new_layers /* nullable */);
int  bf_lua_insert_many_changes(bf_lua* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n,
                                uint8_t* per_key_new /* nullable */, uint64_t* new_layers /* nullable */,
                                uint64_t* out_bits, uint64_t cap, uint64_t* count);
#define BF_LUA_LAYER_SHIFT 58   /* out_bits of bf_lua_insert_many_changes: layer << 58 | offset */
int  bf_lua_include_many(bf_lua* h, const uint8_t* key_bytes, const uint64_t* offsets, uint64_t n,
                         uint8_t* out);
int  bf_lua_insert_many_dev(bf_lua* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                            uint8_t* d_per_key_new /* nullable */, uint64_t* new_layers /* nullable */,
                            void* stream);
int  bf_lua_include_many_dev(bf_lua* h, const uint8_t* d_key_bytes, const uint64_t* d_offsets, uint64_t n,
                             uint8_t* d_out, void* stream);
int  bf_lua_profile(bf_lua* h, uint32_t enable);
int  bf_lua_profile_read(bf_lua* h, char* names, double* total_ms, uint64_t* launches, uint32_t cap,
                         uint32_t* n_out, uint32_t reset);
int  bf_lua_clear(bf_lua* h);
int  bf_lua_get_count(const bf_lua* h, uint64_t* count);
int  bf_lua_set_count(bf_lua* h, uint64_t count);
int  bf_lua_layers(const bf_lua* h, uint32_t* nlayers);
int  bf_lua_export_layer(bf_lua* h, uint32_t layer, uint8_t* buf, uint64_t cap, uint64_t* len_out);
int  bf_lua_import_layer(bf_lua* h, uint32_t layer, const uint8_t* buf, uint64_t len);
int  bf_lua_layer_params(double entries, double precision, uint32_t layer, uint64_t* bits, uint32_t* k);
int  bf_lua_index(double entries, uint64_t count, uint32_t* layer);

/* ---- one key's k offsets without a filter (Ruby#indexes_for, ruby.rb:41-55): computed
 *      by the same device kernel as bf_indexes_many, on the calling thread's current
 *      HIP device; out holds k uint64.  m = 0 or k = 0: BF_EINVAL (the reference raises
 *      ZeroDivisionError at ruby.rb:51).  Not a hot path: it allocates per call.
 *      Errors read back through bf_last_error(NULL). */
int  bf_indexes(const uint8_t* key, uint64_t len, uint64_t m_bits, uint32_t k, uint64_t* out);

/* ---- sizing helpers with the facade's exact semantics (bloomfilter.rb:50-58).
 *      bf_optimal_m returns BF_OPTIMAL_M_INVALID when the result is not a finite int64
 *      (error_rate 0 -> Infinity: the reference raises FloatDomainError at Float#round). */
#define BF_OPTIMAL_M_INVALID INT64_MIN
int64_t bf_optimal_m(double n, double error_rate);
int64_t bf_optimal_k(int64_t n, int64_t m_bits);     /* Integer n: floor division, 0 -> 1 */

#ifdef __cplusplus
}
#endif
#endif /* BFHIP_H */
