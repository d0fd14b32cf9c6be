// bf_multi.h — multi-device handles (bf_config.device_count > 0): one process, several
// GPUs, built from per-device bf_handles (bf_multi.cpp), and the bf_api.cpp internals they
// use on those handles.
#pragma once
#include "bfhip.h"

#include <stdint.h>

#include <string>
#include <vector>

struct BfMulti;

int bfm_create(uint64_t m_bits, uint32_t k, const bf_config& cfg, BfMulti** out, std::string* err);
void bfm_destroy(BfMulti* mh);
const char* bfm_last_error(const BfMulti* mh);
int bfm_info(const BfMulti* mh, uint64_t* m_bits, uint32_t* k, uint64_t* reach_bits, uint64_t* device_bytes);
int bfm_shard_info(const BfMulti* mh, uint32_t* shard_count, uint32_t* shard_index, uint32_t* block_log2,
                   uint64_t* local_bits);
int bfm_insert_many(BfMulti* mh, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* any_new,
                    uint8_t* per_key_new);
int bfm_include_many(BfMulti* mh, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint8_t* out);
int bfm_indexes_many(BfMulti* mh, const uint8_t* keys, const uint64_t* offsets, uint64_t n, uint64_t* out);
int bfm_clear(BfMulti* mh);
int bfm_sync(BfMulti* mh);
int bfm_export_redis(BfMulti* mh, uint8_t* buf, uint64_t cap, uint64_t* len_out);
int bfm_import_redis(BfMulti* mh, const uint8_t* buf, uint64_t len, uint32_t mode);
int bfm_track_dirty(BfMulti* mh, uint32_t enable);
int bfm_dirty_ranges(BfMulti* mh, uint64_t* ranges, uint32_t cap, uint32_t* n_out, uint64_t* redis_len,
                     uint32_t clear);
int bfm_export_range(BfMulti* mh, uint64_t offset, uint64_t len, uint8_t* buf);
int bfm_insert_plan(const BfMulti* mh, uint64_t n, uint32_t* binned, uint64_t* scratch_bytes);
int bfm_fail(BfMulti* mh, int code, const char* msg);

// bf_api.cpp internals, valid on shard handles too (offsets in the handle's local bytes)
int bfi_trimmed_len(bf_handle* h, uint64_t* len);   // last nonzero local byte + 1
int bfi_export_local(bf_handle* h, uint64_t offset, uint64_t len, uint8_t* buf);
int bfi_track_dirty(bf_handle* h, uint32_t enable);
// changed local byte ranges (offset, length pairs, clipped to the local trimmed length)
int bfi_dirty_local(bf_handle* h, std::vector<uint64_t>* ranges, bool clear);
