// Multi-device codec (rs_new_multi): one codec per device ("part"), each
// owning a 64-byte-granular byte range of every shard, driven by one host
// worker thread per part.  Every Leopard operation is column-local
// (leopard16.go:778-792, leopard8.go:899-912), so the parts never exchange
// data: encode and reconstruct write disjoint byte ranges, verify ANDs the
// parts' verdicts on the host, and a reconstruct's error locators are computed
// once by the parent and handed to every part (no collective).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

struct rs_codec;

namespace rs {

enum class HostOp { Encode, Verify, Reconstruct };

// Error locators a reconstruct uses, computed by the caller instead of the
// codec: `ref` = they came from the reference-keyed GF(2^8) inversion cache
// (rs_set_reference_inversion_cache), so they are part of the plan-cache key,
// as for a single-device codec; otherwise they are the exact locators of the
// erasure pattern (which the pattern already keys).
struct ElExt {
    const std::vector<uint32_t> *el = nullptr;
    bool ref = false;
};

// codec.cpp: one part's share of a host-resident call.  The parent has
// validated the call; `shards` point at the part's byte range of every row.
int part_host_call(rs_codec *part, HostOp op, uint8_t *const *shards, uint64_t S, const std::vector<uint8_t> &present,
                   bool recover_all, int *ok, uint64_t *ticket, const ElExt *el);
// codec.cpp: the parent's locators for a reconstruct of the FULL shard size S
// (the reference's useBits depends on it, leopard8.go:475), from its caches.
int parent_error_locators(rs_codec *parent, const std::vector<uint8_t> &present, bool recover_all, uint64_t S,
                          ElExt &out);

// [lo, hi) of shard bytes owned by part g of n: 64-byte blocks dealt as evenly
// as possible, the first blocks % n parts taking one more (dist.byte_range).
void part_byte_range(uint64_t S, int g, int n, uint64_t &lo, uint64_t &hi);

struct Multi;
Multi *multi_create(std::vector<rs_codec *> parts, std::vector<int> devices);
void multi_destroy(Multi *m);
int multi_count(const Multi *m);
rs_codec *multi_part(Multi *m, int g, int *device);
// Host-resident encode / verify / reconstruct over the parts (the parent's
// mutex is held by the caller).  ticket != nullptr: asynchronous.
int multi_host(Multi *m, rs_codec *parent, HostOp op, uint8_t *const *shards, uint64_t S,
               const std::vector<uint8_t> &present, bool recover_all, int *ok, uint64_t *ticket);
int multi_ticket_wait(Multi *m, uint64_t ticket);
int multi_ticket_query(Multi *m, uint64_t ticket, int *done);
int multi_verify_result(Multi *m, uint64_t ticket, int *ok);
int multi_set_host_segment(Multi *m, size_t bytes);

}  // namespace rs
