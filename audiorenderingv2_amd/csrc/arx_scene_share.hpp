// arx_scene_share.hpp -- the rank path's scene hand-over (arx_group_set_scene with one GPU per
// process): rank 0 builds the tree, its byte image goes to every other rank.
//
// A collective that one rank skips hangs the others, so every rank enters every step whatever
// happened locally, and local failures travel inside the collectives:
//   1. rank 0 builds and serializes; the image size, or kShareFailed if the input check or the build
//      failed, is broadcast -- all ranks leave together on kShareFailed;
//   2. every rank stages a buffer of that size; an all-reduce (max) of "staging failed" flags lets
//      all ranks leave together if any rank could not;
//   3. the image is broadcast;
//   4. every other rank deserializes it; a second flag all-reduce makes a rank that could not fail
//      the call on every rank (otherwise the next render would wait in an all-reduce for it).
// The transport is a template parameter: RCCL on device buffers in the product (arx_group.cpp),
// threads in the host test (tests/cpp/scene_share_test.cpp).
#pragma once
#include <cstdint>
#include <vector>

namespace arx {

constexpr uint64_t kShareFailed = ~0ull;

enum class ShareResult {
    ok,
    root_failed,      // rank 0's input check or build failed (rank 0 knows why)
    staging_failed,   // some rank could not stage the image
    consume_failed,   // some rank could not read the image
    transport_failed  // a collective itself failed: the ranks may disagree from here on
};

// Chan provides (all collective over the group, rank 0 the root):
//   bool bcast_u64(uint64_t* v);
//   bool max_u64(uint64_t* v);
//   bool stage(uint64_t bytes);                       // local: make room for the image
//   bool bcast_bytes(uint8_t* host, uint64_t bytes);  // rank 0's host bytes into every rank's
// produce(std::vector<uint8_t>&) -> bool runs on rank 0 only, consume(const std::vector<uint8_t>&)
// -> bool on the others.
template <class Chan, class Produce, class Consume>
ShareResult share_from_rank0(Chan& ch, int rank, Produce&& produce, Consume&& consume) {
    std::vector<uint8_t> bytes;
    uint64_t size = 0;
    if (rank == 0) size = produce(bytes) ? (uint64_t)bytes.size() : kShareFailed;
    if (!ch.bcast_u64(&size)) return ShareResult::transport_failed;
    if (size == kShareFailed) return ShareResult::root_failed;
    uint64_t flag = 0;
    if (rank != 0) {
        try {
            bytes.resize(size);
        } catch (...) {
            flag = 1;
        }
    }
    if (!ch.stage(size)) flag = 1;
    if (!ch.max_u64(&flag)) return ShareResult::transport_failed;
    if (flag) return ShareResult::staging_failed;
    if (!ch.bcast_bytes(bytes.data(), size)) return ShareResult::transport_failed;
    flag = (rank != 0 && !consume(bytes)) ? 1 : 0;
    if (!ch.max_u64(&flag)) return ShareResult::transport_failed;
    return flag ? ShareResult::consume_failed : ShareResult::ok;
}

}  // namespace arx
