// Static DDP bucket plan over a flat gradient arena (host C++).
#pragma once
#include <cstddef>
#include <vector>

namespace ddp_amd {

struct BucketSpec {
  int first_param, last_param;  // [first, last) in parameter order
  size_t offset, count;         // element range in the arena
};

// Buckets in REVERSE parameter order (the order gradients become ready in backward).
// cap_first_bytes limits the first bucket (DDP uses 1 MiB so communication starts early).
std::vector<BucketSpec> plan_buckets(const std::vector<size_t>& offsets,
                                     const std::vector<size_t>& numels, size_t elem_bytes,
                                     size_t cap_bytes, size_t cap_first_bytes);

}  // namespace ddp_amd
