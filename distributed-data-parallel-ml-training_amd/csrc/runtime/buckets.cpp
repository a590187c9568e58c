// Static DDP bucket plan (pure host C++, no HIP/RCCL: unit-tested under ASan/UBSan,
// tests/test_aux_subsystems.py). Reference parity: torch DDP's bucket assignment in reverse
// parameter order with a small first bucket.
#include "buckets.h"

namespace ddp_amd {

std::vector<BucketSpec> plan_buckets(const std::vector<size_t>& offsets,
                                     const std::vector<size_t>& numels, size_t elem_bytes,
                                     size_t cap_bytes, size_t cap_first_bytes) {
  std::vector<BucketSpec> out;
  const int n = (int)numels.size();
  int end = n;  // exclusive
  size_t bytes = 0;
  int start = n;
  auto flush = [&](int s, int e) {
    if (s >= e) return;
    BucketSpec b;
    b.first_param = s;
    b.last_param = e;
    b.offset = offsets[s];
    b.count = offsets[e - 1] + numels[e - 1] - offsets[s];
    out.push_back(b);
  };
  for (int p = n - 1; p >= 0; --p) {
    const size_t cap = out.empty() ? cap_first_bytes : cap_bytes;
    const size_t pb = numels[p] * elem_bytes;
    if (start < end && bytes + pb > cap) {
      flush(start, end);
      end = start;
      bytes = 0;
    }
    start = p;
    bytes += pb;
  }
  flush(start, end);
  return out;
}

}  // namespace ddp_amd
