// DDP bucket plan + launch state machine (pure host C++, no HIP/RCCL: unit-tested under
// ASan/UBSan, tests/test_aux_subsystems.py). Reference parity: torch DDP's bucket assignment in
// reverse parameter order with a small first bucket, and its rebuild after iteration 0
// (SURVEY.md §2.B N5, §2.E).
#include "buckets.h"

#include <algorithm>
#include <stdexcept>
#include <string>

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

BucketScheduler::BucketScheduler(std::vector<BucketSpec> buckets, int n_params)
    : buckets_(std::move(buckets)) {
  if (n_params < 0) throw std::runtime_error("negative parameter count");
  bucket_of_param_.assign(n_params, -1);
  for (size_t b = 0; b < buckets_.size(); ++b) {
    const auto& s = buckets_[b];
    if (s.first_param < 0 || s.last_param > n_params || s.first_param >= s.last_param)
      throw std::runtime_error("bucket " + std::to_string(b) + " has a bad parameter range");
    for (int p = s.first_param; p < s.last_param; ++p) {
      if (bucket_of_param_[p] != -1) throw std::runtime_error("parameter in two buckets");
      bucket_of_param_[p] = (int)b;
    }
  }
  for (int p = 0; p < n_params; ++p)
    if (bucket_of_param_[p] < 0) throw std::runtime_error("parameter in no bucket");
  order_.resize(buckets_.size());
  for (size_t b = 0; b < buckets_.size(); ++b) order_[b] = (int)b;
  prepare();
}

void BucketScheduler::prepare() {
  pending_.assign(buckets_.size(), 0);
  for (size_t b = 0; b < buckets_.size(); ++b)
    pending_[b] = buckets_[b].last_param - buckets_[b].first_param;
  ready_.assign(buckets_.size(), 0);
  seen_.assign(bucket_of_param_.size(), 0);
  seq_.clear();
  log_.clear();
  next_launch_ = 0;
  marked_ = 0;
}

std::vector<int> BucketScheduler::launchable() {
  std::vector<int> out;
  while (next_launch_ < (int)order_.size() && ready_[order_[next_launch_]]) {
    const int b = order_[next_launch_++];
    out.push_back(b);
    log_.emplace_back(b, marked_);
  }
  return out;
}

std::vector<int> BucketScheduler::mark(int p) {
  if (p < 0 || p >= (int)bucket_of_param_.size()) throw std::runtime_error("bad param index");
  if (seen_[p]) throw std::runtime_error("parameter marked ready twice in one backward");
  seen_[p] = 1;
  seq_.push_back(p);
  ++marked_;
  const int b = bucket_of_param_[p];
  if (--pending_[b] == 0) {
    ready_[b] = 1;
    return launchable();
  }
  return {};
}

std::vector<int> BucketScheduler::finish() {
  for (size_t b = 0; b < buckets_.size(); ++b)
    if (!ready_[b])
      throw std::runtime_error("bucket " + std::to_string(b) +
                               " has parameters whose gradient was never produced "
                               "(unused parameters are not supported)");
  std::vector<int> rest = launchable();
  last_seq_ = seq_;
  last_log_ = log_;
  prepare();
  return rest;
}

void BucketScheduler::set_launch_order(const std::vector<int>& order) {
  if (order.size() != buckets_.size()) throw std::runtime_error("launch order: wrong length");
  std::vector<char> hit(buckets_.size(), 0);
  for (int b : order) {
    if (b < 0 || b >= (int)buckets_.size() || hit[b])
      throw std::runtime_error("launch order is not a permutation of the buckets");
    hit[b] = 1;
  }
  if (next_launch_ != 0) throw std::runtime_error("launch order changed during a backward");
  order_ = order;
}

std::vector<int> BucketScheduler::order_from_ready(const std::vector<int>& ready_seq) const {
  std::vector<int> done_at(buckets_.size(), -1), left(buckets_.size(), 0);
  for (size_t b = 0; b < buckets_.size(); ++b)
    left[b] = buckets_[b].last_param - buckets_[b].first_param;
  for (size_t i = 0; i < ready_seq.size(); ++i) {
    const int p = ready_seq[i];
    if (p < 0 || p >= (int)bucket_of_param_.size()) throw std::runtime_error("bad param index");
    const int b = bucket_of_param_[p];
    if (--left[b] == 0) done_at[b] = (int)i;
  }
  std::vector<int> order(buckets_.size());
  for (size_t b = 0; b < buckets_.size(); ++b) {
    if (done_at[b] < 0) throw std::runtime_error("ready sequence does not complete every bucket");
    order[b] = (int)b;
  }
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return done_at[a] < done_at[b]; });
  return order;
}

}  // namespace ddp_amd
