// DDP bucket plan + readiness/launch state machine over a flat gradient arena (host C++, no
// HIP/RCCL: unit-tested under ASan/UBSan and driven from Python on CPU against the Python twin,
// tests/test_aux_subsystems.py, tests/test_bucket_scheduler_cpu.py).
#pragma once
#include <cstddef>
#include <utility>
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

// Readiness counters and launch order of one backward pass.
//   mark(p)        parameter p's gradient is complete; returns the buckets that may be launched
//                  NOW, in launch order (a bucket is launched only after every bucket before it
//                  in the launch order, so all ranks issue collectives identically);
//   finish()       end of backward: every parameter must have been marked; records the
//                  observed ready order and resets for the next pass;
//   rebuild()      torch DDP's post-iteration-0 rebuild in this design's terms: buckets stay
//                  contiguous arena slices (zero-copy), but their LAUNCH order becomes the order
//                  in which they completed in the observed backward (ready_order()), so a
//                  finished bucket never waits behind one that completes later. Every rank
//                  must apply the same order (the caller broadcasts rank 0's).
class BucketScheduler {
 public:
  BucketScheduler(std::vector<BucketSpec> buckets, int n_params);
  const std::vector<BucketSpec>& buckets() const { return buckets_; }
  int n_params() const { return (int)bucket_of_param_.size(); }
  int bucket_of(int p) const { return bucket_of_param_.at(p); }
  std::vector<int> mark(int p);
  std::vector<int> finish();
  void prepare();
  bool complete(int b) const { return ready_[b] != 0; }
  int launched() const { return next_launch_; }
  int marked() const { return marked_; }
  const std::vector<int>& launch_order() const { return order_; }
  void set_launch_order(const std::vector<int>& order);  // throws unless a permutation
  // launch order implied by a ready sequence of parameter indices (bucket completion order;
  // ties keep plan order)
  std::vector<int> order_from_ready(const std::vector<int>& ready_seq) const;
  const std::vector<int>& ready_order() const { return last_seq_; }
  // (bucket, parameters marked when it was launched) of the last completed pass
  const std::vector<std::pair<int, int>>& launch_log() const { return last_log_; }

 private:
  std::vector<int> launchable();
  std::vector<BucketSpec> buckets_;
  std::vector<int> bucket_of_param_;
  std::vector<int> pending_;
  std::vector<char> ready_;
  std::vector<char> seen_;
  std::vector<int> order_;
  std::vector<int> seq_, last_seq_;
  std::vector<std::pair<int, int>> log_, last_log_;
  int next_launch_ = 0;
  int marked_ = 0;
};

}  // namespace ddp_amd
