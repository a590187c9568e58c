// Native communication runtime — see comm.h.
#include "comm.h"
#include "../kernels/api.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace ddp_amd {

#define HIP_OK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess)                                                                \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) +     \
                               " at " __FILE__ ":" + std::to_string(__LINE__));          \
  } while (0)

#define KERNEL_OK(x)                                                                     \
  do {                                                                                   \
    const int k_ = (x);                                                                  \
    if (k_ != 0)                                                                         \
      throw std::runtime_error(std::string("kernel launch failed (") + std::to_string(k_) + \
                               ") at " __FILE__ ":" + std::to_string(__LINE__));         \
  } while (0)

#define NCCL_OK(x)                                                                       \
  do {                                                                                   \
    ncclResult_t r_ = (x);                                                               \
    if (r_ != ncclSuccess)                                                               \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r_) +   \
                               " at " __FILE__ ":" + std::to_string(__LINE__));          \
  } while (0)

// dtype codes shared with parallel/comm.py
static ncclDataType_t to_nccl(int dtype) {
  switch (dtype) {
    case 0: return ncclFloat32;
    case 1: return ncclBfloat16;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclInt64;
    case 5: return ncclUint8;
    default: throw std::runtime_error("unsupported dtype code");
  }
}
static size_t dtype_bytes(int dtype) {
  switch (dtype) {
    case 0: case 3: return 4;
    case 1: case 2: return 2;
    case 4: return 8;
    case 5: return 1;
    default: return 4;
  }
}
// op codes: 0 sum, 1 prod, 2 max, 3 min, 4 avg
static ncclRedOp_t to_op(int op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclAvg;
    default: throw std::runtime_error("unsupported reduction op");
  }
}

RcclComm::RcclComm(int rank, int world, const std::string& uid_bytes, int device)
    : rank_(rank), world_(world), device_(device) {
  HIP_OK(hipSetDevice(device));
  if (world > 1 || !uid_bytes.empty()) {
    if (uid_bytes.size() != sizeof(ncclUniqueId))
      throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid_bytes.data(), sizeof(id));
    NCCL_OK(ncclCommInitRank(&comm_, world, id, rank));
  }
}

RcclComm::~RcclComm() {
  if (comm_ && !aborted_) ncclCommDestroy(comm_);
  if (stage_) hipFree(stage_);
}

int RcclComm::count() const {
  if (!comm_) return 0;
  int n = 0;
  NCCL_OK(ncclCommCount(comm_, &n));
  return n;
}

int RcclComm::version() {
  int v = 0;
  NCCL_OK(ncclGetVersion(&v));
  return v;
}

std::string RcclComm::make_unique_id() {
  ncclUniqueId id;
  NCCL_OK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

void RcclComm::all_reduce(void* buf, size_t count, int dtype, int op, hipStream_t st) {
  if (comm_ == nullptr || count == 0) return;
  NCCL_OK(ncclAllReduce(buf, buf, count, to_nccl(dtype), to_op(op), comm_, st));
}

void RcclComm::broadcast(void* buf, size_t count, int dtype, int root, hipStream_t st) {
  if (comm_ == nullptr || count == 0) return;
  NCCL_OK(ncclBroadcast(buf, buf, count, to_nccl(dtype), root, comm_, st));
}

void RcclComm::all_gather(const void* send, void* recv, size_t count, int dtype, hipStream_t st) {
  if (comm_ == nullptr) {
    if (send != recv) KERNEL_OK(ddp_copy_bytes(recv, send, count * dtype_bytes(dtype), st));
    return;
  }
  NCCL_OK(ncclAllGather(send, recv, count, to_nccl(dtype), comm_, st));
}

void RcclComm::all_gather2(const void* send1, void* recv1, size_t count1, int dtype1,
                           const void* send2, void* recv2, size_t count2, int dtype2,
                           hipStream_t st) {
  if (comm_ == nullptr) {
    if (send1 != recv1) KERNEL_OK(ddp_copy_bytes(recv1, send1, count1 * dtype_bytes(dtype1), st));
    if (send2 != recv2) KERNEL_OK(ddp_copy_bytes(recv2, send2, count2 * dtype_bytes(dtype2), st));
    return;
  }
  NCCL_OK(ncclGroupStart());
  if (count1) NCCL_OK(ncclAllGather(send1, recv1, count1, to_nccl(dtype1), comm_, st));
  if (count2) NCCL_OK(ncclAllGather(send2, recv2, count2, to_nccl(dtype2), comm_, st));
  NCCL_OK(ncclGroupEnd());
}

void RcclComm::reduce_scatter(const void* send, void* recv, size_t count, int dtype, int op,
                              hipStream_t st) {
  if (comm_ == nullptr) {
    if (send != recv) KERNEL_OK(ddp_copy_bytes(recv, send, count * dtype_bytes(dtype), st));
    return;
  }
  NCCL_OK(ncclReduceScatter(send, recv, count, to_nccl(dtype), to_op(op), comm_, st));
}

void RcclComm::gather(const void* send, void* recv, size_t count, int dtype, int root,
                      hipStream_t st) {
  const size_t bytes = count * dtype_bytes(dtype);
  const ncclDataType_t dt = to_nccl(dtype);
  if (world_ == 1) {
    if (comm_ != nullptr && count > 0) {
      // single-rank live communicator (one-GPU box): the root's own slot travels through a
      // grouped self send/recv, so the point-to-point path of 2A runs exactly as on a node
      NCCL_OK(ncclGroupStart());
      NCCL_OK(ncclSend(send, count, dt, rank_, comm_, st));
      NCCL_OK(ncclRecv((char*)recv + (size_t)root * bytes, count, dt, rank_, comm_, st));
      NCCL_OK(ncclGroupEnd());
    } else if ((const char*)recv + (size_t)root * bytes != send) {
      KERNEL_OK(ddp_copy_bytes((char*)recv + (size_t)root * bytes, send, bytes, st));
    }
    return;
  }
  // the root's own slot: a copy KERNEL, not hipMemcpyAsync (a captured step must stay a graph of
  // kernel nodes; see ddp_copy_bytes)
  if (rank_ == root)
    KERNEL_OK(ddp_copy_bytes((char*)recv + (size_t)root * bytes, send, bytes, st));
  NCCL_OK(ncclGroupStart());
  if (rank_ == root) {
    for (int r = 0; r < world_; ++r)
      if (r != root) NCCL_OK(ncclRecv((char*)recv + (size_t)r * bytes, count, dt, r, comm_, st));
  } else {
    NCCL_OK(ncclSend(send, count, dt, root, comm_, st));
  }
  NCCL_OK(ncclGroupEnd());
}

void RcclComm::scatter(const void* send, void* recv, size_t count, int dtype, int root,
                       hipStream_t st) {
  const size_t bytes = count * dtype_bytes(dtype);
  const ncclDataType_t dt = to_nccl(dtype);
  if (world_ == 1) {
    if (comm_ != nullptr && count > 0 && (const char*)send + (size_t)root * bytes != recv) {
      NCCL_OK(ncclGroupStart());  // self send/recv (see gather)
      NCCL_OK(ncclSend((const char*)send + (size_t)root * bytes, count, dt, rank_, comm_, st));
      NCCL_OK(ncclRecv(recv, count, dt, rank_, comm_, st));
      NCCL_OK(ncclGroupEnd());
    } else if ((const char*)send + (size_t)root * bytes != recv) {
      KERNEL_OK(ddp_copy_bytes(recv, (const char*)send + (size_t)root * bytes, bytes, st));
    }
    return;
  }
  if (rank_ == root && (const char*)send + (size_t)root * bytes != recv)
    KERNEL_OK(ddp_copy_bytes(recv, (const char*)send + (size_t)root * bytes, bytes, st));
  NCCL_OK(ncclGroupStart());
  if (rank_ == root) {
    for (int r = 0; r < world_; ++r)
      if (r != root) NCCL_OK(ncclSend((const char*)send + (size_t)r * bytes, count, dt, r, comm_, st));
  } else {
    NCCL_OK(ncclRecv(recv, count, dt, root, comm_, st));
  }
  NCCL_OK(ncclGroupEnd());
}

void RcclComm::scatter_replicated(void* buf, size_t count, int dtype, int root, hipStream_t st) {
  if (count == 0) return;
  const ncclDataType_t dt = to_nccl(dtype);
  if (world_ == 1) {
    if (comm_ == nullptr) return;  // no communicator: the root already holds the data
    // single-rank live communicator (one-GPU box): the root's copy travels through a grouped
    // self send/recv into a staging buffer that starts as all-ones bytes (NaN for every float
    // dtype) and is copied back, so the receive half of 2A's point-to-point plane really runs
    // and a receive that wrote nothing shows up as NaN in buf (tests/test_gpu_rccl_self.py)
    const size_t bytes = count * dtype_bytes(dtype);
    if (bytes > stage_bytes_) {
      // growing the staging buffer is a hipMalloc / hipFree: illegal inside a stream capture.
      // Callers reserve the largest size before capturing (reserve_stage); refuse otherwise
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      HIP_OK(hipStreamIsCapturing(st, &cs));
      if (cs != hipStreamCaptureStatusNone)
        throw std::runtime_error("scatter_replicated: staging buffer must be reserved before "
                                 "graph capture (RcclComm::reserve_stage)");
      reserve_stage(bytes);
    }
    // fill + copy-back are kernels (a captured memset node did not order before its readers)
    KERNEL_OK(ddp_fill_bytes(stage_, 0xff, bytes, st));
    NCCL_OK(ncclGroupStart());
    NCCL_OK(ncclSend(buf, count, dt, rank_, comm_, st));
    NCCL_OK(ncclRecv(stage_, count, dt, rank_, comm_, st));
    NCCL_OK(ncclGroupEnd());
    KERNEL_OK(ddp_copy_bytes(buf, stage_, bytes, st));
    return;
  }
  NCCL_OK(ncclGroupStart());
  if (rank_ == root) {
    for (int r = 0; r < world_; ++r)
      if (r != root) NCCL_OK(ncclSend(buf, count, dt, r, comm_, st));
  } else {
    NCCL_OK(ncclRecv(buf, count, dt, root, comm_, st));
  }
  NCCL_OK(ncclGroupEnd());
}

void RcclComm::reserve_stage(size_t bytes) {
  if (bytes <= stage_bytes_) return;
  if (stage_) {
    HIP_OK(hipDeviceSynchronize());  // the old buffer may still be read by queued work
    HIP_OK(hipFree(stage_));
    stage_ = nullptr;
  }
  HIP_OK(hipMalloc(&stage_, bytes));
  stage_bytes_ = bytes;
}

void RcclComm::send(const void* buf, size_t count, int dtype, int peer, hipStream_t st) {
  NCCL_OK(ncclSend(buf, count, to_nccl(dtype), peer, comm_, st));
}

void RcclComm::recv(void* buf, size_t count, int dtype, int peer, hipStream_t st) {
  NCCL_OK(ncclRecv(buf, count, to_nccl(dtype), peer, comm_, st));
}

int RcclComm::async_error() {
  if (!comm_) return 0;
  ncclResult_t r = ncclSuccess;
  ncclCommGetAsyncError(comm_, &r);
  return (int)r;
}

void RcclComm::abort() {
  if (comm_ && !aborted_) {
    ncclCommAbort(comm_);
    aborted_ = true;
  }
}

// ------------------------------------------------------------------ Reducer
Reducer::Reducer(RcclComm* comm, float* arena, std::vector<size_t> offsets,
                 std::vector<size_t> numels, size_t cap_bytes, size_t cap_first_bytes,
                 bool average)
    : comm_(comm), arena_(arena), offsets_(std::move(offsets)), numels_(std::move(numels)),
      sched_(plan_buckets(offsets_, numels_, sizeof(float), cap_bytes, cap_first_bytes),
             (int)numels_.size()),
      average_(average) {
  const size_t nb = sched_.buckets().size();
  contrib_.assign(nb, {});
  ready_ev_.assign(nb, {});
  done_ev_.resize(nb);
  done_stream_.assign(nb, nullptr);
  for (size_t b = 0; b < nb; ++b)
    HIP_OK(hipEventCreateWithFlags(&done_ev_[b], hipEventDisableTiming));
  // comm stream at the highest stream priority: HIP keeps high-priority streams on their own
  // hardware queues, so the collectives cannot end up behind the backward on a queue shared
  // round-robin with the compute stream (normal priority: 0 us of overlap measured,
  // profiles/r2_pipelined_ddp.md)
  int lo = 0, hi = 0;
  HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  (void)lo;
  HIP_OK(hipStreamCreateWithPriority(&comm_stream_, hipStreamNonBlocking, hi));
  prepare();
}

void Reducer::set_comm_dtype(int dtype) {
  if (dtype != 0 && dtype != 1) throw std::runtime_error("gradient comm dtype: 0 = fp32, 1 = bf16");
  comm_bf16_ = dtype == 1;
  if (comm_bf16_ && !stage_) {
    size_t n = 0;
    for (const auto& b : sched_.buckets()) n = std::max(n, b.offset + b.count);
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&stage_), (n + 64) * sizeof(unsigned short)));
  }
}

void Reducer::set_timing(bool on) {
  timing_ = on;
  if (on && t_start_.empty()) {
    t_start_.resize(done_ev_.size());
    t_end_.resize(done_ev_.size());
    for (size_t b = 0; b < done_ev_.size(); ++b) {
      HIP_OK(hipEventCreate(&t_start_[b]));
      HIP_OK(hipEventCreate(&t_end_[b]));
    }
  }
}

std::vector<std::pair<float, float>> Reducer::bucket_times(hipEvent_t ref) const {
  std::vector<std::pair<float, float>> out;
  for (size_t b = 0; b < t_start_.size(); ++b) {
    float a = 0.f, e = 0.f;
    HIP_OK(hipEventElapsedTime(&a, ref, t_start_[b]));
    HIP_OK(hipEventElapsedTime(&e, ref, t_end_[b]));
    out.emplace_back(a, e);
  }
  return out;
}

Reducer::~Reducer() {
  for (auto e : t_start_) hipEventDestroy(e);
  for (auto e : t_end_) hipEventDestroy(e);
  if (stage_) hipFree(stage_);
  for (auto& v : ready_ev_)
    for (auto e : v)
      if (e) hipEventDestroy(e);
  for (auto e : done_ev_) hipEventDestroy(e);
  if (comm_stream_) hipStreamDestroy(comm_stream_);
}

void Reducer::prepare() {
  sched_.prepare();
  for (auto& c : contrib_) c.clear();
}

void Reducer::mark_ready(int p, hipStream_t compute) {
  if (p < 0 || p >= sched_.n_params()) throw std::runtime_error("bad param index");
  auto& cs = contrib_[sched_.bucket_of(p)];
  if (std::find(cs.begin(), cs.end(), compute) == cs.end()) cs.push_back(compute);
  for (int b : sched_.mark(p)) launch(b);
}

// Buckets launch in the scheduler's launch order (plan order, or the rebuilt completion order)
// so every rank issues collectives identically. The comm stream waits on an event recorded NOW
// on every stream that produced part of the bucket: that covers each producer's work up to its
// last contribution.
void Reducer::launch(int b) {
  const BucketSpec& bs = sched_.buckets()[b];
  auto& evs = ready_ev_[b];
  // overlap: the collective runs on the comm stream; inline: on the stream that completed the
  // bucket (stream order = no cross-stream edge in a captured graph)
  // (world 1 without emulation has no collective: nothing to order against)
  const bool real = comm_->live() || emulate_;
  hipStream_t target = (overlap_ && real) ? comm_stream_ : contrib_[b].back();
  for (size_t i = 0; i < contrib_[b].size(); ++i) {
    if (contrib_[b][i] == target) continue;
    if (i >= evs.size()) evs.resize(i + 1, nullptr);
    if (!evs[i]) HIP_OK(hipEventCreateWithFlags(&evs[i], hipEventDisableTiming));
    HIP_OK(hipEventRecord(evs[i], contrib_[b][i]));
    HIP_OK(hipStreamWaitEvent(target, evs[i], 0));
  }
  float* buf = arena_ + bs.offset;
  if (timing_) HIP_OK(hipEventRecord(t_start_[b], target));
  if (real && comm_bf16_) {
    unsigned short* sb = stage_ + bs.offset;
    if (ddp_pack_bf16(buf, bs.count, sb, target) != 0)
      throw std::runtime_error("bf16 pack of a gradient bucket failed (alignment)");
    if (comm_->live()) comm_->all_reduce(sb, bs.count, /*bf16*/ 1, average_ ? 4 : 0, target);
    if (ddp_unpack_bf16(sb, bs.count, buf, target) != 0)
      throw std::runtime_error("bf16 unpack of a gradient bucket failed (alignment)");
  } else if (comm_->live()) {
    comm_->all_reduce(buf, bs.count, /*fp32*/ 0, average_ ? 4 : 0, target);
  } else if (emulate_) {
    // world 1 stand-in for the collective (graph-structure / overlap studies on one GPU):
    // one pass over the bucket, like the reduction kernel of an all-reduce
    if (emulate_gbps_ > 0.0) {
      const float us = (float)(4.0 * bs.count / (emulate_gbps_ * 1e3));
      if (ddp_comm_standin(buf, bs.count, emulate_blocks_, us, 1.0f, 1, target) != 0)
        throw std::runtime_error("emulated collective launch failed");
    } else {
      for (int i = 0; i < emulate_passes_; ++i)
        if (ddp_scale(buf, bs.count, 1.0f, target) != 0)
          throw std::runtime_error("emulated collective launch failed");
    }
  }
  done_stream_[b] = target;
  if (timing_) HIP_OK(hipEventRecord(t_end_[b], target));
  HIP_OK(hipEventRecord(done_ev_[b], target));
  if (debug_sync_) HIP_OK(hipStreamSynchronize(target));
}

void Reducer::finalize(hipStream_t compute) {
  for (int b : sched_.finish()) launch(b);  // throws if a parameter never got a gradient
  for (size_t b = 0; b < done_stream_.size(); ++b)
    if (done_stream_[b] != compute) HIP_OK(hipStreamWaitEvent(compute, done_ev_[b], 0));
  for (auto& c : contrib_) c.clear();
}

}  // namespace ddp_amd
