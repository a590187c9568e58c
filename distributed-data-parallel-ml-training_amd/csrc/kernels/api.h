// C ABI of the gfx950 kernel library: argument structs + launcher declarations.
// Shared by the .hip kernel translation units and the pybind11 binding (bind.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ddp_amd {

// BatchNorm statistics are accumulated into kStatRep replicas [rep][2][C] (sum, sum of squares)
// to spread float-atomic contention over many addresses; consumers sum the replicas in replica
// order. Deterministic-statistics build (_build.py variant "det": -DDDP_AMD_DETERMINISTIC,
// loaded with DDP_AMD_DETERMINISTIC=1): every block owns a replica of its own (block id <
// kStatRep), so each address receives exactly one float add onto zero and the consumers' fixed
// order makes the statistics — and the whole step — bitwise reproducible (test mode; a block id
// beyond kStatRep poisons replica 0 with NaN so it cannot pass silently).
#ifdef DDP_AMD_DETERMINISTIC
constexpr int kStatRep = 4096;
constexpr bool kDeterministic = true;
#else
constexpr int kStatRep = 16;
constexpr bool kDeterministic = false;
#endif

struct ConvGeom {
  int N, H, W, C;     // input (NHWC, C % 8 == 0)
  int K;              // output channels
  int R, S, stride, pad;
  int P, Q;           // output spatial
  int Creal;          // real (unpadded) input channels — weight-gradient layout
  int wkrsc;          // fp32 weight / weight-gradient layout: 0 = [K][Cr][R][S], 1 = [K][R][S][Cr]
};

struct BnArgs {
  int N, H, W, C;               // z / pre-pool shape
  int pool;                     // 0: none, 1: 2x2 stride-2 max-pool
  int relu;                     // apply ReLU
  float eps;
  const unsigned short* z;      // conv output (bf16)
  const unsigned short* res;    // optional residual added before ReLU (bf16, same shape as z)
  const float* stats;           // [kStatRep][2][C] sum, sumsq over N*H*W
  const float* gamma;           // [C]
  const float* beta;            // [C]
  unsigned short* out;          // forward output (bf16, pooled shape)
  const unsigned short* dout;   // backward: grad wrt block output (pooled shape)
  float* sums;                  // backward scratch [kStatRep][2][C]: S1 = sum dy_bn, S2 = sum dy_bn*xhat
  unsigned short* dz;           // backward: grad wrt conv output
  unsigned short* dres;         // backward: grad wrt residual (optional)
  float* dgamma;                // grad arena slices (accumulated)
  float* dbeta;
  float* dbias;                 // conv bias grad (optional)
  float* running_mean;          // optional (track_running_stats=True): updated in training fwd
  float* running_var;
  float momentum;
  int use_running;              // eval with running statistics instead of batch statistics
  float* coef;                  // [6][C] scale, shift, mean, invstd (fwd) and k1, k2 (bwd); the
                                // backward reads the table its forward wrote
  int sums_ready;               // backward: sums already accumulated (BnBwdFuse in the next
                                // layer's dgrad) -> finalize + apply only
  unsigned char* mask;          // residual blocks (res, ReLU, no pool): [N*H*W][C/8] bytes, bit e
                                // of a channel group = its pre-ReLU value was > 0. Forward writes
                                // it; the backward reads it INSTEAD of the residual (1/16 of the
                                // bytes) — the residual only ever served the ReLU mask there
  // Projection shortcut folded in (ResNet's downsample Conv -> BN, no ReLU): res is the
  // shortcut conv's PRE-BatchNorm output and these name its BatchNorm, so the shortcut's BN
  // output is never stored and its backward rides in this block's passes (ddp_bn_act_*_res)
  float* rcoef;                 // its coef table [6][C]
  float* rsums;                 // backward: its S2 row ([kStatRep][2][C]; S1 is this BN's own)
  unsigned short* rdz;          // backward: grad wrt the shortcut conv output
  float* rdgamma;               // its grad arena slices (accumulated)
  float* rdbeta;
  int red_gb;                   // backward reduce launch: channel groups per block (0 = min(C/8, 256))
};

// BatchNorm-backward statistics fused into a conv dgrad: the dgrad output IS the gradient at the
// output of the preceding Conv->BN->ReLU(->2x2 max-pool) block, so its epilogue can accumulate
// that block's backward sums S1 = sum dy_bn, S2 = sum dy_bn * xhat (recomputing the ReLU mask /
// pool routing from the block's conv output z) — the block's BN backward then skips its reduce
// pass (BnArgs::sums_ready).
struct BnBwdFuse {
  const unsigned short* z;  // preceding block's conv output [N][Hz][Wz][C] (bf16, pre-pool)
  const float* coef;        // its coefficient table [6][C] (scale, shift, mean, invstd, ..)
  float* sums;              // its backward sums [kStatRep][2][C] (zeroed per forward)
  int pool, relu;           // 2x2/s2 max-pool between z and the dgrad output; ReLU
  int Hz, Wz;               // z spatial dims (2x the dgrad output's when pooled)
  // VGG input block (conv_l0.hip, z never stored): ``code`` = the forward's per-window gradient
  // destinations (lane-major bytes, conv_l0.hip Args::code) and ``z`` = its zw (the winner's z,
  // POOLED shape): the sums are l0_sums_kernel's, taken in the dgrad's split-K finish only
  const unsigned* code;
};

// The COMPLETE BatchNorm backward of that preceding block fused into a small dgrad's split-K
// finish (conv_igemm.hip splitk_finish_bnbwd_kernel): with the sums complete inside each block,
// the finish also writes the block's dgamma / dbeta and its conv-output gradient dz — the dgrad
// output itself is never stored and the block skips its BN backward (finalize + apply).
struct BnBwdApply {
  unsigned short* dz;       // gradient wrt the preceding block's conv output [N][Hz][Wz][C]
  float* dgamma;            // its BatchNorm weight / bias gradients (accumulated, may be null)
  float* dbeta;
};

// Training-mode BatchNorm (+ReLU, +2x2/s2 max-pool) forward fused into the split-K finish of a
// small conv GEMM (conv_igemm.hip splitk_finish_bnfwd_kernel): one block owns 16 channels over
// every GEMM row, so the batch statistics are complete inside the block — no atomics, no
// finalize, no separate apply pass. The conv output z is still written (the backward reads it).
struct BnFwdFuse {
  const float* gamma;       // [C]
  const float* beta;        // [C]
  float eps;
  int relu, pool;
  float* coef;              // [6][C] table for the backward: scale, shift, mean, invstd
  unsigned short* y;        // block output [N][P/pool][Q/pool][C] (bf16)
  int P, Q;                 // conv output spatial dims (pre-pool)
};

// Fused input of the tap-reuse 3x3 forward (conv_tr.hip): the conv input is
// [2x2/s2 max-pool](ReLU(BatchNorm(z))) of the preceding block, computed while the input patch
// is loaded (the preceding block's bn_act_fwd launch disappears). Training-mode batch
// statistics only (no running statistics).
struct TrFwdIn {
  const unsigned short* z;  // preceding block's conv output [N][Hz][Wz][C] (Hz = 2H when pooled)
  const float* stats;       // its statistics replicas [kStatRep][2][C]
  const float* gamma;       // [C]
  const float* beta;
  float eps;
  int relu, pool;
  float* coef;              // [6][C] coefficient table written for its backward
  unsigned short* y;        // materialised conv input [N][H][W][C] (the wgrad operand)
};

// The last Conv->BN->ReLU->2x2-pool block over 2x2 images computed inside the classifier head's
// forward (linear_ce.hip): x = the pooled features it writes
struct HeadBnIn {
  const unsigned short* z;  // [B][2][2][F] the block's conv output (bf16)
  const float* stats;       // its statistics replicas [kStatRep][2][F]
  const float* gamma;
  const float* beta;
  float eps;
  int relu;
  float* coef;              // [6][F]: block 0 writes scale, shift, mean, invstd
  unsigned short* y;        // [B][F] pooled features (written)
};

// SGD in the backward (conv_igemm.hip wgrad_finish_krsc_body): the optimizer step of one conv
// weight, applied by the WGRAD split-K finish that produces its complete gradient
// (torch.optim.SGD, dampening 0: d = g * grad_scale + wd * p; buf = momentum * buf + d;
// d = nesterov ? d + momentum * buf : buf; p -= lr * d) + the bf16 forward operand copy.
struct SgdFuse {
  float* p;             // fp32 master weight, same [K][R][S][Cr] index order as the gradient
  float* buf;           // its momentum buffer
  unsigned short* wc;   // bf16 forward operand [K][R][S][C] (C >= Cr, pad channels untouched)
  float lr, momentum, wd, grad_scale;
  int nesterov;
};

// VGG input block (conv_l0.hip): conv 3x3 (8 padded channels -> 64) + train-mode BN + ReLU +
// 2x2 max-pool with z recomputed instead of stored
struct L0Io {
  const void* x;        // [N][H][W][8] bf16
  const void* wc;       // [64][3][3][8] bf16
  const float* bias;    // [64] or null
  float eps;
  int relu;
  float* stats;         // [kStatRep][2][64] (zeroed per step)
  const float* gamma;
  const float* beta;
  float* coef;          // [6][64] scale, shift, mean, invstd, k1, k2
  void* y;              // [N][H/2][W/2][64] bf16 (forward output)
  const void* dy;       // [N][H/2][W/2][64] bf16 (backward input)
  float* sums;          // [kStatRep][2][64] (zeroed per step)
  void* dz;             // [N][H][W][64] bf16 (backward output)
  void* code;           // [N][H/2][W/2][64] uint8: per pooled value, where its gradient goes
  void* zw;             // [N][H/2][W/2][64] bf16: z of that pixel (forward -> backward sums)
  float* dgamma;
  float* dbeta;
  int sums_ready;       // backward: ``sums`` already accumulated (the next block's dgrad finish,
                        // BnBwdFuse::code) -> the dz pass only
};

struct PackDesc {
  const float* p;          // fp32 master [K][Cr][R][S] (krsc == 0) or [K][R][S][Cr] (krsc == 1)
  unsigned short* wc;      // bf16 [K][R][S][C]   (may be null)
  unsigned short* wt;      // bf16 [C][R][S][K]   (may be null)
  int K, Cr, C, R, S;
  int krsc;
};

struct AugArgs {
  const unsigned char* images;  // [Nd][H][W][3] uint8
  const int* labels;            // [Nd]
  const int* indices;           // [L] sample order for this rank/epoch
  const int* cursor;            // device batch counter (may be null -> 0)
  int L, B, H, W, Cp, pad, flip;
  uint32_t seed, epoch;
  float mean[3], inv_std[3];
  unsigned short* x;            // [B][H][W][Cp] bf16
  long long* y;                 // [B]
  float* zero;                  // optional side job: zero this many floats (the next forward's
  size_t zero_n;                //   per-step accumulator scratch, ops/common.py StepScratch)
};

}  // namespace ddp_amd

extern "C" {
int ddp_conv_fwd(const ddp_amd::ConvGeom* g, const void* x, const void* wc, const float* bias,
                 void* y, float* stats, float* ws, size_t ws_elems, int splits, hipStream_t st);
// as ddp_conv_fwd; when the GEMM is split-K and small enough, its finish also runs the BatchNorm
// forward of ``bn`` (returns 1: y and the coefficient table are written, no bn_act_fwd needed),
// else the plain conv with statistics (returns 0); negative: invalid arguments; >= 2: HIP error
// (rc - 2)
int ddp_conv_fwd_bn(const ddp_amd::ConvGeom* g, const void* x, const void* wc, const float* bias,
                    void* z, float* stats, float* ws, size_t ws_elems, const ddp_amd::BnFwdFuse* bn,
                    hipStream_t st);
// split-K finish of a forward GEMM computed elsewhere (slabs [splits][M][K] -> z + statistics,
// or the BatchNorm-fused finish with ``bn``); returns the HIP error code
int ddp_conv_fwd_finish(const ddp_amd::ConvGeom* g, float* ws, int splits, const float* bias,
                        void* z, float* stats, const ddp_amd::BnFwdFuse* bn, int* bn_done,
                        hipStream_t st);
// 3x3/s1/p1 forward through the tap-reuse kernel (conv_tr.hip): 1 served (*bn_done as
// ddp_conv_fwd_bn), 0 not served (use ddp_conv_fwd[_bn]), < 0 invalid, >= 2 HIP error (rc - 2)
int ddp_conv_fwd_tr(const ddp_amd::ConvGeom* g, const void* x, const void* wc, const float* bias,
                    void* z, float* stats, float* ws, size_t ws_elems,
                    const ddp_amd::BnFwdFuse* bn, int* bn_done, const ddp_amd::TrFwdIn* in,
                    hipStream_t st);
int ddp_conv_tr_would_serve(const ddp_amd::ConvGeom* g, size_t ws_elems, int in_mode);
// tap-reuse policy: mode -1 clear table, 0/1 disable/enable (table entries), 4 enable with the
// heuristic for untabled shapes, 2 table entry (M, K, C, H) ->
// (bm, bn, splits, stages) (bm = 0: use the implicit-GEMM kernel), 3 force the same (sweeps)
void ddp_conv_tr_set(int mode, int M, int K, int C, int H, int bm, int bn, int splits, int stages);
int ddp_conv_tr_geometry(int BM, int N, int H, int W, int* out7);
// classifier-head dx fused with the preceding block's whole BN backward + dW / db in one launch
// (conv_igemm.hip linear_head_bwd_kernel): 1 launched, 0 not served, < 0 invalid, >= 2 HIP
// error (rc - 2)
int ddp_linear_head_bwd_bn(const float* dl, const float* W, const void* x, int B, int F, int J,
                           const float* gscale, const ddp_amd::BnBwdFuse* bn,
                           const ddp_amd::BnBwdApply* ba, float* dW, float* db, hipStream_t st);
// row limit of the BN-fused split-K finishes (default 128)
void ddp_conv_bn_fuse_rows(int rows);
int ddp_conv_dgrad(const ddp_amd::ConvGeom* g, const void* dy, const void* wt, void* dx,
                   float* ws, size_t ws_elems, int splits, int accumulate, hipStream_t st);
// dx = result + (first gradient branch never stored: acc_dy through the ReLU mask bits acc_mask,
// bn_act.hip BnArgs::mask); stride 1 only; dx is written, not read
int ddp_conv_dgrad_acc(const ddp_amd::ConvGeom* g, const void* dy, const void* wt, void* dx,
                       float* ws, size_t ws_elems, int splits, const void* acc_dy,
                       const unsigned char* acc_mask, hipStream_t st);
// ba (optional): also run the preceding block's whole BN backward in the finish when the dgrad
// is split-K and small (*bn_done = 1: dz / dgamma / dbeta written, dx NOT written)
int ddp_conv_dgrad_bn(const ddp_amd::ConvGeom* g, const void* dy, const void* wt, void* dx,
                      float* ws, size_t ws_elems, int splits, const ddp_amd::BnBwdFuse* bn,
                      const ddp_amd::BnBwdApply* ba, int* bn_done, hipStream_t st);
int ddp_conv_wgrad(const ddp_amd::ConvGeom* g, const void* dy, const void* x, float* dw,
                   float* ws, size_t ws_elems, int splits, hipStream_t st);
int ddp_bn_act_fwd(const ddp_amd::BnArgs* a, hipStream_t st);
int ddp_bn_act_bwd(const ddp_amd::BnArgs* a, hipStream_t st);
// residual block with the projection shortcut's BatchNorm folded in (BnArgs::rcoef ..): forward
// y = relu(bn(z) + bn_r(res)), r = the shortcut BN (its stats / gamma / beta / running buffers /
// coef; the rest of r is ignored); backward writes dz and rdz from one reduce + finalize + apply
int ddp_bn_act_fwd_res(const ddp_amd::BnArgs* a, const ddp_amd::BnArgs* r, hipStream_t st);
int ddp_bn_act_bwd_res(const ddp_amd::BnArgs* a, hipStream_t st);
// small layers: the whole BatchNorm backward in one launch, one block per 8 channels
// (bn_act_bwd_local_kernel); ok = this layer takes that path; set = its loads-per-thread
// limit (0 = off)
int ddp_bn_bwd_local_ok(int N, int H, int W, int C, int pool);
void ddp_bn_bwd_local_set(long long max_loads);
// mid-size layers: the same in one launch over up to kStatRep blocks per 64 channels that meet at
int ddp_bn_pool_linear_ce_fwd(const ddp_amd::HeadBnIn* bn, const float* W, const float* b,
                              const long long* labels, int B, int F, int J, float* dlogits,
                              float* loss_sum, int* correct, float* loss_acc, hipStream_t st);
int ddp_linear_ce_fwd(const void* x, const float* W, const float* b, const long long* labels,
                      int B, int F, int J, float* logits, float* dlogits, float* loss_sum,
                      int* correct, float* loss_acc, hipStream_t st);
int ddp_linear_bwd(const float* dlogits, const void* x, const float* W, int B, int F, int J,
                   const float* gscale, void* dx, float* dW, float* db, hipStream_t st);
int ddp_softmax_ce(const void* logits, int logits_bf16, const long long* labels, int B, int J,
                   float* loss_sum, int* correct, void* dlogits, int dlogits_bf16,
                   hipStream_t st);
int ddp_sgd(float* p, const float* g, float* buf, size_t n, float lr, float momentum, float wd,
            float grad_scale, int nesterov, hipStream_t st);
int ddp_conv_fwd_smallk(const ddp_amd::ConvGeom* g, const void* x, const void* wc,
                        const float* bias, void* y, float* stats, hipStream_t st);
void ddp_conv_options(int stages);
void ddp_conv_epi_stage_set(int on);
int ddp_bn_pool3_fwd(const ddp_amd::BnArgs* a, unsigned char* idx, hipStream_t st);
int ddp_bn_pool3_bwd(const ddp_amd::BnArgs* a, const unsigned char* idx, hipStream_t st);
void ddp_conv_pair_mode(int mode, int items);
void ddp_sgd_fuse_register(float* dw, const ddp_amd::SgdFuse* f, int clear);
void ddp_sgd_fuse_begin();
int ddp_l0_ok(const ddp_amd::ConvGeom* g);
int ddp_l0_fwd(const ddp_amd::ConvGeom* g, const ddp_amd::L0Io* io, hipStream_t st);
int ddp_l0_bwd(const ddp_amd::ConvGeom* g, const ddp_amd::L0Io* io, hipStream_t st);
int ddp_conv_wgrad_final(const ddp_amd::ConvGeom* g, const void* dy, const void* x, float* dw,
                         float* ws, size_t ws_elems, int splits, hipStream_t st);
int ddp_sgd_fuse_taken(uintptr_t* out, int cap);
// gradient views whose MASTER a pair's unsplit WGRAD epilogue updated (operand re-pack pending)
int ddp_sgd_fuse_taken_master(uintptr_t* out, int cap);
// sweeps (tools/conv_tune.py --pairs): force the paired launch with these split-K factors (0 = off)
void ddp_conv_pair_force(int splits_dg, int splits_wg, int tile);
int ddp_conv_bwd_pair(const ddp_amd::ConvGeom* g, const void* dy, const void* wc, void* dx,
                      const void* x, float* dw, float* ws, size_t ws_elems,
                      const ddp_amd::BnBwdFuse* bn, const ddp_amd::BnBwdApply* ba, int* bn_done,
                      hipStream_t st);
void ddp_conv_tune_set(int mode, int M, int N, int K, int tile, int splits, int stages);
void ddp_conv_pair_tune_set(int M, int N, int K, int hw, int tile, int sd, int sw);
void ddp_conv_wgrad_pm_set(int on);
void ddp_conv_rows_pm_set(int on);
// BatchNorm backward: fold the finalize into the apply while the grid's replica re-reads stay
// within this many MB (default 32)
void ddp_bn_fold_bwd_mb(int mb);
// big BatchNorm layers: finalize folded into the apply on a capped grid of this many blocks
// (0, default: separate finalize launch)
void ddp_bn_fold_grid(int blocks);
// dense 2x2 form of 3x3 / s1 / p1 convs over 2x2 images (conv_igemm.hip ConvArgs::d2x2): ok =
// this geometry takes it (FWD and DGRAD), set = switch it on / off (tests)
int ddp_conv_dense2x2_ok(const ddp_amd::ConvGeom* g);
void ddp_conv_dense2x2_set(int on);
void ddp_conv_tune_clear();
void ddp_conv_force_tile(int tile_plus_one, int stages);
int ddp_pack_conv_weights(const ddp_amd::PackDesc* descs, int n, hipStream_t st);
int ddp_sgd_pack(const void* items, int n_items, const long long* descs, float* p, float* g,
                 float* buf, float lr, float momentum, float wd, float grad_scale, int nesterov,
                 int zero_grad, int* counter, int delta, const unsigned* skip,
                 unsigned short* shadow, float* slot, unsigned* done, unsigned* signal,
                 hipStream_t st);
// tail of a pipelined step with sharded buckets: gathered small-tensor slots -> fp32 arena,
// re-pack of channel-padded conv operands, then release-increment ``signal`` (optim.hip)
int ddp_shard_tail(const void* segs, int n_segs, const float* src, float* dst,
                   const ddp_amd::PackDesc* pack, int n_pack, unsigned* done, unsigned* signal,
                   const unsigned* skip, hipStream_t st);
void ddp_sgd_tile_dims(int RS, int* TK, int* TC);
int ddp_counter_add(int* c, int delta, hipStream_t st);
int ddp_synth_generate(unsigned char* images, int* labels, int n, int pix_per_img,
                       unsigned int seed, int classes, hipStream_t st);
int ddp_augment(const ddp_amd::AugArgs* a, hipStream_t st);
int ddp_nchw_to_nhwc(const float* x, int N, int C, int H, int W, int Cp, void* out,
                     hipStream_t st);
int ddp_maxpool_fwd(const void* x, int N, int H, int W, int C, int KH, int KW, int stride,
                    int pad, int Ho, int Wo, void* y, void* idx, hipStream_t st);
int ddp_maxpool_bwd(const void* dy, const void* idx, int N, int H, int W, int C, int KH, int KW,
                    int stride, int pad, int Ho, int Wo, void* dx, hipStream_t st);
int ddp_avgpool_fwd(const void* x, int N, int HW, int C, void* y, hipStream_t st);
int ddp_avgpool_bwd(const void* dy, int N, int HW, int C, void* dx, hipStream_t st);
int ddp_colsum(const void* dl, int B, int J, float* db, hipStream_t st);
int ddp_mean_ws(const float* in, size_t n, int ws, float* out, hipStream_t st);
int ddp_scale(float* x, size_t n, float s, hipStream_t st);
// kernel copy / byte fill (graph-capture-safe stand-ins for hipMemcpyAsync / hipMemsetAsync)
int ddp_copy_bytes(void* dst, const void* src, size_t n, hipStream_t st);
int ddp_fill_bytes(void* dst, int value, size_t n, hipStream_t st);
int ddp_comm_standin(float* x, size_t n, int blocks, float usec, float scale, int passes,
                     hipStream_t st);
int ddp_flag_signal(unsigned* flag, hipStream_t st);
int ddp_flag_wait(const unsigned* flag, unsigned* expected, unsigned* err, float timeout_s,
                  hipStream_t st);
int ddp_pack_bf16(const float* x, size_t n, unsigned short* y, hipStream_t st);
// segment copy of fp32 runs: table of int4 {src_index, dst_index, count, -}, one block each
int ddp_seg_copy_f32(const void* table, int n, const float* src, float* dst, hipStream_t st);
int ddp_unpack_bf16(const unsigned short* y, size_t n, float* x, hipStream_t st);
}
