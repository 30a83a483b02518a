/*
 * sqr.h — C ABI of libsqr.so, the MI355X (gfx950) hot path of sq-recovery.
 *
 * Every entry point is a plain C function over plain pointers and sizes (no
 * torch types).  Conventions for all calls:
 *   - pointers are DEVICE pointers owned by the caller; the library allocates
 *     nothing and never synchronises the host;
 *   - `stream` is a hipStream_t passed as void* (NULL = the legacy default stream);
 *     kernels are enqueued on it, so calls are graph-capturable;
 *   - return 0 on success, otherwise a negative SQR_E* code or a positive
 *     hipError_t; sqr_last_error_string() describes the last failure on the
 *     calling thread.
 *
 * Reference interfaces replaced (timoblak/sq-recovery, file:line):
 *   sqr_implicit_loss_fwd_bwd  torch/classes.py:203-295  ImplicitLoss (__init__ grid :217-222,
 *                              preprocess_sq :224-230, depth_projection :232-282, __call__ :284-295)
 *                              + its autograd backward (analytic here)
 *   sqr_implicit_render        torch/classes.py:232-282  ImplicitLoss.depth_projection (forward only)
 *   sqr_explicit_loss_fwd_bwd  torch/classes.py:109-201  ExplicitLoss (occupancy :138-189, __call__ :191-201)
 *   sqr_iou_counts             torch/classes.py:374-447  IoUAccuracy (ins_outs :394-426, __call__ :428-447)
 *   sqr_conv2d_fwd / _bwd_data / _bwd_weight
 *                              torch.nn.Conv2d as used by torchvision resnet18 inside ResNetSQ
 *                              (torch/models.py:181-184) and by GenericNetSQ (torch/models.py:134-152)
 *                              — forward and the two autograd backward products.
 *   sqr_bn_fwd / sqr_bn_bwd    torch.nn.BatchNorm2d (+ residual add + ReLU) of torchvision resnet18's
 *                              BasicBlock (ResNetSQ encoder, torch/models.py:181), training and eval.
 *   sqr_stem_fwd / _bwd        resnet18 stem bn1 -> relu -> maxpool(3,2,1) (torch/models.py:181).
 *   sqr_stem_fused_fwd / _bwd  the same stem + conv1 (torch/models.py:181-184) in one pass, bf16.
 *   sqr_adam_step              torch.optim.Adam step of torch/train.py:50-54 (+ conv weight packing).
 *   sqr_amp_*, sqr_adam_step_amp  torch.amp.GradScaler around that step (fp16 config 5; the reference
 *                              trains fp32 and has no scaler — this is the scaler torch pairs with fp16).
 *   sqr_tail_fwd / _bwd        ResNetSQ avgpool + encoder.fc + output heads (torch/models.py:7-99,186-204).
 *   sqr_comm_*                 the gradient all-reduce a DistributedDataParallel wrap of train.py's net
 *                              (torch/train.py:43) would issue, on a libsqr-owned RCCL communicator.
 */
#ifndef SQR_H
#define SQR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes (negative; positive values are hipError_t) */
#define SQR_OK 0
#define SQR_E_INVALID_ARG (-1)
#define SQR_E_UNSUPPORTED (-2)
#define SQR_E_WORKSPACE (-3)

/* element types for the conv entry points */
#define SQR_DTYPE_F32 0
#define SQR_DTYPE_BF16 1
#define SQR_DTYPE_F16 2 /* IEEE half (BASELINE config 5: fp16 + dynamic loss scaling) */

int sqr_version(void);
const char* sqr_last_error_string(void);

/* Measurement hook (bench.py): arm two hipEvent_t (passed as void*) to be recorded on the launch
 * stream immediately before and after the NEXT main conv kernel (the implicit-GEMM / direct
 * kernel of a sqr_conv2d_* call, not its im2col / split-K reduction launches); the hook then
 * disarms itself.  NULL, NULL disarms.  Per calling thread. */
int sqr_probe_arm(void* start_event, void* stop_event);
/* Clock probe (bench.py's roofline timing inside the replayed step graph, where events cannot
 * bracket one kernel node): the NEXT main conv kernel launched by this thread (then the hook
 * disarms) records, into the device slots[0] / slots[1] (u64; the caller sets them to UINT64_MAX / 0
 * before the kernel runs), the wall clock of its first workgroup's start (atomic min) and of its last
 * workgroup's end after its stores drained (atomic max).  Kernel node parameters are fixed at graph
 * capture, so every replay of a captured launch records into the same slots.  Supported by the
 * direct 3x3 kernels (the others ignore it).  slots = NULL disarms. */
int sqr_probe_arm_clock(unsigned long long* slots);
/* ticks per millisecond of that clock (hipDeviceAttributeWallClockRate) */
int sqr_wall_clock_khz(int* khz);

/* ---------------------------------------------------------------- losses */

/* Workspace (bytes, device) needed by sqr_implicit_loss_fwd_bwd for B samples at render size R. */
size_t sqr_implicit_loss_workspace_bytes(int B, int R);

/* ImplicitLoss(R, tau, sharpness)(target, params) and d loss / d params.
 *   params  [B,12] f32 : a(3) e(2) t(3) q(4, xyzw) — raw network output (clamped inside)
 *   target  [B,H,W] f32 : the depth image (channel dim squeezed); nearest-resampled to RxR
 *   loss_per_sample [B] f64 : mean_{r,c} |target_resized - render|; the reference loss is their mean
 *   grad_params [B,12] f32 : d(mean_b loss_b)/d params   (written only when need_grad != 0)
 * 2 <= R <= 256 when need_grad, R >= 2 otherwise; H,W >= 1. */
int sqr_implicit_loss_fwd_bwd(const float* params, const float* target, int B, int H, int W, int R,
                              float tau, float sharpness, int need_grad, double* loss_per_sample,
                              float* grad_params, void* workspace, size_t workspace_bytes, void* stream);

/* The same plus loss_mean [1] f64 = mean_b loss_per_sample (the reference's returned value,
 * classes.py:293-295) from the finalize launch itself (B <= 1024; otherwise one more launch).
 * loss_mean may be NULL. */
int sqr_implicit_loss_fwd_bwd_mean(const float* params, const float* target, int B, int H, int W, int R,
                                   float tau, float sharpness, int need_grad, double* loss_per_sample,
                                   double* loss_mean, float* grad_params, void* workspace,
                                   size_t workspace_bytes, void* stream);

/* Autograd backward of the losses: out[i] = grad[i] * (float)(*gout) for the f64 upstream gradient
 * gout of the scalar loss (one launch; out may alias grad). */
int sqr_loss_grad_scale(const float* grad, const double* gout, long long n, float* out, void* stream);

/* depth_projection only: images [B,R,R] f32 in the reference's image orientation (row = R-1-y, col = x). */
int sqr_implicit_render(const float* params, int B, int R, float tau, float sharpness, float* images,
                        void* stream);

size_t sqr_explicit_loss_workspace_bytes(int B, int R);

/* ExplicitLoss(R)(p_true, p_pred): loss_per_sample [B] f64 = 100*mean (occ_true-occ_pred)^2 on the
 * (n)^3 grid, n = len(arange(0, 1+1/R, 1/R)); grad_pred [B,12] f32 = d(mean_b loss_b)/d p_pred. */
int sqr_explicit_loss_fwd_bwd(const float* p_true, const float* p_pred, int B, int R, int need_grad,
                              double* loss_per_sample, float* grad_pred, void* workspace,
                              size_t workspace_bytes, void* stream);
/* ... with the batch mean (as sqr_implicit_loss_fwd_bwd_mean) */
int sqr_explicit_loss_fwd_bwd_mean(const float* p_true, const float* p_pred, int B, int R, int need_grad,
                                   double* loss_per_sample, double* loss_mean, float* grad_pred, void* workspace,
                                   size_t workspace_bytes, void* stream);

/* IoUAccuracy(R): per-sample voxel counts [B,2] int64 = (|in_true & in_pred|, |in_true | in_pred|),
 * computed in float64 like the reference. */
int sqr_iou_counts(const float* p_true, const float* p_pred, int B, int R, long long* counts,
                   void* stream);
/* the same for float64 parameters (torch/visu.py:142-159 feeds f64 params; no rounding to f32) */
int sqr_iou_counts_f64(const double* p_true, const double* p_pred, int B, int R, long long* counts,
                       void* stream);

/* ---------------------------------------------------------------- conv2d (implicit GEMM, NHWC) */

/* Activations are NHWC (torch channels_last), weights KRSC for fwd/wgrad and CRSK for dgrad
 * (sqr_conv2d_pack_weight produces both from torch's KCRS fp32 master weight).
 * dtype SQR_DTYPE_BF16: bf16 in/out, fp32 accumulation (MFMA 16x16x32 / 32x32x16 bf16).
 * dtype SQR_DTYPE_F16 : fp16 in/out, fp32 accumulation (MFMA 16x16x32 / 32x32x16 f16), same kernels.
 * dtype SQR_DTYPE_F32 : f32 in/out, exact-f32 MFMA (16x16x4 f32) — the parity mode. */
typedef struct sqr_conv_desc {
  int N, C, H, W;   /* input */
  int K, R, S;      /* filters */
  int stride, pad;  /* symmetric */
  int dtype;        /* SQR_DTYPE_* */
} sqr_conv_desc;

int sqr_conv2d_out_hw(const sqr_conv_desc* d, int* Ho, int* Wo);
size_t sqr_conv2d_workspace_bytes(const sqr_conv_desc* d, int which /*0 fwd,1 dgrad,2 wgrad*/);

/* w_kcrs f32 [K,C,R,S] -> w_krsc [K,R,S,C] and (optionally) the backward-data weight w_crsk in
 * d->dtype (C*R*S*K elements).  For stride 1 w_crsk is [C,R,S,K]; for stride st it holds the st*st
 * output-parity classes (ph,pw) back to back, each [C][Rc][Sc][K] with the taps r = r0 + st*t,
 * r0 = (ph + pad) % st (those are the only taps that reach an output pixel of that parity).
 * For C<8 convs w_krsc is the im2col weight [K][Kp], Kp = next pow2 >= max(64, R*S*C). */
int sqr_conv2d_pack_weight(const float* w_kcrs, const sqr_conv_desc* d, void* w_krsc, void* w_crsk,
                           void* stream);
/* Several pack_weight calls in ONE launch (njobs <= 20, stride <= 2; jobs is a host array read at call time;
 * only desc K,C,R,S,stride,pad,dtype matter). */
typedef struct sqr_pack_job {
  const float* w_kcrs;
  sqr_conv_desc desc;
  void* w_krsc;
  void* w_crsk; /* nullable */
} sqr_pack_job;
int sqr_conv2d_pack_weights(const sqr_pack_job* jobs, int njobs, void* stream);

/* x [N,H,W,C], y [N,Ho,Wo,K].  C must be a power of two >= 8, or < 8 (then the conv runs as
 * im2col into the workspace + a 1x1 GEMM; the im2col matrix stays in the workspace). */
int sqr_conv2d_fwd(const void* x, const void* w_krsc, void* y, const sqr_conv_desc* d, void* workspace,
                   size_t workspace_bytes, void* stream);
/* Forward that also emits BatchNorm batch-statistics partials of the (dtype-rounded) output:
 * stats[rows][2][K] f32 = (sum, sum of squares) per output channel over disjoint pixel sets (M tiles,
 * or the per-workgroup bands of the persistent layer-1 kernel), *stats_rows = rows.
 * stats must hold sqr_conv2d_stats_floats(d) floats.  Feed them to sqr_bn_fwd_stats /
 * sqr_stem_fwd_stats so the BatchNorm that follows the conv never re-reads the activation. */
size_t sqr_conv2d_stats_floats(const sqr_conv_desc* d);
/* Routing of bf16 3x3/stride-1/pad-1 forward and backward-data convs to the direct halo-window
 * kernels (C = K = 64, W = 64 or 128: the persistent resident-weight kernel; otherwise the tiled one),
 * and of bf16 3x3/stride-2/pad-1 backward-data convs of ResNetSQ's layer 2-4 shapes to the direct
 * parity-class kernel: 1 (default) when the shape tiles and the grid fills the chip (stride 2:
 * whenever it tiles), 2 whenever the shape tiles, 0 never (implicit-GEMM kernel for every shape).  Returns the previous mode.
 * Process-wide; meant for A/B tests. */
int sqr_conv_set_direct(int mode);
/* Tile choice of the tiled direct 3x3 kernels (layers 2-4): 1 = the deep weight rings (4- / 6- /
 * 9-stage), 0 = the same tiles with 3-stage rings.  Returns the previous setting.  Process-wide; meant
 * for A/B tests (results are bitwise the same: only the DMA pipelining differs). */
int sqr_conv_set_deep_ring(int on);
int sqr_conv2d_fwd_stats(const void* x, const void* w_krsc, void* y, const sqr_conv_desc* d, float* stats,
                         int* stats_rows, void* workspace, size_t workspace_bytes, void* stream);
/* sqr_conv2d_fwd_stats of x_act = relu(x_pre * scale + shift), the preceding BatchNorm + ReLU applied
 * while the conv stages its input (a BasicBlock's bn1 -> relu -> conv2, torchvision resnet18 in
 * torch/models.py:181).  coef = [scale C][shift C] (sqr_bn_fwd_finalize).  With x_act and x_mask (1 bit
 * per element, as sqr_bn_fwd writes it) they are written as side outputs, bitwise what sqr_bn_apply
 * writes: persistent layer-1 shapes only (16-bit, C = K = 64, 3x3 / s1 / p1, 64- or 128-wide maps).
 * With both NULL nothing but y and the statistics is written (the activation never reaches memory in
 * the forward; sqr_conv2d_bwd_data_bn_act rebuilds it in the backward): the shapes of
 * sqr_conv2d_bnin_nso_supported.  SQR_E_UNSUPPORTED otherwise, nothing launched. */
int sqr_conv2d_fwd_stats_bnin(const void* x_pre, const float* coef, void* x_act, uint8_t* x_mask,
                              const void* w_krsc, void* y, const sqr_conv_desc* d, float* stats, int* stats_rows,
                              void* stream);
/* 1 if conv d (C -> K) as the consumer of a BatchNorm + ReLU should run without the activation in
 * memory: sqr_conv2d_fwd_stats_bnin with x_act = x_mask = NULL and sqr_conv2d_bwd_data_bn_act are
 * handled by direct kernels at this shape AND that beats the apply pass (side outputs) there --
 * ResNetSQ's layer-2/3 convs at 256^2 input, layers 2-4 at 512^2, batch 64.  sqr_conv2d_fwd_stats_bnin
 * without side outputs also takes the persistent layer-1 shapes, and both entry points the 8x8
 * layer-4 tiles; the query answers 0 there (the side-output / apply-pass path is faster). */
int sqr_conv2d_bnin_nso_supported(const sqr_conv_desc* d);
/* dy [N,Ho,Wo,K], w_crsk (see pack_weight) -> dx [N,H,W,C]; strided convs run one stride-1
 * implicit GEMM per output-parity class (no work on structurally zero taps), all classes in one
 * launch; bf16 3x3/s2 shapes of ResNetSQ's layers 2-4 take the direct window kernel instead. */
int sqr_conv2d_bwd_data(const void* dy, const void* w_crsk, void* dx, const sqr_conv_desc* d,
                        void* workspace, size_t workspace_bytes, void* stream);
/* dx = bwd_data(dy) + addend (addend [N,H,W,C] in the conv dtype, distinct from dx): the gradient
 * of a residual block's input, whose identity / downsample branch contributes `addend`
 * (torchvision BasicBlock `out += identity`, torch/models.py:181).  The direct 3x3 kernels add in
 * their epilogues (the sum is never a separate pass); other shapes add after the GEMM. */
int sqr_conv2d_bwd_data_acc(const void* dy, const void* w_crsk, void* dx, const void* addend,
                            const sqr_conv_desc* d, void* workspace, size_t workspace_bytes, void* stream);
/* The same for a stride-2 conv whose input also feeds a stride-2 1x1 downsample conv (a BasicBlock
 * with a downsample, torch/models.py:181): that branch's input gradient is non-zero only on the
 * (even, even) pixels, so it is passed compact, addend_c [N, H/2, W/2, C] (the downsample's
 * backward-data as a stride-1 1x1 conv on the output grid), and added there: dx[n, 2i, 2j, c] +=
 * addend_c[n, i, j, c].  The direct stride-2 kernel adds it in its copy-out. */
int sqr_conv2d_bwd_data_acc_s2(const void* dy, const void* w_crsk, void* dx, const void* addend_c,
                               const sqr_conv_desc* d, void* workspace, size_t workspace_bytes, void* stream);
/* As sqr_conv2d_bwd_data_acc with the addend ReLU-masked on the fly: dx = bwd_data(dy) + addend *
 * [bit of addend_mask] (1 bit per element, NHWC order, bit k of byte i = element 8i + k): an identity
 * block's residual gradient g = dy_out * [y_out > 0] read as (dy_out, mask) instead of a
 * materialised copy (torchvision BasicBlock `out += identity; relu(out)`, models.py:181).  Direct
 * 3x3 / stride-1 16-bit kernels only: SQR_E_UNSUPPORTED otherwise (the caller masks and calls
 * sqr_conv2d_bwd_data_acc). */
int sqr_conv2d_bwd_data_acc_masked(const void* dy, const void* w_crsk, void* dx, const void* addend,
                                   const uint8_t* addend_mask, const sqr_conv_desc* d, void* workspace,
                                   size_t workspace_bytes, void* stream);
/* Backward-data of a conv whose input is a BatchNorm+ReLU output — a BasicBlock's conv2 into bn1
 * (torch/models.py:181): g_out = bwd_data(dy) * relu_mask (the BatchNorm's ReLU mask, 1 bit per
 * element) and stats receives that BatchNorm's backward sums (sum g, sum g*(bn_x - bn_mean)) as
 * f32 partial rows [*stats_rows][2][C] — computed in the direct kernels' epilogues, so
 * sqr_bn_bwd_stats needs no reduction pass over (g, x).  stats must hold
 * sqr_conv2d_bwd_data_bn_stats_floats(d) floats. */
size_t sqr_conv2d_bwd_data_bn_stats_floats(const sqr_conv_desc* d);
int sqr_conv2d_bwd_data_bn(const void* dy, const void* w_crsk, void* g_out, const void* bn_x,
                           const uint8_t* relu_mask, const float* bn_mean, float* stats, int* stats_rows,
                           const sqr_conv_desc* d, void* workspace, size_t workspace_bytes, void* stream);
/* sqr_conv2d_bwd_data_bn for a BatchNorm + ReLU applied on load without side outputs (the forward was
 * sqr_conv2d_fwd_stats_bnin with x_act = x_mask = NULL): the ReLU mask is recomputed from bn_x and the
 * forward coefficients bn_coef = [scale C][shift C] (the rounded activation > 0, as sqr_bn_apply forms
 * it), and act_out (nullable) receives the activation relu(bn_x * scale + shift) itself -- bitwise what
 * sqr_bn_apply writes -- for the conv's weight gradient.  Tiled direct kernels only (not the
 * persistent layer-1 shapes): SQR_E_UNSUPPORTED otherwise, nothing launched. */
int sqr_conv2d_bwd_data_bn_act(const void* dy, const void* w_crsk, void* g_out, const void* bn_x,
                               const float* bn_coef, const float* bn_mean, void* act_out, float* stats,
                               int* stats_rows, const sqr_conv_desc* d, void* stream);
/* x [N,H,W,C], dy [N,Ho,Wo,K] -> dw_kcrs f32 [K,C,R,S] (torch's weight-grad layout) */
int sqr_conv2d_bwd_weight(const void* x, const void* dy, float* dw_kcrs, const sqr_conv_desc* d,
                          void* workspace, size_t workspace_bytes, void* stream);
/* A BatchNorm backward finalize riding along a weight-gradient launch: the BatchNorm whose
 * backward sums sqr_conv2d_bwd_data_bn produced (stats [stats_rows][2][C] f32, over M pixels) gets
 * dgamma / dbeta and coef = [k1 C][k2 C][k3 C] for sqr_bn_bwd_apply, computed by extra workgroups
 * of the weight gradient's split-K reduction instead of a launch of their own. */
typedef struct sqr_bn_bwd_fin {
  const float* stats;
  int stats_rows;
  long long M;
  int C;
  const float* gamma;       /* nullable (affine=False) */
  const float* save_mean;
  const float* save_invstd;
  float* dgamma;            /* nullable */
  float* dbeta;             /* nullable */
  float* coef;              /* out, 3*C floats */
} sqr_bn_bwd_fin;
/* A BatchNorm backward reduction riding along a weight-gradient launch: dy is the gradient this
 * conv's backward-data just wrote for the BatchNorm(+ReLU) output that feeds it (a BasicBlock's
 * input: the previous block's bn2 output, kind 1, or its bn2 + downsample-bn output, kind 2);
 * part receives (sum g, sum g*(x_a - mean_a)[, sum g*(x_b - mean_b)]) per block, g = dy*mask,
 * for sqr_bn_bwd_part / sqr_bn_add_bwd_part.  part must hold sqr_bn_bwd_red_doubles(M, C, kind). */
typedef struct sqr_bn_bwd_red {
  int kind;
  const void* dy;
  const uint8_t* relu_mask;
  const void* x_a;
  const float* mean_a;
  const void* x_b;          /* kind 2 */
  const float* mean_b;      /* kind 2 */
  long long M;
  int C;
  double* part;             /* out */
  int* part_rows;           /* out (host memory) */
} sqr_bn_bwd_red;
size_t sqr_bn_bwd_red_doubles(long long M, int C, int kind);
/* the weight gradient with either job (or both, or neither: then = sqr_conv2d_bwd_weight) riding
 * along its split-K reduction launch */
int sqr_conv2d_bwd_weight_bn(const void* x, const void* dy, float* dw_kcrs, const sqr_conv_desc* d,
                             const sqr_bn_bwd_fin* fin, const sqr_bn_bwd_red* red, void* workspace,
                             size_t workspace_bytes, void* stream);
/* C<8 (im2col) convs only: the same from the im2col matrix the forward left at the start of its
 * workspace (sqr_conv2d_workspace_bytes(d,0) bytes), skipping the re-gather; this call's own
 * workspace needs sqr_conv2d_workspace_bytes(d,2) - sqr_conv2d_workspace_bytes(d,0) bytes. */
int sqr_conv2d_bwd_weight_col(const void* col, const void* dy, float* dw_kcrs, const sqr_conv_desc* d,
                              void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- batch norm (NHWC, fused) */

/* x [M][C] (M = N*H*W pixels, NHWC), C a multiple of 8 with C/8 dividing 256; gamma/beta/stats f32.
 * training != 0: batch statistics; save_mean/save_invstd [C] are written and running_mean/var
 *   (nullable) are updated as nn.BatchNorm2d does (momentum, unbiased running variance);
 * training == 0: normalises with running_mean/var.
 * y = relu?(gamma*(x-mean)*invstd + beta [+ residual]); residual nullable.
 * relu_mask (nullable, used only with relu): uint8 [M*C/8], bit k of byte i = (y[8i+k] > 0) of the
 * stored values — what sqr_bn_bwd needs instead of re-reading y. */
size_t sqr_bn_workspace_bytes(long long M, int C);
int sqr_bn_fwd(const void* x, long long M, int C, int dtype, const float* gamma, const float* beta,
               float* running_mean, float* running_var, float momentum, float eps, int training,
               const void* residual, int relu, void* y, uint8_t* relu_mask, float* save_mean, float* save_invstd,
               void* workspace, size_t workspace_bytes, void* stream);
/* training-mode sqr_bn_fwd with the batch statistics taken from sqr_conv2d_fwd_stats partials */
int sqr_bn_fwd_stats(const void* x, long long M, int C, int dtype, const float* stats, int stats_rows,
                     const float* gamma, const float* beta, float* running_mean, float* running_var, float momentum,
                     float eps, const void* residual, int relu, void* y, uint8_t* relu_mask, float* save_mean,
                     float* save_invstd, void* workspace, size_t workspace_bytes, void* stream);
/* sqr_bn_fwd_stats in two halves: the finalize (batch statistics -> save_mean / save_invstd, running
 * statistics, coef = [scale C][shift C]) and the apply pass y = relu?(x * scale + shift [+ residual]);
 * the apply half is skipped when the consuming conv applies on load (sqr_conv2d_fwd_stats_bnin). */
int sqr_bn_fwd_finalize(const float* stats, int stats_rows, long long M, int C, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                        float* save_invstd, float* coef, void* stream);
int sqr_bn_apply(const void* x, long long M, int C, int dtype, const float* coef, const void* residual, int relu,
                 void* y, uint8_t* relu_mask, void* stream);
/* backward of sqr_bn_fwd (training statistics): g = dy * [y > 0] with the forward's relu_mask (NULL
 * when the forward had no ReLU); dx, dgamma = sum g*xhat, dbeta = sum g; dres (nullable) = g. */
int sqr_bn_bwd(const void* dy, const uint8_t* relu_mask, const void* x, long long M, int C, int dtype, const float* gamma,
               const float* save_mean, const float* save_invstd, void* dx, void* dres, float* dgamma,
               float* dbeta, void* workspace, size_t workspace_bytes, void* stream);
/* sqr_bn_bwd from sqr_conv2d_bwd_data_bn's partials: g already masked; dx = k1*g + k3*x + k2,
 * dgamma, dbeta.  workspace >= 3*C floats. */
int sqr_bn_bwd_stats(const void* g, const void* x, long long M, int C, int dtype, const float* stats, int stats_rows,
                     const float* gamma, const float* save_mean, const float* save_invstd, void* dx, float* dgamma,
                     float* dbeta, void* workspace, size_t workspace_bytes, void* stream);
/* dx = k1*g + k3*x + k2 from finalized coefficients (sqr_conv2d_bwd_weight_bnfin's coef) */
int sqr_bn_bwd_apply(const void* g, const void* x, long long M, int C, int dtype, const float* coef, void* dx,
                     void* stream);
/* sqr_bn_bwd from riding-reduction partials (sqr_conv2d_bwd_weight_bn's red job, kind 1) */
int sqr_bn_bwd_part(const void* dy, const uint8_t* relu_mask, const void* x, long long M, int C, int dtype,
                    const double* part, int rows, const float* gamma, const float* save_mean,
                    const float* save_invstd, void* dx, void* dres, float* dgamma, float* dbeta, void* workspace,
                    size_t workspace_bytes, void* stream);

/* Two-branch BatchNorm: y = act(bn_a(a.x) + bn_b(b.x)) — torchvision BasicBlock with a downsample,
 * relu(bn2(conv2(.)) + bn_ds(conv_ds(x))) (torch/models.py:181).  One apply pass reads both conv
 * outputs (the downsample branch's normalised tensor is never written); the backward reduces both
 * BatchNorms in one pass over (dy, mask, a.x, b.x) and writes both input gradients in one pass.
 * Training takes the batch statistics from each conv's sqr_conv2d_fwd_stats partials. */
typedef struct sqr_bn_operand {
  const void* x;            /* [M][C] conv output (NHWC), the op's dtype */
  const float* stats;       /* training: [stats_rows][2][C] partials; eval: unused */
  int stats_rows;
  const float* gamma;       /* nullable (affine=False) */
  const float* beta;
  float* running_mean;      /* nullable when not tracking (training) */
  float* running_var;
  float momentum, eps;
  float* save_mean;         /* training: written by fwd, read by bwd */
  float* save_invstd;
} sqr_bn_operand;
size_t sqr_bn_add_workspace_bytes(long long M, int C);
int sqr_bn_add_fwd(const sqr_bn_operand* a, const sqr_bn_operand* b, long long M, int C, int dtype, int training,
                   int relu, void* y, uint8_t* relu_mask, void* workspace, size_t workspace_bytes, void* stream);
/* training backward: g = dy * [y > 0]; dx_a / dx_b, dgamma / dbeta of both BatchNorms */
int sqr_bn_add_bwd(const sqr_bn_operand* a, const sqr_bn_operand* b, const void* dy, const uint8_t* relu_mask,
                   long long M, int C, int dtype, void* dx_a, void* dx_b, float* dgamma_a, float* dbeta_a,
                   float* dgamma_b, float* dbeta_b, void* workspace, size_t workspace_bytes, void* stream);
/* sqr_bn_add_bwd from riding-reduction partials (kind 2); workspace >= 6*C floats */
int sqr_bn_add_bwd_part(const sqr_bn_operand* a, const sqr_bn_operand* b, const void* dy, const uint8_t* relu_mask,
                        long long M, int C, int dtype, const double* part, int rows, void* dx_a, void* dx_b,
                        float* dgamma_a, float* dbeta_a, float* dgamma_b, float* dbeta_b, void* workspace,
                        size_t workspace_bytes, void* stream);

/* resnet stem: y = maxpool3x3/s2/p1(relu(bn(x))), x [N][H][W][C] NHWC; argmax [N][Ho][Wo][C] uint8
 * = window tap (dh*3+dw) of the first maximum (torch's tie rule), written when training. */
size_t sqr_stem_workspace_bytes(int N, int H, int W, int C);
int sqr_stem_fwd(const void* x, int N, int H, int W, int C, int dtype, const float* gamma, const float* beta,
                 float* running_mean, float* running_var, float momentum, float eps, int training, void* y,
                 uint8_t* argmax, float* save_mean, float* save_invstd, void* workspace, size_t workspace_bytes,
                 void* stream);
int sqr_stem_fwd_stats(const void* x, int N, int H, int W, int C, int dtype, const float* stats, int stats_rows,
                       const float* gamma, const float* beta, float* running_mean, float* running_var, float momentum,
                       float eps, void* y, uint8_t* argmax, float* save_mean, float* save_invstd, void* workspace,
                       size_t workspace_bytes, void* stream);
/* dpool/ypool [N][Ho][Wo][C] (gradient and value of the pooled output), x = conv1 output. */
int sqr_stem_bwd(const void* dpool, const void* ypool, const uint8_t* argmax, const void* x, int N, int H, int W,
                 int C, int dtype, const float* gamma, const float* save_mean, const float* save_invstd, void* dx,
                 float* dgamma, float* dbeta, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- fused stem (bf16 / fp16) */

/* resnet18 stem of ResNetSQ (torch/models.py:181-184) for 16-bit training / inference:
 * y = maxpool3x3/s2/p1(relu(bn1(conv1(x)))), conv1 = 1 -> 64 channels, 7x7, stride 2, pad 3, no
 * bias, computed in y_dtype (bf16 or fp16; fp32 accumulation) WITHOUT materialising the conv1
 * activation: the forward recomputes conv1 for the BatchNorm statistics and for the pooling.  The
 * backward does not recompute conv1: per tile it accumulates, over the input patches A, the Gram
 * matrix S = sum A A^T and T1 = sum g A (g = the pooled gradient routed to its argmax pixel), then
 * T2 = W S and sum g*x = rowsum(W o T1) give dW / dgamma / dbeta in closed form (BatchNorm's
 * backward is linear in g, x and 1; no input gradient).  Known deviation from torch: x in these
 * sums is the f32 conv value, where torch's BatchNorm backward reads the 16-bit-rounded stored
 * conv1 output; the difference is within the 16-bit rounding of x and is covered by the
 * tolerance tests/test_step_gpu.py derives from a CPU float32 emulation that rounds at the GPU
 * step's storage points (every parameter gradient within 3x of that emulation's error vs float64).
 *   x [N][H][W] (x_dtype f32, bf16 or fp16), w [64][1][7][7] f32, y [N][Hp][Wp][64] y_dtype (NHWC),
 *   argmax [N][Hp][Wp][64] u8 (window tap of the first maximum; written when training).
 * Shapes: the conv1 output (H/2 x W/2) must tile by 8 x 32 and the pooled one by 8 x 16
 * (sqr_stem_fused_supported).  BatchNorm semantics as sqr_stem_fwd (momentum, running stats). */
int sqr_stem_fused_supported(int N, int H, int W);
size_t sqr_stem_fused_workspace_bytes(int N, int H, int W);
int sqr_stem_fused_fwd(const void* x, int x_dtype, int y_dtype, int N, int H, int W, const float* w, const float* gamma,
                       const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                       int training, void* y, uint8_t* argmax, float* save_mean, float* save_invstd,
                       void* workspace, size_t workspace_bytes, void* stream);
/* dy, y, argmax: the pooled gradient / output / argmax of the forward; dw [64][1][7][7] f32 */
int sqr_stem_fused_bwd(const void* x, int x_dtype, int y_dtype, int N, int H, int W, const float* w, const float* gamma,
                       const float* save_mean, const float* save_invstd, const void* dy, const void* y,
                       const uint8_t* argmax, float* dw, float* dgamma, float* dbeta, void* workspace,
                       size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- optimizer */

/* One torch.optim.Adam step (weight_decay 0, no amsgrad / maximize; torch/train.py:50-54) over up to
 * 80 fp32 parameters, fused with the bf16 packing of conv weights: when w_krsc is set (desc: the
 * conv geometry, dtype BF16) the updated weight is also written as sqr_conv2d_pack_weight's w_krsc
 * (and w_crsk when set; K, C multiples of 64).  step: the parameter's device step counter (float),
 * read as t = step + 1 for the bias corrections and incremented.  grad_scale multiplies every
 * gradient as it is read (1 = torch.optim.Adam; 1/N averages gradients all-reduced with SUM over N
 * data-parallel ranks).  params is a host array. */
typedef struct sqr_adam_param {
  float* p;
  const float* g;
  float* exp_avg;
  float* exp_avg_sq;
  float* step;
  long long n;
  sqr_conv_desc desc;
  void* w_krsc; /* nullable */
  void* w_crsk; /* nullable */
} sqr_adam_param;
int sqr_adam_step(const sqr_adam_param* params, int nparams, double lr, double beta1, double beta2, double eps,
                  double grad_scale, void* stream);

/* ---------------------------------------------------------------- dynamic loss scaling (fp16)
 * torch.amp.GradScaler (init_scale 2^16, growth 2, backoff 0.5, interval 2000) as three stream-ordered,
 * graph-capturable device steps around a backward of `loss * (*loss_scale)`:
 *   sqr_amp_check_finite  found_inf |= any non-finite element in the gradients (host arrays of device
 *                         pointers / sizes; *found_inf must be 0 before the first call of a step);
 *   sqr_amp_check_finite_scaled  the same on the values the fused Adam will use, g * grad_scale *
 *                         fp32(1 / *loss_scale) (loss_scale nullable): torch checks after unscaling, so a
 *                         finite g that overflows once multiplied (scale backed off below 1) counts;
 *   sqr_adam_step_amp     sqr_adam_step on gradients g / (*loss_scale) that does nothing at all (no
 *                         update, no step-counter increment, no packing) when *found_inf != 0;
 *   sqr_amp_update_scale  GradScaler.update(): *found_inf ? scale *= backoff, tracker = 0
 *                         : ++tracker == interval ? scale *= growth, tracker = 0; then *found_inf = 0.
 * loss_scale f32, found_inf / growth_tracker int32, all device pointers. */
int sqr_amp_check_finite(const float* const* grads, const long long* sizes, int n, int* found_inf, void* stream);
int sqr_amp_check_finite_scaled(const float* const* grads, const long long* sizes, int n, const float* loss_scale,
                                double grad_scale, int* found_inf, void* stream);
int sqr_adam_step_amp(const sqr_adam_param* params, int nparams, double lr, double beta1, double beta2, double eps,
                      double grad_scale, const float* loss_scale, const int* found_inf, void* stream);
int sqr_amp_update_scale(float* loss_scale, int* growth_tracker, int* found_inf, float growth_factor,
                         float backoff_factor, int growth_interval, void* stream);

/* ---------------------------------------------------------------- ResNetSQ tail (fused) */

/* adaptive avg-pool + encoder.fc (Linear-LeakyReLU-Linear-LeakyReLU) + the 4 heads of ResNetSQ
 * (torch/models.py:186-204, heads :7-99): x [B][P][C0] (NHWC layer-4 output, P = H*W pixels, dtype)
 * -> a [B,3], e [B,2], t [B,3] (sigmoid), q [B,4] (L2-normalised), all f32.  Parameters are the
 * fp32 nn.Linear weights [out][in] / biases.  Constraints: C0 a power of 2 <= 1024, F1, F2
 * multiples of 4 <= 1024. */
typedef struct sqr_tail_desc {
  int B, P, C0, F1, F2, dtype;
  const float *w0, *b0;   /* encoder.fc.0: [F1][C0], [F1] */
  const float *w1, *b1;   /* encoder.fc.2: [F2][F1], [F2] */
  const float* wh[4];     /* output_{size,shape,position,rotation}.out_layer.0.weight [3|2|3|4][F2] */
  const float* bh[4];
} sqr_tail_desc;
/* save: sqr_tail_save_floats(t) floats written by the forward, read by the backward */
size_t sqr_tail_save_floats(const sqr_tail_desc* t);
int sqr_tail_fwd(const sqr_tail_desc* t, const void* x, float* out_a, float* out_e, float* out_t, float* out_q,
                 float* save, void* stream);
/* the same with the four heads written side by side into pred [B][12] = (a, e, t, q): the
 * reference's torch.cat of the heads (torch/train.py:88-89) without a copy */
int sqr_tail_fwd_packed(const sqr_tail_desc* t, const void* x, float* pred, float* save, void* stream);
typedef struct sqr_tail_grads {
  const float* g_out[4];  /* upstream grads of a, e, t, q: rows of ld[h] floats; NULL = zero */
  int ld[4];
  void* dx;               /* [B][P][C0] dtype: d loss / d x */
  float *dw0, *db0, *dw1, *db1;
  float* dwh[4];
  float* dbh[4];
} sqr_tail_grads;
size_t sqr_tail_workspace_bytes(const sqr_tail_desc* t);
int sqr_tail_bwd(const sqr_tail_desc* t, const float* save, const sqr_tail_grads* g, void* workspace,
                 size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- data-parallel gradient exchange
 * One RCCL communicator per rank, owned by libsqr (not by torch's ProcessGroupNCCL), carrying the
 * bucketed gradient all-reduce of a data-parallel step (north_star: "RCCL all-reduce
 * of gradients over xGMI overlapped with backward on a side HIP stream").  The reference trains on one
 * GPU (torch/train.py:42-54); these calls replace what a DistributedDataParallel wrap around its
 * `net` (train.py:43) would issue.  The collectives are stream-ordered and graph-capturable: a
 * captured step holds plain RCCL kernels and no host-side completion tracking (no watchdog).
 *   sqr_comm_load        dlopen the process's RCCL (path, NULL = "librccl.so.1", i.e. the copy
 *                        already mapped by torch); *version = ncclGetVersion (nullable);
 *   sqr_comm_unique_id   rank 0: a fresh SQR_COMM_ID_BYTES id, to be sent to every rank (host group);
 *   sqr_comm_init_rank   collective over all ranks, on the calling thread's current HIP device;
 *   sqr_comm_allreduce_sum_f32  in-place sum of count floats over the ranks;
 *   sqr_comm_broadcast   in-place byte broadcast from root (parameter / buffer init);
 *   sqr_comm_async_error 0, or the communicator's asynchronous failure as an error;
 *   sqr_comm_destroy     finalize + destroy (after every graph holding its collectives is destroyed);
 *   sqr_comm_abort       ncclCommAbort + free: a rank whose host deadline expired or whose peer failed
 *                        (sqr.dist.wait_device) releases its in-flight collectives and exits.
 * Errors from RCCL are returned as 1000 + ncclResult_t. */
#define SQR_COMM_ID_BYTES 128
typedef struct sqr_comm* sqr_comm_t;
int sqr_comm_load(const char* rccl_path, int* version);
int sqr_comm_unique_id(unsigned char* id_out);
int sqr_comm_init_rank(sqr_comm_t* comm, const unsigned char* id, int nranks, int rank);
int sqr_comm_allreduce_sum_f32(sqr_comm_t comm, float* buf, size_t count, void* stream);
int sqr_comm_broadcast(sqr_comm_t comm, void* buf, size_t bytes, int root, void* stream);
int sqr_comm_async_error(sqr_comm_t comm);
int sqr_comm_destroy(sqr_comm_t comm);
int sqr_comm_abort(sqr_comm_t comm);

/* Measurement stand-in for one bucket all-reduce at N = 1 (bench.py --dp-proxy, sqr.dist.ProxyComm;
 * no training path calls it): `channels` 256-thread workgroups copy `bytes` from src to scratch and
 * hold their CU until hold_us has passed since they started -- the CU slots and HBM traffic an RCCL
 * ring all-reduce of that bucket takes on an N-GPU node, so the interference of the overlapped
 * all-reduce with the backward kernels can be measured on a one-GPU box. */
int sqr_comm_proxy(const void* src, void* scratch, size_t bytes, int channels, double hold_us, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SQR_H */
