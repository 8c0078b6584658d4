/* spff.h -- C ABI of the MI355X-native SPFF-UNet engine (libspff_hip.so).
 *
 * This is the drop-in boundary for the reference's hot path: the SPFF-UNet
 * forward (innovative3D/models.py:693-701 UNet3D_SpectralCore.forward with the
 * _DoubleConvSpectral_Novel blocks of models.py:1448-1544, built by
 * build_spct_energyfilm_fourier models.py:1547-1555 behind
 * LitSPCT_EFiLM_FourierGate models.py:1558-1564), the loss
 * ce_plus_macro_dice_loss (helpers.py:797-803) and autograd's backward of both.
 * The reference binds these through PyTorch; the Python mirror in
 * spff-unet-spcct_amd/innovative3D binds them with ctypes.
 *
 * Conventions: plain device pointers + sizes, no torch types.  All calls are
 * stream-ordered and asynchronous (hipStream_t passed as void*; NULL = default
 * stream).  Activations are fp32; the network input is the reference layout
 * [B][Cin][D][H][W]; logits/dlogits are channel-last [B][D][H][W][K] (a
 * torch.channels_last_3d view of the reference's [B][K][D][H][W]).  Params /
 * dparams are ONE flat fp32 buffer in reference state-dict order (see
 * spff_param_info; the lazily created FourierGate mask appears once, under
 * "...fgate.freq_mask", and stands for the aliased "...fgate._mask" key).
 * Functions return 0 on success, a negative SPFF_E* code otherwise (never
 * throw); spff_last_error() describes the last failure of the calling thread.
 * A plan is not thread-safe and holds one forward's saved activations inside
 * the caller's workspace until the matching backward.
 */
#ifndef SPFF_H_
#define SPFF_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPFF_OK 0
#define SPFF_EINVAL (-1)
#define SPFF_EHIP (-2)
#define SPFF_ESHAPE (-3)
#define SPFF_ECOLL (-4) /* a shard-group collective callback (spff_coll) returned non-zero */

/* arithmetic of the 3x3x3 conv contractions (spff_cfg.math):
 *   SPFF_MATH_F32     fp32 MFMA (v_mfma_f32_32x32x2_f32, an exact fp32 fma chain)
 *   SPFF_MATH_BF16X6  fp32 operands split exactly into 3 bf16 planes, 6 cross
 *                     products on the bf16 MFMA, fp32 accumulate: dropped terms
 *                     < 2^-24 |xy| per product (fp32 accuracy class), ~2.7x the rate
 *   SPFF_MATH_BF16X3  2 planes, 3 products: ~2^-17 relative per product (opt-in)
 *   SPFF_MATH_F16X3   each operand scaled by a power of two (max |x| 2^e < 2^14, from an
 *                     on-device absmax) and split into 2 fp16 planes, 3 products on the
 *                     fp16 MFMA: <= 2^-22 |x| per operand, dropped l*l <= 2^-22 |xy|,
 *                     at the bf16x3 rate (the 1x1x1 / ConvTranspose GEMMs keep bf16x6) */
/* largest num_classes of the SPFF / 3DUNet plans and of spff_loss / spff_confusion
 * (the SwinUNETR plan's soft-Dice loss: 32) */
#define SPFF_MAX_CLASSES 128

#define SPFF_MATH_F32 0
#define SPFF_MATH_BF16X6 1
#define SPFF_MATH_BF16X3 2
#define SPFF_MATH_F16X3 3

typedef struct spff_cfg {
  int batch, in_ch, depth, height, width;  /* input [B][Cin][D][H][W] */
  int num_classes;                          /* K, 1 .. SPFF_MAX_CLASSES */
  int base;                                 /* f: a multiple of 8 (>= 8) */
  int ksd;                                  /* spectral kernel depth: 1 or 3 */
  int use_efilm, use_fgate;                 /* novel block (models.py:1448) */
  int use_se, use_specse;                   /* encoder post (models.py:684) */
  int math;                                 /* SPFF_MATH_* (0 = fp32 MFMA) */
  /* depth sharding (BASELINE config 4): this plan holds global depths
   * [shard_rank * depth, (shard_rank + 1) * depth) of a volume of depth
   * shard_world * depth; requires batch == 1 and a collectives table, see spff_coll below.
   * shard_world <= 1: unsharded. */
  int shard_world, shard_rank;
  /* saved-activation layout: SPFF_MEM_FULL keeps every block's conv outputs, IN /
   * gate outputs and up-conv outputs (~2.8 KB per input voxel); SPFF_MEM_LEAN keeps
   * only the conv outputs y1, y2 and per-(b,c[,d]) coefficients and recomputes the
   * rest in the backward (~1.7 KB per voxel: one 5 x 512^3 volume fits one MI355X;
   * +~3 % step time); SPFF_MEM_AUTO (0) = lean from 2^26 voxels per plan. */
  int memory_mode;
  /* the axis a sharded plan (shard_world > 1) splits: SPFF_SHARD_DEPTH (0) -- above;
   * SPFF_SHARD_HEIGHT (1) -- the registry layout [B, 1, 5, H, W]: this
   * plan holds global rows [shard_rank * height, (shard_rank + 1) * height) of a volume
   * of height shard_world * height; height and width multiples of 8 (the three (1,2,2)
   * pools stay rank-local), any batch.  Same collectives table. */
  int shard_axis;
  /* the novel block's EnergyFiLM3D(hidden, pe_dims) and FourierGate3D(learn_phase)
   * (models.py:1484-1489, 1521-1541), the same in every block; 0 = the reference's
   * defaults (32, 16, off: what _DoubleConvSpectral_Novel builds).  hidden 1..64,
   * pe_dims 2..32 ((hidden + pe_dims) * depth * 4 B of LDS <= 160 KiB) */
  int efilm_hidden, efilm_pe_dims, fgate_learn_phase;
} spff_cfg;

#define SPFF_SHARD_DEPTH 0
#define SPFF_SHARD_HEIGHT 1

#define SPFF_MEM_AUTO 0
#define SPFF_MEM_FULL 1
#define SPFF_MEM_LEAN 2

/* The shard group's collectives, implemented by the caller (e.g. RCCL through
 * torch.distributed) and called by the engine in stream order on the stream
 * argument: the stream of the current spff_forward / spff_backward, or -- for a
 * halo that overlaps a convolution's interior depth tiles -- the plan's side
 * stream, which the engine has made wait for the data and whose completion the
 * main stream waits for.  Issue the work on the stream given.  Return 0 on success.
 *   allreduce: in-place sum over the group of n elements at device pointer buf
 *              (dtype 0 = fp32, 1 = fp64).
 *   halo:      interior points at slice 0 of a [d_local][slice_floats] slab
 *              that has one writable slice before it and one after it: send
 *              slice 0 to rank - 1 and slice d_local - 1 to rank + 1, and receive
 *              rank - 1's last slice into interior[-slice_floats ..) and
 *              rank + 1's first slice into interior[d_local * slice_floats ..).
 *              Slices beyond the global ends are zeroed by the engine. */
typedef struct spff_coll {
  void* ctx;
  int (*allreduce)(void* ctx, void* buf, int64_t n, int dtype, void* stream);
  int (*halo)(void* ctx, float* interior, int64_t slice_floats, int d_local, void* stream);
} spff_coll;

typedef struct spff_plan spff_plan;

/* plan lifetime (replaces build_class(...)() -> module construction, config.py:159-182) */
int spff_plan_create(const spff_cfg* cfg, spff_plan** out);
void spff_plan_destroy(spff_plan* plan);
/* attach the shard group's collectives (required before the first forward of a
 * plan with shard_world > 1; the table is copied) */
int spff_plan_set_coll(spff_plan* plan, const spff_coll* coll);
/* gradient-ready hook (data parallelism; replaces the bucketed gradient
 * all-reduce torch DDP hangs on autograd for the reference's module, SURVEY
 * §8(e) DP row): during spff_backward the engine calls fn(ctx, off, n, stream)
 * in stream order as soon as dparams[off, off + n) is final (one call per
 * block's parameters, per SE / up-conv / head group; together they cover every
 * float once), so the caller can issue that range's all-reduce on a
 * collective stream that waits on `stream` while the backward continues.
 * fn == NULL removes the hook.  Return 0 from fn, else the backward fails. */
typedef int (*spff_grad_ready_fn)(void* ctx, int64_t off, int64_t n, void* stream);
int spff_plan_set_grad_hook(spff_plan* plan, spff_grad_ready_fn fn, void* ctx);
const char* spff_last_error(void);

/* flat parameter layout (reference state-dict order, models.py:655-681) */
int spff_num_params(const spff_plan* plan);
int spff_param_info(const spff_plan* plan, int i, const char** name, int* ndim,
                    int64_t shape[5], int64_t* offset, int64_t* numel);
int64_t spff_param_floats(const spff_plan* plan);
size_t spff_workspace_bytes(const spff_plan* plan);

/* forward: x [B][Cin][D][H][W] -> logits [B][D][H][W][K]  (models.py:693-701) */
int spff_forward(spff_plan* plan, const float* x, const float* params, float* logits,
                 void* workspace, void* stream);
/* backward of the last forward: dlogits [B][D][H][W][K] -> dparams (flat, every
 * entry written).  Input gradient is not produced (the hot path never needs it). */
int spff_backward(spff_plan* plan, const float* dlogits, const float* params, float* dparams,
                  void* workspace, void* stream);
/* device pointer + shape of a saved intermediate (debug / tests), e.g. "enc1.out"
 * (fp32 [nvox][channels]); "pool1.idx" .. "pool3.idx" are the max-pools' argmax BYTES
 * [nvox][channels] (k = 2 dh + dw of each 2 x 2 window, first max in scan order) */
int spff_saved_tensor(const spff_plan* plan, void* workspace, const char* name,
                      const float** ptr, int64_t* nvox, int* channels);

/* debug knobs (tests): key 0 = stop the backward after N decoder blocks (-1 off);
 * key 1 = also store the block outputs the up-conv / head GEMMs apply on the fly
 * (bott/dec*.out; otherwise spff_saved_tensor reports them as not stored) */
int spff_debug_set(spff_plan* plan, int key, int value);

/* optional HIP-event timing of the engine's kernels on the plan's stream (bench.py):
 * classes 0 = conv3d fwd, 1 = conv3d dgrad (same kernel), 2 = conv3d wgrad,
 * 3 = ConvTranspose / 1x1 head GEMMs, and the HBM-bound passes 4 = per-(b,c,d)
 * slab reductions (IN statistics, gate sums; incl. the split combine),
 * 5 = IN/gate apply (act_apply), 6 = IN backward apply (in_bwd_apply), 7 = the
 * SPFF_MATH_F16X3 operand-max passes of the weight gradients' scales (the weights, the
 * block inputs, the a1 bound; per launch in sharded plans).
 * collect() syncs on the recorded events and writes out[4*c + {0,1,2,3}] =
 * {total ms, algorithmic FLOPs, launches, algorithmic HBM bytes (operands read
 * once, result written once)}. */
int spff_prof_enable(spff_plan* plan, int on);
int spff_prof_collect(spff_plan* plan, double* out, int nclass);
/* Library-wide conv timing: HIP events around every 3x3x3 conv launch (forward, input
 * gradient, weight gradient) on the stream it runs on, whichever plan or op entry point
 * issues it (the 3DUNet / SwinUNETR plans included).  collect: out[4 c + {0,1,2,3}] =
 * (ms, algorithmic fp32 flops 2 V Cin Cout T, launches, 0) for class c = 0 fwd, 1 dgrad,
 * 2 wgrad; synchronises on the recorded events and resets the record. */
int spff_conv_prof_enable(int on);
int spff_conv_prof_collect(double* out, int nclass);

/* ce_plus_macro_dice_loss (helpers.py:797-803) on channel-last logits [V][K].
 * out4 (device) = [ce, ce + 0.5*hard_dice_loss, hard_dice_loss, n_valid];
 * dlogits = d(ce)/dlogits (softmax - onehot)/N_valid (0 for ignored voxels);
 * conf (device) = K*(K+1) int64: conf[pred*(K+1) + label] over non-ignored
 * voxels (argmax, first max wins), column K = labels outside [0,K) (the
 * reference raises on those in the loss; they are excluded from CE here).
 * count_override (device int64*, may be NULL): global N_valid for data-parallel
 * runs (all-reduced by the caller); NULL -> counted locally. */
size_t spff_loss_ws_bytes(int64_t nvox, int num_classes);
int spff_loss(const float* logits, const int64_t* labels, int64_t nvox, int num_classes,
              int ignore_index, double smooth, const int64_t* count_override, float* out4,
              float* dlogits, int64_t* conf, void* ws, void* stream);
/* argmax confusion only (per_class_metrics_3d, helpers.py:668-725) */
int spff_confusion(const float* logits, const int64_t* labels, int64_t nvox, int num_classes,
                   int ignore_index, int64_t* conf, void* stream);
int spff_count_valid(const int64_t* labels, int64_t nvox, int ignore_index, int64_t* count,
                     void* stream);
/* x[i] *= *scale (scale is a device scalar) */
int spff_scale(float* x, int64_t n, const float* scale, void* stream);

/* fused Adam / AdamW step over n contiguous fp32 elements (replaces the
 * torch.optim.Adam of BaseLitModel.configure_optimizers, models.py:591-594, and
 * unified_optimizer.py:5-60): decoupled = 1 is AdamW; step = the 1-based step
 * count after this update; arithmetic in torch's fp32 operation order. */
int spff_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                   int64_t n, double lr, double beta1, double beta2, double eps,
                   double weight_decay, int decoupled, int64_t step, void* stream);

/* op-level entry points (parity tests): channel-last activations, reference
 * weight layout W[Cout][Cin][ksd][3][3].  ws >= spff_conv3d_ws_bytes(...). */
size_t spff_conv3d_ws_bytes(int B, int D, int H, int W, int cin, int cout, int ksd);
int spff_conv3d_fwd(const float* x, int ldx, const float* w, float* y, int B, int D, int H, int W,
                    int cin, int cout, int ksd, void* ws, void* stream);
int spff_conv3d_dgrad(const float* dy, const float* w, float* dx, int B, int D, int H, int W,
                      int cin, int cout, int ksd, void* ws, void* stream);
/* the same with an explicit SPFF_MATH_* arithmetic (the two above use SPFF_MATH_F32) */
int spff_conv3d_fwd_ex(const float* x, int ldx, const float* w, float* y, int B, int D, int H,
                       int W, int cin, int cout, int ksd, int math, void* ws, void* stream);
int spff_conv3d_dgrad_ex(const float* dy, const float* w, float* dx, int B, int D, int H, int W,
                         int cin, int cout, int ksd, int math, void* ws, void* stream);
int spff_conv3d_wgrad(const float* x, int ldx, const float* dy, float* dw, int B, int D, int H,
                      int W, int cin, int cout, int ksd, void* ws, void* stream);
int spff_conv3d_wgrad_ex(const float* x, int ldx, const float* dy, float* dw, int B, int D,
                         int H, int W, int cin, int cout, int ksd, int math, void* ws,
                         void* stream);
/* Op-level ConvTranspose3d(cin -> cout, kernel = stride = (1,2,2)) + bias (reference
 * models.py:668-672, the decoder up-convolutions) on channel-last tensors: x [B][D][H][W][cin]
 * low resolution, y [B][D][2H][2W][cout]; weight W[cin][cout][1][2][2], bias [cout].
 * math = SPFF_MATH_*: the GEMM arithmetic (f32 MFMA, the exact bf16x6 split, or f16x3 with
 * per-chunk power-of-two scales).  dgrad: dx = the input gradient of dy; wgrad: dw, db
 * (overwritten).  ws >= spff_upconv_ws_bytes(...). */
size_t spff_upconv_ws_bytes(int B, int D, int H, int W, int cin, int cout);
int spff_upconv_fwd(const float* x, const float* w, const float* b, float* y, int B, int D, int H,
                    int W, int cin, int cout, int math, void* ws, void* stream);
int spff_upconv_dgrad(const float* dy, const float* w, float* dx, int B, int D, int H, int W,
                      int cin, int cout, int math, void* ws, void* stream);
int spff_upconv_wgrad(const float* x, const float* dy, float* dw, float* db, int B, int D, int H,
                      int W, int cin, int cout, int math, void* ws, void* stream);

/* ---------------------------------------------------------------------------
 * 3D U-Net baseline variant (BASELINE config 3; registry entry "3DUNet",
 * config.py:283-311): LitCicek3DUNet_DepthAdapter_Published (models.py:756-853)
 * = _resize_depth_like (models.py:153-157) -> Cicek3DUNet (models.py:718-753:
 * 4 x [Conv3d(3, bias=False) -> BatchNorm3d -> ReLU] x 2 + MaxPool3d(2) down,
 * ConvTranspose3d(2, stride 2) + concat [up, skip] up, 1x1x1 head) ->
 * _resize_logits_depth_like (models.py:159-163).  Same conventions as above:
 * params flat in reference state-dict order (names without the "backbone."
 * prefix), BatchNorm running_mean / running_var in a second flat fp32 buffer
 * (spff_unet3d_buffer_info; num_batches_tracked stays with the caller).
 * -------------------------------------------------------------------------- */
typedef struct spff_unet3d_cfg {
  int batch, in_ch, depth, height, width;  /* input [B][Cin][D][H][W] */
  int target_depth;  /* depth adapter: D is resampled to this before the backbone and the
                        logits back to D (trilinear, align_corners=False); 0 = none.  The
                        backbone depth, H and W must be multiples of 16 (4 poolings). */
  int num_classes;   /* K (<= 32) */
  int base;          /* f (power of two, >= 8); the reference wrapper uses 32 */
  int math;          /* SPFF_MATH_* for the 3x3x3 convolutions */
  int reserved[7];   /* zero */
} spff_unet3d_cfg;

typedef struct spff_unet3d spff_unet3d;

int spff_unet3d_create(const spff_unet3d_cfg* cfg, spff_unet3d** out);
void spff_unet3d_destroy(spff_unet3d* net);
int spff_unet3d_num_params(const spff_unet3d* net);
int spff_unet3d_param_info(const spff_unet3d* net, int i, const char** name, int* ndim,
                           int64_t shape[5], int64_t* offset, int64_t* numel);
int64_t spff_unet3d_param_floats(const spff_unet3d* net);
int spff_unet3d_num_buffers(const spff_unet3d* net);
int spff_unet3d_buffer_info(const spff_unet3d* net, int i, const char** name, int64_t* offset,
                            int64_t* numel);
int64_t spff_unet3d_buffer_floats(const spff_unet3d* net);
size_t spff_unet3d_workspace_bytes(const spff_unet3d* net);
/* forward: x [B][Cin][D][H][W] -> logits [B][D][H][W][K].  training = 1:
 * BatchNorm normalises with batch statistics and updates running_mean /
 * running_var in `buffers` (momentum 0.1, unbiased variance); 0: normalises
 * with the running statistics (buffers read only). */
int spff_unet3d_forward(spff_unet3d* net, const float* x, const float* params, float* buffers,
                        int training, float* logits, void* workspace, void* stream);
/* backward of the last forward: dlogits [B][D][H][W][K] -> dparams (every entry written) */
int spff_unet3d_backward(spff_unet3d* net, const float* dlogits, const float* params,
                         float* dparams, void* workspace, void* stream);
/* Synchronised BatchNorm for data parallelism (torch.nn.SyncBatchNorm semantics): with a
 * table (only its allreduce is used; in-place fp64 sum over the group, in stream order) and
 * world > 1, every train-mode BatchNorm3d all-reduces its per-channel batch moments and its
 * backward's two per-channel sums, so each rank normalises with the global batch statistics
 * and updates identical running statistics; the BN weight / bias gradients stay this
 * rank's partial sums (the caller SUM-all-reduces the flat gradient).  Every rank must run
 * the plan's shape.  NULL or world <= 1: per-replica statistics (the default). */
int spff_unet3d_set_sync_bn(spff_unet3d* net, const spff_coll* coll, int world);
int spff_unet3d_saved_tensor(const spff_unet3d* net, void* workspace, const char* name,
                             const float** ptr, int64_t* nvox, int* channels);

/* the weighted softmax CE of the 3DUNet wrapper (_weighted_softmax_ce,
 * models.py:779-799): as spff_loss, plus optional per-class weights
 * (class_weights: K device floats or NULL) and clamp_denominator = 1 for the
 * wrapper's sum / max(N_valid, 1). */
int spff_loss_ex(const float* logits, const int64_t* labels, int64_t nvox, int num_classes,
                 int ignore_index, double smooth, const int64_t* count_override,
                 const float* class_weights, int clamp_denominator, float* out4,
                 float* dlogits, int64_t* conf, void* ws, void* stream);

/* ------------------------------------------------------------------------
 * SwinUNETR variant (BASELINE config 5; registry "SwinUNETR", config.py:366-386
 * -> LitSwinUNETR_Published / SwinUNETR_Published, models.py:858-982, i.e.
 * MONAI 1.5.2 SwinUNETR).  Replaces SwinUNETR_Published.forward
 * (models.py:877) and its autograd backward, and LitSwinUNETR_Published._loss
 * (models.py:910-928).  Parameters: a flat fp32 buffer in MONAI's state-dict
 * order / names without the "model.model." prefix (spff_swin_param_info);
 * the relative_position_index buffers are not needed.  D, H, W must be
 * multiples of 32.  Parity is unpinned (MONAI is not available offline);
 * semantics in oracle/swin_oracle.py.
 * ------------------------------------------------------------------------ */
typedef struct spff_swin_cfg {
  int batch, in_ch, depth, height, width;  /* input [B][Cin][D][H][W], Cin <= 8 */
  int num_classes;   /* K (<= 32) */
  int feature_size;  /* 12 on the registry path */
  int window;        /* MONAI window_size (7: the registry's (2,2,2) never reaches MONAI) */
  int heads[4];      /* (1, 2, 4, 8) */
  float mlp_ratio;   /* 2.0 */
  int math;          /* SPFF_MATH_* for the 3x3x3 convolutions */
  int reserved[6];   /* zero */
} spff_swin_cfg;

typedef struct spff_swin spff_swin;

int spff_swin_create(const spff_swin_cfg* cfg, spff_swin** out);
void spff_swin_destroy(spff_swin* net);
int spff_swin_num_params(const spff_swin* net);
int spff_swin_param_info(const spff_swin* net, int i, const char** name, int* ndim,
                         int64_t shape[5], int64_t* offset, int64_t* numel);
int64_t spff_swin_param_floats(const spff_swin* net);
size_t spff_swin_workspace_bytes(const spff_swin* net);
/* forward: x [B][Cin][D][H][W] -> logits [B][D][H][W][K] (channel-last) */
int spff_swin_forward(spff_swin* net, const float* x, const float* params, float* logits,
                      void* workspace, void* stream);
/* backward of the last forward: dlogits [B][D][H][W][K] -> dparams (every entry written) */
int spff_swin_backward(spff_swin* net, const float* dlogits, const float* params,
                       float* dparams, void* workspace, void* stream);
int spff_swin_saved_tensor(const spff_swin* net, void* workspace, const char* name,
                           const float** ptr, int64_t* rows, int* channels);
/* (1 - ce_weight) * soft-Dice loss (classes >= 1 unless include_bg) + ce_weight * CE
 * (ignore_index), LitSwinUNETR_Published._loss: out4 = [ce, loss, dice_loss, N_valid],
 * dlogits [V][K] = dloss/dlogits.  ws >= spff_swin_loss_ws_bytes device bytes. */
size_t spff_swin_loss_ws_bytes(int batch, int num_classes);
int spff_swin_loss(const float* logits, const int64_t* labels, int batch, int64_t vox_per_sample,
                   int num_classes, int ignore_index, int include_bg, double ce_weight,
                   float* out4, float* dlogits, void* ws, void* stream);

/* ------------------------------------------------------------------------
 * Training data path on the device (oracle/data_oracle.py).
 * ------------------------------------------------------------------------ */
/* label map of the ellipse ROIs (x0, y0, w0, h0, label) [nroi][5] (device int32), later
 * ROIs overwriting earlier ones, replicated over `frames`: labels [frames][H][W] int64.
 * Replaces the ROI loop of create_image_and_labels_for_dataset (helpers.py:125-129, 199-204). */
int spff_rasterize_ellipses(const int* rois, int nroi, int frames, int height, int width,
                            int64_t* labels, void* stream);
/* [n][hin][win] -> [n][hout][wout] antialiased bilinear (align_corners=False), PyTorch's
 * weights: TF.resize(t, (H, W)) of helpers.py:196.  tmp >= n*hin*wout floats. */
int spff_resize_bilinear_aa(const float* in, int n, int hin, int win, float* out, int hout,
                            int wout, float* tmp, void* stream);
/* TrainGridAug.__call__ (datasets.py:158-209) on a batch x [B][F][H][W] (+ labels y, may be
 * NULL): per sample, prm[8] = {flip_w, flip_h, rot_k, jitter_on, scale, shift, noise_cap
 * (0: no noise), stamp} and maps[H + W] = source row / column of the stripe shuffle in the
 * rotated frame (device arrays; the random draws are the caller's).  xo / yo [B][F][Ho][Wo].
 * ws >= spff_grid_aug_ws_bytes(B). */
size_t spff_grid_aug_ws_bytes(int batch);
int spff_grid_aug(const float* x, const int64_t* y, int batch, int frames, int height, int width,
                  const int* maps, const float* prm, uint64_t seed, float* xo, int64_t* yo,
                  void* ws, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SPFF_H_ */
