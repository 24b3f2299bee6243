/*
 * vqa.h — C-ABI of libvqa.so, the MI355X (gfx950) VQ-VAE audio training path.
 *
 * This is the drop-in boundary for the reference's hot path
 * (sunzeyucmu/VAE-based-Music--Deep-Generative-Models). The reference has no
 * FFI: its "operator API" is the set of TensorFlow/Keras ops that its layers
 * call. Each entry point below names the reference call site it replaces.
 *
 * Conventions (all entry points):
 *  - Every pointer is a DEVICE pointer owned by the caller. The library never
 *    allocates on the hot path; ops that need scratch take (workspace, bytes)
 *    and expose a *_workspace() size query.
 *  - Activations are channels-last (N, T, C) contiguous ("NTC"), exactly the
 *    Keras layout. Their element type is `dtype` (VQA_F32 or VQA_BF16) unless a
 *    VQA_X_F32 / VQA_Y_F32 flag forces fp32 on one side. Weights, biases,
 *    gradients of weights, optimizer state and VQ state are always fp32.
 *  - Keras kernel layouts: Conv1D (K, C_in, C_out); Conv1DTranspose
 *    (K, C_out, C_in). Padding is TF "same" (see vqa_same_pad_left).
 *  - Calls are asynchronous on `stream` (a hipStream_t; NULL = default stream)
 *    and never synchronise. Every entry point returns VQA_OK (0) or a negative
 *    VQA_E_* code; the message is in the thread-local vqa_get_last_error().
 *    No C++ exception crosses the ABI. Entry points are reentrant.
 */
#ifndef VQA_H
#define VQA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* vqa_stream_t; /* hipStream_t */

enum { VQA_OK = 0, VQA_E_INVALID_ARG = -1, VQA_E_UNSUPPORTED = -2, VQA_E_HIP = -3 };
enum { VQA_F32 = 0, VQA_BF16 = 1 };

/* conv flags */
enum {
  VQA_PRE_RELU = 1,     /* fwd / bwd_weight: use relu(x) (resnet.py:12,16 layers.ReLU before Conv1D) */
  VQA_ADD_RESIDUAL = 2, /* out = residual + conv(...)   (resnet.py:29 layers.add)                     */
  VQA_POST_MASK = 4,    /* out = (mask > 0) ? conv : 0  (ReLU backward, mask = pre-ReLU tensor)         */
  VQA_X_F32 = 8,        /* the x / dx side tensor is fp32 regardless of dtype                          */
  VQA_Y_F32 = 16        /* the y / dy side tensor is fp32 regardless of dtype                          */
};

/* ---- library -------------------------------------------------------------------------------- */
const char* vqa_get_last_error(void);
const char* vqa_version(void);
/* ABI revision of the signatures in this header. It is raised whenever an existing entry point's argument
 * list changes (revision 2: vqa_adam_keras gained lr_dev, vqa_dropout / vqa_prior_embed_fwd elem_offset,
 * vqa_prior_decode out_ld); a binding built against another revision must refuse the library. */
#define VQA_ABI_VERSION 2
int vqa_abi_version(void);
/* TF SAME padding (Appendix A.2 of SURVEY.md): left pad of a conv with these parameters. Host-only. */
int vqa_same_pad_left(int T_in, int K, int stride, int dilation);
int vqa_same_out_len(int T_in, int stride);

/* ---- Conv1D: replaces keras layers.Conv1D(filters, K, strides, dilation_rate, padding="same")
 *      resnet.py:13, resnet.py:17, encdec.py:33 (down-sampling), encdec.py:38 (projection),
 *      encdec.py:60 (decoder pre-conv), encdec.py:148 (decoder output conv)                      */
int vqa_conv1d_fwd(const void* x, const float* w, const float* bias, const void* residual, void* y,
                   int B, int T_in, int T_out, int C_in, int C_out, int K, int stride, int dilation,
                   int pad_left, int flags, int dtype, vqa_stream_t stream);
/* d(loss)/dx given dy (the GradientTape backward of the same layer, vqvae.py:143).
 * flags: VQA_POST_MASK (mask has dx's shape), VQA_ADD_RESIDUAL (residual has dx's shape). */
int vqa_conv1d_bwd_data(const void* dy, const float* w, const void* mask, const void* residual, void* dx,
                        int B, int T_in, int T_out, int C_in, int C_out, int K, int stride, int dilation,
                        int pad_left, int flags, int dtype, vqa_stream_t stream);
/* dw (K, C_in, C_out) and db (C_out, nullable) — overwritten, not accumulated. flags: VQA_PRE_RELU. */
int vqa_conv1d_bwd_weight(const void* x, const void* dy, float* dw, float* db,
                          int B, int T_in, int T_out, int C_in, int C_out, int K, int stride, int dilation,
                          int pad_left, int flags, int dtype, void* workspace, size_t ws_bytes,
                          vqa_stream_t stream);
size_t vqa_conv1d_bwd_weight_workspace(int B, int T_in, int T_out, int C_in, int C_out, int K, int stride,
                                       int dilation, int pad_left, int flags, int dtype);

/* ---- Conv1DTranspose: replaces keras layers.Conv1DTranspose(filters, 2*stride, strides=stride,
 *      padding="same"), encdec.py:67-68. Supported: stride 2, K 4 (the reference's only use).
 *      w is (K, C_out, C_in); T_out = stride*T_in.                                              */
int vqa_conv1d_transpose_fwd(const void* x, const float* w, const float* bias, const void* residual, void* y,
                             int B, int T_in, int T_out, int C_in, int C_out, int K, int stride,
                             int pad_left, int flags, int dtype, vqa_stream_t stream);
int vqa_conv1d_transpose_bwd_data(const void* dy, const float* w, const void* mask, const void* residual,
                                  void* dx, int B, int T_in, int T_out, int C_in, int C_out, int K,
                                  int stride, int pad_left, int flags, int dtype, vqa_stream_t stream);
int vqa_conv1d_transpose_bwd_weight(const void* x, const void* dy, float* dw, float* db,
                                    int B, int T_in, int T_out, int C_in, int C_out, int K, int stride,
                                    int pad_left, int flags, int dtype, void* workspace, size_t ws_bytes,
                                    vqa_stream_t stream);
size_t vqa_conv1d_transpose_bwd_weight_workspace(int B, int T_in, int T_out, int C_in, int C_out, int K,
                                                 int stride, int pad_left, int flags, int dtype);

/* ---- deferred weight-gradient reduction -------------------------------------------------------------
 * The *_partials variants of the two bwd_weight calls write per-workgroup partial sums into the caller's
 * workspace and fill *desc (host memory) instead of reducing; one vqa_reduce_partials call later reduces
 * any number of them in a single launch (fixed summation order: deterministic). The workspaces must
 * stay allocated until that call has executed on the stream. */
typedef struct {
  const float* partials; /* workspace written by the *_partials call                      */
  float* dw;             /* destination of elements [0, n_w)                                  */
  float* db;             /* destination of elements [n_w, n) (bias), may be NULL              */
  int nparts;            /* partial rows                                                      */
  int n;                 /* elements per partial row                                          */
  int n_w;               /* weight elements per partial row                                   */
  int reserved;
} vqa_partials_desc;
int vqa_conv1d_bwd_weight_partials(const void* x, const void* dy, float* dw, float* db, int B, int T_in, int T_out,
                                   int C_in, int C_out, int K, int stride, int dilation, int pad_left, int flags,
                                   int dtype, void* workspace, size_t ws_bytes, vqa_partials_desc* desc,
                                   vqa_stream_t stream);
int vqa_conv1d_transpose_bwd_weight_partials(const void* x, const void* dy, float* dw, float* db, int B, int T_in,
                                             int T_out, int C_in, int C_out, int K, int stride, int pad_left,
                                             int flags, int dtype, void* workspace, size_t ws_bytes,
                                             vqa_partials_desc* desc, vqa_stream_t stream);
int vqa_reduce_partials(const vqa_partials_desc* descs, int count, vqa_stream_t stream);

/* ---- fused backward of one Conv1D whose input x enters through an optional ReLU (resnet.py:12-17: the
 *      two convs of ResnetConv1DBlock; backward = GradientTape.gradient, vqvae.py:143):
 *      dx = (conv_data_grad(dy) * (x > 0 if VQA_PRE_RELU)) (+ residual if VQA_ADD_RESIDUAL),
 *      dw/db = the weight gradient with relu(x) (VQA_PRE_RELU) or x.
 * Stride-1 convs with 32/64 channels run as ONE kernel that reads dy, x (and residual) once; other shapes
 * fall back to vqa_conv1d_bwd_data + vqa_conv1d_bwd_weight. desc != NULL defers the weight-gradient
 * reduction as in the *_partials calls. */
int vqa_conv1d_bwd_data_weight(const void* dy, const float* w, const void* x, const void* residual, void* dx,
                               float* dw, float* db, int B, int T_in, int T_out, int C_in, int C_out, int K,
                               int stride, int dilation, int pad_left, int flags, int dtype, void* workspace,
                               size_t ws_bytes, vqa_partials_desc* desc, vqa_stream_t stream);
size_t vqa_conv1d_bwd_data_weight_workspace(int B, int T_in, int T_out, int C_in, int C_out, int K, int stride,
                                            int dilation, int pad_left, int flags, int dtype);

/* ---- fused residual block: replaces resnet.py:7-29 ResnetConv1DBlock (C = 32):
 *      h = conv_a(relu(x)) + b_a (k3, dilation), y = x + conv_b(relu(h)) + b_b (k3, dilation 1), SAME padding.
 * Weights in Keras layout (3, C, C). The forward keeps h on chip; h_out (nullable) receives relu(h).
 * The backward recomputes h from x, so it reads dy and x and writes dx = d loss / d x; the four weight
 * gradients (overwritten) are reduced from per-workgroup partials — or, with desc != NULL (2 entries:
 * conv_a, conv_b), left for a later vqa_reduce_partials call. */
int vqa_resblock_supported(int C, int dilation, int dtype);
int vqa_resblock_fwd(const void* x, const float* wa, const float* ba, const float* wb, const float* bb, void* y,
                     void* h_out, int B, int T, int C, int dilation, int dtype, vqa_stream_t stream);
int vqa_resblock_bwd(const void* dy, const void* x, const float* wa, const float* ba, const float* wb, const float* bb,
                     void* dx, float* dwa, float* dba, float* dwb, float* dbb, int B, int T, int C, int dilation,
                     int dtype, void* workspace, size_t ws_bytes, vqa_partials_desc* desc, vqa_stream_t stream);
size_t vqa_resblock_bwd_workspace(int B, int T, int C, int dilation, int dtype);

/* ---- decoder tail: the last Conv1DTranspose (K=4, stride 2, C -> Cu) of the last decoder block followed by
 *      the decoder's output Conv1D (K=3, Cu -> 1), encdec.py:67-68 then :148, with nothing in between, run as
 *      ONE thin 3-tap convolution from h (B, T, C) to y (B, 2T, 1) fp32 (the two linear maps composed; the
 *      Cu-channel full-rate tensor is never formed). Backward: dh (B, T, C) and the four parameter gradients
 *      (written, not accumulated) from dy (B, 2T, 1) fp32. C must be 32. */
int vqa_dtail_supported(int C, int Cu, int K_up, int stride_up, int K_out, int C_out, int dtype);
size_t vqa_dtail_workspace(int B, int T, int C, int Cu, int dtype);
int vqa_dtail_fwd(const void* h, const float* w_up, const float* b_up, const float* w_out, const float* b_out,
                  float* y, int B, int T, int C, int Cu, int dtype, void* workspace, size_t ws_bytes,
                  vqa_stream_t stream);
int vqa_dtail_bwd(const float* dy, const void* h, const float* w_up, const float* b_up, const float* w_out,
                  const float* b_out, void* dh, float* dw_up, float* db_up, float* dw_out, float* db_out, int B,
                  int T, int C, int Cu, int dtype, void* workspace, size_t ws_bytes, vqa_stream_t stream);

/* ---- Vector quantizer (VectorQuantizer.py) ---------------------------------------------------- */
/* e_sqnorm[k] = sum_d E[d][k]^2  (VectorQuantizer.py:180). E is (D, K). */
int vqa_vq_sqnorm(const float* E, float* e_sqnorm, int D, int K, vqa_stream_t stream);
/* idx[n] = argmin_k (sum_d z[n][d]^2 + e_sqnorm[k]) - 2 * (z @ E)[n][k]; ties -> lowest k.
 * Replaces get_code_indices, VectorQuantizer.py:170-186. min_dist nullable. z is (N, D) in dtype. */
int vqa_vq_argmin(const void* z, const float* E, const float* e_sqnorm, int64_t* idx, float* min_dist,
                  int64_t N, int D, int K, int dtype, vqa_stream_t stream);
/* The same argmin for bf16 z (D in {32, 64}) on bf16 MFMA: E3 (K, 3, D) bf16 holds hi, mid, lo planes with
 * hi + mid + lo = E exactly (vqa_vq_split_bf16x3, run after every codebook update), so each z.e is a sum of
 * exact products accumulated in fp32, as with the fp32 path. */
int vqa_vq_argmin_split(const void* z, const void* E3, const float* e_sqnorm, int64_t* idx, float* min_dist,
                        int64_t N, int D, int K, vqa_stream_t stream);
int vqa_vq_split_bf16x3(const float* E, void* E3, int D, int K, vqa_stream_t stream);
/* q = ET[idx] (one_hot @ E^T, :86-90); q_st = z + (q - z) (:114);
 * commit_out[0] = beta * mean((q - z)^2) (:97-99);
 * if m_sumT != NULL: m_sumT[k][d] += sum_{n: idx[n]=k} z[n][d], n_sum[k] += count (:123-124; the
 * caller zeroes them first). ET is the (K, D) transpose of E kept by vqa_vq_ema_apply. */
int vqa_vq_quantize(const void* z, const float* ET, const int64_t* idx, void* q_st, float* commit_out,
                    float* m_sumT, float* n_sum, int64_t N, int D, int K, float beta, int dtype,
                    void* workspace, size_t ws_bytes, vqa_stream_t stream);
size_t vqa_vq_quantize_workspace(int64_t N, int D, int K, int dtype);
/* Gradient of the quantizer: dz = dq_st + scale * (z - ET[idx])  (straight-through :114 plus the
 * commitment term :97-99; scale = 2*beta/(N_global*D)). */
int vqa_vq_backward(const void* dq, const void* z, const float* ET, const int64_t* idx, void* dz, float scale,
                    int64_t N, int D, int dtype, vqa_stream_t stream);
/* Dead-code reset candidates (VectorQuantizer.py:137 shuffle(_tile(flat))[:K], _tile :191-199) with an
 * injected permutation: RT[k][:] = z_global[perm(k) mod N_global] if that row lives on this rank
 * (global rows [row_offset, row_offset + N_local)), else 0. perm = vqa_reset_perm_index(seed,
 * *counter, level, M, k) with M = N_global (or N_global*ceil(K/N_global) when N_global < K). */
int vqa_vq_reset_rows(const void* z, float* RT, int64_t N_local, int64_t row_offset, int64_t N_global,
                      int D, int K, uint64_t seed, const int64_t* counter, int level, int dtype,
                      vqa_stream_t stream);
/* EMA codebook update (VectorQuantizer.py:126-145) from (all-reduced) m_sumT/n_sum/RT:
 * N_t = g*N_t + omg*n_sum; m_t = g*m_t + omg*m_sum; usage = N_t >= thresh;
 * E = usage ? m_t / clip(N_t, 1e-8, 1e8) : R; ET = E^T. Increments *counter.
 * metrics[0..2] = batch usage, running usage, entropy (VectorQuantizer.py:149-159). */
int vqa_vq_ema_apply(float* E, float* ET, float* m_t, float* N_t, const float* m_sumT, const float* n_sum,
                     const float* RT, float gamma, float one_minus_gamma, float thresh, float* metrics,
                     int64_t* counter, int D, int K, vqa_stream_t stream);
/* vqa_vq_ema_apply that also writes the codebook's derived state the next argmin reads, in the same pass:
 * e_sqnorm (K) = |e_k|^2 (vqa_vq_sqnorm's bits) and E3 (K, 3, D) bf16 = the hi/mid/lo planes
 * (vqa_vq_split_bf16x3's bits); either may be NULL. Replaces the :144-145 update plus the two follow-up launches. */
int vqa_vq_ema_apply_derived(float* E, float* ET, float* m_t, float* N_t, const float* m_sumT, const float* n_sum,
                             const float* RT, float gamma, float one_minus_gamma, float thresh, float* metrics,
                             int64_t* counter, float* e_sqnorm, void* E3, int D, int K, vqa_stream_t stream);
/* The reset permutation (host-callable; the device uses the same code): a keyed 4-round Feistel
 * bijection on [0, M) with cycle walking. Returns the k-th sampled row of the tiled batch. */
int64_t vqa_reset_perm_index(uint64_t seed, int64_t counter, int level, int64_t M, int64_t k);

/* ---- upper-level conditioner (src/conditioner/conditioners.py:42-72 ConditionerNet) ---------------
 * Embedding (layers.Embedding(bins, width), :64): out[n][:] = table[idx[n]][:] (table (K, D) fp32, out in the
 * activation dtype; an index outside [0, K) gives a zero row). Backward: dtable[k][:] += sum_{n: idx[n]=k}
 * dy[n][:] in a fixed order (the counting sort + segment sums of the EMA statistics; deterministic). */
int vqa_embedding_fwd(const float* table, const int64_t* idx, void* out, int64_t N, int D, int K, int dtype,
                      vqa_stream_t stream);
int vqa_embedding_bwd(const void* dy, const int64_t* idx, float* dtable, int64_t N, int D, int K, int dtype,
                      void* workspace, size_t ws_bytes, vqa_stream_t stream);
size_t vqa_embedding_bwd_workspace(int64_t N, int D, int K);
/* LayerNormalization(axis=-1, epsilon) (:70): y = (x - mean) / sqrt(var + eps) * gamma + beta over the last
 * axis (C <= 1024), biased variance, fp32 statistics; x, y in the activation dtype. Backward: dx, and
 * dgamma = sum dy*xhat, dbeta = sum dy written (per-workgroup partials reduced in a fixed order; desc != NULL
 * defers that reduction as in the *_partials calls). */
int vqa_layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, int64_t rows, int C, float eps,
                      int dtype, vqa_stream_t stream);
int vqa_layernorm_bwd(const void* x, const void* dy, const float* gamma, void* dx, float* dgamma, float* dbeta,
                      int64_t rows, int C, float eps, int dtype, void* workspace, size_t ws_bytes,
                      vqa_partials_desc* desc, vqa_stream_t stream);
size_t vqa_layernorm_bwd_workspace(int64_t rows, int C);

/* ---- losses / optimizer ------------------------------------------------------------------------ */
/* loss_out[0] = mean((r - x)^2) (vqvae.py:91,125); dr = 2*(r - x)/n + extra (extra nullable). fp32. */
int vqa_mse_loss(const float* x, const float* r, const float* extra_grad, float* dr, float* loss_out,
                 int64_t n, void* workspace, size_t ws_bytes, vqa_stream_t stream);
size_t vqa_mse_loss_workspace(int64_t n);
/* Keras 2.7 Adam (vqvae.py:144, compile at :362; TF ApplyAdam): t = *step + 1,
 * alpha = lr*sqrt(1-b2^t)/(1-b1^t); m += (g*s - m)(1-b1); v += ((g*s)^2 - v)(1-b2);
 * w -= alpha*m/(sqrt(v)+eps), with s = grad_scale. Does not touch *step. lr_dev (nullable): a device scalar
 * that replaces lr (a LearningRateSchedule's value for this step, written by vqa_lr_schedule). */
int vqa_adam_keras(float* w, const float* g, float* m, float* v, int64_t n, const int64_t* step, float lr,
                   const float* lr_dev, float beta1, float beta2, float eps, float grad_scale, vqa_stream_t stream);
/* keras LearningRateSchedule at the optimizer's device step counter (OptimizerV2._decayed_lr: schedule(float(
 * iterations)), before the step's increment): *lr = f(*step), so a captured train step replays with the right rate.
 * kind 0: p0. kind 1, CustomSchedule (src/transformer/multi_head_attention.py:82-101): p0 = rsqrt(d_model),
 * p1 = warmup_steps^-1.5: p0 * min(rsqrt(s), s * p1). kind 2, keras ExponentialDecay: p0 = initial rate,
 * p1 = decay_steps, p2 = decay_rate, p3 = staircase: p0 * p2^(s / p1) (exponent floored when staircase). */
int vqa_lr_schedule(const int64_t* step, float* lr, int kind, float p0, float p1, float p2, float p3,
                    vqa_stream_t stream);
/* The train step's metric trackers in one launch (replaces update_metrics, vqvae.py:262-304, and the VQ
 * trackers, VectorQuantizer.py:149-159): macc is (4 + 7*levels) x (total, count) — rows loss, recon_loss,
 * vqvae_loss, spectral_loss, then per level level/recon/vq/spectral loss, batch usage, usage, entropy;
 * loss_slots (levels x 3: recon, commit, spectral) are scaled by `scale` (1/world) first; vq_metrics is
 * levels x 3 (vqa_vq_ema_apply's metrics). Each row gets total += value, count += 1 (keras Mean). */
int vqa_step_metrics(const float* loss_slots, const float* vq_metrics, float* macc, int levels, float scale,
                     vqa_stream_t stream);
/* On-device synthetic feed (replaces the host chunk feed of data_utils.py:65-206 and the
 * notebook tf.data pipeline): x (B, T) fp32 = clip(0.5 sin(2 pi f_b t / sr + phi_b) + 0.05 N(0,1), -1, 1) with
 * f_b ~ U[55, 2000) Hz, phi_b ~ U[0, 2 pi); counter-based draws keyed by (seed, rank, item, sample). */
int vqa_synthetic_batch(float* x, int B, int64_t T, uint64_t seed, int rank, float sample_rate,
                        vqa_stream_t stream);
/* *counter += delta on the stream (graph-capturable step counters). */
int vqa_counter_add(int64_t* counter, int64_t delta, vqa_stream_t stream);

/* ---- multi-resolution spectral loss --------------------------------------------------------------
 * Replaces vqvae.py:309-326 (_multispectral_loss) over data_utils.py:25-30 (spectral = |tf.signal.stft|)
 * and data_utils.py:33-40 (norm = tf.norm 'fro'), plus its GradientTape backward (vqvae.py:143):
 *   loss_out[0] = mean_b mean_res ||S_x[b] - S_r[b]||_F / ||S_x[b]||_F,
 *   S = |rfft(frame * hann_periodic(win), n_fft)|, frame f = sig[f*hop : f*hop + win], F = 1 + (T-win)/hop
 *   (no centering, pad_end=False), dr = d loss_out / d r (nullable: loss only; abs'(0) = 0 as in TF),
 *   item_loss[b] = mean_res of item b's loss (nullable).
 * x, r, dr: (B, T) fp32. STFT parameters are host arrays of nres (<= 8) entries; n_fft in {256, 512, 1024,
 * 2048}, win <= n_fft, win <= T. with_grad selects the workspace size with (1) or without (0) dr. */
int vqa_spectral_loss(const float* x, const float* r, float* loss_out, float* dr, float* item_loss, int B, int T,
                      const int* n_fft, const int* hop, const int* win, int nres, void* workspace, size_t ws_bytes,
                      vqa_stream_t stream);
size_t vqa_spectral_loss_workspace(int B, int T, const int* n_fft, const int* hop, const int* win, int nres,
                                   int with_grad);
/* The same loss in two parts, for a target shared by several reconstructions (the levels of one train
 * step): vqa_spectral_target writes the FFT tables and |S_x| of every resolution into `target`
 * (vqa_spectral_target_workspace bytes); vqa_spectral_loss_target then takes that buffer instead of x
 * (workspace: vqa_spectral_loss_target_workspace). vqa_spectral_loss = both in one call. */
size_t vqa_spectral_target_workspace(int B, int T, const int* n_fft, const int* hop, const int* win, int nres);
int vqa_spectral_target(const float* x, void* target, size_t target_bytes, int B, int T, const int* n_fft,
                        const int* hop, const int* win, int nres, vqa_stream_t stream);
size_t vqa_spectral_loss_target_workspace(int B, int T, const int* n_fft, const int* hop, const int* win, int nres,
                                          int with_grad);
int vqa_spectral_loss_target(const void* target, const float* r, float* loss_out, float* dr, float* item_loss, int B,
                             int T, const int* n_fft, const int* hop, const int* win, int nres, void* workspace,
                             size_t ws_bytes, vqa_stream_t stream);
/* data_utils.py:25-30 spectral(x) for one resolution: mag (B, F, n_fft/2 + 1) fp32 = |tf.signal.stft(x)|. */
int vqa_stft_magnitude(const float* x, float* mag, int B, int T, int n_fft, int hop, int win, vqa_stream_t stream);

/* ==== factorized-attention prior (BASELINE configs 4-5) ==================== *
 * src/transformer/{factorized_attention,transformer}.py, src/autoregressive/autoregressive_fmha.py, prior.py.
 * Rows are (nseq, T) sequences of channels-last vectors in the activation dtype; weights fp32, Keras layouts. */

/* Sequence-linear layer (MFMA): y[r][n] = sum_tap sum_k x[src(r,tap)][k] * Wv[tap][k][n] + bias[n]
 * (+ residual[r][n]) (+ y[r][n] when accumulate), src(r,tap) = the same sequence at t + dir*(taps-1-tap), zero
 * outside [0, T). Wv[tap][k][n] = wtrans ? w[(tap*N + n)*K + k] : w[(tap*K + k)*N + n].
 *   dir=-1, taps=3, wtrans=0: Conv1D(3w, 3, padding="causal") (factorized_attention.py:36)
 *   dir=+1, taps=3, wtrans=1: its data gradient
 *   taps=1: layers.Dense / MultiHeadAttention EinsumDense (factorized_attention.py:39-50, transformer.py:30)
 *           and, wtrans=1, their data gradients.
 * ldx/ldr/ldy are row strides in elements (column slices of a wider tensor are allowed). K <= 256, N <= 128,
 * N % 16 == 0, K % 32 (bf16) / 4 (fp32) == 0. */
int vqa_seqlin_fwd(const void* x, int64_t ldx, const float* w, const float* bias, const void* residual, int64_t ldr,
                   void* y, int64_t ldy, int nseq, int T, int K, int N, int taps, int dir, int wtrans, int accumulate,
                   int dtype, vqa_stream_t stream);
/* The same layer with weights prepared once per step by vqa_seqlin_prep: wp = Wv laid out [taps][N][K] in the
 * activation dtype (the kernel stages it with plain 16-byte copies). vqa_seqlin_prep converts a batch of
 * layers in one launch: out[tap][n][k] = wtrans ? w[(tap*N + n)*K + k] : w[(tap*K + k)*N + n]. */
typedef struct {
  const float* w;
  void* out;
  int taps, K, N, wtrans;
} vqa_seqlin_prep_desc;
int vqa_seqlin_prep(const vqa_seqlin_prep_desc* descs, int count, int dtype, vqa_stream_t stream);
int vqa_seqlin_fwd_prepped(const void* x, int64_t ldx, const void* wp, const float* bias, const void* residual,
                           int64_t ldr, void* y, int64_t ldy, int nseq, int T, int K, int N, int taps, int dir,
                           int accumulate, int dtype, vqa_stream_t stream);
/* vqa_seqlin_fwd_prepped of LayerNorm(x; gamma, beta, eps) without materialising it: transformer.py:24-30's
 * LayerNorm -> FactorizedAttention qkv Conv1D and LayerNorm -> mlp Dense (+ x1) in one launch. Bit-identical to
 * vqa_layernorm_fwd followed by vqa_seqlin_fwd_prepped (rows outside [0, T) are zero, not beta). bf16, K = 128
 * only; VQA_E_UNSUPPORTED otherwise (callers then run the two launches). */
int vqa_seqlin_fwd_ln_prepped(const void* x, int64_t ldx, const float* gamma, const float* beta, float eps,
                              const void* wp, const float* bias, const void* residual, int64_t ldr, void* y,
                              int64_t ldy, int nseq, int T, int K, int N, int taps, int dir, int dtype,
                              vqa_stream_t stream);
/* dW[tap][k][n] = sum_t x[t-(taps-1-tap)][k] dy[t][n], db = sum_t dy[t] (deterministic partials; desc != NULL
 * defers the reduction as for the conv weight gradients). K <= 128, N <= 128, multiples of 16. */
size_t vqa_seqlin_wgrad_workspace(int nseq, int T, int K, int N, int taps);
int vqa_seqlin_wgrad(const void* x, int64_t ldx, const void* dy, int64_t lddy, float* dw, float* db, int nseq, int T,
                     int K, int N, int taps, int dtype, void* workspace, size_t ws_bytes, vqa_partials_desc* desc,
                     vqa_stream_t stream);
/* autoregressive_fmha.py:119-151: out = table[tokens] (row 0 <- ycond when given) * scale + pos[t]; keras
 * Dropout(rate) with a counter-based mask (seed, and the device step counter when given, so a replayed graph
 * draws a new mask each step); + xcond (N, T, W) when given. The mask is vqa_dropout's over the flat
 * (N, T, W) index (+ elem_offset: under data parallelism the rank's first global index, rank * N*T*W, so the
 * ranks draw the single-process mask of the global batch) with salt VQA_EMB_DROPOUT_SALT: the gradient of the
 * dropout is vqa_dropout(dx, N*T*W, rate, seed, VQA_EMB_DROPOUT_SALT, elem_offset, counter). */
#define VQA_EMB_DROPOUT_SALT 0x454d42ull
int vqa_prior_embed_fwd(const float* table, const float* pos, const int64_t* tokens, const float* ycond,
                        const void* xcond, void* out, int N, int T, int W, int bins, float scale, float rate,
                        uint64_t seed, int64_t elem_offset, const int64_t* counter, int dtype, vqa_stream_t stream);
/* out[i] (+)= sum_{n < nout} x[n*ostride + i], i < inner (fp32 out, fixed order): positional-embedding and
 * bias gradients. */
int vqa_colsum(const void* x, float* out, int nout, int64_t ostride, int64_t inner, int accumulate, int dtype,
               vqa_stream_t stream);
int vqa_axpy(const void* x, const void* y, void* z, int64_t n, int dtype, vqa_stream_t stream); /* z = x + y */
/* keras Dropout(rate) in place (src/transformer/transformer.py:31-33, autoregressive_fmha.py:151):
 * x * 1/(1-rate) where uniform(seed, salt, elem_offset + i) >= rate, else 0. elem_offset: the global flat index of
 * x[0] (data parallel: rank * n), so DP ranks apply the single-process mask of the global batch. */
int vqa_dropout(void* x, int64_t n, float rate, uint64_t seed, uint64_t salt, int64_t elem_offset,
                const int64_t* counter, int dtype, vqa_stream_t stream);
int vqa_scale_f32(float* x, int64_t n, float s, vqa_stream_t stream);
/* prior.py:262-290 teacher forcing: latent = [start, codes[:-1]]; pred = [start, amax[:-1]];
 * out = m ? pred : latent, m = mask[r] (uint8, when given) or uniform(seed, step + *counter, row_offset + r)
 * < rate (row_offset: the rank's first row of the global batch under data parallelism); amax NULL: out =
 * latent. */
int vqa_tf_mix(const int64_t* codes, const int64_t* amax, const uint8_t* mask, int64_t* out, int N, int T,
               int64_t start, float rate, uint64_t seed, uint64_t step, int64_t row_offset, const int64_t* counter,
               vqa_stream_t stream);
/* Factorized attention core of keras MultiHeadAttention (softmax(q k^T * scale + mask) v per head) on the
 * projected q, k, v (N, T, H*head_dim), head_dim 16. mode 0 row (causal within blocks of l,
 * factorized_attention.py:74-141), 1 col (causal over blocks at a fixed position, :210-286), 2 prev-row
 * (block b attends block b-1; block 0 attends the zero block, so o = vbias, :308-388). lse (N, T, H) fp32
 * (log2 domain) is saved for the backward. Modes 0/2 need l % 64 == 0; mode 1 needs T/l <= 8. */
int vqa_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const float* vbias, int N, int T,
                 int H, int head_dim, int l, int mode, float scale, int dtype, vqa_stream_t stream);
/* dq, dk, dv from dout (deterministic: one kernel per query tile for dq, one per key tile for dk/dv).
 * dsum: (N, T, H) fp32 scratch (modes 0/2). For mode 2 the zero block's value-bias gradient is the column
 * sum of dout over block 0 (vqa_colsum); dq of block 0 is zero. */
int vqa_attn_bwd(const void* q, const void* k, const void* v, const void* o, const float* lse, const void* dout,
                 float* dsum, void* dq, void* dk, void* dv, int N, int T, int H, int head_dim, int l, int mode,
                 float scale, int dtype, vqa_stream_t stream);
/* Output head Dense(bins) fused with SparseCategoricalCrossentropy(from_logits) / accuracy
 * (autoregressive_fmha.py:80,158; autoregressive.py:189-212); logits are never written. wt = W^T (V, K) in
 * the activation dtype (vqa_head_wt). K = 128. head_fwd: per row lse, argmax (first maximum), and with
 * targets the row loss lse - logit[target] and correctness (1/0). head_bwd: dx = dlogits W^T, dW, db with
 * dlogits = (softmax - onehot) * inv_count. */
int vqa_head_wt(const float* w, void* wt, int K, int V, int dtype, vqa_stream_t stream);
int vqa_head_fwd(const void* x, const void* wt, const float* bias, const int64_t* targets, float* lse, int64_t* amax,
                 float* loss_row, float* correct, int64_t M, int K, int V, int dtype, vqa_stream_t stream);
size_t vqa_head_bwd_workspace(int64_t M, int K, int V);
int vqa_head_bwd(const void* x, const void* wt, const float* bias, const int64_t* targets, const float* lse,
                 float inv_count, void* dx, float* dw, float* db, int64_t M, int K, int V, int dtype, void* workspace,
                 size_t ws_bytes, vqa_partials_desc* desc, vqa_stream_t stream);
/* out[i] = scale * sum_j x[i*n + j] (fixed-order two-stage reduction; workspace vqa_rowsum_workspace bytes). */
size_t vqa_rowsum_workspace(int64_t rows, int64_t n);
int vqa_rowsum(const float* x, int64_t rows, int64_t n, float scale, float* out, void* workspace, size_t ws_bytes,
               vqa_stream_t stream);

/* Autoregressive sampling (autoregressive_fmha.py:162-240, Sampler.py): one persistent workgroup per sample
 * walks `steps` positions with a key/value cache, z = logits + Gumbel(uniform(seed, sample, step, bin)),
 * next token = argmax z. tokens (N, steps+1) int64 with tokens[:, 0] = start. Optional: ycond (N, width)
 * label embedding for position 0, xcond (N, ctx, width) fp32 upper-level conditioning, forced (N, steps+1)
 * input tokens (teacher-forced check), logits (N, steps, bins) output. width 128, attention width 32.
 * out_kernel is (width, out_ld) row-major with out_ld >= bins a multiple of 4 and out_bias has out_ld entries
 * (a vocabulary that is not a multiple of 4, e.g. the sampler's default 513 bins, is passed zero-padded; the
 * padded columns are never sampled). */
typedef struct {
  const float *ln1_gamma, *ln1_beta, *qkv_kernel, *qkv_bias, *query_kernel, *query_bias, *key_kernel, *key_bias,
      *value_kernel, *value_bias, *out_kernel, *out_bias, *proj_kernel, *proj_bias, *ln2_gamma, *ln2_beta,
      *mlp_kernel, *mlp_bias;
  int attn_type; /* 0 row, 1 col, 2 prev-row (transformer.py:82-86) */
} vqa_prior_layer;
size_t vqa_prior_decode_cache_bytes(int N, int depth, int ctx);
int vqa_prior_decode(const vqa_prior_layer* layers, int depth, const float* x_embedding, const float* pos_embedding,
                     const float* out_kernel, const float* out_bias, const float* ycond, const float* xcond,
                     const int64_t* forced, float* logits, int64_t* tokens, void* cache, size_t cache_bytes, int N,
                     int steps, int ctx, int width, int heads, int blocks, int bins, int out_ld, int64_t start,
                     uint64_t seed, vqa_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* VQA_H */
