// vqa_runtime.hip — error reporting, losses and the Keras-Adam optimizer kernel (gfx950).
//
//   vqa_mse_loss   : keras MeanSquaredError(reduction=NONE) + tf.reduce_mean (vqvae.py:91,125) fused with
//                    its gradient and the spectral-loss gradient add.
//   vqa_adam_keras : keras.optimizers.Adam() defaults as applied by TF's ApplyAdam (vqvae.py:144,362):
//                    one launch over the flat fp32 parameter buffer of all levels.
#include "vqa_common.h"
#include <stdarg.h>
#include <stdio.h>
#include <algorithm>

namespace vqa {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

__global__ __launch_bounds__(256) void mse_kernel(const float* x, const float* r, const float* extra, float* dr,
                                                 long long n, float gscale, float* ws) {
  __shared__ float red[4];
  float part = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float d = r[i] - x[i];
    part += d * d;
    float g = gscale * d;
    if (extra) g = g + extra[i];
    dr[i] = g;
  }
  const float s = block_sum_256(part, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

// float4 form (n % 4 == 0, 16-byte aligned buffers): two float4 of every buffer per thread and trip, both
// loaded before either is used (the second clamped to a valid index, its terms dropped past the end)
__global__ __launch_bounds__(256) void mse4_kernel(const float* x, const float* r, const float* extra, float* dr,
                                                  long long n4, float gscale, float* ws) {
  __shared__ float red[4];
  float part = 0.f;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += 2 * stride) {
    const long long j = i + stride < n4 ? i + stride : i;
    const f32x4 r0 = ((const f32x4*)r)[i], x0 = ((const f32x4*)x)[i];
    const f32x4 r1 = ((const f32x4*)r)[j], x1 = ((const f32x4*)x)[j];
    f32x4 e0 = {0.f, 0.f, 0.f, 0.f}, e1 = e0;
    if (extra) {
      e0 = ((const f32x4*)extra)[i];
      e1 = ((const f32x4*)extra)[j];
    }
    const f32x4 d0 = r0 - x0, d1 = r1 - x1;
    f32x4 g0 = gscale * d0, g1 = gscale * d1;
    if (extra) {
      g0 = g0 + e0;
      g1 = g1 + e1;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) part += d0[k] * d0[k];
    ((f32x4*)dr)[i] = g0;
    if (j != i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) part += d1[k] * d1[k];
      ((f32x4*)dr)[j] = g1;
    }
  }
  const float s = block_sum_256(part, red);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void mse_reduce_kernel(const float* ws, int n, float scale, float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += ws[i];
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) out[0] = s * scale;
}

// TF ApplyAdam (training_ops.cc, non-nesterov): alpha = lr*sqrt(1-b2^t)/(1-b1^t);
// m += (g - m)*(1-b1); v += (g*g - v)*(1-b2); var -= (m*alpha)/(sqrt(v) + eps).
__global__ __launch_bounds__(256) void adam_kernel(float* w, const float* g, float* m, float* v, long long n,
                                                  const int64_t* step, float lr0, const float* lr_dev, float b1,
                                                  float b2, float eps, float gs) {
  const float lr = lr_dev ? lr_dev[0] : lr0;  // a LearningRateSchedule's value at this step (vqa_lr_schedule)
  const float t = (float)(step[0] + 1);
  const float b1p = powf(b1, t), b2p = powf(b2, t);
  const float alpha = lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float omb1 = 1.f - b1, omb2 = 1.f - b2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float gi = g[i] * gs;
    float mi = m[i], vi = v[i];
    mi = mi + (gi - mi) * omb1;
    vi = vi + (gi * gi - vi) * omb2;
    m[i] = mi;
    v[i] = vi;
    w[i] = w[i] - (mi * alpha) / (sqrtf(vi) + eps);
  }
}

// keras LearningRateSchedule evaluated on the device at the optimizer's step counter (OptimizerV2._decayed_lr
// calls the schedule with float(iterations), the count BEFORE this step's increment), so a captured step replays
// with the right rate. Host-precomputed float32 constants keep the arithmetic TF's:
//   kind 1  CustomSchedule (src/transformer/multi_head_attention.py:82-101): p0 = rsqrt(d_model),
//           p1 = warmup_steps ** -1.5 -> p0 * min(rsqrt(s), s * p1)
//   kind 2  keras ExponentialDecay: p0 = initial rate, p1 = decay_steps, p2 = decay_rate, p3 = staircase (0 / 1)
//           -> p0 * p2 ** (s / p1), the exponent floored when staircase
__global__ void lr_schedule_kernel(const int64_t* step, float* lr, int kind, float p0, float p1, float p2, float p3) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const float s = (float)step[0];
  float r = p0;
  if (kind == 1) {
    r = p0 * fminf(1.0f / sqrtf(s), s * p1);
  } else if (kind == 2) {
    float e = s / p1;
    if (p3 != 0.f) e = floorf(e);
    r = p0 * powf(p2, e);
  }
  lr[0] = r;
}

__global__ void counter_add_kernel(int64_t* c, int64_t delta) {
  if (threadIdx.x == 0 && blockIdx.x == 0) c[0] += delta;
}

// The step's metric trackers (vqvae.py:262-304 update_metrics, VectorQuantizer.py:149-159) as one launch:
// macc rows [loss, recon, vqvae, spectral] then per level [level, recon, vq, spectral, batch_usage, usage,
// entropy], each (total, count). loss_slots = per level (recon, commit, spectral) sums over ranks, scaled by
// 1/world; the Python sums of the reference are left folds: level = (recon + commit) + spectral,
// total = ((0 + level_0) + level_1) + ...
__global__ void step_metrics_kernel(const float* loss_slots, const float* vqm, float* macc, int levels,
                                    float scale) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float tot = 0.f, tr = 0.f, tc = 0.f, ts = 0.f;
  for (int l = 0; l < levels; ++l) {
    const float r = loss_slots[3 * l] * scale, c = loss_slots[3 * l + 1] * scale, sp = loss_slots[3 * l + 2] * scale;
    const float lv = (r + c) + sp;
    tot += lv;
    tr += r;
    tc += c;
    ts += sp;
    const float v[7] = {lv, r, c, sp, vqm[3 * l], vqm[3 * l + 1], vqm[3 * l + 2]};
    float* row = macc + 2 * (4 + 7 * l);
    for (int i = 0; i < 7; ++i) {
      row[2 * i] += v[i];
      row[2 * i + 1] += 1.f;
    }
  }
  const float g[4] = {tot, tr, tc, ts};
  for (int i = 0; i < 4; ++i) {
    macc[2 * i] += g[i];
    macc[2 * i + 1] += 1.f;
  }
}

// ---- on-device synthetic waveform feed (replaces the host-side chunk feed of
// data_utils.py:65-206 splitsongs / read_data and the notebook's tf.data pipeline) --------------------------
// x[b][t] = clip(0.5 sin(2 pi f_b t / sr + phi_b) + 0.05 eps, -1, 1), f_b ~ U[55, 2000) Hz, phi_b ~ U[0, 2 pi),
// eps ~ N(0, 1): every draw is a counter-based hash of (seed, rank, item, sample) — no state, any launch
// shape gives the same batch, ranks draw disjoint streams. The phase is reduced in fp64 (t up to 2^31).
__device__ __forceinline__ float u01(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }  // [0, 1)
__device__ __forceinline__ uint64_t feed_key(uint64_t seed, int rank, long long item) {
  return splitmix64(splitmix64(seed ^ 0x5DEECE66DULL) + ((uint64_t)(unsigned)rank << 40) + (uint64_t)item);
}
__global__ __launch_bounds__(256) void synth_kernel(float* x, int B, long long T, uint64_t seed, int rank,
                                                   double inv_sr) {
  const int b = blockIdx.y;
  const uint64_t key = feed_key(seed, rank, b);
  const double f = 55.0 + (2000.0 - 55.0) * (double)u01(splitmix64(key ^ 1));
  const float ph = 6.2831853071795864f * u01(splitmix64(key ^ 2));
  const double cyc_per_sample = f * inv_sr;
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < T; t += (long long)gridDim.x * 256) {
    double c = cyc_per_sample * (double)t;
    c -= floor(c);
    const float s = sinf(6.2831853071795864f * (float)c + ph);
    // Box-Muller from two independent hashes of (key, t)
    const uint64_t h = splitmix64(key + 0x9E3779B97F4A7C15ULL * (uint64_t)(t + 1));
    const float u1 = fmaxf(u01(h), 1.0f / 16777216.0f), u2 = u01(splitmix64(h));
    const float eps = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853071795864f * u2);
    x[(long long)b * T + t] = fminf(fmaxf(0.5f * s + 0.05f * eps, -1.0f), 1.0f);
  }
}

static int blocks_for(long long n, int cap) {
  long long b = (n + 255) / 256;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace vqa

using namespace vqa;

extern "C" const char* vqa_get_last_error(void) { return g_err; }
extern "C" const char* vqa_version(void) { return "libvqa 0.2 gfx950 abi 2"; }
extern "C" int vqa_abi_version(void) { return VQA_ABI_VERSION; }

extern "C" size_t vqa_mse_loss_workspace(int64_t n) { return n < 1 ? 0 : (size_t)blocks_for(n, 1024) * sizeof(float); }

extern "C" int vqa_mse_loss(const float* x, const float* r, const float* extra_grad, float* dr, float* loss_out,
                            int64_t n, void* workspace, size_t ws_bytes, vqa_stream_t stream) {
  VQA_ARG(x && r && dr && loss_out && n > 0, "mse_loss: bad arguments");
  const int nb = blocks_for(n, 1024);
  VQA_ARG(workspace && ws_bytes >= (size_t)nb * sizeof(float), "mse_loss: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const float inv_n = (float)(1.0 / (double)n);
  const float gscale = (float)(2.0 / (double)n);
  if (n % 4 == 0 && ((uintptr_t)x | (uintptr_t)r | (uintptr_t)extra_grad | (uintptr_t)dr) % 16 == 0) {
    hipLaunchKernelGGL(mse4_kernel, dim3(nb), dim3(256), 0, s, x, r, extra_grad, dr, (long long)(n / 4), gscale,
                       (float*)workspace);
    VQA_LAUNCHED("mse4_kernel");
  } else {
    hipLaunchKernelGGL(mse_kernel, dim3(nb), dim3(256), 0, s, x, r, extra_grad, dr, (long long)n, gscale,
                       (float*)workspace);
    VQA_LAUNCHED("mse_kernel");
  }
  hipLaunchKernelGGL(mse_reduce_kernel, dim3(1), dim3(256), 0, s, (const float*)workspace, nb, inv_n, loss_out);
  VQA_LAUNCHED("mse_reduce_kernel");
  return VQA_OK;
}

extern "C" int vqa_adam_keras(float* w, const float* g, float* m, float* v, int64_t n, const int64_t* step, float lr,
                              const float* lr_dev, float beta1, float beta2, float eps, float grad_scale,
                              vqa_stream_t stream) {
  VQA_ARG(w && g && m && v && step && n > 0, "adam: bad arguments");
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n, 4096)), dim3(256), 0, (hipStream_t)stream, w, g, m, v,
                     (long long)n, step, lr, lr_dev, beta1, beta2, eps, grad_scale);
  VQA_LAUNCHED("adam_kernel");
  return VQA_OK;
}

extern "C" int vqa_lr_schedule(const int64_t* step, float* lr, int kind, float p0, float p1, float p2, float p3,
                               vqa_stream_t stream) {
  VQA_ARG(step && lr && kind >= 0 && kind <= 2, "lr_schedule: bad arguments (kind %d)", kind);
  VQA_ARG(kind != 2 || p1 > 0.f, "lr_schedule: decay_steps must be > 0");
  hipLaunchKernelGGL(lr_schedule_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step, lr, kind, p0, p1, p2, p3);
  VQA_LAUNCHED("lr_schedule_kernel");
  return VQA_OK;
}

extern "C" int vqa_counter_add(int64_t* counter, int64_t delta, vqa_stream_t stream) {
  VQA_ARG(counter, "counter_add: null pointer");
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, counter, delta);
  VQA_LAUNCHED("counter_add_kernel");
  return VQA_OK;
}

extern "C" int vqa_step_metrics(const float* loss_slots, const float* vq_metrics, float* macc, int levels, float scale,
                                vqa_stream_t stream) {
  VQA_ARG(loss_slots && vq_metrics && macc && levels > 0, "step_metrics: bad arguments");
  hipLaunchKernelGGL(step_metrics_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, loss_slots, vq_metrics, macc,
                     levels, scale);
  VQA_LAUNCHED("step_metrics_kernel");
  return VQA_OK;
}

extern "C" int vqa_synthetic_batch(float* x, int B, int64_t T, uint64_t seed, int rank, float sample_rate,
                                   vqa_stream_t stream) {
  VQA_ARG(x && B > 0 && T > 0 && B <= 65535 && sample_rate > 0.f, "synthetic_batch: bad arguments");
  const unsigned gx = (unsigned)std::min<long long>((T + 255) / 256, 1024);
  hipLaunchKernelGGL(synth_kernel, dim3(gx, (unsigned)B), dim3(256), 0, (hipStream_t)stream, x, B, (long long)T, seed,
                     rank, 1.0 / (double)sample_rate);
  VQA_LAUNCHED("synth_kernel");
  return VQA_OK;
}
