// adamw.hip — the step's optimizer tail in three launches: global-norm gradient clipping
// and AdamW over a table of parameter tensors.
//
// Reference: onebit_asr/train.py:116-118 (clip_grad_norm_(model.parameters(), 5.0);
// optimizer.step()) with the optimizer of train.py:259 (AdamW, betas (0.9, 0.98),
// weight_decay 1e-2, eps 1e-8). torch runs these as a per-tensor norm, a norm of norms, a
// scale of every gradient and the AdamW update, i.e. hundreds of small launches per step
// for the ~800 parameter tensors of Conformer-S; here:
//   (every gradient is first multiplied by grad_scale: 1/world after a SUM all-reduce)
//   1. adamw_norm_kernel     one block per 4096-element chunk of one tensor: sum g^2
//                            (fixed order) -> partial[block];
//   2. adamw_finalize_kernel one block: total norm (fixed order, fp64), clip coefficient
//                            min(1, max_norm / (norm + 1e-6)), step += 1, bias corrections;
//   3. adamw_update_kernel   per chunk: g *= coef; AdamW with torch's operation order
//                            (decoupled decay, lerp for m, addcmul for v, sqrt(v)/sqrt(bc2)
//                            + eps, addcdiv) -- torch/optim/adamw.py _single_tensor_adam.
// The clipped gradient is used in registers; grads are not rewritten. lr and the step
// counter live on the device, so the three launches replay unchanged in a HIP graph.
#include <math.h>

#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 4096;  // elements per block (16 per thread)

struct Scalars {  // written by the finalize kernel, read by the update kernel
  float coef, decay, step_size, bc2_sqrt;
  float total_norm, pad0, pad1, pad2;
};

__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float s = 0.0f;
  if (threadIdx.x == 0) {
    for (int w = 0; w < kThreads / 64; ++w) s += red[w];
  }
  return s;  // valid in thread 0
}

__global__ __launch_bounds__(kThreads) void adamw_norm_kernel(const AdamwTensor* __restrict__ tab,
                                                              const int64_t* __restrict__ map,
                                                              float grad_scale,
                                                              float* __restrict__ partial) {
  __shared__ float red[kThreads / 64];
  const int64_t t = map[2 * blockIdx.x];
  const int64_t s0 = map[2 * blockIdx.x + 1];
  const AdamwTensor d = tab[t];
  const int64_t end = min<int64_t>(s0 + kChunk, d.numel);
  float acc = 0.0f;
  for (int64_t i = s0 + threadIdx.x; i < end; i += kThreads) {
    const float g = d.grad[i] * grad_scale;
    acc = fmaf(g, g, acc);
  }
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(kThreads) void adamw_finalize_kernel(
    const float* __restrict__ partial, int64_t nb, const float* __restrict__ lr_dev,
    float* __restrict__ step_dev, double beta1, double beta2, double weight_decay, float max_norm,
    Scalars* __restrict__ sc, float* __restrict__ total_norm_out) {
  __shared__ double red[kThreads];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < nb; i += kThreads) acc += (double)partial[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = kThreads / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const float norm = (float)sqrt(red[0]);
  float coef = 1.0f;
  if (max_norm > 0.0f) {  // torch: clip_coef = max_norm / (total_norm + 1e-6), clamp(max=1)
    coef = max_norm / (norm + 1e-6f);
    coef = fminf(coef, 1.0f);
  }
  const float step = *step_dev + 1.0f;
  *step_dev = step;
  const double lr = (double)*lr_dev;
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  sc->coef = coef;
  sc->decay = (float)(1.0 - lr * weight_decay);
  sc->step_size = (float)(lr / bc1);
  sc->bc2_sqrt = (float)sqrt(bc2);
  sc->total_norm = norm;
  if (total_norm_out) *total_norm_out = norm;
}

__global__ __launch_bounds__(kThreads) void adamw_update_kernel(
    const AdamwTensor* __restrict__ tab, const int64_t* __restrict__ map,
    const Scalars* __restrict__ sc, float grad_scale, float w1, float beta2,
    float one_minus_beta2, float eps) {
  const int64_t t = map[2 * blockIdx.x];
  const int64_t s0 = map[2 * blockIdx.x + 1];
  const AdamwTensor d = tab[t];
  const int64_t end = min<int64_t>(s0 + kChunk, d.numel);
  const float coef = sc->coef, decay = sc->decay, step_size = sc->step_size,
              bc2s = sc->bc2_sqrt;
  for (int64_t i = s0 + threadIdx.x; i < end; i += kThreads) {
    const float g = (d.grad[i] * grad_scale) * coef;  // clip_grad_norm_: grads.mul_(coef)
    float p = d.param[i] * decay;                     // param.mul_(1 - lr * wd)
    float m = d.exp_avg[i];
    m = m + w1 * (g - m);                             // exp_avg.lerp_(grad, 1 - beta1)
    float v = d.exp_avg_sq[i] * beta2;                // exp_avg_sq.mul_(beta2)
    v = v + one_minus_beta2 * g * g;                  //   .addcmul_(grad, grad, 1 - beta2)
    const float denom = sqrtf(v) / bc2s + eps;        // (sqrt(v) / sqrt(bc2)).add_(eps)
    p = p + (-step_size) * (m / denom);               // param.addcdiv_(m, denom, -step_size)
    d.param[i] = p;
    d.exp_avg[i] = m;
    d.exp_avg_sq[i] = v;
  }
}

}  // namespace

int64_t adamw_plan(const int64_t* numels, int64_t n, int64_t* map) {
  int64_t nb = 0;
  for (int64_t t = 0; t < n; ++t) {
    for (int64_t s = 0; s < numels[t]; s += kChunk) {
      if (map) {
        map[2 * nb] = t;
        map[2 * nb + 1] = s;
      }
      ++nb;
    }
  }
  return nb;
}

size_t adamw_workspace(int64_t n_blocks) {
  return sizeof(float) * (size_t)n_blocks + 2 * sizeof(Scalars) + 64;
}

void launch_adamw(const AdamwTensor* tab, const int64_t* map, int64_t nb, const float* lr,
                  float* step, float grad_scale, double beta1, double beta2, double eps,
                  double weight_decay, double max_norm, float* total_norm_out, void* ws,
                  hipStream_t s) {
  float* partial = (float*)ws;
  Scalars* sc = (Scalars*)((char*)ws + ((sizeof(float) * (size_t)nb + 63) / 64) * 64);
  hipLaunchKernelGGL(adamw_norm_kernel, dim3((unsigned)nb), dim3(kThreads), 0, s, tab, map,
                     grad_scale, partial);
  hipLaunchKernelGGL(adamw_finalize_kernel, dim3(1), dim3(kThreads), 0, s, partial, nb, lr, step,
                     beta1, beta2, weight_decay, (float)max_norm, sc, total_norm_out);
  // torch's scalars are Python doubles cast to fp32 inside each op
  const float w1 = (float)(1.0 - beta1);
  const float omb2 = (float)(1.0 - beta2);
  hipLaunchKernelGGL(adamw_update_kernel, dim3((unsigned)nb), dim3(kThreads), 0, s, tab, map, sc,
                     grad_scale, w1, (float)beta2, omb2, (float)eps);
}

}  // namespace ob
