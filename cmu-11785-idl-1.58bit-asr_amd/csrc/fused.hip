// fused.hip — elementwise backward companions of the fused BitLinear epilogues (tgemm.hip).
//
//   dY = rscale * rowvalid * drop(dOut)
// is the gradient of kEpiResidual's output w.r.t. its GEMM output y (C = R + rscale *
// rowvalid * drop(y)): the backward of conformer.py:39-45 (x + 0.5 * dropout(lin2(.))) and
// :131-138 (x + pad_zero(dropout(out_proj(.)))), regenerating the forward's keep mask from
// the same (seed, counter). HBM-bound: one read, one write per element, dwordx4 when N % 4
// == 0.
#include "ob_drop.h"
#include "ob_fp.h"
#include "ob_launch.h"

namespace ob {

namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void drop_scale_bwd_kernel(
    const float* __restrict__ dout, int64_t rows, int64_t N, float rscale, DropCfg dc,
    const uint64_t* __restrict__ rng, uint64_t rng_off, const int* __restrict__ lens, int T,
    float* __restrict__ dy) {
  const uint32_t dkey = dc.on ? drop_key(rng[0], rng[1] + rng_off) : 0u;
  const int64_t total = rows * N;
  const int64_t nvec = (N % 4 == 0) ? total / 4 : 0;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  auto one = [&](int64_t i, float g) -> float {
    const int64_t row = i / N;
    float v = g;
    if (dc.on) v = nc_mul(v, drop_keep(dkey, (uint64_t)i, dc.thresh) ? dc.scale : 0.0f);
    if (lens) {
      const int64_t b = row / T;
      if (row - b * T >= lens[b]) v = nc_mul(v, 0.0f);
    }
    return rscale == 1.0f ? v : nc_mul(rscale, v);
  };
  for (int64_t q = blockIdx.x * (int64_t)kThreads + threadIdx.x; q < nvec; q += stride) {
    float4 g = reinterpret_cast<const float4*>(dout)[q];
    const int64_t i = 4 * q;
    g.x = one(i, g.x);
    g.y = one(i + 1, g.y);
    g.z = one(i + 2, g.z);
    g.w = one(i + 3, g.w);
    reinterpret_cast<float4*>(dy)[q] = g;
  }
  for (int64_t i = 4 * nvec + blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += stride)
    dy[i] = one(i, dout[i]);
}

__global__ __launch_bounds__(kThreads) void residual_drop_fwd_kernel(
    const float* __restrict__ R, const float* __restrict__ Y, int64_t rows, int64_t N,
    float rscale, DropCfg dc, const uint64_t* __restrict__ rng, uint64_t rng_off,
    const int* __restrict__ lens, int T, float* __restrict__ out) {
  const uint32_t dkey = dc.on ? drop_key(rng[0], rng[1] + rng_off) : 0u;
  const int64_t total = rows * N;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += stride) {
    float v = Y[i];
    if (dc.on) v = nc_mul(v, drop_keep(dkey, (uint64_t)i, dc.thresh) ? dc.scale : 0.0f);
    if (lens) {
      const int64_t row = i / N, b = row / T;
      if (row - b * T >= lens[b]) v = nc_mul(v, 0.0f);
    }
    out[i] = nc_add(R[i], rscale == 1.0f ? v : nc_mul(rscale, v));
  }
}


// ---------------------------------------------------------------------------------------
// Conv2dSubsampling's `conv -> +bias -> ReLU` tails (conformer.py:183-186) on NCHW planes:
// forward y = max(x + b[c], 0) in place; backward g' = g * (y > 0) and db[c] = sum over
// the batch's planes of g' (per-plane partials, then a fixed-order sum over b). One pass
// each instead of torch's add + clamp / threshold_backward + sum.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void bias_relu_fwd_kernel(float* __restrict__ y,
                                                                 const float* __restrict__ bias,
                                                                 int64_t planes, int C,
                                                                 int64_t hw) {
  const int64_t total = planes * hw;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  if (hw % 4 == 0) {
    float4* y4 = reinterpret_cast<float4*>(y);
    const int64_t hw4 = hw / 4;
    for (int64_t q = blockIdx.x * (int64_t)kThreads + threadIdx.x; q < total / 4; q += stride) {
      const float b = bias[(q / hw4) % C];
      float4 v = y4[q];
      v.x = fmaxf(v.x + b, 0.0f);
      v.y = fmaxf(v.y + b, 0.0f);
      v.z = fmaxf(v.z + b, 0.0f);
      v.w = fmaxf(v.w + b, 0.0f);
      y4[q] = v;
    }
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += stride)
    y[i] = fmaxf(y[i] + bias[(i / hw) % C], 0.0f);
}

// block = one (b, c) plane: g' = g * (y > 0) written to gout, plane sum -> part[plane].
__global__ __launch_bounds__(kThreads) void relu_bias_bwd_kernel(
    const float* __restrict__ g, const float* __restrict__ y, int64_t hw,
    float* __restrict__ gout, float* __restrict__ part) {
  __shared__ float red[kThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * hw;
  float acc = 0.0f;
  for (int64_t i = threadIdx.x; i < hw; i += kThreads) {
    const float v = y[base + i] > 0.0f ? g[base + i] : 0.0f;
    gout[base + i] = v;
    acc += v;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// out[i] = sum over slices of part[slice * n + i] (fixed order): one wave per output, lanes
// take slices lane, lane + 64, ..., then a fixed shuffle tree (a thread per output summing
// 128 slices serially was latency-bound: 30 us).
__global__ __launch_bounds__(64) void slice_sum_kernel(const float* __restrict__ part,
                                                       int slices, int n,
                                                       float* __restrict__ out) {
  const int i = blockIdx.x;
  float acc = 0.0f;
  for (int sl = threadIdx.x; sl < slices; sl += 64) acc += part[(int64_t)sl * n + i];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (threadIdx.x == 0) out[i] = acc;
}

// Column sums of a [rows][N] matrix (the bias gradient of a GEMM on rows): block = (row
// slice, 64-column group); lane = column, waves split the slice's rows; fixed order.
constexpr int kColSlices = 128;

__global__ __launch_bounds__(kThreads) void colsum_part_kernel(const float* __restrict__ x,
                                                               int64_t rows, int n,
                                                               float* __restrict__ part) {
  __shared__ float red[kThreads / 64][64];
  const int col = blockIdx.y * 64 + (threadIdx.x & 63);
  const int w = threadIdx.x >> 6;
  const int64_t r0 = rows * blockIdx.x / kColSlices, r1 = rows * (blockIdx.x + 1) / kColSlices;
  float acc = 0.0f;
  if (col < n) {
#pragma unroll 4
    for (int64_t r = r0 + w; r < r1; r += kThreads / 64) acc += x[r * n + col];
  }
  red[w][threadIdx.x & 63] = acc;
  __syncthreads();
  if (w == 0 && col < n)
    part[(int64_t)blockIdx.x * n + col] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}

// Zero n 32-bit words. Used instead of hipMemsetAsync, which, captured into a HIP graph
// on ROCm 7.2, leaves garbage in buffers below ~4 MB on every replay after the first
// (tools/memset_graph_repro.py).
__global__ __launch_bounds__(kThreads) void zero_words_kernel(uint32_t* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
    p[i] = 0u;
}

}  // namespace

void launch_zero_words(void* p, int64_t n_words, hipStream_t s) {
  if (n_words <= 0) return;
  int64_t blocks = ceil_div(n_words, kThreads);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(zero_words_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s,
                     static_cast<uint32_t*>(p), n_words);
}

void launch_drop_scale_bwd(const float* dout, int64_t rows, int64_t N, float rscale,
                           float p_drop, const uint64_t* rng, uint64_t rng_off, const int* lens,
                           int T, float* dy, hipStream_t s) {
  const int64_t total = rows * N;
  if (total == 0) return;
  int64_t blocks = ceil_div((N % 4 == 0) ? total / 4 : total, kThreads);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(drop_scale_bwd_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, dout,
                     rows, N, rscale, make_drop(p_drop), rng, rng_off, lens, T > 0 ? T : 1, dy);
}

void launch_residual_drop_fwd(const float* R, const float* Y, int64_t rows, int64_t N,
                              float rscale, float p_drop, const uint64_t* rng, uint64_t rng_off,
                              const int* lens, int T, float* out, hipStream_t s) {
  const int64_t total = rows * N;
  if (total == 0) return;
  int64_t blocks = ceil_div(total, kThreads);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(residual_drop_fwd_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, R, Y,
                     rows, N, rscale, make_drop(p_drop), rng, rng_off, lens, T > 0 ? T : 1, out);
}

void launch_bias_relu_fwd(float* y, const float* bias, int64_t B, int64_t C, int64_t hw,
                          hipStream_t s) {
  const int64_t total = B * C * hw;
  if (total == 0) return;
  int64_t blocks = ceil_div(hw % 4 == 0 ? total / 4 : total, kThreads);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(bias_relu_fwd_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, y, bias,
                     B * C, (int)C, hw);
}

size_t relu_bias_bwd_workspace(int64_t B, int64_t C) { return sizeof(float) * (size_t)(B * C) + 256; }

void launch_relu_bias_bwd(const float* g, const float* y, int64_t B, int64_t C, int64_t hw,
                          float* gout, float* dbias, void* ws, hipStream_t s) {
  if (B * C == 0) return;
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(relu_bias_bwd_kernel, dim3((unsigned)(B * C)), dim3(kThreads), 0, s, g, y,
                     hw, gout, part);
  if (dbias)
    hipLaunchKernelGGL(slice_sum_kernel, dim3((unsigned)C), dim3(64), 0, s, (const float*)part,
                       (int)B, (int)C, dbias);
}

size_t colsum_workspace(int64_t N) { return sizeof(float) * (size_t)(kColSlices * N) + 256; }

void launch_colsum(const float* x, int64_t rows, int64_t N, float* out, void* ws, hipStream_t s) {
  if (N == 0) return;
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(colsum_part_kernel, dim3(kColSlices, (unsigned)ceil_div(N, 64)),
                     dim3(kThreads), 0, s, x, rows, (int)N, part);
  hipLaunchKernelGGL(slice_sum_kernel, dim3((unsigned)N), dim3(64), 0, s, (const float*)part,
                     kColSlices, (int)N, out);
}

}  // namespace ob
