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
    if (dc.on) v = nc_mul(v, drop_hash(dkey, (uint64_t)i) >= dc.thresh ? dc.scale : 0.0f);
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
    if (dc.on) v = nc_mul(v, drop_hash(dkey, (uint64_t)i) >= dc.thresh ? dc.scale : 0.0f);
    if (lens) {
      const int64_t row = i / N, b = row / T;
      if (row - b * T >= lens[b]) v = nc_mul(v, 0.0f);
    }
    out[i] = nc_add(R[i], rscale == 1.0f ? v : nc_mul(rscale, v));
  }
}

}  // namespace

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

}  // namespace ob
