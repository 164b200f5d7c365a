// k_linear.hip — the PPO learner's small dense layers (Decima's MLPs: widths <= 64) on hand-written kernels.
//
// The learner (trainers/ppo.py, schedulers/decima.py evaluate_actions) runs ~200 nn.Linear forward / backward GEMMs
// per minibatch over 1e5..3e5 node rows with 5..64 features. Through hipBLASLt each call cost ~70 us of host time
// (per-shape heuristics for row counts that change every minibatch) and its tall-skinny weight gradients ran on a
// handful of workgroups (0.38 s of the learner's 0.71 s of GPU time, profiles/r04/learner_profile.log). Here:
//   * ssim_linear_fwd: y[r][j] = b[j] + sum_i x[r][i] w(i, j) with the <= 64 x 64 weight staged in LDS, four outputs
//     per thread (the forward: w(i, j) = W[j][i]; the input gradient: w(i, j) = W[i][j], no bias);
//   * ssim_linear_wgrad: gW[j][i] = sum_r gy[r][j] x[r][i] and gb[j] = sum_r gy[r][j], split over 256-row chunks into
//     per-chunk partial sums (LDS-staged row tiles, 4 x 4 output tiles per thread), then
//     reduced in chunk order: deterministic, no atomics.
// f32 in, f32 fma accumulation in index order; the learner's tolerance tests compare with torch (tests/test_linear_gpu).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sparksched.h"

namespace {

constexpr int kLinMax = 64;   // widest layer
constexpr int kFwdThreads = 256;
constexpr int kWgThreads = 256;
constexpr int kWgRows = 256;  // rows per chunk of the weight-gradient pass (one partial per chunk)
constexpr int kWgTile = 64;   // rows per LDS tile within a chunk

// y[r][j..j+3] per thread (4 outputs of one row: the row's inputs are read once per 4 outputs, the weights as one
// 16-B LDS read per input)
__global__ __launch_bounds__(kFwdThreads) void k_linear_fwd(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ b, float* __restrict__ y,
                                                           int64_t rows, int in_dim, int out_dim, int transpose_w) {
  __shared__ float4 m[kLinMax * (kLinMax / 4)];  // m[i][q] = w(i, 4q .. 4q + 3), zero past out_dim
  const int nq = (out_dim + 3) / 4;
  for (int t = threadIdx.x; t < in_dim * nq * 4; t += kFwdThreads) {
    const int i = t / (nq * 4), j = t - i * nq * 4;
    const float v = j >= out_dim ? 0.0f : transpose_w ? w[(int64_t)j * in_dim + i] : w[(int64_t)i * out_dim + j];
    reinterpret_cast<float*>(m)[t] = v;
  }
  __syncthreads();
  const int64_t total = rows * nq;
  for (int64_t g = (int64_t)blockIdx.x * kFwdThreads + threadIdx.x; g < total; g += (int64_t)gridDim.x * kFwdThreads) {
    const int64_t r = g / nq;
    const int q = (int)(g - r * nq), j0 = 4 * q;
    const float* xr = x + r * in_dim;
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
    if (b != nullptr) {
      a0 = b[j0];
      if (j0 + 1 < out_dim) a1 = b[j0 + 1];
      if (j0 + 2 < out_dim) a2 = b[j0 + 2];
      if (j0 + 3 < out_dim) a3 = b[j0 + 3];
    }
    for (int i = 0; i < in_dim; ++i) {
      const float xv = xr[i];
      const float4 mv = m[i * nq + q];
      a0 = __builtin_fmaf(xv, mv.x, a0);
      a1 = __builtin_fmaf(xv, mv.y, a1);
      a2 = __builtin_fmaf(xv, mv.z, a2);
      a3 = __builtin_fmaf(xv, mv.w, a3);
    }
    float* yr = y + r * out_dim + j0;
    yr[0] = a0;
    if (j0 + 1 < out_dim) yr[1] = a1;
    if (j0 + 2 < out_dim) yr[2] = a2;
    if (j0 + 3 < out_dim) yr[3] = a3;
  }
}

// partial[p][j * (in_dim + 1) + i] over the rows of chunk p (kWgRows): i < in_dim the weight gradient, i == in_dim
// the bias gradient (an input column of ones). Each thread owns 4 x 4 output tiles (rows j, columns i) and per row
// reads 4 gradients and 4 inputs (two 16-B LDS reads) for 16 fmas.
__global__ __launch_bounds__(kWgThreads) void k_linear_wgrad_part(const float* __restrict__ gy,
                                                                 const float* __restrict__ x, float* __restrict__ part,
                                                                 int64_t rows, int in_dim, int out_dim) {
  __shared__ float4 gs[kWgTile * (kLinMax / 4)];
  __shared__ float4 xs[kWgTile * ((kLinMax + 4) / 4)];
  const int w1 = in_dim + 1, n_out = out_dim * w1;
  const int tj = (out_dim + 3) / 4, ti = (w1 + 3) / 4, n_tiles = tj * ti;
  const int64_t r0 = (int64_t)blockIdx.x * kWgRows;
  const int64_t r1 = r0 + kWgRows < rows ? r0 + kWgRows : rows;
  // up to 2 tiles per thread (64 x 65 outputs: 16 x 17 = 272 tiles on 256 threads)
  float acc[2][16];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[u][v] = 0.0f;
  for (int64_t t0 = r0; t0 < r1; t0 += kWgTile) {
    const int nt = (int)(r1 - t0 < kWgTile ? r1 - t0 : kWgTile);
    __syncthreads();
    for (int t = threadIdx.x; t < nt * tj * 4; t += kWgThreads) {
      const int rr = t / (tj * 4), j = t - rr * tj * 4;
      reinterpret_cast<float*>(gs)[t] = j < out_dim ? gy[(t0 + rr) * out_dim + j] : 0.0f;
    }
    for (int t = threadIdx.x; t < nt * ti * 4; t += kWgThreads) {
      const int rr = t / (ti * 4), i = t - rr * ti * 4;
      reinterpret_cast<float*>(xs)[t] = i < in_dim ? x[(t0 + rr) * in_dim + i] : i == in_dim ? 1.0f : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tile = threadIdx.x + u * kWgThreads;
      if (tile < n_tiles) {
        const int a = tile / ti, c = tile - a * ti;
        for (int rr = 0; rr < nt; ++rr) {
          const float4 g4 = gs[rr * tj + a];
          const float4 x4 = xs[rr * ti + c];
          const float gv[4] = {g4.x, g4.y, g4.z, g4.w}, xv[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
          for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[u][4 * p + q] = __builtin_fmaf(gv[p], xv[q], acc[u][4 * p + q]);
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int tile = threadIdx.x + u * kWgThreads;
    if (tile < n_tiles) {
      const int a = tile / ti, c = tile - a * ti;
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = 4 * a + p, i = 4 * c + q;
          if (j < out_dim && i < w1) part[(int64_t)blockIdx.x * n_out + j * w1 + i] = acc[u][4 * p + q];
        }
    }
  }
}

// gw / gb from the partials: a block sums 64 outputs, 8 slices of threads each over every 8th chunk (coalesced 256-B
// rows), then the slices are added in slice order (a fixed order: deterministic)
constexpr int kRedOut = 64, kRedSlices = 8;
__global__ __launch_bounds__(kRedOut * kRedSlices) void k_linear_wgrad_reduce(const float* __restrict__ part,
                                                                            float* __restrict__ gw,
                                                                            float* __restrict__ gb, int parts,
                                                                            int in_dim, int out_dim) {
  __shared__ float sl[kRedSlices][kRedOut];
  const int w1 = in_dim + 1, n_out = out_dim * w1;
  const int o = threadIdx.x % kRedOut, s = threadIdx.x / kRedOut;
  const int e = blockIdx.x * kRedOut + o;
  float acc = 0.0f;
  if (e < n_out)
    for (int p = s; p < parts; p += kRedSlices) acc += part[(int64_t)p * n_out + e];
  sl[s][o] = acc;
  __syncthreads();
  if (s != 0 || e >= n_out) return;
  float t = 0.0f;
#pragma unroll
  for (int k = 0; k < kRedSlices; ++k) t += sl[k][o];
  const int j = e / w1, i = e - j * w1;
  if (i < in_dim)
    gw[j * in_dim + i] = t;
  else if (gb != nullptr)
    gb[j] = t;
}

bool dims_ok(int in_dim, int out_dim) {
  return in_dim >= 1 && in_dim <= kLinMax && out_dim >= 1 && out_dim <= kLinMax;
}

}  // namespace

extern "C" {

int ssim_linear_fwd(const float* x, const float* w, const float* b, float* y, int64_t rows, int32_t in_dim,
                    int32_t out_dim, int32_t transpose_w, void* stream) {
  if (!dims_ok(in_dim, out_dim) || rows < 0) return -1;
  if (rows == 0) return 0;
  const int64_t total = rows * ((out_dim + 3) / 4);
  int64_t blocks = (total + kFwdThreads - 1) / kFwdThreads;  // (total: rows x output quads)
  if (blocks > 8192) blocks = 8192;  // grid-stride beyond: 32 workgroups per CU
  hipLaunchKernelGGL(k_linear_fwd, dim3((unsigned)blocks), dim3(kFwdThreads), 0, (hipStream_t)stream, x, w, b, y,
                     rows, (int)in_dim, (int)out_dim, (int)transpose_w);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int32_t ssim_linear_wgrad_parts(int64_t rows) {  // one partial per kWgRows-row chunk
  const int64_t p = (rows + kWgRows - 1) / kWgRows;
  return (int32_t)(p < 1 ? 1 : p);
}

int ssim_linear_wgrad(const float* gy, const float* x, float* gw, float* gb, int64_t rows, int32_t in_dim,
                      int32_t out_dim, float* partial, int32_t parts, void* stream) {
  if (!dims_ok(in_dim, out_dim) || rows < 0 || parts != ssim_linear_wgrad_parts(rows)) return -1;
  hipLaunchKernelGGL(k_linear_wgrad_part, dim3((unsigned)parts), dim3(kWgThreads), 0, (hipStream_t)stream, gy, x,
                     partial, rows, (int)in_dim, (int)out_dim);
  const int n_out = out_dim * (in_dim + 1);
  hipLaunchKernelGGL(k_linear_wgrad_reduce, dim3((unsigned)((n_out + kRedOut - 1) / kRedOut)),
                     dim3(kRedOut * kRedSlices), 0, (hipStream_t)stream, partial, gw, gb, (int)parts, (int)in_dim,
                     (int)out_dim);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
