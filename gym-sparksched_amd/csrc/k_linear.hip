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

// One layer of a weight-gradient pass: gw[j][i] = sum_r gy[r][j] x[r][i], gb[j] = sum_r gy[r][j]. x is a row-major
// [rows, in_dim] matrix, or (base != nullptr) the exec-score grid's generated input: row r = (decision r / grid_n,
// action r % grid_n) holds base[r / grid_n][0 .. in_dim - 2] and the action fraction (r % grid_n) / grid_n.
struct WgLayer {
  const float* gy;
  const float* x;
  const float* base;
  float* part;  // parts x out_dim x (in_dim + 1)
  float* gw;
  float* gb;
  int in_dim, out_dim, grid_n, pad_;
};
struct WgLayers {
  WgLayer l[3];
};

__device__ __forceinline__ float wg_x(const WgLayer& L, int64_t r, int i) {
  if (L.base == nullptr) return L.x[r * L.in_dim + i];
  const int64_t k = r / L.grid_n;
  const int a = (int)(r - k * L.grid_n);
  return i < L.in_dim - 1 ? L.base[k * (L.in_dim - 1) + i] : (float)a / (float)L.grid_n;
}

// partial[p][j * (in_dim + 1) + i] over the rows of chunk p (kWgRows) of layer blockIdx.y: i < in_dim the weight
// gradient, i == in_dim the bias gradient (an input column of ones). Each thread owns 4 x 4 output tiles (rows j,
// columns i) and per row reads 4 gradients and 4 inputs (two 16-B LDS reads) for 16 fmas.
__global__ __launch_bounds__(kWgThreads) void k_linear_wgrad_part(WgLayers layers, int64_t rows) {
  __shared__ float4 gs[kWgTile * (kLinMax / 4)];
  __shared__ float4 xs[kWgTile * ((kLinMax + 4) / 4)];
  const WgLayer& L = layers.l[blockIdx.y];
  const int in_dim = L.in_dim, out_dim = L.out_dim;
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
      reinterpret_cast<float*>(gs)[t] = j < out_dim ? L.gy[(t0 + rr) * out_dim + j] : 0.0f;
    }
    for (int t = threadIdx.x; t < nt * ti * 4; t += kWgThreads) {
      const int rr = t / (ti * 4), i = t - rr * ti * 4;
      reinterpret_cast<float*>(xs)[t] = i < in_dim ? wg_x(L, t0 + rr, i) : i == in_dim ? 1.0f : 0.0f;
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
          if (j < out_dim && i < w1) L.part[(int64_t)blockIdx.x * n_out + j * w1 + i] = acc[u][4 * p + q];
        }
    }
  }
}

// gw / gb from the partials: a block sums 64 outputs, 8 slices of threads each over every 8th chunk (coalesced 256-B
// rows), then the slices are added in slice order (a fixed order: deterministic)
constexpr int kRedOut = 64, kRedSlices = 8;
__global__ __launch_bounds__(kRedOut * kRedSlices) void k_linear_wgrad_reduce(WgLayers layers, int parts) {
  __shared__ float sl[kRedSlices][kRedOut];
  const WgLayer& L = layers.l[blockIdx.y];
  const int w1 = L.in_dim + 1, n_out = L.out_dim * w1;
  if ((int)blockIdx.x * kRedOut >= n_out) return;  // (grid sized for the widest layer; uniform per block)
  const int o = threadIdx.x % kRedOut, s = threadIdx.x / kRedOut;
  const int e = blockIdx.x * kRedOut + o;
  float acc = 0.0f;
  if (e < n_out)
    for (int p = s; p < parts; p += kRedSlices) acc += L.part[(int64_t)p * n_out + e];
  sl[s][o] = acc;
  __syncthreads();
  if (s != 0 || e >= n_out) return;
  float t = 0.0f;
#pragma unroll
  for (int k = 0; k < kRedSlices; ++k) t += sl[k][o];
  const int j = e / w1, i = e - j * w1;
  if (i < L.in_dim)
    L.gw[j * L.in_dim + i] = t;
  else if (L.gb != nullptr)
    L.gb[j] = t;
}

// both passes of a weight-gradient computation over n layers sharing the row count (and one partial per chunk)
int wgrad_launch(const WgLayers& layers, int n, int64_t rows, int parts, hipStream_t stream) {
  int widest = 0;
  for (int k = 0; k < n; ++k) {
    const int o = layers.l[k].out_dim * (layers.l[k].in_dim + 1);
    widest = o > widest ? o : widest;
  }
  hipLaunchKernelGGL(k_linear_wgrad_part, dim3((unsigned)parts, (unsigned)n), dim3(kWgThreads), 0, stream, layers,
                     rows);
  hipLaunchKernelGGL(k_linear_wgrad_reduce, dim3((unsigned)((widest + kRedOut - 1) / kRedOut), (unsigned)n),
                     dim3(kRedOut * kRedSlices), 0, stream, layers, parts);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

bool dims_ok(int in_dim, int out_dim) {
  return in_dim >= 1 && in_dim <= kLinMax && out_dim >= 1 && out_dim <= kLinMax;
}

// ---- fused three-layer MLPs: Linear(d0, D1), act, Linear(D1, D2), act, Linear(D2, D3) (make_mlp with two hidden
// layers, schedulers/decima/utils.py:51-70). One thread per row runs the whole chain in registers, the weights as
// wave-uniform (scalar) loads; the forward keeps the two post-activation hidden rows for the backward, which
// computes the pre-activation gradients of both hidden layers (and the input gradient) in one pass, then the three
// weight gradients in one pair of launches. 1 + 3 launches per MLP instead of 5 + 11 for the per-layer form.
enum { kActLeaky = 0, kActTanh = 1 };
constexpr int kMlpThreads = 256;

struct Mlp3Args {
  const float* x;     // [rows, d0], or nullptr: the exec-score grid (base [rows / grid_n, d0 - 1] + action fraction)
  const float* base;
  const float *w0, *b0, *w1, *b1, *w2, *b2;  // nn.Linear layouts: w0 [D1][d0], w1 [D2][D1], w2 [D3][D2]
  float *h1, *h2, *y;                        // forward: post-activation hidden rows (nullptr: not kept), output
  const float* gy;                           // backward: [rows, D3]
  float *g1, *g2, *gx;                       // backward: pre-activation gradients, input gradient (nullptr: none)
  int64_t rows;
  int d0, grid_n;
  float slope;
};

// tanh to a few ulp: odd Taylor polynomial below |v| = 1/8 (next term < 1e-12 relative), (1 - e) / (1 + e) with
// e = exp(-2|v|) above (at most ~2 bits lost to the subtraction). ocml's tanhf, inlined 64 times into the unrolled
// row chain, made the compiler spill ~15 KB per lane.
__device__ __forceinline__ float mlp_tanh(float v) {
  const float ax = __builtin_fabsf(v);
  const float x2 = v * v;
  const float p = v * __builtin_fmaf(
                          x2,
                          __builtin_fmaf(x2, __builtin_fmaf(x2, __builtin_fmaf(x2, 62.0f / 2835.0f, -17.0f / 315.0f),
                                                            2.0f / 15.0f),
                                         -1.0f / 3.0f),
                          1.0f) ;
  const float e = __expf(-2.0f * ax);
  const float q = __builtin_copysignf(__fdividef(1.0f - e, 1.0f + e), v);
  return ax < 0.125f ? p : q;
}

template <int ACT>
__device__ __forceinline__ float mlp_act(float v, float slope) {
  if constexpr (ACT == kActTanh)
    return mlp_tanh(v);
  else
    return v > 0.0f ? v : v * slope;
}
// the derivative from the activation's OUTPUT (what torch's in-place LeakyReLU and Tanh backward use)
template <int ACT>
__device__ __forceinline__ float mlp_act_d(float h, float slope) {
  if constexpr (ACT == kActTanh)
    return 1.0f - h * h;
  else
    return h > 0.0f ? 1.0f : slope;
}

template <int N>
__device__ __forceinline__ void mlp_store(float* dst, const float (&v)[N]) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int q = 0; q < N / 4; ++q)
      reinterpret_cast<float4*>(dst)[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  } else {
#pragma unroll
    for (int q = 0; q < N; ++q) dst[q] = v[q];
  }
}
template <int N>
__device__ __forceinline__ void mlp_load(const float* src, float (&v)[N]) {
  if constexpr (N % 4 == 0) {
#pragma unroll
    for (int q = 0; q < N / 4; ++q) {
      const float4 f = reinterpret_cast<const float4*>(src)[q];
      v[4 * q] = f.x;
      v[4 * q + 1] = f.y;
      v[4 * q + 2] = f.z;
      v[4 * q + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = src[q];
  }
}

// the row's input value i < d0 (row-major x, or the exec grid's base row + action fraction)
__device__ __forceinline__ float mlp_x(const Mlp3Args& a, int64_t r, int i) {
  if (a.x != nullptr) return a.x[r * a.d0 + i];
  const int64_t k = r / a.grid_n;
  const int an = (int)(r - k * a.grid_n);
  return i < a.d0 - 1 ? a.base[k * (a.d0 - 1) + i] : (float)an / (float)a.grid_n;
}

// LDS copies of the three layers (staged once per block; every read below is wave-uniform: a broadcast):
//   forward: W0t[i][j] = w0[j][i] (rows i >= d0 zero), W1t[i][j] = w1[j][i], W2 row-major, biases;
//   backward: W2 and W1 row-major, W0t as in the forward (row k: the weights of input column k).
template <int D0P, int D1, int D2, int D3>
struct MlpLds {
  float w0[D0P * D1];
  float w1[D1 * D2];
  float w2[D3 * D2];
  float b0[D1], b1[D2], b2[D3];
};

template <int D0P, int D1, int D2, int D3>
__device__ __forceinline__ void mlp_stage(const Mlp3Args& a, MlpLds<D0P, D1, D2, D3>& m, bool fwd) {
  for (int t = threadIdx.x; t < D0P * D1; t += kMlpThreads) {  // W0t[i][j] = w0[j][i]
    const int i = t / D1, j = t - i * D1;
    m.w0[t] = i < a.d0 ? a.w0[j * a.d0 + i] : 0.0f;
  }
  for (int t = threadIdx.x; t < D1 * D2; t += kMlpThreads) {
    if (fwd) {  // W1t[i][j] = w1[j][i]
      const int i = t / D2, j = t - i * D2;
      m.w1[t] = a.w1[j * D1 + i];
    } else {
      m.w1[t] = a.w1[t];
    }
  }
  for (int t = threadIdx.x; t < D3 * D2; t += kMlpThreads) m.w2[t] = a.w2[t];
  if (fwd) {
    for (int t = threadIdx.x; t < D1; t += kMlpThreads) m.b0[t] = a.b0[t];
    for (int t = threadIdx.x; t < D2; t += kMlpThreads) m.b1[t] = a.b1[t];
    for (int t = threadIdx.x; t < D3; t += kMlpThreads) m.b2[t] = a.b2[t];
  }
  __syncthreads();
}

// An opaque zero added to every LDS weight row address: the weights are loop-invariant, and without it the compiler
// hoists (or front-loads) every weight read of the unrolled chain at once (thousands of registers: spills).
__device__ __forceinline__ int mlp_zero() {
  int z = 0;
  asm volatile("" : "+v"(z));
  return z;
}

// acc[0 .. N) += s * row[0 .. N) (row: LDS, 16-B aligned, N % 4 == 0)
template <int N>
__device__ __forceinline__ void mlp_axpy(float (&acc)[N], float s, const float* row) {
#pragma unroll
  for (int q = 0; q < N / 4; ++q) {
    const float4 w = reinterpret_cast<const float4*>(row)[q];
    acc[4 * q] = __builtin_fmaf(s, w.x, acc[4 * q]);
    acc[4 * q + 1] = __builtin_fmaf(s, w.y, acc[4 * q + 1]);
    acc[4 * q + 2] = __builtin_fmaf(s, w.z, acc[4 * q + 2]);
    acc[4 * q + 3] = __builtin_fmaf(s, w.w, acc[4 * q + 3]);
  }
  __builtin_amdgcn_sched_barrier(0);  // one weight row in flight at a time (other waves hide the LDS latency)
}

template <int D0P, int D1, int D2, int D3, int ACT>
__global__ __launch_bounds__(kMlpThreads) void k_mlp3_fwd(Mlp3Args a) {
  __shared__ __attribute__((aligned(16))) MlpLds<D0P, D1, D2, D3> m;
  mlp_stage<D0P, D1, D2, D3>(a, m, true);
  for (int64_t r = (int64_t)blockIdx.x * kMlpThreads + threadIdx.x; r < a.rows;
       r += (int64_t)gridDim.x * kMlpThreads) {
    const int z = mlp_zero();
    const float *b0 = m.b0 + z, *b1 = m.b1 + z, *b2 = m.b2 + z;
    float h1[D1];
#pragma unroll
    for (int j = 0; j < D1; ++j) h1[j] = b0[j];
#pragma unroll
    for (int i = 0; i < D0P; ++i)
      if (i < a.d0) mlp_axpy<D1>(h1, mlp_x(a, r, i), m.w0 + i * D1 + mlp_zero());
#pragma unroll
    for (int j = 0; j < D1; ++j) h1[j] = mlp_act<ACT>(h1[j], a.slope);
    if (a.h1 != nullptr) mlp_store(a.h1 + r * D1, h1);  // (inference: not kept)
    float h2[D2];
#pragma unroll
    for (int j = 0; j < D2; ++j) h2[j] = b1[j];
#pragma unroll
    for (int i = 0; i < D1; ++i) mlp_axpy<D2>(h2, h1[i], m.w1 + i * D2 + mlp_zero());
#pragma unroll
    for (int j = 0; j < D2; ++j) h2[j] = mlp_act<ACT>(h2[j], a.slope);
    if (a.h2 != nullptr) mlp_store(a.h2 + r * D2, h2);  // (inference: not kept)
    float y[D3];
#pragma unroll
    for (int o = 0; o < D3; ++o) {
      float s = b2[o];
#pragma unroll
      for (int q = 0; q < D2 / 4; ++q) {
        const float4 w = reinterpret_cast<const float4*>(m.w2 + o * D2 + mlp_zero())[q];
        s = __builtin_fmaf(h2[4 * q], w.x, s);
        s = __builtin_fmaf(h2[4 * q + 1], w.y, s);
        s = __builtin_fmaf(h2[4 * q + 2], w.z, s);
        s = __builtin_fmaf(h2[4 * q + 3], w.w, s);
      }
      y[o] = s;
    }
    mlp_store(a.y + r * D3, y);
  }
}

template <int D0P, int D1, int D2, int D3, int ACT>
__global__ __launch_bounds__(kMlpThreads) void k_mlp3_bwd_data(Mlp3Args a) {
  __shared__ __attribute__((aligned(16))) MlpLds<D0P, D1, D2, D3> m;
  mlp_stage<D0P, D1, D2, D3>(a, m, false);
  for (int64_t r = (int64_t)blockIdx.x * kMlpThreads + threadIdx.x; r < a.rows;
       r += (int64_t)gridDim.x * kMlpThreads) {
    float g2[D2];
#pragma unroll
    for (int j = 0; j < D2; ++j) g2[j] = 0.0f;
    {
      float gy[D3];
      mlp_load(a.gy + r * D3, gy);
#pragma unroll
      for (int o = 0; o < D3; ++o) mlp_axpy<D2>(g2, gy[o], m.w2 + o * D2 + mlp_zero());
    }
    {
      float h2[D2];
      mlp_load(a.h2 + r * D2, h2);
#pragma unroll
      for (int j = 0; j < D2; ++j) g2[j] *= mlp_act_d<ACT>(h2[j], a.slope);
    }
    mlp_store(a.g2 + r * D2, g2);
    float g1[D1];
#pragma unroll
    for (int i = 0; i < D1; ++i) g1[i] = 0.0f;
#pragma unroll
    for (int j = 0; j < D2; ++j) mlp_axpy<D1>(g1, g2[j], m.w1 + j * D1 + mlp_zero());
    {
      float h1[D1];
      mlp_load(a.h1 + r * D1, h1);
#pragma unroll
      for (int i = 0; i < D1; ++i) g1[i] *= mlp_act_d<ACT>(h1[i], a.slope);
    }
    mlp_store(a.g1 + r * D1, g1);
    if (a.gx != nullptr) {  // gx[k] = sum_i g1[i] w0[i][k]: one dot product per input column (W0t row k)
      float* gxr = a.gx + r * a.d0;
#pragma unroll 1
      for (int k = 0; k < a.d0; ++k) {
        const float* wk = m.w0 + k * D1 + mlp_zero();
        float s = 0.0f;
#pragma unroll
        for (int q = 0; q < D1 / 4; ++q) {
          const float4 w = reinterpret_cast<const float4*>(wk)[q];
          s = __builtin_fmaf(g1[4 * q], w.x, s);
          s = __builtin_fmaf(g1[4 * q + 1], w.y, s);
          s = __builtin_fmaf(g1[4 * q + 2], w.z, s);
          s = __builtin_fmaf(g1[4 * q + 3], w.w, s);
        }
        gxr[k] = s;
      }
    }
  }
}

// the exec-score grid's input gradient: gbase[k][c] = sum_i (sum_a g1[k * grid_n + a][i]) w0[i][c], c < d0 - 1 (the
// action column is generated, not an input). A block of 256 threads = 4 decisions x 64 hidden units.
template <int D1>
__global__ __launch_bounds__(256) void k_mlp3_grid_gx(const float* __restrict__ g1, const float* __restrict__ w0,
                                                     float* __restrict__ gbase, int64_t decisions, int grid_n,
                                                     int d0) {
  __shared__ float gs[4][D1];
  const int slot = threadIdx.x / 64, u = threadIdx.x % 64;
  const int64_t k = (int64_t)blockIdx.x * 4 + slot;
  if (k < decisions && u < D1) {
    float s = 0.0f;
    const float* gr = g1 + k * grid_n * D1 + u;
    for (int an = 0; an < grid_n; ++an) s += gr[(int64_t)an * D1];
    gs[slot][u] = s;
  }
  __syncthreads();
  if (k >= decisions || u >= d0 - 1) return;
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < D1; ++i) s = __builtin_fmaf(gs[slot][i], w0[i * d0 + u], s);
  gbase[k * (d0 - 1) + u] = s;
}

int mlp_blocks(int64_t rows) {
  int64_t b = (rows + kMlpThreads - 1) / kMlpThreads;
  return (int)(b > 16384 ? 16384 : b < 1 ? 1 : b);
}

template <int D1, int D2, int D3, int ACT>
int mlp3_dispatch(bool fwd, const Mlp3Args& a, hipStream_t s) {
  const dim3 g((unsigned)mlp_blocks(a.rows)), b(kMlpThreads);
  const int d0p = (a.d0 + 7) / 8 * 8;
#define SSIM_MLP3_CASE(P)                                                   \
  case P:                                                                   \
    if (fwd)                                                                \
      hipLaunchKernelGGL((k_mlp3_fwd<P, D1, D2, D3, ACT>), g, b, 0, s, a);  \
    else                                                                    \
      hipLaunchKernelGGL((k_mlp3_bwd_data<P, D1, D2, D3, ACT>), g, b, 0, s, a); \
    break;
  switch (d0p) {
    SSIM_MLP3_CASE(8)
    SSIM_MLP3_CASE(16)
    SSIM_MLP3_CASE(24)
    SSIM_MLP3_CASE(32)
    SSIM_MLP3_CASE(40)
    SSIM_MLP3_CASE(48)
    SSIM_MLP3_CASE(56)
    SSIM_MLP3_CASE(64)
    default:
      return -1;
  }
#undef SSIM_MLP3_CASE
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// the shapes the Decima MLPs take (decima_tpch.yaml): GNN (hid [32, 16], embed 16, LeakyReLU) and policy (hid [64, 64],
// one score, Tanh); any other MLP takes the per-layer kernels
int mlp3_kind(int d1, int d2, int d3, int act) {
  if (d1 == 32 && d2 == 16 && d3 == 16 && act == kActLeaky) return 0;
  if (d1 == 64 && d2 == 64 && d3 == 1 && act == kActTanh) return 1;
  return -1;
}
int mlp3_run(bool fwd, int kind, const Mlp3Args& a, hipStream_t s) {
  return kind == 0 ? mlp3_dispatch<32, 16, 16, kActLeaky>(fwd, a, s) : mlp3_dispatch<64, 64, 1, kActTanh>(fwd, a, s);
}

// ---- discounted returns (trainers/utils/returns_calculator.py:37-52): R_k = r_k + decay_k R_{k+1}, backward over each
// trajectory row. One thread per row runs the serial recursion with the same two roundings as the reference's
// per-column `r[:, k] + decay[:, k] * R` (a product, then a sum: no fused multiply-add), so the returns are
// bit-identical to it; the loads of a row run ahead of the dependent chain (they do not depend on R). Replaces 3
// launches per trajectory step (~25k per decima_tpch.yaml iteration).
template <class T>
__device__ __forceinline__ T ret_step(T r, T d, T R);
template <>
__device__ __forceinline__ double ret_step<double>(double r, double d, double R) {
#pragma clang fp contract(off)
  return r + d * R;  // (contraction off: __dmul_rn / __dadd_rn alone still fused into an fma)
}
template <>
__device__ __forceinline__ float ret_step<float>(float r, float d, float R) {
#pragma clang fp contract(off)
  return r + d * R;
}

template <class T>
__global__ __launch_bounds__(64) void k_discounted_returns(const T* __restrict__ r, const T* __restrict__ decay,
                                                          T* __restrict__ out, int64_t rows, int64_t cols) {
  const int64_t row = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (row >= rows) return;
  const T* rr = r + row * cols;
  const T* dr = decay + row * cols;
  T* o = out + row * cols;
  T R = T(0);
  int64_t k = cols - 1;
  for (; k >= 7; k -= 8) {  // 8 columns of loads in flight ahead of the chain
    T rv[8], dv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      rv[u] = rr[k - u];
      dv[u] = dr[k - u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      R = ret_step<T>(rv[u], dv[u], R);
      o[k - u] = R;
    }
  }
  for (; k >= 0; --k) {
    R = ret_step<T>(rr[k], dr[k], R);
    o[k] = R;
  }
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
  WgLayers L{};
  L.l[0] = WgLayer{gy, x, nullptr, partial, gw, gb, (int)in_dim, (int)out_dim, 0, 0};
  return wgrad_launch(L, 1, rows, parts, (hipStream_t)stream);
}


int32_t ssim_mlp3_supported(int32_t d0, int32_t d1, int32_t d2, int32_t d3, int32_t act) {
  return d0 >= 1 && d0 <= kLinMax && mlp3_kind(d1, d2, d3, act) >= 0 ? 1 : 0;
}

int ssim_mlp3_fwd(const float* x, const float* base, int32_t grid_n, const float* w0, const float* b0,
                  const float* w1, const float* b1, const float* w2, const float* b2, float* h1, float* h2, float* y,
                  int64_t rows, int32_t d0, int32_t d1, int32_t d2, int32_t d3, int32_t act, float slope,
                  void* stream) {
  if (!ssim_mlp3_supported(d0, d1, d2, d3, act) || rows < 0) return -1;
  if (rows == 0) return 0;  // (an empty tensor's data pointer may be NULL)
  if ((x == nullptr) == (base == nullptr) || (base != nullptr && (grid_n < 1 || d0 < 2 || rows % grid_n != 0)))
    return -1;
  Mlp3Args a{};
  a.x = x;
  a.base = base;
  a.w0 = w0; a.b0 = b0; a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2;
  a.h1 = h1; a.h2 = h2; a.y = y;
  a.rows = rows;
  a.d0 = d0;
  a.grid_n = base != nullptr ? grid_n : 1;
  a.slope = slope;
  return mlp3_run(true, mlp3_kind(d1, d2, d3, act), a, (hipStream_t)stream);
}

int32_t ssim_mlp3_parts(int64_t rows) { return ssim_linear_wgrad_parts(rows); }

int ssim_mlp3_bwd(const float* gy, const float* x, const float* base, int32_t grid_n, const float* w0,
                  const float* w1, const float* w2, const float* h1, const float* h2, float* g1, float* g2, float* gx,
                  float* gw0, float* gb0, float* gw1, float* gb1, float* gw2, float* gb2, int64_t rows, int32_t d0,
                  int32_t d1, int32_t d2, int32_t d3, int32_t act, float slope, float* partial, int32_t parts,
                  void* stream) {
  if (!ssim_mlp3_supported(d0, d1, d2, d3, act) || rows < 0 || parts != ssim_mlp3_parts(rows)) return -1;
  if (rows == 0) {  // nothing flows back: zero weight / bias gradients (the input gradient is empty)
    hipStream_t s = (hipStream_t)stream;
    float* gz[6] = {gw0, gb0, gw1, gb1, gw2, gb2};
    const int64_t nz[6] = {(int64_t)d1 * d0, d1, (int64_t)d2 * d1, d2, (int64_t)d3 * d2, d3};
    for (int k = 0; k < 6; ++k)
      if (gz[k] != nullptr && hipMemsetAsync(gz[k], 0, nz[k] * sizeof(float), s) != hipSuccess) return -2;
    return 0;
  }
  if ((x == nullptr) == (base == nullptr) || (base != nullptr && (grid_n < 1 || d0 < 2 || rows % grid_n != 0)))
    return -1;
  hipStream_t s = (hipStream_t)stream;
  Mlp3Args a{};
  a.x = x;
  a.base = base;
  a.w0 = w0; a.w1 = w1; a.w2 = w2;
  a.h1 = const_cast<float*>(h1); a.h2 = const_cast<float*>(h2);
  a.gy = gy;
  a.g1 = g1; a.g2 = g2;
  a.gx = base != nullptr ? nullptr : gx;
  a.rows = rows;
  a.d0 = d0;
  a.grid_n = base != nullptr ? grid_n : 1;
  a.slope = slope;
  const int rc = mlp3_run(false, mlp3_kind(d1, d2, d3, act), a, s);
  if (rc != 0) return rc;
  if (base != nullptr && gx != nullptr) {  // the grid's input gradient: per decision, summed over its actions
    const int64_t dec = rows / grid_n;
    const unsigned blocks = (unsigned)((dec + 3) / 4);
    if (d1 == 32)
      hipLaunchKernelGGL(k_mlp3_grid_gx<32>, dim3(blocks), dim3(256), 0, s, g1, w0, gx, dec, (int)grid_n, (int)d0);
    else
      hipLaunchKernelGGL(k_mlp3_grid_gx<64>, dim3(blocks), dim3(256), 0, s, g1, w0, gx, dec, (int)grid_n, (int)d0);
  }
  if (partial == nullptr) return -1;
  // partials: layer 2, layer 1, layer 0 regions back to back
  const int64_t n2 = (int64_t)parts * d3 * (d2 + 1), n1 = (int64_t)parts * d2 * (d1 + 1);
  WgLayers L{};
  L.l[0] = WgLayer{gy, h2, nullptr, partial, gw2, gb2, (int)d2, (int)d3, 0, 0};
  L.l[1] = WgLayer{g2, h1, nullptr, partial + n2, gw1, gb1, (int)d1, (int)d2, 0, 0};
  L.l[2] = WgLayer{g1, x, base, partial + n2 + n1, gw0, gb0, (int)d0, (int)d1, base != nullptr ? (int)grid_n : 0, 0};
  return wgrad_launch(L, 3, rows, parts, s);
}

int64_t ssim_mlp3_partial_floats(int64_t rows, int32_t d0, int32_t d1, int32_t d2, int32_t d3) {
  return (int64_t)ssim_mlp3_parts(rows) * ((int64_t)d3 * (d2 + 1) + (int64_t)d2 * (d1 + 1) + (int64_t)d1 * (d0 + 1));
}


int ssim_discounted_returns(const void* r, const void* decay, void* out, int64_t rows, int64_t cols, int32_t f64,
                            void* stream) {
  if (rows < 0 || cols < 0) return -1;
  if (rows == 0 || cols == 0) return 0;
  const dim3 g((unsigned)((rows + 63) / 64)), b(64);
  if (f64)
    hipLaunchKernelGGL(k_discounted_returns<double>, g, b, 0, (hipStream_t)stream, (const double*)r,
                       (const double*)decay, (double*)out, rows, cols);
  else
    hipLaunchKernelGGL(k_discounted_returns<float>, g, b, 0, (hipStream_t)stream, (const float*)r,
                       (const float*)decay, (float*)out, rows, cols);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
