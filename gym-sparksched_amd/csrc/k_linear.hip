// k_linear.hip — the PPO learner's small dense layers (Decima's MLPs: widths <= 64) on hand-written kernels.
//
// The learner (trainers/ppo.py, schedulers/decima.py evaluate_actions) runs ~200 nn.Linear forward / backward GEMMs
// per minibatch over 1e5..3e5 node rows with 5..64 features. Through hipBLASLt each call cost ~70 us of host time
// (per-shape heuristics for row counts that change every minibatch) and its tall-skinny weight gradients ran on a
// handful of workgroups (0.38 s of the learner's 0.71 s of GPU time, profiles/r04/learner_profile.log). Here:
//   * ssim_linear_fwd: y[r][j] = b[j] + sum_i x[r][i] w(i, j) on the matrix cores (16-row tiles per wave, the <= 64 x 64
//     weight staged in LDS in operand order; the forward: w(i, j) = W[j][i]; the input gradient: w(i, j) = W[i][j]);
//   * ssim_linear_wgrad: gW[j][i] = sum_r gy[r][j] x[r][i] and gb[j] = sum_r gy[r][j] on the matrix cores, split over
//     256-row chunks into per-chunk partial sums (LDS-staged row tiles), then reduced in chunk order: deterministic.
// f32 operands, f32 accumulation (v_mfma_f32_16x16x4_f32: no reduced precision); the learner's tolerance tests compare
// with torch (tests/test_linear_gpu). (Round 4's scalar forms read each row's inputs with stride in_dim per lane.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sparksched.h"

namespace {

constexpr int kLinMax = 64;   // widest layer
constexpr int kFwdThreads = 256;
constexpr int kFwdWaves = kFwdThreads / 64;
constexpr int kWgThreads = 256;
constexpr int kWgRows = 256;  // rows per chunk of the weight-gradient pass (one partial per chunk)
constexpr int kWgTile = 64;   // rows per LDS tile within a chunk
constexpr int kXs = 68;       // LDS row stride (floats) of the staged gy tiles: 64 + 4 (16-B aligned, bank-skewed)
constexpr int kXs2 = 80;      // ... of [x | 1] in the weight-gradient pass (in_dim + 1 <= 65 columns)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// y[r][j] = b[j] + sum_i x[r][i] w(i, j) on the matrix cores (v_mfma_f32_16x16x4_f32: f32 operands, f32 accumulate).
// Each wave computes 16-row tiles: Y^T[16 units x 16 rows] = W^T . X^T per 16-unit output tile, the k order of the
// steps being 16g + 4q + r (lane quarter q, word r): lane (row, q) loads its row's inputs 16g + 4q .. + 3 straight
// into registers (the B operand of four steps), the weights are staged once per workgroup in the A operand's order
// (wp: one 16-B LDS word per lane per four steps), and the <= 4 output tiles' accumulator chains are interleaved step
// by step (independent MFMAs back to back instead of each waiting on its predecessor's result).
__global__ __launch_bounds__(kFwdThreads) void k_linear_fwd(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ b, float* __restrict__ y,
                                                           int64_t rows, int in_dim, int out_dim, int transpose_w) {
  __shared__ f32x4 wp[4][4][64];  // [out tile t][k group g][lane]: word r = w(16g + 4(l >> 4) + r, 16t + (l & 15))
  __shared__ __attribute__((aligned(16))) float bs[kLinMax];
  const int tid = threadIdx.x;
  for (int e = tid; e < 4 * 4 * 64 * 4; e += kFwdThreads) {
    const int r = e & 3, l = (e >> 2) & 63, g = (e >> 8) & 3, t = e >> 10;
    const int j = 16 * t + (l & 15), i = 16 * g + 4 * (l >> 4) + r;
    float v = 0.0f;
    if (i < in_dim && j < out_dim) v = transpose_w ? w[(int64_t)j * in_dim + i] : w[(int64_t)i * out_dim + j];
    reinterpret_cast<float*>(wp)[e] = v;
  }
  for (int j = tid; j < kLinMax; j += kFwdThreads) bs[j] = (b != nullptr && j < out_dim) ? b[j] : 0.0f;
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63, row = lane & 15, q = lane >> 4;
  const int KG = (in_dim + 15) / 16, NT = (out_dim + 15) / 16;
  const int64_t tiles = (rows + 15) / 16;
  for (int64_t tile = (int64_t)blockIdx.x * kFwdWaves + wave; tile < tiles; tile += (int64_t)gridDim.x * kFwdWaves) {
    const int64_t r0 = tile * 16;
    const bool valid = r0 + row < rows;
    const float* xr = x + (r0 + row) * in_dim;
    f32x4 xv[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = 16 * g + 4 * q + j;
        xv[g][j] = (g < KG && valid && k < in_dim) ? xr[k] : 0.0f;
      }
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = *reinterpret_cast<const f32x4*>(&bs[16 * t + 4 * q]);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (g >= KG) break;
      f32x4 a[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) a[t] = wp[t][g][lane];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (t < NT) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t][r], xv[g][r], acc[t], 0, 0, 0);
    }
    if (valid) {  // lane holds y[r0 + row][16t + 4q + r]
      float* yr = y + (r0 + row) * out_dim;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j0 = 16 * t + 4 * q;
        if (t >= NT) break;
        if ((out_dim & 3) == 0 && j0 + 3 < out_dim) {
          *reinterpret_cast<f32x4*>(yr + j0) = acc[t];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (j0 + r < out_dim) yr[j0 + r] = acc[t][r];
        }
      }
    }
  }
}

// partial[p][j * (in_dim + 1) + i] over the rows of chunk p (kWgRows): i < in_dim the weight gradient, i == in_dim the
// bias gradient (an input column of ones), on the matrix cores: D[16 j x 16 i] += gY^T[j][4 rows] . X[4 rows][i] per
// step, over the chunk's rows in order (deterministic). The chunk's rows are staged in 64-row LDS tiles (gy and
// [x | 1], coalesced); the <= 4 x 5 output tiles are spread over the 4 waves.
__global__ __launch_bounds__(kWgThreads) void k_linear_wgrad_part(const float* __restrict__ gy,
                                                                 const float* __restrict__ x, float* __restrict__ part,
                                                                 int64_t rows, int in_dim, int out_dim) {
  __shared__ __attribute__((aligned(16))) float gs[kWgTile][kXs];
  __shared__ __attribute__((aligned(16))) float xs2[kWgTile][kXs2];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, li = lane & 15, q = lane >> 4;
  const int w1 = in_dim + 1, n_out = out_dim * w1;
  const int IT = (w1 + 15) / 16, tiles = ((out_dim + 15) / 16) * IT;
  const int64_t r0 = (int64_t)blockIdx.x * kWgRows;
  const int64_t r1 = r0 + kWgRows < rows ? r0 + kWgRows : rows;
  f32x4 acc[5];  // this wave's output tiles wave, wave + 4, ... (<= 5 of the <= 20)
  int tj_j[5], ti_i[5];  // their operand columns: gy column 16 tj + li, [x | 1] column 16 ti + li
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    acc[u] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const int tile = wave + 4 * u, tj = tile / IT, ti = tile - tj * IT;
    tj_j[u] = tile < tiles ? 16 * tj + li : 0;
    ti_i[u] = tile < tiles ? 16 * ti + li : 0;
  }
  for (int64_t t0 = r0; t0 < r1; t0 += kWgTile) {
    const int nt = (int)(r1 - t0 < kWgTile ? r1 - t0 : kWgTile);
    __syncthreads();
    for (int e = tid; e < kWgTile * 64; e += kWgThreads) {
      const int rr = e >> 6, j = e & 63;
      gs[rr][j] = (rr < nt && j < out_dim) ? gy[(t0 + rr) * out_dim + j] : 0.0f;
    }
    for (int e = tid; e < kWgTile * kXs2; e += kWgThreads) {
      const int rr = e / kXs2, i = e - rr * kXs2;
      xs2[rr][i] = rr >= nt ? 0.0f : i < in_dim ? x[(t0 + rr) * in_dim + i] : i == in_dim ? 1.0f : 0.0f;
    }
    __syncthreads();
#pragma unroll 2
    for (int s = 0; s < kWgTile / 4; ++s)  // (the wave's tiles interleaved: independent accumulator chains)
#pragma unroll
      for (int u = 0; u < 5; ++u)
        if (wave + 4 * u < tiles)
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(gs[4 * s + q][tj_j[u]], xs2[4 * s + q][ti_i[u]], acc[u], 0, 0, 0);
  }
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int tile = wave + 4 * u;
    if (tile < tiles) {
      const int tj = tile / IT, ti = tile - tj * IT;
      const int i = 16 * ti + li;
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // lane holds D[4q + r][li] = gW[16 tj + 4q + r][16 ti + li]
        const int j = 16 * tj + 4 * q + r;
        if (j < out_dim && i < w1) part[(int64_t)blockIdx.x * n_out + j * w1 + i] = acc[u][r];
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
  const int64_t tiles = (rows + 15) / 16;  // 16-row tiles, one per wave at a time
  int64_t blocks = (tiles + kFwdWaves - 1) / kFwdWaves;
  if (blocks > 2048) blocks = 2048;  // grid-stride beyond: 8 workgroups per CU
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
