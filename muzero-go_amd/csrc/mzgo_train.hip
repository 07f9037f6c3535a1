// mzgo_train.hip -- the trainer's backward of the dynamics conv on fp32 MFMA
// (main.py's training step, main.py:478-482's
// loss.backward() through DynamicsNetwork.forward, main.py:97-103).
//
// Forward (k_recurrent_inference):  x' = relu(conv3x3(x) + b),  x = latent + emb[a]
// broadcast over the board (zero padding 1).  Given g = dL/dx', with the ReLU
// mask taken from the saved output (gp = g * [x' > 0]):
//
//   gx[b][ci][q]          = sum_{co,ky,kx} W[co][ci][ky][kx] gp[b][co][q - (ky-1, kx-1)]   (conv2d_input)
//   gw[co][ci][ky][kx]    = sum_{b,p} gp[b][co][p] x[b][ci][p + (ky-1, kx-1)]              (conv2d_weight)
//   gb[co]                = sum_{b,p} gp[b][co][p]
//
// both as implicit GEMMs on v_mfma_f32_16x16x4_f32 (exact f32 products, f32
// accumulation; the summation order differs from MIOpen's, so the tolerance
// against torch is fp32 rounding).  gx: one wave per (board, 16 cells, 16 ci)
// tile, K = 9 taps x C co in k-steps of 4.  gw: one wave per (16 co, 16 ci,
// tap) tile and chunk of boards, K = the chunk's boards x cells; the chunks'
// partial tiles land in a workspace and k_dyn_bwd_reduce sums them in chunk
// order (deterministic, no atomics) together with gb.
//
// Operand fragments (16x16x4 f32): lane l holds A[l & 15][k = l >> 4] and
// B[k = l >> 4][l & 15]; the result C[(l >> 4) * 4 + r][l & 15] in register r.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace mzgo {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kBwdChunk = 8;   // boards per gw partial (a chunk's K = 8 x cells)

// gp at (b, co, cell (y, x)) or 0 off the board
__device__ __forceinline__ float masked_grad(const float* __restrict__ g, const float* __restrict__ out,
                                             size_t plane, int N, int y, int x) {
  if (y < 0 || y >= N || x < 0 || x >= N) return 0.f;
  const size_t i = plane + (size_t)y * N + x;
  return out[i] > 0.f ? g[i] : 0.f;
}

// grid (ceil(CELLS/16), C/16, B), one wave per block
__global__ void __launch_bounds__(64) k_dyn_bwd_input(const float* __restrict__ g, const float* __restrict__ out,
                                                      const float* __restrict__ w, float* __restrict__ gx, int C,
                                                      int N) {
  const int lane = threadIdx.x;
  const int CELLS = N * N;
  const int b = blockIdx.z, ci0 = blockIdx.y * 16, p0 = blockIdx.x * 16;
  const int i = lane & 15, k = lane >> 4;
  const int p = p0 + i;                           // this lane's A row (cell)
  const int py = p / N, px = p - py * N;
  const bool prow = p < CELLS;
  const int ci = ci0 + i;                         // this lane's B column
  const size_t bplane = (size_t)b * C * CELLS;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (int tap = 0; tap < 9; ++tap) {
    const int ky = tap / 3, kx = tap - ky * 3;
    const int qy = py - ky + 1, qx = px - kx + 1;
    for (int co0 = 0; co0 < C; co0 += 4) {
      const int co = co0 + k;
      const float a = prow ? masked_grad(g, out, bplane + (size_t)co * CELLS, N, qy, qx) : 0.f;
      const float bw = w[((size_t)co * C + ci) * 9 + tap];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bw, acc, 0, 0, 0);
    }
  }
  const int col = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int pr = p0 + (lane >> 4) * 4 + r;
    if (pr < CELLS) gx[bplane + (size_t)(ci0 + col) * CELLS + pr] = acc[r];
  }
}

// grid (C/16 co tiles * C/16 ci tiles, 9 taps, chunks), one wave per block:
// partial[chunk][co][ci][tap] over the chunk's boards
__global__ void __launch_bounds__(64) k_dyn_bwd_weight(const float* __restrict__ g, const float* __restrict__ out,
                                                       const float* __restrict__ latent,
                                                       const int64_t* __restrict__ action,
                                                       const float* __restrict__ emb, float* __restrict__ part,
                                                       int B, int C, int N) {
  const int lane = threadIdx.x;
  const int CELLS = N * N;
  const int CT = C / 16;
  const int co0 = (blockIdx.x / CT) * 16, ci0 = (blockIdx.x % CT) * 16;
  const int tap = blockIdx.y, ky = tap / 3, kx = tap - ky * 3;
  const int chunk = blockIdx.z;
  const int i = lane & 15, k = lane >> 4;
  const int co = co0 + i, ci = ci0 + i;           // A row (co) / B column (ci) of this lane
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const int b1 = min(B, (chunk + 1) * kBwdChunk);
  for (int b = chunk * kBwdChunk; b < b1; ++b) {
    const size_t bplane = (size_t)b * C * CELLS;
    const float e = emb[(size_t)action[b] * C + ci];
    for (int p0 = 0; p0 < CELLS; p0 += 4) {
      const int p = p0 + k;                       // K index: this lane's cell
      float a = 0.f, bx = 0.f;
      if (p < CELLS) {
        const int py = p / N, px = p - py * N;
        a = masked_grad(g, out, bplane + (size_t)co * CELLS, N, py, px);
        const int sy = py + ky - 1, sx = px + kx - 1;
        if (sy >= 0 && sy < N && sx >= 0 && sx < N) bx = latent[bplane + (size_t)ci * CELLS + sy * N + sx] + e;
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bx, acc, 0, 0, 0);
    }
  }
  const int col = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int cor = co0 + (lane >> 4) * 4 + r;
    part[(((size_t)chunk * C + cor) * C + ci0 + col) * 9 + tap] = acc[r];
  }
}

// gw = the chunks' partials summed in chunk order; gb[co] = sum_{b,p} gp
// (one thread per (co, ci, tap); threads with ci = tap = 0 also form gb[co])
__global__ void __launch_bounds__(256) k_dyn_bwd_reduce(const float* __restrict__ part, const float* __restrict__ g,
                                                        const float* __restrict__ out, float* __restrict__ gw,
                                                        float* __restrict__ gb, int chunks, int B, int C, int N) {
  const size_t n = (size_t)C * C * 9;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < n) {
    float s = 0.f;
    for (int c = 0; c < chunks; ++c) s += part[(size_t)c * n + idx];
    gw[idx] = s;
  }
  if (idx < (size_t)C) {
    const int CELLS = N * N;
    float s = 0.f;
    for (int b = 0; b < B; ++b) {
      const size_t plane = ((size_t)b * C + idx) * CELLS;
      for (int p = 0; p < CELLS; ++p) s += out[plane + p] > 0.f ? g[plane + p] : 0.f;
    }
    gb[idx] = s;
  }
}

size_t dyn_bwd_workspace_bytes(int B, int C) {
  const size_t chunks = (size_t)(B + kBwdChunk - 1) / kBwdChunk;
  return chunks * (size_t)C * C * 9 * sizeof(float);
}

hipError_t dyn_conv_backward(const float* g, const float* out, const float* latent, const int64_t* action,
                             const float* emb, const float* w, int B, int C, int N, float* gx, float* gw,
                             float* gb, void* workspace, hipStream_t s) {
  const int CELLS = N * N;
  const int chunks = (B + kBwdChunk - 1) / kBwdChunk;
  hipLaunchKernelGGL(k_dyn_bwd_input, dim3((CELLS + 15) / 16, C / 16, B), dim3(64), 0, s, g, out, w, gx, C, N);
  hipLaunchKernelGGL(k_dyn_bwd_weight, dim3((C / 16) * (C / 16), 9, chunks), dim3(64), 0, s, g, out, latent,
                     action, emb, static_cast<float*>(workspace), B, C, N);
  const size_t n = (size_t)C * C * 9;
  hipLaunchKernelGGL(k_dyn_bwd_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     static_cast<const float*>(workspace), g, out, gw, gb, chunks, B, C, N);
  return hipGetLastError();
}

}  // namespace mzgo
