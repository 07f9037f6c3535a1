// mzgo_train.hip -- the trainer's 3x3 conv layers on fp32 MFMA: forward
// (activation recomputation) and backward (main.py's
// training step, main.py:478-482's loss.backward() through
// RepresentationNetwork.forward, main.py:72-84, and DynamicsNetwork.forward,
// main.py:97-103).
//
// A layer:  y = relu(conv3x3(x) + b), padding 1, x [B][Cin][N][N] -- for the
// dynamics x = latent + emb[a] broadcast over the board (emb given).  Given
// g = dL/dy, with the ReLU mask taken from the saved output (gp = g * [y > 0]):
//
//   gx[b][ci][q]          = sum_{co,ky,kx} W[co][ci][ky][kx] gp[b][co][q - (ky-1, kx-1)]   (conv2d_input)
//   gw[co][ci][ky][kx]    = sum_{b,p} gp[b][co][p] x[b][ci][p + (ky-1, kx-1)]              (conv2d_weight)
//   gb[co]                = sum_{b,p} gp[b][co][p]
//
// All as implicit GEMMs on v_mfma_f32_16x16x4_f32 (exact f32 products, f32
// accumulation; the summation order differs from MIOpen's, so the tolerance
// against torch is fp32 rounding).  Channel counts need not be multiples of
// 16 (the representation's conv1 has Cin = 6): tiles are masked.
//   forward: one wave per (board, 16 cells, 16 co) tile, K = Cin x 9 taps.
//   gx:      one wave per (board, 16 cells, 16 ci) tile, K = 9 taps x Cout.
//   gw:      one workgroup of 9 waves (one per tap) per (16 co, 16 ci) tile and
//            chunk of boards: the chunk's gp rows and zero-haloed x planes are
//            staged in LDS with coalesced loads, K = the chunk's boards x
//            cells; the chunks' partial tiles land in a workspace and
//            k_conv_bwd_reduce sums them in chunk order (deterministic, no
//            atomics).
//   gb:      one workgroup per co, a fixed-order tree reduction.
//
// Operand fragments (16x16x4 f32): lane l holds A[l & 15][k = l >> 4] and
// B[k = l >> 4][l & 15]; the result C[(l >> 4) * 4 + r][l & 15] in register r.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace mzgo {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kBwdChunk = 8;   // boards per gw partial (a chunk's K = 8 x cells)
constexpr int kMaxN = 19;

// gp at (b, co, cell (y, x)) or 0 off the board
__device__ __forceinline__ float masked_grad(const float* __restrict__ g, const float* __restrict__ out,
                                             size_t plane, int N, int y, int x) {
  if (y < 0 || y >= N || x < 0 || x >= N) return 0.f;
  const size_t i = plane + (size_t)y * N + x;
  return out[i] > 0.f ? g[i] : 0.f;
}

// y = relu(conv3x3(x (+ emb[action]) ) + bias); grid (ceil(CELLS/16), ceil(Cout/16), B), one wave
__global__ void __launch_bounds__(64) k_conv_fwd(const float* __restrict__ x, const int64_t* __restrict__ action,
                                                 const float* __restrict__ emb, const float* __restrict__ w,
                                                 const float* __restrict__ bias, float* __restrict__ y, int Cin,
                                                 int Cout, int N) {
  const int lane = threadIdx.x;
  const int CELLS = N * N;
  const int b = blockIdx.z, co0 = blockIdx.y * 16, p0 = blockIdx.x * 16;
  const int i = lane & 15, k = lane >> 4;
  const int p = p0 + i;                           // this lane's A row (cell)
  const int py = p / N, px = p - py * N;
  const bool prow = p < CELLS;
  const int co = co0 + i;                         // this lane's B column
  const bool ccol = co < Cout;
  const float* xb = x + (size_t)b * Cin * CELLS;
  const float* eb = emb ? emb + (size_t)action[b] * Cin : nullptr;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (int tap = 0; tap < 9; ++tap) {
    const int ky = tap / 3, kx = tap - ky * 3;
    const int sy = py + ky - 1, sx = px + kx - 1;
    const bool on = prow && sy >= 0 && sy < N && sx >= 0 && sx < N;
    for (int c0 = 0; c0 < Cin; c0 += 4) {
      const int ci = c0 + k;
      const bool okc = ci < Cin;
      const float a = on && okc ? xb[(size_t)ci * CELLS + sy * N + sx] + (eb ? eb[ci] : 0.f) : 0.f;
      const float bw = ccol && okc ? w[((size_t)co * Cin + ci) * 9 + tap] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bw, acc, 0, 0, 0);
    }
  }
  const int col = co0 + (lane & 15);
  if (col < Cout) {
    const float bb = bias[col];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pr = p0 + (lane >> 4) * 4 + r;
      const float v = acc[r] + bb;
      if (pr < CELLS) y[((size_t)b * Cout + col) * CELLS + pr] = v > 0.f ? v : 0.f;
    }
  }
}

// gx; grid (ceil(CELLS/16), ceil(Cin/16), B), one wave per block
__global__ void __launch_bounds__(64) k_conv_bwd_input(const float* __restrict__ g, const float* __restrict__ out,
                                                       const float* __restrict__ w, float* __restrict__ gx, int Cin,
                                                       int Cout, int N) {
  const int lane = threadIdx.x;
  const int CELLS = N * N;
  const int b = blockIdx.z, ci0 = blockIdx.y * 16, p0 = blockIdx.x * 16;
  const int i = lane & 15, k = lane >> 4;
  const int p = p0 + i;                           // this lane's A row (cell)
  const int py = p / N, px = p - py * N;
  const bool prow = p < CELLS;
  const int ci = ci0 + i;                         // this lane's B column
  const bool ccol = ci < Cin;
  const size_t gplane = (size_t)b * Cout * CELLS;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (int tap = 0; tap < 9; ++tap) {
    const int ky = tap / 3, kx = tap - ky * 3;
    const int qy = py - ky + 1, qx = px - kx + 1;
    for (int co0 = 0; co0 < Cout; co0 += 4) {
      const int co = co0 + k;
      const bool okc = co < Cout;
      const float a = prow && okc ? masked_grad(g, out, gplane + (size_t)co * CELLS, N, qy, qx) : 0.f;
      const float bw = ccol && okc ? w[((size_t)co * Cin + ci) * 9 + tap] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bw, acc, 0, 0, 0);
    }
  }
  const int col = ci0 + (lane & 15);
  if (col < Cin) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pr = p0 + (lane >> 4) * 4 + r;
      if (pr < CELLS) gx[((size_t)b * Cin + col) * CELLS + pr] = acc[r];
    }
  }
}

// partial[chunk][co][ci][tap] over the chunk's boards; grid (coT * ciT, chunks),
// 9 waves (wave = tap)
constexpr int kGpStride = kMaxN * kMaxN + 3;            // gp row in LDS (cells, padded to a float4 of K)
constexpr int kXPlane = (kMaxN + 2) * (kMaxN + 2);      // zero-haloed x plane in LDS
__global__ void __launch_bounds__(576) k_conv_bwd_weight(const float* __restrict__ g, const float* __restrict__ out,
                                                         const float* __restrict__ x,
                                                         const int64_t* __restrict__ action,
                                                         const float* __restrict__ emb, float* __restrict__ part,
                                                         int B, int Cin, int Cout, int N) {
  __shared__ float gpl[16 * kGpStride];
  __shared__ float xl[16 * kXPlane];
  const int tid = threadIdx.x, lane = tid & 63, tap = tid >> 6;
  const int CELLS = N * N, PW = N + 2, PLANE = PW * PW;
  const int CT = (Cin + 15) / 16;
  const int co0 = (blockIdx.x / CT) * 16, ci0 = (blockIdx.x % CT) * 16;
  const int chunk = blockIdx.y;
  const int ky = tap / 3, kx = tap - ky * 3;
  const int i = lane & 15, k = lane >> 4;
  // zero halo of the x planes (interior rewritten per board) and the K pad of gp
  for (int j = tid; j < 16 * kXPlane; j += 576) xl[j] = 0.f;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const int b1 = min(B, (chunk + 1) * kBwdChunk);
  for (int b = chunk * kBwdChunk; b < b1; ++b) {
    __syncthreads();                                  // the previous board's reads are done
    // stage: gp rows of the 16 co, x planes of the 16 ci (row-contiguous loads)
    for (int j = tid; j < 16 * CELLS; j += 576) {
      const int r = j / CELLS, p = j - r * CELLS;
      const int co = co0 + r, ci = ci0 + r;
      float gv = 0.f, xv = 0.f;
      if (co < Cout) {
        const size_t idx = ((size_t)b * Cout + co) * CELLS + p;
        gv = out[idx] > 0.f ? g[idx] : 0.f;
      }
      if (ci < Cin) xv = x[((size_t)b * Cin + ci) * CELLS + p] + (emb ? emb[(size_t)action[b] * Cin + ci] : 0.f);
      gpl[r * kGpStride + p] = gv;
      const int py = p / N, px = p - py * N;
      xl[r * kXPlane + (py + 1) * PW + px + 1] = xv;
    }
    for (int j = tid; j < 16 * 3; j += 576) gpl[(j / 3) * kGpStride + CELLS + j % 3] = 0.f;
    __syncthreads();
    for (int p0 = 0; p0 < CELLS; p0 += 4) {
      const int p = p0 + k;                           // K index: this lane's cell
      const float a = gpl[i * kGpStride + p];         // (p >= CELLS: the zero pad)
      float bx = 0.f;
      if (p < CELLS) {
        const int py = p / N, px = p - py * N;
        bx = xl[i * kXPlane + (py + ky) * PW + px + kx];
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bx, acc, 0, 0, 0);
    }
  }
  (void)PLANE;
  const int ci = ci0 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int co = co0 + (lane >> 4) * 4 + r;
    if (co < Cout && ci < Cin) part[(((size_t)chunk * Cout + co) * Cin + ci) * 9 + tap] = acc[r];
  }
}

// gw = the chunks' partials summed in chunk order
__global__ void __launch_bounds__(256) k_conv_bwd_reduce(const float* __restrict__ part, float* __restrict__ gw,
                                                         int chunks, size_t n) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n) return;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += part[(size_t)c * n + idx];
  gw[idx] = s;
}

// gb[co] = sum_{b,p} gp: one workgroup per co; each thread sums a fixed
// strided subset in order, then a fixed-order tree (deterministic)
__global__ void __launch_bounds__(256) k_conv_bwd_bias(const float* __restrict__ g, const float* __restrict__ out,
                                                       float* __restrict__ gb, int B, int Cout, int N) {
  __shared__ float red[256];
  const int co = blockIdx.x, tid = threadIdx.x, CELLS = N * N;
  float s = 0.f;
  for (int j = tid; j < B * CELLS; j += 256) {
    const int b = j / CELLS, p = j - b * CELLS;
    const size_t idx = ((size_t)b * Cout + co) * CELLS + p;
    s += out[idx] > 0.f ? g[idx] : 0.f;
  }
  red[tid] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (tid < h) red[tid] += red[tid + h];
    __syncthreads();
  }
  if (tid == 0) gb[co] = red[0];
}

size_t conv_bwd_workspace_bytes(int B, int Cin, int Cout) {
  const size_t chunks = (size_t)(B + kBwdChunk - 1) / kBwdChunk;
  return chunks * (size_t)Cout * Cin * 9 * sizeof(float);
}

hipError_t conv_forward(const float* x, const int64_t* action, const float* emb, const float* w, const float* bias,
                        int B, int Cin, int Cout, int N, float* y, hipStream_t s) {
  const int CELLS = N * N;
  hipLaunchKernelGGL(k_conv_fwd, dim3((CELLS + 15) / 16, (Cout + 15) / 16, B), dim3(64), 0, s, x, action, emb, w,
                     bias, y, Cin, Cout, N);
  return hipGetLastError();
}

hipError_t conv_backward(const float* g, const float* out, const float* x, const int64_t* action, const float* emb,
                         const float* w, int B, int Cin, int Cout, int N, float* gx, float* gw, float* gb,
                         void* workspace, hipStream_t s) {
  const int CELLS = N * N;
  const int chunks = (B + kBwdChunk - 1) / kBwdChunk;
  if (gx)
    hipLaunchKernelGGL(k_conv_bwd_input, dim3((CELLS + 15) / 16, (Cin + 15) / 16, B), dim3(64), 0, s, g, out, w, gx,
                       Cin, Cout, N);
  hipLaunchKernelGGL(k_conv_bwd_weight, dim3(((Cout + 15) / 16) * ((Cin + 15) / 16), chunks), dim3(576), 0, s, g,
                     out, x, action, emb, static_cast<float*>(workspace), B, Cin, Cout, N);
  const size_t n = (size_t)Cout * Cin * 9;
  hipLaunchKernelGGL(k_conv_bwd_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     static_cast<const float*>(workspace), gw, chunks, n);
  hipLaunchKernelGGL(k_conv_bwd_bias, dim3(Cout), dim3(256), 0, s, g, out, gb, B, Cout, N);
  return hipGetLastError();
}

}  // namespace mzgo
