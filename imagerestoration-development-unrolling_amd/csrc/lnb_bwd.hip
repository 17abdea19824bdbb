// Reverse pass of LocalNonLinearBlock (nsubnets = 1; REF:911-964, REF13:541-575) for training.
//
// Forward (lnb_ops.hip fuses all of it; the reverse recomputes the pieces it needs):
//   n   = ln_w * x * isd,  isd = 1/sqrt(var_c x + 1e-5)  (unbiased, x NOT centred: REF:919-925)
//   h   = W1 n                         (1x1 GEMM, HIP conv1x1)
//   h'  = dw3x3_replicate(h)           (depthwise, 2 hid channels)
//   gate = sigmoid(m) m v,  (m, v) = h'[:hid], h'[hid:]
//   out = s0 x + s1 W2 gate
// Kernels here: the per-pixel LN forward, depthwise 3x3 forward, gate forward / reverse,
// depthwise reverse (data: exact adjoint of the clamped gather; weights: per-channel
// reductions) and the LN reverse.  The GEMMs of the reverse (W2^T go, W1^T gh) run on the
// HIP conv1x1; their weight gradients are library GEMMs (host side).
#include <algorithm>

#include "grr_common.h"

namespace grr {
namespace {

constexpr int NT = 256;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ void block_atomic_add(float* dst, float v) {
  __shared__ float red[NT / 64];
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    if (t != 0.f) atomicAdd(dst, t);
  }
}

// n = ln_w x isd, isd per pixel.   grid-stride over B*P pixels
__global__ __launch_bounds__(NT) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ lnw,
                                                    float* __restrict__ n, float* __restrict__ isd, int C,
                                                    int64_t P, int64_t npix) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < npix; i += (int64_t)gridDim.x * NT) {
    const int64_t b = i / P, p = i - b * P;
    const float* xp = x + b * C * P + p;
    float s = 0.f;
#pragma unroll 8
    for (int c = 0; c < C; ++c) s += xp[(int64_t)c * P];
    const float mean = s / (float)C;
    float q = 0.f;
#pragma unroll 8
    for (int c = 0; c < C; ++c) {
      const float d = xp[(int64_t)c * P] - mean;
      q += d * d;
    }
    const float r = 1.0f / sqrtf(q / (float)(C - 1) + 1e-5f);
    isd[i] = r;
    float* np_ = n + b * C * P + p;
#pragma unroll 8
    for (int c = 0; c < C; ++c) np_[(int64_t)c * P] = lnw[c] * xp[(int64_t)c * P] * r;
  }
}

// gx_k (+)= ln_w_k gn_k isd - (x_k - mean) isd^3 / (C-1) * sum_c ln_w_c gn_c x_c
__global__ __launch_bounds__(NT) void ln_bwd_kernel(const float* __restrict__ x, const float* __restrict__ lnw,
                                                    const float* __restrict__ isd, const float* __restrict__ gn,
                                                    float* __restrict__ gx, int C, int64_t P, int64_t npix) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < npix; i += (int64_t)gridDim.x * NT) {
    const int64_t b = i / P, p = i - b * P;
    const float* xp = x + b * C * P + p;
    const float* gp = gn + b * C * P + p;
    float s = 0.f, dot = 0.f;
#pragma unroll 8
    for (int c = 0; c < C; ++c) {
      const float xv = xp[(int64_t)c * P];
      s += xv;
      dot += lnw[c] * gp[(int64_t)c * P] * xv;
    }
    const float mean = s / (float)C, r = isd[i];
    const float k = dot * r * r * r / (float)(C - 1);
    float* gxp = gx + b * C * P + p;
#pragma unroll 8
    for (int c = 0; c < C; ++c) {
      const int64_t o = (int64_t)c * P;
      gxp[o] += lnw[c] * gp[o] * r - (xp[o] - mean) * k;
    }
  }
}

// gw[c] += sum_{b,p} u v isd(b,p)          grid (chunks, B*C)
__global__ __launch_bounds__(NT) void ln_wgrad_kernel(const float* __restrict__ u, const float* __restrict__ v,
                                                      const float* __restrict__ isd, float* __restrict__ gw, int C,
                                                      int64_t P) {
  const int plane = blockIdx.y, c = plane % C, b = plane / C;
  const float* up = u + (int64_t)plane * P;
  const float* vp = v + (int64_t)plane * P;
  const float* sp = isd + (int64_t)b * P;
  float acc = 0.f;
  for (int64_t p = blockIdx.x * (int64_t)NT + threadIdx.x; p < P; p += (int64_t)gridDim.x * NT)
    acc += up[p] * vp[p] * sp[p];
  block_atomic_add(gw + c, acc);
}

// h'(p) = sum_t w_t h(clamp(p + t)), t = (dy, dx) in {-1,0,1}^2, tap index (dy+1)*3 + dx+1
__global__ __launch_bounds__(NT) void dw3_fwd_kernel(const float* __restrict__ h, const float* __restrict__ wdw,
                                                     float* __restrict__ out, int C, int H, int W) {
  const int HW = H * W;
  const int p = blockIdx.x * NT + threadIdx.x;
  if (p >= HW) return;
  const int plane = blockIdx.y, c = plane % C;
  const int r = p / W, col = p - r * W;
  const float* hp = h + (int64_t)plane * HW;
  float acc = 0.f;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx)
      acc += wdw[c * 9 + (dy + 1) * 3 + dx + 1] * hp[clampi(r + dy, 0, H - 1) * W + clampi(col + dx, 0, W - 1)];
  out[(int64_t)plane * HW + p] = acc;
}

// adjoint of the clamped gather along one axis: the source rows s with clamp(s + d) = q
__device__ __forceinline__ int axis_sources(int q, int d, int n, int (&s)[2]) {
  if (d == 0) { s[0] = q; return 1; }
  int k = 0;
  if (q - d >= 0 && q - d < n) s[k++] = q - d;
  if ((d > 0 && q == n - 1) || (d < 0 && q == 0)) s[k++] = q;
  return k;
}

// gh(q) = sum_t w_t sum_{p: clamp(p+t) = q} g(p)   (exact adjoint of dw3_fwd)
__global__ __launch_bounds__(NT) void dw3_bwd_data_kernel(const float* __restrict__ g, const float* __restrict__ wdw,
                                                          float* __restrict__ gh, int C, int H, int W) {
  const int HW = H * W;
  const int p = blockIdx.x * NT + threadIdx.x;
  if (p >= HW) return;
  const int plane = blockIdx.y, c = plane % C;
  const int r = p / W, col = p - r * W;
  const float* gp = g + (int64_t)plane * HW;
  float acc = 0.f;
  if (r > 0 && r < H - 1 && col > 0 && col < W - 1) {   // interior: correlation with the flipped taps
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) acc += wdw[c * 9 + (dy + 1) * 3 + dx + 1] * gp[(r - dy) * W + col - dx];
    gh[(int64_t)plane * HW + p] = acc;
    return;
  }
  for (int dy = -1; dy <= 1; ++dy) {
    int sy[2];
    const int ny = axis_sources(r, dy, H, sy);
    for (int dx = -1; dx <= 1; ++dx) {
      int sx[2];
      const int nx = axis_sources(col, dx, W, sx);
      const float wt = wdw[c * 9 + (dy + 1) * 3 + dx + 1];
      float s = 0.f;
      for (int a = 0; a < ny; ++a)
        for (int e = 0; e < nx; ++e) s += gp[sy[a] * W + sx[e]];
      acc += wt * s;
    }
  }
  gh[(int64_t)plane * HW + p] = acc;
}

// gw[c, t] += sum_{b,p} g(p) h(clamp(p + t))        grid (chunks, B*C)
__global__ __launch_bounds__(NT) void dw3_wgrad_kernel(const float* __restrict__ g, const float* __restrict__ h,
                                                       float* __restrict__ gw, int C, int H, int W) {
  const int HW = H * W;
  const int plane = blockIdx.y, c = plane % C;
  const float* gp = g + (int64_t)plane * HW;
  const float* hp = h + (int64_t)plane * HW;
  float acc[9] = {};
  for (int p = blockIdx.x * NT + threadIdx.x; p < HW; p += gridDim.x * NT) {
    const int r = p / W, col = p - r * W;
    const float gv = gp[p];
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx)
        acc[(dy + 1) * 3 + dx + 1] += gv * hp[clampi(r + dy, 0, H - 1) * W + clampi(col + dx, 0, W - 1)];
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) block_atomic_add(gw + c * 9 + t, acc[t]);
}

// gate = sigmoid(m) m v (if gate != NULL); gm, gv from ggate (if ggate != NULL).   hp [B, 2hid, P]
__global__ __launch_bounds__(NT) void gate_kernel(const float* __restrict__ hp, const float* __restrict__ ggate,
                                                  float* __restrict__ gate, float* __restrict__ ghp, int hid,
                                                  int64_t P, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t b = i / ((int64_t)hid * P), rem = i - b * hid * P;   // rem = j P + p
    const int64_t om = b * 2 * hid * P + rem, ov = om + (int64_t)hid * P;
    const float m = hp[om], v = hp[ov];
    const float sg = 1.0f / (1.0f + expf(-m));
    if (gate) gate[i] = (sg * m) * v;
    if (ggate) {
      const float gg = ggate[i];
      ghp[om] = gg * v * (sg + m * sg * (1.0f - sg));
      ghp[ov] = gg * sg * m;
    }
  }
}

int grid_for(int64_t n) { return (int)std::min<int64_t>((n + NT - 1) / NT, 1 << 16); }
int chunks_for(int64_t n, int64_t planes) {
  const int64_t want = (4096 + planes - 1) / planes;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, (n + NT - 1) / NT));
}

}  // namespace
}  // namespace grr

using namespace grr;

extern "C" {

grr_status grr_lnb_norm(const float* x, const float* ln_w, float* n, float* isd, int B, int C, int64_t P,
                        void* stream) {
  clear_error();
  GRR_REQUIRE(x && ln_w && n && isd && B > 0 && C > 1 && P > 0, GRR_ERR_INVALID_ARG, "grr_lnb_norm: bad args");
  const int64_t np = (int64_t)B * P;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3(grid_for(np)), dim3(NT), 0, (hipStream_t)stream, x, ln_w, n, isd, C, P, np);
  return launch_status("grr_lnb_norm");
}

grr_status grr_lnb_norm_bwd(const float* x, const float* ln_w, const float* isd, const float* gn, float* gx,
                            float* gln_w, int B, int C, int64_t P, void* stream) {
  clear_error();
  GRR_REQUIRE(x && ln_w && isd && gn && gx && gln_w && B > 0 && C > 1 && P > 0, GRR_ERR_INVALID_ARG,
              "grr_lnb_norm_bwd: bad args");
  GRR_REQUIRE((int64_t)B * C <= 65535, GRR_ERR_UNSUPPORTED, "grr_lnb_norm_bwd: B*C > 65535");
  const int64_t np = (int64_t)B * P;
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(grid_for(np)), dim3(NT), 0, (hipStream_t)stream, x, ln_w, isd, gn, gx, C,
                     P, np);
  grr_status st = launch_status("grr_lnb_norm_bwd/data");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(ln_wgrad_kernel, dim3(chunks_for(P, (int64_t)B * C), B * C), dim3(NT), 0, (hipStream_t)stream,
                     gn, x, isd, gln_w, C, P);
  return launch_status("grr_lnb_norm_bwd/weight");
}

grr_status grr_dwconv3(const float* h, const float* wdw, float* out, int B, int C, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(h && wdw && out && B > 0 && C > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG, "grr_dwconv3: bad args");
  GRR_REQUIRE((int64_t)B * C <= 65535, GRR_ERR_UNSUPPORTED, "grr_dwconv3: B*C > 65535");
  hipLaunchKernelGGL(dw3_fwd_kernel, dim3((H * W + NT - 1) / NT, B * C), dim3(NT), 0, (hipStream_t)stream, h, wdw,
                     out, C, H, W);
  return launch_status("grr_dwconv3");
}

grr_status grr_dwconv3_bwd(const float* g, const float* h, const float* wdw, float* gh, float* gwdw, int B, int C,
                           int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(g && h && wdw && gh && gwdw && B > 0 && C > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_dwconv3_bwd: bad args");
  GRR_REQUIRE((int64_t)B * C <= 65535, GRR_ERR_UNSUPPORTED, "grr_dwconv3_bwd: B*C > 65535");
  hipLaunchKernelGGL(dw3_bwd_data_kernel, dim3((H * W + NT - 1) / NT, B * C), dim3(NT), 0, (hipStream_t)stream, g,
                     wdw, gh, C, H, W);
  grr_status st = launch_status("grr_dwconv3_bwd/data");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(dw3_wgrad_kernel, dim3(chunks_for((int64_t)H * W, (int64_t)B * C), B * C), dim3(NT), 0,
                     (hipStream_t)stream, g, h, gwdw, C, H, W);
  return launch_status("grr_dwconv3_bwd/weight");
}

grr_status grr_lnb_gate(const float* hp, const float* ggate, float* gate, float* ghp, int B, int hid, int64_t P,
                        void* stream) {
  clear_error();
  GRR_REQUIRE(hp && B > 0 && hid > 0 && P > 0 && (gate || ggate) && (!ggate || ghp), GRR_ERR_INVALID_ARG,
              "grr_lnb_gate: bad args");
  const int64_t n = (int64_t)B * hid * P;
  hipLaunchKernelGGL(gate_kernel, dim3(grid_for(n)), dim3(NT), 0, (hipStream_t)stream, hp, ggate, gate, ghp, hid, P,
                     n);
  return launch_status("grr_lnb_gate");
}

}  // extern "C"
