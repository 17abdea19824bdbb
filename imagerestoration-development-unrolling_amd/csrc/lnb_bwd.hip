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
// one partial per block (grr_common.h, fixed-order reductions): wave sums -> LDS -> thread 0 adds
// them in wave order and stores the block's slot
__device__ __forceinline__ void block_red_put(const Red& r, int idx, uint32_t slot, float v) {
  __shared__ float red[NT / 64];
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    red_put(r, idx, slot, t);
  }
}
// slot of block (blockIdx.x, blockIdx.y) of a (chunks, B * per) grid: one per (b, chunk)
__device__ __forceinline__ uint32_t chunk_slot(int per) {
  return (uint32_t)(blockIdx.y / per) * gridDim.x + blockIdx.x;
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
// SKIP: the block's skip term in the same pass, gx_k = s0 gout_k + (...) (written, not accumulated) and
// gdot += <gout, x> (the skip weight's gradient) -- no separate scale and dot passes over gout
template <bool SKIP>
__global__ __launch_bounds__(NT) void ln_bwd_kernel(const float* __restrict__ x, const float* __restrict__ lnw,
                                                    const float* __restrict__ isd, const float* __restrict__ gn,
                                                    const float* __restrict__ gout, const float* __restrict__ skip,
                                                    float* __restrict__ gx, Red gdot, int C, int64_t P,
                                                    int64_t npix) {
  const float s0 = SKIP ? skip[0] : 0.f;
  float dacc = 0.f;
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
    if constexpr (SKIP) {
      const float* op = gout + b * C * P + p;
#pragma unroll 8
      for (int c = 0; c < C; ++c) {
        const int64_t o = (int64_t)c * P;
        const float go = op[o];
        dacc += go * xp[o];
        gxp[o] = __fmul_rn(s0, go) + (lnw[c] * gp[o] * r - (xp[o] - mean) * k);
      }
    } else {
#pragma unroll 8
      for (int c = 0; c < C; ++c) {
        const int64_t o = (int64_t)c * P;
        gxp[o] += lnw[c] * gp[o] * r - (xp[o] - mean) * k;
      }
    }
  }
  if constexpr (SKIP) block_red_put(gdot, 0, blockIdx.x, dacc);
}

// gw[c] += sum_{b,p} u v isd(b,p)          grid (chunks, B*C)
__global__ __launch_bounds__(NT) void ln_wgrad_kernel(const float* __restrict__ u, const float* __restrict__ v,
                                                      const float* __restrict__ isd, Red gw, int C, int64_t P) {
  const int plane = blockIdx.y, c = plane % C, b = plane / C;
  const float* up = u + (int64_t)plane * P;
  const float* vp = v + (int64_t)plane * P;
  const float* sp = isd + (int64_t)b * P;
  float acc = 0.f;
  for (int64_t p = blockIdx.x * (int64_t)NT + threadIdx.x; p < P; p += (int64_t)gridDim.x * NT)
    acc += up[p] * vp[p] * sp[p];
  block_red_put(gw, c, chunk_slot(C), acc);
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
                                                       Red gw, int C, int H, int W) {
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
  for (int t = 0; t < 9; ++t) block_red_put(gw, c * 9 + t, chunk_slot(C), acc[t]);
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

// Reverse of the gate with the skip scale folded in: ghp = scale * d(gate)/d(hp) . gq and
// gdot += <gq, gate>, gq = W2^T gout (so that <gout, W2 gate> = <gq, gate> needs no W2 gate).
// Grid-stride over all elements, one partial per block.
__global__ __launch_bounds__(NT) void gate_bwd_scaled_kernel(const float* __restrict__ hp, const float* __restrict__ gq,
                                                             const float* __restrict__ scale, float* __restrict__ ghp,
                                                             Red gdot, int hid, int64_t P, int64_t n) {
  const float s = scale[0];
  float dot = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t b = i / ((int64_t)hid * P), rem = i - b * hid * P;
    const int64_t om = b * 2 * hid * P + rem, ov = om + (int64_t)hid * P;
    const float m = hp[om], v = hp[ov];
    const float sg = 1.0f / (1.0f + expf(-m));
    const float q = gq[i];
    dot += q * ((sg * m) * v);
    const float gg = s * q;
    ghp[om] = gg * v * (sg + m * sg * (1.0f - sg));
    ghp[ov] = gg * sg * m;
  }
  block_red_put(gdot, 0, blockIdx.x, dot);
}

// ---------------------------------------------------------------------------
// Row-streaming depthwise 3x3 (W <= 64 V, W % V == 0): one wave = one (b, channel) plane and a
// segment of rows, lane = V adjacent columns; rows r-1, r, r+1 of the operands stay in
// registers (one row load per row and operand, prefetched one row ahead), horizontal
// neighbours come from DPP lane shifts.  The per-pixel kernels above issue nine scalar
// loads per output pixel and are L1-bound (dwconv3 2.3 TB/s, dwconv3_bwd 1.6 TB/s).
// ---------------------------------------------------------------------------
template <int V> struct RowVec;
template <> struct RowVec<1> { typedef float T; };
template <> struct RowVec<2> { typedef float __attribute__((ext_vector_type(2))) T; };
template <> struct RowVec<4> { typedef float __attribute__((ext_vector_type(4))) T; };
template <> struct RowVec<8> { typedef float __attribute__((ext_vector_type(8))) T; };

template <int V>
__device__ __forceinline__ void row_load(float (&d)[V], const float* p) {
  const typename RowVec<V>::T t = *reinterpret_cast<const typename RowVec<V>::T*>(p);
  if constexpr (V == 1) {
    d[0] = t;
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) d[j] = t[j];
  }
}
template <int V>
__device__ __forceinline__ void row_store(float* p, const float (&v)[V]) {
  typename RowVec<V>::T t;
  if constexpr (V == 1) {
    t = v[0];
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) t[j] = v[j];
  }
  *reinterpret_cast<typename RowVec<V>::T*>(p) = t;
}
// value of lane -1 / +1 (0 past the wave's ends); the asm pins the DPP at its definition
__device__ __forceinline__ float dpp_prev(float v) {
  float r = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xF, 0xF, true));
  asm volatile("" : "+v"(r));
  return r;
}
__device__ __forceinline__ float dpp_next(float v) {
  float r = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xF, 0xF, true));
  asm volatile("" : "+v"(r));
  return r;
}

// Rows wider than one wave (W > 64 V, W % V == 0) run as column strips: strip k's waves hold columns
// [x0, x0 + 64 V), x0 = k STEP - V (0 for the first), and own the output columns [k STEP, (k + 1) STEP):
// the V columns of each side are a halo (the depthwise reach is one column; DPP shifts stop at the
// wave's ends), so no value the owned columns depend on crosses a wave.  Image-edge rules use the
// global column.  Waves of neighbouring strips are neighbours in the grid (same row segment).
__host__ __device__ inline int dw3_row_strips(int W, int V) {
  const int step = 62 * V;
  return W <= 64 * V ? 1 : (W + step - 1) / step;
}
struct Dw3RowGeom {
  int lane, c0, cl0;
  bool on;
  int plane, c, r0, r1;
  uint32_t wid, slot;   // wave index; slot of the per-channel reductions = (b, segment, strip)
};
template <int V>
__device__ __forceinline__ bool dw3_row_geom(Dw3RowGeom& q, int C, int H, int W, int sseg, int nsegs, uint32_t nwaves) {
  q.lane = threadIdx.x & 63;
  const uint32_t wid = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (wid >= nwaves) return false;   // whole waves only
  constexpr int STEP = 62 * V;
  const int nstrips = dw3_row_strips(W, V);
  const int strip = (int)(wid % (uint32_t)nstrips);
  const uint32_t rest = wid / (uint32_t)nstrips;
  const int seg = (int)(rest % nsegs);
  q.plane = (int)(rest / nsegs);
  q.c = q.plane % C;
  q.wid = wid;
  q.slot = ((uint32_t)(q.plane / C) * nsegs + seg) * nstrips + strip;
  q.r0 = seg * sseg;
  q.r1 = min(q.r0 + sseg, H);
  const int x0 = strip == 0 ? 0 : strip * STEP - V;
  const int lo = nstrips == 1 ? 0 : strip * STEP;
  const int hi = nstrips == 1 ? W : min(lo + STEP, W);
  q.c0 = x0 + V * q.lane;
  q.on = q.c0 >= lo && q.c0 < hi;
  q.cl0 = clampi(q.c0, 0, W - V);
  return true;
}

// out(r, c) = sum_t w_t h(clamp(r + dy), clamp(c + dx))  (same taps and order as dw3_fwd_kernel)
template <int V>
__global__ __launch_bounds__(NT) void dw3_row_fwd_kernel(const float* __restrict__ h, const float* __restrict__ wdw,
                                                         float* __restrict__ out, int C, int H, int W, int sseg,
                                                         int nsegs, uint32_t nwaves) {
  Dw3RowGeom q;
  if (!dw3_row_geom<V>(q, C, H, W, sseg, nsegs, nwaves)) return;
  const int64_t HW = (int64_t)H * W;
  const float* hp = h + q.plane * HW + q.cl0;
  float* op = out + q.plane * HW + q.cl0;
  float wt[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wt[t] = wdw[q.c * 9 + t];
  float R[3][V], N[V];
  row_load<V>(R[0], hp + (int64_t)clampi(q.r0 - 1, 0, H - 1) * W);
  row_load<V>(R[1], hp + (int64_t)q.r0 * W);
  row_load<V>(N, hp + (int64_t)clampi(q.r0 + 1, 0, H - 1) * W);
  for (int r = q.r0; r < q.r1; ++r) {
#pragma unroll
    for (int j = 0; j < V; ++j) R[2][j] = N[j];
    row_load<V>(N, hp + (int64_t)clampi(r + 2, 0, H - 1) * W);
    float o[V];
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float pv = dpp_prev(R[dy][V - 1]), nx = dpp_next(R[dy][0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int col = q.c0 + j;
        const float l = col > 0 ? (j > 0 ? R[dy][j - 1] : pv) : R[dy][j];
        const float rr = col < W - 1 ? (j < V - 1 ? R[dy][j + 1] : nx) : R[dy][j];
        o[j] += wt[dy * 3 + 0] * l;
        o[j] += wt[dy * 3 + 1] * R[dy][j];
        o[j] += wt[dy * 3 + 2] * rr;
      }
    }
    if (q.on) row_store<V>(op + (int64_t)r * W, o);
#pragma unroll
    for (int j = 0; j < V; ++j) { R[0][j] = R[1][j]; R[1][j] = R[2][j]; }
  }
}

// One pass for both gradients of the depthwise conv:
//   gh(q) = sum_t w_t sum_{p: clamp(p + t) = q} g(p)   (adjoint of the clamped gather, separable:
//           rows then columns; along an axis the sources of q for offset d are q - d when inside,
//           plus q itself at the edge the clamp folds onto)
//   gw[c, t] += sum_p g(p) h(clamp(p + t))              (wave sums, one partial per tap and wave)
template <int V>
__global__ __launch_bounds__(NT) void dw3_row_bwd_kernel(const float* __restrict__ g, const float* __restrict__ h,
                                                         const float* __restrict__ wdw, float* __restrict__ gh,
                                                         Red gw, int C, int H, int W, int sseg,
                                                         int nsegs, uint32_t nwaves) {
  Dw3RowGeom q;
  if (!dw3_row_geom<V>(q, C, H, W, sseg, nsegs, nwaves)) return;
  const int64_t HW = (int64_t)H * W;
  const float* gp = g + q.plane * HW + q.cl0;
  const float* hp = h + q.plane * HW + q.cl0;
  float* ghp = gh + q.plane * HW + q.cl0;
  float wt[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) wt[t] = wdw[q.c * 9 + t];
  float acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = 0.f;
  // g rows r-1, r, r+1 (zero outside the image: the adjoint has no sources there), h rows clamped
  float G[3][V], Hh[3][V], NG[V], NH[V];
  auto gload = [&](float (&d)[V], int rr) {
    if (rr >= 0 && rr < H) {
      row_load<V>(d, gp + (int64_t)rr * W);
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) d[j] = 0.f;
    }
  };
  gload(G[0], q.r0 - 1);
  gload(G[1], q.r0);
  gload(NG, q.r0 + 1);
  row_load<V>(Hh[0], hp + (int64_t)clampi(q.r0 - 1, 0, H - 1) * W);
  row_load<V>(Hh[1], hp + (int64_t)q.r0 * W);
  row_load<V>(NH, hp + (int64_t)clampi(q.r0 + 1, 0, H - 1) * W);
  for (int r = q.r0; r < q.r1; ++r) {
#pragma unroll
    for (int j = 0; j < V; ++j) { G[2][j] = NG[j]; Hh[2][j] = NH[j]; }
    gload(NG, r + 2);
    row_load<V>(NH, hp + (int64_t)clampi(r + 2, 0, H - 1) * W);
    // row adjoint: tap row dy (0: -1, 1: 0, 2: +1) reads g at row r - (dy - 1)
    float A[3][V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      A[0][j] = r == 0 ? G[2][j] + G[1][j] : G[2][j];        // dy = -1: sources r + 1, and r at the top
      A[1][j] = G[1][j];
      A[2][j] = r == H - 1 ? G[0][j] + G[1][j] : G[0][j];    // dy = +1: sources r - 1, and r at the bottom
    }
    float o[V];
#pragma unroll
    for (int j = 0; j < V; ++j) o[j] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float pv = dpp_prev(A[dy][V - 1]), nx = dpp_next(A[dy][0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int col = q.c0 + j;
        const float a = A[dy][j];
        const float al = j > 0 ? A[dy][j - 1] : pv;      // column c - 1 (0 left of the image)
        const float ar = j < V - 1 ? A[dy][j + 1] : nx;  // column c + 1
        const float sm = col + 1 < W ? (col == 0 ? ar + a : ar) : (col == 0 ? a : 0.f);   // dx = -1
        const float sp = col >= 1 ? (col == W - 1 ? al + a : al) : (col == W - 1 ? a : 0.f);  // dx = +1
        o[j] += wt[dy * 3 + 0] * sm;
        o[j] += wt[dy * 3 + 1] * a;
        o[j] += wt[dy * 3 + 2] * sp;
      }
    }
    if (q.on) row_store<V>(ghp + (int64_t)r * W, o);
    // weight gradient: g(r, c) h(clamp(r + dy), clamp(c + dx))
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float pv = dpp_prev(Hh[dy][V - 1]), nx = dpp_next(Hh[dy][0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int col = q.c0 + j;
        const float gv = q.on ? G[1][j] : 0.f;
        const float l = col > 0 ? (j > 0 ? Hh[dy][j - 1] : pv) : Hh[dy][j];
        const float rr = col < W - 1 ? (j < V - 1 ? Hh[dy][j + 1] : nx) : Hh[dy][j];
        acc[dy * 3 + 0] += gv * l;
        acc[dy * 3 + 1] += gv * Hh[dy][j];
        acc[dy * 3 + 2] += gv * rr;
      }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
      G[0][j] = G[1][j]; G[1][j] = G[2][j];
      Hh[0][j] = Hh[1][j]; Hh[1][j] = Hh[2][j];
    }
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const float s = wave_sum(acc[t]);
    if (q.lane == 0) red_put(gw, q.c * 9 + t, q.slot, s);
  }
}

// one depthwise output row from input rows r-1, r, r+1 (R[0..2], replicate-clamped by the
// caller): the expressions and order of dw3_row_fwd_kernel
// ZERO (the window models' FeedForward, nn.Conv2d padding=1): zero padding instead of replicate -- the
// caller passes zero rows above / below the image, the column neighbours past the edges are 0
template <int V, bool ZERO = false>
__device__ __forceinline__ void dw3_row_out(const float (&R0)[V], const float (&R1)[V], const float (&R2)[V],
                                            const float (&wt)[9], int c0, int W, float (&o)[V]) {
  const float* Rs[3] = {R0, R1, R2};
#pragma unroll
  for (int k = 0; k < V; ++k) o[k] = 0.f;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const float* R = Rs[dy];
    const float pv = dpp_prev(R[V - 1]), nx = dpp_next(R[0]);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const int col = c0 + k;
      const float l = col > 0 ? (k > 0 ? R[k - 1] : pv) : (ZERO ? 0.f : R[k]);
      const float rr = col < W - 1 ? (k < V - 1 ? R[k + 1] : nx) : (ZERO ? 0.f : R[k]);
      o[k] += wt[dy * 3 + 0] * l;
      o[k] += wt[dy * 3 + 1] * R[k];
      o[k] += wt[dy * 3 + 2] * rr;
    }
  }
}

// row rr of a plane (replicate: clamped; ZERO: zeros outside the image)
template <int V, bool ZERO>
__device__ __forceinline__ void row_load_pad(float (&d)[V], const float* base, int rr, int H, int W) {
  if (ZERO && (rr < 0 || rr >= H)) {
#pragma unroll
    for (int k = 0; k < V; ++k) d[k] = 0.f;
  } else {
    row_load<V>(d, base + (int64_t)clampi(rr, 0, H - 1) * W);
  }
}

// the gate and its derivative: FFN (REF7:42-46) gelu(m) v with the exact erf gelu; else (REF:934-947)
// sigmoid(m) m v.  gate_d returns d gate / dm (per unit v) and the gate factor f with gate = f v.
template <bool FFN>
__device__ __forceinline__ float gate_f(float m) {
  if constexpr (FFN) return m * 0.5f * (1.0f + erff(m * 0.70710678118654752440f));
  const float sg = 1.0f / (1.0f + expf(-m));
  return sg * m;
}
template <bool FFN>
__device__ __forceinline__ void gate_d(float m, float& f, float& df) {
  if constexpr (FFN) {   // torch's gelu backward: cdf + x pdf
    const float cdf = 0.5f * (1.0f + erff(m * 0.70710678118654752440f));
    const float pdf = expf(-0.5f * m * m) * 0.39894228040143267794f;
    f = m * cdf;
    df = cdf + m * pdf;
  } else {
    const float sg = 1.0f / (1.0f + expf(-m));
    f = sg * m;
    df = sg + m * sg * (1.0f - sg);
  }
}

// depthwise 3x3 + gate in one row pass: gate = sigmoid(m) m v of (m, v) = dw3(hh)[j], [hid + j];
// one wave = one channel pair of one image and a segment of rows (the depthwise output is not
// written: the reverse recomputes it from hh)
template <int V, bool FFN>
__global__ __launch_bounds__(NT) void dw3_gate_row_fwd_kernel(const float* __restrict__ hh,
                                                              const float* __restrict__ wdw, float* __restrict__ gate,
                                                              int hid, int H, int W, int sseg, int nsegs,
                                                              uint32_t nwaves) {
  Dw3RowGeom q;
  if (!dw3_row_geom<V>(q, hid, H, W, sseg, nsegs, nwaves)) return;
  const int64_t HW = (int64_t)H * W;
  const int64_t bq = q.plane / hid, j = q.c;
  const int64_t pm = (bq * 2 * hid + j) * HW + q.cl0, pv = pm + (int64_t)hid * HW;
  const float* hmp = hh + pm;
  const float* hvp = hh + pv;
  float* gp = gate + q.plane * HW + q.cl0;
  float wm[9], wv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    wm[t] = wdw[j * 9 + t];
    wv[t] = wdw[(hid + j) * 9 + t];
  }
  float Rm[3][V], Rv[3][V], Nm[V], Nv[V];
  row_load_pad<V, FFN>(Rm[0], hmp, q.r0 - 1, H, W);
  row_load_pad<V, FFN>(Rv[0], hvp, q.r0 - 1, H, W);
  row_load<V>(Rm[1], hmp + (int64_t)q.r0 * W);
  row_load<V>(Rv[1], hvp + (int64_t)q.r0 * W);
  row_load_pad<V, FFN>(Nm, hmp, q.r0 + 1, H, W);
  row_load_pad<V, FFN>(Nv, hvp, q.r0 + 1, H, W);
  for (int r = q.r0; r < q.r1; ++r) {
#pragma unroll
    for (int k = 0; k < V; ++k) { Rm[2][k] = Nm[k]; Rv[2][k] = Nv[k]; }
    row_load_pad<V, FFN>(Nm, hmp, r + 2, H, W);
    row_load_pad<V, FFN>(Nv, hvp, r + 2, H, W);
    float m[V], v[V], o[V];
    dw3_row_out<V, FFN>(Rm[0], Rm[1], Rm[2], wm, q.c0, W, m);
    dw3_row_out<V, FFN>(Rv[0], Rv[1], Rv[2], wv, q.c0, W, v);
#pragma unroll
    for (int k = 0; k < V; ++k) o[k] = gate_f<FFN>(m[k]) * v[k];
    if (q.on) row_store<V>(gp + (int64_t)r * W, o);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      Rm[0][k] = Rm[1][k]; Rm[1][k] = Rm[2][k];
      Rv[0][k] = Rv[1][k]; Rv[1][k] = Rv[2][k];
    }
  }
}

// The gate's reverse and the depthwise reverse in one row pass (LocalNonLinearBlock reverse,
// REF:934-947): one wave = one hidden channel pair (mask plane j, value plane hid + j) of one
// image and a segment of rows.  The ghp rows are formed in registers from hp = [m; v] and
// gq = W2^T gout as the rows arrive (ghp_m = s gq v (sg + m sg (1 - sg)), ghp_v = s gq sg m,
// sg = sigmoid(m)), so ghp never reaches HBM; <gq, gate> is accumulated for the skip weight
// (rows of the wave's own segment only); then, per plane, the depthwise data adjoint and weight
// gradient of dw3_row_bwd_kernel with the same expressions.
template <int V, bool REC, bool FFN = false>
__global__ __launch_bounds__(NT) void dw3_gate_row_bwd_kernel(
    const float* hp, const float* __restrict__ gq, const float* __restrict__ scale,
    const float* __restrict__ hh, const float* __restrict__ wdw, float* __restrict__ gh, Red gw,
    Red gdot, int hid, int H, int W, int sseg, int nsegs, uint32_t nwaves) {
  Dw3RowGeom q;
  if (!dw3_row_geom<V>(q, hid, H, W, sseg, nsegs, nwaves)) return;   // q.plane = b hid + j, q.c = j
  const int64_t HW = (int64_t)H * W;
  const int64_t bq = q.plane / hid, j = q.c;
  const int64_t pm = (bq * 2 * hid + j) * HW + q.cl0, pv = pm + (int64_t)hid * HW;
  const float* mp = hp ? hp + pm : nullptr;
  const float* vp = hp ? hp + pv : nullptr;
  const float* qp = gq + q.plane * HW + q.cl0;
  const float* hmp = hh + pm;
  const float* hvp = hh + pv;
  const float s = scale[0];
  float wm[9], wv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    wm[t] = wdw[j * 9 + t];
    wv[t] = wdw[(hid + j) * 9 + t];
  }
  float accm[9], accv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) accm[t] = accv[t] = 0.f;
  float dot = 0.f;
  // ghp rows r-1, r, r+1 of both planes (zero outside the image), hh rows clamped
  float Gm[3][V], Gv[3][V], Hm[3][V], Hv[3][V];
  float NM[V], NV[V], NQ[V], NHm[V], NHv[V];
  // hp == nullptr: the depthwise output rows are recomputed from hh rows (ring X*: rows
  // rr-1, rr, rr+1 of the row rr being formed), so hp never has to be stored
  constexpr bool rec = REC;   // hp not given
  float Xm[3][V], Xv[3][V];
  if constexpr (REC) {
#pragma unroll
    for (int k = 0; k < V; ++k) Xm[0][k] = Xv[0][k] = Xm[1][k] = Xv[1][k] = 0.f;
  }
  int xrow = INT32_MIN;   // hh row held in X*[2] (rows xrow-2, xrow-1, xrow in X*[0..2])
  auto raw_load = [&](int rr) {   // operands of ghp row rr (clamped; rows outside give ghp 0)
    const int64_t o = (int64_t)clampi(rr, 0, H - 1) * W;
    row_load<V>(NQ, qp + o);
    if constexpr (!REC) {
      row_load<V>(NM, mp + o);
      row_load<V>(NV, vp + o);
      return;
    }
    // hh rows up to rr + 1 into the ring (rows are consecutive after the first call)
    const int want = rr + 1;
    if (xrow == INT32_MIN) {
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        row_load_pad<V, FFN>(Xm[d], hmp, want - 2 + d, H, W);
        row_load_pad<V, FFN>(Xv[d], hvp, want - 2 + d, H, W);
      }
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) {
        Xm[0][k] = Xm[1][k]; Xm[1][k] = Xm[2][k];
        Xv[0][k] = Xv[1][k]; Xv[1][k] = Xv[2][k];
      }
      row_load_pad<V, FFN>(Xm[2], hmp, want, H, W);
      row_load_pad<V, FFN>(Xv[2], hvp, want, H, W);
    }
    xrow = want;
    dw3_row_out<V, FFN>(Xm[0], Xm[1], Xm[2], wm, q.c0, W, NM);
    dw3_row_out<V, FFN>(Xv[0], Xv[1], Xv[2], wv, q.c0, W, NV);
  };
  auto ghp_row = [&](int rr, float (&dm)[V], float (&dv)[V]) {
    const bool in = rr >= 0 && rr < H;
    const bool own = q.on && rr >= q.r0 && rr < q.r1;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float m = NM[k], v = NV[k], g = NQ[k];
      float gf, dgf;
      gate_d<FFN>(m, gf, dgf);
      if (own) dot += g * (gf * v);
      const float gg = s * g;
      dm[k] = in ? gg * v * dgf : 0.f;
      dv[k] = in ? gg * gf : 0.f;
    }
  };
  raw_load(q.r0 - 1);
  ghp_row(q.r0 - 1, Gm[0], Gv[0]);
  raw_load(q.r0);
  ghp_row(q.r0, Gm[1], Gv[1]);
  raw_load(q.r0 + 1);
  row_load_pad<V, FFN>(Hm[0], hmp, q.r0 - 1, H, W);
  row_load_pad<V, FFN>(Hv[0], hvp, q.r0 - 1, H, W);
  row_load<V>(Hm[1], hmp + (int64_t)q.r0 * W);
  row_load<V>(Hv[1], hvp + (int64_t)q.r0 * W);
  row_load_pad<V, FFN>(NHm, hmp, q.r0 + 1, H, W);
  row_load_pad<V, FFN>(NHv, hvp, q.r0 + 1, H, W);
  // one plane's data adjoint (row r) and weight-gradient contribution
  auto plane = [&](const float (&G)[3][V], const float (&Hp)[3][V], const float (&wt)[9], float (&acc)[9], int r,
                   float* dst) {
    float A[3][V];
#pragma unroll
    for (int k = 0; k < V; ++k) {   // zero padding: no folding of the clamped edge rows
      A[0][k] = (!FFN && r == 0) ? G[2][k] + G[1][k] : G[2][k];
      A[1][k] = G[1][k];
      A[2][k] = (!FFN && r == H - 1) ? G[0][k] + G[1][k] : G[0][k];
    }
    float o[V];
#pragma unroll
    for (int k = 0; k < V; ++k) o[k] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float pvv = dpp_prev(A[dy][V - 1]), nx = dpp_next(A[dy][0]);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const int col = q.c0 + k;
        const float a = A[dy][k];
        const float al = k > 0 ? A[dy][k - 1] : pvv;
        const float ar = k < V - 1 ? A[dy][k + 1] : nx;
        const float sm = FFN ? (col + 1 < W ? ar : 0.f) : (col + 1 < W ? (col == 0 ? ar + a : ar) : (col == 0 ? a : 0.f));
        const float sp = FFN ? (col >= 1 ? al : 0.f) : (col >= 1 ? (col == W - 1 ? al + a : al) : (col == W - 1 ? a : 0.f));
        o[k] += wt[dy * 3 + 0] * sm;
        o[k] += wt[dy * 3 + 1] * a;
        o[k] += wt[dy * 3 + 2] * sp;
      }
    }
    if (q.on) row_store<V>(dst + (int64_t)r * W, o);
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float pvv = dpp_prev(Hp[dy][V - 1]), nx = dpp_next(Hp[dy][0]);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const int col = q.c0 + k;
        const float gv = q.on ? G[1][k] : 0.f;
        const float l = col > 0 ? (k > 0 ? Hp[dy][k - 1] : pvv) : (FFN ? 0.f : Hp[dy][k]);
        const float rr = col < W - 1 ? (k < V - 1 ? Hp[dy][k + 1] : nx) : (FFN ? 0.f : Hp[dy][k]);
        acc[dy * 3 + 0] += gv * l;
        acc[dy * 3 + 1] += gv * Hp[dy][k];
        acc[dy * 3 + 2] += gv * rr;
      }
    }
  };
  float* const ghm = gh + pm;
  float* const ghv = gh + pv;
  for (int r = q.r0; r < q.r1; ++r) {
    ghp_row(r + 1, Gm[2], Gv[2]);
#pragma unroll
    for (int k = 0; k < V; ++k) { Hm[2][k] = NHm[k]; Hv[2][k] = NHv[k]; }
    raw_load(r + 2);
    row_load_pad<V, FFN>(NHm, hmp, r + 2, H, W);
    row_load_pad<V, FFN>(NHv, hvp, r + 2, H, W);
    plane(Gm, Hm, wm, accm, r, ghm);
    plane(Gv, Hv, wv, accv, r, ghv);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      Gm[0][k] = Gm[1][k]; Gm[1][k] = Gm[2][k];
      Gv[0][k] = Gv[1][k]; Gv[1][k] = Gv[2][k];
      Hm[0][k] = Hm[1][k]; Hm[1][k] = Hm[2][k];
      Hv[0][k] = Hv[1][k]; Hv[1][k] = Hv[2][k];
    }
  }
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const float a = wave_sum(accm[t]), b = wave_sum(accv[t]);
    if (q.lane == 0) {
      red_put(gw, (int)j * 9 + t, q.slot, a);
      red_put(gw, (hid + (int)j) * 9 + t, q.slot, b);
    }
  }
  const float d = wave_sum(dot);
  if (q.lane == 0) red_put(gdot, 0, q.wid, d);
}

// The same reverse (recomputing the depthwise output from hh, the training path) with its operand rows
// through a per-wave LDS ring (round 5): each wave DMAs the rows of iteration r + 3 -- gq row r + 4 and the
// two hh rows r + 5 -- into slot (r + 3) mod 4 of its own ring (16-byte LDS-DMA, one scalar base per row,
// a loop-invariant lane offset; lanes >= 16 V idle at V < 4) and waits with a counted vmcnt, so no load
// latency sits on the row loop (the register kernel loaded its hh rows and used them at once: 0.34 of HBM
// at C4).  The hh rows of the window (r - 1 .. r + 2) serve both the recomputed depthwise output and the
// weight gradient (the register kernel loaded them twice).  Same expressions and order as
// dw3_gate_row_bwd_kernel<V, true>: the outputs agree to fp32 contraction, the reductions bitwise.
constexpr int DW3R_D = 4;   // ring slots (DMAs DW3R_D - 1 iterations ahead)
// ring slots per V: three at V = 8 (2-KB rows: 72 KB per 4-wave workgroup, two workgroups per CU)
__host__ __device__ constexpr int dw3_ring_depth(int V) { return V == 8 ? 3 : DW3R_D; }
// grr_lnb_set_bwd_ring: 1 (default) the ring kernel where it applies (W % 4 == 0, 16-byte aligned planes),
// 0 the register kernel (A/B and tests)
int g_dw3_bwd_ring = 1;
#define HW_ALIGNED(H, W) (((int64_t)(H) * (W)) % 4 == 0)
__device__ __forceinline__ void dma_row16s(const float* sbase, uint32_t voff, float* lds_dst) {
  const uint32_t m0v = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds_dst;
  asm volatile("global_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "{m0}"(__builtin_amdgcn_readfirstlane(m0v))
               : "memory");
}
// a wave-uniform pointer the compiler cannot prove uniform (derived from threadIdx.x >> 6) into SGPRs
__device__ __forceinline__ const float* uniform_ptr(const float* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const float*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
// DMA geometry of a ring row (shared by the kernel and the host replay grr_dw3_ring_check): a ring row holds
// RW = 64 V floats; one global_load_lds_dwordx4 moves 16 bytes per lane into consecutive LDS, so a row takes
// NDMA instructions of LANES lanes, DMA d lane l writing row bytes [16 (d LANES + l), + 16) from image column
// x0 + 4 (d LANES + l), clamped into [0, W - 4].  The invariants (static_assert below, replayed on the host
// over every strip of a launch): every DMA byte lands inside its ring row, every source lies inside its image
// row.  Round 5's fault (r05v8: hipErrorIllegalAddress in test_gate_dw3_rows_vs_autograd[b2hid3h9w32-lnb], the
// V = 1 instance, right after a change that let the issue path run two DMAs per ring row for an 8-column
// lane) is the violation of both at V < 4: one 1-KB DMA already covers 4 V rows' worth of lanes' data at V = 1,
// so a second DMA per row (or all 64 lanes in the first) writes past the 256-B ring row into the next slot --
// for the last wave's last slot past the workgroup's LDS -- and reads 1 KB past the image row, off the end of
// the tensor at its last row (the test's 9 x 32 planes end 1 KB before the next page boundary only by chance).
// The faulting diff was not kept; this reconstruction rests on the arithmetic above, which the replay checks.
template <int V>
struct Dw3RingGeom {
  static constexpr int RW = 64 * V;
  static constexpr int NDMA = (RW * 4 + 1023) / 1024;
  static constexpr int LANES = RW / 4 / NDMA;
  static_assert(NDMA * LANES * 16 == RW * 4 && LANES <= 64, "ring row DMAs must tile the row exactly");
};
__host__ __device__ inline int dw3_ring_src_col(int x0, int dl, int W) {   // dl = d LANES + l
  const int c = x0 + 4 * dl;
  return c < W - 4 ? c : W - 4;
}

template <int V>
__global__ __launch_bounds__(NT) void dw3_gate_row_bwd_ring_kernel(
    const float* __restrict__ gq, const float* __restrict__ scale, const float* __restrict__ hh,
    const float* __restrict__ wdw, float* __restrict__ gh, Red gw, Red gdot, int hid, int H, int W, int sseg,
    int nsegs, uint32_t nwaves) {
  extern __shared__ __attribute__((aligned(16))) float dw3_ring[];
  Dw3RowGeom q;
  if (!dw3_row_geom<V>(q, hid, H, W, sseg, nsegs, nwaves)) return;   // q.plane = b hid + j, q.c = j
  constexpr int RW = 64 * V;                                          // floats per ring row
  constexpr int D = dw3_ring_depth(V);                                // ring slots
  float* const ring = dw3_ring + (threadIdx.x >> 6) * (D * 3 * RW);
  const int64_t HW = (int64_t)H * W;
  const int64_t bq = q.plane / hid, j = q.c;
  const int64_t pm0 = (bq * 2 * hid + j) * HW, pv0 = pm0 + (int64_t)hid * HW;
  const float* const gq0 = gq + (int64_t)q.plane * HW;   // plane bases (wave-uniform; SGPRs at the DMA)
  const float* const hm0 = hh + pm0;
  const float* const hv0 = hh + pv0;
  // DMA d of a ring row, lane l: the 16-byte chunk d LANES + l, the strip's columns x0 + 4 (d LANES + l)
  // (Dw3RingGeom; W % 4 == 0): one DMA per row at V <= 4, two at V = 8
  typedef Dw3RingGeom<V> RG;
  static_assert(RG::RW == RW, "ring row size");
  const int x0 = q.c0 - V * q.lane;
  const uint32_t voff = (uint32_t)dw3_ring_src_col(x0, q.lane, W) * 4u;                    // DMA 0
  const uint32_t voff1 = (uint32_t)dw3_ring_src_col(x0, RG::LANES + q.lane, W) * 4u;      // DMA 1 (V = 8)
  const bool dma_lane = q.lane < RG::LANES;
  auto issue = [&](int r, int sl) {   // rows of iteration r: gq row r + 1, hh rows r + 2
    if (dma_lane) {
      float* dst = ring + sl * (3 * RW);
      dma_row16s(uniform_ptr(gq0 + (int64_t)clampi(r + 1, 0, H - 1) * W), voff, dst);
      dma_row16s(uniform_ptr(hm0 + (int64_t)clampi(r + 2, 0, H - 1) * W), voff, dst + RW);
      dma_row16s(uniform_ptr(hv0 + (int64_t)clampi(r + 2, 0, H - 1) * W), voff, dst + 2 * RW);
      if constexpr (RG::NDMA == 2) {   // the second KB of each 2-KB row
        dma_row16s(uniform_ptr(gq0 + (int64_t)clampi(r + 1, 0, H - 1) * W), voff1, dst + RG::LANES * 4);
        dma_row16s(uniform_ptr(hm0 + (int64_t)clampi(r + 2, 0, H - 1) * W), voff1, dst + RW + RG::LANES * 4);
        dma_row16s(uniform_ptr(hv0 + (int64_t)clampi(r + 2, 0, H - 1) * W), voff1, dst + 2 * RW + RG::LANES * 4);
      }
    }
  };
  static_assert(RG::NDMA <= 2, "ring kernel issue path: one or two DMAs per ring row");
  // the first D - 1 iterations' rows
#pragma unroll
  for (int k = 0; k < D - 1; ++k) issue(q.r0 + k, k);
  const float s = scale[0];
  float wm[9], wv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    wm[t] = wdw[j * 9 + t];
    wv[t] = wdw[(hid + j) * 9 + t];
  }
  float accm[9], accv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) accm[t] = accv[t] = 0.f;
  float dot = 0.f;
  const float* const qp = gq0 + q.cl0;
  const float* const hmp = hm0 + q.cl0;
  const float* const hvp = hv0 + q.cl0;
  // windows: hh rows r-1 .. r+2 (Hm / Hv[0..3]), ghp rows r-1 .. r+1 (Gm / Gv[0..2])
  float Hm[4][V], Hv[4][V], Gm[3][V], Gv[3][V];
  auto ghp_row = [&](int rr, const float (&g)[V], const float (&R0m)[V], const float (&R1m)[V], const float (&R2m)[V],
                     const float (&R0v)[V], const float (&R1v)[V], const float (&R2v)[V], float (&dm)[V],
                     float (&dv)[V]) {
    float NM[V], NV[V];
    dw3_row_out<V, false>(R0m, R1m, R2m, wm, q.c0, W, NM);
    dw3_row_out<V, false>(R0v, R1v, R2v, wv, q.c0, W, NV);
    const bool in = rr >= 0 && rr < H;
    const bool own = q.on && rr >= q.r0 && rr < q.r1;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float m = NM[k], v = NV[k], gg0 = g[k];
      float gf, dgf;
      gate_d<false>(m, gf, dgf);
      if (own) dot += gg0 * (gf * v);
      const float gg = s * gg0;
      dm[k] = in ? gg * v * dgf : 0.f;
      dv[k] = in ? gg * gf : 0.f;
    }
  };
  {   // prologue: hh rows r0-2 .. r0+1 and gq rows r0-1, r0 by plain loads; ghp rows r0-1, r0
    float X0m[V], X0v[V], g0[V], g1[V];
    row_load_pad<V, false>(X0m, hmp, q.r0 - 2, H, W);
    row_load_pad<V, false>(X0v, hvp, q.r0 - 2, H, W);
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      row_load_pad<V, false>(Hm[d], hmp, q.r0 - 1 + d, H, W);
      row_load_pad<V, false>(Hv[d], hvp, q.r0 - 1 + d, H, W);
    }
    row_load_pad<V, false>(g0, qp, q.r0 - 1, H, W);
    row_load_pad<V, false>(g1, qp, q.r0, H, W);
    ghp_row(q.r0 - 1, g0, X0m, Hm[0], Hm[1], X0v, Hv[0], Hv[1], Gm[0], Gv[0]);
    ghp_row(q.r0, g1, Hm[0], Hm[1], Hm[2], Hv[0], Hv[1], Hv[2], Gm[1], Gv[1]);
  }
  // one plane's data adjoint (row r) and weight-gradient contribution: dw3_gate_row_bwd_kernel's
  auto plane = [&](const float (&G)[3][V], const float (&Hp0)[V], const float (&Hp1)[V], const float (&Hp2)[V],
                   const float (&wt)[9], float (&acc)[9], int r, float* dst) {
    const float* Hp[3] = {Hp0, Hp1, Hp2};
    float A[3][V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
      A[0][k] = r == 0 ? G[2][k] + G[1][k] : G[2][k];
      A[1][k] = G[1][k];
      A[2][k] = r == H - 1 ? G[0][k] + G[1][k] : G[0][k];
    }
    float o[V];
#pragma unroll
    for (int k = 0; k < V; ++k) o[k] = 0.f;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float pvv = dpp_prev(A[dy][V - 1]), nx = dpp_next(A[dy][0]);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const int col = q.c0 + k;
        const float a = A[dy][k];
        const float al = k > 0 ? A[dy][k - 1] : pvv;
        const float ar = k < V - 1 ? A[dy][k + 1] : nx;
        const float sm = col + 1 < W ? (col == 0 ? ar + a : ar) : (col == 0 ? a : 0.f);
        const float sp = col >= 1 ? (col == W - 1 ? al + a : al) : (col == W - 1 ? a : 0.f);
        o[k] += wt[dy * 3 + 0] * sm;
        o[k] += wt[dy * 3 + 1] * a;
        o[k] += wt[dy * 3 + 2] * sp;
      }
    }
    if (q.on) row_store<V>(dst + (int64_t)r * W, o);
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float* Hd = Hp[dy];
      const float pvv = dpp_prev(Hd[V - 1]), nx = dpp_next(Hd[0]);
#pragma unroll
      for (int k = 0; k < V; ++k) {
        const int col = q.c0 + k;
        const float gv = q.on ? G[1][k] : 0.f;
        const float l = col > 0 ? (k > 0 ? Hd[k - 1] : pvv) : Hd[k];
        const float rr = col < W - 1 ? (k < V - 1 ? Hd[k + 1] : nx) : Hd[k];
        acc[dy * 3 + 0] += gv * l;
        acc[dy * 3 + 1] += gv * Hd[k];
        acc[dy * 3 + 2] += gv * rr;
      }
    }
  };
  float* const ghm = gh + pm0 + q.cl0;
  float* const ghv = gh + pv0 + q.cl0;
  int sl = 0;
  for (int r = q.r0; r < q.r1; ++r) {
    // iteration r's rows landed: after them the wave issued the next D - 2 iterations' DMAs (3 NDMA each)
    // and its own stores (vmcnt counts those too: the wait is conservative)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * RG::NDMA * (D - 2)) : "memory");
    const float* slot = ring + sl * (3 * RW) + V * q.lane;
    float g2[V];
    row_load<V>(g2, slot);                  // gq row r + 1
    row_load<V>(Hm[3], slot + RW);          // hh rows r + 2
    row_load<V>(Hv[3], slot + 2 * RW);
    ghp_row(r + 1, g2, Hm[1], Hm[2], Hm[3], Hv[1], Hv[2], Hv[3], Gm[2], Gv[2]);
    plane(Gm, Hm[0], Hm[1], Hm[2], wm, accm, r, ghm);
    plane(Gv, Hv[0], Hv[1], Hv[2], wv, accv, r, ghv);
    issue(r + D - 1, sl == 0 ? D - 1 : sl - 1);   // the slot iteration r - 1 read
    sl = sl == D - 1 ? 0 : sl + 1;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      Gm[0][k] = Gm[1][k]; Gm[1][k] = Gm[2][k];
      Gv[0][k] = Gv[1][k]; Gv[1][k] = Gv[2][k];
      Hm[0][k] = Hm[1][k]; Hm[1][k] = Hm[2][k]; Hm[2][k] = Hm[3][k];
      Hv[0][k] = Hv[1][k]; Hv[1][k] = Hv[2][k]; Hv[2][k] = Hv[3][k];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA in flight into LDS at the wave's end
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const float a = wave_sum(accm[t]), b = wave_sum(accv[t]);
    if (q.lane == 0) {
      red_put(gw, (int)j * 9 + t, q.slot, a);
      red_put(gw, (hid + (int)j) * 9 + t, q.slot, b);
    }
  }
  const float d = wave_sum(dot);
  if (q.lane == 0) red_put(gdot, 0, q.wid, d);
}

// V for the row kernels (0: not applicable -> per-pixel kernels)
// W > 256: column strips of 4-wide lanes with a V-column halo (the fused gate + depthwise reverse reaches
// two columns: V >= 2)
int dw3_row_vec(int W) {
  if (W <= 64) return 1;
  if (W <= 128 && W % 2 == 0) return 2;
  if (W % 4 == 0) return 4;
  return 0;
}
// the ring kernel's one-strip instance: 256 < W <= 512, W % 8 == 0 -- 8 columns per lane cover the row, no halo
// columns (round 5's V = 4 strips read 1.5x the columns at W = 512)
#ifndef GRR_DW3_V8
#define GRR_DW3_V8 1   // 32 x 512^2: hid 96 5.61 -> 4.58 ms, hid 192 11.16 -> 9.03 ms per launch (scripts/gpu_r06_u.sh)
#endif
bool dw3_ring_v8_shape(int W) { return W > 256 && W <= 512 && W % 8 == 0; }
bool dw3_ring_v8(int W) { return GRR_DW3_V8 && dw3_ring_v8_shape(W); }
// rows per wave: whole planes while the grid has >= 4096 waves, else segments of >= 32 rows
int dw3_row_seg(int H, int64_t planes) {
  static const int64_t min_waves = [] {   // GRR_DW3_MIN_WAVES / GRR_DW3_MAX_SEG: A/B of the segment split
    const char* e = getenv("GRR_DW3_MIN_WAVES");
    return e ? (int64_t)atoll(e) : (int64_t)4096;
  }();
  static const int max_seg = [] {
    const char* e = getenv("GRR_DW3_MAX_SEG");
    return e ? atoi(e) : (1 << 30);
  }();
  int sseg = H;
  while (sseg > 32 && (planes * ((H + sseg - 1) / sseg) < min_waves || sseg > max_seg)) sseg = (sseg + 1) / 2;
  return sseg;
}
// Host replay of the ring kernel's DMA geometry for a launch shape (Dw3RingGeom, dw3_row_geom's strips):
// 0 when every DMA of every strip lands inside its ring row and reads inside its image row, else the first
// violation as GRR_ERR_SHAPE.  Cheap integer arithmetic; tests/test_abi.py runs it over the test shapes.
template <int V>
static grr_status dw3_ring_replay(int W) {
  typedef Dw3RingGeom<V> RG;
  const int nstrips = dw3_row_strips(W, V), step = 62 * V;
  for (int strip = 0; strip < nstrips; ++strip) {
    const int x0 = strip == 0 ? 0 : strip * step - V;
    for (int d = 0; d < RG::NDMA; ++d)
      for (int l = 0; l < RG::LANES; ++l) {
        const int dl = d * RG::LANES + l, lds_end = 16 * (dl + 1), c = dw3_ring_src_col(x0, dl, W);
        GRR_REQUIRE(lds_end <= RG::RW * 4, GRR_ERR_SHAPE, "dw3 ring: V=%d W=%d strip %d DMA %d lane %d writes byte %d of a %d-byte ring row",
                    V, W, strip, d, l, lds_end, RG::RW * 4);
        GRR_REQUIRE(c >= 0 && c + 4 <= W, GRR_ERR_SHAPE, "dw3 ring: V=%d W=%d strip %d DMA %d lane %d reads columns %d..%d",
                    V, W, strip, d, l, c, c + 3);
      }
  }
  return GRR_OK;
}

template <int V>
grr_status launch_dw3_row(bool bwd, const float* g, const float* h, const float* wdw, float* out, float* gwd, int B,
                          int C, int H, int W, hipStream_t s, const char* what) {
  const int nstrips = dw3_row_strips(W, V);
  const int64_t planes = (int64_t)B * C * nstrips;   // (plane, strip) pairs
  const int sseg = dw3_row_seg(H, planes), nsegs = (H + sseg - 1) / sseg;
  const uint32_t nwaves = (uint32_t)(planes * nsegs);
  const dim3 grid((nwaves + NT / 64 - 1) / (NT / 64));
  if (!bwd) {
    hipLaunchKernelGGL(dw3_row_fwd_kernel<V>, grid, dim3(NT), 0, s, h, wdw, out, C, H, W, sseg, nsegs, nwaves);
    return launch_status(what);
  }
  RedScratch rs(s);
  const int iw = rs.plan(gwd, C * 9, (uint32_t)((int64_t)B * nsegs * nstrips));
  grr_status st = rs.alloc(what);
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(dw3_row_bwd_kernel<V>, grid, dim3(NT), 0, s, g, h, wdw, out, rs.red(iw), C, H, W, sseg, nsegs,
                     nwaves);
  st = launch_status(what);
  return st != GRR_OK ? st : rs.finish(what);
}
bool dw3_row_ok(const float* g, const float* h, const float* out, int B, int C, int H, int W) {
  const int V = dw3_row_vec(W);
  if (V == 0) return false;
  // vector row loads: plane bases aligned to 4 V bytes
  const void* ptrs[] = {g, h, out};
  for (const void* p : ptrs)
    if (p && (uintptr_t)p % (4u * V) != 0) return false;
  return (int64_t)B * C * dw3_row_strips(W, V) * ((H + 31) / 32) < (1ll << 31);
}
grr_status dw3_row(bool bwd, const float* g, const float* h, const float* wdw, float* out, float* gw, int B, int C,
                   int H, int W, hipStream_t s, const char* what) {
  switch (dw3_row_vec(W)) {
    case 1: return launch_dw3_row<1>(bwd, g, h, wdw, out, gw, B, C, H, W, s, what);
    case 2: return launch_dw3_row<2>(bwd, g, h, wdw, out, gw, B, C, H, W, s, what);
    default: return launch_dw3_row<4>(bwd, g, h, wdw, out, gw, B, C, H, W, s, what);
  }
}

template <int V, bool FFN = false>
grr_status launch_dw3_gate_row(const float* hp, const float* gq, const float* scale, const float* hh, const float* wdw,
                               float* gh, float* gwd, float* gdotd, int B, int hid, int H, int W, hipStream_t s,
                               const char* what) {
  const int nstrips = dw3_row_strips(W, V);
  const int64_t planes = (int64_t)B * hid * nstrips;   // (plane, strip) pairs
  const int sseg = dw3_row_seg(H, planes), nsegs = (H + sseg - 1) / sseg;
  const uint32_t nwaves = (uint32_t)(planes * nsegs);
  const dim3 grid((nwaves + NT / 64 - 1) / (NT / 64));
  RedScratch rs(s);
  const int iw = rs.plan(gwd, 2 * hid * 9, (uint32_t)((int64_t)B * nsegs * nstrips));
  const int id = rs.plan(gdotd, 1, nwaves);
  grr_status st = rs.alloc(what);
  if (st != GRR_OK) return st;
  const Red gw = rs.red(iw), gdot = rs.red(id);
  if constexpr (V == 8) {   // ring kernel only (grr_lnb_gate_dw3_bwd checked dw3_ring_v8)
    hipLaunchKernelGGL(dw3_gate_row_bwd_ring_kernel<8>, grid, dim3(NT),
                       (NT / 64) * dw3_ring_depth(8) * 3 * 64 * 8 * sizeof(float), s, gq, scale, hh, wdw, gh, gw, gdot,
                       hid, H, W, sseg, nsegs, nwaves);
  } else if (!FFN && !hp && g_dw3_bwd_ring && W % 4 == 0 && (uintptr_t)gq % 16 == 0 && (uintptr_t)hh % 16 == 0 &&
      HW_ALIGNED(H, W)) {
    hipLaunchKernelGGL(dw3_gate_row_bwd_ring_kernel<V>, grid, dim3(NT),
                       (NT / 64) * dw3_ring_depth(V) * 3 * 64 * V * sizeof(float), s, gq, scale, hh, wdw, gh, gw, gdot,
                       hid, H, W, sseg, nsegs, nwaves);
  } else if constexpr (FFN) {   // the FeedForward reverse always recomputes the depthwise output
    hipLaunchKernelGGL((dw3_gate_row_bwd_kernel<V, true, true>), grid, dim3(NT), 0, s, hp, gq, scale, hh, wdw, gh, gw,
                       gdot, hid, H, W, sseg, nsegs, nwaves);
  } else if (hp) {
    hipLaunchKernelGGL((dw3_gate_row_bwd_kernel<V, false>), grid, dim3(NT), 0, s, hp, gq, scale, hh, wdw, gh, gw, gdot,
                       hid, H, W, sseg, nsegs, nwaves);
  } else {
    hipLaunchKernelGGL((dw3_gate_row_bwd_kernel<V, true>), grid, dim3(NT), 0, s, hp, gq, scale, hh, wdw, gh, gw, gdot,
                       hid, H, W, sseg, nsegs, nwaves);
  }
  st = launch_status(what);
  return st != GRR_OK ? st : rs.finish(what);
}

template <int V, bool FFN = false>
void launch_dw3_gate_fwd_row(const float* hh, const float* wdw, float* gate, int B, int hid, int H, int W,
                             hipStream_t s) {
  const int64_t planes = (int64_t)B * hid * dw3_row_strips(W, V);   // (plane, strip) pairs
  const int sseg = dw3_row_seg(H, planes), nsegs = (H + sseg - 1) / sseg;
  const uint32_t nwaves = (uint32_t)(planes * nsegs);
  const dim3 grid((nwaves + NT / 64 - 1) / (NT / 64));
  hipLaunchKernelGGL((dw3_gate_row_fwd_kernel<V, FFN>), grid, dim3(NT), 0, s, hh, wdw, gate, hid, H, W, sseg, nsegs,
                     nwaves);
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
  hipLaunchKernelGGL(ln_bwd_kernel<false>, dim3(grid_for(np)), dim3(NT), 0, (hipStream_t)stream, x, ln_w, isd, gn,
                     nullptr, nullptr, gx, Red{nullptr, 0}, C, P, np);
  grr_status st = launch_status("grr_lnb_norm_bwd/data");
  if (st != GRR_OK) return st;
  const int chunks = chunks_for(P, (int64_t)B * C);
  RedScratch rs((hipStream_t)stream);
  const int iw = rs.plan(gln_w, C, (uint32_t)B * chunks);
  st = rs.alloc("grr_lnb_norm_bwd/weight");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(ln_wgrad_kernel, dim3(chunks, B * C), dim3(NT), 0, (hipStream_t)stream, gn, x, isd, rs.red(iw), C,
                     P);
  st = launch_status("grr_lnb_norm_bwd/weight");
  return st != GRR_OK ? st : rs.finish("grr_lnb_norm_bwd/weight");
}

grr_status grr_lnb_norm_bwd_skip(const float* x, const float* ln_w, const float* isd, const float* gn,
                                 const float* gout, const float* skip, float* gx, float* gln_w, float* gskip0, int B,
                                 int C, int64_t P, void* stream) {
  clear_error();
  GRR_REQUIRE(x && ln_w && isd && gn && gout && skip && gx && gln_w && gskip0 && gx != gout && B > 0 && C > 1 && P > 0,
              GRR_ERR_INVALID_ARG, "grr_lnb_norm_bwd_skip: bad args");
  GRR_REQUIRE((int64_t)B * C <= 65535, GRR_ERR_UNSUPPORTED, "grr_lnb_norm_bwd_skip: B*C > 65535");
  const int64_t np = (int64_t)B * P;
  const int grid = grid_for(np), chunks = chunks_for(P, (int64_t)B * C);
  hipStream_t s = (hipStream_t)stream;
  RedScratch rs(s);
  const int id = rs.plan(gskip0, 1, (uint32_t)grid), iw = rs.plan(gln_w, C, (uint32_t)B * chunks);
  grr_status st = rs.alloc("grr_lnb_norm_bwd_skip");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(ln_bwd_kernel<true>, dim3(grid), dim3(NT), 0, s, x, ln_w, isd, gn, gout, skip, gx, rs.red(id), C,
                     P, np);
  hipLaunchKernelGGL(ln_wgrad_kernel, dim3(chunks, B * C), dim3(NT), 0, s, gn, x, isd, rs.red(iw), C, P);
  st = launch_status("grr_lnb_norm_bwd_skip");
  return st != GRR_OK ? st : rs.finish("grr_lnb_norm_bwd_skip");
}

grr_status grr_dwconv3(const float* h, const float* wdw, float* out, int B, int C, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(h && wdw && out && B > 0 && C > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG, "grr_dwconv3: bad args");
  if (dw3_row_ok(nullptr, h, out, B, C, H, W))
    return dw3_row(false, nullptr, h, wdw, out, nullptr, B, C, H, W, (hipStream_t)stream, "grr_dwconv3");
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
  if (dw3_row_ok(g, h, gh, B, C, H, W))
    return dw3_row(true, g, h, wdw, gh, gwdw, B, C, H, W, (hipStream_t)stream, "grr_dwconv3_bwd");
  GRR_REQUIRE((int64_t)B * C <= 65535, GRR_ERR_UNSUPPORTED, "grr_dwconv3_bwd: B*C > 65535");
  hipLaunchKernelGGL(dw3_bwd_data_kernel, dim3((H * W + NT - 1) / NT, B * C), dim3(NT), 0, (hipStream_t)stream, g,
                     wdw, gh, C, H, W);
  grr_status st = launch_status("grr_dwconv3_bwd/data");
  if (st != GRR_OK) return st;
  const int chunks = chunks_for((int64_t)H * W, (int64_t)B * C);
  RedScratch rs((hipStream_t)stream);
  const int iw = rs.plan(gwdw, C * 9, (uint32_t)B * chunks);
  st = rs.alloc("grr_dwconv3_bwd/weight");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(dw3_wgrad_kernel, dim3(chunks, B * C), dim3(NT), 0, (hipStream_t)stream, g, h, rs.red(iw), C, H,
                     W);
  st = launch_status("grr_dwconv3_bwd/weight");
  return st != GRR_OK ? st : rs.finish("grr_dwconv3_bwd/weight");
}

grr_status grr_lnb_gate_bwd_scaled(const float* hp, const float* gq, const float* scale, float* ghp, float* gdot, int B,
                                   int hid, int64_t P, void* stream) {
  clear_error();
  GRR_REQUIRE(hp && gq && scale && ghp && gdot && B > 0 && hid > 0 && P > 0, GRR_ERR_INVALID_ARG,
              "grr_lnb_gate_bwd_scaled: bad args");
  const int64_t n = (int64_t)B * hid * P;
  const int grid = (int)std::min<int64_t>((n + NT - 1) / NT, 4096);
  RedScratch rs((hipStream_t)stream);
  const int id = rs.plan(gdot, 1, (uint32_t)grid);
  grr_status st = rs.alloc("grr_lnb_gate_bwd_scaled");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(gate_bwd_scaled_kernel, dim3(grid), dim3(NT), 0, (hipStream_t)stream, hp, gq, scale, ghp,
                     rs.red(id), hid, P, n);
  st = launch_status("grr_lnb_gate_bwd_scaled");
  return st != GRR_OK ? st : rs.finish("grr_lnb_gate_bwd_scaled");
}

grr_status grr_lnb_dw3_gate(const float* hh, const float* wdw, float* gate, int B, int hid, int H, int W,
                            void* stream) {
  clear_error();
  GRR_REQUIRE(hh && wdw && gate && B > 0 && hid > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_lnb_dw3_gate: bad args");
  const int V = dw3_row_vec(W);
  const bool aligned = V > 0 && (uintptr_t)hh % (4u * V) == 0 && (uintptr_t)gate % (4u * V) == 0;
  GRR_REQUIRE(aligned && (int64_t)B * hid * dw3_row_strips(W, V > 0 ? V : 1) * ((H + 31) / 32) < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_lnb_dw3_gate: needs W <= 64, even W <= 128 or W %% 4 == 0, and 4V-byte aligned planes");
  hipStream_t s = (hipStream_t)stream;
  switch (V) {
    case 1: launch_dw3_gate_fwd_row<1>(hh, wdw, gate, B, hid, H, W, s); break;
    case 2: launch_dw3_gate_fwd_row<2>(hh, wdw, gate, B, hid, H, W, s); break;
    default: launch_dw3_gate_fwd_row<4>(hh, wdw, gate, B, hid, H, W, s); break;
  }
  return launch_status("grr_lnb_dw3_gate");
}

grr_status grr_dw3_ring_check(int W) {
  clear_error();
  GRR_REQUIRE(W >= 4 && W % 4 == 0, GRR_ERR_INVALID_ARG, "grr_dw3_ring_check: the ring kernel needs W %% 4 == 0");
  if (grr::dw3_ring_v8_shape(W)) {   // (checked whether or not the build launches it)
    const grr_status st = grr::dw3_ring_replay<8>(W);
    if (st != GRR_OK) return st;
  }
  switch (grr::dw3_row_vec(W)) {
    case 1: return grr::dw3_ring_replay<1>(W);
    case 2: return grr::dw3_ring_replay<2>(W);
    case 4: return grr::dw3_ring_replay<4>(W);
    default: return GRR_ERR_UNSUPPORTED;
  }
}

grr_status grr_lnb_set_bwd_ring(int enable) {
  clear_error();
  GRR_REQUIRE(enable == 0 || enable == 1, GRR_ERR_INVALID_ARG, "grr_lnb_set_bwd_ring: 0 or 1");
  g_dw3_bwd_ring = enable;
  return GRR_OK;
}

grr_status grr_lnb_gate_dw3_bwd(const float* hp, const float* gq, const float* scale, const float* hh,
                                const float* wdw, float* gh, float* gwdw, float* gdot, int B, int hid, int H, int W,
                                void* stream) {
  clear_error();
  GRR_REQUIRE(gq && scale && hh && wdw && gh && gwdw && gdot && B > 0 && hid > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_lnb_gate_dw3_bwd: bad args");
  const int V = dw3_row_vec(W);
  const void* ptrs[] = {hp, gq, hh, gh};
  bool aligned = true;
  for (const void* p : ptrs) aligned = aligned && (uintptr_t)p % (4u * (V > 0 ? V : 1)) == 0;   // NULL hp passes
  GRR_REQUIRE(V > 0 && aligned && (int64_t)B * hid * dw3_row_strips(W, V > 0 ? V : 1) * ((H + 31) / 32) < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_lnb_gate_dw3_bwd: needs W <= 64, even W <= 128 or W %% 4 == 0, and 4V-byte aligned planes");
  hipStream_t s = (hipStream_t)stream;
  const char* what = "grr_lnb_gate_dw3_bwd";
  if (!hp && g_dw3_bwd_ring && dw3_ring_v8(W) && (uintptr_t)gq % 32 == 0 && (uintptr_t)hh % 32 == 0 &&
      (uintptr_t)gh % 32 == 0)
    return launch_dw3_gate_row<8>(hp, gq, scale, hh, wdw, gh, gwdw, gdot, B, hid, H, W, s, what);
  switch (V) {
    case 1: return launch_dw3_gate_row<1>(hp, gq, scale, hh, wdw, gh, gwdw, gdot, B, hid, H, W, s, what);
    case 2: return launch_dw3_gate_row<2>(hp, gq, scale, hh, wdw, gh, gwdw, gdot, B, hid, H, W, s, what);
    default: return launch_dw3_gate_row<4>(hp, gq, scale, hh, wdw, gh, gwdw, gdot, B, hid, H, W, s, what);
  }
}

grr_status grr_ffn_dw3_gate(const float* hh, const float* wdw, float* gate, int B, int hid, int H, int W,
                            void* stream) {
  clear_error();
  GRR_REQUIRE(hh && wdw && gate && B > 0 && hid > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_ffn_dw3_gate: bad args");
  const int V = dw3_row_vec(W);
  const bool aligned = V > 0 && (uintptr_t)hh % (4u * V) == 0 && (uintptr_t)gate % (4u * V) == 0;
  GRR_REQUIRE(aligned && (int64_t)B * hid * dw3_row_strips(W, V > 0 ? V : 1) * ((H + 31) / 32) < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_ffn_dw3_gate: needs W <= 64, even W <= 128 or W %% 4 == 0, and 4V-byte aligned planes");
  hipStream_t s = (hipStream_t)stream;
  switch (V) {
    case 1: launch_dw3_gate_fwd_row<1, true>(hh, wdw, gate, B, hid, H, W, s); break;
    case 2: launch_dw3_gate_fwd_row<2, true>(hh, wdw, gate, B, hid, H, W, s); break;
    default: launch_dw3_gate_fwd_row<4, true>(hh, wdw, gate, B, hid, H, W, s); break;
  }
  return launch_status("grr_ffn_dw3_gate");
}

grr_status grr_ffn_gate_dw3_bwd(const float* gq, const float* scale, const float* hh, const float* wdw, float* gh,
                                float* gwdw, float* gdot, int B, int hid, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(gq && scale && hh && wdw && gh && gwdw && gdot && B > 0 && hid > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_ffn_gate_dw3_bwd: bad args");
  const int V = dw3_row_vec(W);
  const void* ptrs[] = {gq, hh, gh};
  bool aligned = true;
  for (const void* p : ptrs) aligned = aligned && (uintptr_t)p % (4u * (V > 0 ? V : 1)) == 0;
  GRR_REQUIRE(V > 0 && aligned && (int64_t)B * hid * dw3_row_strips(W, V > 0 ? V : 1) * ((H + 31) / 32) < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_ffn_gate_dw3_bwd: needs W <= 64, even W <= 128 or W %% 4 == 0, and 4V-byte aligned planes");
  hipStream_t s = (hipStream_t)stream;
  const char* what = "grr_ffn_gate_dw3_bwd";
  switch (V) {
    case 1: return launch_dw3_gate_row<1, true>(nullptr, gq, scale, hh, wdw, gh, gwdw, gdot, B, hid, H, W, s, what);
    case 2: return launch_dw3_gate_row<2, true>(nullptr, gq, scale, hh, wdw, gh, gwdw, gdot, B, hid, H, W, s, what);
    default: return launch_dw3_gate_row<4, true>(nullptr, gq, scale, hh, wdw, gh, gwdw, gdot, B, hid, H, W, s, what);
  }
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
