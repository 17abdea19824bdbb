// Reverse (training) kernels of the window-graph solver (REF7 = exploration/
// model_multiscale_mixture_GLR/lib/model_GLR_GTV_deep_v7.py, MixtureGTV :802-1016).
//
// The forward (window_ops.hip) applies per graph g and signal channel c
//   P   s(p) = sum_t k_t x(reflect(p + d_t))                 stats stencil, reflect frame (REF7:449-467)
//   T   y(p) = sum_t k_t v(p - d_t)  [p - d_t inside]         its conv_transpose, zero frame (:469-488)
//   GLR l(q) = s(q) - sum_e w_e(q) s(n_e(q)),  n_e(q) = clamp(q + delta_e)            (:374-398)
//   GTV o(q) = sum_e w_e(q) ph_e(q) - sum_e [q - delta_e in] w_e(q - delta_e) ph_e(q - delta_e),
//       ph_e(p) = phi(w_e(p) s(p) - w_e(p) s(n_e(p))), phi = id or 2 soft(., gamma) - .   (:536-774)
// so a term's output is scale[g] * T(l) or scale[g] * T(o).  Given the gradient g of that
// output the reverse runs as
//   b = T* g (zero-frame correlation)  ->  Z-reverse (this file: glr / gtv pass 1, gather pass 2)
//   ->  x-gradient P* gs (reflect adjoint), tap gradients of T and P, weight / scalar gradients.
// The clamped neighbour reads of l / C are differentiated exactly: the scatter onto
// clamp(p + delta_e) is evaluated as a gather over the source pixels of each q (per axis: q - d
// when inside, plus the pixels the clamp folds onto the frame row / column).
//
// Every kernel here is a per-pixel kernel (grid-stride over the elements, reductions by wave
// sums and one fixed-order partial per block); the K-edge windows (K = 8, 12, 24, reach <= 2) make the
// per-pixel working set large, and this path trains the older window models, not the metric's.
#include "grr_common.h"

namespace grr {
namespace {

constexpr int NTB = 256;
constexpr int kWinMaxEdges = 24;

struct WinDeltaB {
  int8_t dy[kWinMaxEdges];
  int8_t dx[kWinMaxEdges];
};

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// Block-wide sums of N per-thread values, one partial per value and block (grr_common.h, fixed-order
// reductions): value i goes to row idx[i] of r[i], slot `slot`.  Every thread of the block must call
// it (the grid-stride loops end before it).
template <int N>
__device__ __forceinline__ void block_red(float (&v)[N], const Red (&r)[N], const int (&idx)[N], uint32_t slot) {
  __shared__ float red[NTB / 64][N];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float s = wsum(v[i]);
    if (lane == 0) red[wave][i] = s;
  }
  __syncthreads();
  if (threadIdx.x < N) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NTB / 64; ++w) t += red[w][threadIdx.x];
    Red rr{nullptr, 1};
    int ii = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (i == (int)threadIdx.x) { rr = r[i]; ii = idx[i]; }
    red_put(rr, ii, slot, t);
  }
}
// slot of block (blockIdx.x, blockIdx.y) of a (chunks, B * per) grid: one per (b, chunk)
__device__ __forceinline__ uint32_t chunk_slot(int per) {
  return (uint32_t)(blockIdx.y / per) * gridDim.x + blockIdx.x;
}
__device__ __forceinline__ int refl(int v, int n) {   // one-pixel reflect frame
  v = v < 0 ? -v : v;
  return v > n - 1 ? 2 * (n - 1) - v : v;
}
// tap t = (centre, up, left, right, down): offsets d_t
__device__ __forceinline__ int tdy(int t) { return t == 1 ? -1 : (t == 4 ? 1 : 0); }
__device__ __forceinline__ int tdx(int t) { return t == 2 ? -1 : (t == 3 ? 1 : 0); }

// sources along one axis of the clamped read clamp(p + d) = q, |d| <= 2: q - d when inside,
// plus the pixels whose read the clamp folds onto the frame (q == 0 for d < 0, q == n-1 for d > 0)
__device__ __forceinline__ int clamp_sources(int q, int d, int n, int (&s)[3]) {
  int k = 0;
  if (q - d >= 0 && q - d < n) s[k++] = q - d;
  if (d < 0 && q == 0)
    for (int p = 0; p < -d && p < n; ++p) if (p != q - d) s[k++] = p;        // p + d < 0
  if (d > 0 && q == n - 1)
    for (int p = n - 1; p > n - 1 - d && p >= 0; --p) if (p != q - d) s[k++] = p;   // p + d > n - 1
  return k;
}
// sources of the reflect read refl(p + d) = q, |d| <= 1
__device__ __forceinline__ int reflect_sources(int q, int d, int n, int (&s)[2]) {
  int k = 0;
  if (q - d >= 0 && q - d < n) s[k++] = q - d;
  if (d == 1 && q == n - 2 && n >= 2) s[k++] = n - 1;   // refl(n) = n - 2
  if (d == -1 && q == 1 && n >= 2) s[k++] = 0;          // refl(-1) = 1
  return k;
}

// ---- stencils.  mode 0 P (reflect), 1 T* (zero-frame correlation), 2 P* (reflect adjoint).
// out = (acc ? out : 0) + (scale ? scale[g] : 1) y,  planes [B, G, Fs], g = (plane / Fs) % G
template <int MODE>
__global__ __launch_bounds__(NTB) void win_stencil_bwd_kernel(const float* __restrict__ x, const float* __restrict__ taps,
                                                              const float* __restrict__ scale, int acc,
                                                              float* __restrict__ out, int G, int Fs, int H, int W,
                                                              int64_t n) {
  const int64_t HW = (int64_t)H * W;
  float k[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) k[t] = taps[t];
  for (int64_t i = blockIdx.x * (int64_t)NTB + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTB) {
    const int64_t plane = i / HW;
    const int p = (int)(i - plane * HW);
    const int r = p / W, c = p - r * W;
    const float* xp = x + plane * HW;
    float y = 0.f;
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const int dy = tdy(t), dx = tdx(t);
      if constexpr (MODE == 0) {
        y += k[t] * xp[refl(r + dy, H) * W + refl(c + dx, W)];
      } else if constexpr (MODE == 1) {
        const int rr = r + dy, cc = c + dx;
        if (rr >= 0 && rr < H && cc >= 0 && cc < W) y += k[t] * xp[rr * W + cc];
      } else {
        int sy[2], sx[2];
        const int ny = reflect_sources(r, dy, H, sy), nx = reflect_sources(c, dx, W, sx);
        float s = 0.f;
        for (int a = 0; a < ny; ++a)
          for (int b = 0; b < nx; ++b) s += xp[sy[a] * W + sx[b]];
        y += k[t] * s;
      }
    }
    if (scale) y *= scale[(plane / Fs) % G];
    out[i] = acc ? out[i] + y : y;
  }
}

// tap gradients: gt[t] += sum over planes of scale[g] sum_p u(p) z(src_t(p));
// mode 0 (P): z(reflect(p + d_t));  mode 1 (T): z(p - d_t) [inside]
template <int MODE>
__global__ __launch_bounds__(NTB) void win_tapgrad_kernel(const float* __restrict__ u, const float* __restrict__ z,
                                                          const float* __restrict__ scale, Red gt,
                                                          int G, int Fs, int H, int W, int64_t n) {
  const int64_t HW = (int64_t)H * W;
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t i = blockIdx.x * (int64_t)NTB + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTB) {
    const int64_t plane = i / HW;
    const int p = (int)(i - plane * HW);
    const int r = p / W, c = p - r * W;
    const float* zp = z + plane * HW;
    const float uv = u[i] * (scale ? scale[(plane / Fs) % G] : 1.f);
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const int dy = tdy(t), dx = tdx(t);
      if constexpr (MODE == 0) {
        acc[t] += uv * zp[refl(r + dy, H) * W + refl(c + dx, W)];
      } else {
        const int rr = r - dy, cc = c - dx;
        if (rr >= 0 && rr < H && cc >= 0 && cc < W) acc[t] += uv * zp[rr * W + cc];
      }
    }
  }
  const Red r[5] = {gt, gt, gt, gt, gt};
  const int idx[5] = {0, 1, 2, 3, 4};
  block_red<5>(acc, r, idx, blockIdx.x);
}

// ---- GLR pass 1.  Per (b, g) and pixel q, channels in turn; sc = scale[g] (mu coef):
//   l(q) = s(q) - sum_e w_e(q) s(n_e(q));  gl = sc b(q)
//   gw_e(q) += -sum_c gl s(n_e(q));  gdot[g] += coef sum b l;  gsd(q) = gl;  E_e(q) = gl w_e(q)
__global__ __launch_bounds__(NTB) void win_glr_bwd_kernel(const float* __restrict__ s, const float* __restrict__ b,
                                                          const float* __restrict__ w, WinDeltaB d, int K,
                                                          const float* __restrict__ scale, float coef,
                                                          float* __restrict__ l_out, float* __restrict__ E,
                                                          float* __restrict__ gsd, float* __restrict__ gw,
                                                          Red gdot, int G, int Fs, int H, int W) {
  // grid (x, B*G): every lane of a block works on the same graph, so the per-graph
  // reduction is one wave sum after the loop, with every lane active
  const int64_t HW = (int64_t)H * W;
  const int64_t bg = blockIdx.y;
  const int g = (int)(bg % G);
  const float sc = scale ? scale[g] : 1.f;
  float dot = 0.f;
  for (int q = blockIdx.x * NTB + threadIdx.x; q < HW; q += gridDim.x * NTB) {
    const int r = q / W, c = q - r * W;
    const float* wq = w + bg * K * HW + q;
    float gwa[kWinMaxEdges];
    for (int e = 0; e < K; ++e) gwa[e] = 0.f;
    for (int ch = 0; ch < Fs; ++ch) {
      const int64_t plane = (bg * Fs + ch) * HW;
      const float* sp = s + plane;
      const float bv = b[plane + q], gl = sc * bv;
      float wx = 0.f;
      for (int e = 0; e < K; ++e) {
        const int nq = clampi(r + d.dy[e], 0, H - 1) * W + clampi(c + d.dx[e], 0, W - 1);
        const float we = wq[e * HW], sn = sp[nq];
        wx += we * sn;
        gwa[e] -= gl * sn;
        if (E) E[((bg * Fs + ch) * K + e) * HW + q] = gl * we;
      }
      const float lv = sp[q] - wx;
      l_out[plane + q] = lv;
      gsd[plane + q] = gl;
      dot += bv * lv;
    }
    for (int e = 0; e < K; ++e) gw[bg * K * HW + e * HW + q] += gwa[e];
  }
  float v[1] = {coef * dot};
  const Red r[1] = {gdot};
  const int idx[1] = {g};
  block_red<1>(v, r, idx, chunk_slot(G));
}

// ---- GTV pass 1 (linear C^T C or the prox C^T phi(C .)).  sc = scale[g] (ro coef):
//   z_e(p) = w_e s(p) - w_e s(n_e(p)), ph_e = phi(z_e), da_e = sc (b(p) - [p + d_e in] b(p + d_e))
//   gph = w_e da_e, gz = phi'(z) gph;  gw_e += ph_e da_e + gz (s(p) - s(n_e(p)))
//   gsd(p) = sum_e gz w_e;  E_e(p) = gz w_e (subtracted at n_e(p) by the gather);  PW_e(p) = w_e ph_e
//   gdot[g] += coef sum_{p,e} ph_e w_e (b(p) - [in] b(p + d_e))  (= coef <b, o>);  ggam[g] += sum gph dphi/dgamma
__global__ __launch_bounds__(NTB) void win_gtv_bwd_kernel(const float* __restrict__ s, const float* __restrict__ b,
                                                          const float* __restrict__ w, WinDeltaB d, int K, int prox,
                                                          const float* __restrict__ log_gamma,
                                                          const float* __restrict__ scale, float coef,
                                                          float* __restrict__ PW, float* __restrict__ E,
                                                          float* __restrict__ gsd, float* __restrict__ gw,
                                                          Red gdot, Red ggam, int G,
                                                          int Fs, int H, int W) {
  const int64_t HW = (int64_t)H * W;                 // grid (x, B*G) as the GLR kernel
  const int64_t bg = blockIdx.y;
  const int g = (int)(bg % G);
  const float sc = scale ? scale[g] : 1.f;
  const float gm = prox ? expf(log_gamma[g]) : 0.f;
  float dot = 0.f, dgam = 0.f;
  for (int p = blockIdx.x * NTB + threadIdx.x; p < HW; p += gridDim.x * NTB) {
    const int r = p / W, c = p - r * W;
    const float* wp = w + bg * K * HW + p;
    float gwa[kWinMaxEdges];
    for (int e = 0; e < K; ++e) gwa[e] = 0.f;
    for (int ch = 0; ch < Fs; ++ch) {
      const int64_t plane = (bg * Fs + ch) * HW;
      const float* sp = s + plane;
      const float* bp = b + plane;
      const float sv = sp[p], bv = bp[p];
      float gs = 0.f;
      for (int e = 0; e < K; ++e) {
        const int ry = r + d.dy[e], cx = c + d.dx[e];
        const bool in = ry >= 0 && ry < H && cx >= 0 && cx < W;
        const int nq = clampi(ry, 0, H - 1) * W + clampi(cx, 0, W - 1);
        const float we = wp[e * HW], sn = sp[nq];
        const float z = __builtin_fmaf(sv, we, -__fmul_rn(we, sn));   // (win_gather_fused_kernel rounds z alike)
        float ph = z, gz;
        const float bd = bv - (in ? bp[ry * W + cx] : 0.f);
        const float gph = we * (sc * bd);
        if (prox) {
          const float lo = z < -gm ? z + gm : 0.f, hi = z > gm ? z - gm : 0.f;
          const float eps = lo + hi;
          ph = eps - (z - eps);
          const bool beyond = z < -gm || z > gm;
          gz = beyond ? gph : -gph;
          dgam += gph * (z < -gm ? 2.f : (z > gm ? -2.f : 0.f));
        } else {
          gz = gph;
        }
        gwa[e] += ph * (sc * bd) + gz * (sv - sn);
        gs += gz * we;
        if (E) E[((bg * Fs + ch) * K + e) * HW + p] = gz * we;
        if (PW) PW[((bg * Fs + ch) * K + e) * HW + p] = we * ph;
        dot += ph * we * bd;
      }
      gsd[plane + p] = gs;
    }
    for (int e = 0; e < K; ++e) gw[bg * K * HW + e * HW + p] += gwa[e];
  }
  float v[2] = {coef * dot, dgam};
  const Red r[2] = {gdot, ggam};
  const int idx[2] = {g, g};
  block_red<2>(v, r, idx, chunk_slot(G));
}

// ---- pass 2 (gather):  gs(q) = gsd(q) - sum_e sum_{p: clamp(p + d_e) = q} E_e(p)
// and, with PW: o(q) = sum_e PW_e(q) - sum_e [q - d_e inside] PW_e(q - d_e)
__global__ __launch_bounds__(NTB) void win_gather_bwd_kernel(const float* __restrict__ E, const float* __restrict__ PW,
                                                             WinDeltaB d, int K, float* __restrict__ gs,
                                                             float* __restrict__ o_out, int H, int W, int64_t n) {
  const int64_t HW = (int64_t)H * W;
  for (int64_t i = blockIdx.x * (int64_t)NTB + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTB) {
    const int64_t plane = i / HW;
    const int q = (int)(i - plane * HW);
    const int r = q / W, c = q - r * W;
    const float* Ep = E + plane * K * HW;
    float acc = 0.f;
    for (int e = 0; e < K; ++e) {
      int sy[3], sx[3];
      const int ny = clamp_sources(r, d.dy[e], H, sy), nx = clamp_sources(c, d.dx[e], W, sx);
      for (int a = 0; a < ny; ++a)
        for (int bb = 0; bb < nx; ++bb) acc += Ep[e * HW + sy[a] * W + sx[bb]];
    }
    gs[i] -= acc;
    if (PW) {
      const float* Pp = PW + plane * K * HW;
      float o = 0.f;
      for (int e = 0; e < K; ++e) o += Pp[e * HW + q];
      for (int e = 0; e < K; ++e) {
        const int py = r - d.dy[e], px = c - d.dx[e];
        if (py >= 0 && py < H && px >= 0 && px < W) o -= Pp[e * HW + py * W + px];
      }
      o_out[i] = o;
    }
  }
}

// ---- pass 2 without the E / PW planes: each E_e(p) / PW_e(p) the gather needs is recomputed at its
// target from s, b and w (pass 1's expressions, in its order).  Every source p of q under edge e has
// clamp(p + d_e) = q, so s(n_e(p)) = s(q), and p + d_e is inside exactly when it equals q (then
// b(p + d_e) = b(q)).  Pass 1 then writes neither plane set (2 Fs K floats per pixel written and read back).
//   GLR: E_e(p) = (sc b(p)) w_e(p)
//   GTV: E_e(p) = gz_e(p) w_e(p), PW_e(p) = w_e(p) ph_e(p)  (win_gtv_bwd_kernel)
template <bool GTV>
__global__ __launch_bounds__(NTB) void win_gather_fused_kernel(const float* __restrict__ s, const float* __restrict__ b,
                                                               const float* __restrict__ w, WinDeltaB d, int K,
                                                               int prox, const float* __restrict__ log_gamma,
                                                               const float* __restrict__ scale,
                                                               float* __restrict__ gs, float* __restrict__ o_out, int G,
                                                               int Fs, int H, int W, int64_t n) {
  const int64_t HW = (int64_t)H * W;
  for (int64_t i = blockIdx.x * (int64_t)NTB + threadIdx.x; i < n; i += (int64_t)gridDim.x * NTB) {
    const int64_t plane = i / HW;                   // (b, g, channel)
    const int64_t bg = plane / Fs;
    const int g = (int)(bg % G);
    const float sc = scale ? scale[g] : 1.f;
    const float gm = GTV && prox ? expf(log_gamma[g]) : 0.f;
    const int q = (int)(i - plane * HW);
    const int r = q / W, c = q - r * W;
    const float* sp = s + plane * HW;
    const float* bp = b + plane * HW;
    const float* wb = w + bg * K * HW;
    const float sq = sp[q], bq = bp[q];
    // E_e(p) (and PW_e(p) for GTV) of source p of q under edge e
    auto edge = [&](int e, int p, bool in, float& pw) {
      const float we = wb[e * HW + p];
      if constexpr (!GTV) {
        pw = 0.f;
        const float gl = sc * bp[p];
        return gl * we;
      } else {
        const float sv = sp[p], sn = sq;
        // pass 1's rounding of z exactly (it compiles to fma(s(p), w, -round(w s(n)))): at tiny gamma the soft
        // threshold's branch follows the last bit of z, so both passes must see the same z
        const float z = __builtin_fmaf(sv, we, -__fmul_rn(we, sn));
        float ph = z, gz;
        const float bd = bp[p] - (in ? bq : 0.f);
        const float gph = we * (sc * bd);
        if (prox) {
          const float lo = z < -gm ? z + gm : 0.f, hi = z > gm ? z - gm : 0.f;
          const float eps = lo + hi;
          ph = eps - (z - eps);
          const bool beyond = z < -gm || z > gm;
          gz = beyond ? gph : -gph;
        } else {
          gz = gph;
        }
        pw = we * ph;
        return gz * we;
      }
    };
    float acc = 0.f;
    for (int e = 0; e < K; ++e) {
      int sy[3], sx[3];
      const int dy = d.dy[e], dx = d.dx[e];
      const int ny = clamp_sources(r, dy, H, sy), nx = clamp_sources(c, dx, W, sx);
      for (int a = 0; a < ny; ++a)
        for (int bb = 0; bb < nx; ++bb) {
          const int py = sy[a], px = sx[bb];
          const bool in = py + dy >= 0 && py + dy < H && px + dx >= 0 && px + dx < W;
          float pw;
          acc += edge(e, py * W + px, in, pw);
        }
    }
    gs[i] -= acc;
    if (GTV && o_out) {
      // o(q) = sum_e PW_e(q) - sum_e [q - d_e inside] PW_e(q - d_e)  (pass 2's order: the first sum, then
      // the subtraction term by term)
      float o = 0.f;
      for (int e = 0; e < K; ++e) {
        const int ny2 = clampi(r + d.dy[e], 0, H - 1), nx2 = clampi(c + d.dx[e], 0, W - 1);
        const float we = wb[e * HW + q], sv = sq, sn = sp[ny2 * W + nx2];
        const float z = __builtin_fmaf(sv, we, -__fmul_rn(we, sn));
        float ph = z;
        if (prox) {
          const float lo = z < -gm ? z + gm : 0.f, hi = z > gm ? z - gm : 0.f;
          const float eps = lo + hi;
          ph = eps - (z - eps);
        }
        o += we * ph;
      }
      for (int e = 0; e < K; ++e) {
        const int py = r - d.dy[e], px = c - d.dx[e];
        if (py >= 0 && py < H && px >= 0 && px < W) {
          float pw;
          const bool in = true;   // p + d_e = q
          edge(e, py * W + px, in, pw);
          o -= pw;
        }
      }
      o_out[i] = o;
    }
  }
}

// ---- edge-weight reverse (REF7:418-446).  Pass 1, in place: gw_e <- gsim_e = w_e (gw_e - sum w gw)
__global__ __launch_bounds__(NTB) void win_softmax_bwd_kernel(const float* __restrict__ w, float* __restrict__ gw, int K,
                                                              int64_t HW, int64_t npix) {
  for (int64_t i = blockIdx.x * (int64_t)NTB + threadIdx.x; i < npix; i += (int64_t)gridDim.x * NTB) {
    const int64_t bg = i / HW, p = i - bg * HW;
    const float* wp = w + bg * K * HW + p;
    float* gp = gw + bg * K * HW + p;
    float s = 0.f;
    for (int e = 0; e < K; ++e) s += wp[e * HW] * gp[e * HW];
    for (int e = 0; e < K; ++e) gp[e * HW] = wp[e * HW] * (gp[e * HW] - s);
  }
}
// Pass 2: fh_f = M_f f_f / max(|f|, 1e-12), sim_e(p) = sum_f fh_f(p) fh_f(n_e(p)):
//   gfh_f(q) = sum_e gsim_e(q) fh_f(n_e(q)) + sum_e sum_{p: n_e(p) = q} gsim_e(p) fh_f(p)
//   gM[g,f] += gfh_f n_f;  gf = (gn - n (n . gn)) / |f| (gn / eps below eps), gn = M gfh
template <int FMAX>
__global__ __launch_bounds__(NTB) void win_feat_bwd_kernel(const float* __restrict__ feat, int64_t fstride,
                                                           const float* __restrict__ multiM,
                                                           const float* __restrict__ gsim, WinDeltaB d, int K,
                                                           float* __restrict__ gfeat, int64_t gstride,
                                                           Red gM, int G, int F, int H, int W) {
  // grid (x, B*G): the graph is fixed per block, so gM reduces per block (one partial per f)
  const int64_t HW = (int64_t)H * W;
  const int bg = blockIdx.y, g = bg % G, b = bg / G;
  const float* fp = feat + (int64_t)b * fstride + (int64_t)g * F * HW;
  float* gfp = gfeat + (int64_t)b * gstride + (int64_t)g * F * HW;
  const float* gsp = gsim + (int64_t)bg * K * HW;
  float M[FMAX], gMa[FMAX];
#pragma unroll
  for (int f = 0; f < FMAX; ++f) {
    M[f] = f < F ? multiM[g * F + f] : 0.f;
    gMa[f] = 0.f;
  }
  // fh(pix) = M f(pix) / max(|f(pix)|, eps), accumulated as  acc += wt * fh(pix)
  auto add_fh = [&](float (&acc)[FMAX], int pix, float wt) {
    float v[FMAX], ss = 0.f;
#pragma unroll
    for (int f = 0; f < FMAX; ++f) {
      v[f] = f < F ? fp[f * HW + pix] : 0.f;
      ss += v[f] * v[f];
    }
    const float c = wt / fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
    for (int f = 0; f < FMAX; ++f) acc[f] += c * (v[f] * M[f]);
  };
  for (int q = blockIdx.x * NTB + threadIdx.x; q < HW; q += gridDim.x * NTB) {
    const int r = q / W, c = q - r * W;
    float gfh[FMAX];
#pragma unroll
    for (int f = 0; f < FMAX; ++f) gfh[f] = 0.f;
    for (int e = 0; e < K; ++e) {
      const int nq = clampi(r + d.dy[e], 0, H - 1) * W + clampi(c + d.dx[e], 0, W - 1);
      add_fh(gfh, nq, gsp[e * HW + q]);
      int sy[3], sx[3];
      const int ny = clamp_sources(r, d.dy[e], H, sy), nx = clamp_sources(c, d.dx[e], W, sx);
      for (int a = 0; a < ny; ++a)
        for (int bb = 0; bb < nx; ++bb) {
          const int pp = sy[a] * W + sx[bb];
          add_fh(gfh, pp, gsp[e * HW + pp]);
        }
    }
    float v[FMAX], nrm = 0.f;
#pragma unroll
    for (int f = 0; f < FMAX; ++f) {
      v[f] = f < F ? fp[f * HW + q] : 0.f;
      nrm += v[f] * v[f];
    }
    const float inv = 1.f / fmaxf(sqrtf(nrm), 1e-12f);
    const bool small = sqrtf(nrm) <= 1e-12f;
    float ndg = 0.f;
#pragma unroll
    for (int f = 0; f < FMAX; ++f) {
      const float n = v[f] * inv;
      gMa[f] += gfh[f] * n;
      ndg += n * (gfh[f] * M[f]);
    }
#pragma unroll
    for (int f = 0; f < FMAX; ++f) {
      if (f < F) {
        const float n = v[f] * inv, gn = gfh[f] * M[f];
        gfp[f * HW + q] += small ? gn * inv : (gn - n * ndg) * inv;   // GTV and GLR share a slab
      }
    }
  }
  Red r[FMAX];
  int idx[FMAX];
#pragma unroll
  for (int f = 0; f < FMAX; ++f) {
    r[f] = f < F ? gM : Red{nullptr, 1};
    idx[f] = g * F + f;
  }
  block_red<FMAX>(gMa, r, idx, chunk_slot(G));
}

// ---- mixture reverse (REF7:1006-1009): out[b,c] = sum_g score[b,g] x[b,g,c] + dc[b,c]
//   gx[b,g,c] = gout[b,c] score[b,g];  gscore[b,g] = sum_c gout[b,c] x[b,g,c]
__global__ __launch_bounds__(NTB) void win_mix_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ x,
                                                          const float* __restrict__ score, float* __restrict__ gx,
                                                          float* __restrict__ gscore, int G, int Fs, int64_t HW,
                                                          int64_t npix) {
  for (int64_t i = blockIdx.x * (int64_t)NTB + threadIdx.x; i < npix; i += (int64_t)gridDim.x * NTB) {
    const int64_t bg = i / HW, p = i - bg * HW;
    const int64_t b = bg / G;
    const float sv = score[bg * HW + p];
    float gsc = 0.f;
    for (int c = 0; c < Fs; ++c) {
      const float go = gout[(b * Fs + c) * HW + p];
      gx[(bg * Fs + c) * HW + p] = go * sv;
      gsc += go * x[(bg * Fs + c) * HW + p];
    }
    gscore[bg * HW + p] = gsc;
  }
}

int grid_1d(int64_t n) { return (int)std::min<int64_t>((n + NTB - 1) / NTB, 1 << 16); }
// reduction kernels: about 4096 blocks in all (16 per CU), grid-stride beyond, so the per-block
// partials stay few
int grid_red(int64_t n) { return (int)std::min<int64_t>((n + NTB - 1) / NTB, 4096); }
dim3 plane_grid(int H, int W, int planes) {
  const int64_t per = std::max<int64_t>(1, 4096 / std::max(planes, 1));
  return dim3((unsigned)std::min<int64_t>(((int64_t)H * W + NTB - 1) / NTB, per), (unsigned)planes);
}

// delta: int32 [K,2] (dy, dx), the layout grr_win_edge_weights / grr_win_solver take
bool fill_delta(const int32_t* delta, int K, WinDeltaB& d) {
  if (!delta || K <= 0 || K > kWinMaxEdges) return false;
  for (int e = 0; e < K; ++e) {
    const int dy = delta[2 * e], dx = delta[2 * e + 1];
    if (dy < -2 || dy > 2 || dx < -2 || dx > 2) return false;
    d.dy[e] = (int8_t)dy;
    d.dx[e] = (int8_t)dx;
  }
  return true;
}

}  // namespace
}  // namespace grr

using namespace grr;

extern "C" {

grr_status grr_win_bwd_stencil(const float* x, const float* taps, int mode, const float* scale, int accumulate,
                               float* out, int B, int G, int Fs, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && taps && out && B > 0 && G > 0 && Fs > 0 && H > 1 && W > 1 && mode >= 0 && mode <= 2,
              GRR_ERR_INVALID_ARG, "grr_win_bwd_stencil: bad args");
  const int64_t n = (int64_t)B * G * Fs * H * W;
  hipStream_t s = (hipStream_t)stream;
  if (mode == 0)
    hipLaunchKernelGGL(win_stencil_bwd_kernel<0>, dim3(grid_1d(n)), dim3(NTB), 0, s, x, taps, scale, accumulate, out, G, Fs, H, W, n);
  else if (mode == 1)
    hipLaunchKernelGGL(win_stencil_bwd_kernel<1>, dim3(grid_1d(n)), dim3(NTB), 0, s, x, taps, scale, accumulate, out, G, Fs, H, W, n);
  else
    hipLaunchKernelGGL(win_stencil_bwd_kernel<2>, dim3(grid_1d(n)), dim3(NTB), 0, s, x, taps, scale, accumulate, out, G, Fs, H, W, n);
  return launch_status("grr_win_bwd_stencil");
}

grr_status grr_win_bwd_tapgrad(const float* u, const float* z, int mode, const float* scale, float* gtaps, int B,
                               int G, int Fs, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(u && z && gtaps && B > 0 && G > 0 && Fs > 0 && H > 1 && W > 1 && (mode == 0 || mode == 1),
              GRR_ERR_INVALID_ARG, "grr_win_bwd_tapgrad: bad args");
  const int64_t n = (int64_t)B * G * Fs * H * W;
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_red(n);
  RedScratch rs(s);
  const int it = rs.plan(gtaps, 5, (uint32_t)grid);
  grr_status st = rs.alloc("grr_win_bwd_tapgrad");
  if (st != GRR_OK) return st;
  if (mode == 0)
    hipLaunchKernelGGL(win_tapgrad_kernel<0>, dim3(grid), dim3(NTB), 0, s, u, z, scale, rs.red(it), G, Fs, H, W, n);
  else
    hipLaunchKernelGGL(win_tapgrad_kernel<1>, dim3(grid), dim3(NTB), 0, s, u, z, scale, rs.red(it), G, Fs, H, W, n);
  st = launch_status("grr_win_bwd_tapgrad");
  return st != GRR_OK ? st : rs.finish("grr_win_bwd_tapgrad");
}

grr_status grr_win_bwd_glr(const float* s, const float* b, const float* w, const int32_t* delta, int K,
                           const float* scale, float coef, float* l_out, float* E, float* gsd, float* gw, float* gdot,
                           int B, int G, int Fs, int H, int W, void* stream) {
  clear_error();
  WinDeltaB d{};
  GRR_REQUIRE(s && b && w && l_out && gsd && gw && B > 0 && G > 0 && Fs > 0 && H > 1 && W > 1 &&
                  fill_delta(delta, K, d),
              GRR_ERR_INVALID_ARG, "grr_win_bwd_glr: bad args");
  GRR_REQUIRE((int64_t)B * G <= 65535, GRR_ERR_UNSUPPORTED, "grr_win_bwd_glr: B*G > 65535");
  const dim3 grid = plane_grid(H, W, B * G);
  RedScratch rs((hipStream_t)stream);
  const int id = rs.plan(gdot, G, (uint32_t)B * grid.x);
  grr_status st = rs.alloc("grr_win_bwd_glr");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(win_glr_bwd_kernel, grid, dim3(NTB), 0, (hipStream_t)stream, s, b, w, d, K, scale, coef, l_out, E,
                     gsd, gw, rs.red(id), G, Fs, H, W);
  st = launch_status("grr_win_bwd_glr");
  return st != GRR_OK ? st : rs.finish("grr_win_bwd_glr");
}

grr_status grr_win_bwd_gtv(const float* s, const float* b, const float* w, const int32_t* delta, int K,
                           int prox, const float* log_gamma, const float* scale, float coef, float* PW, float* E,
                           float* gsd, float* gw, float* gdot, float* ggamma, int B, int G, int Fs, int H, int W,
                           void* stream) {
  clear_error();
  WinDeltaB d{};
  GRR_REQUIRE(s && b && w && gsd && gw && B > 0 && G > 0 && Fs > 0 && H > 1 && W > 1 &&
                  (!prox || log_gamma) && fill_delta(delta, K, d),
              GRR_ERR_INVALID_ARG, "grr_win_bwd_gtv: bad args");
  GRR_REQUIRE((int64_t)B * G <= 65535, GRR_ERR_UNSUPPORTED, "grr_win_bwd_gtv: B*G > 65535");
  const dim3 grid = plane_grid(H, W, B * G);
  RedScratch rs((hipStream_t)stream);
  const int id = rs.plan(gdot, G, (uint32_t)B * grid.x), ig = rs.plan(prox ? ggamma : nullptr, G, (uint32_t)B * grid.x);
  grr_status st = rs.alloc("grr_win_bwd_gtv");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(win_gtv_bwd_kernel, grid, dim3(NTB), 0, (hipStream_t)stream, s, b, w, d, K, prox, log_gamma,
                     scale, coef, PW, E, gsd, gw, rs.red(id), rs.red(ig), G, Fs, H, W);
  st = launch_status("grr_win_bwd_gtv");
  return st != GRR_OK ? st : rs.finish("grr_win_bwd_gtv");
}

grr_status grr_win_bwd_gather(const float* E, const float* PW, const int32_t* delta, int K, float* gs,
                              float* o_out, int B, int G, int Fs, int H, int W, void* stream) {
  clear_error();
  WinDeltaB d{};
  GRR_REQUIRE(E && gs && (!PW || o_out) && B > 0 && G > 0 && Fs > 0 && H > 1 && W > 1 && fill_delta(delta, K, d),
              GRR_ERR_INVALID_ARG, "grr_win_bwd_gather: bad args");
  const int64_t n = (int64_t)B * G * Fs * H * W;
  hipLaunchKernelGGL(win_gather_bwd_kernel, dim3(grid_1d(n)), dim3(NTB), 0, (hipStream_t)stream, E, PW, d, K, gs, o_out,
                     H, W, n);
  return launch_status("grr_win_bwd_gather");
}

grr_status grr_win_bwd_gather_fused(const float* s, const float* b, const float* w, const int32_t* delta, int K,
                                    int gtv, int prox, const float* log_gamma, const float* scale, float* gs,
                                    float* o_out, int B, int G, int Fs, int H, int W, void* stream) {
  clear_error();
  WinDeltaB d{};
  GRR_REQUIRE(s && b && w && gs && (gtv || !o_out) && (!gtv || !prox || log_gamma) && B > 0 && G > 0 && Fs > 0 &&
                  H > 1 && W > 1 && fill_delta(delta, K, d),
              GRR_ERR_INVALID_ARG, "grr_win_bwd_gather_fused: bad args");
  const int64_t n = (int64_t)B * G * Fs * H * W;
  if (gtv)
    hipLaunchKernelGGL(win_gather_fused_kernel<true>, dim3(grid_1d(n)), dim3(NTB), 0, (hipStream_t)stream, s, b, w, d,
                       K, prox, log_gamma, scale, gs, o_out, G, Fs, H, W, n);
  else
    hipLaunchKernelGGL(win_gather_fused_kernel<false>, dim3(grid_1d(n)), dim3(NTB), 0, (hipStream_t)stream, s, b, w,
                       d, K, 0, nullptr, scale, gs, nullptr, G, Fs, H, W, n);
  return launch_status("grr_win_bwd_gather_fused");
}

grr_status grr_win_bwd_edge_weights(const float* feat, int64_t feat_bstride, const float* multiM, const float* w,
                                    float* gw, const int32_t* delta, int K, float* gfeat,
                                    int64_t gfeat_bstride, float* gmultiM, int B, int G, int F, int H, int W,
                                    void* stream) {
  clear_error();
  WinDeltaB d{};
  GRR_REQUIRE(feat && multiM && w && gw && gfeat && gmultiM && B > 0 && G > 0 && F > 0 && H > 0 && W > 0 &&
                  fill_delta(delta, K, d),
              GRR_ERR_INVALID_ARG, "grr_win_bwd_edge_weights: bad args");
  GRR_REQUIRE(F <= GRR_MAX_NODE_FTS, GRR_ERR_UNSUPPORTED, "grr_win_bwd_edge_weights: F=%d > %d", F,
              GRR_MAX_NODE_FTS);
  const int64_t npix = (int64_t)B * G * H * W;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(win_softmax_bwd_kernel, dim3(grid_1d(npix)), dim3(NTB), 0, s, w, gw, K, (int64_t)H * W, npix);
  GRR_REQUIRE((int64_t)B * G <= 65535, GRR_ERR_UNSUPPORTED, "grr_win_bwd_edge_weights: B*G > 65535");
  grr_status st = launch_status("grr_win_bwd_edge_weights");
  if (st != GRR_OK) return st;
  const dim3 grid = plane_grid(H, W, B * G);
  RedScratch rs(s);
  const int im = rs.plan(gmultiM, G * F, (uint32_t)B * grid.x);
  st = rs.alloc("grr_win_bwd_edge_weights");
  if (st != GRR_OK) return st;
  const Red rm = rs.red(im);
#define WIN_FEAT_BWD(FM_)                                                                                          \
  hipLaunchKernelGGL(win_feat_bwd_kernel<FM_>, grid, dim3(NTB), 0, s, feat, feat_bstride, multiM, gw, d, K, gfeat, \
                     gfeat_bstride, rm, G, F, H, W)
  if (F <= 4)
    WIN_FEAT_BWD(4);
  else if (F <= 12)
    WIN_FEAT_BWD(12);
  else
    WIN_FEAT_BWD(GRR_MAX_NODE_FTS);
#undef WIN_FEAT_BWD
  st = launch_status("grr_win_bwd_edge_weights");
  return st != GRR_OK ? st : rs.finish("grr_win_bwd_edge_weights");
}

grr_status grr_win_bwd_mix(const float* gout, const float* x, const float* score, float* gx, float* gscore, int B,
                           int G, int Fs, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(gout && x && score && gx && gscore && B > 0 && G > 0 && Fs > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_win_bwd_mix: bad args");
  const int64_t npix = (int64_t)B * G * H * W;
  hipLaunchKernelGGL(win_mix_bwd_kernel, dim3(grid_1d(npix)), dim3(NTB), 0, (hipStream_t)stream, gout, x, score, gx,
                     gscore, G, Fs, (int64_t)H * W, npix);
  return launch_status("grr_win_bwd_mix");
}

}  // extern "C"
