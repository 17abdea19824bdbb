// Backward (adjoint) kernels of the GGTV/GGLR solver for training (config C4).
//
// The forward solver (graph_ops.hip) fuses whole operator applications into streaming
// kernels.  Its reverse pass is written here as a small set of per-pixel kernels that
// the host (irdu_amd/solver_grad.py) composes into the reverse of every operator
// application (REF = exploration/GGTV_GGLR_v1.0/deep_multiscale_GGLR_GGTV_v1x0.py):
//
//   stencil_kernel       S = replicate-pad 3x3 cross correlation (REF:177-195), its
//                        conv_transpose partner S^T (zero frame, REF:197-215) and the
//                        exact adjoints of both (4 modes)
//   tapgrad_kernel       d/d(tap) of S or S^T, reduced per channel
//   glr_bwd_kernel       reverse of (I - W) inside GLR  (REF:218-237)
//   pair_bwd_kernel      reverse of the symmetric pair Laplacian inside C^T C (REF:452-523)
//   prox_bwd_kernel      reverse of C^T phi(C s) with the soft-threshold prox (REF:684-704, :757-781)
//   pair_weights_bwd     c = w_right^2 + w_left(p+1)^2 ... -> raw edge weights
//   edge_weights_bwd     softmax + normalise + multiM (REF:146-175)
//   graph_dot / lincomb / unpool2_acc / conv2x2s2_bwd_data: recurrence and feature-conv glue
//
// All are HBM-bound streaming passes with one thread per pixel; the F node features of
// one graph are looped inside the thread so the graph's edge weights are read once.
// Reductions (per-graph scalars, per-channel taps, multiM) are accumulated in registers
// over a grid-strided pixel range, reduced across the wave with shuffles and across the
// workgroup through LDS in wave order, and stored into the contributor's own slot of a
// partials array; red_finish_kernel adds the slots in order (grr_common.h, "Fixed-order
// reductions"): bitwise run-to-run reproducible, no float atomics.
//
// Tap order (host computes taps [C,5] from stats_kernel_p01/p02a/p02b/p03):
//   0 centre (0,0), 1 up (-1,0), 2 left (0,-1), 3 right (0,+1), 4 down (+1,0).
// Edge order (REF:42-53): 0 up, 1 left, 2 right, 3 down; opposite(e) = 3 - e.
#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "grr_common.h"

namespace grr {
namespace {

constexpr int NT = 256;
constexpr int TARGET_BLOCKS = 4096;   // grid size of the pixel-looping reduction kernels

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// one partial per block: wave sums -> LDS -> thread 0 adds them in wave order and stores the
// block's slot.  Every thread of the block must call it (it synchronises); consecutive calls
// reuse the LDS slots safely.
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

__device__ __forceinline__ bool inside_e(int e, int r, int c, int H, int W) {
  switch (e) {
    case 0: return r > 0;
    case 1: return c > 0;
    case 2: return c + 1 < W;
    default: return r + 1 < H;
  }
}
__device__ __forceinline__ int off_e(int e, int W) {
  switch (e) {
    case 0: return -W;
    case 1: return -1;
    case 2: return 1;
    default: return W;
  }
}
// tap t: offsets (dy, dx)
__device__ __forceinline__ int tap_dy(int t) { return t == 1 ? -1 : (t == 4 ? 1 : 0); }
__device__ __forceinline__ int tap_dx(int t) { return t == 2 ? -1 : (t == 3 ? 1 : 0); }

// ---------------------------------------------------------------------------
// Stencil apply.  mode 0 P:  y(p) = sum_t k_t x(clamp(p + t))            (S, REF:177-195)
//                 mode 1 T:  y(q) = sum_t k_t x(q - t) [q - t inside]     (S^T, REF:197-215)
//                 mode 2 Tt: y(p) = sum_t k_t x(p + t) [p + t inside]     (adjoint of T)
//                 mode 3 Pt: y(q) = sum_t k_t ([q - t in] x(q - t) + [t != 0, q + t out] x(q))  (adjoint of P)
// out = (acc ? out : 0) + (scale ? scale[g] : 1) * y.   grid (ceil(HW/NT), B*C).
// ---------------------------------------------------------------------------
template <int mode>
__global__ __launch_bounds__(NT) void stencil_kernel(const float* __restrict__ x, const float* __restrict__ taps,
                                                     const float* __restrict__ scale, int acc,
                                                     float* __restrict__ out, int C, int F, int H, int W) {
  const int HW = H * W;
  const int p = blockIdx.x * NT + threadIdx.x;
  if (p >= HW) return;
  const int plane = blockIdx.y, ch = plane % C;
  const int r = p / W, col = p - r * W;
  const float* xp = x + (int64_t)plane * HW;
  float k[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) k[t] = taps[ch * 5 + t];
  float y = 0.f;
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const int dy = tap_dy(t), dx = tap_dx(t);
    if constexpr (mode == 0) {
      y += k[t] * xp[clampi(r + dy, 0, H - 1) * W + clampi(col + dx, 0, W - 1)];
    } else if constexpr (mode == 1) {
      const int rr = r - dy, cc = col - dx;
      if (rr >= 0 && rr < H && cc >= 0 && cc < W) y += k[t] * xp[rr * W + cc];
    } else if constexpr (mode == 2) {
      const int rr = r + dy, cc = col + dx;
      if (rr >= 0 && rr < H && cc >= 0 && cc < W) y += k[t] * xp[rr * W + cc];
    } else {
      const int rr = r - dy, cc = col - dx;
      if (rr >= 0 && rr < H && cc >= 0 && cc < W) y += k[t] * xp[rr * W + cc];
      const int ro = r + dy, co = col + dx;
      if (t != 0 && (ro < 0 || ro >= H || co < 0 || co >= W)) y += k[t] * xp[p];
    }
  }
  if (scale) y *= scale[ch / F];
  float* o = out + (int64_t)plane * HW + p;
  *o = acc ? *o + y : y;
}

// The same four stencils, four adjacent columns per thread (W % 4 == 0, 16-byte aligned planes):
// rows r-1, r, r+1 as float4 plus the two flanking columns of row r.  grid (ceil(HW/4/NT), B*C).
typedef float f4 __attribute__((ext_vector_type(4)));
template <int mode>
__global__ __launch_bounds__(NT) void stencil4_kernel(const float* __restrict__ x, const float* __restrict__ taps,
                                                      const float* __restrict__ scale, int acc,
                                                      float* __restrict__ out, int C, int F, int H, int W) {
  const int HW = H * W, W4 = W / 4;
  const int q4 = blockIdx.x * NT + threadIdx.x;
  if (q4 >= HW / 4) return;
  const int plane = blockIdx.y, ch = plane % C;
  const int r = q4 / W4, c0 = (q4 - r * W4) * 4;
  const float* xp = x + (int64_t)plane * HW;
  const float k0 = taps[ch * 5], ku = taps[ch * 5 + 1], kl = taps[ch * 5 + 2], kr = taps[ch * 5 + 3],
              kd = taps[ch * 5 + 4];
  const bool top = r == 0, bot = r == H - 1, lft = c0 == 0, rgt = c0 + 4 == W;
  const f4 cv = *reinterpret_cast<const f4*>(xp + r * W + c0);
  f4 uv, dv;
  float lv, rv;
  if constexpr (mode == 0) {   // replicate
    uv = *reinterpret_cast<const f4*>(xp + (top ? r : r - 1) * W + c0);
    dv = *reinterpret_cast<const f4*>(xp + (bot ? r : r + 1) * W + c0);
    lv = lft ? cv[0] : xp[r * W + c0 - 1];
    rv = rgt ? cv[3] : xp[r * W + c0 + 4];
  } else {                     // zero frame
    uv = top ? f4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f4*>(xp + (r - 1) * W + c0);
    dv = bot ? f4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f4*>(xp + (r + 1) * W + c0);
    lv = lft ? 0.f : xp[r * W + c0 - 1];
    rv = rgt ? 0.f : xp[r * W + c0 + 4];
  }
  f4 y;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float l = j > 0 ? cv[j - 1] : lv, rr = j < 3 ? cv[j + 1] : rv;
    float v;
    if constexpr (mode == 0 || mode == 2) {   // sum_t k_t x(p + t)
      v = k0 * cv[j];
      v += ku * uv[j]; v += kl * l; v += kr * rr; v += kd * dv[j];
    } else {                                  // sum_t k_t x(q - t)
      v = k0 * cv[j];
      v += ku * dv[j]; v += kl * rr; v += kr * l; v += kd * uv[j];
      if constexpr (mode == 3) {              // replicate adjoint: clamped reads at the frame land on q
        const int col = c0 + j;
        if (top) v += ku * cv[j];
        if (bot) v += kd * cv[j];
        if (col == 0) v += kl * cv[j];
        if (col == W - 1) v += kr * cv[j];
      }
    }
    y[j] = v;
  }
  if (scale) y *= scale[ch / F];
  f4* o = reinterpret_cast<f4*>(out + (int64_t)plane * HW + r * W + c0);
  *o = acc ? *o + y : y;
}

// The x-gradient pass of the GLR and the GTV term of one level in one sweep (both are P* of the
// replicate stencil, mode 3, with the module's own taps and scale):
//   out += s1[g] P1*(v1) + s2[g] P2*(v2)
// reads v1, v2, out and writes out once (two stencil4_kernel<3> launches read out twice and write it
// twice).  Four adjacent columns per thread, W % 4 == 0.  grid (ceil(HW/4/NT), B*C).
__device__ __forceinline__ f4 padj4(const float* xp, float k0, float ku, float kl, float kr, float kd, int r, int c0,
                                    int H, int W) {
  const bool top = r == 0, bot = r == H - 1, lft = c0 == 0, rgt = c0 + 4 == W;
  const f4 cv = *reinterpret_cast<const f4*>(xp + r * W + c0);
  const f4 uv = top ? f4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f4*>(xp + (r - 1) * W + c0);
  const f4 dv = bot ? f4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const f4*>(xp + (r + 1) * W + c0);
  const float lv = lft ? 0.f : xp[r * W + c0 - 1];
  const float rv = rgt ? 0.f : xp[r * W + c0 + 4];
  f4 y;
#pragma unroll
  for (int j = 0; j < 4; ++j) {   // stencil4_kernel<3>'s expression, term by term
    const float l = j > 0 ? cv[j - 1] : lv, rr = j < 3 ? cv[j + 1] : rv;
    float v = k0 * cv[j];
    v += ku * dv[j]; v += kl * rr; v += kr * l; v += kd * uv[j];
    const int col = c0 + j;
    if (top) v += ku * cv[j];
    if (bot) v += kd * cv[j];
    if (col == 0) v += kl * cv[j];
    if (col == W - 1) v += kr * cv[j];
    y[j] = v;
  }
  return y;
}
__global__ __launch_bounds__(NT) void padj2_kernel(const float* __restrict__ x1, const float* __restrict__ taps1,
                                                   const float* __restrict__ scale1, const float* __restrict__ x2,
                                                   const float* __restrict__ taps2, const float* __restrict__ scale2,
                                                   float* __restrict__ out, int C, int F, int H, int W) {
  const int HW = H * W, W4 = W / 4;
  const int q4 = blockIdx.x * NT + threadIdx.x;
  if (q4 >= HW / 4) return;
  const int plane = blockIdx.y, ch = plane % C;
  const int r = q4 / W4, c0 = (q4 - r * W4) * 4;
  const float* t1 = taps1 + ch * 5;
  const float* t2 = taps2 + ch * 5;
  f4 y1 = padj4(x1 + (int64_t)plane * HW, t1[0], t1[1], t1[2], t1[3], t1[4], r, c0, H, W);
  f4 y2 = padj4(x2 + (int64_t)plane * HW, t2[0], t2[1], t2[2], t2[3], t2[4], r, c0, H, W);
  y1 *= scale1[ch / F];
  y2 *= scale2[ch / F];
  f4* o = reinterpret_cast<f4*>(out + (int64_t)plane * HW + r * W + c0);
  *o = (*o + y1) + y2;   // the order of two accumulating stencil launches
}

// Tap gradients of y = mode(z) contracted with u: gt[c, t] += scale[g] * sum_{b,q} u(q) dy(q)/dk_t.
// mode 0 (P): dy(q)/dk_t = z(clamp(q + t));  mode 1 (T): z(q - t) [inside].   grid (chunks, B*C).
template <int mode>
__global__ __launch_bounds__(NT) void tapgrad_kernel(const float* __restrict__ u, const float* __restrict__ z,
                                                     const float* __restrict__ scale,
                                                     Red gt, int C, int F, int H, int W) {
  const int HW = H * W;
  const int plane = blockIdx.y, ch = plane % C;
  const float* up = u + (int64_t)plane * HW;
  const float* zp = z + (int64_t)plane * HW;
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = blockIdx.x * NT + threadIdx.x; p < HW; p += gridDim.x * NT) {
    const int r = p / W, col = p - r * W;
    const float uv = up[p];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const int dy = tap_dy(t), dx = tap_dx(t);
      if constexpr (mode == 0) {
        acc[t] += uv * zp[clampi(r + dy, 0, H - 1) * W + clampi(col + dx, 0, W - 1)];
      } else {
        const int rr = r - dy, cc = col - dx;
        if (rr >= 0 && rr < H && cc >= 0 && cc < W) acc[t] += uv * zp[rr * W + cc];
      }
    }
  }
  const float sc = scale ? scale[ch / F] : 1.f;
#pragma unroll
  for (int t = 0; t < 5; ++t) block_red_put(gt, ch * 5 + t, chunk_slot(C), sc * acc[t]);
}

// ---------------------------------------------------------------------------
// GLR reverse.  Forward inside GLR: z = (I - W) s,  (W s)(p) = sum_e w_e(p) s(nb_e(p)),
// nb_e(p) = clamp(p + delta_e) (REF:218-237).  Given s = P x and a = Tt(g):
//   z_out  = (I - W) s                      (for the T-tap gradient)
//   ap_out = (I - W)^T a                    (then x-gradient = Pt(ap), P-tap gradient)
//   gw[e](p) += scale[g] * (-sum_f a_f(p) s_f(nb_e p))
//   gdot[g]  += coef * sum a . z            (d/d mu of <g, T z>)
// grid (ceil(HW/NT), B*G)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void glr_bwd_kernel(const float* __restrict__ s, const float* __restrict__ a,
                                                     const float* __restrict__ w, const float* __restrict__ scale,
                                                     float coef, float* __restrict__ z_out,
                                                     float* __restrict__ ap_out, float* __restrict__ gw,
                                                     Red gdot, int G, int F, int H, int W) {
  const int HW = H * W;
  const int bg = blockIdx.y, g = bg % G;
  float dot = 0.f;
  for (int p = blockIdx.x * NT + threadIdx.x; p < HW; p += gridDim.x * NT) {
    const int r = p / W, col = p - r * W;
    const float* wb = w + (int64_t)bg * 4 * HW;
    float we[4], wn[4];
    bool in[4];
    int nb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      in[e] = inside_e(e, r, col, H, W);
      nb[e] = in[e] ? p + off_e(e, W) : p;
      we[e] = wb[e * HW + p];
    }
    // w_e(p - delta_e) = w of edge e at the opposite neighbour (exists iff that neighbour is inside)
#pragma unroll
    for (int e = 0; e < 4; ++e) wn[e] = in[3 - e] ? wb[e * HW + nb[3 - e]] : 0.f;
    float gwa[4] = {0.f, 0.f, 0.f, 0.f};
    for (int f = 0; f < F; ++f) {
      const int64_t base = ((int64_t)bg * F + f) * HW;
      const float* sp = s + base;
      const float* ap = a + base;
      const float sv = sp[p], av = ap[p];
      float z = sv, wta = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float sn = sp[nb[e]];
        z -= we[e] * sn;
        gwa[e] -= av * sn;
        wta += in[3 - e] ? wn[e] * ap[nb[3 - e]] : 0.f;   // scatter-adjoint, interior part
        wta += in[e] ? 0.f : we[e] * av;                  // clamped (self) reads at the frame
      }
      z_out[base + p] = z;
      ap_out[base + p] = av - wta;
      dot += av * z;
    }
    const float sc = scale ? scale[g] : 1.f;
    float* gwb = gw + (int64_t)bg * 4 * HW + p;
#pragma unroll
    for (int e = 0; e < 4; ++e) gwb[e * HW] += sc * gwa[e];
  }
  if (gdot.p) block_red_put(gdot, g, chunk_slot(G), coef * dot);
}

// Pair-Laplacian reverse (GTV C^T C, linear part).  K s(p) = sum over the 4 incident edges
// of c_edge (s(p) - s(other)); c[0] = edge (p, p+right), c[1] = edge (p, p+down).  K is
// symmetric, so ap_out = K a.  gc[d](p) += scale[g] sum_f (a(p) - a(p+d)) (s(p) - s(p+d)).
__global__ __launch_bounds__(NT) void pair_bwd_kernel(const float* __restrict__ s, const float* __restrict__ a,
                                                      const float* __restrict__ cw, const float* __restrict__ scale,
                                                      float coef, float* __restrict__ z_out,
                                                      float* __restrict__ ap_out, float* __restrict__ gc,
                                                      Red gdot, int G, int F, int H, int W) {
  const int HW = H * W;
  const int bg = blockIdx.y, g = bg % G;
  float dot = 0.f;
  for (int p = blockIdx.x * NT + threadIdx.x; p < HW; p += gridDim.x * NT) {
    const int r = p / W, col = p - r * W;
    const float* cb = cw + (int64_t)bg * 2 * HW;
    const bool hr = col + 1 < W, hl = col > 0, vd = r + 1 < H, vu = r > 0;
    const float cr = hr ? cb[p] : 0.f, cl = hl ? cb[p - 1] : 0.f;
    const float cd = vd ? cb[HW + p] : 0.f, cu = vu ? cb[HW + p - W] : 0.f;
    const int pr = hr ? p + 1 : p, pl = hl ? p - 1 : p, pd = vd ? p + W : p, pu = vu ? p - W : p;
    float gh = 0.f, gv = 0.f;
    for (int f = 0; f < F; ++f) {
      const int64_t base = ((int64_t)bg * F + f) * HW;
      const float* sp = s + base;
      const float* ap = a + base;
      const float sv = sp[p], av = ap[p];
      const float sr = sp[pr], sl = sp[pl], sd = sp[pd], su = sp[pu];
      const float ar = ap[pr], al = ap[pl], ad = ap[pd], au = ap[pu];
      const float z = cr * (sv - sr) + cl * (sv - sl) + cd * (sv - sd) + cu * (sv - su);
      const float ka = cr * (av - ar) + cl * (av - al) + cd * (av - ad) + cu * (av - au);
      z_out[base + p] = z;
      ap_out[base + p] = ka;
      gh += (av - ar) * (sv - sr);
      gv += (av - ad) * (sv - sd);
      dot += av * z;
    }
    const float sc = scale ? scale[g] : 1.f;
    float* gcb = gc + (int64_t)bg * 2 * HW + p;
    if (hr) gcb[0] += sc * gh;
    if (vd) gcb[HW] += sc * gv;
  }
  if (gdot.p) block_red_put(gdot, g, chunk_slot(G), coef * dot);
}

// ---------------------------------------------------------------------------
// Prox reverse: o = Ct(phi(C s)) before the final S^T, with
//   t_e(p) = w_e(p) (s(p) - s(p + delta_e))  (0 when p + delta_e is outside)      REF:452-467
//   phi(t) = 2 soft(t, gamma) - t,  soft = the reference's two wheres               REF:684-704, :766-771
//   o(q)   = sum_e w_e(q) phi_e(q) - sum_e [q - delta_e in] w_e(q - delta_e) phi_e(q - delta_e)   REF:469-516
// Given a = Tt(g):
//   o_out(q), gs_out(q) = d<a, o>/ds(q),  gw[e](q) += scale * d<a,o>/dw_e(q),
//   ggam[g] += scale * d<a,o>/dgamma,     gdot[g] += coef * <a, o>
// ---------------------------------------------------------------------------
// soft threshold as t - clamp(t, -gm, gm): the same fp32 value as the two-sided select (one v_med3)
__device__ __forceinline__ float soft_t(float t, float gm) { return t - __builtin_amdgcn_fmed3f(t, -gm, gm); }

__global__ __launch_bounds__(NT) void prox_bwd_kernel(const float* __restrict__ s, const float* __restrict__ a,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ log_gamma,
                                                      const float* __restrict__ scale, float coef,
                                                      float* __restrict__ o_out, float* __restrict__ gs_out,
                                                      float* __restrict__ gw, Red ggam,
                                                      Red gdot, int G, int F, int H, int W) {
  const int HW = H * W;
  const int bg = blockIdx.y, g = bg % G;
  float dot = 0.f, dgam = 0.f;
  const float gm = expf(log_gamma[g]);
  for (int p = blockIdx.x * NT + threadIdx.x; p < HW; p += gridDim.x * NT) {
    const int r = p / W, col = p - r * W;
    const float* wb = w + (int64_t)bg * 4 * HW;
    float we[4], wn[4];
    bool in[4];
    int nb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      in[e] = inside_e(e, r, col, H, W);
      nb[e] = in[e] ? p + off_e(e, W) : p;
      we[e] = wb[e * HW + p];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) wn[e] = in[3 - e] ? wb[e * HW + nb[3 - e]] : 0.f;   // w_e(p - delta_e)
    float gwa[4] = {0.f, 0.f, 0.f, 0.f};
    for (int f = 0; f < F; ++f) {
      const int64_t base = ((int64_t)bg * F + f) * HW;
      const float* sp = s + base;
      const float* ap = a + base;
      const float sv = sp[p], av = ap[p];
      float o = 0.f, gs = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // edge e leaving p
        if (in[e]) {
          const float sn = sp[nb[e]], an = ap[nb[e]];
          const float ds = sv - sn, t = we[e] * ds;
          const float ph = 2.f * soft_t(t, gm) - t;
          const float da = av - an;
          const float gph = we[e] * da;
          const bool beyond = t < -gm || t > gm;
          const float gt = beyond ? gph : -gph;
          o += we[e] * ph;
          gs += gt * we[e];
          gwa[e] += ph * da + gt * ds;
          dgam += gph * (t < -gm ? 2.f : (t > gm ? -2.f : 0.f));
        }   // else t = 0, phi = 0: no contribution to o, w or gamma
        // edge e arriving at p from q' = p - delta_e (neighbour in direction 3-e)
        if (in[3 - e]) {
          const int q = nb[3 - e];
          const float sq = sp[q], aq = ap[q];
          const float t = wn[e] * (sq - sv);
          const float ph = 2.f * soft_t(t, gm) - t;
          const float gph = wn[e] * (aq - av);
          const bool beyond = t < -gm || t > gm;
          const float gt = beyond ? gph : -gph;
          o -= wn[e] * ph;
          gs -= gt * wn[e];
        }
      }
      o_out[base + p] = o;
      gs_out[base + p] = gs;
      dot += av * o;
    }
    const float sc = scale ? scale[g] : 1.f;
    float* gwb = gw + (int64_t)bg * 4 * HW + p;
#pragma unroll
    for (int e = 0; e < 4; ++e) gwb[e * HW] += sc * gwa[e];
  }
  dgam *= scale ? scale[g] : 1.f;
  if (gdot.p) block_red_put(gdot, g, chunk_slot(G), coef * dot);
  if (ggam.p) block_red_put(ggam, g, chunk_slot(G), dgam);
}

// c[0](p) = w_right(p)^2 + w_left(p+1)^2, c[1](p) = w_down(p)^2 + w_up(p+W)^2 (0 at the frame):
// gw[right](p) += 2 w_right(p) gc0(p);  gw[left](q) += 2 w_left(q) gc0(q-1);
// gw[down](p)  += 2 w_down(p) gc1(p);   gw[up](q)   += 2 w_up(q) gc1(q-W).      grid (ceil(HW/NT), B*G)
__global__ __launch_bounds__(NT) void pair_weights_bwd_kernel(const float* __restrict__ w, const float* __restrict__ gc,
                                                              float* __restrict__ gw, int H, int W) {
  const int HW = H * W;
  const int bg = blockIdx.y;
  const int p = blockIdx.x * NT + threadIdx.x;
  if (p >= HW) return;
  const int r = p / W, col = p - r * W;
  const float* wb = w + (int64_t)bg * 4 * HW;
  const float* gcb = gc + (int64_t)bg * 2 * HW;
  float* gwb = gw + (int64_t)bg * 4 * HW;
  if (r > 0) gwb[p] += 2.f * wb[p] * gcb[HW + p - W];
  if (col > 0) gwb[HW + p] += 2.f * wb[HW + p] * gcb[p - 1];
  if (col + 1 < W) gwb[2 * HW + p] += 2.f * wb[2 * HW + p] * gcb[p];
  if (r + 1 < H) gwb[3 * HW + p] += 2.f * wb[3 * HW + p] * gcb[HW + p];
}

// ---------------------------------------------------------------------------
// Edge-weight reverse (REF:146-175): fh_f = M_f f_f / max(|f|, 1e-12);
// sim_e(p) = sum_f fh_f(p) fh_f(nb_e p);  w = softmax_e(sim).
//   gsim_e(p) = w_e(p) (gw_e(p) - sum_e' w_e'(p) gw_e'(p))
//   gfh_f(q)  = sum_e gsim_e(q) fh_f(nb_e q) + sum_e [q - delta_e in] gsim_e(q - delta_e) fh_f(q - delta_e)
//             + sum_e [q + delta_e out] gsim_e(q) fh_f(q)
//   gM[g,f]  += gfh_f n_f ;  gf = (gn - n (n . gn)) / |f|  (gn / eps below eps), gn = M gfh
// feat / gfeat: channel-0 pointers of the module's [G*F] slab, batch strides in elements.
// grid (chunks, B*G)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float inv_den(const float* fp, int64_t HW, int F, int p) {
  float ss = 0.f;
  for (int f = 0; f < F; ++f) {
    const float v = fp[f * HW + p];
    ss += v * v;
  }
  return 1.f / fmaxf(sqrtf(ss), 1e-12f);
}
__device__ __forceinline__ float gsim_at(const float* wb, const float* gwb, int64_t HW, int e, int p) {
  const float w0 = wb[p], w1 = wb[HW + p], w2 = wb[2 * HW + p], w3 = wb[3 * HW + p];
  const float s = w0 * gwb[p] + w1 * gwb[HW + p] + w2 * gwb[2 * HW + p] + w3 * gwb[3 * HW + p];
  return wb[e * HW + p] * (gwb[e * HW + p] - s);
}

__global__ __launch_bounds__(NT) void edge_weights_bwd_kernel(const float* __restrict__ feat, int64_t fstride,
                                                              const float* __restrict__ multiM,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ gw,
                                                              float* __restrict__ gfeat, int64_t gstride,
                                                              Red gM, int G, int F, int H, int W) {
  const int HW = H * W;
  const int bg = blockIdx.y, g = bg % G, b = bg / G;
  const float* fp = feat + (int64_t)b * fstride + (int64_t)g * F * HW;
  float* gfp = gfeat + (int64_t)b * gstride + (int64_t)g * F * HW;
  const float* wb = w + (int64_t)bg * 4 * HW;
  const float* gwb = gw + (int64_t)bg * 4 * HW;
  const float* M = multiM + g * F;
  // per-thread multiM gradient partials in LDS (F <= GRR_MAX_NODE_FTS), reduced once per block
  __shared__ float gm_sm[GRR_MAX_NODE_FTS * NT];
  for (int f = 0; f < F; ++f) gm_sm[f * NT + threadIdx.x] = 0.f;
  for (int p = blockIdx.x * NT + threadIdx.x; p < HW; p += gridDim.x * NT) {
    const int r = p / W, col = p - r * W;
    bool in[4];
    int nb[4];
    float inb[4], gs_out[4], gs_in[4];
    const float ic = inv_den(fp, HW, F, p);
    float gsum = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      in[e] = inside_e(e, r, col, H, W);
      nb[e] = in[e] ? p + off_e(e, W) : p;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      inb[e] = in[e] ? inv_den(fp, HW, F, nb[e]) : ic;
      gs_out[e] = gsim_at(wb, gwb, HW, e, p);
      // gsim of edge e at q' = p - delta_e (the neighbour in direction 3-e), whose e-neighbour is p
      gs_in[e] = in[3 - e] ? gsim_at(wb, gwb, HW, e, nb[3 - e]) : 0.f;
      gsum += in[e] ? 0.f : gs_out[e];          // self term at the frame
    }
    // pass A: n . gn
    float ndg = 0.f;
    for (int f = 0; f < F; ++f) {
      const float* ff = fp + (int64_t)f * HW;
      const float m = M[f];
      const float n = ff[p] * ic;
      float gfh = gsum * n * m;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gfh += gs_out[e] * ff[nb[e]] * inb[e] * m;
        if (in[3 - e]) gfh += gs_in[e] * ff[nb[3 - e]] * inb[3 - e] * m;
      }
      gm_sm[f * NT + threadIdx.x] += gfh * n;
      ndg += n * (gfh * m);
    }
    // pass B: gf
    const bool small = 1.f / ic <= 1e-12f;
    for (int f = 0; f < F; ++f) {
      const float* ff = fp + (int64_t)f * HW;
      const float m = M[f];
      const float n = ff[p] * ic;
      float gfh = gsum * n * m;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gfh += gs_out[e] * ff[nb[e]] * inb[e] * m;
        if (in[3 - e]) gfh += gs_in[e] * ff[nb[3 - e]] * inb[3 - e] * m;
      }
      const float gn = gfh * m;
      gfp[(int64_t)f * HW + p] = small ? gn * ic : (gn - n * ndg) * ic;
    }
  }
  for (int f = 0; f < F; ++f) block_red_put(gM, g * F + f, chunk_slot(G), gm_sm[f * NT + threadIdx.x]);
}

typedef float f4v __attribute__((ext_vector_type(4)));

// gdot[g] += coef * sum_{b,f,p} u v.      grid (chunks, B*G); V4: float4 loads (n % 4 == 0, aligned)
template <bool V4>
__global__ __launch_bounds__(NT) void graph_dot_kernel(const float* __restrict__ u, const float* __restrict__ v,
                                                       float coef, Red gdot, int G, int F,
                                                       int64_t HW) {
  const int bg = blockIdx.y, g = bg % G;
  const int64_t n = (int64_t)F * HW;
  const float* up = u + (int64_t)bg * n;
  const float* vp = v + (int64_t)bg * n;
  float acc = 0.f;
  if constexpr (V4) {
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * NT) {
      const f4v a = *reinterpret_cast<const f4v*>(up + 4 * i), b = *reinterpret_cast<const f4v*>(vp + 4 * i);
      acc += a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) acc += up[i] * vp[i];
  }
  block_red_put(gdot, g, chunk_slot(G), coef * acc);
}

// out = sa[g] * x + sb[g] * y  (sa/sb NULL -> 1; y NULL -> term dropped); acc: out += ...
// grid (chunks, B*G): one (b, graph) slab of n = F H W floats per block row; V4 as graph_dot_kernel
template <bool V4>
__global__ __launch_bounds__(NT) void lincomb_kernel(const float* __restrict__ x, const float* __restrict__ sa,
                                                     const float* __restrict__ y, const float* __restrict__ sb,
                                                     float* __restrict__ out, int acc, int G, int64_t n) {
  const int bg = blockIdx.y, g = bg % G;
  const float a = sa ? sa[g] : 1.f, bb = sb ? sb[g] : 1.f;
  const int64_t base = (int64_t)bg * n;
  if constexpr (V4) {
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * NT) {
      const int64_t o = base + 4 * i;
      f4v v = a * *reinterpret_cast<const f4v*>(x + o);
      if (y) v += bb * *reinterpret_cast<const f4v*>(y + o);
      f4v* dst = reinterpret_cast<f4v*>(out + o);
      *dst = acc ? *dst + v : v;
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
      const int64_t o = base + i;
      float v = a * x[o];
      if (y) v += bb * y[o];
      out[o] = acc ? out[o] + v : v;
    }
  }
}

// One reverse step of the stage recurrence x' = x + alpha u, u = r - A x + beta u_prev, without
// the operator term (REF:784-807), in one pass over the (b, g) slab:
//   galpha[g] += <gx', u>;  gu = alpha[g] gx' + beta_next[g] gu_next;  gbeta[g] += <gu, u_prev>;
//   gbb += gu;  gx_out = gx' - gu  (gx_out may alias gx).                 grid (chunks, B*G)
// gxh (optional): the previous stage's half-level x-gradient not yet added, gx' = gx + U gxh (the 2x2
// unpool-accumulate, unpool2_acc_kernel's arithmetic) -- one read of gx instead of U's read + write.
// pj (optional, V4 only): the previous stage's full-level x-gradient pass not yet applied,
// gx' = (gx + s1 P1*(v1)) + s2 P2*(v2) before U -- padj2_kernel's arithmetic and order.
struct GluePadj {
  const float *v1, *t1, *s1, *v2, *t2, *s2;
};
// gud (optional, V4, even H): D gu as well (pool2_kernel's arithmetic), the half-level operand of the
// operator reverse that reads gu next -- each thread takes the same four columns of a row pair.
template <bool V4>
__global__ __launch_bounds__(NT) void cg_glue_kernel(const float* gx, const float* __restrict__ gxh, GluePadj pj,
                                                     int F, const float* __restrict__ u,
                                                     const float* __restrict__ gun, const float* __restrict__ up,
                                                     const float* __restrict__ alpha,
                                                     const float* __restrict__ beta_next, float* __restrict__ gu_out,
                                                     float* __restrict__ gbb, float* gx_out,
                                                     float* __restrict__ gud, Red galpha, Red gbeta, int G,
                                                     int64_t n, int H, int W) {
  const int bg = blockIdx.y, g = bg % G;
  const int64_t base = (int64_t)bg * n;
  const float al = alpha[g], be = gun ? beta_next[g] : 0.f;
  const int HW = H * W, w2 = W / 2;
  const int64_t hbase = (int64_t)bg * (n / 4);   // the slab's half-level planes: F (H/2) (W/2) floats
  auto half_at = [&](int li) {   // offset of the half-level value under slab element li
    const int f = li / HW, p = li - f * HW, r = p / W, c = p - r * W;
    return hbase + (int64_t)f * (HW / 4) + (r >> 1) * w2 + (c >> 1);
  };
  float da = 0.f, db = 0.f;
  if constexpr (V4) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    typedef float f2 __attribute__((ext_vector_type(2)));
    // four columns at slab element li (W % 4 == 0 where pj / gxh / gud are given)
    auto glue4 = [&](int li) __attribute__((always_inline)) {
      const int64_t o = base + li;
      f4 x = *reinterpret_cast<const f4*>(gx + o);
      const f4 uv = *reinterpret_cast<const f4*>(u + o);
      if (pj.v1) {
        const int f = li / HW, p = li - f * HW, r = p / W, c = p - r * W;
        const int ch = g * F + f;
        const int64_t po = ((int64_t)bg * F + f) * HW;
        const float *k1 = pj.t1 + ch * 5, *k2 = pj.t2 + ch * 5;
        f4 y1 = padj4(pj.v1 + po, k1[0], k1[1], k1[2], k1[3], k1[4], r, c, H, W);
        f4 y2 = padj4(pj.v2 + po, k2[0], k2[1], k2[2], k2[3], k2[4], r, c, H, W);
        y1 *= pj.s1[g];
        y2 *= pj.s2[g];
        x = (x + y1) + y2;
      }
      if (gxh) {   // the four columns sit over two half-level columns
        const f2 q = *reinterpret_cast<const f2*>(gxh + half_at(li));
        x.x += 0.25f * q.x; x.y += 0.25f * q.x; x.z += 0.25f * q.y; x.w += 0.25f * q.y;
      }
      f4 gu = al * x;
      if (gun) gu += be * *reinterpret_cast<const f4*>(gun + o);
      da += x.x * uv.x + x.y * uv.y + x.z * uv.z + x.w * uv.w;
      if (up) {
        const f4 pv = *reinterpret_cast<const f4*>(up + o);
        db += gu.x * pv.x + gu.y * pv.y + gu.z * pv.z + gu.w * pv.w;
      }
      if (gbb) *reinterpret_cast<f4*>(gbb + o) += gu;
      *reinterpret_cast<f4*>(gu_out + o) = gu;
      *reinterpret_cast<f4*>(gx_out + o) = x - gu;
      return gu;
    };
    if (gud) {   // (f, half row, column quad) per step
      const int W4 = W / 4, hq = (H / 2) * W4;
      const int64_t nq = n / 8;
      for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < nq; i += (int64_t)gridDim.x * NT) {
        const int q = (int)i, f = q / hq, rem = q - f * hq, hr = rem / W4, c4 = rem - hr * W4;
        const int li = f * HW + 2 * hr * W + 4 * c4;
        const f4 g0 = glue4(li), g1 = glue4(li + W);
        f2 d;
        d.x = 0.25f * g0.x + 0.25f * g0.y + 0.25f * g1.x + 0.25f * g1.y;
        d.y = 0.25f * g0.z + 0.25f * g0.w + 0.25f * g1.z + 0.25f * g1.w;
        *reinterpret_cast<f2*>(gud + hbase + (int64_t)f * (HW / 4) + hr * w2 + 2 * c4) = d;
      }
    } else {
      const int64_t n4 = n / 4;
      for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT)
        glue4((int)(4 * i));
    }
  } else {
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
      const int64_t o = base + i;
      float x = gx[o];
      if (gxh) x += 0.25f * gxh[half_at((int)i)];
      float gu = al * x;
      if (gun) gu += be * gun[o];
      da += x * u[o];
      if (up) db += gu * up[o];
      if (gbb) gbb[o] += gu;
      gu_out[o] = gu;
      gx_out[o] = x - gu;
    }
  }
  block_red_put(galpha, g, chunk_slot(G), da);
  if (up) block_red_put(gbeta, g, chunk_slot(G), db);
}

// out(q) += 0.25 * xd(q / 2)   (U = conv_transpose2d of the 0.25 2x2 kernel, stride 2; REF:676-679)
__global__ __launch_bounds__(NT) void unpool2_acc_kernel(const float* __restrict__ xd, float* __restrict__ out, int H,
                                                         int W, int64_t n) {
  const int h = H / 2, w = W / 2;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t plane = i / ((int64_t)H * W);
    const int p = (int)(i - plane * H * W);
    const int r = p / W, c = p - r * W;
    out[i] += 0.25f * xd[plane * h * w + (r >> 1) * w + (c >> 1)];
  }
}

// the same, four output columns per thread (W % 4 == 0, aligned): grid (chunks, planes)
__global__ __launch_bounds__(NT) void unpool2_acc4_kernel(const float* __restrict__ xd, float* __restrict__ out,
                                                          int H, int W) {
  const int w = W / 2, W4 = W / 4, n4 = H * W4;
  const int64_t plane = blockIdx.y;
  const float* xp = xd + plane * (H / 2) * w;
  float* op = out + plane * H * W;
  for (int i = blockIdx.x * NT + threadIdx.x; i < n4; i += gridDim.x * NT) {
    const int r = i / W4, c4 = i - r * W4;
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 q = *reinterpret_cast<const f2*>(xp + (r >> 1) * w + 2 * c4);
    f4v* dst = reinterpret_cast<f4v*>(op + r * W + 4 * c4);
    f4v v = *dst;
    v.x += 0.25f * q.x; v.y += 0.25f * q.x; v.z += 0.25f * q.y; v.w += 0.25f * q.y;
    *dst = v;
  }
}

// data gradient of the 2x2 stride-2 conv (REF:593-602):
// gx[b,k,2i+di,2j+dj] = sum_m wt[m,k,di,dj] g[b,m,i,j]
__global__ __launch_bounds__(NT) void conv2x2s2_bwd_data_kernel(const float* __restrict__ g,
                                                                const float* __restrict__ wt,
                                                                float* __restrict__ gx, int K, int M, int H, int W) {
  const int HW = H * W, h = H / 2, w = W / 2;
  const int p = blockIdx.x * NT + threadIdx.x;
  if (p >= HW) return;
  const int bk = blockIdx.y, b = bk / K, k = bk % K;
  const int r = p / W, c = p - r * W;
  const int tap = (r & 1) * 2 + (c & 1);
  const float* gp = g + (int64_t)b * M * h * w + (r >> 1) * w + (c >> 1);
  float acc = 0.f;
  for (int m = 0; m < M; ++m) acc += wt[(m * K + k) * 4 + tap] * gp[(int64_t)m * h * w];
  gx[(int64_t)bk * HW + p] = acc;
}

// gx[b,k,2i+di,2j+dj] = t[b, (2 di + dj) K + k, i, j]: the four tap planes of the 2x2 stride-2 conv's
// data gradient, computed as one 1x1 GEMM with 4K output rows, interleaved to full resolution.
// One thread per 4 consecutive output pixels of a row (float4 store; two float2 source reads).
__global__ __launch_bounds__(NT) void interleave2x2_kernel(const float* __restrict__ t, float* __restrict__ gx, int K,
                                                           int H, int W, int64_t nq) {
  const int h = H / 2, w = W / 2, W4 = W / 4;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < nq; i += (int64_t)gridDim.x * NT) {
    const int64_t row = i / W4;                        // (b, k, r)
    const int c4 = (int)(i - row * W4) * 4;
    const int r = (int)(row % H);
    const int64_t bk = row / H;
    const int64_t b = bk / K, k = bk - b * K;
    const int di = r & 1;
    const float* t0 = t + ((b * 4 + 2 * di) * K + k) * h * w + (int64_t)(r >> 1) * w + c4 / 2;
    const float* t1 = t0 + (int64_t)K * h * w;        // dj = 1
    const float2 e = *reinterpret_cast<const float2*>(t0), o = *reinterpret_cast<const float2*>(t1);
    *reinterpret_cast<float4*>(gx + row * W + c4) = make_float4(e.x, o.x, e.y, o.y);
  }
}

// ---------------------------------------------------------------------------
// Fused term reverse: one pass per operator term instead of five.  s = P x and a = T* g
// are recomputed on the fly at the pixel and its four neighbours (radius-2 reads that hit
// L1/L2), the term's reverse runs as in glr_bwd / pair_bwd / prox_bwd above, and both
// tap gradients are accumulated in the same pass in their gather forms:
//   T taps:  sum_q g(q) z(q - t) [inside]  = sum_p z(p) g(p + t) [p + t inside]
//   P taps:  sum_q v(q) x(clamp(q + t))     with v = (I-W)^T a, K a or d<a,o>/ds
// Output v_out = that v (the x-gradient is then one adjoint-stencil pass, P* v).
// MODE 0: GLR (w raw),  1: pair Laplacian (w = pair weights),  2: prox (w raw, gamma).
// F is a template parameter so the per-channel tap partials stay in registers.
// grid (chunks, B*G)
// ---------------------------------------------------------------------------
template <int MODE, int F>
__global__ __launch_bounds__(NT) void term_bwd_fused_kernel(
    const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ taps,
    const float* __restrict__ w, const float* __restrict__ log_gamma, const float* __restrict__ scale, float coef,
    float* __restrict__ v_out, float* __restrict__ gw, Red ggam, Red gdot,
    Red gtaps, int G, int H, int W) {
  const int HW = H * W;
  const int bg = blockIdx.y, gi = bg % G;
  const float sc = scale ? scale[gi] : 1.f;
  const float gm = MODE == 2 ? expf(log_gamma[gi]) : 0.f;
  float k[F][5];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int t = 0; t < 5; ++t) k[f][t] = taps[(gi * F + f) * 5 + t];
  float accT[F][5], accP[F][5];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int t = 0; t < 5; ++t) { accT[f][t] = 0.f; accP[f][t] = 0.f; }
  float dot = 0.f, dgam = 0.f;
  const int wplanes = MODE == 1 ? 2 : 4;
  const float* wb = w + (int64_t)bg * wplanes * HW;
  float* gwb = gw + (int64_t)bg * wplanes * HW;

  for (int p = blockIdx.x * NT + threadIdx.x; p < HW; p += gridDim.x * NT) {
    const int r = p / W, col = p - r * W;
    bool in[4];
    int nb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      in[e] = inside_e(e, r, col, H, W);
      nb[e] = in[e] ? p + off_e(e, W) : p;
    }
    // neighbour coordinates of the 5 positions {p, up, left, right, down} (clamped)
    const int pr[5] = {r, in[0] ? r - 1 : r, r, r, in[3] ? r + 1 : r};
    const int pc[5] = {col, col, in[1] ? col - 1 : col, in[2] ? col + 1 : col, col};
    float we[4] = {0.f, 0.f, 0.f, 0.f}, wn[4] = {0.f, 0.f, 0.f, 0.f};
    float cr = 0.f, cl = 0.f, cd = 0.f, cu = 0.f;
    if constexpr (MODE == 1) {
      cr = in[2] ? wb[p] : 0.f; cl = in[1] ? wb[p - 1] : 0.f;
      cd = in[3] ? wb[HW + p] : 0.f; cu = in[0] ? wb[HW + p - W] : 0.f;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) we[e] = wb[e * HW + p];
#pragma unroll
      for (int e = 0; e < 4; ++e) wn[e] = in[3 - e] ? wb[e * HW + nb[3 - e]] : 0.f;
    }
    float gwa[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int f = 0; f < F; ++f) {
      const int64_t base = ((int64_t)bg * F + f) * HW;
      const float* xp = x + base;
      const float* gp = g + base;
      // s = P x (replicate) and a = T* g (zero frame) at the 5 positions
      float s5[5], a5[5], xt[5], gt5[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const int rr = pr[i], cc = pc[i];
        const float* xr = xp + rr * W;
        const float xc = xr[cc];
        const float xu = xp[max(rr - 1, 0) * W + cc], xd = xp[min(rr + 1, H - 1) * W + cc];
        const float xl = xr[max(cc - 1, 0)], xrr = xr[min(cc + 1, W - 1)];
        s5[i] = k[f][0] * xc + k[f][1] * xu + k[f][2] * xl + k[f][3] * xrr + k[f][4] * xd;
        const float* gr = gp + rr * W;
        const float gc = gr[cc];
        const float gu = rr > 0 ? gp[(rr - 1) * W + cc] : 0.f, gd = rr + 1 < H ? gp[(rr + 1) * W + cc] : 0.f;
        const float gl = cc > 0 ? gr[cc - 1] : 0.f, grr = cc + 1 < W ? gr[cc + 1] : 0.f;
        a5[i] = k[f][0] * gc + k[f][1] * gu + k[f][2] * gl + k[f][3] * grr + k[f][4] * gd;
        if (i == 0) {
          xt[0] = xc; xt[1] = xu; xt[2] = xl; xt[3] = xrr; xt[4] = xd;   // x(clamp(p + t))
          gt5[0] = gc; gt5[1] = gu; gt5[2] = gl; gt5[3] = grr; gt5[4] = gd;   // g(p + t), 0 outside
        }
      }
      const float sv = s5[0], av = a5[0];
      float z = 0.f, v = 0.f;
      if constexpr (MODE == 0) {
        float wta = 0.f;
        z = sv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float sn = s5[e + 1];            // s(nb_e p): positions 1..4 are up, left, right, down
          z -= we[e] * sn;
          gwa[e] -= av * sn;
          wta += in[3 - e] ? wn[e] * a5[(3 - e) + 1] : 0.f;
          wta += in[e] ? 0.f : we[e] * av;
        }
        v = av - wta;
      } else if constexpr (MODE == 1) {
        const float su = s5[1], sl = s5[2], sr = s5[3], sd = s5[4];
        const float au = a5[1], al = a5[2], ar = a5[3], ad = a5[4];
        z = cr * (sv - sr) + cl * (sv - sl) + cd * (sv - sd) + cu * (sv - su);
        v = cr * (av - ar) + cl * (av - al) + cd * (av - ad) + cu * (av - au);
        gwa[0] += (av - ar) * (sv - sr);
        gwa[1] += (av - ad) * (sv - sd);
      } else {
        float o = 0.f, gs = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (in[e]) {
            const float sn = s5[e + 1], an = a5[e + 1];
            const float ds = sv - sn, t = we[e] * ds;
            const float ph = 2.f * soft_t(t, gm) - t;
            const float da = av - an;
            const float gph = we[e] * da;
            const float gtv = (t < -gm || t > gm) ? gph : -gph;
            o += we[e] * ph;
            gs += gtv * we[e];
            gwa[e] += ph * da + gtv * ds;
            dgam += gph * (t < -gm ? 2.f : (t > gm ? -2.f : 0.f));
          }
          if (in[3 - e]) {
            const float sq = s5[(3 - e) + 1], aq = a5[(3 - e) + 1];
            const float t = wn[e] * (sq - sv);
            const float ph = 2.f * soft_t(t, gm) - t;
            const float gph = wn[e] * (aq - av);
            const float gtv = (t < -gm || t > gm) ? gph : -gph;
            o -= wn[e] * ph;
            gs -= gtv * wn[e];
          }
        }
        z = o;
        v = gs;
      }
      v_out[base + p] = v;
      dot += av * z;
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        accT[f][t] += z * gt5[t];
        accP[f][t] += v * xt[t];
      }
    }
    if constexpr (MODE == 1) {
      if (in[2]) gwb[p] += sc * gwa[0];
      if (in[3]) gwb[HW + p] += sc * gwa[1];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) gwb[e * HW + p] += sc * gwa[e];
    }
  }
  const uint32_t slot = chunk_slot(G);
  if (gdot.p) block_red_put(gdot, gi, slot, coef * dot);
  if constexpr (MODE == 2) {
    if (ggam.p) block_red_put(ggam, gi, slot, sc * dgam);
  }
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int t = 0; t < 5; ++t) block_red_put(gtaps, (gi * F + f) * 5 + t, slot, sc * (accT[f][t] + accP[f][t]));
}

// ---------------------------------------------------------------------------
// The same term reverse as a row-streaming kernel (W <= 64 V, W % V == 0): one workgroup = the
// F channel waves of one (b, graph, row segment), lane = V adjacent columns.  Each wave keeps
// x and g rows t-3..t, s = P x and a = T* g rows t-3..t-1 in registers (vertical neighbours)
// and takes horizontal neighbours by DPP lane shifts; per output row r = t-2 it evaluates the
// per-pixel arithmetic of term_bwd_fused_kernel (same expressions, same order) for its
// channel.  The weight gradient sums over the F channels of the graph: each wave writes its
// row of partials to LDS (double-buffered by row parity, one barrier per row) and the sum in
// channel order is added to gw by the wave that owns the plane.  x, g, w are read once and v,
// gw written once per launch (the per-pixel kernel re-reads every operand 5-25 times from
// L1/L2 and runs at ≈ 1.7 TB/s).
// ---------------------------------------------------------------------------
// grr_bwd_set_term_rows: 0 = per-pixel term reverses, 1 = the register-prefetch row kernel, 2 (default) = the
// LDS-ring row kernel where it applies (A/B and tests)
int g_term_rows = 2;
// ring kernel: the x-gradient pass inside up to this width (the half levels, where it replaces a stencil
// pass); wider levels fold it into the CG glue pass instead (training steps, same box,
// profiles/r05/term/ab_acc_policy.txt: msgf 65.2 -> 63.8 ms, C4 942 -> 933 ms against the pass inside at
// every width).  grr_bwd_set_term_acc_max_w (A/B and tests)
int g_term_acc_max_w = 128;
// ring kernel: the narrow V = 1 tail launch for a row's last strip (launch_term_row); GRR_TERM_TAIL=0 or
// grr_bwd_set_term_tail(0) turns it off (A/B and tests)
int g_term_tail = [] {
  const char* e = getenv("GRR_TERM_TAIL");
  return e ? atoi(e) : 1;
}();

template <int V> struct RowT;
template <> struct RowT<1> { typedef float T; };
template <> struct RowT<2> { typedef float __attribute__((ext_vector_type(2))) T; };
template <> struct RowT<4> { typedef float __attribute__((ext_vector_type(4))) T; };
template <int V>
__device__ __forceinline__ void rload(float (&d)[V], const float* p) {
  const typename RowT<V>::T t = *reinterpret_cast<const typename RowT<V>::T*>(p);
  if constexpr (V == 1) {
    d[0] = t;
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) d[j] = t[j];
  }
}
template <int V>
__device__ __forceinline__ void rstore(float* p, const float (&v)[V]) {
  typename RowT<V>::T t;
  if constexpr (V == 1) {
    t = v[0];
  } else {
#pragma unroll
    for (int j = 0; j < V; ++j) t[j] = v[j];
  }
  *reinterpret_cast<typename RowT<V>::T*>(p) = t;
}
__device__ __forceinline__ float lprev(float v) {   // lane - 1 (0 at lane 0)
  float r = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xF, 0xF, true));
  asm volatile("" : "+v"(r));
  return r;
}
__device__ __forceinline__ float lnext(float v) {   // lane + 1 (0 at lane 63)
  float r = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xF, 0xF, true));
  asm volatile("" : "+v"(r));
  return r;
}

// Workgroup = F channel waves: up to 12 for V = 4 (a 768-thread bound caps the kernel at 168
// VGPRs = 3 waves per SIMD, which also gives 4 three-wave workgroups per CU instead of 2 at the
// 176-182 VGPRs the compiler picks unconstrained), up to 16 for V <= 2 (128 VGPRs).
template <int V> struct TermRowMax { static constexpr int F = V == 4 ? 12 : 16; };
// gw rows of the read-modify-write through LDS-DMA one row ahead: the summing wave copies gw row r + 1 of
// its planes into an LDS ring right after adding row r, so the next row's read-modify-write reads LDS
// instead of waiting on a global load after the partials' barrier; no registers are held across the
// step (an early global read into VGPRs spilled, §4.r4)
// Only where it measured faster (profiles/r04/term/ab_gw_dma.txt): not in GGTV's instance (MODE 2, the
// register-heaviest: the ring costs it spills) nor in the one-strip 4-column instances (W = 256, 3-4 %
// slower); 12 % faster at W = 128, 7 % at W = 512 (strips)
__host__ __device__ constexpr bool term_gw_dma(int mode, int v, bool strips) {
  return mode != 2 && (strips || v < 4);
}
typedef __attribute__((address_space(3))) float* lds_f32_t;
__device__ __forceinline__ void dma_dword(const float* src, float* lds_wave_base) {
  const uint32_t m0v = (uint32_t)(uintptr_t)(lds_f32_t)lds_wave_base;
  asm volatile("global_load_lds_dword %0, off" ::"v"(src), "{m0}"(__builtin_amdgcn_readfirstlane(m0v)) : "memory");
}
// PADJ: no v_out; the x-gradient pass that follows it (gx += scale[g] P*(v), grr_bwd_stencil mode 3 /
// padj2) runs in the kernel one row behind v: v rows go to an LDS ring (P* reaches one row and one
// column), gx rows come one row ahead by LDS-DMA, and each segment computes v for the rows either side
// of it (their weight-gradient partials and reductions are not taken).
//
// RING (round 5): every operand row reaches the channel waves through an LDS ring filled by one extra
// producer wave (wave F) with 16-byte LDS-DMA, ring_d - 1 steps ahead: per step the x and g rows of the
// F channels, the graph's WPL weight rows and the WPL gw rows of the read-modify-write.  The channel
// waves issue no loads in the row loop (no prefetch registers, no load latency on their path): the
// register-prefetch kernel was latency-bound (one row of prefetch; waves waiting 59 % of their cycles,
// sq_term_row_512.json).  Each step has exactly one barrier (the partials'), which the producer joins:
// it waits (counted vmcnt) until the next step's rows have landed, passes the barrier, then refills the
// slot the previous step read.  Column strips (W > 64 V) start on 16-byte boundaries: 64 V - 8 owned
// columns, 4 halo columns per side.  Same arithmetic, same order: results equal the non-ring kernel's.
constexpr int kRingRows(int V) { return 4 / V; }   // rows one 64-lane 16-byte DMA moves
// scalar base + a loop-invariant per-lane byte offset: the VGPR operand is never rewritten while DMAs that
// read it are in flight (a rewritten address VGPR drew compiler vmcnt(0) waits inside the issue loop)
__device__ __forceinline__ void dma_row16(const float* sbase, uint32_t voff, float* lds_dst) {
  const uint32_t m0v = (uint32_t)(uintptr_t)(lds_f32_t)lds_dst;
  asm volatile("global_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "{m0}"(__builtin_amdgcn_readfirstlane(m0v))
               : "memory");
}
// s_waitcnt vmcnt(n) for a wave-uniform run-time n (the immediate is 6 bits)
__device__ __forceinline__ void vm_wait_rt(int n) {
  switch (n) {
#define GRR_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    GRR_VMW(0) GRR_VMW(1) GRR_VMW(2) GRR_VMW(3) GRR_VMW(4) GRR_VMW(5) GRR_VMW(6) GRR_VMW(7) GRR_VMW(8)
    GRR_VMW(9) GRR_VMW(10) GRR_VMW(11) GRR_VMW(12) GRR_VMW(13) GRR_VMW(14) GRR_VMW(15) GRR_VMW(16)
    GRR_VMW(17) GRR_VMW(18) GRR_VMW(19) GRR_VMW(20) GRR_VMW(21) GRR_VMW(22) GRR_VMW(23) GRR_VMW(24)
    GRR_VMW(25) GRR_VMW(26) GRR_VMW(27) GRR_VMW(28) GRR_VMW(29) GRR_VMW(30) GRR_VMW(31) GRR_VMW(32)
    GRR_VMW(33) GRR_VMW(34) GRR_VMW(35) GRR_VMW(36) GRR_VMW(37) GRR_VMW(38) GRR_VMW(39) GRR_VMW(40)
    GRR_VMW(41) GRR_VMW(42) GRR_VMW(43) GRR_VMW(44) GRR_VMW(45) GRR_VMW(46) GRR_VMW(47) GRR_VMW(48)
    GRR_VMW(49) GRR_VMW(50) GRR_VMW(51) GRR_VMW(52) GRR_VMW(53) GRR_VMW(54) GRR_VMW(55) GRR_VMW(56)
    GRR_VMW(57) GRR_VMW(58) GRR_VMW(59) GRR_VMW(60) GRR_VMW(61) GRR_VMW(62)
#undef GRR_VMW
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
  }
}
__device__ __forceinline__ void ring_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// channel waves per workgroup of the ring kernel: F + 1 <= 8 waves for V = 4 (two per SIMD: 256 VGPRs),
// <= 13 for V <= 2 (128 VGPRs)
template <int V> struct TermRingMax { static constexpr int F = V == 4 ? 7 : 12; };
template <int MODE, int V, bool STRIPS = false, bool PADJ = false, bool RING = false>
__global__ __launch_bounds__(RING ? 64 * (TermRingMax<V>::F + 1) : 64 * TermRowMax<V>::F) void term_row_kernel(
    const float* __restrict__ x, const float* __restrict__ g, const float* __restrict__ taps,
    const float* __restrict__ w, const float* __restrict__ log_gamma, const float* __restrict__ scale, float coef,
    float* __restrict__ v_out, float* __restrict__ gx_out, float* __restrict__ gw, Red ggam, Red gdot,
    Red gtaps, int G, int F, int H, int W, int sseg, int nsegs, uint32_t nblk, int ring_d, int cbeg, int nstr,
    uint32_t slot0) {
  constexpr int WPL = MODE == 1 ? 2 : 4;   // weight planes per graph
  constexpr bool kGwDma = !RING && term_gw_dma(MODE, V, STRIPS);
  // weight-gradient partials [row parity][channel][plane][64 V columns] (dynamic: 2 F WPL 64 V floats),
  // then (term_gw_dma) the gw row ring [row parity][plane][element j][lane] (2 WPL 64 V floats)
  extern __shared__ __attribute__((aligned(16))) float part_dyn[];
  auto part = [&](int pr, int ff, int e) { return part_dyn + ((pr * F + ff) * WPL + e) * (64 * V); };
  auto gring = [&](int pr, int e) { return part_dyn + (2 * F * WPL + pr * WPL + e) * (64 * V); };
  const int lane = threadIdx.x & 63;
  const int f = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // (PADJ) then this wave's v rows [3][64 V] (lane-major) and gx rows [2][element j][lane]; RING: the v rows
  // after the ring's slots (gx rows come in the slots)
  const int ring_fx0 = (F + kRingRows(V) - 1) / kRingRows(V) * kRingRows(V);
  const int ring_wx0 = (WPL + kRingRows(V) - 1) / kRingRows(V) * kRingRows(V);
  const int ring0 = RING ? 2 * F * WPL + ring_d * (2 * (ring_fx0 + ring_wx0) + (PADJ ? ring_fx0 : 0))
                         : 2 * F * WPL + (kGwDma ? 2 * WPL : 0);
  auto vring = [&](int q) { return part_dyn + (ring0 + f * 3 + q % 3) * (64 * V); };
  auto oring = [&](int q) { return part_dyn + (ring0 + 3 * F + f * 2 + (q & 1)) * (64 * V); };
  uint32_t unit = xcd_remap(blockIdx.x, nblk);
  // W > 64 V: column strips owning 62 V columns with V halo columns per side (the term's reach is two
  // columns: s = P x and a = T* g at the pixel's neighbours), as the depthwise row kernels
  // (a separate instance, so that the one-strip kernel keeps its registers).  RING: 64 V - 8 owned
  // columns, 4 halo columns per side (16-byte aligned DMA chunks)
  constexpr int STEP = RING ? 64 * V - 8 : 62 * V;
  constexpr int HALO = RING ? 4 : V;
  // (STRIPS) nstr strips owning columns cbeg + STEP s ..; a launch may cover only part of the row (the
  // ring kernel's narrow tail launch, launch_term_row)
  int strip = 0, nstrips = 1;
  if constexpr (STRIPS) {
    nstrips = nstr;
    strip = (int)(unit % (uint32_t)nstrips);
    unit /= (uint32_t)nstrips;
  }
  const int seg = unit % nsegs;
  const int bg = unit / nsegs, gi = bg % G;
  const int r0 = seg * sseg, r1 = min(r0 + sseg, H);
  const int rs = PADJ ? max(r0 - 1, 0) : r0, re = PADJ ? min(r1 + 1, H) : r1;   // rows whose v is formed
  const int lc0 = V * lane;                  // the lane's slot in the LDS partial rows
  int c0 = lc0;                              // global column
  bool on = c0 < W;
  int cl0 = on ? c0 : W - V;
  int x0 = 0;                                // the strip's first column
  if constexpr (STRIPS) {
    const int lo = cbeg + strip * STEP, hi = min(lo + STEP, W);
    x0 = lo == 0 ? 0 : lo - HALO;
    c0 = x0 + lc0;
    on = c0 >= lo && c0 < hi;
    cl0 = clampi(c0, 0, W - V);
  }
  const int64_t HW = (int64_t)H * W;
  // RING: rows per ring slot (x, g of the F channels, WPL weight rows, WPL gw rows, (PADJ) the F channels'
  // gx rows; each block padded to whole DMAs)
  const int ring_fx = ring_fx0, ring_wx = ring_wx0;   // x, g (gx) / w, gw block rows
  const int ring_rows = 2 * (ring_fx + ring_wx) + (PADJ ? ring_fx : 0);
  float* const ring = part_dyn + 2 * F * WPL * (64 * V);
  auto rslot = [&](int sl) { return ring + sl * ring_rows * (64 * V); };
  const int t0 = rs - 1, te = re + 1;        // the row loop's steps (output row t - 2)
  if constexpr (RING) {
    if (f == F) {   // producer: the operand rows of step t into slot (t - t0) mod ring_d
      // The slot's rows come in four blocks (x, g: F rows each; w, gw: WPL rows each), each padded to
      // whole DMAs of RPD = 4 / V rows (16 V lanes per row): DMA q of a block moves its rows q RPD ..
      // q RPD + RPD - 1, the lane row sub's 16-byte chunk ck.  Scalar base: the block's plane q RPD at
      // the step's row; per-lane offset: plane sub and the column (the last DMA of a block clamps the
      // plane: padding rows repeat the block's last row).  The w block's plane 0 (MODE 0 / 2) is the
      // row t - 1 one: its own scalar row at V = 4, one row down in the lane offset at V < 4.
      constexpr int RPD = kRingRows(V);
      const int sub = lane / (16 * V), ck = lane % (16 * V);
      const int col = min(x0 + 4 * ck, W - 4);
      const int nfx = (F + RPD - 1) / RPD, nfw = (WPL + RPD - 1) / RPD;
      auto lane_off = [&](int q, int np) {
        return (uint32_t)(((min(q * RPD + sub, np - 1) - q * RPD) * HW + col) * 4);
      };
      const uint32_t vo_main = (uint32_t)((sub * HW + col) * 4);
      const uint32_t vo_lastf = lane_off(nfx - 1, F), vo_lastw = lane_off(nfw - 1, WPL);
      constexpr bool kLag1 = MODE != 1;
      // V < 4: the DMA holding plane 0 reads row clamp(t - 2) + delta at lane row 0, delta = clamp(t - 1) -
      // clamp(t - 2) in {0, 1} (uniform per step: one of two loop-invariant offsets)
      const uint32_t vo_w0 = nfw == 1 ? vo_lastw : vo_main;
      const uint32_t vo_w0d = vo_w0 + ((V < 4 && kLag1 && sub == 0) ? (uint32_t)W * 4u : 0u);
      const float* const xb = x + (int64_t)bg * F * HW;
      const float* const gb = g + (int64_t)bg * F * HW;
      const float* const wb0 = w + (int64_t)bg * WPL * HW;
      const float* const gwb0 = gw + (int64_t)bg * WPL * HW;
      const float* const gxb = PADJ ? gx_out + (int64_t)bg * F * HW : nullptr;
      const int64_t qstep = (int64_t)RPD * HW;   // floats between consecutive DMAs of a block
      auto issue = [&](int t, int sl) {
        float* dst = rslot(sl);
        constexpr int DS = RPD * (64 * V);
        const int64_t ro0 = (int64_t)clampi(t, 0, H - 1) * W, ro2 = (int64_t)clampi(t - 2, 0, H - 1) * W;
        // x, g: rows t
        for (int q = 0; q < nfx - 1; ++q, dst += DS) dma_row16(xb + q * qstep + ro0, vo_main, dst);
        dma_row16(xb + (nfx - 1) * qstep + ro0, vo_lastf, dst);
        dst += DS;
        for (int q = 0; q < nfx - 1; ++q, dst += DS) dma_row16(gb + q * qstep + ro0, vo_main, dst);
        dma_row16(gb + (nfx - 1) * qstep + ro0, vo_lastf, dst);
        dst += DS;
        // w: rows t - 2 (plane 0 of MODE 0 / 2: t - 1)
        const int64_t ro_w0 = (V == 4 && kLag1) ? (int64_t)clampi(t - 1, 0, H - 1) * W : ro2;
        if (V < 4 && kLag1 && clampi(t - 1, 0, H - 1) != clampi(t - 2, 0, H - 1)) dma_row16(wb0 + ro_w0, vo_w0d, dst);
        else dma_row16(wb0 + ro_w0, vo_w0, dst);
        dst += DS;
        for (int q = 1; q < nfw - 1; ++q, dst += DS) dma_row16(wb0 + q * qstep + ro2, vo_main, dst);
        if (nfw > 1) {
          dma_row16(wb0 + (nfw - 1) * qstep + ro2, vo_lastw, dst);
          dst += DS;
        }
        // gw: rows t - 2
        for (int q = 0; q < nfw - 1; ++q, dst += DS) dma_row16(gwb0 + q * qstep + ro2, vo_main, dst);
        dma_row16(gwb0 + (nfw - 1) * qstep + ro2, vo_lastw, dst);
        if constexpr (PADJ) {   // gx: rows t - 3 (the row P*(v) reaches this step)
          dst += DS;
          const int64_t ro3 = (int64_t)clampi(t - 3, 0, H - 1) * W;
          for (int q = 0; q < nfx - 1; ++q, dst += DS) dma_row16(gxb + q * qstep + ro3, vo_main, dst);
          dma_row16(gxb + (nfx - 1) * qstep + ro3, vo_lastf, dst);
        }
      };
      const int ndma = 2 * nfx + 2 * nfw + (PADJ ? nfx : 0);
      const int D = ring_d;
      for (int k = 0; k < D - 1; ++k) issue(t0 + k, k);
      vm_wait_rt(ndma * (D - 2));   // step t0's rows landed
      ring_barrier();
      int sl = D - 1;
      for (int t = t0; t <= te; ++t) {
        vm_wait_rt(ndma * (D - 3));   // step t + 1's rows landed
        ring_barrier();               // (the partials' barrier of step t)
        issue(t + D - 1, sl);         // the slot step t - 1 read
        sl = sl + 1 == D ? 0 : sl + 1;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
  }
  const float sc = scale ? scale[gi] : 1.f;
  const float gm = MODE == 2 ? expf(log_gamma[gi]) : 0.f;
  float k[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) k[t] = taps[(gi * F + f) * 5 + t];
  const int64_t base = ((int64_t)bg * F + f) * HW + cl0;
  const float* xp = x + base;
  const float* gp = g + base;
  float* vp = PADJ ? nullptr : v_out + base;
  float* gxp = PADJ ? gx_out + base : nullptr;
  const float* wb = w + (int64_t)bg * WPL * HW + cl0;
  float* gwb = gw + (int64_t)bg * WPL * HW + cl0;

  float X[4][V], Gr[4][V], S[3][V], A[3][V];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) X[i][j] = Gr[i][j] = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) S[i][j] = A[i][j] = 0.f;
  // weight rows: MODE 0/2: plane 0 rows r, r+1; plane 3 rows r-1, r; planes 1, 2 row r.
  //              MODE 1:   plane 0 row r; plane 1 rows r-1, r.
  float W0[2][V], W3[2][V], W1[V], W2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) W0[0][j] = W0[1][j] = W3[0][j] = W3[1][j] = W1[j] = W2[j] = 0.f;
  float accT[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, accP[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float dot = 0.f, dgam = 0.f;

  auto xrow = [&](float (&d)[V], int rr) { rload<V>(d, xp + (int64_t)clampi(rr, 0, H - 1) * W); };
  // always one load (a clamped row, zeroed outside the image): the prefetch's load count is fixed, which
  // the counted vmcnt of the gw / gx LDS-DMA rings below relies on (kAfter)
  auto grow = [&](float (&d)[V], int rr) {
    rload<V>(d, gp + (int64_t)clampi(rr, 0, H - 1) * W);
    if (rr < 0 || rr >= H) {
#pragma unroll
      for (int j = 0; j < V; ++j) d[j] = 0.f;
    }
  };
  auto wrow = [&](float (&d)[V], int e, int rr) {   // rows outside the image are never used (selects)
    rload<V>(d, wb + e * HW + (int64_t)clampi(rr, 0, H - 1) * W);
  };
  // prefetched operands of the next step
  float NX[V], NG[V], NW0[V], NW3[V], NW1[V], NW2[V];
  auto prefetch = [&](int t) {   // step t: x, g row t; weights of output row t - 2 (plane 0 row t - 1)
    xrow(NX, t);
    grow(NG, t);
    if constexpr (MODE == 1) {
      wrow(NW0, 0, t - 2);
      wrow(NW3, 1, t - 2);
    } else {
      wrow(NW0, 0, t - 1);
      wrow(NW1, 1, t - 2);
      wrow(NW2, 2, t - 2);
      wrow(NW3, 3, t - 2);
    }
  };
  // fill: steps r0 - 3 .. r0 - 2 (x, g rows; no output)
  xrow(X[2], rs - 3);
  grow(Gr[2], rs - 3);
  xrow(X[3], rs - 2);
  grow(Gr[3], rs - 2);
  if constexpr (MODE != 1) wrow(W0[1], 0, rs - 2);
  // element j of the lane's V columns of gw row rr, plane e -> ring slot rr & 1 (lane-contiguous)
  auto gw_dma = [&](int rr) {
    for (int e = f; e < WPL; e += F)
#pragma unroll
      for (int j = 0; j < V; ++j) dma_dword(gwb + e * HW + (int64_t)rr * W + j, gring(rr & 1, e) + j * 64);
  };
  if constexpr (kGwDma) gw_dma(r0);
  // (PADJ) gx row q += scale P*(v) (grr_bwd_stencil mode 3's expression, term by term), v rows q - 1 .. q + 1
  // from the ring, gx row q from its LDS-DMA slot
  auto padj_row = [&](int q, const float* gx_lane) {   // gx_lane: RING, this lane's V columns of gx row q
    const float* vc = vring(q);
    const bool top = q == 0, bot = q == H - 1;
    float cv[V], uv[V], dv[V];
    rload<V>(cv, vc + lc0);
    if (top) {
#pragma unroll
      for (int j = 0; j < V; ++j) uv[j] = 0.f;
    } else {
      rload<V>(uv, vring(q + 2) + lc0);
    }
    if (bot) {
#pragma unroll
      for (int j = 0; j < V; ++j) dv[j] = 0.f;
    } else {
      rload<V>(dv, vring(q + 1) + lc0);
    }
    const float lv = (c0 > 0 && lane > 0) ? vc[lc0 - 1] : 0.f;
    const float rv = (c0 + V < W && lane < 63) ? vc[lc0 + V] : 0.f;
    const float* os = oring(q) + lane;
    float gq[V];
    if constexpr (RING) {
      rload<V>(gq, gx_lane);
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) gq[j] = os[j * 64];
    }
    float o[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int col = c0 + j;
      const float l = j > 0 ? cv[j - 1] : lv, rr = j < V - 1 ? cv[j + 1] : rv;
      float y = k[0] * cv[j];
      y += k[1] * dv[j]; y += k[2] * rr; y += k[3] * l; y += k[4] * uv[j];
      if (top) y += k[1] * cv[j];
      if (bot) y += k[4] * cv[j];
      if (col == 0) y += k[2] * cv[j];
      if (col == W - 1) y += k[3] * cv[j];
      o[j] = gq[j] + y * sc;
    }
    if (on) rstore<V>(gxp + (int64_t)q * W, o);
  };
  auto gx_dma = [&](int q) {
#pragma unroll
    for (int j = 0; j < V; ++j) dma_dword(gxp + (int64_t)q * W + j, oring(q) + j * 64);
  };
  if constexpr (RING) ring_barrier();   // step t0's rows have landed
  else prefetch(t0);
  int par = 0;
  int sl = 0;   // (RING) this step's ring slot
  for (int t = t0; t <= te; ++t) {
    const float* const slot_lane = rslot(sl) + lc0;
    if constexpr (RING) {
      sl = sl + 1 == ring_d ? 0 : sl + 1;
      rload<V>(NX, slot_lane + f * (64 * V));
      if (t >= 0 && t < H) {
        rload<V>(NG, slot_lane + (ring_fx + f) * (64 * V));
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) NG[j] = 0.f;
      }
      const float* const wr = slot_lane + 2 * ring_fx * (64 * V);
      if constexpr (MODE == 1) {
        rload<V>(NW0, wr);
        rload<V>(NW3, wr + 64 * V);
      } else {
        rload<V>(NW0, wr);
        rload<V>(NW1, wr + 64 * V);
        rload<V>(NW2, wr + 2 * (64 * V));
        rload<V>(NW3, wr + 3 * (64 * V));
      }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
      X[0][j] = X[1][j]; X[1][j] = X[2][j]; X[2][j] = X[3][j]; X[3][j] = NX[j];
      Gr[0][j] = Gr[1][j]; Gr[1][j] = Gr[2][j]; Gr[2][j] = Gr[3][j]; Gr[3][j] = NG[j];
      if constexpr (MODE == 1) {
        W0[0][j] = NW0[j];
        W3[0][j] = W3[1][j]; W3[1][j] = NW3[j];
      } else {
        W0[0][j] = W0[1][j]; W0[1][j] = NW0[j];
        W3[0][j] = W3[1][j]; W3[1][j] = NW3[j];
        W1[j] = NW1[j]; W2[j] = NW2[j];
      }
    }
    if constexpr (!RING) {
      if (t + 1 <= re + 1) prefetch(t + 1);
    }
    // s = P x (replicate) and a = T* g (zero frame) at row t - 1
    {
      const float xp_ = lprev(X[2][V - 1]), xn_ = lnext(X[2][0]);
      const float gp_ = lprev(Gr[2][V - 1]), gn_ = lnext(Gr[2][0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int col = c0 + j;
        const float xl = col > 0 ? (j > 0 ? X[2][j - 1] : xp_) : X[2][j];
        const float xr = col < W - 1 ? (j < V - 1 ? X[2][j + 1] : xn_) : X[2][j];
        const float gl = col > 0 ? (j > 0 ? Gr[2][j - 1] : gp_) : 0.f;
        const float gr = col + 1 < W ? (j < V - 1 ? Gr[2][j + 1] : gn_) : 0.f;
        S[0][j] = S[1][j]; S[1][j] = S[2][j];
        A[0][j] = A[1][j]; A[1][j] = A[2][j];
        S[2][j] = k[0] * X[2][j] + k[1] * X[1][j] + k[2] * xl + k[3] * xr + k[4] * X[3][j];
        A[2][j] = k[0] * Gr[2][j] + k[1] * Gr[1][j] + k[2] * gl + k[3] * gr + k[4] * Gr[3][j];
      }
    }
    const int r = t - 2;
    if (r < rs) {   // pipeline fill (uniform over the workgroup)
      if constexpr (RING) ring_barrier();
      continue;
    }
    const bool own = !PADJ || (r >= r0 && r < r1);   // (PADJ) rows r0 - 1 and r1: v only
    // output row r: s, a rows r-1, r, r+1 = S[0..2]; x, g rows r-1, r, r+1 = X[0..2], Gr[0..2]
    const bool in0 = r > 0, in3 = r + 1 < H;
    const float s_p = lprev(S[1][V - 1]), s_n = lnext(S[1][0]);
    const float a_p = lprev(A[1][V - 1]), a_n = lnext(A[1][0]);
    const float x_p = lprev(X[1][V - 1]), x_n = lnext(X[1][0]);
    const float g_p = lprev(Gr[1][V - 1]), g_n = lnext(Gr[1][0]);
    float w1n = 0.f, w2p = 0.f, c0p = 0.f;
    if constexpr (MODE == 1) c0p = lprev(W0[0][V - 1]);
    else { w1n = lnext(W1[0]); w2p = lprev(W2[V - 1]); }
    float vrow[V], gwa[WPL][V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int col = c0 + j;
      const bool in1 = col > 0, in2 = col + 1 < W;
      const float sv = S[1][j], av = A[1][j];
      float s5[5], a5[5], xt[5], gt5[5];
      s5[0] = sv;
      s5[1] = in0 ? S[0][j] : sv;
      s5[2] = in1 ? (j > 0 ? S[1][j - 1] : s_p) : sv;
      s5[3] = in2 ? (j < V - 1 ? S[1][j + 1] : s_n) : sv;
      s5[4] = in3 ? S[2][j] : sv;
      a5[0] = av;
      a5[1] = in0 ? A[0][j] : av;
      a5[2] = in1 ? (j > 0 ? A[1][j - 1] : a_p) : av;
      a5[3] = in2 ? (j < V - 1 ? A[1][j + 1] : a_n) : av;
      a5[4] = in3 ? A[2][j] : av;
      xt[0] = X[1][j]; xt[1] = X[0][j]; xt[4] = X[2][j];
      xt[2] = in1 ? (j > 0 ? X[1][j - 1] : x_p) : X[1][j];
      xt[3] = in2 ? (j < V - 1 ? X[1][j + 1] : x_n) : X[1][j];
      gt5[0] = Gr[1][j]; gt5[1] = Gr[0][j]; gt5[4] = Gr[2][j];
      gt5[2] = in1 ? (j > 0 ? Gr[1][j - 1] : g_p) : 0.f;
      gt5[3] = in2 ? (j < V - 1 ? Gr[1][j + 1] : g_n) : 0.f;
      float z = 0.f, v = 0.f;
      if constexpr (MODE == 0) {
        const bool in[4] = {in0, in1, in2, in3};
        const float we[4] = {W0[0][j], W1[j], W2[j], W3[1][j]};
        const float wn[4] = {in3 ? W0[1][j] : 0.f, in2 ? (j < V - 1 ? W1[j + 1] : w1n) : 0.f,
                             in1 ? (j > 0 ? W2[j - 1] : w2p) : 0.f, in0 ? W3[0][j] : 0.f};
        float wta = 0.f;
        z = sv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float sn = s5[e + 1];
          z -= we[e] * sn;
          gwa[e][j] = -(av * sn);
          wta += in[3 - e] ? wn[e] * a5[(3 - e) + 1] : 0.f;
          wta += in[e] ? 0.f : we[e] * av;
        }
        v = av - wta;
      } else if constexpr (MODE == 1) {
        const float cr = in2 ? W0[0][j] : 0.f, cl = in1 ? (j > 0 ? W0[0][j - 1] : c0p) : 0.f;
        const float cd = in3 ? W3[1][j] : 0.f, cu = in0 ? W3[0][j] : 0.f;
        const float su = s5[1], sl = s5[2], sr = s5[3], sd = s5[4];
        const float au = a5[1], al = a5[2], ar = a5[3], ad = a5[4];
        z = cr * (sv - sr) + cl * (sv - sl) + cd * (sv - sd) + cu * (sv - su);
        v = cr * (av - ar) + cl * (av - al) + cd * (av - ad) + cu * (av - au);
        gwa[0][j] = (av - ar) * (sv - sr);
        gwa[1][j] = (av - ad) * (sv - sd);
      } else {
        const bool in[4] = {in0, in1, in2, in3};
        const float we[4] = {W0[0][j], W1[j], W2[j], W3[1][j]};
        const float wn[4] = {in3 ? W0[1][j] : 0.f, in2 ? (j < V - 1 ? W1[j + 1] : w1n) : 0.f,
                             in1 ? (j > 0 ? W2[j - 1] : w2p) : 0.f, in0 ? W3[0][j] : 0.f};
        float o = 0.f, gs = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gwa[e][j] = 0.f;
          if (in[e]) {
            const float sn = s5[e + 1], an = a5[e + 1];
            const float ds = sv - sn, tt = we[e] * ds;
            const float ph = 2.f * soft_t(tt, gm) - tt;
            const float da = av - an;
            const float gph = we[e] * da;
            const float gtv = (tt < -gm || tt > gm) ? gph : -gph;
            o += we[e] * ph;
            gs += gtv * we[e];
            gwa[e][j] = ph * da + gtv * ds;
            if (on && own) dgam += gph * (tt < -gm ? 2.f : (tt > gm ? -2.f : 0.f));
          }
          if (in[3 - e]) {
            const float sq = s5[(3 - e) + 1], aq = a5[(3 - e) + 1];
            const float tt = wn[e] * (sq - sv);
            const float ph = 2.f * soft_t(tt, gm) - tt;
            const float gph = wn[e] * (aq - av);
            const float gtv = (tt < -gm || tt > gm) ? gph : -gph;
            o -= wn[e] * ph;
            gs -= gtv * wn[e];
          }
        }
        z = o;
        v = gs;
      }
      const float zz = on && own ? z : 0.f, vv = on && own ? v : 0.f;
      vrow[j] = v;
      dot += av * zz;
#pragma unroll
      for (int tt = 0; tt < 5; ++tt) {
        accT[tt] += zz * gt5[tt];
        accP[tt] += vv * xt[tt];
      }
    }
    if constexpr (PADJ) rstore<V>(vring(r) + lc0, vrow);
    else if (on) rstore<V>(vp + (int64_t)r * W, vrow);
    // weight gradient: partials of the F channels -> LDS -> sum in channel order -> gw
    if (own) {
#pragma unroll
      for (int e = 0; e < WPL; ++e) rstore<V>(part(par, f, e) + lc0, gwa[e]);
      if constexpr (!RING) __syncthreads();
    }
    if constexpr (RING) ring_barrier();   // every step, halo rows included (the producer counts them)
    if constexpr (kGwDma || (PADJ && !RING)) {
      // gw row r / gx row r - 1 landed: copied before this step's prefetch loads, which issue exactly
      // 2 + WPL vector loads (x row, g row -- clamped, never skipped --, WPL weight rows: prefetch()), + the v
      // row store without PADJ; none in the last steps -- the vector memory counter drains in order.  kAfter
      // counts 1 + WPL of them (<= the issued count: a conservative wait)
      constexpr int kAfter = (MODE == 1 ? 3 : 5) + (PADJ ? 0 : 1);
      static_assert(kAfter <= 2 + WPL + (PADJ ? 0 : 1), "kAfter must not exceed the loads issued after the DMA");
      if (t + 1 <= re + 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kAfter) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PADJ ? 0 : 1) : "memory");
    }
    if (own) {
    for (int e = f; e < WPL; e += F) {
      float sum[V];
      rload<V>(sum, part(par, 0, e) + lc0);
      for (int ff = 1; ff < F; ++ff) {
        float pv[V];
        rload<V>(pv, part(par, ff, e) + lc0);
#pragma unroll
        for (int j = 0; j < V; ++j) sum[j] += pv[j];
      }
      if (on) {
        float* dst = gwb + e * HW + (int64_t)r * W;
        float cv[V];
        if constexpr (RING) {
          rload<V>(cv, slot_lane + (2 * ring_fx + ring_wx + e) * (64 * V));
        } else if constexpr (kGwDma) {
          const float* sl = gring(r & 1, e) + lane;
#pragma unroll
          for (int j = 0; j < V; ++j) cv[j] = sl[j * 64];
        } else {
          rload<V>(cv, dst);
        }
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const int col = c0 + j;
          const bool keep = MODE != 1 || (e == 0 ? col + 1 < W : r + 1 < H);
          if (keep) cv[j] += sc * sum[j];
        }
        rstore<V>(dst, cv);
      }
    }
    if constexpr (kGwDma) {
      if (r + 1 < r1) gw_dma(r + 1);
    }
    par ^= 1;
    }
    if constexpr (PADJ) {
      if (r - 1 >= r0 && r - 1 < r1) padj_row(r - 1, slot_lane + (2 * (ring_fx + ring_wx) + f) * (64 * V));
      if constexpr (!RING) {
        if (r >= r0 && r < r1) gx_dma(r);
      }
    }
  }
  if constexpr (PADJ) {
    if (r1 == H) {   // the image's last row: no v row below it
      if constexpr (RING) {
        padj_row(H - 1, gxp + (int64_t)(H - 1) * W);
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        padj_row(H - 1, nullptr);
      }
    }
  }
  // per-graph / per-channel reductions: wave sums into this wave's slots.  Slot of the workgroup:
  // (b, segment, strip); the per-graph scalars take one slot per channel wave of it.
  const uint32_t wslot = slot0 + ((uint32_t)(bg / G) * nsegs + seg) * nstrips + strip;
  {
    const float d = wave_sum(dot);
    if (lane == 0) red_put(gdot, gi, wslot * F + f, coef * d);
  }
  if constexpr (MODE == 2) {
    const float d = wave_sum(dgam);
    if (lane == 0) red_put(ggam, gi, wslot * F + f, sc * d);
  }
#pragma unroll
  for (int tt = 0; tt < 5; ++tt) {
    const float d = wave_sum(accT[tt] + accP[tt]);
    if (lane == 0) red_put(gtaps, (gi * F + f) * 5 + tt, wslot, sc * d);
  }
}

int term_row_vec(int W) {
  if (W <= 64) return 1;
  if (W <= 128 && W % 2 == 0) return 2;
  if (W <= 256 && W % 4 == 0) return 4;
  return 0;
}
// W > 256 runs as column strips (the term's reach is two columns: lanes of V >= 2 columns, a V-column
// halo per side).  The GLR and prox terms on 2-column lanes (124 owned columns per strip: 640 columns
// loaded for W = 512 against 768 with 4-column lanes, and 128 VGPRs, four waves per SIMD), the pair term
// on 4-column lanes (measured, B32 G8 F6 512^2: GLR 4.15 -> 3.64 ms, prox 6.69 -> 4.61, pair 2.88 -> 3.33;
// profiles/r04/term/ab_wide_v.txt); the edge-weight reverse on 4-column lanes
// Round 6 (the LDS-ring kernel with the tail launch, C4 shapes, scripts/term_sweep.py, profiles/r06/tv/): the GLR
// term at W > 256 on 4-column lanes where the ring takes it (F <= 7) without the x-gradient pass (W above the
// pass's width cap: at 4-column lanes that pass no longer fits the ring's LDS) (512^2 F = 6: 2.15 -> 1.97 ms;
// prox unchanged, stays on 2-column lanes), and the ring for the prox term at one-column lanes too (64^2
// F = 12: 0.37 -> 0.24 ms, 0.72 -> 0.41; 32^2: 0.30 -> 0.21).  GRR_TERM_POLICY=0 restores the round-5
// choices (A/B).
static int term_policy() {
  static const int v = [] {
    const char* e = getenv("GRR_TERM_POLICY");
    return e ? atoi(e) : 1;
  }();
  return v;
}
int term_strip_vec(int W, int mode = 1, int F = 0) {
  if (term_row_vec(W)) return term_row_vec(W);
  if (term_policy() != 0 && mode == 0 && W % 4 == 0 && F <= TermRingMax<4>::F && W > g_term_acc_max_w) return 4;
  if (mode != 1 && W % 2 == 0) return 2;
  return W % 4 == 0 ? 4 : 0;
}
// The same reverse as a row-streaming kernel (W <= 64 V, F in {1, 2, 3, 4, 6}): one wave = one
// (b, graph) and a segment of rows, lane = V adjacent columns.  Feature rows r-1..r+1 of the F
// channels, their inverse norms and gsim (4 planes) stay in registers; horizontal neighbours
// come from DPP lane shifts.  feat, w, gw read once, gfeat written once (the per-pixel kernel
// re-reads each feature plane ~12 times through L1/L2, 1.1 TB/s).
template <int F, int V, bool STRIPS = false>
__global__ __launch_bounds__(NT) void edge_row_bwd_kernel(const float* __restrict__ feat, int64_t fstride,
                                                          const float* __restrict__ multiM,
                                                          const float* __restrict__ w, const float* __restrict__ gw,
                                                          float* __restrict__ gfeat, int64_t gstride,
                                                          Red gM, int G, int H, int W, int sseg,
                                                          int nsegs, uint32_t nwaves) {
  const int lane = threadIdx.x & 63;
  const uint32_t wid = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (wid >= nwaves) return;   // whole waves; no barriers below
  // STRIPS (W > 64 V): 62 V owned columns per wave with V halo columns per side (reach: one column),
  // as term_row_kernel
  uint32_t unit = wid;
  int strip = 0, nstrips = 1;
  constexpr int STEP = 62 * V;
  if constexpr (STRIPS) {
    nstrips = (W + STEP - 1) / STEP;
    strip = (int)(unit % (uint32_t)nstrips);
    unit /= (uint32_t)nstrips;
  }
  const int seg = (int)(unit % nsegs);
  const int bg = (int)(unit / nsegs), g = bg % G, b = bg / G;
  const int r0 = seg * sseg, r1 = min(r0 + sseg, H);
  int c0 = V * lane;
  bool on = c0 < W;
  int cl0 = on ? c0 : W - V;
  if constexpr (STRIPS) {
    const int x0 = strip == 0 ? 0 : strip * STEP - V;
    const int lo = strip * STEP, hi = min(lo + STEP, W);
    c0 = x0 + V * lane;
    on = c0 >= lo && c0 < hi;
    cl0 = clampi(c0, 0, W - V);
  }
  const int64_t HW = (int64_t)H * W;
  const float* fp = feat + (int64_t)b * fstride + (int64_t)g * F * HW + cl0;
  float* gfp = gfeat + (int64_t)b * gstride + (int64_t)g * F * HW + cl0;
  const float* wb = w + (int64_t)bg * 4 * HW + cl0;
  const float* gwb = gw + (int64_t)bg * 4 * HW + cl0;
  float M[F];
#pragma unroll
  for (int f = 0; f < F; ++f) M[f] = multiM[g * F + f];
  float gm[F];
#pragma unroll
  for (int f = 0; f < F; ++f) gm[f] = 0.f;

  // windows: rows t-2, t-1, t (slot 0, 1, 2)
  float FE[3][F][V], IC[3][V], GS[3][4][V];
  auto load_row = [&](int slot, int rr) {
    const int64_t ro = (int64_t)clampi(rr, 0, H - 1) * W;
    float ss[V];
#pragma unroll
    for (int j = 0; j < V; ++j) ss[j] = 0.f;
#pragma unroll
    for (int f = 0; f < F; ++f) {
      rload<V>(FE[slot][f], fp + f * HW + ro);
#pragma unroll
      for (int j = 0; j < V; ++j) ss[j] += FE[slot][f][j] * FE[slot][f][j];
    }
#pragma unroll
    for (int j = 0; j < V; ++j) IC[slot][j] = 1.f / fmaxf(sqrtf(ss[j]), 1e-12f);
    float wv[4][V], gv[4][V];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      rload<V>(wv[e], wb + e * HW + ro);
      rload<V>(gv[e], gwb + e * HW + ro);
    }
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float s = wv[0][j] * gv[0][j] + wv[1][j] * gv[1][j] + wv[2][j] * gv[2][j] + wv[3][j] * gv[3][j];
#pragma unroll
      for (int e = 0; e < 4; ++e) GS[slot][e][j] = wv[e][j] * (gv[e][j] - s);
    }
  };
  auto shift = [&]() {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        IC[k][j] = IC[k + 1][j];
#pragma unroll
        for (int f = 0; f < F; ++f) FE[k][f][j] = FE[k + 1][f][j];
#pragma unroll
        for (int e = 0; e < 4; ++e) GS[k][e][j] = GS[k + 1][e][j];
      }
    }
  };
  load_row(1, r0 - 1);
  load_row(2, r0);
  for (int r = r0; r < r1; ++r) {
    shift();
    load_row(2, r + 1);
    // output row r: rows r-1, r, r+1 in slots 0, 1, 2
    const bool in0 = r > 0, in3 = r + 1 < H;
    float gout[F][V];
    const float icp = lprev(IC[1][V - 1]), icn = lnext(IC[1][0]);
    const float g1n = lnext(GS[1][1][0]), g2p = lprev(GS[1][2][V - 1]);
    float fpv[F], fnx[F];
#pragma unroll
    for (int f = 0; f < F; ++f) { fpv[f] = lprev(FE[1][f][V - 1]); fnx[f] = lnext(FE[1][f][0]); }
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int col = c0 + j;
      const bool in1 = col > 0, in2 = col + 1 < W;
      const bool in[4] = {in0, in1, in2, in3};
      const float ic = IC[1][j];
      const float icl = j > 0 ? IC[1][j - 1] : icp, icr = j < V - 1 ? IC[1][j + 1] : icn;
      const float inb[4] = {in0 ? IC[0][j] : ic, in1 ? icl : ic, in2 ? icr : ic, in3 ? IC[2][j] : ic};
      float gs_out[4], gs_in[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) gs_out[e] = GS[1][e][j];
      gs_in[0] = in3 ? GS[2][0][j] : 0.f;                                  // edge up of the pixel below
      gs_in[1] = in2 ? (j < V - 1 ? GS[1][1][j + 1] : g1n) : 0.f;          // edge left of the right pixel
      gs_in[2] = in1 ? (j > 0 ? GS[1][2][j - 1] : g2p) : 0.f;              // edge right of the left pixel
      gs_in[3] = in0 ? GS[0][3][j] : 0.f;                                  // edge down of the pixel above
      float gsum = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) gsum += in[e] ? 0.f : gs_out[e];
      float gfh[F], ndg = 0.f;
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const float m = M[f];
        const float xc = FE[1][f][j];
        const float n = xc * ic;
        // feature f at the 4 (clamped) neighbours: up, left, right, down
        const float xl = j > 0 ? FE[1][f][j - 1] : fpv[f], xr = j < V - 1 ? FE[1][f][j + 1] : fnx[f];
        const float xn[4] = {in0 ? FE[0][f][j] : xc, in1 ? xl : xc, in2 ? xr : xc, in3 ? FE[2][f][j] : xc};
        float v = gsum * n * m;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v += gs_out[e] * xn[e] * inb[e] * m;
          if (in[3 - e]) v += gs_in[e] * xn[3 - e] * inb[3 - e] * m;
        }
        gfh[f] = v;
        if (on) gm[f] += v * n;
        ndg += n * (v * m);
      }
      const bool small = 1.f / ic <= 1e-12f;
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const float n = FE[1][f][j] * ic;
        const float gn = gfh[f] * M[f];
        gout[f][j] = small ? gn * ic : (gn - n * ndg) * ic;
      }
    }
    if (on) {
#pragma unroll
      for (int f = 0; f < F; ++f) rstore<V>(gfp + f * HW + (int64_t)r * W, gout[f]);
    }
  }
  const uint32_t wslot = ((uint32_t)b * nsegs + seg) * nstrips + strip;   // (b, segment, strip)
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const float s = wave_sum(gm[f]);
    if (lane == 0) red_put(gM, g * F + f, wslot, s);
  }
}

bool edge_row_bwd_ok(const float* feat, int64_t fstride, const float* w, const float* gw, float* gfeat,
                     int64_t gstride, int F, int H, int W) {
  const int V = term_strip_vec(W);
  if (V == 0) return false;
  if (fstride % V != 0 || gstride % V != 0 || ((int64_t)H * W) % V != 0) return false;
  const void* ptrs[] = {feat, w, gw, gfeat};
  for (const void* p : ptrs)
    if ((uintptr_t)p % (4u * V) != 0) return false;
  return F == 1 || F == 2 || F == 3 || F == 4 || F == 6;
}
// launches edge_row_bwd_kernel (edge_row_bwd_ok() holds); gM's partials: one slot per wave
grr_status launch_edge_row_bwd(const float* feat, int64_t fstride, const float* multiM, const float* w,
                               const float* gw, float* gfeat, int64_t gstride, float* gMd, int B, int G, int F, int H,
                               int W, hipStream_t s) {
  const int V = term_strip_vec(W);
  const int nstrips = W <= 64 * V ? 1 : (W + 62 * V - 1) / (62 * V);
  const int64_t planes = (int64_t)B * G * nstrips;   // (b, graph, strip) units
  int sseg = H;
  while (sseg > 32 && planes * ((H + sseg - 1) / sseg) < 4096) sseg = (sseg + 1) / 2;
  const int nsegs = (H + sseg - 1) / sseg;
  const uint32_t nwaves = (uint32_t)(planes * nsegs);
  const dim3 grid((nwaves + NT / 64 - 1) / (NT / 64));
  RedScratch rs(s);
  const int im = rs.plan(gMd, G * F, (uint32_t)((int64_t)B * nsegs * nstrips));
  grr_status st = rs.alloc("grr_bwd_edge_weights");
  if (st != GRR_OK) return st;
  const Red gM = rs.red(im);
#define GRR_EDGE_BWD_CASE(FF, VV)                                                                              \
  if (F == FF && V == VV) {                                                                                    \
    if (nstrips > 1)                                                                                           \
      hipLaunchKernelGGL((edge_row_bwd_kernel<FF, VV, true>), grid, dim3(NT), 0, s, feat, fstride, multiM, w, gw, \
                         gfeat, gstride, gM, G, H, W, sseg, nsegs, nwaves);                                    \
    else                                                                                                       \
      hipLaunchKernelGGL((edge_row_bwd_kernel<FF, VV, false>), grid, dim3(NT), 0, s, feat, fstride, multiM, w, gw, \
                         gfeat, gstride, gM, G, H, W, sseg, nsegs, nwaves);                                    \
  }
  GRR_EDGE_BWD_CASE(1, 4) GRR_EDGE_BWD_CASE(2, 4) GRR_EDGE_BWD_CASE(3, 4) GRR_EDGE_BWD_CASE(4, 4)
  GRR_EDGE_BWD_CASE(6, 4) GRR_EDGE_BWD_CASE(1, 2) GRR_EDGE_BWD_CASE(2, 2) GRR_EDGE_BWD_CASE(3, 2)
  GRR_EDGE_BWD_CASE(4, 2) GRR_EDGE_BWD_CASE(6, 2) GRR_EDGE_BWD_CASE(1, 1) GRR_EDGE_BWD_CASE(2, 1)
  GRR_EDGE_BWD_CASE(3, 1) GRR_EDGE_BWD_CASE(4, 1) GRR_EDGE_BWD_CASE(6, 1)
#undef GRR_EDGE_BWD_CASE
  st = launch_status("grr_bwd_edge_weights");
  if (st != GRR_OK) return st;
  return rs.finish("grr_bwd_edge_weights");
}

// The term reverse's three reductions (gdot, ggamma: per graph; gtaps: per channel and tap), planned
// and allocated once the launch geometry is known
struct TermReds {
  RedScratch rs;
  int id = 0, ig = 0, it = 0;
  explicit TermReds(hipStream_t s) : rs(s) {}
  grr_status setup(int mode, float* gdot, float* ggam, float* gtaps, int G, int F, uint32_t slots_scalar,
                   uint32_t slots_taps) {
    id = rs.plan(gdot, G, slots_scalar);
    ig = rs.plan(mode == 2 ? ggam : nullptr, G, slots_scalar);
    it = rs.plan(gtaps, G * F * 5, slots_taps);
    return rs.alloc("grr_bwd_term_fused");
  }
};

// LDS of one term_row_kernel workgroup: the partials, the gw ring, (PADJ) the v and gx rings
size_t term_row_lds(int mode, int V, int F, bool strips, bool padj) {
  const int wpl = mode == 1 ? 2 : 4;
  const int rows = 2 * F * wpl + (term_gw_dma(mode, V, strips) ? 2 * wpl : 0) + (padj ? 5 * F : 0);
  return (size_t)rows * 64 * V * sizeof(float);
}
constexpr size_t kTermLdsMax = 160 * 1024;
// Shapes the ring kernel takes (g_term_rows == 2): W % 4 == 0 (16-byte DMAs), F + 1 waves within its
// launch bound, and not the one-column lanes where it measured slower for the GLR and pair terms (W <= 32:
// profiles/r05/term/ab_ring_vs_register.txt; the prox term takes the ring there since round 6, term_policy)
bool term_ring_shape_ok(int mode, int F, int W) {
  const int V = term_strip_vec(W, mode, F);
  if (g_term_rows != 2 || V == 0 || W % 4 != 0 || F > (V == 4 ? TermRingMax<4>::F : TermRingMax<1>::F)) return false;
  if (term_policy() == 0) return V >= 2 || (W >= 64 && mode != 2);
  return V >= 2 || W >= 64 || mode == 2;
}
// The ring kernel's depth (steps of rows in LDS) where it applies, else 0: the shape (above) and 16-byte
// aligned planes.  Depth 4 (three steps of rows ahead): deeper rings measured no faster and cost
// workgroups per CU (GRR_TERM_RING_D overrides it for A/B).
// padj: the x-gradient pass inside (gx rows in the slots, three v rows per channel wave after them)
size_t term_ring_lds(int mode, int V, int F, bool padj, int d, int* ndma_out) {
  const int wpl = mode == 1 ? 2 : 4, rpd = 4 / V;
  const int fx = (F + rpd - 1) / rpd, wx = (wpl + rpd - 1) / rpd;
  const int rows = (2 * (fx + wx) + (padj ? fx : 0)) * rpd;
  if (ndma_out) *ndma_out = rows / rpd;
  const size_t row_b = (size_t)64 * V * sizeof(float);
  return (size_t)2 * F * wpl * row_b + (size_t)d * rows * row_b + (padj ? (size_t)3 * F * row_b : 0);
}
int term_ring_setting() {
  static const int forced = [] {
    const char* e = getenv("GRR_TERM_RING_D");
    return e ? atoi(e) : 0;
  }();
  return forced >= 4 ? forced : 4;
}
// the ring's shape-only conditions at depth d: the counted vmcnt of d - 3 steps of DMAs, the LDS
bool term_ring_fits(int mode, int V, int F, bool padj, int d, size_t* lds_out) {
  int ndma = 0;
  const size_t lds = term_ring_lds(mode, V, F, padj, d, &ndma);
  if (lds_out) *lds_out = lds;
  return ndma * (d - 3) <= 63 && lds <= kTermLdsMax;
}
int term_ring_depth(int mode, int V, int F, int W, const float* x, const float* g, const float* w, const float* gw,
                    const float* gx, size_t* lds_out) {
  if (!term_ring_shape_ok(mode, F, W)) return 0;
  const void* ptrs[] = {x, g, w, gw, gx};
  for (const void* p : ptrs)
    if ((uintptr_t)p % 16u != 0) return 0;
  const int d = term_ring_setting();
  size_t lds = 0;
  if (!term_ring_fits(mode, V, F, gx != nullptr, d, &lds)) return 0;
  if (lds_out) *lds_out = lds;
  return d;
}
template <int MODE, int V>
grr_status launch_term_row(int B, int F, const float* x, const float* g, const float* taps, const float* w,
                           const float* lg, const float* scale, float coef, float* v, float* gx, float* gw,
                           float* ggam, float* gdot, float* gtaps, int G, int H, int W, hipStream_t s) {
  size_t ring_lds = 0;
  const int ring_d = g_term_rows == 2 ? term_ring_depth(MODE, V, F, W, x, g, w, gw, gx, &ring_lds) : 0;
  GRR_REQUIRE(ring_d || gx == nullptr || (V < 4 && W <= 64 * V), GRR_ERR_UNSUPPORTED,
              "grr_bwd_term_fused_acc: the x-gradient pass at this width needs the LDS-ring kernel "
              "(16-byte aligned planes, W %% 4 == 0)");
  // rows per workgroup: segments of <= 128 rows, halved further while the grid holds < 2048 waves (floor 32
  // rows).  Round 6 on the ring kernel (C4 shapes, sum of one launch per shape and term,
  // profiles/r06/seg/): 16.19 ms at the round-5 rule (whole planes while >= 8192 waves) against 15.40 here;
  // GRR_TERM_MIN_WAVES / GRR_TERM_MAX_SEG override both (A/B)
  int sseg = H;
  const int step = ring_d ? 64 * V - 8 : 62 * V;   // owned columns per strip
  const int nstrips = W <= 64 * V ? 1 : (W + step - 1) / step;
  const int64_t graphs = (int64_t)B * G * nstrips;   // (b, graph, strip) units
  static const int64_t min_waves = [] {
    const char* e = getenv("GRR_TERM_MIN_WAVES");
    return e ? (int64_t)atoll(e) : (int64_t)2048;
  }();
  static const int max_seg = [] {
    const char* e = getenv("GRR_TERM_MAX_SEG");
    return e ? atoi(e) : 128;
  }();
  while (sseg > 32 && (graphs * F * ((H + sseg - 1) / sseg) < min_waves || sseg > max_seg)) sseg = (sseg + 1) / 2;
  const int nsegs = (H + sseg - 1) / sseg;
  const uint32_t nblk = (uint32_t)(graphs * nsegs);
  const bool padj = gx != nullptr;
  const size_t lds = ring_d ? ring_lds : term_row_lds(MODE, V, F, nstrips > 1, padj);
  // slots: one per (b, segment, strip) workgroup for the taps, one per channel wave of it for the
  // per-graph scalars
  const uint32_t wgs = (uint32_t)((int64_t)B * nsegs * nstrips);
  TermReds R(s);
  grr_status st = R.setup(MODE, gdot, ggam, gtaps, G, F, wgs * F, wgs);
  if (st != GRR_OK) return st;
  // Narrow tail (ring kernel, V > 1): when the last strip owns no more columns than a one-column-lane strip
  // (64 - 8), the row's first nstrips - 1 strips run here and the last one as a V = 1 launch on the same
  // stream (W = 512: 2 x 256 + 64 lane columns instead of 3 x 256 at V = 4, 4 x 128 + 64 instead of 5 x 128
  // at V = 2); its reduction slots follow the main launch's.  Same per-column arithmetic.
  size_t tail_lds = 0;
  const bool tail = ring_d && V > 1 && nstrips > 1 && W - (nstrips - 1) * step <= 56 && g_term_tail &&
                    F <= TermRingMax<1>::F && term_ring_fits(MODE, 1, F, padj, ring_d, &tail_lds);
  const int nmain = tail ? nstrips - 1 : nstrips;
  const uint32_t nblk_main = (uint32_t)((int64_t)B * G * nmain * nsegs);
#define GRR_TERM_ROW_LAUNCH(STRIPS, PADJ)                                                                   \
  hipLaunchKernelGGL((term_row_kernel<MODE, V, STRIPS, PADJ>), dim3(nblk), dim3(64 * F), lds, s, x, g, taps, w, lg, \
                     scale, coef, v, gx, gw, R.rs.red(R.ig), R.rs.red(R.id), R.rs.red(R.it), G, F, H, W, sseg,   \
                     nsegs, nblk, 0, 0, nstrips, 0u)
#define GRR_TERM_RING_LAUNCH(VV, STRIPS, PADJ, NB, LDS, CB, NS, SL0)                                           \
  hipLaunchKernelGGL((term_row_kernel<MODE, VV, STRIPS, PADJ, true>), dim3(NB), dim3(64 * (F + 1)), LDS, s, x, g, \
                     taps, w, lg, scale, coef, v, gx, gw, R.rs.red(R.ig), R.rs.red(R.id), R.rs.red(R.it), G, F, H, \
                     W, sseg, nsegs, NB, ring_d, CB, NS, SL0)
  if (ring_d) {
    if (padj) {
      if (nstrips > 1) GRR_TERM_RING_LAUNCH(V, true, true, nblk_main, lds, 0, nmain, 0u);
      else GRR_TERM_RING_LAUNCH(V, false, true, nblk, lds, 0, 1, 0u);
    } else {
      if (nstrips > 1) GRR_TERM_RING_LAUNCH(V, true, false, nblk_main, lds, 0, nmain, 0u);
      else GRR_TERM_RING_LAUNCH(V, false, false, nblk, lds, 0, 1, 0u);
    }
    if constexpr (V > 1) {
      if (tail) {
        const uint32_t nblk_tail = (uint32_t)((int64_t)B * G * nsegs);
        const uint32_t slot_tail = (uint32_t)((int64_t)B * nsegs * nmain);
        if (padj) GRR_TERM_RING_LAUNCH(1, true, true, nblk_tail, tail_lds, nmain * step, 1, slot_tail);
        else GRR_TERM_RING_LAUNCH(1, true, false, nblk_tail, tail_lds, nmain * step, 1, slot_tail);
      }
    }
  } else if (padj) {
    if constexpr (V < 4) GRR_TERM_ROW_LAUNCH(false, true);   // term_acc_shape_ok: one strip, V <= 2
  } else if (nstrips > 1) {
    GRR_TERM_ROW_LAUNCH(true, false);
  } else {
    GRR_TERM_ROW_LAUNCH(false, false);
  }
#undef GRR_TERM_ROW_LAUNCH
#undef GRR_TERM_RING_LAUNCH
  st = launch_status("grr_bwd_term_fused");
  if (st != GRR_OK) return st;
  return R.rs.finish("grr_bwd_term_fused");
}
bool term_row_ok(int mode, int F, const float* x, const float* g, const float* w, const float* v, const float* gw,
                 int W) {
  const int V = term_strip_vec(W, mode, F);
  if (V == 0 || F > (V == 4 ? TermRowMax<4>::F : TermRowMax<1>::F)) return false;
  const void* ptrs[] = {x, g, w, v, gw};
  for (const void* p : ptrs)
    if ((uintptr_t)p % (4u * V) != 0) return false;
  return true;
}
// the row kernel with the x-gradient pass inside (PADJ) where it measured faster than the kernel + the
// stencil / padj2 pass: one strip of 1- or 2-column lanes (W <= 128; e.g. B16 G32 F3 128^2: 0.467 against
// 0.477 ms for GLR + pair + padj2, prox 0.339 against 0.359).  The 4-column instances (W = 256, strips)
// are at the 168-VGPR cap and spill more with it: GLR + pair 1.75 against 1.67 ms, prox 1.36 against
// 1.22 at B16 G32 F3 256^2 (profiles/r04/term/ab_term_acc.txt).  (Strips would also need V >= 3: P* at
// an owned edge column reads v one halo column out.)
bool term_acc_shape_ok(int mode, int F, int W) {
  const int V = term_strip_vec(W, mode, F);
  if (V == 0 || V == 4 || W > 64 * V || F > TermRowMax<1>::F) return false;
  return term_row_lds(mode, V, F, false, true) <= kTermLdsMax;
}
template <int MODE>
grr_status launch_term_row_v(int B, int F, const float* x, const float* g, const float* taps, const float* w,
                             const float* lg, const float* scale, float coef, float* v, float* gx, float* gw,
                             float* ggam, float* gdot, float* gtaps, int G, int H, int W, hipStream_t s) {
  switch (term_strip_vec(W, MODE, F)) {
    case 1: return launch_term_row<MODE, 1>(B, F, x, g, taps, w, lg, scale, coef, v, gx, gw, ggam, gdot, gtaps, G, H, W, s);
    case 2: return launch_term_row<MODE, 2>(B, F, x, g, taps, w, lg, scale, coef, v, gx, gw, ggam, gdot, gtaps, G, H, W, s);
    default: return launch_term_row<MODE, 4>(B, F, x, g, taps, w, lg, scale, coef, v, gx, gw, ggam, gdot, gtaps, G, H, W, s);
  }
}

template <int MODE>
bool launch_term_fused(int F, dim3 grid, hipStream_t s, const float* x, const float* g, const float* taps,
                       const float* w, const float* lg, const float* scale, float coef, float* v, float* gw,
                       Red ggam, Red gdot, Red gtaps, int G, int H, int W) {
#define GRR_TERM_CASE(FF)                                                                                      \
  case FF:                                                                                                     \
    hipLaunchKernelGGL((term_bwd_fused_kernel<MODE, FF>), grid, dim3(NT), 0, s, x, g, taps, w, lg, scale, coef, \
                       v, gw, ggam, gdot, gtaps, G, H, W);                                                     \
    return true;
  switch (F) {
    GRR_TERM_CASE(1)
    GRR_TERM_CASE(2)
    GRR_TERM_CASE(3)
    GRR_TERM_CASE(4)
    default: return false;   // F > 4: the tap partials spill registers; the multi-pass path is faster there

  }
#undef GRR_TERM_CASE
}

// pixel chunks per plane for the reduction kernels: ~TARGET_BLOCKS blocks in total, so each
// block loops over many pixels and issues few atomics
int chunks_for(int64_t n, int64_t planes) {
  const int64_t want = (TARGET_BLOCKS + planes - 1) / planes;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, (n + NT - 1) / NT));
}
int blocks_for(int64_t n) { return (int)std::min<int64_t>((n + NT - 1) / NT, 1 << 16); }

// dst[i] += sum_s part[i][s] for every planned reduction of a launch, slots in order: lane l adds
// slots l, l + 64, ... in order, then the fixed shuffle tree.   grid (sum of n), one wave per value
struct RedFinishArgs {
  const float* part[RedScratch::kMax];
  float* dst[RedScratch::kMax];
  uint32_t nslot[RedScratch::kMax];
  int first[RedScratch::kMax + 1];   // value ranges of the reductions in the grid
  int k;
};
__global__ __launch_bounds__(64) void red_finish_kernel(RedFinishArgs a) {
  int i = 0;
  while (i + 1 < a.k && (int)blockIdx.x >= a.first[i + 1]) ++i;
  const int idx = blockIdx.x - a.first[i];
  const uint32_t nslot = a.nslot[i];
  const float* row = a.part[i] + (size_t)idx * nslot;
  float v = 0.f;
  for (uint32_t s = threadIdx.x; s < nslot; s += 64) v += row[s];
  v = wave_sum(v);
  if (threadIdx.x == 0) a.dst[i][idx] += v;
}

}  // namespace

// ---- RedScratch (grr_common.h) ---------------------------------------------
// Scratch leases.  Each (device, stream) owns grow-only buffers, each leased by one RedScratch at a time
// (alloc() to finish()); normally one per stream, a second one only while a lease is nested inside
// another on the same stream.  Later calls on the same stream reuse a buffer: their kernels run after
// the earlier finish kernel in stream order.  Memory comes from the allocator registered by
// grr_set_scratch_allocator (the Python package registers PyTorch's caching allocator, so the scratch
// is visible to and reclaimable through torch), else from hipMalloc / hipFree.  An outgrown buffer is
// retired, not freed (a queued kernel may still read it), until grr_release_scratch.
// A lease taken while its stream is being captured into a HIP graph is the graph's own: a
// hipMallocAsync / hipFreeAsync pair on the capturing stream (memory nodes of the graph), never one of
// the stream's buffers, so replays do not share memory with eager calls on that stream or with another
// graph, and grr_release_scratch cannot free memory a graph still points at.
namespace {
struct ScratchBuf {
  int dev;
  hipStream_t s;
  void* p;
  size_t bytes;
  bool cb;        // from the registered allocator
  bool leased;
};
struct ScratchState {
  grr_scratch_alloc_fn alloc = nullptr;
  grr_scratch_free_fn free = nullptr;
  void* ctx = nullptr;
  std::vector<ScratchBuf> bufs;      // live buffers, by (device, stream)
  std::vector<ScratchBuf> retired;   // outgrown, freed by grr_release_scratch
  size_t total = 0;
};
ScratchState g_scratch;
std::mutex g_scratch_mu;
struct CaptureLease {
  void* p;
  hipStream_t s;
};
std::vector<CaptureLease> g_capture_leases;   // leased inside a stream capture, freed by scratch_return

grr_status scratch_raw_alloc(int dev, hipStream_t s, size_t bytes, ScratchBuf* out, const char* what) {
  void* p = nullptr;
  bool cb = false;
  if (g_scratch.alloc) {
    p = g_scratch.alloc((uint64_t)bytes, dev, (void*)s, g_scratch.ctx);
    cb = true;
  } else if (hipMalloc(&p, bytes) != hipSuccess) {
    p = nullptr;
  }
  if (!p) {
    set_error("%s: reduction scratch of %zu bytes: allocation failed", what, bytes);
    return GRR_ERR_HIP;
  }
  *out = ScratchBuf{dev, s, p, bytes, cb, false};
  g_scratch.total += bytes;
  return GRR_OK;
}
void scratch_raw_free(const ScratchBuf& b) {
  if (b.cb) {
    if (g_scratch.free) g_scratch.free(b.p, b.dev, (void*)b.s, g_scratch.ctx);
  } else {
    (void)hipFree(b.p);
  }
  g_scratch.total -= b.bytes;
}

// lease >= bytes for stream s (returned by scratch_return)
grr_status scratch_lease(hipStream_t s, size_t bytes, void** out, const char* what) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    set_error("%s: hipGetDevice failed", what);
    return GRR_ERR_HIP;
  }
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  GRR_REQUIRE(hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusInvalidated,
              GRR_ERR_HIP, "%s: the stream's capture state is invalid", what);
  if (cap == hipStreamCaptureStatusActive) {
    void* p = nullptr;
    if (hipMallocAsync(&p, std::max<size_t>(bytes, 256), s) != hipSuccess || !p) {
      set_error("%s: reduction scratch of %zu bytes inside a stream capture: hipMallocAsync failed", what, bytes);
      return GRR_ERR_HIP;
    }
    g_capture_leases.push_back(CaptureLease{p, s});
    *out = p;
    return GRR_OK;
  }
  ScratchBuf* small = nullptr;
  for (auto& b : g_scratch.bufs) {
    if (b.dev != dev || b.s != s || b.leased) continue;
    if (b.bytes >= bytes) {
      b.leased = true;
      *out = b.p;
      return GRR_OK;
    }
    small = &b;
  }
  size_t want = std::max<size_t>(bytes, (size_t)1 << 20);
  if (small) want = std::max(want, 2 * small->bytes);
  ScratchBuf nb{};
  grr_status st = scratch_raw_alloc(dev, s, want, &nb, what);
  if (st != GRR_OK) return st;
  nb.leased = true;
  if (small) {   // outgrown: retired (queued kernels may still read it), replaced
    g_scratch.retired.push_back(*small);
    *small = nb;
  } else {       // first lease on this stream, or nested inside a live one
    g_scratch.bufs.push_back(nb);
  }
  *out = nb.p;
  return GRR_OK;
}
void scratch_return(void* p) {
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  for (size_t i = 0; i < g_capture_leases.size(); ++i)
    if (g_capture_leases[i].p == p) {   // after the finish kernel on the capturing stream: a free node
      (void)hipFreeAsync(p, g_capture_leases[i].s);
      g_capture_leases.erase(g_capture_leases.begin() + (std::ptrdiff_t)i);
      return;
    }
  for (auto& b : g_scratch.bufs)
    if (b.p == p) b.leased = false;
}
}  // namespace

int RedScratch::plan(float* dst, int n, uint32_t nslot) {
  const int i = k_++;
  dst_[i] = dst;
  n_[i] = n;
  nslot_[i] = nslot < 1 ? 1 : nslot;
  return i;
}

grr_status RedScratch::alloc(const char* what) {
  size_t total = 0;
  for (int i = 0; i < k_; ++i)
    if (dst_[i]) total += (size_t)n_[i] * nslot_[i];
  if (total == 0) return GRR_OK;
  grr_status st = scratch_lease(s_, total * sizeof(float), &base_, what);
  if (st != GRR_OK) {
    base_ = nullptr;
    return st;
  }
  float* p = static_cast<float*>(base_);
  for (int i = 0; i < k_; ++i)
    if (dst_[i]) {
      part_[i] = p;
      p += (size_t)n_[i] * nslot_[i];
    }
  // no fill: every contributor of a launch stores its slot (zero partials included)
  return GRR_OK;
}

grr_status RedScratch::finish(const char* what) {
  RedFinishArgs a{};
  int total = 0;
  for (int i = 0; i < k_; ++i)
    if (dst_[i] && part_[i] && n_[i] > 0) {
      a.part[a.k] = part_[i];
      a.dst[a.k] = dst_[i];
      a.nslot[a.k] = nslot_[i];
      a.first[a.k] = total;
      total += n_[i];
      ++a.k;
    }
  a.first[a.k] = total;
  if (total > 0) hipLaunchKernelGGL(red_finish_kernel, dim3(total), dim3(64), 0, s_, a);
  grr_status st = launch_status(what);
  if (base_) {
    scratch_return(base_);
    base_ = nullptr;
  }
  return st;
}

RedScratch::~RedScratch() {
  if (base_) scratch_return(base_);   // an error path before finish(): nothing was added
}

}  // namespace grr

using namespace grr;

extern "C" {

grr_status grr_set_scratch_allocator(grr_scratch_alloc_fn alloc, grr_scratch_free_fn free_fn, void* ctx) {
  clear_error();
  GRR_REQUIRE((alloc == nullptr) == (free_fn == nullptr), GRR_ERR_INVALID_ARG,
              "grr_set_scratch_allocator: give both functions or neither");
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  // buffers already handed out stay with the allocator that made them (ScratchBuf::cb); a buffer made
  // by the previous registered allocator is freed through the new one only if that is the same pair
  g_scratch.alloc = alloc;
  g_scratch.free = free_fn;
  g_scratch.ctx = ctx;
  return GRR_OK;
}

grr_status grr_release_scratch(void) {
  clear_error();
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  for (const auto& b : g_scratch.bufs)
    GRR_REQUIRE(!b.leased, GRR_ERR_INVALID_ARG, "grr_release_scratch: a reduction scratch is in use");
  for (const auto& b : g_scratch.bufs) scratch_raw_free(b);
  for (const auto& b : g_scratch.retired) scratch_raw_free(b);
  g_scratch.bufs.clear();
  g_scratch.retired.clear();
  return GRR_OK;
}

int64_t grr_scratch_bytes(void) {
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  return (int64_t)g_scratch.total;
}

grr_status grr_bwd_set_term_acc_max_w(int w) {
  clear_error();
  GRR_REQUIRE(w >= 0, GRR_ERR_INVALID_ARG, "grr_bwd_set_term_acc_max_w: w >= 0");
  g_term_acc_max_w = w;
  return GRR_OK;
}

grr_status grr_bwd_set_term_tail(int enable) {
  clear_error();
  GRR_REQUIRE(enable == 0 || enable == 1, GRR_ERR_INVALID_ARG, "grr_bwd_set_term_tail: 0 or 1");
  g_term_tail = enable;
  return GRR_OK;
}

grr_status grr_bwd_set_term_rows(int enable) {
  clear_error();
  GRR_REQUIRE(enable >= 0 && enable <= 2, GRR_ERR_INVALID_ARG, "grr_bwd_set_term_rows: 0, 1 or 2");
  g_term_rows = enable;
  return GRR_OK;
}

grr_status grr_bwd_term_fused(int mode, const float* x, const float* g, const float* taps, const float* w,
                              const float* log_gamma, const float* scale, float coef, float* v_out, float* gw,
                              float* ggamma, float* gdot, float* gtaps, int B, int G, int F, int H, int W,
                              void* stream) {
  clear_error();
  GRR_REQUIRE(x && g && taps && w && v_out && gw && gtaps && B > 0 && G > 0 && F > 0 && H > 0 && W > 0 &&
                  mode >= 0 && mode <= 2 && (mode != 2 || log_gamma),
              GRR_ERR_INVALID_ARG, "grr_bwd_term_fused: bad args");
  hipStream_t s = (hipStream_t)stream;
  // row-streaming kernel where the shape allows
  if (g_term_rows && (int64_t)B * G * H < (1ll << 31) && term_row_ok(mode, F, x, g, w, v_out, gw, W)) {
    switch (mode) {
      case 0: return launch_term_row_v<0>(B, F, x, g, taps, w, log_gamma, scale, coef, v_out, nullptr, gw, ggamma, gdot, gtaps, G, H, W, s);
      case 1: return launch_term_row_v<1>(B, F, x, g, taps, w, log_gamma, scale, coef, v_out, nullptr, gw, ggamma, gdot, gtaps, G, H, W, s);
      default: return launch_term_row_v<2>(B, F, x, g, taps, w, log_gamma, scale, coef, v_out, nullptr, gw, ggamma, gdot, gtaps, G, H, W, s);
    }
  }
  GRR_REQUIRE((int64_t)B * G <= 65535, GRR_ERR_UNSUPPORTED, "grr_bwd_term_fused: B*G > 65535");
  GRR_REQUIRE(F >= 1 && F <= 4, GRR_ERR_UNSUPPORTED,
              "grr_bwd_term_fused: F=%d needs the row kernel (W <= 256 with W %% V == 0, F <= 12 / 16) or F <= 4", F);
  const int chunks = chunks_for((int64_t)H * W, (int64_t)B * G);
  const dim3 grid(chunks, B * G);
  TermReds R(s);
  const uint32_t slots = (uint32_t)B * chunks;   // one per (b, chunk) workgroup
  grr_status st = R.setup(mode, gdot, ggamma, gtaps, G, F, slots, slots);
  if (st != GRR_OK) return st;
  const Red rg = R.rs.red(R.ig), rd = R.rs.red(R.id), rt = R.rs.red(R.it);
  switch (mode) {
    case 0: launch_term_fused<0>(F, grid, s, x, g, taps, w, log_gamma, scale, coef, v_out, gw, rg, rd, rt, G, H, W); break;
    case 1: launch_term_fused<1>(F, grid, s, x, g, taps, w, log_gamma, scale, coef, v_out, gw, rg, rd, rt, G, H, W); break;
    default: launch_term_fused<2>(F, grid, s, x, g, taps, w, log_gamma, scale, coef, v_out, gw, rg, rd, rt, G, H, W);
  }
  st = launch_status("grr_bwd_term_fused");
  if (st != GRR_OK) return st;
  return R.rs.finish("grr_bwd_term_fused");
}

int grr_bwd_term_acc_supported(int mode, int F, int H, int W) {
  // the LDS-ring kernel takes the pass wherever it applies (any width: gx rows come in its slots), the
  // register kernel at one strip of <= 2-column lanes
  // (16-byte aligned planes are the caller's part: kernels.term_acc_ok checks them).  Everything else
  // grr_bwd_term_fused_acc and launch_term_row ask for is checked here, so a shape this accepts with
  // aligned planes never fails with GRR_ERR_UNSUPPORTED: term_row_ok's channel bound, then either the
  // ring (enabled, within the width cap, its DMA count and LDS at the depth it will run) or the
  // register kernel's one strip of <= 2-column lanes
  if (mode < 0 || mode > 2 || F <= 0 || H <= 0 || W <= 0 || !g_term_rows) return 0;
  const int V = term_strip_vec(W, mode, F);
  if (V == 0 || F > (V == 4 ? TermRowMax<4>::F : TermRowMax<1>::F)) return 0;
  if (term_ring_shape_ok(mode, F, W)) {
    if (W > g_term_acc_max_w) return 0;   // the policy cap (wider levels fold the pass into the CG glue)
    if (g_term_rows == 2 && term_ring_fits(mode, V, F, true, term_ring_setting(), nullptr)) return 1;
  }
  return term_acc_shape_ok(mode, F, W) ? 1 : 0;
}

grr_status grr_bwd_term_fused_acc(int mode, const float* x, const float* g, const float* taps, const float* w,
                                  const float* log_gamma, const float* scale, float coef, float* gx, float* gw,
                                  float* ggamma, float* gdot, float* gtaps, int B, int G, int F, int H, int W,
                                  void* stream) {
  clear_error();
  GRR_REQUIRE(x && g && taps && w && gx && gw && gtaps && scale && B > 0 && G > 0 && F > 0 && H > 0 && W > 0 &&
                  mode >= 0 && mode <= 2 && (mode != 2 || log_gamma),
              GRR_ERR_INVALID_ARG, "grr_bwd_term_fused_acc: bad args");
  GRR_REQUIRE(grr_bwd_term_acc_supported(mode, F, H, W) && (int64_t)B * G * H < (1ll << 31) &&
                  term_row_ok(mode, F, x, g, w, gx, gw, W),
              GRR_ERR_UNSUPPORTED, "grr_bwd_term_fused_acc: mode %d F=%d %dx%d needs the row kernel (see "
              "grr_bwd_term_acc_supported) and 4 V-byte aligned planes", mode, F, H, W);
  hipStream_t s = (hipStream_t)stream;
  switch (mode) {
    case 0: return launch_term_row_v<0>(B, F, x, g, taps, w, log_gamma, scale, coef, nullptr, gx, gw, ggamma, gdot, gtaps, G, H, W, s);
    case 1: return launch_term_row_v<1>(B, F, x, g, taps, w, log_gamma, scale, coef, nullptr, gx, gw, ggamma, gdot, gtaps, G, H, W, s);
    default: return launch_term_row_v<2>(B, F, x, g, taps, w, log_gamma, scale, coef, nullptr, gx, gw, ggamma, gdot, gtaps, G, H, W, s);
  }
}

grr_status grr_bwd_stencil(const float* x, const float* taps, int mode, const float* scale, int accumulate,
                           float* out, int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && taps && out && B > 0 && G > 0 && F > 0 && H > 0 && W > 0 && mode >= 0 && mode <= 3,
              GRR_ERR_INVALID_ARG, "grr_bwd_stencil: bad args");
  const int C = G * F;
  GRR_REQUIRE((int64_t)B * C <= 65535 && (int64_t)H * W < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_bwd_stencil: grid too large");
  hipStream_t s = (hipStream_t)stream;
  if (W % 4 == 0 && (uintptr_t)x % 16 == 0 && (uintptr_t)out % 16 == 0) {
    const dim3 g4((H * W / 4 + NT - 1) / NT, B * C);
    switch (mode) {
      case 0: hipLaunchKernelGGL(stencil4_kernel<0>, g4, dim3(NT), 0, s, x, taps, scale, accumulate, out, C, F, H, W); break;
      case 1: hipLaunchKernelGGL(stencil4_kernel<1>, g4, dim3(NT), 0, s, x, taps, scale, accumulate, out, C, F, H, W); break;
      case 2: hipLaunchKernelGGL(stencil4_kernel<2>, g4, dim3(NT), 0, s, x, taps, scale, accumulate, out, C, F, H, W); break;
      default: hipLaunchKernelGGL(stencil4_kernel<3>, g4, dim3(NT), 0, s, x, taps, scale, accumulate, out, C, F, H, W);
    }
    return launch_status("grr_bwd_stencil");
  }
  const dim3 grid((H * W + NT - 1) / NT, B * C);
  switch (mode) {
    case 0: hipLaunchKernelGGL(stencil_kernel<0>, grid, dim3(NT), 0, s, x, taps, scale, accumulate, out, C, F, H, W); break;
    case 1: hipLaunchKernelGGL(stencil_kernel<1>, grid, dim3(NT), 0, s, x, taps, scale, accumulate, out, C, F, H, W); break;
    case 2: hipLaunchKernelGGL(stencil_kernel<2>, grid, dim3(NT), 0, s, x, taps, scale, accumulate, out, C, F, H, W); break;
    default: hipLaunchKernelGGL(stencil_kernel<3>, grid, dim3(NT), 0, s, x, taps, scale, accumulate, out, C, F, H, W);
  }
  return launch_status("grr_bwd_stencil");
}

grr_status grr_bwd_padj2(const float* v1, const float* taps1, const float* scale1, const float* v2, const float* taps2,
                         const float* scale2, float* out, int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(v1 && taps1 && scale1 && v2 && taps2 && scale2 && out && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_bwd_padj2: bad args");
  GRR_REQUIRE(W % 4 == 0 && (uintptr_t)v1 % 16 == 0 && (uintptr_t)v2 % 16 == 0 && (uintptr_t)out % 16 == 0,
              GRR_ERR_UNSUPPORTED, "grr_bwd_padj2: W %% 4 != 0 or planes not 16-byte aligned");
  const int C = G * F;
  GRR_REQUIRE((int64_t)B * C <= 65535 && (int64_t)H * W < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_bwd_padj2: grid too large");
  const dim3 g4((H * W / 4 + NT - 1) / NT, B * C);
  hipLaunchKernelGGL(padj2_kernel, g4, dim3(NT), 0, (hipStream_t)stream, v1, taps1, scale1, v2, taps2, scale2, out, C,
                     F, H, W);
  return launch_status("grr_bwd_padj2");
}

grr_status grr_bwd_tapgrad(const float* u, const float* z, int mode, const float* scale, float* gtaps, int B, int G,
                           int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(u && z && gtaps && B > 0 && G > 0 && F > 0 && H > 0 && W > 0 && (mode == 0 || mode == 1),
              GRR_ERR_INVALID_ARG, "grr_bwd_tapgrad: bad args");
  GRR_REQUIRE((int64_t)B * G * F <= 65535, GRR_ERR_UNSUPPORTED, "grr_bwd_tapgrad: B*G*F > 65535");
  const int chunks = chunks_for((int64_t)H * W, (int64_t)B * G * F);
  const dim3 grid(chunks, B * G * F);
  RedScratch rs((hipStream_t)stream);
  const int it = rs.plan(gtaps, G * F * 5, (uint32_t)B * chunks);
  grr_status st = rs.alloc("grr_bwd_tapgrad");
  if (st != GRR_OK) return st;
  if (mode == 0)
    hipLaunchKernelGGL(tapgrad_kernel<0>, grid, dim3(NT), 0, (hipStream_t)stream, u, z, scale, rs.red(it), G * F, F, H, W);
  else
    hipLaunchKernelGGL(tapgrad_kernel<1>, grid, dim3(NT), 0, (hipStream_t)stream, u, z, scale, rs.red(it), G * F, F, H, W);
  st = launch_status("grr_bwd_tapgrad");
  return st != GRR_OK ? st : rs.finish("grr_bwd_tapgrad");
}

grr_status grr_bwd_glr(const float* s, const float* a, const float* w, const float* scale, float coef, float* z_out,
                       float* ap_out, float* gw, float* gdot, int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(s && a && w && z_out && ap_out && gw && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_bwd_glr: bad args");
  GRR_REQUIRE((int64_t)B * G * F <= 65535, GRR_ERR_UNSUPPORTED, "grr_bwd_glr: B*G*F > 65535");
  const int chunks = chunks_for((int64_t)H * W, (int64_t)B * G);
  RedScratch rs((hipStream_t)stream);
  const int id = rs.plan(gdot, G, (uint32_t)B * chunks);
  grr_status st = rs.alloc("grr_bwd_glr");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(glr_bwd_kernel, dim3(chunks, B * G), dim3(NT), 0, (hipStream_t)stream, s, a, w, scale, coef,
                     z_out, ap_out, gw, rs.red(id), G, F, H, W);
  st = launch_status("grr_bwd_glr");
  return st != GRR_OK ? st : rs.finish("grr_bwd_glr");
}

grr_status grr_bwd_pair(const float* s, const float* a, const float* c, const float* scale, float coef, float* z_out,
                        float* ap_out, float* gc, float* gdot, int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(s && a && c && z_out && ap_out && gc && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_bwd_pair: bad args");
  GRR_REQUIRE((int64_t)B * G * F <= 65535, GRR_ERR_UNSUPPORTED, "grr_bwd_pair: B*G*F > 65535");
  const int chunks = chunks_for((int64_t)H * W, (int64_t)B * G);
  RedScratch rs((hipStream_t)stream);
  const int id = rs.plan(gdot, G, (uint32_t)B * chunks);
  grr_status st = rs.alloc("grr_bwd_pair");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(pair_bwd_kernel, dim3(chunks, B * G), dim3(NT), 0, (hipStream_t)stream, s, a, c, scale, coef,
                     z_out, ap_out, gc, rs.red(id), G, F, H, W);
  st = launch_status("grr_bwd_pair");
  return st != GRR_OK ? st : rs.finish("grr_bwd_pair");
}

grr_status grr_bwd_prox(const float* s, const float* a, const float* w, const float* log_gamma, const float* scale,
                        float coef, float* o_out, float* gs_out, float* gw, float* ggamma, float* gdot, int B, int G,
                        int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(s && a && w && log_gamma && o_out && gs_out && gw && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_bwd_prox: bad args");
  GRR_REQUIRE((int64_t)B * G * F <= 65535, GRR_ERR_UNSUPPORTED, "grr_bwd_prox: B*G*F > 65535");
  const int chunks = chunks_for((int64_t)H * W, (int64_t)B * G);
  RedScratch rs((hipStream_t)stream);
  const int ig = rs.plan(ggamma, G, (uint32_t)B * chunks), id = rs.plan(gdot, G, (uint32_t)B * chunks);
  grr_status st = rs.alloc("grr_bwd_prox");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(prox_bwd_kernel, dim3(chunks, B * G), dim3(NT), 0, (hipStream_t)stream, s, a, w, log_gamma, scale,
                     coef, o_out, gs_out, gw, rs.red(ig), rs.red(id), G, F, H, W);
  st = launch_status("grr_bwd_prox");
  return st != GRR_OK ? st : rs.finish("grr_bwd_prox");
}

grr_status grr_bwd_pair_weights(const float* w, const float* gc, float* gw, int B, int G, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(w && gc && gw && B > 0 && G > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_bwd_pair_weights: bad args");
  GRR_REQUIRE((int64_t)B * G <= 65535, GRR_ERR_UNSUPPORTED, "grr_bwd_pair_weights: B*G > 65535");
  hipLaunchKernelGGL(pair_weights_bwd_kernel, dim3((H * W + NT - 1) / NT, B * G), dim3(NT), 0, (hipStream_t)stream, w,
                     gc, gw, H, W);
  return launch_status("grr_bwd_pair_weights");
}

grr_status grr_bwd_edge_weights(const float* feat, int64_t feat_bstride, const float* multiM, const float* w,
                                const float* gw, float* gfeat, int64_t gfeat_bstride, float* gmultiM, int B, int G,
                                int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(feat && multiM && w && gw && gfeat && gmultiM && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_bwd_edge_weights: bad args");
  GRR_REQUIRE(F <= GRR_MAX_NODE_FTS, GRR_ERR_UNSUPPORTED, "grr_bwd_edge_weights: F=%d > %d", F, GRR_MAX_NODE_FTS);
  if (g_term_rows && edge_row_bwd_ok(feat, feat_bstride, w, gw, gfeat, gfeat_bstride, F, H, W))
    return launch_edge_row_bwd(feat, feat_bstride, multiM, w, gw, gfeat, gfeat_bstride, gmultiM, B, G, F, H, W,
                               (hipStream_t)stream);
  GRR_REQUIRE((int64_t)B * G * F <= 65535, GRR_ERR_UNSUPPORTED, "grr_bwd_edge_weights: B*G*F > 65535");
  const int chunks = chunks_for((int64_t)H * W, (int64_t)B * G);
  RedScratch rs((hipStream_t)stream);
  const int im = rs.plan(gmultiM, G * F, (uint32_t)B * chunks);
  grr_status st = rs.alloc("grr_bwd_edge_weights");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(edge_weights_bwd_kernel, dim3(chunks, B * G), dim3(NT), 0, (hipStream_t)stream, feat,
                     feat_bstride, multiM, w, gw, gfeat, gfeat_bstride, rs.red(im), G, F, H, W);
  st = launch_status("grr_bwd_edge_weights");
  return st != GRR_OK ? st : rs.finish("grr_bwd_edge_weights");
}

grr_status grr_bwd_graph_dot(const float* u, const float* v, float coef, float* gdot, int B, int G, int F, int H,
                             int W, void* stream) {
  clear_error();
  GRR_REQUIRE(u && v && gdot && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_bwd_graph_dot: bad args");
  GRR_REQUIRE((int64_t)B * G * F <= 65535, GRR_ERR_UNSUPPORTED, "grr_bwd_graph_dot: B*G*F > 65535");
  const int64_t n = (int64_t)F * H * W;
  const bool v4 = n % 4 == 0 && ((uintptr_t)u & 15) == 0 && ((uintptr_t)v & 15) == 0;
  const int chunks = chunks_for(v4 ? n / 4 : n, (int64_t)B * G);
  const dim3 grid(chunks, B * G);
  RedScratch rs((hipStream_t)stream);
  const int id = rs.plan(gdot, G, (uint32_t)B * chunks);
  grr_status st = rs.alloc("grr_bwd_graph_dot");
  if (st != GRR_OK) return st;
  if (v4)
    hipLaunchKernelGGL(graph_dot_kernel<true>, grid, dim3(NT), 0, (hipStream_t)stream, u, v, coef, rs.red(id), G, F,
                       (int64_t)H * W);
  else
    hipLaunchKernelGGL(graph_dot_kernel<false>, grid, dim3(NT), 0, (hipStream_t)stream, u, v, coef, rs.red(id), G, F,
                       (int64_t)H * W);
  st = launch_status("grr_bwd_graph_dot");
  return st != GRR_OK ? st : rs.finish("grr_bwd_graph_dot");
}

static grr_status cg_glue_impl(const float* gx, const float* gx_half, const float* v1, const float* taps1,
                               const float* scale1, const float* v2, const float* taps2, const float* scale2,
                               const float* u, const float* gu_next, const float* u_prev, const float* alpha,
                               const float* beta_next, float* gu, float* gbb, float* gx_out, float* gu_half,
                               float* galpha, float* gbeta, int B, int G, int F, int H, int W, void* stream) {
  GRR_REQUIRE(gx && u && alpha && gu && gx_out && galpha && (!gu_next || beta_next) && (!u_prev || gbeta) && B > 0 &&
                  G > 0 && F > 0 && H > 0 && W > 0 && (!gx_half || (H % 2 == 0 && W % 2 == 0)),
              GRR_ERR_INVALID_ARG, "grr_bwd_cg_glue: bad args");
  GRR_REQUIRE(!v1 == !v2 && (!v1 || (taps1 && scale1 && taps2 && scale2)), GRR_ERR_INVALID_ARG,
              "grr_bwd_cg_glue: v1, v2 with their taps and scales, or neither");
  GRR_REQUIRE((int64_t)B * G <= 65535 && (int64_t)F * H * W < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_bwd_cg_glue: B*G > 65535 or a (b, graph) slab of 2^31 floats");
  const int64_t n = (int64_t)F * H * W;
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  const bool v4 = n % 4 == 0 && al16(gx) && al16(u) && al16(gu) && al16(gx_out) && (!gu_next || al16(gu_next)) &&
                  (!u_prev || al16(u_prev)) && (!gbb || al16(gbb)) &&
                  (!gx_half || (W % 4 == 0 && ((uintptr_t)gx_half & 7) == 0)) &&
                  (!v1 || (W % 4 == 0 && al16(v1) && al16(v2)));
  GRR_REQUIRE(!v1 || v4, GRR_ERR_UNSUPPORTED,
              "grr_bwd_cg_glue: the x-gradient pass needs W %% 4 == 0 and 16-byte aligned planes (W = %d)", W);
  GRR_REQUIRE(!gu_half || (v4 && W % 4 == 0 && H % 2 == 0 && ((uintptr_t)gu_half & 7) == 0), GRR_ERR_UNSUPPORTED,
              "grr_bwd_cg_glue_pool: needs W %% 4 == 0, even H, 16-byte aligned planes, 8-byte aligned gu_half (H %d, W %d)", H, W);
  const GluePadj pj{v1, taps1, scale1, v2, taps2, scale2};
  const int chunks = chunks_for(v4 ? n / (gu_half ? 8 : 4) : n, (int64_t)B * G);
  const dim3 grid(chunks, B * G);
  RedScratch rs((hipStream_t)stream);
  const int ia = rs.plan(galpha, G, (uint32_t)B * chunks), ib = rs.plan(u_prev ? gbeta : nullptr, G, (uint32_t)B * chunks);
  grr_status st = rs.alloc("grr_bwd_cg_glue");
  if (st != GRR_OK) return st;
  if (v4)
    hipLaunchKernelGGL(cg_glue_kernel<true>, grid, dim3(NT), 0, (hipStream_t)stream, gx, gx_half, pj, F, u, gu_next,
                       u_prev, alpha, beta_next, gu, gbb, gx_out, gu_half, rs.red(ia), rs.red(ib), G, n, H, W);
  else
    hipLaunchKernelGGL(cg_glue_kernel<false>, grid, dim3(NT), 0, (hipStream_t)stream, gx, gx_half, pj, F, u, gu_next,
                       u_prev, alpha, beta_next, gu, gbb, gx_out, nullptr, rs.red(ia), rs.red(ib), G, n, H, W);
  st = launch_status("grr_bwd_cg_glue");
  return st != GRR_OK ? st : rs.finish("grr_bwd_cg_glue");
}

grr_status grr_bwd_cg_glue(const float* gx, const float* gx_half, const float* v1, const float* taps1,
                           const float* scale1, const float* v2, const float* taps2, const float* scale2,
                           const float* u, const float* gu_next, const float* u_prev, const float* alpha,
                           const float* beta_next, float* gu, float* gbb, float* gx_out, float* galpha, float* gbeta,
                           int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  return cg_glue_impl(gx, gx_half, v1, taps1, scale1, v2, taps2, scale2, u, gu_next, u_prev, alpha, beta_next, gu,
                      gbb, gx_out, nullptr, galpha, gbeta, B, G, F, H, W, stream);
}

grr_status grr_bwd_cg_glue_pool(const float* gx, const float* gx_half, const float* v1, const float* taps1,
                                const float* scale1, const float* v2, const float* taps2, const float* scale2,
                                const float* u, const float* gu_next, const float* u_prev, const float* alpha,
                                const float* beta_next, float* gu, float* gbb, float* gx_out, float* gu_half,
                                float* galpha, float* gbeta, int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(gu_half, GRR_ERR_INVALID_ARG, "grr_bwd_cg_glue_pool: gu_half required");
  return cg_glue_impl(gx, gx_half, v1, taps1, scale1, v2, taps2, scale2, u, gu_next, u_prev, alpha, beta_next, gu,
                      gbb, gx_out, gu_half, galpha, gbeta, B, G, F, H, W, stream);
}

grr_status grr_bwd_lincomb(const float* x, const float* sa, const float* y, const float* sb, float* out,
                           int accumulate, int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && out && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_bwd_lincomb: bad args");
  GRR_REQUIRE((int64_t)B * G <= 65535, GRR_ERR_UNSUPPORTED, "grr_bwd_lincomb: B*G > 65535");
  const int64_t n = (int64_t)F * H * W;   // one (b, graph) slab
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  const bool v4 = n % 4 == 0 && al16(x) && al16(out) && (!y || al16(y));
  const dim3 grid(chunks_for(v4 ? n / 4 : n, (int64_t)B * G), B * G);
  if (v4)
    hipLaunchKernelGGL(lincomb_kernel<true>, grid, dim3(NT), 0, (hipStream_t)stream, x, sa, y, sb, out, accumulate, G,
                       n);
  else
    hipLaunchKernelGGL(lincomb_kernel<false>, grid, dim3(NT), 0, (hipStream_t)stream, x, sa, y, sb, out, accumulate,
                       G, n);
  return launch_status("grr_bwd_lincomb");
}

grr_status grr_bwd_unpool2_acc(const float* xd, float* out, int B, int C, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(xd && out && B > 0 && C > 0 && H > 1 && W > 1, GRR_ERR_INVALID_ARG, "grr_bwd_unpool2_acc: bad args");
  GRR_REQUIRE(H % 2 == 0 && W % 2 == 0, GRR_ERR_SHAPE, "grr_bwd_unpool2_acc: H, W must be even");
  const int64_t n = (int64_t)B * C * H * W;
  if (W % 4 == 0 && (int64_t)B * C <= 65535 && (int64_t)H * W < (1ll << 31) && ((uintptr_t)xd & 7) == 0 &&
      ((uintptr_t)out & 15) == 0) {
    const dim3 grid(chunks_for((int64_t)H * W / 4, (int64_t)B * C), B * C);
    hipLaunchKernelGGL(unpool2_acc4_kernel, grid, dim3(NT), 0, (hipStream_t)stream, xd, out, H, W);
  } else {
    hipLaunchKernelGGL(unpool2_acc_kernel, dim3(blocks_for(n)), dim3(NT), 0, (hipStream_t)stream, xd, out, H, W, n);
  }
  return launch_status("grr_bwd_unpool2_acc");
}

grr_status grr_interleave2x2(const float* t, float* gx, int B, int K, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(t && gx && t != gx && B > 0 && K > 0 && H > 1 && W > 1, GRR_ERR_INVALID_ARG,
              "grr_interleave2x2: bad args");
  GRR_REQUIRE(H % 2 == 0 && W % 4 == 0, GRR_ERR_SHAPE, "grr_interleave2x2: H even and W %% 4 == 0 required");
  GRR_REQUIRE(((uintptr_t)t & 7) == 0 && ((uintptr_t)gx & 15) == 0, GRR_ERR_INVALID_ARG,
              "grr_interleave2x2: t 8-byte / gx 16-byte alignment required");
  const int64_t nq = (int64_t)B * K * H * (W / 4);
  hipLaunchKernelGGL(interleave2x2_kernel, dim3(blocks_for(nq)), dim3(NT), 0, (hipStream_t)stream, t, gx, K, H, W, nq);
  return launch_status("grr_interleave2x2");
}

grr_status grr_conv2x2s2_bwd_data(const float* g, const float* wt, float* gx, int B, int K, int M, int H, int W,
                                  void* stream) {
  clear_error();
  GRR_REQUIRE(g && wt && gx && B > 0 && K > 0 && M > 0 && H > 1 && W > 1, GRR_ERR_INVALID_ARG,
              "grr_conv2x2s2_bwd_data: bad args");
  GRR_REQUIRE(H % 2 == 0 && W % 2 == 0, GRR_ERR_SHAPE, "grr_conv2x2s2_bwd_data: H, W must be even");
  GRR_REQUIRE((int64_t)B * K <= 65535, GRR_ERR_UNSUPPORTED, "grr_conv2x2s2_bwd_data: grid too large");
  hipLaunchKernelGGL(conv2x2s2_bwd_data_kernel, dim3((H * W + NT - 1) / NT, B * K), dim3(NT), 0, (hipStream_t)stream,
                     g, wt, gx, K, M, H, W);
  return launch_status("grr_conv2x2s2_bwd_data");
}

}  // extern "C"
