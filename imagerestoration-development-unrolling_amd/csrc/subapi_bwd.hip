// Reverses of the GLRFast / GTVFast sub-API kernels (subapi_ops.hip), so the reference's module
// methods stay differentiable (REF = exploration/GGTV_GGLR_v1.0/deep_multiscale_GGLR_GGTV_v1x0.py;
// in the reference they are ATen compositions under autograd, REF:128-228, :452-516):
//   get_neighbors_pixels       gx(q) = sum_e sum_{p: clamp(p + d_e) = q} g_e(p)
//   normalize_and_transform    gf = (M g - y <M g, y>) / |f|  (|f| > eps; else M g / eps), gM += g y
//   stats_conv (_transpose)    gx = S* g (S^T* g), gtaps += <g, the tap's shifted input>
//   op_L_norm                  gx = g - sum_e scatter(w_e g), gw_e = -sum_f g x(clamp(p + d_e))
//   op_C                       gs = sum_e w_e gE_e - scatter(w_e gE_e), gw_e = sum_f gE_e (s - s(clamp)), gx = S* gs
//   op_C_transpose             gz = S^T* g;  gE_e = w_e (gz - [p + d_e inside] gz(p + d_e)), gw_e = sum_f E_e (...)
// "scatter" is the adjoint of the replicate-clamped gather: the sources of q along edge e are
// q - d_e (when inside) and q itself (when q + d_e falls outside, the clamp maps it back to q).
// Per-channel tap and per-graph multiM gradients are block reductions with one fixed-order partial per
// block (grr_common.h).
// These are off the solver's path (it fuses the same arithmetic in graph_bwd.hip); one thread per
// output pixel, HBM-bound.
#include "grr_common.h"

namespace grr {

namespace {

constexpr int SB_NT = 256;
constexpr int SDY[4] = {-1, 0, 0, 1}, SDX[4] = {0, -1, 1, 0};   // REF edge order: up, left, right, down

struct BTaps {
  float c, u, l, r, d;
};

__device__ __forceinline__ BTaps btaps(const grr_stencil& s, int ch) {
  const float p01 = s.p01[ch], p2a = s.p02a[ch], p2b = s.p02b[ch], p3 = s.p03[ch];
  BTaps t;
  t.c = ((p01 - p2a) - p2b) + 4.0f * p3;
  t.r = p2a - p3;
  t.d = p2b - p3;
  t.u = -p3;
  t.l = -p3;
  return t;
}

// sum over the sources p of q along edge e (clamp adjoint) of fn(p)
template <class Fn>
__device__ __forceinline__ float clamp_adj(int y, int x, int e, int H, int W, Fn fn) {
  const int sy = y - SDY[e], sx = x - SDX[e];
  float v = (sy >= 0 && sy < H && sx >= 0 && sx < W) ? fn(sy, sx) : 0.f;
  const int ny = y + SDY[e], nx = x + SDX[e];
  if (ny < 0 || ny >= H || nx < 0 || nx >= W) v += fn(y, x);
  return v;
}

// block sum of NV floats per thread -> one partial per value (thread k: row idx0 + k of r, slot `slot`;
// grr_common.h, fixed-order reductions)
template <int NV>
__device__ __forceinline__ void block_red(float (&v)[NV], const Red& r, int idx0, int nv, uint32_t slot) {
  __shared__ float red[NV][SB_NT / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float s = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) red[k][wv] = s;
  }
  __syncthreads();
  if ((int)threadIdx.x < nv) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < SB_NT / 64; ++i) s += red[threadIdx.x][i];
    red_put(r, idx0 + (int)threadIdx.x, slot, s);
  }
  __syncthreads();
}
// slot of block (blockIdx.x, blockIdx.y) of a (chunks, B * per) grid: one per (b, chunk)
__device__ __forceinline__ uint32_t chunk_slot(int per) {
  return (uint32_t)(blockIdx.y / per) * gridDim.x + blockIdx.x;
}

// grid: (blocks per plane, planes); the pixels of one plane per block row
__device__ __forceinline__ int64_t plane_of() { return blockIdx.y; }

__global__ __launch_bounds__(SB_NT) void neighbor_gather_bwd_kernel(const float* __restrict__ g, float* __restrict__ gx,
                                                                    int H, int W) {
  const int64_t HW = (int64_t)H * W, pl = plane_of();
  const float* gp = g + pl * 4 * HW;
  for (int64_t p = blockIdx.x * (int64_t)SB_NT + threadIdx.x; p < HW; p += (int64_t)gridDim.x * SB_NT) {
    const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
    float v = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v += clamp_adj(y, x, e, H, W, [&](int sy, int sx) { return gp[e * HW + (int64_t)sy * W + sx]; });
    gx[pl * HW + p] = v;
  }
}

// grid (blocks, B*G): gf for the F channels of a graph, gM[g, f] += sum g_f y_f
__global__ __launch_bounds__(SB_NT) void normalize_features_bwd_kernel(const float* __restrict__ f,
                                                                       const float* __restrict__ multiM,
                                                                       const float* __restrict__ gout,
                                                                       float* __restrict__ gf, Red gM,
                                                                       int G, int F, int64_t HW) {
  constexpr int FMAX = 16;
  const int64_t bg = blockIdx.y;
  const int gi = (int)(bg % G);
  float acc[FMAX];
#pragma unroll
  for (int k = 0; k < FMAX; ++k) acc[k] = 0.f;
  for (int64_t p = blockIdx.x * (int64_t)SB_NT + threadIdx.x; p < HW; p += (int64_t)gridDim.x * SB_NT) {
    const float* src = f + bg * F * HW + p;
    const float* gs = gout + bg * F * HW + p;
    float ss = 0.f;
    for (int k = 0; k < F; ++k) ss = __builtin_fmaf(src[k * HW], src[k * HW], ss);
    const float nrm = sqrtf(ss), den = fmaxf(nrm, 1e-12f);
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < FMAX; ++k) {
      if (k < F) {
        const float y = src[k * HW] / den, gy = gs[k * HW] * multiM[gi * F + k];
        acc[k] += gs[k * HW] * y;
        dot += gy * y;
      }
    }
    for (int k = 0; k < F; ++k) {
      const float y = src[k * HW] / den, gy = gs[k * HW] * multiM[gi * F + k];
      // d(f / max(|f|, eps)): the clamp passes no gradient to |f| below eps
      gf[(bg * F + k) * HW + p] = nrm > 1e-12f ? (gy - y * dot) / den : gy / den;
    }
  }
  block_red<FMAX>(acc, gM, gi * F, F, chunk_slot(G));
}

// stats_conv reverse: gx = S* g (replicate) or S^T* g (zero frame); gtaps[ch] (c, u, l, r, d) += <g, shifted x>
__global__ __launch_bounds__(SB_NT) void stats_conv_bwd_kernel(const float* __restrict__ x, grr_stencil s,
                                                               int transpose, const float* __restrict__ g,
                                                               float* __restrict__ gx, Red gtaps,
                                                               int C, int H, int W) {
  const int64_t HW = (int64_t)H * W, pl = plane_of();
  const int ch = (int)(pl % C);
  const BTaps t = btaps(s, ch);
  const float* xp = x + pl * HW;
  const float* gp = g + pl * HW;
  float tg[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t p = blockIdx.x * (int64_t)SB_NT + threadIdx.x; p < HW; p += (int64_t)gridDim.x * SB_NT) {
    const int y = (int)(p / W), xx = (int)(p - (int64_t)y * W);
    const float gv = gp[p];
    auto X = [&](int yy, int xc) { return xp[(int64_t)yy * W + xc]; };
    auto Gv = [&](int yy, int xc) { return gp[(int64_t)yy * W + xc]; };
    float v;
    if (!transpose) {
      // out(p) = u x(clamp(p-dy)) + l x(clamp(p-dx)) + c x(p) + r x(clamp(p+dx)) + d x(clamp(p+dy))
      tg[0] += gv * X(y, xx);
      tg[1] += gv * X(max(y - 1, 0), xx);
      tg[2] += gv * X(y, max(xx - 1, 0));
      tg[3] += gv * X(y, min(xx + 1, W - 1));
      tg[4] += gv * X(min(y + 1, H - 1), xx);
      v = t.c * gv;
      v += t.u * clamp_adj(y, xx, 0, H, W, Gv);
      v += t.l * clamp_adj(y, xx, 1, H, W, Gv);
      v += t.r * clamp_adj(y, xx, 2, H, W, Gv);
      v += t.d * clamp_adj(y, xx, 3, H, W, Gv);
    } else {
      // out(p) = u x(p+dy) + l x(p+dx) + c x(p) + r x(p-dx) + d x(p-dy), zero outside
      tg[0] += gv * X(y, xx);
      if (y + 1 < H) tg[1] += gv * X(y + 1, xx);
      if (xx + 1 < W) tg[2] += gv * X(y, xx + 1);
      if (xx > 0) tg[3] += gv * X(y, xx - 1);
      if (y > 0) tg[4] += gv * X(y - 1, xx);
      v = t.c * gv;
      if (y > 0) v += t.u * Gv(y - 1, xx);
      if (xx > 0) v += t.l * Gv(y, xx - 1);
      if (xx + 1 < W) v += t.r * Gv(y, xx + 1);
      if (y + 1 < H) v += t.d * Gv(y + 1, xx);
    }
    gx[pl * HW + p] = v;
  }
  if (gtaps.p) block_red<5>(tg, gtaps, ch * 5, 5, chunk_slot(C));
}

// op_L_norm reverse, grid (blocks, B*G): the F planes of a graph share w
__global__ __launch_bounds__(SB_NT) void op_L_norm_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                              const float* __restrict__ g, float* __restrict__ gx,
                                                              float* __restrict__ gw, int F, int H, int W) {
  const int64_t HW = (int64_t)H * W, bg = blockIdx.y;
  const float* wp = w + bg * 4 * HW;
  for (int64_t p = blockIdx.x * (int64_t)SB_NT + threadIdx.x; p < HW; p += (int64_t)gridDim.x * SB_NT) {
    const int y = (int)(p / W), xx = (int)(p - (int64_t)y * W);
    float gwe[4] = {0.f, 0.f, 0.f, 0.f};
    for (int f = 0; f < F; ++f) {
      const float* xp = x + (bg * F + f) * HW;
      const float* gp = g + (bg * F + f) * HW;
      float v = gp[p];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v -= clamp_adj(y, xx, e, H, W, [&](int sy, int sx) {
          const int64_t q = (int64_t)sy * W + sx;
          return wp[e * HW + q] * gp[q];
        });
        gwe[e] -= gp[p] * xp[(int64_t)clampi(y + SDY[e], 0, H - 1) * W + clampi(xx + SDX[e], 0, W - 1)];
      }
      gx[(bg * F + f) * HW + p] = v;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) gw[bg * 4 * HW + e * HW + p] = gwe[e];
  }
}

// op_C reverse, first part, grid (blocks, B*G): gs (before S*) and gw from gE and s = S x
__global__ __launch_bounds__(SB_NT) void op_C_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         grr_stencil s, const float* __restrict__ gE,
                                                         float* __restrict__ gs, float* __restrict__ gw, int G, int F,
                                                         int H, int W) {
  const int64_t HW = (int64_t)H * W, bg = blockIdx.y;
  const float* wp = w + bg * 4 * HW;
  for (int64_t p = blockIdx.x * (int64_t)SB_NT + threadIdx.x; p < HW; p += (int64_t)gridDim.x * SB_NT) {
    const int y = (int)(p / W), xx = (int)(p - (int64_t)y * W);
    float gwe[4] = {0.f, 0.f, 0.f, 0.f};
    for (int f = 0; f < F; ++f) {
      const int64_t pl = bg * F + f;
      const BTaps t = btaps(s, (int)(pl % (G * F)));
      const float* xp = x + pl * HW;
      const float* ge = gE + pl * 4 * HW;
      auto S = [&](int yy, int xc) {
        const int yu = max(yy - 1, 0), yd = min(yy + 1, H - 1), xl = max(xc - 1, 0), xr = min(xc + 1, W - 1);
        float v = t.u * xp[(int64_t)yu * W + xc];
        v += t.l * xp[(int64_t)yy * W + xl];
        v += t.c * xp[(int64_t)yy * W + xc];
        v += t.r * xp[(int64_t)yy * W + xr];
        v += t.d * xp[(int64_t)yd * W + xc];
        return v;
      };
      const float sc = S(y, xx);
      float v = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float gv = ge[e * HW + p];
        v += wp[e * HW + p] * gv;
        v -= clamp_adj(y, xx, e, H, W, [&](int sy, int sx) {
          const int64_t q = (int64_t)sy * W + sx;
          return wp[e * HW + q] * ge[e * HW + q];
        });
        gwe[e] += gv * (sc - S(clampi(y + SDY[e], 0, H - 1), clampi(xx + SDX[e], 0, W - 1)));
      }
      gs[pl * HW + p] = v;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) gw[bg * 4 * HW + e * HW + p] = gwe[e];
  }
}

// op_C_transpose reverse, second part, grid (blocks, B*G): gE, gw from gz = S^T* g
__global__ __launch_bounds__(SB_NT) void op_Ct_bwd_kernel(const float* __restrict__ e6, const float* __restrict__ w,
                                                          const float* __restrict__ gz, float* __restrict__ gE,
                                                          float* __restrict__ gw, int F, int H, int W) {
  const int64_t HW = (int64_t)H * W, bg = blockIdx.y;
  const float* wp = w + bg * 4 * HW;
  for (int64_t p = blockIdx.x * (int64_t)SB_NT + threadIdx.x; p < HW; p += (int64_t)gridDim.x * SB_NT) {
    const int y = (int)(p / W), xx = (int)(p - (int64_t)y * W);
    float gwe[4] = {0.f, 0.f, 0.f, 0.f};
    for (int f = 0; f < F; ++f) {
      const int64_t pl = bg * F + f;
      const float* zp = gz + pl * HW;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ny = y + SDY[e], nx = xx + SDX[e];
        const bool in = ny >= 0 && ny < H && nx >= 0 && nx < W;
        const float d = zp[p] - (in ? zp[(int64_t)ny * W + nx] : 0.f);
        gE[(pl * 4 + e) * HW + p] = wp[e * HW + p] * d;
        gwe[e] += e6[(pl * 4 + e) * HW + p] * d;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) gw[bg * 4 * HW + e * HW + p] = gwe[e];
  }
}

dim3 grid2(int64_t hw, int64_t rows) {
  const int64_t bx = std::min<int64_t>((hw + SB_NT - 1) / SB_NT, std::max<int64_t>(1, 8192 / std::max<int64_t>(rows, 1)));
  return dim3((unsigned)std::max<int64_t>(bx, 1), (unsigned)rows);
}

bool taps_set(const grr_stencil& s) { return s.p01 && s.p02a && s.p02b && s.p03; }

}  // namespace

}  // namespace grr

using namespace grr;

extern "C" {

grr_status grr_neighbor_gather_bwd(const float* g, float* gx, int B, int C, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(g && gx && B > 0 && C > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG, "grr_neighbor_gather_bwd: bad args");
  GRR_REQUIRE((int64_t)B * C < 65536, GRR_ERR_UNSUPPORTED, "grr_neighbor_gather_bwd: B*C >= 65536");
  hipLaunchKernelGGL(neighbor_gather_bwd_kernel, grid2((int64_t)H * W, (int64_t)B * C), dim3(SB_NT), 0,
                     (hipStream_t)stream, g, gx, H, W);
  return launch_status("grr_neighbor_gather_bwd");
}

grr_status grr_normalize_features_bwd(const float* f, const float* multiM, const float* gout, float* gf, float* gM,
                                      int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(f && multiM && gout && gf && gM && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_normalize_features_bwd: bad args");
  GRR_REQUIRE(F <= 16 && (int64_t)B * G < 65536, GRR_ERR_UNSUPPORTED, "grr_normalize_features_bwd: F > 16");
  const dim3 grid = grid2((int64_t)H * W, (int64_t)B * G);
  RedScratch rs((hipStream_t)stream);
  const int im = rs.plan(gM, G * F, (uint32_t)B * grid.x);
  grr_status st = rs.alloc("grr_normalize_features_bwd");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(normalize_features_bwd_kernel, grid, dim3(SB_NT), 0, (hipStream_t)stream, f, multiM, gout, gf,
                     rs.red(im), G, F, (int64_t)H * W);
  st = launch_status("grr_normalize_features_bwd");
  return st != GRR_OK ? st : rs.finish("grr_normalize_features_bwd");
}

grr_status grr_stats_conv_bwd(const float* x, grr_stencil s, int transpose, const float* g, float* gx, float* gtaps,
                              int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && g && gx && taps_set(s) && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_stats_conv_bwd: bad args");
  GRR_REQUIRE(gx != g && (int64_t)B * G * F < 65536, GRR_ERR_INVALID_ARG, "grr_stats_conv_bwd: aliasing / size");
  const dim3 grid = grid2((int64_t)H * W, (int64_t)B * G * F);
  RedScratch rs((hipStream_t)stream);
  const int it = rs.plan(gtaps, G * F * 5, (uint32_t)B * grid.x);
  grr_status st = rs.alloc("grr_stats_conv_bwd");
  if (st != GRR_OK) return st;
  hipLaunchKernelGGL(stats_conv_bwd_kernel, grid, dim3(SB_NT), 0, (hipStream_t)stream, x, s, transpose, g, gx,
                     rs.red(it), G * F, H, W);
  st = launch_status("grr_stats_conv_bwd");
  return st != GRR_OK ? st : rs.finish("grr_stats_conv_bwd");
}

grr_status grr_glr_op_l_norm_bwd(const float* x, const float* w, const float* g, float* gx, float* gw, int B, int G,
                                 int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && w && g && gx && gw && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_glr_op_l_norm_bwd: bad args");
  GRR_REQUIRE(gx != g && (int64_t)B * G < 65536, GRR_ERR_INVALID_ARG, "grr_glr_op_l_norm_bwd: aliasing / size");
  hipLaunchKernelGGL(op_L_norm_bwd_kernel, grid2((int64_t)H * W, (int64_t)B * G), dim3(SB_NT), 0, (hipStream_t)stream,
                     x, w, g, gx, gw, F, H, W);
  return launch_status("grr_glr_op_l_norm_bwd");
}

// gx = S* gs with gs from op_C_bwd_kernel (work: caller's [B,G,F,H,W] buffer); gtaps accumulate
grr_status grr_gtv_op_c_bwd(const float* x, const float* w, grr_stencil s, const float* gE, float* work, float* gx,
                            float* gw, float* gtaps, int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && w && gE && work && gx && gw && gtaps && taps_set(s) && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_gtv_op_c_bwd: bad args");
  GRR_REQUIRE(work != gx && (int64_t)B * G * F < 65536, GRR_ERR_INVALID_ARG, "grr_gtv_op_c_bwd: aliasing / size");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(op_C_bwd_kernel, grid2((int64_t)H * W, (int64_t)B * G), dim3(SB_NT), 0, st, x, w, s, gE, work, gw,
                     G, F, H, W);
  grr_status rc = launch_status("grr_gtv_op_c_bwd");
  if (rc != GRR_OK) return rc;
  const dim3 grid = grid2((int64_t)H * W, (int64_t)B * G * F);
  RedScratch rs(st);
  const int it = rs.plan(gtaps, G * F * 5, (uint32_t)B * grid.x);
  rc = rs.alloc("grr_gtv_op_c_bwd");
  if (rc != GRR_OK) return rc;
  hipLaunchKernelGGL(stats_conv_bwd_kernel, grid, dim3(SB_NT), 0, st, x, s, 0, work, gx, rs.red(it), G * F, H, W);
  rc = launch_status("grr_gtv_op_c_bwd");
  return rc != GRR_OK ? rc : rs.finish("grr_gtv_op_c_bwd");
}

// z: the op_C_transpose forward's pre-S^T value (its `work` buffer); work2: caller's [B,G,F,H,W] buffer
grr_status grr_gtv_op_c_transpose_bwd(const float* edges, const float* w, grr_stencil s, const float* z,
                                      const float* g, float* work2, float* gE, float* gw, float* gtaps, int B, int G,
                                      int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(edges && w && z && g && work2 && gE && gw && gtaps && taps_set(s) && B > 0 && G > 0 && F > 0 && H > 0 &&
                  W > 0, GRR_ERR_INVALID_ARG, "grr_gtv_op_c_transpose_bwd: bad args");
  GRR_REQUIRE(work2 != g && (int64_t)B * G * F < 65536, GRR_ERR_INVALID_ARG,
              "grr_gtv_op_c_transpose_bwd: aliasing / size");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid = grid2((int64_t)H * W, (int64_t)B * G * F);
  RedScratch rs(st);
  const int it = rs.plan(gtaps, G * F * 5, (uint32_t)B * grid.x);
  grr_status rc = rs.alloc("grr_gtv_op_c_transpose_bwd");
  if (rc != GRR_OK) return rc;
  hipLaunchKernelGGL(stats_conv_bwd_kernel, grid, dim3(SB_NT), 0, st, z, s, 1, g, work2, rs.red(it), G * F, H, W);
  rc = launch_status("grr_gtv_op_c_transpose_bwd");
  if (rc == GRR_OK) rc = rs.finish("grr_gtv_op_c_transpose_bwd");
  if (rc != GRR_OK) return rc;
  hipLaunchKernelGGL(op_Ct_bwd_kernel, grid2((int64_t)H * W, (int64_t)B * G), dim3(SB_NT), 0, st, edges, w, work2, gE,
                     gw, F, H, W);
  return launch_status("grr_gtv_op_c_transpose_bwd");
}

}  // extern "C"
