// The GLRFast / GTVFast sub-API of the reference as standalone gfx950 kernels (REF =
// exploration/GGTV_GGLR_v1.0/deep_multiscale_GGLR_GGTV_v1x0.py):
//   get_neighbors_pixels        REF:128-144 / :359-374     [B,C,H,W] -> [B,C,4,H,W]
//   normalize_and_transform...  REF:146-157 / :377-388     [B,G,F,H,W] -> [B,G*F,H,W]
//   stats_conv / _transpose     REF:177-215 / :410-449     S (replicate frame), S^T (zero frame)
//   GLRFast.op_L_norm           REF:218-228                x - sum_e w_e x(clamp(p + delta_e))
//   GTVFast.op_C                REF:452-467                [B,G,F,H,W] -> edge signals [B,G,F,4,H,W]
//   GTVFast.op_C_transpose      REF:469-516                edge signals -> [B,G,F,H,W]
// The solver never calls these (graph_ops.hip fuses the same arithmetic so the 4x edge tensors
// never reach HBM); they exist so code written against the reference's module API runs on the
// engine unchanged.  Each is a streaming gather: one thread per output pixel, lanes along W
// (coalesced rows), neighbour rows served by L1/L2; HBM-bound.
#include "grr_common.h"

namespace grr {

namespace {

constexpr int SUB_NT = 256;

struct SubTaps {
  float c, u, l, r, d;
};

// taps of p01*k01 + p02a*k02a + p02b*k02b + p03*k03 (REF:178-183), same roundings as graph_ops.hip
__device__ __forceinline__ SubTaps sub_taps(const grr_stencil& s, int ch) {
  const float p01 = s.p01[ch], p2a = s.p02a[ch], p2b = s.p02b[ch], p3 = s.p03[ch];
  SubTaps t;
  t.c = ((p01 - p2a) - p2b) + 4.0f * p3;
  t.r = p2a - p3;
  t.d = p2b - p3;
  t.u = -p3;
  t.l = -p3;
  return t;
}

// S x at (y, x) of one plane, replicate frame (REF:186)
__device__ __forceinline__ float s_rep(const float* pl, const SubTaps& t, int y, int x, int H, int W) {
  const int yu = max(y - 1, 0), yd = min(y + 1, H - 1), xl = max(x - 1, 0), xr = min(x + 1, W - 1);
  float v = t.u * pl[(int64_t)yu * W + x];
  v += t.l * pl[(int64_t)y * W + xl];
  v += t.c * pl[(int64_t)y * W + x];
  v += t.r * pl[(int64_t)y * W + xr];
  v += t.d * pl[(int64_t)yd * W + x];
  return v;
}

// S^T y at (y, x): conv_transpose2d(padding 1) of the same kernel, zero outside (REF:207-213)
__device__ __forceinline__ float st_zero(const float* pl, const SubTaps& t, int y, int x, int H, int W) {
  float v = y + 1 < H ? t.u * pl[(int64_t)(y + 1) * W + x] : 0.f;
  v += x + 1 < W ? t.l * pl[(int64_t)y * W + x + 1] : 0.f;
  v += t.c * pl[(int64_t)y * W + x];
  v += x > 0 ? t.r * pl[(int64_t)y * W + x - 1] : 0.f;
  v += y > 0 ? t.d * pl[(int64_t)(y - 1) * W + x] : 0.f;
  return v;
}

constexpr int DY[4] = {-1, 0, 0, 1}, DX[4] = {0, -1, 1, 0};   // REF edge order: up, left, right, down

__global__ __launch_bounds__(SUB_NT) void neighbor_gather_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                                 int64_t planes, int H, int W) {
  const int64_t HW = (int64_t)H * W, n = planes * HW;
  for (int64_t i = blockIdx.x * (int64_t)SUB_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * SUB_NT) {
    const int64_t pl = i / HW, p = i - pl * HW;
    const int y = (int)(p / W), xx = (int)(p - (int64_t)y * W);
    const float* src = x + pl * HW;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int yy = clampi(y + DY[e], 0, H - 1), xe = clampi(xx + DX[e], 0, W - 1);
      out[(pl * 4 + e) * HW + p] = src[(int64_t)yy * W + xe];
    }
  }
}

__global__ __launch_bounds__(SUB_NT) void normalize_features_kernel(const float* __restrict__ f,
                                                                    const float* __restrict__ multiM,
                                                                    float* __restrict__ out, int64_t BG, int G,
                                                                    int F, int64_t HW) {
  const int64_t n = BG * HW;
  for (int64_t i = blockIdx.x * (int64_t)SUB_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * SUB_NT) {
    const int64_t bg = i / HW, p = i - bg * HW;
    const int g = (int)(bg % G);
    const float* src = f + bg * F * HW + p;
    float ss = 0.f;
    for (int k = 0; k < F; ++k) ss = __builtin_fmaf(src[k * HW], src[k * HW], ss);
    const float den = fmaxf(sqrtf(ss), 1e-12f);   // F.normalize(dim=2, eps 1e-12)
    for (int k = 0; k < F; ++k) out[(bg * F + k) * HW + p] = (src[k * HW] / den) * multiM[g * F + k];
  }
}

__global__ __launch_bounds__(SUB_NT) void stats_conv_kernel(const float* __restrict__ x, grr_stencil s, int transpose,
                                                            float* __restrict__ out, int64_t planes, int C, int H,
                                                            int W) {
  const int64_t HW = (int64_t)H * W, n = planes * HW;
  for (int64_t i = blockIdx.x * (int64_t)SUB_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * SUB_NT) {
    const int64_t pl = i / HW, p = i - pl * HW;
    const int y = (int)(p / W), xx = (int)(p - (int64_t)y * W);
    const SubTaps t = sub_taps(s, (int)(pl % C));
    out[i] = transpose ? st_zero(x + pl * HW, t, y, xx, H, W) : s_rep(x + pl * HW, t, y, xx, H, W);
  }
}

// op_L_norm: out = x - sum_e w_e x(clamp(p + delta_e))  (the einsum of REF:222-226)
__global__ __launch_bounds__(SUB_NT) void op_L_norm_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           float* __restrict__ out, int64_t planes, int G, int F,
                                                           int H, int W) {
  const int64_t HW = (int64_t)H * W, n = planes * HW;
  for (int64_t i = blockIdx.x * (int64_t)SUB_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * SUB_NT) {
    const int64_t pl = i / HW, p = i - pl * HW;
    const int y = (int)(p / W), xx = (int)(p - (int64_t)y * W);
    const int64_t bg = pl / F;
    const float* src = x + pl * HW;
    const float* wp = w + bg * 4 * HW + p;
    float wx = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int yy = clampi(y + DY[e], 0, H - 1), xe = clampi(xx + DX[e], 0, W - 1);
      wx = __builtin_fmaf(wp[e * HW], src[(int64_t)yy * W + xe], wx);
    }
    out[i] = src[p] - wx;
  }
}

// op_C: E_e(p) = w_e(p) s(p) - w_e(p) s(clamp(p + delta_e)), s = S x  (REF:452-467)
__global__ __launch_bounds__(SUB_NT) void gtv_op_C_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          grr_stencil s, float* __restrict__ out, int64_t planes,
                                                          int C, int F, int H, int W) {
  const int64_t HW = (int64_t)H * W, n = planes * HW;
  for (int64_t i = blockIdx.x * (int64_t)SUB_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * SUB_NT) {
    const int64_t pl = i / HW, p = i - pl * HW;
    const int y = (int)(p / W), xx = (int)(p - (int64_t)y * W);
    const SubTaps t = sub_taps(s, (int)(pl % C));
    const float* src = x + pl * HW;
    const float* wp = w + (pl / F) * 4 * HW + p;
    const float sc = s_rep(src, t, y, xx, H, W);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float sn = s_rep(src, t, clampi(y + DY[e], 0, H - 1), clampi(xx + DX[e], 0, W - 1), H, W);
      const float we = wp[e * HW];
      out[(pl * 4 + e) * HW + p] = sc * we - sn * we;
    }
  }
}

// op_C_transpose, first part: o(q) = sum_e z_e(q) - sum_e [q - delta_e inside] z_e(q - delta_e),
// z_e = E_e w_e; the subtractions in edge order as REF:484-510 applies them (scatters that land in
// the replicate frame are cropped away, REF:513)
__global__ __launch_bounds__(SUB_NT) void gtv_op_Ct_scatter_kernel(const float* __restrict__ e6,
                                                                   const float* __restrict__ w,
                                                                   float* __restrict__ o, int64_t planes, int F,
                                                                   int H, int W) {
  const int64_t HW = (int64_t)H * W, n = planes * HW;
  for (int64_t i = blockIdx.x * (int64_t)SUB_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * SUB_NT) {
    const int64_t pl = i / HW, p = i - pl * HW;
    const int y = (int)(p / W), xx = (int)(p - (int64_t)y * W);
    const float* ep = e6 + pl * 4 * HW;
    const float* wp = w + (pl / F) * 4 * HW;
    float z[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = ep[e * HW + p] * wp[e * HW + p];
    float v = ((z[0] + z[1]) + z[2]) + z[3];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int sy = y - DY[e], sx = xx - DX[e];
      if (sy >= 0 && sy < H && sx >= 0 && sx < W) {
        const int64_t q = (int64_t)sy * W + sx;
        v -= ep[e * HW + q] * wp[e * HW + q];
      }
    }
    o[i] = v;
  }
}

unsigned sub_grid(int64_t n) { return (unsigned)std::min<int64_t>((n + SUB_NT - 1) / SUB_NT, 1 << 16); }

bool stencil_set(const grr_stencil& s) { return s.p01 && s.p02a && s.p02b && s.p03; }

}  // namespace

}  // namespace grr

using namespace grr;

extern "C" {

grr_status grr_neighbor_gather(const float* x, float* out, int B, int C, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && out && B > 0 && C > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG, "grr_neighbor_gather: bad args");
  GRR_REQUIRE(out != x, GRR_ERR_INVALID_ARG, "grr_neighbor_gather: out must not alias x");
  const int64_t planes = (int64_t)B * C;
  hipLaunchKernelGGL(neighbor_gather_kernel, dim3(sub_grid(planes * H * W)), dim3(SUB_NT), 0, (hipStream_t)stream, x,
                     out, planes, H, W);
  return launch_status("grr_neighbor_gather");
}

grr_status grr_normalize_features(const float* f, const float* multiM, float* out, int B, int G, int F, int H, int W,
                                  void* stream) {
  clear_error();
  GRR_REQUIRE(f && multiM && out && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_normalize_features: bad args");
  const int64_t bg = (int64_t)B * G, hw = (int64_t)H * W;
  hipLaunchKernelGGL(normalize_features_kernel, dim3(sub_grid(bg * hw)), dim3(SUB_NT), 0, (hipStream_t)stream, f,
                     multiM, out, bg, G, F, hw);
  return launch_status("grr_normalize_features");
}

grr_status grr_stats_conv(const float* x, grr_stencil s, int transpose, float* out, int B, int G, int F, int H, int W,
                          void* stream) {
  clear_error();
  GRR_REQUIRE(x && out && stencil_set(s) && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_stats_conv: bad args");
  GRR_REQUIRE(out != x, GRR_ERR_INVALID_ARG, "grr_stats_conv: out must not alias x");
  const int64_t planes = (int64_t)B * G * F;
  hipLaunchKernelGGL(stats_conv_kernel, dim3(sub_grid(planes * H * W)), dim3(SUB_NT), 0, (hipStream_t)stream, x, s,
                     transpose, out, planes, G * F, H, W);
  return launch_status("grr_stats_conv");
}

grr_status grr_glr_op_l_norm(const float* x, const float* w, float* out, int B, int G, int F, int H, int W,
                             void* stream) {
  clear_error();
  GRR_REQUIRE(x && w && out && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_glr_op_l_norm: bad args");
  GRR_REQUIRE(out != x, GRR_ERR_INVALID_ARG, "grr_glr_op_l_norm: out must not alias x");
  const int64_t planes = (int64_t)B * G * F;
  hipLaunchKernelGGL(op_L_norm_kernel, dim3(sub_grid(planes * H * W)), dim3(SUB_NT), 0, (hipStream_t)stream, x, w,
                     out, planes, G, F, H, W);
  return launch_status("grr_glr_op_l_norm");
}

grr_status grr_gtv_op_c(const float* x, const float* w, grr_stencil s, float* edges, int B, int G, int F, int H, int W,
                        void* stream) {
  clear_error();
  GRR_REQUIRE(x && w && edges && stencil_set(s) && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_gtv_op_c: bad args");
  const int64_t planes = (int64_t)B * G * F;
  hipLaunchKernelGGL(gtv_op_C_kernel, dim3(sub_grid(planes * H * W)), dim3(SUB_NT), 0, (hipStream_t)stream, x, w, s,
                     edges, planes, G * F, F, H, W);
  return launch_status("grr_gtv_op_c");
}

grr_status grr_gtv_op_c_transpose(const float* edges, const float* w, grr_stencil s, float* work, float* out, int B,
                                  int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(edges && w && work && out && stencil_set(s) && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_gtv_op_c_transpose: bad args");
  GRR_REQUIRE(work != out, GRR_ERR_INVALID_ARG, "grr_gtv_op_c_transpose: work must not alias out");
  const int64_t planes = (int64_t)B * G * F;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(gtv_op_Ct_scatter_kernel, dim3(sub_grid(planes * H * W)), dim3(SUB_NT), 0, st, edges, w, work,
                     planes, F, H, W);
  grr_status rc = launch_status("grr_gtv_op_c_transpose");
  if (rc != GRR_OK) return rc;
  hipLaunchKernelGGL(stats_conv_kernel, dim3(sub_grid(planes * H * W)), dim3(SUB_NT), 0, st, work, s, 1, out, planes,
                     G * F, H, W);
  return launch_status("grr_gtv_op_c_transpose");
}

}  // extern "C"
