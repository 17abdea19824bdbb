// gfx950 kernels of the unrolled GGTV/GGLR solver (a1-a18 of SURVEY.md §8).
//
// Data layout in HBM (all fp32, caller-allocated, contiguous):
//   signals       [B, C = G*F, H, W]     (the reference's NCHW, REF:707-809)
//   edge weights  [B, G, 4, H, W]        (REF:160-175; shared by the F channels of a graph)
//   pair weights  [B, G, 2, H, W]        (symmetrised w^2 of the linear graph-TV operator)
//   half level    [B, C, H/2, W/2]       (2x2 mean pool D, REF:613)
//
// Work decomposition of the fused operator kernel: one 256-thread workgroup = one
// (batch b, channel, 32x32 output tile).  All of its global loads (input tile with
// a 3-pixel replicate halo, the graph's edge weights at the 34x34 pass-B points,
// the epilogue operands) are issued up front, so their latency overlaps; the F
// channel-workgroups of one (b, graph, tile) are consecutive logical blocks placed
// on one XCD, so the shared edge weights come from HBM once and from L2 F-1 times.
// The chain  x -> s = S x (halo 2) -> {l = (I-W) s, o = C^T C s} (halo 1) -> S^T
// is evaluated LDS-to-LDS, followed by a fused epilogue (rhs / CG stage /
// half-level term).  Everything is memory-bound (≈3.5 flop/B), so the design goal is HBM
// bytes: each launch reads each of its inputs once and writes each output once.
#include <cstdarg>

#include "grr_common.h"

namespace grr {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

void clear_error() { g_err.clear(); }

grr_status launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return GRR_ERR_HIP;
  }
  return GRR_OK;
}

constexpr int NT = 256;     // threads per workgroup (4 waves)
constexpr int TILE = 32;    // output tile edge
constexpr int XS = TILE + 6, XA = XS * XS;  // input tile, halo 3
constexpr int SS = TILE + 4, SA = SS * SS;  // s = S x, halo 2
constexpr int LS = TILE + 2, LA = LS * LS;  // l / o, halo 1
constexpr int NPB = (LA + NT - 1) / NT;     // pass-B positions per thread (5)

// ---------------------------------------------------------------------------
// a1: neighbour table
// ---------------------------------------------------------------------------
__global__ void neighbor_table_kernel(int32_t* __restrict__ out, int H, int W) {
  const int64_t n = (int64_t)H * W;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
    out[p] = clampi(y - 1, 0, H - 1) * W + x;            // up
    out[n + p] = y * W + clampi(x - 1, 0, W - 1);        // left
    out[2 * n + p] = y * W + clampi(x + 1, 0, W - 1);    // right
    out[3 * n + p] = clampi(y + 1, 0, H - 1) * W + x;    // down
  }
}

// ---------------------------------------------------------------------------
// a3+a4: edge weights.  One workgroup = (b, g, 32x32 tile); the F feature planes
// of the graph are staged with a 1-pixel replicate halo, normalised in LDS, and
// each output pixel takes a 4-way softmax of its neighbour similarities.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void edge_weights_kernel(
    const float* __restrict__ feat, int64_t bstride, const float* __restrict__ multiM,
    float* __restrict__ w, float* __restrict__ deg, int G, int F, int H, int W,
    int tiles_x, int tiles_y, uint32_t nblk) {
  extern __shared__ float fsm[];  // [F][LA]
  uint32_t lb = xcd_remap(blockIdx.x, nblk);
  const int tx = lb % tiles_x; lb /= tiles_x;
  const int ty = lb % tiles_y; lb /= tiles_y;
  const int g = lb % G;
  const int b = lb / G;
  const int y0 = ty * TILE, x0 = tx * TILE;
  const int64_t HW = (int64_t)H * W;
  const float* fb = feat + (int64_t)b * bstride + (int64_t)g * F * HW;

  for (int i = threadIdx.x; i < F * LA; i += NT) {
    const int f = i / LA, r = i - f * LA;
    const int ry = r / LS, rx = r - ry * LS;
    const int gy = clampi(y0 - 1 + ry, 0, H - 1), gx = clampi(x0 - 1 + rx, 0, W - 1);
    fsm[i] = fb[f * HW + (int64_t)gy * W + gx];
  }
  __syncthreads();
  // F.normalize(dim=F, eps=1e-12) then * multiM[g, f]  (REF:146-157)
  for (int r = threadIdx.x; r < LA; r += NT) {
    float ss = 0.f;
    for (int f = 0; f < F; ++f) {
      const float v = fsm[f * LA + r];
      ss += v * v;
    }
    const float den = fmaxf(sqrtf(ss), 1e-12f);
    for (int f = 0; f < F; ++f) fsm[f * LA + r] = (fsm[f * LA + r] / den) * multiM[g * F + f];
  }
  __syncthreads();
  float* wb = w + (int64_t)(b * G + g) * 4 * HW;
  for (int i = threadIdx.x; i < TILE * TILE; i += NT) {
    const int oy = i / TILE, ox = i - oy * TILE;
    const int gy = y0 + oy, gx = x0 + ox;
    if (gy >= H || gx >= W) continue;
    const int c = (oy + 1) * LS + ox + 1;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    for (int f = 0; f < F; ++f) {
      const float* p = fsm + f * LA;
      const float v = p[c];
      s0 += v * p[c - LS];
      s1 += v * p[c - 1];
      s2 += v * p[c + 1];
      s3 += v * p[c + LS];
    }
    const float m = fmaxf(fmaxf(s0, s1), fmaxf(s2, s3));
    const float e0 = expf(s0 - m), e1 = expf(s1 - m), e2 = expf(s2 - m), e3 = expf(s3 - m);
    const float sum = ((e0 + e1) + e2) + e3;
    const float w0 = e0 / sum, w1 = e1 / sum, w2 = e2 / sum, w3 = e3 / sum;
    const int64_t o = (int64_t)gy * W + gx;
    wb[o] = w0;
    wb[HW + o] = w1;
    wb[2 * HW + o] = w2;
    wb[3 * HW + o] = w3;
    if (deg) deg[(int64_t)(b * G + g) * HW + o] = ((w0 + w1) + w2) + w3;
  }
}

// symmetric pair weights of C^T C (see grr.h)
__global__ void gtv_pair_weights_kernel(const float* __restrict__ w, float* __restrict__ c, int64_t nplanes,
                                        int H, int W) {
  const int64_t HW = (int64_t)H * W, n = nplanes * HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pl = i / HW, p = i - pl * HW;
    const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
    const float* wp = w + pl * 4 * HW;
    float ch = 0.f, cv = 0.f;
    if (x + 1 < W) {
      const float a = wp[2 * HW + p], bb = wp[HW + p + 1];  // w_right(p), w_left(p+right)
      ch = a * a + bb * bb;
    }
    if (y + 1 < H) {
      const float a = wp[3 * HW + p], bb = wp[p + W];       // w_down(p), w_up(p+down)
      cv = a * a + bb * bb;
    }
    c[pl * 2 * HW + p] = ch;
    c[pl * 2 * HW + HW + p] = cv;
  }
}

// D: 2x2 mean pool
__global__ void pool2_kernel(const float* __restrict__ x, float* __restrict__ xd, int64_t planes, int H, int W) {
  const int h = H / 2, w = W / 2;
  const int64_t n = planes * h * w;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pl = i / ((int64_t)h * w), q = i - pl * h * w;
    const int y = (int)(q / w), xx = (int)(q - (int64_t)y * w);
    const float* p = x + pl * H * W + (int64_t)(2 * y) * W + 2 * xx;
    xd[i] = 0.25f * p[0] + 0.25f * p[1] + 0.25f * p[W] + 0.25f * p[W + 1];
  }
}

// ---------------------------------------------------------------------------
// The fused graph operator
// ---------------------------------------------------------------------------
enum { GTV_NONE = 0, GTV_PAIR = 1, GTV_PROX = 2 };
enum { EPI_HALF = 0, EPI_RHS = 1, EPI_STEP = 2 };

struct OpArgs {
  const float* x;
  const float* wL;      // GLR edge weights [B,G,4,H,W]
  const float* wG;      // GTV pair weights [B,G,2,H,W] or raw [B,G,4,H,W] (prox)
  grr_stencil sL, sG;
  const float* log_l;   // GLR term scale (log), NULL -> 1
  const float* log_g;   // GTV term scale (log), NULL -> 1
  const float* log_gamma;
  const float* log_half;  // scale of U(t_half) (log), NULL -> 1
  const float* y;
  const float* b;
  const float* u_prev;
  const float* t_half;
  const float* alpha;
  const float* beta;
  const float* skip;
  float* out;
  float* u_out;
  float* xd_out;
  int G, F, H, W, tiles_x, tiles_y;
  uint32_t nblk;
};

struct Taps {
  float c, u, l, r, d;
};

// K = p01*k01 + p02a*k02a + p02b*k02b + p03*k03 tap by tap (REF:178-183); every
// basis coefficient is 0/±1/4 so these are the reference's exact roundings.
__device__ __forceinline__ Taps make_taps(const grr_stencil& s, int ch) {
  const float p01 = s.p01[ch], p2a = s.p02a[ch], p2b = s.p02b[ch], p3 = s.p03[ch];
  Taps t;
  t.c = ((p01 - p2a) - p2b) + 4.0f * p3;
  t.r = p2a - p3;
  t.d = p2b - p3;
  t.u = -p3;
  t.l = -p3;
  return t;
}

// S x at a tile point: taps in the kernel's raster order (up, left, centre, right, down)
__device__ __forceinline__ float stencil(const Taps& t, const float* a, int i, int stride) {
  float s = t.u * a[i - stride];
  s += t.l * a[i - 1];
  s += t.c * a[i];
  s += t.r * a[i + 1];
  s += t.d * a[i + stride];
  return s;
}

// S^T y (conv_transpose2d, padding 1): out(i,j) = sum K(a,b) y(i+1-a, j+1-b)
__device__ __forceinline__ float stencil_t(const Taps& t, const float* a, int i, int stride) {
  float s = t.u * a[i + stride];
  s += t.l * a[i + 1];
  s += t.c * a[i];
  s += t.r * a[i - 1];
  s += t.d * a[i - stride];
  return s;
}

// phi of the GTV proximal rhs: eps - (t - eps), eps = soft_threshold(t, gamma) (REF:684-704, :765-774)
__device__ __forceinline__ float prox_phi(float t, float gm) {
  const float lo = t < -gm ? t + gm : 0.f;
  const float hi = t > gm ? t - gm : 0.f;
  const float eps = lo + hi;
  return eps - (t - eps);
}

template <bool GLR, int GTV, int EPI>
__global__ __launch_bounds__(NT) void graph_op_kernel(OpArgs a) {
  __shared__ float Xs[XA];
  __shared__ float SLs[GLR ? SA : 1];
  __shared__ float SGs[GTV ? SA : 1];
  __shared__ float Ls[GLR ? LA : 1];
  __shared__ float Gs[GTV ? LA : 1];
  constexpr int NW = GTV == GTV_PROX ? 8 : 4;
  constexpr int NXL = (XA + NT - 1) / NT;  // input-tile loads per thread (6)

  // One workgroup = one (b, channel, 32x32 tile).  The F channel-workgroups of a
  // (b, graph, tile) are consecutive logical blocks, so after the XCD remap they run
  // together on one XCD and the graph's edge weights are fetched from HBM once.
  const int tid = threadIdx.x;
  const int F = a.F;
  uint32_t lb = xcd_remap(blockIdx.x, a.nblk);
  const int f = lb % F; lb /= F;
  const int tx = lb % a.tiles_x; lb /= a.tiles_x;
  const int ty = lb % a.tiles_y; lb /= a.tiles_y;
  const int g = lb % a.G;
  const int b = lb / a.G;
  const int H = a.H, W = a.W, C = a.G * F;
  const int64_t HW = (int64_t)H * W;
  const int y0 = ty * TILE, x0 = tx * TILE;
  const int ch = g * F + f;
  const int64_t plane = ((int64_t)b * C + ch) * HW;
  const int hh = H / 2, hw = W / 2;

  // ---- issue every global load of the workgroup up front ----------------------
  // (1) input tile, halo 3, replicate-clamped (REF:186 replicate pad)
  float xr[NXL];
  {
    const float* xp = a.x + plane;
#pragma unroll
    for (int j = 0; j < NXL; ++j) {
      const int i = tid + j * NT;
      const int ii = i < XA ? i : XA - 1;
      const int ry = ii / XS, rx = ii - ry * XS;
      const int gy = clampi(y0 - 3 + ry, 0, H - 1), gx = clampi(x0 - 3 + rx, 0, W - 1);
      xr[j] = xp[(int64_t)gy * W + gx];
    }
  }
  // (2) this graph's edge weights at the pass-B points
  float wl[NPB][4];
  float wg[NPB][NW];
  {
    const float* wLb = GLR ? a.wL + (int64_t)(b * a.G + g) * 4 * HW : nullptr;
    const float* wGb = GTV ? a.wG + (int64_t)(b * a.G + g) * (GTV == GTV_PROX ? 4 : 2) * HW : nullptr;
#pragma unroll
    for (int j = 0; j < NPB; ++j) {
      const int i = tid + j * NT;
      const int ry = i / LS, rx = i - ry * LS;
      const int gy = y0 - 1 + ry, gx = x0 - 1 + rx;
      const bool in = i < LA && gy >= 0 && gy < H && gx >= 0 && gx < W;
      const int64_t o = (int64_t)gy * W + gx;
      if constexpr (GLR) {
#pragma unroll
        for (int e = 0; e < 4; ++e) wl[j][e] = in ? wLb[e * HW + o] : 0.f;
      }
      if constexpr (GTV == GTV_PAIR) {
        wg[j][0] = in ? wGb[o] : 0.f;                              // c_h(q)      right edge
        wg[j][1] = (in && gx > 0) ? wGb[o - 1] : 0.f;              // c_h(q-1)    left edge
        wg[j][2] = in ? wGb[HW + o] : 0.f;                         // c_v(q)      down edge
        wg[j][3] = (in && gy > 0) ? wGb[HW + o - W] : 0.f;         // c_v(q-W)    up edge
      }
      if constexpr (GTV == GTV_PROX) {
        // own edges e at q (zero where q+delta_e leaves the image: the reference's
        // clamped neighbour is q itself, so E_e = w*s(q) - w*s(q) = 0)
        wg[j][0] = (in && gy > 0) ? wGb[o] : 0.f;
        wg[j][1] = (in && gx > 0) ? wGb[HW + o] : 0.f;
        wg[j][2] = (in && gx < W - 1) ? wGb[2 * HW + o] : 0.f;
        wg[j][3] = (in && gy < H - 1) ? wGb[3 * HW + o] : 0.f;
        // edges e of the pixel p = q - delta_e whose scatter lands on q (REF:482-500)
        wg[j][4] = (in && gy < H - 1) ? wGb[o + W] : 0.f;               // w_up(q+down)
        wg[j][5] = (in && gx < W - 1) ? wGb[HW + o + 1] : 0.f;          // w_left(q+right)
        wg[j][6] = (in && gx > 0) ? wGb[2 * HW + o - 1] : 0.f;          // w_right(q-right)
        wg[j][7] = (in && gy > 0) ? wGb[3 * HW + o - W] : 0.f;          // w_down(q-down)
      }
    }
  }
  // (3) epilogue operands of this thread's 2x2 output block
  const int by = tid >> 4, bx = tid & 15;
  const int gy0 = y0 + 2 * by, gx0 = x0 + 2 * bx;
  float eb[2][2] = {}, eu[2][2] = {}, ey[2][2] = {};
  float th = 0.f;
  const bool has_half = EPI != EPI_HALF && a.t_half != nullptr;
  const bool use_beta = EPI == EPI_STEP && a.beta != nullptr && a.u_prev != nullptr;
  const bool need_y = (EPI == EPI_RHS) || (EPI == EPI_STEP && a.skip != nullptr);
  if (EPI != EPI_HALF) {
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int gy = gy0 + dy, gx = gx0 + dx;
        if (gy < H && gx < W) {
          const int64_t o = plane + (int64_t)gy * W + gx;
          if (EPI == EPI_STEP) eb[dy][dx] = a.b[o];
          if (use_beta) eu[dy][dx] = a.u_prev[o];
          if (need_y) ey[dy][dx] = a.y[o];
        }
      }
    if (has_half && gy0 < H && gx0 < W)
      th = 0.25f * a.t_half[((int64_t)b * C + ch) * hh * hw + (int64_t)(gy0 >> 1) * hw + (gx0 >> 1)];
  }
  float sc_l = 1.f, sc_g = 1.f, sc_h = 1.f, gam = 0.f, alpha = 0.f, beta = 0.f, sk0 = 0.f, sk1 = 1.f;
  if (a.log_l) sc_l = expf(a.log_l[g]);
  if (a.log_g) sc_g = expf(a.log_g[g]);
  if (a.log_half) sc_h = expf(a.log_half[g]);
  if constexpr (GTV == GTV_PROX) gam = expf(a.log_gamma[g]);
  if constexpr (EPI == EPI_STEP) {
    alpha = a.alpha[g];
    if (use_beta) beta = a.beta[g];
    if (a.skip) { sk0 = a.skip[0]; sk1 = a.skip[1]; }
  }
  Taps tL{}, tG{};
  if constexpr (GLR) tL = make_taps(a.sL, ch);
  if constexpr (GTV != GTV_NONE) tG = make_taps(a.sG, ch);

  // ---- pass 0: input tile to LDS
#pragma unroll
  for (int j = 0; j < NXL; ++j) {
    const int i = tid + j * NT;
    if (i < XA) Xs[i] = xr[j];
  }
  __syncthreads();
  // ---- pass A: s = S x on the halo-2 region (values outside the image are never read)
  for (int i = tid; i < SA; i += NT) {
    const int ry = i / SS, rx = i - ry * SS;
    const int xi = (ry + 1) * XS + rx + 1;
    if constexpr (GLR) SLs[i] = stencil(tL, Xs, xi, XS);
    if constexpr (GTV != GTV_NONE) SGs[i] = stencil(tG, Xs, xi, XS);
  }
  __syncthreads();
  // ---- pass B: l = s - W s (GLR, REF:218-228) and o = C^T phi(C s) (GTV, REF:452-516)
#pragma unroll
  for (int j = 0; j < NPB; ++j) {
    const int i = tid + j * NT;
    if (i < LA) {
      const int ry = i / LS, rx = i - ry * LS;
      const int gy = y0 - 1 + ry, gx = x0 - 1 + rx;
      const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
      const int si = (ry + 1) * SS + rx + 1;
      if constexpr (GLR) {
        float l = 0.f;
        if (in) {
          const int nu = gy > 0 ? si - SS : si, nl = gx > 0 ? si - 1 : si;
          const int nr = gx < W - 1 ? si + 1 : si, nd = gy < H - 1 ? si + SS : si;
          const float wx = ((wl[j][0] * SLs[nu] + wl[j][1] * SLs[nl]) + wl[j][2] * SLs[nr]) + wl[j][3] * SLs[nd];
          l = SLs[si] - wx;
        }
        Ls[i] = l;
      }
      if constexpr (GTV == GTV_PAIR) {
        float o = 0.f;
        if (in) {
          const float s = SGs[si];
          o = wg[j][0] * (s - SGs[si + 1]) + wg[j][1] * (s - SGs[si - 1]) +
              wg[j][2] * (s - SGs[si + SS]) + wg[j][3] * (s - SGs[si - SS]);
        }
        Gs[i] = o;
      }
      if constexpr (GTV == GTV_PROX) {
        float o = 0.f;
        if (in) {
          const float s = SGs[si];
          const int nb[4] = {si - SS, si - 1, si + 1, si + SS};
          float z[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float we = wg[j][e];
            z[e] = prox_phi(we * s - we * SGs[nb[e]], gam) * we;   // z_e(q)
          }
          o = ((z[0] + z[1]) + z[2]) + z[3];
          // subtract z_e(q - delta_e) in edge order (REF:482-500)
          const int pb[4] = {si + SS, si + 1, si - 1, si - SS};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float we = wg[j][4 + e];
            o = o - prox_phi(we * SGs[pb[e]] - we * s, gam) * we;
          }
        }
        Gs[i] = o;
      }
    }
  }
  __syncthreads();
  // ---- pass C: S^T and the epilogue, one 2x2 output block per thread
  float outv[2][2];
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int oy = 2 * by + dy, ox = 2 * bx + dx;
      const int li = (oy + 1) * LS + ox + 1;
      float tl = 0.f, tg = 0.f;
      if constexpr (GLR) tl = stencil_t(tL, Ls, li, LS);
      if constexpr (GTV != GTV_NONE) tg = stencil_t(tG, Gs, li, LS);
      const float xv = Xs[(oy + 3) * XS + ox + 3];
      float r;
      if constexpr (EPI == EPI_HALF) {
        // mu * S_L^T l + ro * S_G^T o   (REF:666-675)
        r = 0.f;
        if constexpr (GLR) r = tl * sc_l;
        if constexpr (GTV != GTV_NONE) r = GLR ? r + tg * sc_g : tg * sc_g;
      } else if constexpr (EPI == EPI_RHS) {
        // (y + ro0 * C^T phi(C x)) + ro1 * U(t_half)   (REF:744-749 / :776-781)
        r = ey[dy][dx] + tg * sc_g;
        if (has_half) r = r + th * sc_h;
      } else {
        // A x = ((x + mu0 L0 x) + ro0 G0 x) + U(t_half)   (REF:648-680)
        float ax = xv;
        if constexpr (GLR) ax = ax + tl * sc_l;
        if constexpr (GTV != GTV_NONE) ax = ax + tg * sc_g;
        if (has_half) ax = ax + th;
        float u = eb[dy][dx] - ax;                    // residual b - A x
        if (use_beta) u = u + beta * eu[dy][dx];      // heavy-ball direction (REF:789)
        eu[dy][dx] = u;
        r = xv + alpha * u;                           // x_{k+1}
      }
      outv[dy][dx] = r;
    }
  // D of the (pre-skip) result for the next stage's half level
  if (a.xd_out && gy0 + 1 < H && gx0 + 1 < W) {
    const float d = 0.25f * outv[0][0] + 0.25f * outv[0][1] + 0.25f * outv[1][0] + 0.25f * outv[1][1];
    a.xd_out[((int64_t)b * C + ch) * hh * hw + (int64_t)(gy0 >> 1) * hw + (gx0 >> 1)] = d;
  }
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int gy = gy0 + dy, gx = gx0 + dx;
      if (gy < H && gx < W) {
        const int64_t o = plane + (int64_t)gy * W + gx;
        float r = outv[dy][dx];
        if (EPI == EPI_STEP) {
          if (a.u_out) a.u_out[o] = eu[dy][dx];
          if (a.skip) r = sk0 * ey[dy][dx] + sk1 * r;   // REF:987
        }
        a.out[o] = r;
      }
    }
}

template <bool GLR, int GTV, int EPI>
static grr_status launch_op(const OpArgs& a0, int B, hipStream_t s, const char* name) {
  OpArgs a = a0;
  a.tiles_x = (a.W + TILE - 1) / TILE;
  a.tiles_y = (a.H + TILE - 1) / TILE;
  const uint64_t n = (uint64_t)B * a.G * a.F * a.tiles_x * a.tiles_y;
  GRR_REQUIRE(n < (1ull << 31), GRR_ERR_UNSUPPORTED, "%s: grid too large", name);
  a.nblk = (uint32_t)n;
  hipLaunchKernelGGL((graph_op_kernel<GLR, GTV, EPI>), dim3(a.nblk), dim3(NT), 0, s, a);
  return launch_status(name);
}

static bool stencil_ok(const grr_stencil& s) { return s.p01 && s.p02a && s.p02b && s.p03; }

}  // namespace grr

using namespace grr;

extern "C" {

int grr_version(void) { return 1; }
const char* grr_last_error(void) { return g_err.c_str(); }

grr_status grr_neighbor_table(int32_t* out, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(out && H > 0 && W > 0, GRR_ERR_INVALID_ARG, "grr_neighbor_table: bad args");
  const int64_t n = (int64_t)H * W;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(neighbor_table_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, H, W);
  return launch_status("grr_neighbor_table");
}

grr_status grr_edge_weights(const float* feat, int64_t feat_bstride, const float* multiM, float* w, float* deg,
                            int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(feat && multiM && w && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_edge_weights: bad args");
  GRR_REQUIRE(F <= GRR_MAX_NODE_FTS, GRR_ERR_UNSUPPORTED, "grr_edge_weights: F=%d > %d", F, GRR_MAX_NODE_FTS);
  const int tx = (W + TILE - 1) / TILE, ty = (H + TILE - 1) / TILE;
  const uint64_t n = (uint64_t)B * G * tx * ty;
  GRR_REQUIRE(n < (1ull << 31), GRR_ERR_UNSUPPORTED, "grr_edge_weights: grid too large");
  const size_t lds = (size_t)F * LA * sizeof(float);
  hipLaunchKernelGGL(edge_weights_kernel, dim3((uint32_t)n), dim3(NT), lds, (hipStream_t)stream, feat, feat_bstride,
                     multiM, w, deg, G, F, H, W, tx, ty, (uint32_t)n);
  return launch_status("grr_edge_weights");
}

grr_status grr_gtv_pair_weights(const float* w, float* c, int B, int G, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(w && c && B > 0 && G > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG, "grr_gtv_pair_weights: bad args");
  const int64_t n = (int64_t)B * G * H * W;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1 << 16);
  hipLaunchKernelGGL(gtv_pair_weights_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, c,
                     (int64_t)B * G, H, W);
  return launch_status("grr_gtv_pair_weights");
}

grr_status grr_pool2(const float* x, float* xd, int B, int C, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && xd && B > 0 && C > 0 && H > 1 && W > 1, GRR_ERR_INVALID_ARG, "grr_pool2: bad args");
  GRR_REQUIRE(H % 2 == 0 && W % 2 == 0, GRR_ERR_SHAPE, "grr_pool2: H, W must be even (got %dx%d)", H, W);
  const int64_t n = (int64_t)B * C * (H / 2) * (W / 2);
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1 << 16);
  hipLaunchKernelGGL(pool2_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, xd, (int64_t)B * C, H, W);
  return launch_status("grr_pool2");
}

grr_status grr_system_half(const float* xd, const float* wL, const float* cG, grr_stencil sL, grr_stencil sG,
                           const float* log_mu, const float* log_ro, float* t, int B, int G, int F, int h, int w,
                           void* stream) {
  clear_error();
  GRR_REQUIRE(xd && t && B > 0 && G > 0 && F > 0 && h > 0 && w > 0, GRR_ERR_INVALID_ARG,
              "grr_system_half: bad args");
  GRR_REQUIRE(wL || cG, GRR_ERR_INVALID_ARG, "grr_system_half: need GLR and/or GTV weights");
  GRR_REQUIRE(!wL || stencil_ok(sL), GRR_ERR_INVALID_ARG, "grr_system_half: GLR stencil missing");
  GRR_REQUIRE(!cG || stencil_ok(sG), GRR_ERR_INVALID_ARG, "grr_system_half: GTV stencil missing");
  OpArgs a{};
  a.x = xd; a.wL = wL; a.wG = cG; a.sL = sL; a.sG = sG;
  a.log_l = log_mu; a.log_g = log_ro; a.out = t;
  a.G = G; a.F = F; a.H = h; a.W = w;
  hipStream_t s = (hipStream_t)stream;
  if (wL && cG) return launch_op<true, GTV_PAIR, EPI_HALF>(a, B, s, "grr_system_half");
  if (wL) return launch_op<true, GTV_NONE, EPI_HALF>(a, B, s, "grr_system_half");
  return launch_op<false, GTV_PAIR, EPI_HALF>(a, B, s, "grr_system_half");
}

grr_status grr_gtv_rhs_half(const float* xd, const float* wG, grr_stencil sG, int prox, const float* log_gamma,
                            float* t, int B, int G, int F, int h, int w, void* stream) {
  clear_error();
  GRR_REQUIRE(xd && wG && t && stencil_ok(sG) && B > 0 && G > 0 && F > 0 && h > 0 && w > 0, GRR_ERR_INVALID_ARG,
              "grr_gtv_rhs_half: bad args");
  GRR_REQUIRE(!prox || log_gamma, GRR_ERR_INVALID_ARG, "grr_gtv_rhs_half: prox needs log_gamma");
  OpArgs a{};
  a.x = xd; a.wG = wG; a.sG = sG; a.log_gamma = log_gamma; a.out = t;
  a.G = G; a.F = F; a.H = h; a.W = w;
  hipStream_t s = (hipStream_t)stream;
  if (prox) return launch_op<false, GTV_PROX, EPI_HALF>(a, B, s, "grr_gtv_rhs_half");
  return launch_op<false, GTV_PAIR, EPI_HALF>(a, B, s, "grr_gtv_rhs_half");
}

grr_status grr_gtv_rhs_full(const float* x, const float* y, const float* wG, grr_stencil sG, int prox,
                            const float* log_gamma, const float* log_ro0, const float* t_half, const float* log_ro1,
                            float* b_out, float* xd_out, int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && y && wG && b_out && log_ro0 && stencil_ok(sG) && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_gtv_rhs_full: bad args");
  GRR_REQUIRE(!prox || log_gamma, GRR_ERR_INVALID_ARG, "grr_gtv_rhs_full: prox needs log_gamma");
  GRR_REQUIRE(!t_half || log_ro1, GRR_ERR_INVALID_ARG, "grr_gtv_rhs_full: t_half needs log_ro1");
  GRR_REQUIRE(!(t_half || xd_out) || (H % 2 == 0 && W % 2 == 0), GRR_ERR_SHAPE,
              "grr_gtv_rhs_full: two-scale operator needs even H, W (got %dx%d)", H, W);
  OpArgs a{};
  a.x = x; a.y = y; a.wG = wG; a.sG = sG; a.log_gamma = log_gamma; a.log_g = log_ro0;
  a.t_half = t_half; a.log_half = log_ro1; a.out = b_out; a.xd_out = xd_out;
  a.G = G; a.F = F; a.H = H; a.W = W;
  hipStream_t s = (hipStream_t)stream;
  if (prox) return launch_op<false, GTV_PROX, EPI_RHS>(a, B, s, "grr_gtv_rhs_full");
  return launch_op<false, GTV_PAIR, EPI_RHS>(a, B, s, "grr_gtv_rhs_full");
}

grr_status grr_system_step(const float* x, const float* b, const float* u_prev, const float* t_half, const float* wL,
                           const float* cG, grr_stencil sL, grr_stencil sG, const float* log_mu0,
                           const float* log_ro0, const float* alpha, const float* beta, const float* skip,
                           const float* y_skip, float* x_out, float* u_out, float* xd_out, int B, int G, int F,
                           int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && b && alpha && x_out && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_system_step: bad args");
  GRR_REQUIRE(wL || cG, GRR_ERR_INVALID_ARG, "grr_system_step: need GLR and/or GTV weights");
  GRR_REQUIRE(!wL || (stencil_ok(sL) && log_mu0), GRR_ERR_INVALID_ARG, "grr_system_step: GLR params missing");
  GRR_REQUIRE(!cG || (stencil_ok(sG) && log_ro0), GRR_ERR_INVALID_ARG, "grr_system_step: GTV params missing");
  GRR_REQUIRE(!skip || y_skip, GRR_ERR_INVALID_ARG, "grr_system_step: skip needs y_skip");
  GRR_REQUIRE(!(t_half || xd_out) || (H % 2 == 0 && W % 2 == 0), GRR_ERR_SHAPE,
              "grr_system_step: two-scale operator needs even H, W (got %dx%d)", H, W);
  GRR_REQUIRE(x_out != x && x_out != b && (!u_prev || x_out != u_prev), GRR_ERR_INVALID_ARG,
              "grr_system_step: x_out must not alias an input (halo reads)");
  OpArgs a{};
  a.x = x; a.b = b; a.u_prev = u_prev; a.t_half = t_half; a.wL = wL; a.wG = cG; a.sL = sL; a.sG = sG;
  a.log_l = log_mu0; a.log_g = log_ro0; a.alpha = alpha; a.beta = beta; a.skip = skip; a.y = y_skip;
  a.out = x_out; a.u_out = u_out; a.xd_out = xd_out;
  a.G = G; a.F = F; a.H = H; a.W = W;
  hipStream_t s = (hipStream_t)stream;
  if (wL && cG) return launch_op<true, GTV_PAIR, EPI_STEP>(a, B, s, "grr_system_step");
  if (wL) return launch_op<true, GTV_NONE, EPI_STEP>(a, B, s, "grr_system_step");
  return launch_op<false, GTV_PAIR, EPI_STEP>(a, B, s, "grr_system_step");
}

}  // extern "C"
