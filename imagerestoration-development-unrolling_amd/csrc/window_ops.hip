// Window-graph operators: the image-domain mixture-GTV solvers of the older reference
// models, whose graphs connect every pixel to K neighbours of a connection window
// (3x3 ring: K = 8, 5x5 diamond: K = 12, full 5x5: K = 24) instead of the 4-neighbour
// graphs of the v1.0 path.
//
// REF7 = exploration/model_multiscale_mixture_GLR/lib/model_GLR_GTV_deep_v7.py
//   GLRFast (:274-511), GTVFast (:514-782), MixtureGTV (:802-1016)
// REF1 = exploration/model_multiscale_mixture_GLR/lib/model_GLR_GTV_deep_v1.py
//   the same solver without the stats stencils (:187-676)
//
// Kernels:
//   win_edge_weights_kernel  one pixel per thread: normalise + M, K similarities, softmax
//   win_solver_kernel        one (b, graph, 16x64 tile) per workgroup, the signal channels of
//                            the graph in turn: x tile (halo R+2) -> S x (reflect frame) for
//                            both modules -> l = S x - W S x and o = C^T phi(C x) (halo 1)
//                            -> S^T (zero frame) and the epilogue (CG step or right-hand
//                            side).  The edge tensors [B,G,F,K,H,W] of the reference never
//                            exist; every intermediate stays in LDS.
//   win_mix_kernel           sum_g x[b,g,c] score[b,g] + dc (REF7:1006-1009)
#include "grr_common.h"

namespace grr {
namespace {

constexpr int kMaxEdges = 24;
constexpr int NTW = 256;

struct WinDelta {
  int8_t dy[kMaxEdges];
  int8_t dx[kMaxEdges];
};

__device__ __forceinline__ float soft_phi(float t, float gm) {
  // 2 soft(t, gamma) - t: the edge signal C^T sees after one ADMM update from bias 0
  // (eps = soft(t), bias = t - eps, eps - bias, REF7:958-965)
  const float lo = t < -gm ? t + gm : 0.f;
  const float hi = t > gm ? t - gm : 0.f;
  const float eps = lo + hi;
  return eps - (t - eps);
}

// ---------------------------------------------------------------------------
// Edge weights (REF7:418-446): f^ = f / max(|f|_2, 1e-12) * M over the F node features,
// s_e(p) = sum_f f^(p) f^(clamp(p + delta_e)), w = softmax_e(s), deg = sum_e w.
// grid (ceil(HW / NTW), B*G)
// ---------------------------------------------------------------------------
template <int FMAX>
__global__ __launch_bounds__(NTW) void win_edge_weights_kernel(const float* __restrict__ feat, int64_t bstride,
                                                               const float* __restrict__ multiM, WinDelta d,
                                                               int K, float* __restrict__ w,
                                                               float* __restrict__ deg, int G, int F, int H,
                                                               int W) {
  const int HW = H * W;
  const int p = blockIdx.x * NTW + threadIdx.x;
  if (p >= HW) return;
  const int bg = blockIdx.y, g = bg % G, b = bg / G;
  const float* fp = feat + (int64_t)b * bstride + (int64_t)g * F * HW;
  const int r = p / W, c = p - r * W;
  float m[FMAX], a[FMAX];
  float nrm = 0.f;
#pragma unroll
  for (int f = 0; f < FMAX; ++f) {
    m[f] = f < F ? multiM[g * F + f] : 0.f;
    a[f] = f < F ? fp[(int64_t)f * HW + p] : 0.f;
    nrm += a[f] * a[f];
  }
  const float inv = 1.f / fmaxf(sqrtf(nrm), 1e-12f);
#pragma unroll
  for (int f = 0; f < FMAX; ++f) a[f] = (a[f] * inv) * m[f];
  float s[kMaxEdges];
  float smax = -INFINITY;
#pragma unroll
  for (int e = 0; e < kMaxEdges; ++e) {
    if (e < K) {
      const int q = clampi(r + d.dy[e], 0, H - 1) * W + clampi(c + d.dx[e], 0, W - 1);
      float bq[FMAX];
      float nq = 0.f;
#pragma unroll
      for (int f = 0; f < FMAX; ++f) {
        bq[f] = f < F ? fp[(int64_t)f * HW + q] : 0.f;
        nq += bq[f] * bq[f];
      }
      const float iq = 1.f / fmaxf(sqrtf(nq), 1e-12f);
      float dot = 0.f;
#pragma unroll
      for (int f = 0; f < FMAX; ++f) dot += a[f] * ((bq[f] * iq) * m[f]);
      s[e] = dot;
      smax = fmaxf(smax, dot);
    }
  }
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < kMaxEdges; ++e)
    if (e < K) {
      s[e] = expf(s[e] - smax);
      sum += s[e];
    }
  const float isum = 1.f / sum;
  float* wp = w + (int64_t)bg * K * HW + p;
  float dsum = 0.f;
#pragma unroll
  for (int e = 0; e < kMaxEdges; ++e)
    if (e < K) {
      const float v = s[e] * isum;
      wp[(int64_t)e * HW] = v;
      dsum += v;
    }
  if (deg) deg[(int64_t)bg * HW + p] = dsum;
}

// ---------------------------------------------------------------------------
// Pair weights of the linear GTV term (solver modes 0, 1, 3).  The frame-dropped C^T scatter pairs
// each directed edge with its reverse: C^T C s (q) = sum_e c_e(q) (s(q) - s(clamp(q + d_e))) with
// c_e(q) = w_e(q)^2 + [q + d_e inside] w_e'(q + d_e)^2, e' the edge of offset -d_e (REF7:748-774
// for the scatter; the window offsets are symmetric).  The solver then loads K weights per
// position instead of K plus K gathered reverse weights.   grid (ceil(HW / NTW), B*G)
// ---------------------------------------------------------------------------
struct WinOpp {
  int8_t e[kMaxEdges];
};
template <int KT>   // KT = K at compile time (8, 12, 24: every load issued up front), 0 = runtime K
__global__ __launch_bounds__(NTW) void win_pair_weights_kernel(const float* __restrict__ w, float* __restrict__ c,
                                                               WinDelta d, WinOpp opp, int K_, int H, int W) {
  constexpr int KE = KT > 0 ? KT : kMaxEdges;
  const int K = KT > 0 ? KT : K_;
  const int HW = H * W;
  const int p = blockIdx.x * NTW + threadIdx.x;
  if (p >= HW) return;
  const int r = p / W, col = p - r * W;
  const float* wp = w + (int64_t)blockIdx.y * K * HW;
  float* cp = c + (int64_t)blockIdx.y * K * HW;
  float we[KE], wr[KE];
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    if (KT == 0 && e >= K) break;
    const int ny = r + d.dy[e], nx = col + d.dx[e];
    const bool in = ny >= 0 && ny < H && nx >= 0 && nx < W;
    we[e] = wp[(int64_t)e * HW + p];
    wr[e] = in ? wp[(int64_t)opp.e[e] * HW + ny * W + nx] : 0.f;
  }
#pragma unroll
  for (int e = 0; e < KE; ++e) {
    if (KT == 0 && e >= K) break;
    cp[(int64_t)e * HW + p] = we[e] * we[e] + wr[e] * wr[e];
  }
}

// ---------------------------------------------------------------------------
// Solver kernel.  Tile TH x TW outputs of one (b, g); R = window reach (1 or 2).
//   MODE 0 (CG step, REF7:892-911, :951-990):  A x = x + mu S_L^T (S_L x - W_L S_L x)
//          + ro S_G^T C^T C S_G x;  u = (b - A x) [+ beta u_prev];  x' = x + alpha u
//   MODE 1 (rhs, REF7:945-949):   out = ro S_G^T C^T C S_G x + y           (eps = C x, bias 0)
//   MODE 2 (prox rhs, REF7:958-967): out = ro S_G^T C^T phi(C S_G x) + y, phi(t) = 2 soft(t) - t
//   MODE 3 (module apply, GLRFast/GTVFast.forward, REF7:503-511, :776-782):
//          out = mu S_L^T (S_L x - W_L S_L x) [if wL] + ro S_G^T C^T C S_G x [if wG]
// The S stencils read x with a reflect frame (REF7:449-467, 'reflect'); the neighbour reads of
// L and C clamp to the frame (replicate pad, REF7:374-398); S^T and the C^T scatter drop what
// lands outside (conv_transpose2d padding 1 / pad-subtract-crop, REF7:469-488, :748-774).
// ---------------------------------------------------------------------------
constexpr int TH = 16, TW = 64;

struct WinArgs {
  const float* x;        // [B,G,Fs,H,W] or, x_rep, [B,Fs,H,W] shared by the graphs
  const float* y;        // MODE 0: rhs b [B,G,Fs,H,W]; MODE 1/2: [B,Fs,H,W] shared by the graphs
  const float* u_prev;   // MODE 0, may be null
  const float* wL;       // [B,G,K,H,W] (MODE 0)
  const float* wG;       // [B,G,K,H,W]
  const float* tapsL;    // [5] c,u,l,r,d (MODE 0)
  const float* tapsG;    // [5]
  const float* mu;       // [G] linear (MODE 0)
  const float* ro;       // [G] linear
  const float* log_gamma;   // [G] (MODE 2)
  const float* alpha;    // [G] (MODE 0)
  const float* beta;     // [G] (MODE 0, with u_prev)
  float* out;            // [B,G,Fs,H,W]
  float* u_out;          // MODE 0, may be null
  int x_rep, K, G, Fs, H, W, tiles_x;
  WinDelta d;
};

__device__ __forceinline__ int reflect1(int v, int n) {   // one-pixel reflect frame
  v = v < 0 ? -v : v;
  return v > n - 1 ? 2 * (n - 1) - v : v;
}

// Block = NTS threads; all Fs <= FSMAX signal channels of the graph stay in LDS together so
// each edge weight is fetched once per position and applied to every channel.  KT = K at
// compile time (8, 12, 24: the edge loops unroll and every weight load is issued up front;
// 0 = runtime K).
constexpr int NTS = 512, FSMAX = 3;
static_assert(FSMAX * TH * TW % NTS == 0, "epilogue slots");

// PAIR (modes 0, 1, 3): wG holds the pair weights of win_pair_weights_kernel.
template <int R, int MODE, int KT, bool PAIR = false>
__global__ __launch_bounds__(NTS, KT == 24 ? 2 : 4) void win_solver_kernel(WinArgs a) {
  constexpr bool GLR = MODE == 0 || MODE == 3;
  constexpr int HS = R + 1, SH = TH + 2 * HS, SW = TW + 2 * HS;   // s region
  constexpr int LH = TH + 2, LW = TW + 2;                          // l / o region (halo 1)
  constexpr int NS = SH * SW, NL = LH * LW;
  __shared__ float sg[FSMAX * NS];
  __shared__ float sl[GLR ? FSMAX * NS : 1];
  __shared__ float os[FSMAX * NL];
  __shared__ float ls[GLR ? FSMAX * NL : 1];

  const int H = a.H, W = a.W, G = a.G, Fs = a.Fs;
  const int K = KT > 0 ? KT : a.K;
  const int64_t HW = (int64_t)H * W;
  const int tile = blockIdx.x, bg = blockIdx.y;
  const int g = bg % G, b = bg / G;
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int tid = threadIdx.x;

  const bool has_gtv = a.wG != nullptr, has_glr = GLR && a.wL != nullptr;
  float kG[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, kL[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  if (has_gtv) {
#pragma unroll
    for (int i = 0; i < 5; ++i) kG[i] = a.tapsG[i];
  }
  if (has_glr) {
#pragma unroll
    for (int i = 0; i < 5; ++i) kL[i] = a.tapsL[i];
  }
  const float ro = a.ro ? a.ro[g] : 1.f;
  const float mu = has_glr ? (a.mu ? a.mu[g] : 1.f) : 0.f;
  const float gam = MODE == 2 ? expf(a.log_gamma[g]) : 0.f;
  const float alpha = MODE == 0 ? a.alpha[g] : 0.f;
  const bool use_beta = MODE == 0 && a.u_prev != nullptr;
  const float beta = use_beta ? a.beta[g] : 0.f;
  const float* wLp = has_glr ? a.wL + (int64_t)bg * K * HW : nullptr;
  const float* wGp = has_gtv ? a.wG + (int64_t)bg * K * HW : nullptr;

  // ---- epilogue operands of this thread's outputs, loaded now so their latency hides
  //      behind the s / l / o phases
  constexpr int EPT = FSMAX * TH * TW / NTS;
  float ex[EPT], eb[EPT], eu[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int i = tid + k * NTS;
    const int c = i / (TH * TW), j = i - c * (TH * TW);
    const int py = y0 + j / TW, px = x0 + (j % TW);
    const bool ok = c < Fs && py < H && px < W;
    const int64_t off = ok ? ((int64_t)bg * Fs + c) * HW + (int64_t)py * W + px : 0;
    ex[k] = eb[k] = eu[k] = 0.f;
    if constexpr (MODE == 0) {
      if (ok) {
        ex[k] = a.x[off];
        eb[k] = a.y[off];
        if (use_beta) eu[k] = a.u_prev[off];
      }
    } else if constexpr (MODE == 1 || MODE == 2) {
      if (ok) eb[k] = a.y[((int64_t)b * Fs + c) * HW + (int64_t)py * W + px];
    }
  }
  // ---- s = S x of every channel on the s region, straight from global memory (the five
  //      taps of all channels in flight together; reflect frame; out-of-frame s is never read)
  for (int i = tid; i < NS; i += NTS) {
    const int ry = i / SW, rx = i - ry * SW;
    const int gy = y0 - HS + ry, gx = x0 - HS + rx;
    const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
    const int cy = clampi(gy, 0, H - 1), cx = clampi(gx, 0, W - 1);
    const int ru = reflect1(cy - 1, H), rd = reflect1(cy + 1, H), rl = reflect1(cx - 1, W), rr = reflect1(cx + 1, W);
    const int oc = cy * W + cx, ou = ru * W + cx, od = rd * W + cx, ol = cy * W + rl, orr = cy * W + rr;
    float xv[FSMAX][5];
#pragma unroll
    for (int c = 0; c < FSMAX; ++c) {
      const float* xp = a.x + (a.x_rep ? ((int64_t)b * Fs + min(c, Fs - 1)) * HW
                                       : ((int64_t)bg * Fs + min(c, Fs - 1)) * HW);
      xv[c][0] = xp[oc]; xv[c][1] = xp[ou]; xv[c][2] = xp[ol]; xv[c][3] = xp[orr]; xv[c][4] = xp[od];
    }
#pragma unroll
    for (int c = 0; c < FSMAX; ++c) {
      if (c < Fs) {
        float v = kG[0] * xv[c][0];
        v += kG[1] * xv[c][1]; v += kG[2] * xv[c][2]; v += kG[3] * xv[c][3]; v += kG[4] * xv[c][4];
        sg[c * NS + i] = in ? v : 0.f;
        if constexpr (GLR) {
          float w = kL[0] * xv[c][0];
          w += kL[1] * xv[c][1]; w += kL[2] * xv[c][2]; w += kL[3] * xv[c][3]; w += kL[4] * xv[c][4];
          sl[c * NS + i] = in ? w : 0.f;
        }
      }
    }
  }
  __syncthreads();
  // ---- l and o of every channel on the tile + 1-pixel halo (zero outside the frame)
  for (int i = tid; i < NL; i += NTS) {
    const int ry = i / LW, rx = i - ry * LW;
    const int qy = y0 - 1 + ry, qx = x0 - 1 + rx;
    const bool in = qy >= 0 && qy < H && qx >= 0 && qx < W;
    const int64_t q = (int64_t)qy * W + qx;
    const int sq = (qy - (y0 - HS)) * SW + (qx - (x0 - HS));
    float ov[FSMAX] = {0.f, 0.f, 0.f}, lv[FSMAX] = {0.f, 0.f, 0.f};
    constexpr int KE = KT > 0 ? KT : kMaxEdges;
    if (PAIR && in && has_gtv) {
      // sum_e c_e(q) (s(q) - s(clamp(q + delta_e))): K pair weights, no reverse-edge gathers
      float cf[KE];
      int sn[KE];
#pragma unroll
      for (int e = 0; e < KE; ++e) {
        if (KT == 0 && e >= K) break;
        const int ny = clampi(qy + a.d.dy[e], 0, H - 1), nx = clampi(qx + a.d.dx[e], 0, W - 1);
        sn[e] = (ny - (y0 - HS)) * SW + (nx - (x0 - HS));
        cf[e] = wGp[e * HW + q];
      }
#pragma unroll
      for (int c = 0; c < FSMAX; ++c) {
        if (c < Fs) {
          const float* sc = sg + c * NS;
          const float sv = sc[sq];
          float acc = 0.f;
#pragma unroll
          for (int e = 0; e < KE; ++e) {
            if (KT == 0 && e >= K) break;
            acc += cf[e] * (sv - sc[sn[e]]);
          }
          ov[c] = acc;
        }
      }
    } else if (in && has_gtv) {
      // every weight of this position first (one batch of loads in flight), then the math:
      // sum_e z_e(q) - sum_e [q - delta_e inside] z_e(q - delta_e), z_e = w_e phi(w_e s - w_e s(+delta_e))
      float wf[KE], wb[KE];
      int sn[KE], sp[KE];
#pragma unroll
      for (int e = 0; e < KE; ++e) {
        if (KT == 0 && e >= K) break;
        const int ny = clampi(qy + a.d.dy[e], 0, H - 1), nx = clampi(qx + a.d.dx[e], 0, W - 1);
        sn[e] = (ny - (y0 - HS)) * SW + (nx - (x0 - HS));
        const int py = qy - a.d.dy[e], px = qx - a.d.dx[e];
        const bool pin = py >= 0 && py < H && px >= 0 && px < W;
        const int cy = pin ? py : qy, cx = pin ? px : qx;
        sp[e] = pin ? (cy - (y0 - HS)) * SW + (cx - (x0 - HS)) : -1;
        wf[e] = wGp[e * HW + q];
        wb[e] = wGp[e * HW + (int64_t)cy * W + cx];
      }
#pragma unroll
      for (int c = 0; c < FSMAX; ++c) {
        if (c < Fs) {
          const float* sc = sg + c * NS;
          const float sv = sc[sq];
          float acc = 0.f;
#pragma unroll
          for (int e = 0; e < KE; ++e) {
            if (KT == 0 && e >= K) break;
            float t = wf[e] * sv - wf[e] * sc[sn[e]];
            if constexpr (MODE == 2) t = soft_phi(t, gam);
            acc += t * wf[e];
          }
#pragma unroll
          for (int e = 0; e < KE; ++e) {
            if (KT == 0 && e >= K) break;
            if (sp[e] >= 0) {
              float t = wb[e] * sc[sp[e]] - wb[e] * sv;   // its neighbour p + delta_e is q
              if constexpr (MODE == 2) t = soft_phi(t, gam);
              acc -= t * wb[e];
            }
          }
          ov[c] = acc;
        }
      }
    }
    if constexpr (GLR) {
      if (in && has_glr) {
        float wl[KE];
        int sn[KE];
#pragma unroll
        for (int e = 0; e < KE; ++e) {
          if (KT == 0 && e >= K) break;
          const int ny = clampi(qy + a.d.dy[e], 0, H - 1), nx = clampi(qx + a.d.dx[e], 0, W - 1);
          sn[e] = (ny - (y0 - HS)) * SW + (nx - (x0 - HS));
          wl[e] = wLp[e * HW + q];
        }
#pragma unroll
        for (int c = 0; c < FSMAX; ++c) {
          if (c < Fs) {
            const float* sc = sl + c * NS;
            float wx = 0.f;
#pragma unroll
            for (int e = 0; e < KE; ++e) {
              if (KT == 0 && e >= K) break;
              wx += wl[e] * sc[sn[e]];
            }
            lv[c] = sc[sq] - wx;
          }
        }
      }
    }
#pragma unroll
    for (int c = 0; c < FSMAX; ++c) {
      if (c < Fs) {
        os[c * NL + i] = ov[c];
        if constexpr (GLR) ls[c * NL + i] = lv[c];
      }
    }
  }
  __syncthreads();
  // ---- S^T (zero frame) and the epilogue on the tile, every channel
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    const int i = tid + k * NTS;
    const int c = i / (TH * TW), j = i - c * (TH * TW);
    const int ry = j / TW, rx = j - ry * TW;
    const int py = y0 + ry, px = x0 + rx;
    if (c >= Fs || py >= H || px >= W) continue;
    const int li = c * NL + (ry + 1) * LW + (rx + 1);
    // sum_t k_t v(p - t): up tap reads p + down, left tap p + right, ...
    float tg = kG[0] * os[li];
    tg += kG[1] * os[li + LW]; tg += kG[2] * os[li + 1]; tg += kG[3] * os[li - 1]; tg += kG[4] * os[li - LW];
    const int64_t plane = ((int64_t)bg * Fs + c) * HW;
    const int64_t p = (int64_t)py * W + px;
    if constexpr (MODE == 0) {
      float tl = kL[0] * ls[li];
      tl += kL[1] * ls[li + LW]; tl += kL[2] * ls[li + 1]; tl += kL[3] * ls[li - 1]; tl += kL[4] * ls[li - LW];
      const float xv = ex[k];
      const float ax = (xv + tl * mu) + tg * ro;
      float u = eb[k] - ax;
      if (use_beta) u = u + beta * eu[k];
      a.out[plane + p] = xv + alpha * u;
      if (a.u_out) a.u_out[plane + p] = u;
    } else if constexpr (MODE == 3) {
      float tl = kL[0] * ls[li];
      tl += kL[1] * ls[li + LW]; tl += kL[2] * ls[li + 1]; tl += kL[3] * ls[li - 1]; tl += kL[4] * ls[li - LW];
      float v = has_glr ? tl * mu : 0.f;
      if (has_gtv) v = has_glr ? v + tg * ro : tg * ro;
      a.out[plane + p] = v;
    } else {
      a.out[plane + p] = tg * ro + eb[k];
    }
  }
}

// out[b,c,p] = sum_g x[b,g,c,p] * score[b,g,p] (+ dc[b,c,p])    grid (ceil(HW/NTW), B*Fs)
__global__ __launch_bounds__(NTW) void win_mix_kernel(const float* __restrict__ x, const float* __restrict__ score,
                                                      const float* __restrict__ dc, float* __restrict__ out, int G,
                                                      int Fs, int HW) {
  const int p = blockIdx.x * NTW + threadIdx.x;
  if (p >= HW) return;
  const int bc = blockIdx.y, c = bc % Fs, b = bc / Fs;
  float acc = 0.f;
  for (int g = 0; g < G; ++g)
    acc += x[(((int64_t)b * G + g) * Fs + c) * HW + p] * score[((int64_t)b * G + g) * HW + p];
  if (dc) acc += dc[(int64_t)bc * HW + p];
  out[(int64_t)bc * HW + p] = acc;
}

grr_status load_delta(const int32_t* delta, int K, WinDelta* d, int* reach) {
  GRR_REQUIRE(delta != nullptr && K >= 1 && K <= kMaxEdges, GRR_ERR_UNSUPPORTED,
              "window graph: 1 <= K <= %d edges required (got %d)", kMaxEdges, K);
  int r = 0;
  for (int e = 0; e < K; ++e) {
    const int dy = delta[2 * e], dx = delta[2 * e + 1];
    GRR_REQUIRE(dy >= -2 && dy <= 2 && dx >= -2 && dx <= 2, GRR_ERR_UNSUPPORTED,
                "window graph: edge offsets must lie in a 5x5 window (edge %d = (%d, %d))", e, dy, dx);
    d->dy[e] = (int8_t)dy;
    d->dx[e] = (int8_t)dx;
    r = max(r, max(abs(dy), abs(dx)));
  }
  *reach = r;
  return GRR_OK;
}

}  // namespace
}  // namespace grr

using namespace grr;

extern "C" {

grr_status grr_win_edge_weights(const float* feat, int64_t feat_bstride, const float* multiM, const int32_t* delta,
                                int K, float* w, float* deg, int B, int G, int F, int H, int W, void* stream) {
  GRR_REQUIRE(feat && multiM && w && B > 0 && G > 0 && F > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_win_edge_weights: bad argument");
  GRR_REQUIRE(F <= GRR_MAX_NODE_FTS, GRR_ERR_UNSUPPORTED, "grr_win_edge_weights: F=%d > %d", F, GRR_MAX_NODE_FTS);
  GRR_REQUIRE((int64_t)B * G <= 65535 && (int64_t)H * W * K < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_win_edge_weights: grid too large");
  WinDelta d{};
  int reach = 0;
  const grr_status st = load_delta(delta, K, &d, &reach);
  if (st != GRR_OK) return st;
  const dim3 grid((H * W + NTW - 1) / NTW, B * G);
  hipStream_t s = (hipStream_t)stream;
  if (F <= 4)
    hipLaunchKernelGGL(win_edge_weights_kernel<4>, grid, dim3(NTW), 0, s, feat, feat_bstride, multiM, d, K, w, deg, G,
                       F, H, W);
  else if (F <= 12)
    hipLaunchKernelGGL(win_edge_weights_kernel<12>, grid, dim3(NTW), 0, s, feat, feat_bstride, multiM, d, K, w, deg,
                       G, F, H, W);
  else
    hipLaunchKernelGGL(win_edge_weights_kernel<GRR_MAX_NODE_FTS>, grid, dim3(NTW), 0, s, feat, feat_bstride, multiM,
                       d, K, w, deg, G, F, H, W);
  return launch_status("grr_win_edge_weights");
}

grr_status grr_win_pair_weights(const float* w, const int32_t* delta, int K, float* c, int B, int G, int H, int W,
                                void* stream) {
  GRR_REQUIRE(w && c && w != c && B > 0 && G > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_win_pair_weights: bad argument");
  GRR_REQUIRE((int64_t)B * G <= 65535 && (int64_t)H * W * K < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_win_pair_weights: grid too large");
  WinDelta d{};
  int reach = 0;
  const grr_status st = load_delta(delta, K, &d, &reach);
  if (st != GRR_OK) return st;
  WinOpp opp{};
  for (int e = 0; e < K; ++e) {
    int o = -1;
    for (int f = 0; f < K; ++f)
      if (d.dy[f] == -d.dy[e] && d.dx[f] == -d.dx[e]) o = f;
    GRR_REQUIRE(o >= 0, GRR_ERR_UNSUPPORTED, "grr_win_pair_weights: edge %d = (%d, %d) has no reverse edge", e,
                (int)d.dy[e], (int)d.dx[e]);
    opp.e[e] = (int8_t)o;
  }
  const dim3 grid((H * W + NTW - 1) / NTW, B * G);
  hipStream_t s = (hipStream_t)stream;
  if (K == 8) hipLaunchKernelGGL(win_pair_weights_kernel<8>, grid, dim3(NTW), 0, s, w, c, d, opp, K, H, W);
  else if (K == 12) hipLaunchKernelGGL(win_pair_weights_kernel<12>, grid, dim3(NTW), 0, s, w, c, d, opp, K, H, W);
  else if (K == 24) hipLaunchKernelGGL(win_pair_weights_kernel<24>, grid, dim3(NTW), 0, s, w, c, d, opp, K, H, W);
  else hipLaunchKernelGGL(win_pair_weights_kernel<0>, grid, dim3(NTW), 0, s, w, c, d, opp, K, H, W);
  return launch_status("grr_win_pair_weights");
}

grr_status grr_win_solver(int mode, const float* x, int x_rep, const float* y, const float* u_prev, const float* wL,
                          const float* wG, const float* tapsL, const float* tapsG, const float* mu, const float* ro,
                          const float* log_gamma, const float* alpha, const float* beta, const int32_t* delta, int K,
                          float* out, float* u_out, int B, int G, int Fs, int H, int W, void* stream) {
  const bool pair = mode >= 4;   // modes 4, 5, 7: 0, 1, 3 with wG = grr_win_pair_weights(w_G)
  GRR_REQUIRE(mode >= 0 && mode <= 7 && mode != 6, GRR_ERR_INVALID_ARG, "grr_win_solver: mode %d", mode);
  mode &= 3;
  GRR_REQUIRE(x && out && B > 0 && G > 0 && Fs > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_win_solver: bad argument");
  GRR_REQUIRE(mode == 3 || (y && wG && tapsG && ro), GRR_ERR_INVALID_ARG, "grr_win_solver: y, wG, tapsG, ro required");
  GRR_REQUIRE(mode != 3 || ((wL || wG) && (!wL || tapsL) && (!wG || tapsG)), GRR_ERR_INVALID_ARG,
              "grr_win_solver: apply needs wL (+ tapsL) and / or wG (+ tapsG)");
  GRR_REQUIRE(mode != 0 || (wL && tapsL && mu && alpha && (!u_prev || beta)), GRR_ERR_INVALID_ARG,
              "grr_win_solver: the CG step needs wL, tapsL, mu, alpha (and beta with u_prev)");
  GRR_REQUIRE(mode != 2 || log_gamma, GRR_ERR_INVALID_ARG, "grr_win_solver: prox needs log_gamma");
  GRR_REQUIRE(!(mode == 0 && x_rep), GRR_ERR_INVALID_ARG, "grr_win_solver: the CG step needs a per-graph x");
  GRR_REQUIRE(H >= 2 && W >= 2, GRR_ERR_SHAPE, "grr_win_solver: reflect padding needs H, W >= 2");
  GRR_REQUIRE(Fs <= FSMAX, GRR_ERR_UNSUPPORTED, "grr_win_solver: at most %d signal channels (got %d)", FSMAX, Fs);
  GRR_REQUIRE((int64_t)B * G <= 65535 && (int64_t)H * W * K < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_win_solver: grid too large");
  WinArgs a{};
  int reach = 0;
  const grr_status st = load_delta(delta, K, &a.d, &reach);
  if (st != GRR_OK) return st;
  a.x = x; a.y = y; a.u_prev = u_prev; a.wL = wL; a.wG = wG; a.tapsL = tapsL; a.tapsG = tapsG;
  a.mu = mu; a.ro = ro; a.log_gamma = log_gamma; a.alpha = alpha; a.beta = beta;
  a.out = out; a.u_out = u_out;
  a.x_rep = x_rep; a.K = K; a.G = G; a.Fs = Fs; a.H = H; a.W = W;
  a.tiles_x = (W + TW - 1) / TW;
  const int tiles = a.tiles_x * ((H + TH - 1) / TH);
  const dim3 grid(tiles, B * G);
  hipStream_t s = (hipStream_t)stream;
#define WIN_LAUNCH(R_, M_, K_, P_) hipLaunchKernelGGL((win_solver_kernel<R_, M_, K_, P_>), grid, dim3(NTS), 0, s, a)
#define WIN_MODES(R_, K_)                                                      \
  do {                                                                         \
    if (mode == 0) { if (pair) WIN_LAUNCH(R_, 0, K_, true); else WIN_LAUNCH(R_, 0, K_, false); }   \
    else if (mode == 1) { if (pair) WIN_LAUNCH(R_, 1, K_, true); else WIN_LAUNCH(R_, 1, K_, false); } \
    else if (mode == 2) WIN_LAUNCH(R_, 2, K_, false);                          \
    else { if (pair) WIN_LAUNCH(R_, 3, K_, true); else WIN_LAUNCH(R_, 3, K_, false); }             \
  } while (0)
  if (reach <= 1) {
    if (K == 8) WIN_MODES(1, 8); else WIN_MODES(1, 0);
  } else {
    if (K == 12) WIN_MODES(2, 12); else if (K == 24) WIN_MODES(2, 24); else WIN_MODES(2, 0);
  }
#undef WIN_MODES
#undef WIN_LAUNCH
  return launch_status("grr_win_solver");
}

grr_status grr_win_mix(const float* x, const float* score, const float* dc, float* out, int B, int G, int Fs, int H,
                       int W, void* stream) {
  GRR_REQUIRE(x && score && out && B > 0 && G > 0 && Fs > 0 && H > 0 && W > 0, GRR_ERR_INVALID_ARG,
              "grr_win_mix: bad argument");
  GRR_REQUIRE((int64_t)B * Fs <= 65535 && (int64_t)H * W < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_win_mix: grid too large");
  const dim3 grid((H * W + NTW - 1) / NTW, B * Fs);
  hipLaunchKernelGGL(win_mix_kernel, grid, dim3(NTW), 0, (hipStream_t)stream, x, score, dc, out, G, Fs, H * W);
  return launch_status("grr_win_mix");
}

}  // extern "C"
