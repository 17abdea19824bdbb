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
#include <type_traits>

#include "grr_common.h"

namespace grr {

static thread_local std::string g_err;
static int g_kernel_variant = 0;   // grr_set_kernel_variant: 0 auto, 1 strip kernels only

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
  const float* log_l;   // GLR term scale (log, or linear when lin_l), NULL -> 1
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
  int nstrips, nsegs, sseg;
  int sw;               // row kernel, wide images: output columns per strip (W when one strip)
  int lin_l;            // log_l holds the scale itself (v10 MixtureGLR stores mu linearly)
  int wpb;              // row kernel: waves per block = channels of one graph walked in lockstep
  int x_rep, y_rep;     // operand is [B, F, H, W], replicated over the G graphs (channel g F + f reads f)
  uint32_t nunits, nblk;
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
// soft_threshold(t) = t - clamp(t, -gamma, gamma) is the same fp32 value as the reference's
// where(t < -g, t + g, 0) + where(t > g, t - g, 0) (t - (-g) == t + g exactly; t - t == +0),
// so one v_med3_f32 + a subtraction replaces two compares, two selects and two adds
__device__ __forceinline__ float prox_phi(float t, float gm) {
  const float eps = t - __builtin_amdgcn_fmed3f(t, -gm, gm);
  return eps - (t - eps);
}

// ---------------------------------------------------------------------------
// Streaming fused graph operator.
//
// One wave = one (b, channel) plane, one 64-column strip, one segment of SSEG output
// rows.  Lane = column.  The wave marches down the rows; each iteration loads one
// input row and advances a 4-stage pipeline held entirely in registers:
//     x row t  ->  s = S x at row t-1  ->  {l, o} at row t-2  ->  S^T + epilogue at row t-3
// Vertical neighbours are the previous iteration's registers; horizontal neighbours
// come from the adjacent lanes through DPP wave shifts (v_mov_b32_dpp wave_shr/shl:1).
// No LDS and no barriers.  Each stage needs one column of halo on each side, so a
// 64-lane strip produces SVALID = 58 output columns.  Row loads (one 256-B coalesced
// line per wave and operand) are issued two iterations ahead of their use (register
// ring of depth 2).
// ---------------------------------------------------------------------------
constexpr int SVALID = 58;   // output columns per strip (3-column halo each side)
// Output rows per wave segment (even; each segment re-reads a 6-row pipeline fill): chosen
// per launch by seg_rows() -- as long as the grid still holds >= SEG_MIN_WAVES waves, so
// the fill overhead shrinks (64 -> 256 rows: 9 % -> 2 % extra row reads) where the batch is large.
constexpr int SSEG = 64;               // shortest segment
constexpr int SEG_MIN_WAVES = 4096;    // 16 waves per CU
static int seg_rows(int H, uint64_t units_per_seg) {
  int sseg = (H + 1) & ~1;
  while (sseg > SSEG && units_per_seg * (uint64_t)((H + sseg - 1) / sseg) < SEG_MIN_WAVES) sseg = ((sseg / 2) + 1) & ~1;
  return sseg < SSEG ? SSEG : sseg;
}

// Cross-lane reads must execute with the whole wave active: a DPP read of a lane that
// is masked off returns 0.  The empty asm pins each result at its definition, so the
// compiler cannot sink the v_mov_b32_dpp into a divergent branch (it turned
// `c > 0 ? lane_prev(v) : 0` into an exec-masked branch before this was added).
__device__ __forceinline__ float lane_prev(float v) {  // value of lane-1 (column c-1)
  float r = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xF, 0xF, true));
  asm volatile("" : "+v"(r));
  return r;
}
__device__ __forceinline__ float lane_next(float v) {  // value of lane+1 (column c+1)
  float r = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xF, 0xF, true));
  asm volatile("" : "+v"(r));
  return r;
}

// Addressing: a wave-uniform row base (SGPRs) + a per-lane 32-bit byte offset, so the
// compiler can use the global_load/store "saddr" form with no per-access 64-bit VALU math.
__device__ __forceinline__ float gload(const float* row_base, uint32_t off_bytes) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(row_base) + off_bytes);
}
__device__ __forceinline__ void gstore(float* row_base, uint32_t off_bytes, float v) {
  *reinterpret_cast<float*>(reinterpret_cast<char*>(row_base) + off_bytes) = v;
}

// Every pipeline iteration issues the same sequence of memory operations, so hipcc's
// s_waitcnt bookkeeping stays exact across the loop and the loads issued two
// iterations ahead remain in flight: absent operands are read from this small
// device-resident line, and stores that must not land (halo lanes, pipeline-fill
// rows, outputs the caller did not ask for) go to a per-lane slot of it.
__device__ __attribute__((aligned(16))) float g_grr_scratch[256];   // 64 lanes x up to 16 B

// loads consumed by one pipeline iteration t (issued two iterations earlier)
struct RowLoads {
  float x;        // x row t
  float wl[4];    // GLR edge weights, row t-2
  float wg[4];    // GTV pair weights (2) or raw weights (4), row t-2
  float wup;      // prox: w_up at row t-1 (the scatter source below)
  float eb, eu, ey, th;  // epilogue operands at row t-3
};

template <bool GLR, int GTV, int EPI>
__global__ __launch_bounds__(NT) void graph_op_kernel(OpArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // channels fastest, then strips: a graph's channel waves are dispatch-adjacent (weights
  // shared through L2) and neighbouring strips (shared halo columns) stay on one XCD.
  uint32_t unit = xcd_remap(blockIdx.x, a.nblk) * 4 + wave;
  if (unit >= a.nunits) return;   // whole wave (uniform); wpb == 1 here, no barrier is met
  const int F = a.F;
  const int f = unit % F; unit /= F;
  const int strip = unit % a.nstrips; unit /= a.nstrips;
  const int seg = unit % a.nsegs; unit /= a.nsegs;
  const int g = unit % a.G;
  const int b = unit / a.G;
  const int H = a.H, W = a.W, C = a.G * F, ch = g * F + f;
  const int hh = H / 2, hw = W / 2;
  const int64_t HW = (int64_t)H * W;
  const int c = strip * SVALID - 3 + lane;
  const int cc = clampi(c, 0, W - 1);
  const bool cin = c >= 0 && c < W;
  const bool owner = lane >= 3 && lane < 3 + SVALID && cin;
  const int r0 = seg * a.sseg, r1 = min(r0 + a.sseg, H);
  float* const scratch = g_grr_scratch;
  const uint32_t vo = (uint32_t)cc * 4u, vo_half = (uint32_t)(cc >> 1) * 4u, vo_lane = (uint32_t)lane * 4u;
  const bool owner_xd = owner && (c & 1) == 0 && c + 1 < W;                       // D(x) writer

  const int64_t plane = ((int64_t)b * C + ch) * HW;
  const int64_t hplane = ((int64_t)b * C + ch) * (int64_t)hh * hw;
  const bool has_half = EPI != EPI_HALF && a.t_half != nullptr;
  const bool use_beta = EPI == EPI_STEP && a.beta != nullptr && a.u_prev != nullptr;
  const bool need_y = (EPI == EPI_RHS) || (EPI == EPI_STEP && a.skip != nullptr);
  const bool want_u = EPI == EPI_STEP && a.u_out != nullptr;
  const bool want_xd = a.xd_out != nullptr;
  const int np = GTV == GTV_PROX ? 4 : 2;
  // plane bases (uniform); absent operands point at the scratch line with row stride 0
  const int64_t rplane = ((int64_t)b * F + f) * HW;   // plane of a graph-replicated operand
  const float* px = a.x + (a.x_rep ? rplane : plane);
  const float* pwl = GLR ? a.wL + (int64_t)(b * a.G + g) * 4 * HW : nullptr;
  const float* pwg = GTV ? a.wG + (int64_t)(b * a.G + g) * np * HW : nullptr;
  const float* pb = EPI == EPI_STEP ? a.b + plane : scratch;
  const float* pu = use_beta ? a.u_prev + plane : scratch;
  const float* py = need_y ? a.y + (a.y_rep ? rplane : plane) : scratch;
  const float* pth = has_half ? a.t_half + hplane : scratch;
  float* pout = a.out + plane;
  float* puo = want_u ? a.u_out + plane : scratch;
  float* pxd = want_xd ? a.xd_out + hplane : scratch;
  const int ws_b = EPI == EPI_STEP ? W : 0, ws_u = use_beta ? W : 0, ws_y = need_y ? W : 0;
  const int ws_th = has_half ? hw : 0, ws_uo = want_u ? W : 0, ws_xd = want_xd ? hw : 0;
  const uint32_t vo_b = EPI == EPI_STEP ? vo : vo_lane, vo_u = use_beta ? vo : vo_lane;
  const uint32_t vo_y = need_y ? vo : vo_lane, vo_th = has_half ? vo_half : vo_lane;

  float sc_l = 1.f, sc_g = 1.f, sc_h = 1.f, gam = 0.f, alpha = 0.f, beta = 0.f, sk0 = 0.f, sk1 = 1.f;
  if (a.log_l) sc_l = a.lin_l ? a.log_l[g] : expf(a.log_l[g]);
  if (a.log_g) sc_g = expf(a.log_g[g]);
  if (a.log_half) sc_h = expf(a.log_half[g]);
  if constexpr (GTV == GTV_PROX) gam = expf(a.log_gamma[g]);
  if constexpr (EPI == EPI_STEP) {
    alpha = a.alpha[g];
    if (use_beta) beta = a.beta[g];
    if (a.skip) { sk0 = a.skip[0]; sk1 = a.skip[1]; }
  }
  const bool use_skip = EPI == EPI_STEP && a.skip != nullptr;
  Taps tL{}, tG{};
  if constexpr (GLR) tL = make_taps(a.sL, ch);
  if constexpr (GTV != GTV_NONE) tG = make_taps(a.sG, ch);

  auto issue = [&](int t, RowLoads& S) {
    S.x = gload(px + clampi(t, 0, H - 1) * W, vo);
    const int rw = clampi(t - 2, 0, H - 1) * W;
    if constexpr (GLR) {
#pragma unroll
      for (int e = 0; e < 4; ++e) S.wl[e] = gload(pwl + e * HW + rw, vo);
    }
    if constexpr (GTV == GTV_PAIR) {
      S.wg[0] = gload(pwg + rw, vo);
      S.wg[1] = gload(pwg + HW + rw, vo);
    }
    if constexpr (GTV == GTV_PROX) {
#pragma unroll
      for (int e = 0; e < 4; ++e) S.wg[e] = gload(pwg + e * HW + rw, vo);
      S.wup = gload(pwg + clampi(t - 1, 0, H - 1) * W, vo);
    }
    const int re = clampi(t - 3, 0, H - 1);
    if constexpr (EPI == EPI_STEP) {
      S.eb = gload(pb + re * ws_b, vo_b);
      S.eu = gload(pu + re * ws_u, vo_u);
    }
    if constexpr (EPI != EPI_HALF) {
      S.ey = gload(py + re * ws_y, vo_y);
      S.th = gload(pth + (re >> 1) * ws_th, vo_th);
    }
  };

  // pipeline registers (rows relative to the current iteration t)
  float X0 = 0.f, X1 = 0.f, X2 = 0.f, X3 = 0.f;   // x rows t-3 .. t
  float SL0 = 0.f, SL1 = 0.f, SL2 = 0.f;          // S_L x rows t-3 .. t-1
  float SG0 = 0.f, SG1 = 0.f, SG2 = 0.f;          // S_G x rows t-3 .. t-1
  float L0 = 0.f, L1 = 0.f, L2 = 0.f;             // l rows t-4 .. t-2
  float O0 = 0.f, O1 = 0.f, O2 = 0.f;             // o rows t-4 .. t-2
  float cv_prev = 0.f, wdn_prev = 0.f, xn_prev = 0.f;

  // ODD_Y: output row y = t-3 is odd in this body (segments start at even rows), so the
  // 2x2 pool of rows (y-1, y) is completed here.
  auto consume = [&](int t, const RowLoads& S, auto odd_tag) {
    constexpr bool ODD_Y = decltype(odd_tag)::value;
    // ---- stage 1: input row t
    X0 = X1; X1 = X2; X2 = X3; X3 = S.x;
    // ---- stage 2: s at row t-1 (replicate: X rows are clamped loads)
    {
      const float xl = lane_prev(X2), xr = lane_next(X2);
      if constexpr (GLR) {
        float sv = tL.u * X1;
        sv += tL.l * xl; sv += tL.c * X2; sv += tL.r * xr; sv += tL.d * X3;
        SL0 = SL1; SL1 = SL2; SL2 = sv;
      }
      if constexpr (GTV != GTV_NONE) {
        float sv = tG.u * X1;
        sv += tG.l * xl; sv += tG.c * X2; sv += tG.r * xr; sv += tG.d * X3;
        SG0 = SG1; SG1 = SG2; SG2 = sv;
      }
    }
    // ---- stage 3: l and o at row r = t-2 (zero outside the image: S^T's zero boundary)
    {
      const int r = t - 2;
      const bool rin = r >= 0 && r < H;
      if constexpr (GLR) {
        // (I - W) s with the replicate-clamped neighbour s(clamp(q + delta_e))  (REF:218-228)
        const float up = r > 0 ? SL0 : SL1;
        const float dn = r < H - 1 ? SL2 : SL1;
        const float pv = lane_prev(SL1), nx = lane_next(SL1);
        const float lf = c > 0 ? pv : SL1;
        const float rt = c < W - 1 ? nx : SL1;
        const float wx = ((S.wl[0] * up + S.wl[1] * lf) + S.wl[2] * rt) + S.wl[3] * dn;
        const float l = (rin && cin) ? SL1 - wx : 0.f;
        L0 = L1; L1 = L2; L2 = l;
      }
      if constexpr (GTV == GTV_PAIR) {
        // C^T C s with symmetrised pair weights (zero on edges leaving the image)
        const float chp = lane_prev(S.wg[0]);
        const float chl = c > 0 ? chp : 0.f;
        const float cvu = r > 0 ? cv_prev : 0.f;
        const float sv = SG1;
        const float snx = lane_next(SG1), spv = lane_prev(SG1);
        const float o = S.wg[0] * (sv - snx) + chl * (sv - spv) + S.wg[1] * (sv - SG2) + cvu * (sv - SG0);
        cv_prev = S.wg[1];
        const float ov = (rin && cin) ? o : 0.f;
        O0 = O1; O1 = O2; O2 = ov;
      }
      if constexpr (GTV == GTV_PROX) {
        // o = sum_e z_e(q) - sum_e z_e(q - delta_e),  z_e = phi(E_e) w_e  (REF:452-516, :765-781)
        const float sv = SG1;
        const float su = r > 0 ? SG0 : sv, sd = r < H - 1 ? SG2 : sv;
        const float spv = lane_prev(SG1), snx = lane_next(SG1);
        const float sl = c > 0 ? spv : sv, sr = c < W - 1 ? snx : sv;
        const float w0 = S.wg[0], w1 = S.wg[1], w2 = S.wg[2], w3 = S.wg[3];
        const float z0 = prox_phi(w0 * sv - w0 * su, gam) * w0;
        const float z1 = prox_phi(w1 * sv - w1 * sl, gam) * w1;
        const float z2 = prox_phi(w2 * sv - w2 * sr, gam) * w2;
        const float z3 = prox_phi(w3 * sv - w3 * sd, gam) * w3;
        float o = ((z0 + z1) + z2) + z3;
        // scatters landing on q, in edge order; frame-dropped when the source is outside
        const float wupb = S.wup;                       // w_up(q + down)
        const float wlfr = lane_next(w1);               // w_left(q + right)
        const float wrtl = lane_prev(w2);               // w_right(q - right)
        const float wdna = wdn_prev;                    // w_down(q - down)
        const float o1 = o - prox_phi(wupb * SG2 - wupb * sv, gam) * wupb;
        o = r < H - 1 ? o1 : o;
        const float o2 = o - prox_phi(wlfr * snx - wlfr * sv, gam) * wlfr;
        o = c < W - 1 ? o2 : o;
        const float o3 = o - prox_phi(wrtl * spv - wrtl * sv, gam) * wrtl;
        o = c > 0 ? o3 : o;
        const float o4 = o - prox_phi(wdna * SG0 - wdna * sv, gam) * wdna;
        o = r > 0 ? o4 : o;
        wdn_prev = w3;
        const float ov = (rin && cin) ? o : 0.f;
        O0 = O1; O1 = O2; O2 = ov;
      }
    }
    // ---- stage 4: S^T and the epilogue at row y = t-3
    const int y = t - 3;
    float tl = 0.f, tg = 0.f;
    if constexpr (GLR) {
      const float ln = lane_next(L1), lp = lane_prev(L1);
      float v = tL.u * L2;
      v += tL.l * ln; v += tL.c * L1; v += tL.r * lp; v += tL.d * L0;
      tl = v;
    }
    if constexpr (GTV != GTV_NONE) {
      const float on = lane_next(O1), op = lane_prev(O1);
      float v = tG.u * O2;
      v += tG.l * on; v += tG.c * O1; v += tG.r * op; v += tG.d * O0;
      tg = v;
    }
    const float th = 0.25f * S.th;
    float res, xn = 0.f, u = 0.f;
    if constexpr (EPI == EPI_HALF) {
      res = 0.f;                                        // mu * S_L^T l + ro * S_G^T o (REF:666-675)
      if constexpr (GLR) res = tl * sc_l;
      if constexpr (GTV != GTV_NONE) res = GLR ? res + tg * sc_g : tg * sc_g;
      xn = res;
    } else if constexpr (EPI == EPI_RHS) {
      res = S.ey + tg * sc_g;                           // (y + ro0 C^T phi(C x)) + ro1 U(t)
      if (has_half) res = res + th * sc_h;
      xn = res;
    } else {
      float ax = X0;                                    // A x = ((x + mu0 L x) + ro0 G x) + U(t)
      if constexpr (GLR) ax = ax + tl * sc_l;
      if constexpr (GTV != GTV_NONE) ax = ax + tg * sc_g;
      if (has_half) ax = ax + th;
      u = S.eb - ax;                                    // residual
      if (use_beta) u = u + beta * S.eu;                // heavy-ball direction (REF:789)
      xn = X0 + alpha * u;                              // x_{k+1}
      res = use_skip ? sk0 * S.ey + sk1 * xn : xn;      // block skip (REF:987)
    }
    // stores: same sequence every iteration; fill rows / halo lanes land in the scratch line
    const bool yv = y >= r0 && y < r1;
    const int yr = yv ? y : 0;
    if (owner) gstore(yv ? pout + yr * W : scratch, yv ? vo : vo_lane, res);
    if constexpr (EPI == EPI_STEP) {
      if (owner) gstore(yv ? puo + yr * ws_uo : scratch, yv ? (want_u ? vo : vo_lane) : vo_lane, u);
    }
    if constexpr (ODD_Y) {
      // D of the (pre-skip) result: 2x2 block = rows y-1, y x columns c, c+1
      const float pn = lane_next(xn_prev), cn = lane_next(xn);
      const float d = 0.25f * xn_prev + 0.25f * pn + 0.25f * xn + 0.25f * cn;
      if (owner_xd) gstore(yv ? pxd + (yr >> 1) * ws_xd : scratch, yv ? (want_xd ? vo_half : vo_lane) : vo_lane, d);
    }
    xn_prev = xn;
  };

  // ts = r0 - 3 is odd (r0 even): body A handles even y, body B odd y.  The trip count is
  // padded to even; the extra row only writes to the scratch line.
  const int ts = r0 - 3;
  const int te = ts + ((r1 + 3 - ts + 1) & ~1);
  RowLoads A, B;
  issue(ts, A);
  issue(ts + 1, B);
  const bool lockstep = a.wpb > 1;
  for (int t = ts; t < te; t += 2) {
    consume(t, A, std::false_type{});
    issue(t + 2, A);
    consume(t + 1, B, std::true_type{});
    issue(t + 3, B);
    if (lockstep) __builtin_amdgcn_s_barrier();
  }
}

// ---------------------------------------------------------------------------
// Row-wave variant (W <= 64 V, W % V == 0): one wave = one (b, channel) plane, one
// segment of SSEG output rows and ALL W columns; lane l holds columns V l .. V l + V-1.
// Same 4-stage register pipeline as graph_op_kernel, but no halo columns: every row
// operand is one coalesced V*256-byte wave-load (global_load_dwordx4 for V = 4) and
// horizontal neighbours are in-lane except a lane's first / last column (one DPP
// shift per row array and direction).  Image-edge columns apply the operators'
// boundary rules explicitly (replicate for S, zero outside for S^T / C^T C).
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) float* lds_f32_t;
template <int V> struct VecT;
template <> struct VecT<1> { typedef float type; };
template <> struct VecT<2> { typedef float __attribute__((ext_vector_type(2))) type; };
template <> struct VecT<4> { typedef float __attribute__((ext_vector_type(4))) type; };

template <int N>
__device__ __forceinline__ void vload(float (&d)[N], const float* row_base, uint32_t off_bytes) {
  typedef typename VecT<N>::type T;
  const T t = *reinterpret_cast<const T*>(reinterpret_cast<const char*>(row_base) + off_bytes);
  if constexpr (N == 1) {
    d[0] = t;
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) d[j] = t[j];
  }
}
template <int N>
__device__ __forceinline__ void vstore(float* row_base, uint32_t off_bytes, const float (&v)[N]) {
  typedef typename VecT<N>::type T;
  T t;
  if constexpr (N == 1) {
    t = v[0];
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) t[j] = v[j];
  }
  *reinterpret_cast<T*>(reinterpret_cast<char*>(row_base) + off_bytes) = t;
}

// Buffer-resource row access for the row kernels: a wave-uniform resource per operand plane
// (base + byte size in SGPRs) and one 32-bit VGPR offset per access, instead of 64-bit VGPR
// row pointers.  Reads past num_records return 0 and writes there are dropped by the
// hardware range check, so absent operands use num_records = 0 and rows / lanes that must
// not be written get an offset past the end (GRR_OOB).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t GRR_OOB = 0x80000000u;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, p ? (int)bytes : 0, 0x00020000);
}
template <int N, int AUX = 0>   // AUX: cache-policy bits (2 = nt)
__device__ __forceinline__ void bload(float (&d)[N], rsrc_t r, uint32_t off) {
  if constexpr (N == 1) {
    d[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX));
  } else {
    typedef typename VecT<N>::type T;
    T t;
    if constexpr (N == 2) t = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX));
    else t = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
#pragma unroll
    for (int j = 0; j < N; ++j) d[j] = t[j];
  }
}
template <int N, int AUX = 0>
__device__ __forceinline__ void bstore(rsrc_t r, uint32_t off, const float (&v)[N]) {
  if constexpr (N == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[0]), r, off, 0, AUX);
  } else {
    typedef typename VecT<N>::type T;
    T t;
#pragma unroll
    for (int j = 0; j < N; ++j) t[j] = v[j];
    if constexpr (N == 2) {
      typedef uint32_t U2 __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(U2, t), r, off, 0, AUX);
    } else {
      typedef uint32_t U4 __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U4, t), r, off, 0, AUX);
    }
  }
}

template <int V>
struct RowLoadsV {
  float x[V];          // x row t
  float wl[4][V];      // GLR edge weights, row t-2
  float wg[4][V];      // GTV pair (2) or raw (4) weights, row t-2
  float wup[V];        // prox: w_up at row t-1
  float eb[V], eu[V], ey[V];
  float th[(V + 1) / 2];   // half-resolution operand at row (t-3)/2
};

// No minimum waves per SIMD asked of the row kernel: without its weight registers the LDS-ring
// step kernel needs 178 VGPRs (2 waves/SIMD); forcing 3 (168 VGPRs) spilled 10-12 VGPRs of store
// addresses into the row loop and measured 2.37 -> 2.81 ms per launch.
template <bool GLR, int GTV, int EPI, int V>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1)))
void graph_row_kernel(OpArgs a) {
  constexpr int NH = (V + 1) / 2;    // half-resolution values per lane
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // LW: the step kernel's edge-weight rows (4 GLR + 2 GTV pair rows per image row) reach the
  // block through an LDS ring filled by one extra producer wave with LDS-DMA, four rows
  // ahead; the channel waves read them with ds_read_b128 and hold no weight registers
  // The half-level operator (system_half, V = 2, W = 128) uses the same ring: there one
  // 1 KiB DMA (lanes 0-31 row t-2, lanes 32-63 row t-1) moves a weight plane's row pair.
  constexpr bool LW = GLR && GTV == GTV_PAIR && ((EPI == EPI_STEP && V == 4) || (EPI == EPI_HALF && V == 2));
  constexpr int LW_ROWS = 6;                     // weight rows per image row
  // ring of 3 row pairs; a plane's rows sit 256 floats apart: V = 4 slot [pair][parity][plane][256],
  // V = 2 slot [pair][plane][parity][128]
  constexpr int LW_PAIR = V == 4 ? 2 * LW_ROWS * 256 : LW_ROWS * 256;   // floats per pair
  constexpr int LW_PAR = V == 4 ? LW_ROWS * 256 : 128;                   // parity offset
  constexpr int LW_NDMA = V == 4 ? 2 * LW_ROWS : LW_ROWS;                // DMAs per pair
  __shared__ __attribute__((aligned(16))) float wring[LW ? 3 * LW_PAIR : 4];
  const bool producer = LW && wave == a.wpb;
  // a block = wpb channel waves of one (b, graph, segment): they walk the rows in lockstep
  // (one barrier per two rows), so the graph's edge-weight rows are fetched from HBM once
  // and served to the other channel waves by L1/L2 (the grid divides exactly: no wave
  // leaves early, every wave reaches every barrier)
  uint32_t unit = xcd_remap(blockIdx.x, a.nblk) * a.wpb + (producer ? 0 : wave);
  const int F = a.F;
  const int f = unit % F; unit /= F;
  const int seg = unit % a.nsegs; unit /= a.nsegs;
  const int strip = unit % a.nstrips; unit /= a.nstrips;
  const int g = unit % a.G;
  const int b = unit / a.G;
  const int H = a.H, W = a.W, C = a.G * F, ch = g * F + f;
  const int hh = H / 2, hw = W / 2;
  const int64_t HW = (int64_t)H * W;
  // Wide rows (W > 64 V): strips of output columns [xs, xe); a strip's wave covers 64 V columns
  // from x0 = xs - 4 (4 halo columns each side, whole lanes; strip 0 starts at the image edge).
  // Lanes past the right halo or the image read nothing (out-of-range offsets read 0).
  const int xs = strip * a.sw, xe = min(xs + a.sw, W);
  const int x0 = strip > 0 ? xs - 4 : 0;
  const int c0 = x0 + V * lane;                  // first column of this lane
  const bool lane_on = c0 >= xs && c0 < xe;      // W % V == 0: a lane is all-in or all-out
  const bool lane_ld = c0 < min(xe + 4, W);      // lanes with columns this strip reads
  const int cl0 = lane_ld ? c0 : W - V;          // clamped column for the weight-row DMAs
  const int r0 = seg * a.sseg, r1 = min(r0 + a.sseg, H);
  const uint32_t vo = lane_ld ? (uint32_t)c0 * 4u : GRR_OOB;
  // half-resolution column(s) of this lane: V=4 -> 2l, 2l+1; V=2 -> l; V=1 -> l/2
  const uint32_t vo_half = lane_ld ? (uint32_t)(c0 >> 1) * 4u : GRR_OOB;
  const bool owner_xd = lane_on && (V > 1 || ((c0 & 1) == 0 && c0 + 1 < W));

  const int64_t plane = ((int64_t)b * C + ch) * HW;
  const int64_t hplane = ((int64_t)b * C + ch) * (int64_t)hh * hw;
  const bool has_half = EPI != EPI_HALF && a.t_half != nullptr;
  const bool use_beta = EPI == EPI_STEP && a.beta != nullptr && a.u_prev != nullptr;
  const bool need_y = (EPI == EPI_RHS) || (EPI == EPI_STEP && a.skip != nullptr);
  const bool want_u = EPI == EPI_STEP && a.u_out != nullptr;
  const bool want_xd = a.xd_out != nullptr;
  const int np = GTV == GTV_PROX ? 4 : 2;
  const int64_t rplane = ((int64_t)b * F + f) * HW;   // plane of a graph-replicated operand
  const int64_t PB = HW * 4, HPB = (int64_t)hh * hw * 4;   // plane bytes (launch_op: < 2^31 / 4)
  const float* pwl = GLR ? a.wL + (int64_t)(b * a.G + g) * 4 * HW : nullptr;
  const float* pwg = GTV ? a.wG + (int64_t)(b * a.G + g) * np * HW : nullptr;
  const rsrc_t rx = make_rsrc(a.x + (a.x_rep ? rplane : plane), PB);
  const rsrc_t rwl = make_rsrc(pwl, 4 * PB), rwg = make_rsrc(pwg, np * PB);
  const rsrc_t rb = make_rsrc(EPI == EPI_STEP ? a.b + plane : nullptr, PB);
  const rsrc_t ru = make_rsrc(use_beta ? a.u_prev + plane : nullptr, PB);
  const rsrc_t ry = make_rsrc(need_y ? a.y + (a.y_rep ? rplane : plane) : nullptr, PB);
  const rsrc_t rth = make_rsrc(has_half ? a.t_half + hplane : nullptr, HPB);
  const rsrc_t rout = make_rsrc(a.out + plane, PB);
  const rsrc_t ruo = make_rsrc(want_u ? a.u_out + plane : nullptr, PB);
  const rsrc_t rxd = make_rsrc(want_xd ? a.xd_out + hplane : nullptr, HPB);
  const uint32_t RB = (uint32_t)W * 4u, HRB = (uint32_t)hw * 4u;   // row bytes

  float sc_l = 1.f, sc_g = 1.f, sc_h = 1.f, gam = 0.f, alpha = 0.f, beta = 0.f, sk0 = 0.f, sk1 = 1.f;
  if (a.log_l) sc_l = a.lin_l ? a.log_l[g] : expf(a.log_l[g]);
  if (a.log_g) sc_g = expf(a.log_g[g]);
  if (a.log_half) sc_h = expf(a.log_half[g]);
  if constexpr (GTV == GTV_PROX) gam = expf(a.log_gamma[g]);
  if constexpr (EPI == EPI_STEP) {
    alpha = a.alpha[g];
    if (use_beta) beta = a.beta[g];
    if (a.skip) { sk0 = a.skip[0]; sk1 = a.skip[1]; }
  }
  const bool use_skip = EPI == EPI_STEP && a.skip != nullptr;
  Taps tL{}, tG{};
  if constexpr (GLR) tL = make_taps(a.sL, ch);
  if constexpr (GTV != GTV_NONE) tG = make_taps(a.sG, ch);

  auto issue = [&](int t, RowLoadsV<V>& S) {
    bload(S.x, rx, vo + clampi(t, 0, H - 1) * RB);
    const uint32_t rw = clampi(t - 2, 0, H - 1) * RB;
    if constexpr (GLR && !LW) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bload(S.wl[e], rwl, vo + e * (uint32_t)PB + rw);
    }
    if constexpr (GTV == GTV_PAIR && !LW) {
      bload(S.wg[0], rwg, vo + rw);
      bload(S.wg[1], rwg, vo + (uint32_t)PB + rw);
    }
    if constexpr (GTV == GTV_PROX) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bload(S.wg[e], rwg, vo + e * (uint32_t)PB + rw);
      bload(S.wup, rwg, vo + clampi(t - 1, 0, H - 1) * RB);
    }
    const int re = clampi(t - 3, 0, H - 1);
    if constexpr (EPI == EPI_STEP) {
      bload(S.eb, rb, vo + re * RB);
      bload(S.eu, ru, vo + re * RB);
    }
    if constexpr (EPI != EPI_HALF) {
      bload(S.ey, ry, vo + re * RB);
      bload(S.th, rth, vo_half + (re >> 1) * HRB);
    }
  };

  // pipeline registers, [V] per row (rows relative to the current iteration t)
  float X0[V] = {}, X1[V] = {}, X2[V] = {}, X3[V] = {};
  float SL0[V] = {}, SL1[V] = {}, SL2[V] = {};
  float SG0[V] = {}, SG1[V] = {}, SG2[V] = {};
  float L0[V] = {}, L1[V] = {}, L2[V] = {};
  float O0[V] = {}, O1[V] = {}, O2[V] = {};
  float cv_prev[V] = {}, wdn_prev[V] = {}, xn_prev[V] = {};

  auto consume = [&](int t, const RowLoadsV<V>& S, const float* lwrow, auto odd_tag) {
    constexpr bool ODD_Y = decltype(odd_tag)::value;
    // edge weights of row t-2: registers, or (LW) this lane's 4 columns of the LDS ring slot
    float WL[4][V], WG[2][V];
    if constexpr (LW) {
      typedef typename VecT<V>::type T;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const T q = *reinterpret_cast<const T*>(lwrow + e * 256);
#pragma unroll
        for (int j = 0; j < V; ++j) WL[e][j] = q[j];
      }
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const T q = *reinterpret_cast<const T*>(lwrow + (4 + e) * 256);
#pragma unroll
        for (int j = 0; j < V; ++j) WG[e][j] = q[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) {
#pragma unroll
        for (int e = 0; e < 4; ++e) WL[e][j] = S.wl[e][j];
        WG[0][j] = S.wg[0][j]; WG[1][j] = S.wg[1][j];
      }
    }
#pragma unroll
    for (int j = 0; j < V; ++j) { X0[j] = X1[j]; X1[j] = X2[j]; X2[j] = X3[j]; X3[j] = S.x[j]; }
    // ---- stage 2: s at row t-1 (rows replicate-clamped by the loads, columns here)
    {
      const float xp = lane_prev(X2[V - 1]), xq = lane_next(X2[0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int col = c0 + j;
        const float xl = col > 0 ? (j > 0 ? X2[j - 1] : xp) : X2[j];
        const float xr = col < W - 1 ? (j < V - 1 ? X2[j + 1] : xq) : X2[j];
        if constexpr (GLR) {
          float sv = tL.u * X1[j];
          sv += tL.l * xl; sv += tL.c * X2[j]; sv += tL.r * xr; sv += tL.d * X3[j];
          SL0[j] = SL1[j]; SL1[j] = SL2[j]; SL2[j] = sv;
        }
        if constexpr (GTV != GTV_NONE) {
          float sv = tG.u * X1[j];
          sv += tG.l * xl; sv += tG.c * X2[j]; sv += tG.r * xr; sv += tG.d * X3[j];
          SG0[j] = SG1[j]; SG1[j] = SG2[j]; SG2[j] = sv;
        }
      }
    }
    // ---- stage 3: l and o at row r = t-2 (zero outside the image)
    {
      const int r = t - 2;
      const bool rin = r >= 0 && r < H;
      if constexpr (GLR) {
        const float pv = lane_prev(SL1[V - 1]), nx = lane_next(SL1[0]);
        float l[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const int col = c0 + j;
          const float up = r > 0 ? SL0[j] : SL1[j];
          const float dn = r < H - 1 ? SL2[j] : SL1[j];
          const float lf = col > 0 ? (j > 0 ? SL1[j - 1] : pv) : SL1[j];
          const float rt = col < W - 1 ? (j < V - 1 ? SL1[j + 1] : nx) : SL1[j];
          const float wx = ((WL[0][j] * up + WL[1][j] * lf) + WL[2][j] * rt) + WL[3][j] * dn;
          l[j] = (rin && col < W) ? SL1[j] - wx : 0.f;
        }
#pragma unroll
        for (int j = 0; j < V; ++j) { L0[j] = L1[j]; L1[j] = L2[j]; L2[j] = l[j]; }
      }
      if constexpr (GTV == GTV_PAIR) {
        const float sp = lane_prev(SG1[V - 1]), sn = lane_next(SG1[0]);
        const float wp = lane_prev(WG[0][V - 1]);
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const int col = c0 + j;
          const float sv = SG1[j];
          const float snx = j < V - 1 ? SG1[j + 1] : sn;     // x c_h = 0 at the last column
          const float spv = j > 0 ? SG1[j - 1] : sp;
          const float chl = col > 0 ? (j > 0 ? WG[0][j - 1] : wp) : 0.f;
          const float cvu = r > 0 ? cv_prev[j] : 0.f;
          const float ov = WG[0][j] * (sv - snx) + chl * (sv - spv) + WG[1][j] * (sv - SG2[j]) +
                           cvu * (sv - SG0[j]);
          o[j] = (rin && col < W) ? ov : 0.f;
        }
#pragma unroll
        for (int j = 0; j < V; ++j) { cv_prev[j] = WG[1][j]; O0[j] = O1[j]; O1[j] = O2[j]; O2[j] = o[j]; }
      }
      if constexpr (GTV == GTV_PROX) {
        const float sp = lane_prev(SG1[V - 1]), sn = lane_next(SG1[0]);
        const float w1n = lane_next(S.wg[1][0]), w2p = lane_prev(S.wg[2][V - 1]);
        float o[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const int col = c0 + j;
          const float sv = SG1[j];
          const float su = r > 0 ? SG0[j] : sv, sd = r < H - 1 ? SG2[j] : sv;
          const float spv = j > 0 ? SG1[j - 1] : sp, snx = j < V - 1 ? SG1[j + 1] : sn;
          const float sl = col > 0 ? spv : sv, sr = col < W - 1 ? snx : sv;
          const float w0 = S.wg[0][j], w1 = S.wg[1][j], w2 = S.wg[2][j], w3 = S.wg[3][j];
          const float z0 = prox_phi(w0 * sv - w0 * su, gam) * w0;
          const float z1 = prox_phi(w1 * sv - w1 * sl, gam) * w1;
          const float z2 = prox_phi(w2 * sv - w2 * sr, gam) * w2;
          const float z3 = prox_phi(w3 * sv - w3 * sd, gam) * w3;
          float ov = ((z0 + z1) + z2) + z3;
          const float wupb = S.wup[j];                                 // w_up(q + down)
          const float wlfr = j < V - 1 ? S.wg[1][j + 1] : w1n;         // w_left(q + right)
          const float wrtl = j > 0 ? S.wg[2][j - 1] : w2p;             // w_right(q - right)
          const float wdna = wdn_prev[j];                              // w_down(q - down)
          const float o1 = ov - prox_phi(wupb * SG2[j] - wupb * sv, gam) * wupb;
          ov = r < H - 1 ? o1 : ov;
          const float o2 = ov - prox_phi(wlfr * snx - wlfr * sv, gam) * wlfr;
          ov = col < W - 1 ? o2 : ov;
          const float o3 = ov - prox_phi(wrtl * spv - wrtl * sv, gam) * wrtl;
          ov = col > 0 ? o3 : ov;
          const float o4 = ov - prox_phi(wdna * SG0[j] - wdna * sv, gam) * wdna;
          ov = r > 0 ? o4 : ov;
          o[j] = (rin && col < W) ? ov : 0.f;
        }
#pragma unroll
        for (int j = 0; j < V; ++j) { wdn_prev[j] = S.wg[3][j]; O0[j] = O1[j]; O1[j] = O2[j]; O2[j] = o[j]; }
      }
    }
    // ---- stage 4: S^T and the epilogue at row y = t-3 (neighbours outside are 0)
    const int y = t - 3;
    float tl[V] = {}, tg[V] = {};
    if constexpr (GLR) {
      const float lp = lane_prev(L1[V - 1]), ln = lane_next(L1[0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float nx = j < V - 1 ? L1[j + 1] : ln, pv = j > 0 ? L1[j - 1] : lp;
        float v = tL.u * L2[j];
        v += tL.l * nx; v += tL.c * L1[j]; v += tL.r * pv; v += tL.d * L0[j];
        tl[j] = v;
      }
    }
    if constexpr (GTV != GTV_NONE) {
      const float op = lane_prev(O1[V - 1]), on = lane_next(O1[0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float nx = j < V - 1 ? O1[j + 1] : on, pv = j > 0 ? O1[j - 1] : op;
        float v = tG.u * O2[j];
        v += tG.l * nx; v += tG.c * O1[j]; v += tG.r * pv; v += tG.d * O0[j];
        tg[j] = v;
      }
    }
    float res[V], xn[V], u[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float th = 0.25f * S.th[V == 4 ? (j >> 1) : 0];
      xn[j] = 0.f; u[j] = 0.f;
      if constexpr (EPI == EPI_HALF) {
        float rv = 0.f;                                   // mu * S_L^T l + ro * S_G^T o (REF:666-675)
        if constexpr (GLR) rv = tl[j] * sc_l;
        if constexpr (GTV != GTV_NONE) rv = GLR ? rv + tg[j] * sc_g : tg[j] * sc_g;
        res[j] = rv; xn[j] = rv;
      } else if constexpr (EPI == EPI_RHS) {
        float rv = S.ey[j] + tg[j] * sc_g;                // (y + ro0 C^T phi(C x)) + ro1 U(t)
        if (has_half) rv = rv + th * sc_h;
        res[j] = rv; xn[j] = rv;
      } else {
        float ax = X0[j];                                 // A x = ((x + mu0 L x) + ro0 G x) + U(t)
        if constexpr (GLR) ax = ax + tl[j] * sc_l;
        if constexpr (GTV != GTV_NONE) ax = ax + tg[j] * sc_g;
        if (has_half) ax = ax + th;
        float uv = S.eb[j] - ax;                          // residual
        if (use_beta) uv = uv + beta * S.eu[j];           // heavy-ball direction (REF:789)
        u[j] = uv;
        xn[j] = X0[j] + alpha * uv;                       // x_{k+1}
        res[j] = use_skip ? sk0 * S.ey[j] + sk1 * xn[j] : xn[j];   // block skip (REF:987)
      }
    }
    const bool yv = y >= r0 && y < r1;
    const int yr = yv ? y : 0;
    const uint32_t so = (yv && lane_on) ? vo + yr * RB : GRR_OOB;
    bstore(rout, so, res);
    if constexpr (EPI == EPI_STEP) bstore(ruo, so, u);
    if constexpr (ODD_Y) {
      // D of the (pre-skip) result: 2x2 blocks of rows y-1, y
      float d[NH];
      if constexpr (V == 1) {
        const float pn = lane_next(xn_prev[0]), cn = lane_next(xn[0]);
        d[0] = 0.25f * xn_prev[0] + 0.25f * pn + 0.25f * xn[0] + 0.25f * cn;
      } else {
#pragma unroll
        for (int k = 0; k < NH; ++k)
          d[k] = 0.25f * xn_prev[2 * k] + 0.25f * xn_prev[2 * k + 1] + 0.25f * xn[2 * k] + 0.25f * xn[2 * k + 1];
      }
      bstore(rxd, (yv && owner_xd) ? vo_half + (yr >> 1) * HRB : GRR_OOB, d);
    }
#pragma unroll
    for (int j = 0; j < V; ++j) xn_prev[j] = xn[j];
  };

  const int ts = r0 - 3;
  const int te = ts + ((r1 + 3 - ts + 1) & ~1);
  if constexpr (LW) {
    // ring slot (pair q, parity) holds the weight rows of step t = ts + 2 q' + parity, q = q' mod 3
    if (producer) {
      auto dma = [&](const float* src, float* dst) {
        const uint32_t m0v = (uint32_t)(uintptr_t)(lds_f32_t)dst;
        asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(__builtin_amdgcn_readfirstlane(m0v))
                     : "memory");
      };
      auto dma_pair = [&](int t, int q) {
        if constexpr (V == 4) {
#pragma unroll
          for (int par = 0; par < 2; ++par) {
            const int rw = clampi(t + par - 2, 0, H - 1) * W + cl0;
            float* slot = wring + q * LW_PAIR + par * LW_PAR;
#pragma unroll
            for (int e = 0; e < LW_ROWS; ++e)
              dma(e < 4 ? pwl + e * HW + rw : pwg + (e - 4) * HW + rw, slot + e * 256);
          }
        } else {   // W == 128: lanes 0-31 row t-2, lanes 32-63 row t-1, 4 columns each
          const int rw = clampi(t + (lane >> 5) - 2, 0, H - 1) * W + (lane & 31) * 4;
          float* slot = wring + q * LW_PAIR;
#pragma unroll
          for (int e = 0; e < LW_ROWS; ++e)
            dma(e < 4 ? pwl + e * HW + rw : pwg + (e - 4) * HW + rw, slot + e * 256);
        }
      };
      dma_pair(ts, 0);
      dma_pair(ts + 2, 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(LW_NDMA) : "memory");   // pair 0 landed
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      int q = 0;
      for (int t = ts; t < te; t += 2) {
        dma_pair(t + 4, q == 0 ? 2 : q - 1);       // the slot the channel waves read last iteration
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(LW_NDMA) : "memory");  // pair of t + 2 landed
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        q = q == 2 ? 0 : q + 1;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
  }
  RowLoadsV<V> A, B;
  issue(ts, A);
  issue(ts + 1, B);
  if constexpr (LW) {
    __builtin_amdgcn_s_barrier();                  // the producer's first ring pair has landed
    asm volatile("" ::: "memory");
  }
  const bool lockstep = LW || a.wpb > 1;
  const float* lwl = wring + lane * V;
  int q = 0;
  for (int t = ts; t < te; t += 2) {
    consume(t, A, lwl + q * LW_PAIR, std::false_type{});
    issue(t + 2, A);
    consume(t + 1, B, lwl + q * LW_PAIR + LW_PAR, std::true_type{});
    issue(t + 3, B);
    if (lockstep) {
      if constexpr (LW) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // ring reads done
      __builtin_amdgcn_s_barrier();
      if constexpr (LW) asm volatile("" ::: "memory");
    }
    q = q == 2 ? 0 : q + 1;
  }
}

// W <= 64 V with W % V == 0 -> row kernel with V columns per lane; otherwise 0 (strips)
static int row_vec(int W) {
  if (W <= 64) return 1;
  if (W <= 128 && W % 2 == 0) return 2;
  if (W <= 256 && W % 4 == 0) return 4;
  return 0;
}

template <bool GLR, int GTV, int EPI, int V>
static void launch_row(OpArgs a, int B, hipStream_t s) {
  // wide images: strips of at most 64 V - 8 output columns (a multiple of V), 4 halo columns each side
  a.nstrips = 1;
  a.sw = a.W;
  if (a.W > 64 * V) {
    a.nstrips = (a.W + 64 * V - 9) / (64 * V - 8);
    a.sw = ((a.W + a.nstrips - 1) / a.nstrips + V - 1) / V * V;
  }
  a.sseg = seg_rows(a.H, (uint64_t)B * a.G * a.F * a.nstrips);
  a.nsegs = (a.H + a.sseg - 1) / a.sseg;
  const uint64_t units = (uint64_t)B * a.G * a.F * a.nsegs * a.nstrips;
  a.nunits = (uint32_t)units;
  // channels of a graph per block: the largest divisor of F that fits NT threads.  Only for
  // V = 4 (W > 128): on 128-wide half-resolution planes the unsynchronised waves measured 4 %
  // faster (0.408 vs 0.426 ms, scripts/micro.py --kernel half), the weight rows being short
  // The LDS-ring kernels (LW: the step kernel and the 128-wide half-level operator) add one
  // producer wave per block that streams the edge-weight rows into an LDS ring, so at most
  // NT / 64 - 1 channel waves
  constexpr bool LW = GLR && GTV == GTV_PAIR && ((EPI == EPI_STEP && V == 4) || (EPI == EPI_HALF && V == 2));
  int wpb = (g_kernel_variant == 2 || (V < 4 && !LW)) ? 1 : NT / 64 - (LW ? 1 : 0);
  while (a.F % wpb) --wpb;
  a.wpb = wpb;
  a.nblk = (uint32_t)(units / wpb);
  hipLaunchKernelGGL((graph_row_kernel<GLR, GTV, EPI, V>), dim3(a.nblk), dim3(64 * (wpb + (LW ? 1 : 0))), 0, s, a);
}

template <bool GLR, int GTV, int EPI>
static grr_status launch_op(const OpArgs& a0, int B, hipStream_t s, const char* name) {
  GRR_REQUIRE((int64_t)a0.H * a0.W * 4 < (1ll << 31), GRR_ERR_UNSUPPORTED, "%s: plane too large", name);
  GRR_REQUIRE((uint64_t)B * a0.G * a0.F * ((a0.H + SSEG - 1) / SSEG) * ((a0.W + SVALID - 1) / SVALID) <
                  (1ull << 32) - 4,
              GRR_ERR_UNSUPPORTED, "%s: grid too large", name);
  int vec = g_kernel_variant == 1 ? 0 : row_vec(a0.W);
  // wider rows: the V = 4 row kernel in column strips (4 halo columns per side)
  if (vec == 0 && g_kernel_variant != 1 && a0.W > 256 && a0.W % 4 == 0) vec = 4;
  // row kernels address a graph's 4 weight planes through one buffer resource (int range)
  if ((int64_t)a0.H * a0.W * 16 >= (1ll << 31)) vec = 0;
  if (vec > 1) {   // vector row loads need every operand base aligned to 4V bytes
    const void* ptrs[] = {a0.x, a0.wL, a0.wG, a0.y, a0.b, a0.u_prev, a0.t_half, a0.out, a0.u_out, a0.xd_out};
    for (const void* q : ptrs)
      if ((uintptr_t)q % (4u * vec) != 0) vec = 0;
    // half-resolution rows are read / written as V/2-float vectors
    if (vec == 4 && (a0.t_half || a0.xd_out) && (((int64_t)(a0.H / 2) * (a0.W / 2)) % 2 != 0)) vec = 0;
    // the LDS-ring half-level operator moves whole 128-float weight row pairs with 16-byte DMAs
    if (vec == 2 && GLR && GTV == GTV_PAIR && EPI == EPI_HALF &&
        (a0.W != 128 || (uintptr_t)a0.wL % 16 != 0 || (uintptr_t)a0.wG % 16 != 0))
      vec = 0;
  }
  switch (vec) {
    case 1: launch_row<GLR, GTV, EPI, 1>(a0, B, s); return launch_status(name);
    case 2: launch_row<GLR, GTV, EPI, 2>(a0, B, s); return launch_status(name);
    case 4: launch_row<GLR, GTV, EPI, 4>(a0, B, s); return launch_status(name);
    default: break;
  }
  OpArgs a = a0;
  a.nstrips = (a.W + SVALID - 1) / SVALID;
  a.sseg = seg_rows(a.H, (uint64_t)B * a.G * a.F * a.nstrips);
  a.nsegs = (a.H + a.sseg - 1) / a.sseg;
  const uint64_t units = (uint64_t)B * a.G * a.F * a.nsegs * a.nstrips;
  GRR_REQUIRE(units < (1ull << 32) - 4, GRR_ERR_UNSUPPORTED, "%s: grid too large", name);
  GRR_REQUIRE((int64_t)a.H * a.W * 4 < (1ll << 31), GRR_ERR_UNSUPPORTED, "%s: plane too large", name);
  a.nunits = (uint32_t)units;
  // lockstep channel waves measured neutral for the 58-column strips (W = 512: 3.27 vs 3.19 ms;
  // the strip halo re-reads dominate), so strips run one wave per channel, 4 waves per block
  a.wpb = 1;
  a.nblk = (uint32_t)((units + 3) / 4);
  hipLaunchKernelGGL((graph_op_kernel<GLR, GTV, EPI>), dim3(a.nblk), dim3(NT), 0, s, a);
  return launch_status(name);
}


// ---------------------------------------------------------------------------
// a3+a4 as a row-wave stream (W <= 256): the GTV slab (raw weights + pair weights) and
// the GLR slab (raw weights) of one feature tensor in ONE launch.  One wave = one
// (b, slab, graph) plane set; lane = V adjacent columns (dwordx4 loads for V = 4); the
// normalised features of rows r-1, r, r+1 stay in registers (vertical neighbours),
// horizontal neighbours come from DPP wave shifts.  Row r's pair weight c_v needs
// w_up of row r+1, so it is written one row late.  Same arithmetic order as
// edge_weights_kernel (REF:146-175).
// ---------------------------------------------------------------------------
#ifndef GRR_EDGE_MIN_WAVES
#define GRR_EDGE_MIN_WAVES 8192
#endif
constexpr uint64_t EDGE_MIN_WAVES = GRR_EDGE_MIN_WAVES;
struct EdgeArgs {
  const float* feat;
  int64_t bstride;
  int slab_off[2];          // first channel of each slab in feat
  const float* multiM[2];   // [G,F] per slab
  float* w[2];              // raw weights [B,G,4,H,W] per slab
  float* c[2];              // pair weights [B,G,2,H,W] per slab, or NULL
  int nslab, G, H, W;
  int sseg, nsegs;          // rows per wave segment, segments per plane
  uint32_t nunits, nblk;
};

template <int F, int V>
__global__ __launch_bounds__(NT) void edge_row_kernel(EdgeArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t unit = xcd_remap(blockIdx.x, a.nblk) * 4 + wave;
  if (unit >= a.nunits) return;   // whole wave (uniform)
  const int seg = unit % a.nsegs; unit /= a.nsegs;
  const int g = unit % a.G; unit /= a.G;
  const int slab = unit % a.nslab;
  const int b = unit / a.nslab;
  const int H = a.H, W = a.W;
  // rows [r0, r1) of the plane; a segment that ends inside the image runs one extra row
  // (weights not stored) for the w_up its last row's pair weight c_v needs
  const int r0 = seg * a.sseg, r1 = min(r0 + a.sseg, H);
  const int rend = r1 < H ? r1 + 1 : H;
  const int64_t HW = (int64_t)H * W;
  const float* fb = a.feat + (int64_t)b * a.bstride + (int64_t)(a.slab_off[slab] + g * F) * HW;
  const float* Mp = a.multiM[slab] + g * F;
  float M[F];
#pragma unroll
  for (int f = 0; f < F; ++f) M[f] = Mp[f];
  const int c0 = V * lane;
  const bool lane_on = c0 < W;
  const int cl0 = lane_on ? c0 : W - V;
  const uint32_t vo = (uint32_t)cl0 * 4u;
  float* wb = a.w[slab] + (int64_t)(b * a.G + g) * 4 * HW;
  float* cb = a.c[slab] ? a.c[slab] + (int64_t)(b * a.G + g) * 2 * HW : nullptr;

  float fP[F][V], fC[F][V], fN[F][V], raw[F][V];
  auto load_raw = [&](int row) {
    const int rr = clampi(row, 0, H - 1);
#pragma unroll
    for (int f = 0; f < F; ++f) vload(raw[f], fb + f * HW + (int64_t)rr * W, vo);
  };
  auto normalise = [&](float (&dst)[F][V]) {   // F.normalize(dim=F, eps 1e-12) * multiM (REF:146-157)
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float ss = 0.f;
#pragma unroll
      // explicit fma: the prologue's and the row loop's copies of this code must round alike
      // (a segment's first rows are normalised by the prologue, elsewhere by the loop)
      for (int f = 0; f < F; ++f) ss = __builtin_fmaf(raw[f][j], raw[f][j], ss);
      const float den = fmaxf(sqrtf(ss), 1e-12f);
#pragma unroll
      for (int f = 0; f < F; ++f) dst[f][j] = (raw[f][j] / den) * M[f];
    }
  };
  load_raw(r0 - 1);                                  // clamped: row 0 is its own up neighbour
  normalise(fP);
  load_raw(r0);
  normalise(fC);
  load_raw(r0 + 1);
  normalise(fN);
  float wdn_prev[V];
#pragma unroll
  for (int j = 0; j < V; ++j) wdn_prev[j] = 0.f;

  for (int r = r0; r < rend; ++r) {
    const bool own = r < r1;                           // wave-uniform: row r belongs to this segment
    load_raw(r + 2);                                   // consumed at the bottom of the iteration
    float fl[F], fr[F];                                // lane-edge neighbours (whole wave active)
#pragma unroll
    for (int f = 0; f < F; ++f) { fl[f] = lane_prev(fC[f][V - 1]); fr[f] = lane_next(fC[f][0]); }
    float w0[V], w1[V], w2[V], w3[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int col = c0 + j;
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const float v = fC[f][j];
        const float lv = col > 0 ? (j > 0 ? fC[f][j - 1] : fl[f]) : v;
        const float rv = col < W - 1 ? (j < V - 1 ? fC[f][j + 1] : fr[f]) : v;
        s0 += v * fP[f][j];
        s1 += v * lv;
        s2 += v * rv;
        s3 += v * fN[f][j];
      }
      const float m = fmaxf(fmaxf(s0, s1), fmaxf(s2, s3));
      const float e0 = expf(s0 - m), e1 = expf(s1 - m), e2 = expf(s2 - m), e3 = expf(s3 - m);
      const float sum = ((e0 + e1) + e2) + e3;
      w0[j] = e0 / sum; w1[j] = e1 / sum; w2[j] = e2 / sum; w3[j] = e3 / sum;
    }
    const int64_t ro = (int64_t)r * W;
    if (lane_on && own) {
      vstore(wb + ro, vo, w0);
      vstore(wb + HW + ro, vo, w1);
      vstore(wb + 2 * HW + ro, vo, w2);
      vstore(wb + 3 * HW + ro, vo, w3);
    }
    if (cb) {   // wave-uniform
      const float wl_next = lane_next(w1[0]);
      float ch[V], cv[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int col = c0 + j;
        const float wln = j < V - 1 ? w1[j + 1] : wl_next;     // w_left(p + right)
        ch[j] = col + 1 < W ? w2[j] * w2[j] + wln * wln : 0.f;
        cv[j] = wdn_prev[j] * wdn_prev[j] + w0[j] * w0[j];     // row r-1: w_down(p)^2 + w_up(p + down)^2
        wdn_prev[j] = w3[j];
      }
      if (lane_on) {
        if (own) vstore(cb + ro, vo, ch);
        if (r > r0) vstore(cb + HW + ro - W, vo, cv);
      }
    }
    // advance the row window (the down neighbour of the last row is itself: clamped load)
#pragma unroll
    for (int f = 0; f < F; ++f)
#pragma unroll
      for (int j = 0; j < V; ++j) { fP[f][j] = fC[f][j]; fC[f][j] = fN[f][j]; }
    normalise(fN);
  }
  if (cb && lane_on && r1 == H) {   // last row: no lower neighbour
    float z[V];
#pragma unroll
    for (int j = 0; j < V; ++j) z[j] = 0.f;
    vstore(cb + HW + (int64_t)(H - 1) * W, vo, z);
  }
}

template <int F>
static void launch_edge_row_f(const EdgeArgs& a, int V, hipStream_t s) {
  const dim3 grid(a.nblk), block(NT);
  if (V == 4) hipLaunchKernelGGL((edge_row_kernel<F, 4>), grid, block, 0, s, a);
  else if (V == 2) hipLaunchKernelGGL((edge_row_kernel<F, 2>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((edge_row_kernel<F, 1>), grid, block, 0, s, a);
}

// true when the row-wave kernel took the launch
static bool launch_edge_row(EdgeArgs a, int B, int F, hipStream_t s) {
  const int V = g_kernel_variant == 1 ? 0 : row_vec(a.W);
  if (V == 0) return false;
  if ((uintptr_t)a.feat % (4u * V) || (a.bstride * 4) % (4 * V) || ((int64_t)a.H * a.W) % V) return false;
  for (int k = 0; k < a.nslab; ++k)
    if ((uintptr_t)a.w[k] % (4u * V) || (a.c[k] && (uintptr_t)a.c[k] % (4u * V))) return false;
  // row segments: at least EDGE_MIN_WAVES waves (the row loop is latency-bound with one row
  // of prefetch), segments of >= 32 rows (each costs 2 extra normalised rows + 1 extra row)
  const uint64_t planes = (uint64_t)B * a.nslab * a.G;
  int nsegs = 1;
  while (planes * nsegs < EDGE_MIN_WAVES && a.H / (2 * nsegs) >= 32) nsegs *= 2;
  a.sseg = (a.H + nsegs - 1) / nsegs;
  a.nsegs = (a.H + a.sseg - 1) / a.sseg;
  const uint64_t units = planes * a.nsegs;
  if (units >= (1ull << 32) - 4) return false;
  a.nunits = (uint32_t)units;
  a.nblk = (uint32_t)((units + 3) / 4);
  switch (F) {
    case 1: launch_edge_row_f<1>(a, V, s); return true;
    case 2: launch_edge_row_f<2>(a, V, s); return true;
    case 3: launch_edge_row_f<3>(a, V, s); return true;
    case 4: launch_edge_row_f<4>(a, V, s); return true;
    case 6: launch_edge_row_f<6>(a, V, s); return true;
    case 8: launch_edge_row_f<8>(a, V, s); return true;
    case 12: launch_edge_row_f<12>(a, V, s); return true;
    case 16: launch_edge_row_f<16>(a, V, s); return true;
    default: return false;
  }
}

static bool stencil_ok(const grr_stencil& s) { return s.p01 && s.p02a && s.p02b && s.p03; }

// ---------------------------------------------------------------------------
// Two CG stages per pass: temporal blocking of grr_system_step (GLR + GTV pair, W = 256).
//
// Stage k+1 consumes stage k's rows a few rows behind inside the same workgroup, so
// x_{k+1} and u_{k+1} never reach HBM and the full-level edge weights are read once for
// both stages.  One workgroup = one (b, graph, row segment): per channel a stage-A and a
// stage-B wave, one producer wave and one half-level wave; one workgroup per CU (≈159 KiB of
// LDS), two waves per SIMD.  Per iteration (two image rows) the waves run register pipelines
// of the operator (OpPipe: x -> s = S x -> {l, o} -> S^T, the arithmetic of graph_row_kernel's
// consume):
//   half A    = the half-level operator (mu1 L1 + ro1 G1) of D x_k (the previous pass's pooled
//               output, from HBM), 128-wide rows, two half columns per lane, all channels in one
//               wave: t_k half rows into a 2-row LDS ring per channel, one iteration ahead (what
//               grr_system_half computed in a launch of its own before round 3);
//   stage A   = stage k at full resolution: x_k rows from HBM, t_k from the ring; writes x_{k+1}
//               and u_{k+1} rows into private LDS rings and D x_{k+1} half rows into a third ring;
//   half B    = the half-level operator of D x_{k+1}: t_{k+1}, kept in registers;
//   stage B   = stage k+1 at full resolution, 8 rows behind stage A: x_{k+1} / u_{k+1} from the
//               rings, t_{k+1} from registers; writes x_{k+2}, u_{k+2} and D x_{k+2} to HBM.
// Row timeline at step t (two steps per iteration): stage A loads x_k row t and emits row
// t-3; half B reads D x half row (t-4)/2 - 1 (one row late, so its replicate clamp at the
// top reads a row that exists) and emits half row (t-11)/2; stage B reads x_{k+1} row t-8 and
// emits row t-11.  The rings are read with the rows clamped to the image (the replicate
// boundary the HBM loads apply), and rows outside the image are never written into them.
// A segment's stage A starts 6 rows before its stage B needs exact rows (ts = r0 - 9).  The
// producer wave streams the full-level weight row pairs (7-pair ring: stage A uses pair i,
// stage B pair i-4, pairs i+1, i+2 in flight) and half B's weight rows (4-row ring) with
// LDS-DMA, two iterations ahead; half A loads its weight rows itself, four half rows earlier
// (the producer's later read of the same rows is an L2 hit).
// ---------------------------------------------------------------------------
struct Step2Args {
  const float* x;
  const float* b;
  const float* u_prev;
  const float* xd;       // D x_k (stage A's half level runs in the kernel)
  const float* wL0;
  const float* cG0;
  const float* wL1;
  const float* cG1;
  grr_stencil sL0, sG0, sL1, sG1;
  const float* log_mu0;
  const float* log_ro0;
  const float* log_mu1;
  const float* log_ro1;
  const float* alpha_a;
  const float* beta_a;
  const float* alpha_b;
  const float* beta_b;
  const float* skip;
  const float* y;
  float* out;
  float* u_out;
  float* xd_out;
  float* x_mid;          // training: x_{k+1} and u_{k+1} (the reverse sweep's saved iterates), or NULL
  float* u_mid;
  float* xd_mid;         // training: D x_{k+1} (the reverse sweep's half-level operand), or NULL
  // first pair (graph_step2_kernel<false, false, true>): stage 0, the prox right-hand side B, stage 1
  const float* wG0;      // raw GTV weights [B,G,4,H,W] / [B,G,4,h,w] of the prox terms
  const float* wG1;
  const float* log_gamma0;
  const float* log_gamma1;
  const float* yr;       // y of right-hand side B: [B,C,H,W], or the [B,F,H,W] image it replicates (yr_rep)
  int yr_rep;
  float* b_out;          // right-hand side B
  int G, F, H, nsegs, sseg;
  int W, nstrips;       // image width; column strips of S2_W lanes (1 at W = S2_W)
  int FG, ngrp;         // channel groups of <= S2_FMAX channels per (b, graph): FG channels each (the last may hold fewer)
  uint32_t nblk;
};

template <int V>
struct OpPipe {
  // Register slots of the row pipeline, 4-periodic: at phase P (step t with t = P mod 4 in
  // the caller's unrolled loop) input row t lands in X[(P+3)&3]; X[P&3] holds row t-3.
  // S (s = S x), L (l) and O (o) keep rows t-3..t-1 / t-4..t-2 in slots (P+1..P+3)&3.
  // Static slot indices: no register moves for the pipeline shifts.
  float X[4][V], SL[4][V], SG[4][V], L[4][V], O[4][V];
  float cv[2][V];   // pair weight c_v of the previous row (parity slots)

  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < V; ++j) X[k][j] = SL[k][j] = SG[k][j] = L[k][j] = O[k][j] = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) cv[0][j] = cv[1][j] = 0.f;
  }

  // x row t-3 (the epilogue's x at the output row)
  template <int P>
  __device__ __forceinline__ const float (&x_out() const)[V] { return X[P & 3]; }

  // push input row t (replicate-clamped by the caller) and the edge-weight row t-2 (4 GLR
  // planes, 2 pair planes); returns S_L^T (I - W) S_L x and S_G^T C^T C S_G x at row t-3
  // (before the mu / ro scales).  Lane = V adjacent columns starting at c0.  The arithmetic
  // of graph_row_kernel's consume (stages 2-4).
  // EDGE = false: the caller guarantees 1 <= t-2 <= H-2 (no row-boundary selects).  An
  // interior-block copy of the step2 loop measured no gain: the duplicated body raised the
  // register pressure into AGPR spills that cost what the selects did.
  // CE (column strips of a wider image): c0 is the image column, the image is Wr wide (columns
  // >= Wr are lanes past the right edge: their l / o are zeroed like rows outside the image)
  template <int P, int W, bool EDGE = true, bool CE = false>
  __device__ __forceinline__ void advance(const float (&xin)[V], const float (&WL)[4][V], const float (&WG)[2][V],
                                          int t, int H, int c0, const Taps& tL, const Taps& tG,
                                          float (&tl)[V], float (&tg)[V], int Wr = W) {
    constexpr int K0 = P & 3, K1 = (P + 1) & 3, K2 = (P + 2) & 3, K3 = (P + 3) & 3;
    const int WW = CE ? Wr : W;
#pragma unroll
    for (int j = 0; j < V; ++j) X[K3][j] = xin[j];
    const float (&X1)[V] = X[K1];
    const float (&X2)[V] = X[K2];
    const float (&X3)[V] = X[K3];
    {  // s at row t-1 -> slot K3 (rows t-3, t-2 in K1, K2)
      const float xp = lane_prev(X2[V - 1]), xq = lane_next(X2[0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int col = c0 + j;
        const float xl = col > 0 ? (j > 0 ? X2[j - 1] : xp) : X2[j];
        const float xr = col < WW - 1 ? (j < V - 1 ? X2[j + 1] : xq) : X2[j];
        float sv = tL.u * X1[j];
        sv += tL.l * xl; sv += tL.c * X2[j]; sv += tL.r * xr; sv += tL.d * X3[j];
        SL[K3][j] = sv;
        float sg = tG.u * X1[j];
        sg += tG.l * xl; sg += tG.c * X2[j]; sg += tG.r * xr; sg += tG.d * X3[j];
        SG[K3][j] = sg;
      }
    }
    {  // l and o at row r = t-2 -> slot K3 (zero outside the image); s rows t-3, t-2, t-1 = K1, K2, K3
      const int r = t - 2;
      const bool rin = r >= 0 && r < H;
      const float (&S0)[V] = SL[K1];
      const float (&S1)[V] = SL[K2];
      const float (&S2)[V] = SL[K3];
      const float (&G0)[V] = SG[K1];
      const float (&G1)[V] = SG[K2];
      const float (&G2)[V] = SG[K3];
      const float pv = lane_prev(S1[V - 1]), nx = lane_next(S1[0]);
      const float sp = lane_prev(G1[V - 1]), sn = lane_next(G1[0]);
      const float wp = lane_prev(WG[0][V - 1]);
      const float (&cvp)[V] = cv[(P + 1) & 1];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int col = c0 + j;
        const float up = (!EDGE || r > 0) ? S0[j] : S1[j];
        const float dn = (!EDGE || r < H - 1) ? S2[j] : S1[j];
        const float lf = col > 0 ? (j > 0 ? S1[j - 1] : pv) : S1[j];
        const float rt = col < WW - 1 ? (j < V - 1 ? S1[j + 1] : nx) : S1[j];
        const float wx = ((WL[0][j] * up + WL[1][j] * lf) + WL[2][j] * rt) + WL[3][j] * dn;
        const float lv = S1[j] - wx;
        const float sv = G1[j];
        const float snx = j < V - 1 ? G1[j + 1] : sn;
        const float spv = j > 0 ? G1[j - 1] : sp;
        const float chl = col > 0 ? (j > 0 ? WG[0][j - 1] : wp) : 0.f;
        const float cvu = (!EDGE || r > 0) ? cvp[j] : 0.f;
        const float ov = WG[0][j] * (sv - snx) + chl * (sv - spv) + WG[1][j] * (sv - G2[j]) + cvu * (sv - G0[j]);
        const bool in = (!EDGE || rin) && (!CE || col < WW);
        L[K3][j] = in ? lv : 0.f;
        O[K3][j] = in ? ov : 0.f;
      }
#pragma unroll
      for (int j = 0; j < V; ++j) cv[P & 1][j] = WG[1][j];
    }
    {  // S^T at row t-3 from l / o rows t-4, t-3, t-2 = slots K1, K2, K3
      const float (&L0)[V] = L[K1];
      const float (&L1)[V] = L[K2];
      const float (&L2)[V] = L[K3];
      const float (&O0)[V] = O[K1];
      const float (&O1)[V] = O[K2];
      const float (&O2)[V] = O[K3];
      const float lp = lane_prev(L1[V - 1]), ln = lane_next(L1[0]);
      const float op = lane_prev(O1[V - 1]), on = lane_next(O1[0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float nx = j < V - 1 ? L1[j + 1] : ln, pv = j > 0 ? L1[j - 1] : lp;
        float v = tL.u * L2[j];
        v += tL.l * nx; v += tL.c * L1[j]; v += tL.r * pv; v += tL.d * L0[j];
        tl[j] = v;
        const float gx = j < V - 1 ? O1[j + 1] : on, gp = j > 0 ? O1[j - 1] : op;
        float w = tG.u * O2[j];
        w += tG.l * gx; w += tG.c * O1[j]; w += tG.r * gp; w += tG.d * O0[j];
        tg[j] = w;
      }
    }
  }
};

// The GTV proximal term C^T phi_gamma(C s) of the same input rows an OpPipe streams (the first-pair
// kernel's right-hand side B, REF:757-781): s = S_G x is the pipe's SG rows (same stencil), so this adds
// only the prox rows o and their S_G^T.  The arithmetic of graph_row_kernel's GTV_PROX consume.
// Weight rows of l / o row r = t-2: W4 = the four raw planes at row r, wup = plane 0 (up) at row r+1,
// wdn = plane 3 (down) at row r-1.
template <int V>
struct ProxExt {
  float O[4][V];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < V; ++j) O[k][j] = 0.f;
  }
  template <int P, int W, bool EDGE = true>
  __device__ __forceinline__ void advance(const OpPipe<V>& pp, const float (&W4)[4][V], const float (&wup)[V],
                                          const float (&wdn)[V], int t, int H, int c0, const Taps& tG, float gam,
                                          float (&tp)[V]) {
    constexpr int K1 = (P + 1) & 3, K2 = (P + 2) & 3, K3 = (P + 3) & 3;
    {  // o at row r = t-2 from s rows t-3, t-2, t-1 = the pipe's SG slots K1, K2, K3
      const int r = t - 2;
      const bool rin = r >= 0 && r < H;
      const float (&G0)[V] = pp.SG[K1];
      const float (&G1)[V] = pp.SG[K2];
      const float (&G2)[V] = pp.SG[K3];
      const float sp = lane_prev(G1[V - 1]), sn = lane_next(G1[0]);
      const float w1n = lane_next(W4[1][0]), w2p = lane_prev(W4[2][V - 1]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int col = c0 + j;
        const float sv = G1[j];
        const float su = (!EDGE || r > 0) ? G0[j] : sv, sd = (!EDGE || r < H - 1) ? G2[j] : sv;
        const float spv = j > 0 ? G1[j - 1] : sp, snx = j < V - 1 ? G1[j + 1] : sn;
        const float sl = col > 0 ? spv : sv, sr = col < W - 1 ? snx : sv;
        const float w0 = W4[0][j], w1 = W4[1][j], w2 = W4[2][j], w3 = W4[3][j];
        const float z0 = prox_phi(w0 * sv - w0 * su, gam) * w0;
        const float z1 = prox_phi(w1 * sv - w1 * sl, gam) * w1;
        const float z2 = prox_phi(w2 * sv - w2 * sr, gam) * w2;
        const float z3 = prox_phi(w3 * sv - w3 * sd, gam) * w3;
        float ov = ((z0 + z1) + z2) + z3;
        const float wupb = wup[j];                                   // w_up(q + down)
        const float wlfr = j < V - 1 ? W4[1][j + 1] : w1n;           // w_left(q + right)
        const float wrtl = j > 0 ? W4[2][j - 1] : w2p;               // w_right(q - right)
        const float wdna = wdn[j];                                   // w_down(q - down)
        const float o1 = ov - prox_phi(wupb * G2[j] - wupb * sv, gam) * wupb;
        ov = (!EDGE || r < H - 1) ? o1 : ov;
        const float o2 = ov - prox_phi(wlfr * snx - wlfr * sv, gam) * wlfr;
        ov = col < W - 1 ? o2 : ov;
        const float o3 = ov - prox_phi(wrtl * spv - wrtl * sv, gam) * wrtl;
        ov = col > 0 ? o3 : ov;
        const float o4 = ov - prox_phi(wdna * G0[j] - wdna * sv, gam) * wdna;
        ov = (!EDGE || r > 0) ? o4 : ov;
        O[K3][j] = (!EDGE || rin) ? ov : 0.f;
      }
    }
    {  // S_G^T at row t-3 from o rows t-4, t-3, t-2 = slots K1, K2, K3
      const float (&O0)[V] = O[K1];
      const float (&O1)[V] = O[K2];
      const float (&O2)[V] = O[K3];
      const float op = lane_prev(O1[V - 1]), on = lane_next(O1[0]);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float gx = j < V - 1 ? O1[j + 1] : on, gp = j > 0 ? O1[j - 1] : op;
        float w = tG.u * O2[j];
        w += tG.l * gx; w += tG.c * O1[j]; w += tG.r * gp; w += tG.d * O0[j];
        tp[j] = w;
      }
    }
  }
};

constexpr int S2_W = 256, S2_HW = 128;    // full / half row width
constexpr int S2_WP = 7;                   // weight-ring row pairs
constexpr int S2_HR = 4;                   // half-weight ring rows
constexpr int S2_XR = 8;                   // x_{k+1} ring rows (per channel)
constexpr int S2_UR = 10;                  // u_{k+1} ring rows (per channel)
constexpr int S2_DR = 4;                   // D x_{k+1} ring half rows (per channel)
constexpr int S2_TR = 2;                   // t_k ring half rows (per channel)
constexpr int S2_FMAX = 3;                 // channel waves per graph
constexpr int S2_PAIR = 2 * 6 * S2_W;      // floats per weight-ring pair
constexpr int S2_HROW = 6 * S2_HW;         // floats per half-weight ring row
constexpr int S2_LDS = S2_WP * S2_PAIR + S2_HR * S2_HROW +
                       S2_FMAX * (S2_XR * S2_W + S2_UR * S2_W + S2_DR * S2_HW + S2_TR * S2_HW);
constexpr int S2_NT = 2;                   // cache policy (nt) of step2's read-once / write-once streams
constexpr int S2_UNROLL = 4;               // iterations per loop body (the pipelines' slot period)
#ifndef GRR_STEP2_AHEAD
#define GRR_STEP2_AHEAD 2
#endif
constexpr int S2_AHEAD = GRR_STEP2_AHEAD;  // iterations between a channel wave's row loads and their use (1 or 2)
static_assert(S2_AHEAD == 1 || S2_AHEAD == 2, "step2 load distance");
static_assert(S2_LDS * 4 <= 163840, "step2 LDS");
// First pair (stage 0, right-hand side B, stage 1; graph_step2_kernel<.., FIRST>): stage 1 has no heavy-ball
// term (no u ring); x_1 ring of 7 rows; the half-weight ring row holds 12 planes (wL1 x4, cG1 x2, the prox
// level's wG1 x4 at the row, plane 0 one row down, plane 3 one row up); the prox weight ring holds two
// row pairs of wG0 (4 planes x 2 rows, plane 0 two rows down, plane 3 one row up: 10 rows each).
constexpr int S2F_XR = 7;
constexpr int S2F_HPL = 12;
constexpr int S2F_PR = 10;
constexpr int S2F_LDS = S2_WP * S2_PAIR + S2_HR * S2F_HPL * S2_HW + S2_FMAX * (S2F_XR * S2_W + S2_DR * S2_HW + S2_TR * S2_HW) +
                        2 * S2F_PR * S2_W;
static_assert(S2F_LDS * 4 <= 163840, "first-pair LDS");
// Waves (wave w runs on SIMD w mod 4): stage B of channel f = wave f, the producer = wave
// S2_FMAX, stage A of channel f = wave S2_FMAX + 1 + f, stage A's half level (all channels) =
// wave 2 S2_FMAX + 1.  The two waves of channel f share a SIMD, so each of SIMDs 0-2 issues its
// vector work from two waves (a lone wave issues at half the VALU rate); SIMD 3 holds the
// producer and the half-level wave.  Everything the waves exchange goes through LDS rings
// (x_{k+1}, u_{k+1}, D x_{k+1}, t_k), written at least one barrier before it is read.
constexpr int S2_PRODUCER = S2_FMAX, S2_HALFW = 2 * S2_FMAX + 1;
constexpr int S2_THREADS = 64 * (2 * S2_FMAX + 2);
// Column strips (W != S2_W, W % 8 == 0): a workgroup covers image columns x0 .. x0 + 255,
// x0 = S2_SOWN * strip, and stores the columns it owns, [x0 + S2_HALO, x0 + S2_W - S2_HALO)
// (from column 0 in the first strip, to W in the last).  The lanes' neighbour exchanges are
// wrong at the window's two outer columns; the error spreads 3 columns per operator at the full
// level, 3 half columns at the half level: t_k 6, x_{k+1} 6, t_{k+1} 12, x_{k+2} 12 columns.  The
// 16-column halo covers that.
constexpr int S2_HALO = 16, S2_SOWN = S2_W - 2 * S2_HALO;

// FIRST: stage A = stage 0 (x_0 = b = the right-hand side A, no u), stage B = the prox right-hand side B
// (REF:757-781) of x_1 and stage 1 on it: the prox terms reuse the stage-B pipes' s rows (same stencils,
// same input rows), b_B is formed in registers at the row stage 1 emits and stored beside x_2, u_2; x_1
// never leaves the CU.  W = S2_W only (no strips), no training instance.
template <bool MID, bool STRIPS, bool FIRST = false>
__global__ __launch_bounds__(S2_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
void graph_step2_kernel(Step2Args a) {
  static_assert(!FIRST || (!MID && !STRIPS), "first pair: inference, W = 256");
  constexpr int V = 4, VH = 2, W = S2_W, hw = S2_HW;
  typedef typename VecT<4>::type F4;
  typedef typename VecT<2>::type F2;
  constexpr int XR = FIRST ? S2F_XR : S2_XR;            // x_{k+1} ring rows
  constexpr int UR = FIRST ? 0 : S2_UR;                 // u_{k+1} ring rows
  constexpr int HPL = FIRST ? S2F_HPL : 6;              // planes per half-weight ring row
  constexpr int HROW = HPL * S2_HW;
  __shared__ __attribute__((aligned(16))) float lds[FIRST ? S2F_LDS : S2_LDS];
  float* const wring = lds;
  float* const hring = wring + S2_WP * S2_PAIR;
  float* const xring = hring + S2_HR * HROW;
  float* const uring = xring + S2_FMAX * XR * S2_W;
  float* const dring = uring + S2_FMAX * UR * S2_W;
  float* const tring = dring + S2_FMAX * S2_DR * S2_HW;
  float* const pring = tring + S2_FMAX * S2_TR * S2_HW;   // (FIRST) prox weight pairs
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int F = a.F;
  uint32_t unit = xcd_remap(blockIdx.x, a.nblk);
  int strip = 0;
  if constexpr (STRIPS) { strip = unit % a.nstrips; unit /= a.nstrips; }
  const int seg = unit % a.nsegs; unit /= a.nsegs;
  const int grp = unit % a.ngrp; unit /= a.ngrp;
  const int fb = grp * a.FG, Fg = min(a.FG, F - fb);   // this workgroup's channels fb .. fb + Fg - 1 of graph g
  const int g = unit % a.G;
  const int b = unit / a.G;
  const int H = a.H, h = H / 2;
  const int Wi = STRIPS ? a.W : W, hwi = Wi / 2;   // image row widths (full / half level)
  const int64_t HW = (int64_t)H * Wi, hHW = (int64_t)h * hwi;
  const int64_t PB = HW * 4, HPB = hHW * 4;
  const uint32_t RB = (uint32_t)Wi * 4u, HRB = (uint32_t)hwi * 4u;
  const int C = a.G * F;
  const int c0 = 4 * lane, ch0 = 2 * lane;   // the lane's columns in the LDS rows
  // image columns of the lane (cg, chg: edge rules; loads clamp into the image) and the
  // columns this workgroup stores
  const int x0 = STRIPS ? S2_SOWN * strip : 0;
  const int cg = x0 + c0, chg = x0 / 2 + ch0;
  const uint32_t vo = (uint32_t)(STRIPS ? clampi(cg, 0, Wi - V) : c0) * 4u;
  const uint32_t vo_half = (uint32_t)(STRIPS ? clampi(chg, 0, hwi - VH) : ch0) * 4u;
  const int own_lo = STRIPS && strip > 0 ? x0 + S2_HALO : 0;
  const int own_hi = STRIPS && strip < a.nstrips - 1 ? x0 + S2_W - S2_HALO : Wi;
  const bool own = !STRIPS || (cg >= own_lo && cg < own_hi);
  const int r0 = seg * a.sseg, r1 = min(r0 + a.sseg, H);
  const int ts = r0 - 9;                 // first step (odd offset from r0: step t emits stage-A row t-3)
  const int NI0 = (r1 + 11 - ts) / 2;    // stage B emits rows up to r1 - 1
  const int NI = (NI0 + S2_UNROLL - 1) / S2_UNROLL * S2_UNROLL;   // extra iterations store nothing
  // In the iteration where stage A pools half row 0 (t = 3, top segment only), the stage-B half
  // level reads that row as its replicate-clamped row -1: one extra barrier for every wave orders
  // the stage-A write before the stage-B read
  const int i_top = r0 == 0 ? (3 - ts) / 2 : -1;
  const float scl1 = expf(a.log_mu1[g]), scg1 = expf(a.log_ro1[g]);

  if (wave == S2_PRODUCER) {   // producer: weight rows -> LDS rings (LDS-DMA), two iterations ahead
    const float* pwl0 = a.wL0 + (int64_t)(b * a.G + g) * 4 * HW;
    const float* pcg0 = a.cG0 + (int64_t)(b * a.G + g) * 2 * HW;
    const float* pwl1 = a.wL1 + (int64_t)(b * a.G + g) * 4 * hHW;
    const float* pcg1 = a.cG1 + (int64_t)(b * a.G + g) * 2 * hHW;
    auto dma = [&](const float* src, float* dst) {
      const uint32_t m0v = (uint32_t)(uintptr_t)(lds_f32_t)dst;
      asm volatile("global_load_lds_dwordx4 %0, off nt" ::"v"(src), "{m0}"(__builtin_amdgcn_readfirstlane(m0v))
                   : "memory");
    };
    auto dma_pair = [&](int p) {   // full-level weight rows of steps ts+2p, ts+2p+1 (rows t-2)
      float* slot = wring + (p % S2_WP) * S2_PAIR;
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        const int64_t rw = (int64_t)clampi(ts + 2 * p + par - 2, 0, H - 1) * Wi + vo / 4u;
#pragma unroll
        for (int e = 0; e < 6; ++e)
          dma(e < 4 ? pwl0 + e * HW + rw : pcg0 + (e - 4) * HW + rw, slot + (par * 6 + e) * S2_W);
      }
    };
    // (FIRST) the prox level's raw weights
    const float* pwg0 = FIRST ? a.wG0 + (int64_t)(b * a.G + g) * 4 * HW : nullptr;
    const float* pwg1 = FIRST ? a.wG1 + (int64_t)(b * a.G + g) * 4 * hHW : nullptr;
    auto dma_half = [&](int p) {   // half-level weight row of iteration p (the stage-B half level's l/o row)
      const int hr0 = (ts + 2 * p - 3) / 2 - 3;
      const int hr = clampi(hr0, 0, h - 1);
      float* slot = hring + (p % S2_HR) * HROW;
      const int pl = lane >> 5;   // lanes 0-31: plane 2e, lanes 32-63: plane 2e+1
#pragma unroll
      for (int e = 0; e < HPL / 2; ++e) {
        const int plane = 2 * e + pl;
        const int hc = STRIPS ? clampi(x0 / 2 + (lane & 31) * 4, 0, hwi - 4) : (lane & 31) * 4;
        const float* src;
        if (plane < 4) src = pwl1 + plane * hHW + (int64_t)hr * hwi;
        else if (plane < 6) src = pcg1 + (plane - 4) * hHW + (int64_t)hr * hwi;
        else if (plane < 10) src = pwg1 + (plane - 6) * hHW + (int64_t)hr * hwi;
        else if (plane == 10) src = pwg1 + (int64_t)clampi(hr0 + 1, 0, h - 1) * hwi;          // w_up, row + 1
        else src = pwg1 + 3 * hHW + (int64_t)clampi(hr0 - 1, 0, h - 1) * hwi;                  // w_down, row - 1
        dma(src + hc, slot + e * 2 * S2_HW);
      }
    };
    // (FIRST) prox weight pair of iteration p: stage B's o rows ra = t - 10, ra + 1 (t = ts + 2p), four planes
    // each, then plane 0 at ra + 2 and plane 3 at ra - 1; into slot p mod 2 (one iteration ahead)
    auto dma_prox = [&](int p) {
      const int ra = ts + 2 * p - 10;
      float* slot = pring + (p & 1) * (S2F_PR * S2_W);
#pragma unroll
      for (int k = 0; k < S2F_PR; ++k) {
        const int e = k < 8 ? (k & 3) : (k == 8 ? 0 : 3);
        const int rr = k < 8 ? ra + (k >> 2) : (k == 8 ? ra + 2 : ra - 1);
        dma(pwg0 + e * HW + (int64_t)clampi(rr, 0, H - 1) * Wi + vo / 4u, slot + k * S2_W);
      }
    };
    // vmcnt immediate: the DMAs of the newest pair + half row may be in flight (15 / 18)
    constexpr int kAheadDmas = 12 + HPL / 2;
    if constexpr (FIRST) dma_prox(0);
    dma_pair(0);
    dma_half(0);
    dma_pair(1);
    dma_half(1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kAheadDmas) : "memory");   // iteration 0's rows landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    for (int i = 0; i < NI; ++i) {
      if constexpr (FIRST) dma_prox(i + 1);   // the slot iteration i - 1 read
      dma_pair(i + 2);
      dma_half(i + 2);
      if (i == i_top) __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kAheadDmas) : "memory");  // iteration i+1's rows landed
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  if (wave == S2_HALFW) {
    // Stage A's half level t_k = mu1 S_L^T l + ro1 S_G^T o of D x_k (the grr_system_half launch
    // the per-stage path runs before each stage), one half row per iteration for every channel:
    // iteration i emits half row hb + 1 + i into t-ring slot (i + 1) & 1 for stage A's iteration
    // i + 1, from D x_k half row hb + 4 + i (HBM) and the half-level weight row hb + 2 + i (plain
    // loads; the producer's LDS-DMA reads the same row for the stage-B half level four
    // iterations later, from L2).  The pipeline is primed with 8 rows before the first barrier.
    const int hb = (ts - 3) / 2;   // the half row stage A reads in iteration 0 (ts - 3 is even)
    const int64_t gq = (int64_t)b * a.G + g;
    const rsrc_t rxq = make_rsrc(a.xd + ((int64_t)b * C + (int64_t)g * F + fb) * hHW, (int64_t)Fg * HPB);
    const rsrc_t rwl = make_rsrc(a.wL1 + gq * 4 * hHW, 4 * HPB);
    const rsrc_t rcg = make_rsrc(a.cG1 + gq * 2 * hHW, 2 * HPB);
    Taps tLh[S2_FMAX], tGh[S2_FMAX];
#pragma unroll
    for (int f = 0; f < S2_FMAX; ++f) {
      const int chf = g * F + fb + min(f, Fg - 1);
      tLh[f] = make_taps(a.sL1, chf);
      tGh[f] = make_taps(a.sG1, chf);
    }
    struct LdH {
      float xq[S2_FMAX][VH], w[6][VH];
    };
    // channels f >= Fg read past the operand's range: 0
    auto issue_h = [&](int hin, LdH& L) {
      const uint32_t ro = vo_half + (uint32_t)clampi(hin, 0, h - 1) * HRB;
#pragma unroll
      for (int f = 0; f < S2_FMAX; ++f) bload<VH, S2_NT>(L.xq[f], rxq, (uint32_t)(f * HPB) + ro);
      const uint32_t rw = vo_half + (uint32_t)clampi(hin - 2, 0, h - 1) * HRB;
#pragma unroll
      for (int e = 0; e < 4; ++e) bload<VH>(L.w[e], rwl, (uint32_t)(e * HPB) + rw);
#pragma unroll
      for (int e = 0; e < 2; ++e) bload<VH>(L.w[4 + e], rcg, (uint32_t)(e * HPB) + rw);
    };
    OpPipe<VH> PF[S2_FMAX];
#pragma unroll
    for (int f = 0; f < S2_FMAX; ++f) PF[f].zero();
    float res[S2_FMAX][VH];
    auto hadv = [&](int hin, const LdH& L, auto ph_tag) {
      constexpr int P = decltype(ph_tag)::value;
      float WL[4][VH], WG[2][VH];
#pragma unroll
      for (int k = 0; k < VH; ++k) {
#pragma unroll
        for (int e = 0; e < 4; ++e) WL[e][k] = L.w[e][k];
        WG[0][k] = L.w[4][k];
        WG[1][k] = L.w[5][k];
      }
#pragma unroll
      for (int f = 0; f < S2_FMAX; ++f) {
        if (f < Fg) {
          float tl[VH], tg[VH];
          PF[f].template advance<P, hw, true, STRIPS>(L.xq[f], WL, WG, hin, h, STRIPS ? chg : ch0, tLh[f], tGh[f],
                                                      tl, tg, hwi);
#pragma unroll
          for (int k = 0; k < VH; ++k) {   // mu * S_L^T l + ro * S_G^T o, grr_system_half's epilogue
            float rv = tl[k] * scl1;
            rv = rv + tg[k] * scg1;
            res[f][k] = rv;
          }
        }
      }
    };
    auto put = [&](int slot) {
#pragma unroll
      for (int f = 0; f < S2_FMAX; ++f)
        if (f < Fg) {
          F2 q;
          q[0] = res[f][0]; q[1] = res[f][1];
          *reinterpret_cast<F2*>(tring + (f * S2_TR + slot) * S2_HW + ch0) = q;
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    LdH Q[4];
    issue_h(hb - 4, Q[0]);
    issue_h(hb - 3, Q[1]);
    issue_h(hb - 2, Q[2]);
    issue_h(hb - 1, Q[3]);
    hadv(hb - 4, Q[0], I0{});
    issue_h(hb, Q[0]);
    hadv(hb - 3, Q[1], I1{});
    issue_h(hb + 1, Q[1]);
    hadv(hb - 2, Q[2], I2{});
    issue_h(hb + 2, Q[2]);
    hadv(hb - 1, Q[3], I3{});
    issue_h(hb + 3, Q[3]);
    hadv(hb, Q[0], I0{});
    hadv(hb + 1, Q[1], I1{});
    issue_h(hb + 4, Q[0]);
    hadv(hb + 2, Q[2], I2{});
    hadv(hb + 3, Q[3], I3{});   // emits half row hb
    put(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    auto hiter = [&](int i, auto pi_tag) {
      constexpr int PI = decltype(pi_tag)::value;
      issue_h(hb + 5 + i, Q[(PI + 1) & 1]);
      hadv(hb + 4 + i, Q[PI & 1], pi_tag);
      put((PI + 1) & 1);
      if (i == i_top) __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    for (int i = 0; i < NI; i += S2_UNROLL) {
      hiter(i, I0{});
      hiter(i + 1, I1{});
      hiter(i + 2, I2{});
      hiter(i + 3, I3{});
    }
    return;
  }

  // ---- channel wave f: stage B = wave f < S2_FMAX, stage A = wave S2_FMAX + 1 + f
  const bool role_a = wave > S2_PRODUCER;
  const int f = role_a ? wave - S2_PRODUCER - 1 : wave;
  if (f >= Fg) {   // spare wave of a group with Fg < S2_FMAX channels: the barriers only
    for (int i = 0; i <= NI + (i_top >= 0); ++i) __builtin_amdgcn_s_barrier();
    return;
  }
  const int ch = g * F + fb + f;
  const int64_t plane = ((int64_t)b * C + ch) * HW, hplane = ((int64_t)b * C + ch) * hHW;
  const bool use_beta_a = a.beta_a != nullptr && a.u_prev != nullptr;
  const bool use_skip = a.skip != nullptr;
  const rsrc_t rx = make_rsrc(a.x + plane, PB);
  const rsrc_t rb = make_rsrc(FIRST ? nullptr : a.b + plane, PB);
  const rsrc_t ru = make_rsrc(use_beta_a && !FIRST ? a.u_prev + plane : nullptr, PB);   // absent: reads 0
  // y: the block skip's (step2) or right-hand side B's (FIRST; [B,F,H,W] when it replicates an image)
  const int64_t yplane = FIRST && a.yr_rep ? ((int64_t)b * F + fb + f) * HW : plane;
  const rsrc_t ry = make_rsrc(FIRST ? a.yr + yplane : (use_skip ? a.y + plane : nullptr), PB);
  const rsrc_t rbo = make_rsrc(FIRST ? a.b_out + plane : nullptr, FIRST ? PB : 0);
  const rsrc_t rout = make_rsrc(a.out + plane, PB);
  const rsrc_t ruo = make_rsrc(a.u_out ? a.u_out + plane : nullptr, PB);
  const rsrc_t rxd = make_rsrc(a.xd_out ? a.xd_out + hplane : nullptr, HPB);
  // MID (training): the middle iterate x_{k+1}, u_{k+1} also goes to HBM (a separate instance, so the
  // inference kernel keeps its registers)
  const rsrc_t rxm = make_rsrc(MID ? a.x_mid + plane : nullptr, MID ? PB : 0);
  const rsrc_t rum = make_rsrc(MID ? a.u_mid + plane : nullptr, MID ? PB : 0);
  const rsrc_t rxdm = make_rsrc(MID && a.xd_mid ? a.xd_mid + hplane : nullptr, MID && a.xd_mid ? HPB : 0);

  const float scl0 = expf(a.log_mu0[g]), scg0 = expf(a.log_ro0[g]);
  // absent terms enter as exact zeros / ones: u_prev reads 0 (beta 0), y reads 0 (skip 0, 1)
  const float alpha_a = a.alpha_a[g], beta_a = use_beta_a ? a.beta_a[g] : 0.f;
  const float alpha_b = a.alpha_b[g], beta_b = a.beta_b ? a.beta_b[g] : 0.f;
  float sk0 = 0.f, sk1 = 1.f;
  if (use_skip) { sk0 = a.skip[0]; sk1 = a.skip[1]; }
  const Taps tL0 = make_taps(a.sL0, ch), tG0 = make_taps(a.sG0, ch);
  const Taps tL1 = make_taps(a.sL1, ch), tG1 = make_taps(a.sG1, ch);
  const float gam0 = FIRST ? expf(a.log_gamma0[g]) : 0.f, gam1 = FIRST ? expf(a.log_gamma1[g]) : 0.f;

  float* const xr = xring + f * XR * S2_W + c0;
  float* const ur = uring + f * UR * S2_W + c0;
  float* const dr = dring + f * S2_DR * S2_HW + ch0;
  const float* const tr = tring + f * S2_TR * S2_HW + ch0;
  const float* const wl_lane = wring + c0;
  const float* const hw_lane = hring + ch0;

  struct Ld {
    float x[V], eb[V], eu[V], b2[V], y2[V];
  };
  // read-once streams (x_k, u_k, weights) are non-temporal so that b's rows stay in L2 for
  // stage B's second read 8 rows later (one HBM read of b per launch)
  auto issue_a = [&](int t, Ld& S) {
    // (FIRST: b = x_0 is the row the pipe already holds; no u)
    bload<V, S2_NT>(S.x, rx, vo + clampi(t, 0, H - 1) * RB);
    if constexpr (!FIRST) {
      const int re = clampi(t - 3, 0, H - 1);
      bload(S.eb, rb, vo + re * RB);
      bload<V, S2_NT>(S.eu, ru, vo + re * RB);
    }
  };
  auto issue_b = [&](int t, Ld& S) {
    const int r2 = clampi(t - 11, 0, H - 1);
    if constexpr (!FIRST) bload(S.b2, rb, vo + r2 * RB);
    bload<V, FIRST ? S2_NT : 0>(S.y2, ry, vo + r2 * RB);
  };
  auto ring_w = [&](const float* row, float (&WL)[4][V], float (&WG)[2][V]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const F4 q = *reinterpret_cast<const F4*>(row + e * S2_W);
#pragma unroll
      for (int j = 0; j < V; ++j) WL[e][j] = q[j];
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const F4 q = *reinterpret_cast<const F4*>(row + (4 + e) * S2_W);
#pragma unroll
      for (int j = 0; j < V; ++j) WG[e][j] = q[j];
    }
  };
  auto st4 = [&](float* p, const float (&v)[V]) {
    F4 q;
#pragma unroll
    for (int j = 0; j < V; ++j) q[j] = v[j];
    *reinterpret_cast<F4*>(p) = q;
  };
  auto ld4 = [&](const float* p, float (&v)[V]) {
    const F4 q = *reinterpret_cast<const F4*>(p);
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = q[j];
  };

  OpPipe<V> PA, PQ;
  OpPipe<VH> PH;
  PA.zero();
  PQ.zero();
  PH.zero();
  float TH[VH] = {};
  // (FIRST) the prox terms of right-hand side B on stage B's pipes: full level (x_1) and half level (D x_1)
  ProxExt<V> XQ;
  ProxExt<VH> XH;
  float TP[VH] = {};
  if constexpr (FIRST) {
    XQ.zero();
    XH.zero();
  }
  float xa0[V], xb0[V];   // the even row of the current iteration (2x2 pooling)

  // stage A (stage k) at step t: emits row t-3 into the x / u rings, D x half rows at odd rows;
  // th = t_k at half row (t-3) >> 1 (from the t ring)
  auto stage_a = [&](int t, const Ld& S, const float (&thv)[VH], int q, auto par_tag, auto ph_tag, auto edge_tag) __attribute__((always_inline)) {
    constexpr int PAR = decltype(par_tag)::value, P = decltype(ph_tag)::value;
    constexpr bool EDGE = decltype(edge_tag)::value;
    float WL[4][V], WG[2][V], tl[V], tg[V];
    ring_w(wl_lane + q * S2_PAIR + PAR * 6 * S2_W, WL, WG);
    PA.template advance<P, W, EDGE, STRIPS>(S.x, WL, WG, t, H, STRIPS ? cg : c0, tL0, tG0, tl, tg, Wi);
    const float (&x0)[V] = PA.template x_out<P>();
    const int y = t - 3;
    float xn[V], u[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float th = 0.25f * thv[j >> 1];
      float ax = x0[j];
      ax = ax + tl[j] * scl0;
      ax = ax + tg[j] * scg0;
      ax = ax + th;
      float uv;
      if constexpr (FIRST) {
        uv = x0[j] - ax;                                  // stage 0: b = x_0 (REF:751-753)
      } else {
        uv = S.eb[j] - ax;
        uv = uv + beta_a * S.eu[j];
      }
      u[j] = uv;
      xn[j] = x0[j] + alpha_a * uv;
    }
    if (y >= 0 && y < H) {   // uniform: rows outside the image never enter the rings
      st4(xr + (FIRST ? y % XR : y & (XR - 1)) * S2_W, xn);
      if constexpr (!FIRST) st4(ur + (y % UR) * S2_W, u);
    }
    if constexpr (MID) {     // training: the middle iterate's rows of this segment to HBM
      const uint32_t so = (y >= r0 && y < r1 && own) ? vo + (uint32_t)y * RB : GRR_OOB;
      bstore<V>(rxm, so, xn);
      bstore<V>(rum, so, u);
    }
    if constexpr (PAR == 0) {
#pragma unroll
      for (int j = 0; j < V; ++j) xa0[j] = xn[j];
    } else {
      const int hA = (y - 1) / 2;
      float d[VH];
#pragma unroll
      for (int k = 0; k < VH; ++k)
        d[k] = 0.25f * xa0[2 * k] + 0.25f * xa0[2 * k + 1] + 0.25f * xn[2 * k] + 0.25f * xn[2 * k + 1];
      if (hA >= 0 && hA < h) *reinterpret_cast<F2*>(dr + (hA & (S2_DR - 1)) * S2_HW) = F2{d[0], d[1]};
      // training: D x_{k+1} to HBM (the reverse sweep's half-level operand), the values stage B read
      if constexpr (MID)
        bstore<VH>(rxdm, (y >= r0 && y < r1 && own) ? vo_half + (uint32_t)hA * HRB : GRR_OOB, d);
    }
  };

  // half level of D x_{k+1}: input half row hA - 1 (clamped), emits t_{k+1} half row hA - 4
  auto stage_h = [&](int hA, int qh, auto ph_tag, auto edge_tag) __attribute__((always_inline)) {
    constexpr int P = decltype(ph_tag)::value;
    constexpr bool EDGE = decltype(edge_tag)::value;
    const int hin = hA - 1;
    float xh[VH], WL[4][VH], WG[2][VH], tl[VH], tg[VH];
    {
      const F2 q = *reinterpret_cast<const F2*>(dr + (clampi(hin, 0, h - 1) & (S2_DR - 1)) * S2_HW);
      xh[0] = q[0]; xh[1] = q[1];
    }
    const float* row = hw_lane + qh * HROW;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const F2 q = *reinterpret_cast<const F2*>(row + e * S2_HW);
      WL[e][0] = q[0]; WL[e][1] = q[1];
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const F2 q = *reinterpret_cast<const F2*>(row + (4 + e) * S2_HW);
      WG[e][0] = q[0]; WG[e][1] = q[1];
    }
    PH.template advance<P, hw, EDGE, STRIPS>(xh, WL, WG, hin, h, STRIPS ? chg : ch0, tL1, tG1, tl, tg, hwi);
#pragma unroll
    for (int k = 0; k < VH; ++k) {
      float rv = tl[k] * scl1;
      rv = rv + tg[k] * scg1;
      TH[k] = rv;
    }
    if constexpr (FIRST) {   // right-hand side B's half level: C^T phi(C s) of D x_1 (grr_gtv_rhs_half, prox)
      float W4[4][VH], wup[VH], wdn[VH], tp[VH];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const F2 q = *reinterpret_cast<const F2*>(row + (6 + e) * S2_HW);
        W4[e][0] = q[0]; W4[e][1] = q[1];
      }
      {
        const F2 q = *reinterpret_cast<const F2*>(row + 10 * S2_HW);
        wup[0] = q[0]; wup[1] = q[1];
        const F2 r = *reinterpret_cast<const F2*>(row + 11 * S2_HW);
        wdn[0] = r[0]; wdn[1] = r[1];
      }
      XH.template advance<P, hw, EDGE>(PH, W4, wup, wdn, hin, h, ch0, tG1, gam1, tp);
#pragma unroll
      for (int k = 0; k < VH; ++k) TP[k] = tp[k];
    }
  };

  // stage B (stage k+1) at step t: input x_{k+1} row t-8, emits row t-11 to HBM
  // FIRST: b = right-hand side B at that row, y + ro0 C^T phi(C s) + ro1 U(t') (grr_gtv_rhs_full's
  // expression), formed from the same x_1 rows (prox weights: pring slot qp) and stored beside x_{k+2}
  auto stage_b = [&](int t, const Ld& S, int q, int qp, auto par_tag, auto ph_tag, auto edge_tag) __attribute__((always_inline)) {
    constexpr int PAR = decltype(par_tag)::value, P = decltype(ph_tag)::value;
    constexpr bool EDGE = decltype(edge_tag)::value;
    const int tb = t - 8;
    float xin[V], WL[4][V], WG[2][V], tl[V], tg[V], up[V];
    ld4(xr + (FIRST ? clampi(tb, 0, H - 1) % XR : clampi(tb, 0, H - 1) & (XR - 1)) * S2_W, xin);
    ring_w(wl_lane + q * S2_PAIR + PAR * 6 * S2_W, WL, WG);
    const int y = t - 11;
    if constexpr (!FIRST) ld4(ur + (((y % UR) + UR) % UR) * S2_W, up);
    PQ.template advance<P, W, EDGE, STRIPS>(xin, WL, WG, tb, H, STRIPS ? cg : c0, tL0, tG0, tl, tg, Wi);
    const float (&x0)[V] = PQ.template x_out<P>();
    float bv[V];
    if constexpr (FIRST) {
      const float* prow = pring + qp * (S2F_PR * S2_W) + c0;
      float W4[4][V], wup[V], wdn[V], tp[V];
#pragma unroll
      for (int e = 0; e < 4; ++e) ld4(prow + (PAR * 4 + e) * S2_W, W4[e]);
      ld4(prow + (PAR == 0 ? 4 : 8) * S2_W, wup);
      ld4(prow + (PAR == 0 ? 9 : 3) * S2_W, wdn);
      XQ.template advance<P, W, EDGE>(PQ, W4, wup, wdn, tb, H, c0, tG0, gam0, tp);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float rv = S.y2[j] + tp[j] * scg0;
        rv = rv + (0.25f * TP[j >> 1]) * scg1;
        bv[j] = rv;
      }
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) bv[j] = S.b2[j];
    }
    float res[V], xn[V], u[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float th = 0.25f * TH[j >> 1];
      float ax = x0[j];
      ax = ax + tl[j] * scl0;
      ax = ax + tg[j] * scg0;
      ax = ax + th;
      float uv = bv[j] - ax;
      if constexpr (!FIRST) uv = uv + beta_b * up[j];
      u[j] = uv;
      xn[j] = x0[j] + alpha_b * uv;
      res[j] = FIRST ? xn[j] : sk0 * S.y2[j] + sk1 * xn[j];
    }
    const bool yv = y >= r0 && y < r1 && own;
    const uint32_t so = yv ? vo + (uint32_t)y * RB : GRR_OOB;
    bstore<V, S2_NT>(rout, so, res);
    bstore<V, S2_NT>(ruo, so, u);
    if constexpr (FIRST) bstore<V, S2_NT>(rbo, so, bv);
    if constexpr (PAR == 0) {
#pragma unroll
      for (int j = 0; j < V; ++j) xb0[j] = xn[j];
    } else {
      float d[VH];
#pragma unroll
      for (int k = 0; k < VH; ++k)
        d[k] = 0.25f * xb0[2 * k] + 0.25f * xb0[2 * k + 1] + 0.25f * xn[2 * k] + 0.25f * xn[2 * k + 1];
      bstore<VH, S2_NT>(rxd, yv ? vo_half + (uint32_t)(y >> 1) * HRB : GRR_OOB, d);
    }
  };

  Ld LA, LB, LC, LD;   // rows of iterations i (A, B) and, at S2_AHEAD = 2, i + 1 (C, D) in flight
  if (role_a) {
    issue_a(ts, LA);
    issue_a(ts + 1, LB);
    if (S2_AHEAD == 2) {
      issue_a(ts + 2, LC);
      issue_a(ts + 3, LD);
    }
    // Ring rows the pipelines read before their first write (rows above the image / before the
    // segment, weight pairs of stage B's fill) only feed rows that are never stored, but through
    // products with a 0 weight: zero them so the garbage is finite.  Weight slots 2..6 are first
    // filled after the barrier below.
    const float zero4[V] = {};
#pragma unroll
    for (int r = 0; r < XR; ++r) st4(xr + r * S2_W, zero4);
#pragma unroll
    for (int r = 0; r < UR; ++r) st4(ur + r * S2_W, zero4);
    *reinterpret_cast<F4*>(dring + f * S2_DR * S2_HW + 4 * lane) = F4{0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<F4*>(dring + f * S2_DR * S2_HW + S2_W + 4 * lane) = F4{0.f, 0.f, 0.f, 0.f};
    for (int r = f; r < (S2_WP - 2) * 12; r += Fg) st4(wring + 2 * S2_PAIR + r * S2_W + c0, zero4);
  } else {
    issue_b(ts, LA);
    issue_b(ts + 1, LB);
    if (S2_AHEAD == 2) {
      issue_b(ts + 2, LC);
      issue_b(ts + 3, LD);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // the producer's first ring rows and the first t_k row have landed
  asm volatile("" ::: "memory");
  int qa = 0;
  // stage-A wave: two rows of stage k per iteration; stage-B wave: the half level and two rows of
  // stage k+1 (8 rows behind, its inputs written into the rings at least one barrier earlier).
  // PI = the iteration's phase in the unrolled body (pipelines A, B advance two slots per
  // iteration, the half level one)
  auto iteration_a = [&](int i, auto pi_tag, auto edge_tag) __attribute__((always_inline)) {
    constexpr int PI = decltype(pi_tag)::value;
    using P0 = std::integral_constant<int, (2 * PI) & 3>;
    using P1 = std::integral_constant<int, (2 * PI + 1) & 3>;
    using E = decltype(edge_tag);
    const int t = ts + 2 * i;
    float thv[VH];
    {
      const F2 q = *reinterpret_cast<const F2*>(tr + (PI & 1) * S2_HW);   // t_k half row (t-3)/2
      thv[0] = q[0]; thv[1] = q[1];
    }
    Ld& LX = (S2_AHEAD == 2 && (PI & 1)) ? LC : LA;
    Ld& LY = (S2_AHEAD == 2 && (PI & 1)) ? LD : LB;
    stage_a(t, LX, thv, qa, std::integral_constant<int, 0>{}, P0{}, E{});
    issue_a(t + 2 * S2_AHEAD, LX);
    stage_a(t + 1, LY, thv, qa, std::integral_constant<int, 1>{}, P1{}, E{});
    issue_a(t + 2 * S2_AHEAD + 1, LY);
    if (i == i_top) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    qa = qa == S2_WP - 1 ? 0 : qa + 1;
  };
  auto iteration_b = [&](int i, auto pi_tag, auto edge_tag) __attribute__((always_inline)) {
    constexpr int PI = decltype(pi_tag)::value;
    using P0 = std::integral_constant<int, (2 * PI) & 3>;
    using P1 = std::integral_constant<int, (2 * PI + 1) & 3>;
    using PHh = std::integral_constant<int, PI & 3>;
    using E = decltype(edge_tag);
    const int t = ts + 2 * i;
    const int qb = qa >= 4 ? qa - 4 : qa + 3;   // pair i - 4 (mod 7)
    if (i == i_top) __builtin_amdgcn_s_barrier();
    stage_h((t - 3) / 2, i & (S2_HR - 1), PHh{}, E{});
    Ld& LX = (S2_AHEAD == 2 && (PI & 1)) ? LC : LA;
    Ld& LY = (S2_AHEAD == 2 && (PI & 1)) ? LD : LB;
    stage_b(t, LX, qb, PI & 1, std::integral_constant<int, 0>{}, P0{}, E{});
    issue_b(t + 2 * S2_AHEAD, LX);
    stage_b(t + 1, LY, qb, PI & 1, std::integral_constant<int, 1>{}, P1{}, E{});
    issue_b(t + 2 * S2_AHEAD + 1, LY);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    qa = qa == S2_WP - 1 ? 0 : qa + 1;
  };
  if (role_a) {
    for (int i = 0; i < NI; i += S2_UNROLL) {
      iteration_a(i, std::integral_constant<int, 0>{}, std::true_type{});
      iteration_a(i + 1, std::integral_constant<int, 1>{}, std::true_type{});
      iteration_a(i + 2, std::integral_constant<int, 2>{}, std::true_type{});
      iteration_a(i + 3, std::integral_constant<int, 3>{}, std::true_type{});
    }
  } else {
    for (int i = 0; i < NI; i += S2_UNROLL) {
      iteration_b(i, std::integral_constant<int, 0>{}, std::true_type{});
      iteration_b(i + 1, std::integral_constant<int, 1>{}, std::true_type{});
      iteration_b(i + 2, std::integral_constant<int, 2>{}, std::true_type{});
      iteration_b(i + 3, std::integral_constant<int, 3>{}, std::true_type{});
    }
  }
}

static int step2_seg_rows(int H, uint64_t blocks_per_seg) {
  // one workgroup per CU: at least 2 workgroups per CU where the batch allows, segments of >= 64 rows
  int sseg = H;
  while (sseg > 64 && blocks_per_seg * (uint64_t)((H + sseg - 1) / sseg) < 512) sseg = ((sseg / 2) + 1) & ~1;
  return sseg;
}

}  // namespace grr

using namespace grr;

// Streaming copy (one float4 per lane, non-temporal): the HBM ceiling the bench reports
// beside the step kernel's rate (measured on the same GPU in the same run).
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void stream_copy_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                          int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) {
    const f32x4 v = __builtin_nontemporal_load(src + i);
    __builtin_nontemporal_store(v, dst + i);
  }
}

extern "C" {

int grr_version(void) { return 1; }

grr_status grr_stream_copy(const float* src, float* dst, int64_t n, void* stream) {
  clear_error();
  GRR_REQUIRE(src && dst && n > 0 && n % 4 == 0 && (uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0,
              GRR_ERR_INVALID_ARG, "grr_stream_copy: bad args");
  const int64_t n4 = n / 4;
  GRR_REQUIRE(n4 / 256 < (1ll << 31) - 1, GRR_ERR_UNSUPPORTED, "grr_stream_copy: too large");
  const int blocks = (int)((n4 + 255) / 256);
  hipLaunchKernelGGL(stream_copy_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const f32x4*>(src), reinterpret_cast<f32x4*>(dst), n4);
  return launch_status("grr_stream_copy");
}

grr_status grr_set_kernel_variant(int variant) {
  clear_error();
  GRR_REQUIRE(variant >= 0 && variant <= 2, GRR_ERR_INVALID_ARG, "grr_set_kernel_variant: %d", variant);
  g_kernel_variant = variant;
  return GRR_OK;
}
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

grr_status grr_edge_weights_block(const float* feat, int64_t feat_bstride, int gtv_off, const float* multiM_gtv,
                                  int glr_off, const float* multiM_glr, float* wG, float* cG, float* wL, int B,
                                  int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(feat && multiM_gtv && multiM_glr && wG && cG && wL && B > 0 && G > 0 && F > 0 && H > 0 && W > 0 &&
                  gtv_off >= 0 && glr_off >= 0,
              GRR_ERR_INVALID_ARG, "grr_edge_weights_block: bad args");
  GRR_REQUIRE(F <= GRR_MAX_NODE_FTS, GRR_ERR_UNSUPPORTED, "grr_edge_weights_block: F=%d > %d", F, GRR_MAX_NODE_FTS);
  hipStream_t s = (hipStream_t)stream;
  EdgeArgs a{};
  a.feat = feat; a.bstride = feat_bstride;
  a.slab_off[0] = gtv_off; a.multiM[0] = multiM_gtv; a.w[0] = wG; a.c[0] = cG;
  a.slab_off[1] = glr_off; a.multiM[1] = multiM_glr; a.w[1] = wL; a.c[1] = nullptr;
  a.nslab = 2; a.G = G; a.H = H; a.W = W;
  if (launch_edge_row(a, B, F, s)) return launch_status("grr_edge_weights_block");
  const int64_t HW = (int64_t)H * W;
  grr_status st = grr_edge_weights(feat + (int64_t)gtv_off * HW, feat_bstride, multiM_gtv, wG, nullptr, B, G, F, H,
                                   W, stream);
  if (st != GRR_OK) return st;
  st = grr_gtv_pair_weights(wG, cG, B, G, H, W, stream);
  if (st != GRR_OK) return st;
  return grr_edge_weights(feat + (int64_t)glr_off * HW, feat_bstride, multiM_glr, wL, nullptr, B, G, F, H, W, stream);
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

grr_status grr_gtv_rhs_full_rep(const float* x, int x_rep, const float* y, int y_rep, const float* wG, grr_stencil sG, int prox,
                            const float* log_gamma, const float* log_ro0, const float* t_half, const float* log_ro1,
                            float* b_out, float* xd_out, int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && y && wG && b_out && log_ro0 && stencil_ok(sG) && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_gtv_rhs_full_rep: bad args");
  GRR_REQUIRE(!prox || log_gamma, GRR_ERR_INVALID_ARG, "grr_gtv_rhs_full_rep: prox needs log_gamma");
  GRR_REQUIRE(!t_half || log_ro1, GRR_ERR_INVALID_ARG, "grr_gtv_rhs_full_rep: t_half needs log_ro1");
  GRR_REQUIRE(!(t_half || xd_out) || (H % 2 == 0 && W % 2 == 0), GRR_ERR_SHAPE,
              "grr_gtv_rhs_full_rep: two-scale operator needs even H, W (got %dx%d)", H, W);
  OpArgs a{};
  a.x = x; a.y = y; a.x_rep = x_rep != 0; a.y_rep = y_rep != 0; a.wG = wG; a.sG = sG; a.log_gamma = log_gamma; a.log_g = log_ro0;
  a.t_half = t_half; a.log_half = log_ro1; a.out = b_out; a.xd_out = xd_out;
  a.G = G; a.F = F; a.H = H; a.W = W;
  hipStream_t s = (hipStream_t)stream;
  if (prox) return launch_op<false, GTV_PROX, EPI_RHS>(a, B, s, "grr_gtv_rhs_full_rep");
  return launch_op<false, GTV_PAIR, EPI_RHS>(a, B, s, "grr_gtv_rhs_full_rep");
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

static grr_status system_step2_impl(const float* x, const float* b, const float* u_prev, const float* xd,
                                    const float* wL0, const float* cG0, grr_stencil sL0, grr_stencil sG0,
                                    const float* log_mu0, const float* log_ro0, const float* wL1, const float* cG1,
                                    grr_stencil sL1, grr_stencil sG1, const float* log_mu1, const float* log_ro1,
                                    const float* alpha_a, const float* beta_a, const float* alpha_b,
                                    const float* beta_b, const float* skip, const float* y_skip, float* x_out,
                                    float* u_out, float* xd_out, float* x_mid, float* u_mid, float* xd_mid, int B,
                                    int G, int F, int H, int W, void* stream) {
  GRR_REQUIRE(x && b && xd && wL0 && cG0 && wL1 && cG1 && log_mu0 && log_ro0 && log_mu1 && log_ro1 && alpha_a &&
                  alpha_b && x_out && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_system_step2: bad args");
  GRR_REQUIRE(stencil_ok(sL0) && stencil_ok(sG0) && stencil_ok(sL1) && stencil_ok(sG1), GRR_ERR_INVALID_ARG,
              "grr_system_step2: stencil missing");
  GRR_REQUIRE(!skip || y_skip, GRR_ERR_INVALID_ARG, "grr_system_step2: skip needs y_skip");
  GRR_REQUIRE(!beta_a || u_prev, GRR_ERR_INVALID_ARG, "grr_system_step2: beta_a needs u_prev");
  GRR_REQUIRE((W == S2_W || (W % 8 == 0 && W >= 8)) && H % 2 == 0 && H >= 2, GRR_ERR_UNSUPPORTED,
              "grr_system_step2: needs W = %d or W %% 8 == 0, and even H (got H %d, W %d)", S2_W, H, W);
  GRR_REQUIRE((int64_t)H * W * 4 < (1ll << 31), GRR_ERR_UNSUPPORTED, "grr_system_step2: plane too large");
  GRR_REQUIRE(x_out != x && x_out != b && x_out != u_prev && (!u_out || (u_out != u_prev && u_out != x && u_out != b)),
              GRR_ERR_INVALID_ARG, "grr_system_step2: outputs must not alias the inputs (rows are read ahead)");
  const void* ptrs[] = {x, b, u_prev, xd, wL0, cG0, wL1, cG1, y_skip, x_out, u_out, xd_out, x_mid, u_mid, xd_mid};
  for (const void* q : ptrs)
    GRR_REQUIRE((uintptr_t)q % 16 == 0, GRR_ERR_INVALID_ARG, "grr_system_step2: operands must be 16-byte aligned");
  Step2Args a{};
  a.x_mid = x_mid; a.u_mid = u_mid; a.xd_mid = xd_mid;
  a.x = x; a.b = b; a.u_prev = u_prev; a.xd = xd;
  a.wL0 = wL0; a.cG0 = cG0; a.wL1 = wL1; a.cG1 = cG1;
  a.sL0 = sL0; a.sG0 = sG0; a.sL1 = sL1; a.sG1 = sG1;
  a.log_mu0 = log_mu0; a.log_ro0 = log_ro0; a.log_mu1 = log_mu1; a.log_ro1 = log_ro1;
  a.alpha_a = alpha_a; a.beta_a = beta_a; a.alpha_b = alpha_b; a.beta_b = beta_b;
  a.skip = skip; a.y = y_skip; a.out = x_out; a.u_out = u_out; a.xd_out = xd_out;
  a.G = G; a.F = F; a.H = H; a.W = W;
  a.nstrips = W <= S2_W ? 1 : 1 + (W - S2_W + S2_SOWN - 1) / S2_SOWN;
  a.ngrp = (F + S2_FMAX - 1) / S2_FMAX;   // F = 6 / 12 (v1.0 blocks): 2 / 4 groups of 3
  a.FG = (F + a.ngrp - 1) / a.ngrp;
  a.sseg = step2_seg_rows(H, (uint64_t)B * G * a.ngrp * a.nstrips);
  a.nsegs = (H + a.sseg - 1) / a.sseg;
  const uint64_t nblk = (uint64_t)B * G * a.ngrp * a.nsegs * a.nstrips;
  GRR_REQUIRE(nblk < (1ull << 32) - 4, GRR_ERR_UNSUPPORTED, "grr_system_step2: grid too large");
  a.nblk = (uint32_t)nblk;
  const dim3 grid(a.nblk), block(S2_THREADS);
  hipStream_t s = (hipStream_t)stream;
  if (W == S2_W) {
    if (x_mid) hipLaunchKernelGGL((graph_step2_kernel<true, false>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((graph_step2_kernel<false, false>), grid, block, 0, s, a);
  } else {   // column strips
    if (x_mid) hipLaunchKernelGGL((graph_step2_kernel<true, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((graph_step2_kernel<false, true>), grid, block, 0, s, a);
  }
  return launch_status("grr_system_step2");
}

grr_status grr_system_step2(const float* x, const float* b, const float* u_prev, const float* xd,
                            const float* wL0, const float* cG0, grr_stencil sL0, grr_stencil sG0,
                            const float* log_mu0, const float* log_ro0, const float* wL1, const float* cG1,
                            grr_stencil sL1, grr_stencil sG1, const float* log_mu1, const float* log_ro1,
                            const float* alpha_a, const float* beta_a, const float* alpha_b, const float* beta_b,
                            const float* skip, const float* y_skip, float* x_out, float* u_out, float* xd_out,
                            int B, int G, int F, int H, int W, void* stream) {
  clear_error();
  return system_step2_impl(x, b, u_prev, xd, wL0, cG0, sL0, sG0, log_mu0, log_ro0, wL1, cG1, sL1, sG1, log_mu1,
                           log_ro1, alpha_a, beta_a, alpha_b, beta_b, skip, y_skip, x_out, u_out, xd_out, nullptr,
                           nullptr, nullptr, B, G, F, H, W, stream);
}

// Stage 0, the prox right-hand side B and stage 1 in one pass (graph_step2_kernel<false, false, true>):
// REF:751-753 (x_1 = b_A + alpha_0 (b_A - A b_A)), REF:757-781 (b_B = y + ro0 C^T phi(C S x_1) +
// ro1 U(C^T phi(C S D x_1))), REF:784-790 at k = 1 (no heavy-ball term).  In: b_A, D b_A (the right-hand
// side A pass's pooled output), y ([B,C,H,W], or the [B,F,H,W] image it replicates: y_rep).  Out: b_B,
// x_2, u_2 (stage 1's residual direction, the next stage's heavy-ball term), D x_2.  x_1 stays on chip.
grr_status grr_system_first_pair(const float* b_a, const float* xd_a, const float* y, int y_rep, const float* wL0,
                                 const float* cG0, const float* wG0, grr_stencil sL0, grr_stencil sG0,
                                 const float* log_mu0, const float* log_ro0, const float* log_gamma0,
                                 const float* wL1, const float* cG1, const float* wG1, grr_stencil sL1,
                                 grr_stencil sG1, const float* log_mu1, const float* log_ro1,
                                 const float* log_gamma1, const float* alpha0, const float* alpha1, float* b_out,
                                 float* x_out, float* u_out, float* xd_out, int B, int G, int F, int H, int W,
                                 void* stream) {
  clear_error();
  GRR_REQUIRE(b_a && xd_a && y && wL0 && cG0 && wG0 && log_mu0 && log_ro0 && log_gamma0 && wL1 && cG1 && wG1 &&
                  log_mu1 && log_ro1 && log_gamma1 && alpha0 && alpha1 && b_out && x_out && u_out && xd_out &&
                  B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_system_first_pair: bad args");
  GRR_REQUIRE(stencil_ok(sL0) && stencil_ok(sG0) && stencil_ok(sL1) && stencil_ok(sG1), GRR_ERR_INVALID_ARG,
              "grr_system_first_pair: stencil missing");
  GRR_REQUIRE(W == S2_W && H % 2 == 0 && H >= 2, GRR_ERR_UNSUPPORTED,
              "grr_system_first_pair: needs W = %d and even H (got H %d, W %d)", S2_W, H, W);
  const void* outs[] = {b_out, x_out, u_out, xd_out};
  const void* ins[] = {b_a, xd_a, y};
  for (const void* o : outs)
    for (const void* i : ins)
      GRR_REQUIRE(o != i, GRR_ERR_INVALID_ARG, "grr_system_first_pair: outputs must not alias the inputs");
  const void* ptrs[] = {b_a, xd_a, y, wL0, cG0, wG0, wL1, cG1, wG1, b_out, x_out, u_out, xd_out};
  for (const void* q : ptrs)
    GRR_REQUIRE((uintptr_t)q % 16 == 0, GRR_ERR_INVALID_ARG, "grr_system_first_pair: operands must be 16-byte aligned");
  Step2Args a{};
  a.x = b_a; a.xd = xd_a;
  a.wL0 = wL0; a.cG0 = cG0; a.wL1 = wL1; a.cG1 = cG1;
  a.sL0 = sL0; a.sG0 = sG0; a.sL1 = sL1; a.sG1 = sG1;
  a.log_mu0 = log_mu0; a.log_ro0 = log_ro0; a.log_mu1 = log_mu1; a.log_ro1 = log_ro1;
  a.alpha_a = alpha0; a.alpha_b = alpha1;
  a.out = x_out; a.u_out = u_out; a.xd_out = xd_out;
  a.wG0 = wG0; a.wG1 = wG1; a.log_gamma0 = log_gamma0; a.log_gamma1 = log_gamma1;
  a.yr = y; a.yr_rep = y_rep != 0; a.b_out = b_out;
  a.G = G; a.F = F; a.H = H; a.W = W;
  a.nstrips = 1;
  a.ngrp = (F + S2_FMAX - 1) / S2_FMAX;
  a.FG = (F + a.ngrp - 1) / a.ngrp;
  a.sseg = step2_seg_rows(H, (uint64_t)B * G * a.ngrp);
  a.nsegs = (H + a.sseg - 1) / a.sseg;
  const uint64_t nblk = (uint64_t)B * G * a.ngrp * a.nsegs;
  GRR_REQUIRE(nblk < (1ull << 32) - 4, GRR_ERR_UNSUPPORTED, "grr_system_first_pair: grid too large");
  a.nblk = (uint32_t)nblk;
  hipLaunchKernelGGL((graph_step2_kernel<false, false, true>), dim3(a.nblk), dim3(S2_THREADS), 0,
                     (hipStream_t)stream, a);
  return launch_status("grr_system_first_pair");
}

grr_status grr_system_step2_train(const float* x, const float* b, const float* u_prev, const float* xd,
                                  const float* wL0, const float* cG0, grr_stencil sL0, grr_stencil sG0,
                                  const float* log_mu0, const float* log_ro0, const float* wL1, const float* cG1,
                                  grr_stencil sL1, grr_stencil sG1, const float* log_mu1, const float* log_ro1,
                                  const float* alpha_a, const float* beta_a, const float* alpha_b,
                                  const float* beta_b, float* x_out, float* u_out, float* xd_out, float* x_mid,
                                  float* u_mid, float* xd_mid, int B, int G, int F, int H, int W,
                                  void* stream) {
  clear_error();
  GRR_REQUIRE(x_mid && u_mid && u_out, GRR_ERR_INVALID_ARG, "grr_system_step2_train: x_mid, u_mid, u_out required");
  GRR_REQUIRE(x_mid != x && x_mid != b && x_mid != u_prev && x_mid != x_out && x_mid != u_out && u_mid != x &&
                  u_mid != b && u_mid != u_prev && u_mid != x_out && u_mid != u_out && x_mid != u_mid,
              GRR_ERR_INVALID_ARG, "grr_system_step2_train: x_mid / u_mid must not alias other operands");
  return system_step2_impl(x, b, u_prev, xd, wL0, cG0, sL0, sG0, log_mu0, log_ro0, wL1, cG1, sL1, sG1, log_mu1,
                           log_ro1, alpha_a, beta_a, alpha_b, beta_b, nullptr, nullptr, x_out, u_out, xd_out, x_mid,
                           u_mid, xd_mid, B, G, F, H, W, stream);
}

grr_status grr_glr_stage(const float* x, const float* b, const float* u_prev, const float* wL, grr_stencil sL,
                         const float* mu, const float* alpha, const float* beta, float* x_out, float* u_out, int B,
                         int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && b && wL && mu && alpha && x_out && stencil_ok(sL) && B > 0 && G > 0 && F > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_glr_stage: bad args");
  GRR_REQUIRE(!u_prev || beta, GRR_ERR_INVALID_ARG, "grr_glr_stage: u_prev needs beta");
  GRR_REQUIRE(x_out != x && x_out != b && (!u_prev || x_out != u_prev) && (!u_out || u_out != x),
              GRR_ERR_INVALID_ARG, "grr_glr_stage: outputs must not alias the stencil inputs");
  OpArgs a{};
  a.x = x; a.b = b; a.u_prev = u_prev; a.wL = wL; a.sL = sL;
  a.log_l = mu; a.lin_l = 1; a.alpha = alpha; a.beta = beta;
  a.out = x_out; a.u_out = u_out;
  a.G = G; a.F = F; a.H = H; a.W = W;
  return launch_op<true, GTV_NONE, EPI_STEP>(a, B, (hipStream_t)stream, "grr_glr_stage");
}

}  // extern "C"
