/*
 * grr.h — C ABI of the MI355X (gfx950) graph-regularizer restoration engine.
 *
 * One shared library (libgrr.so) built with hipcc for gfx950.  Every entry point
 * takes raw DEVICE pointers (fp32, contiguous NCHW unless stated), explicit sizes
 * and the caller's hipStream_t (passed as void*).  The caller allocates every
 * tensor it computes on; the only library state is the training reverse's per-stream reduction
 * scratch (grr_set_scratch_allocator).  It never synchronises, and is safe to call from several host
 * threads (re-entrant).  Each call returns a
 * grr_status; on failure grr_last_error() (thread-local) holds a message.
 *
 * Reference interfaces replaced (REF = exploration/GGTV_GGLR_v1.0/
 * deep_multiscale_GGLR_GGTV_v1x0.py; REF13 = exploration/model_multiscale_mixture_GLR/
 * lib/model_GLR_GTV_deep_v13_no_latent.py) are cited per function.
 *
 * Shapes: B batch, G graphs, F node features per graph, C = G*F channels,
 * H x W the resolution of the level a call runs at.  Edge order is the
 * reference's: 0 up (-1,0), 1 left (0,-1), 2 right (0,+1), 3 down (+1,0).
 */
#ifndef GRR_H
#define GRR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum grr_status {
  GRR_OK = 0,
  GRR_ERR_INVALID_ARG = 1, /* null pointer / non-positive size            */
  GRR_ERR_SHAPE = 2,       /* shape the reference itself cannot run (odd H at a pooled level, ...) */
  GRR_ERR_UNSUPPORTED = 3, /* outside this build's limits (e.g. F > GRR_MAX_NODE_FTS) */
  GRR_ERR_HIP = 4          /* HIP launch error                           */
} grr_status;

#define GRR_MAX_NODE_FTS 24

/* Library / error plumbing. */
int grr_version(void);
const char* grr_last_error(void);

/* Kernel-variant knob for tests and benchmarks (no reference counterpart): 0 = automatic
 * (row-wave graph operators for W <= 256 with the channel waves of a graph in lockstep,
 * column strips above), 1 = column-strip graph operators at every width, 2 = automatic
 * without the lockstep.  Process-wide; results agree to fp32 rounding either way. */
grr_status grr_set_kernel_variant(int variant);
/* Measurement knob (process-wide, like grr_set_kernel_variant): which phases a C <= 128 LocalNonLinearBlock
 * forward (grr_lnb_forward / grr_lnb_forward_rep) launches -- 1 weight packing, 2 head (LN + W1 +
 * depthwise + gate -> the workspace's g), 4 mix (W2 g + skip -> out).  7 (default) = all; a caller
 * times head and mix apart by running mask 3 then mask 4 on the same workspace. */
grr_status grr_lnb_set_phases(int mask);

/* Reduction scratch of the training reverse (no reference counterpart: the reference reverses through
 * autograd).  The reverse entry points (grr_bwd_*, grr_lnb_*_bwd, grr_dwconv3_bwd, grr_win_bwd_*, the
 * sub-API *_bwd) reduce per-graph scalars, taps and LN / depthwise weights in a fixed order through a
 * small device scratch of partial sums.  The library keeps one grow-only scratch buffer per (device,
 * stream) -- a second one only while calls nest on a stream -- and reuses it for later calls on that
 * stream (stream order makes the reuse safe).  The buffers come from the allocator registered here
 * (alloc(bytes, device, stream, ctx) returns a device pointer or NULL; free(ptr, device, stream, ctx)),
 * or from hipMalloc when none is registered (both NULL).  The Python package registers PyTorch's
 * caching allocator, so the scratch is PyTorch memory.  A call made while its stream is being captured
 * into a HIP graph takes its own scratch as a hipMallocAsync / hipFreeAsync pair on that stream (memory
 * nodes the graph owns): a replayed graph shares no scratch with eager calls on the stream or with
 * another graph, and grr_release_scratch never frees memory a graph uses.
 * grr_release_scratch frees every stream buffer (the caller synchronises the streams first);
 * grr_scratch_bytes reports the bytes held. */
typedef void* (*grr_scratch_alloc_fn)(uint64_t bytes, int device, void* stream, void* ctx);
typedef void (*grr_scratch_free_fn)(void* ptr, int device, void* stream, void* ctx);
grr_status grr_set_scratch_allocator(grr_scratch_alloc_fn alloc, grr_scratch_free_fn free_fn, void* ctx);
grr_status grr_release_scratch(void);
int64_t grr_scratch_bytes(void);

/* Measurement helper (not a reference interface): float4 streaming copy of n floats
 * (n % 4 == 0, 16-byte aligned), the HBM ceiling bench.py reports beside the step kernel. */
grr_status grr_stream_copy(const float* src, float* dst, int64_t n, void* stream);

/* a1 — integer neighbour table (bit-exact target).  out[e*H*W + p] = flat index
 * of clamp(p + delta_e): the pixel the reference's replicate-padded gather reads
 * for edge e (REF:128-144, GLRFast.get_neighbors_pixels).  out: int32 [4,H,W]. */
grr_status grr_neighbor_table(int32_t* out, int H, int W, void* stream);

/* a3+a4 — edge weights of one graph module (REF:146-175, GLRFast/GTVFast
 * .extract_edge_weights).  feat points at channel 0 of the module's [G*F] channel
 * slab inside a feature tensor whose batch stride is feat_bstride elements
 * (so the GTV/GLR halves of the 2C feature conv output need no copy, REF:714).
 * multiM [G,F].  Writes w [B,G,4,H,W] and, if deg != NULL, deg [B,G,H,W]. */
grr_status grr_edge_weights(const float* feat, int64_t feat_bstride, const float* multiM,
                            float* w, float* deg, int B, int G, int F, int H, int W, void* stream);

/* Symmetric pair weights of the linear graph-TV operator C^T C: for the edge
 * between p and its right / lower neighbour, c[.,0,p] = w_right(p)^2 + w_left(p+right)^2,
 * c[.,1,p] = w_down(p)^2 + w_up(p+down)^2 (0 where that neighbour is outside).
 * Algebraically identical to REF:452-516 (op_C then op_C_transpose with the
 * frame-dropped scatter).  w [B,G,4,H,W] -> c [B,G,2,H,W]. */
grr_status grr_gtv_pair_weights(const float* w, float* c, int B, int G, int H, int W, void* stream);

/* Both graph modules of one MixtureGTVGLR level in one call (REF:712-729): the GTV slab
 * (channels [gtv_off, gtv_off + G*F) of feat) -> raw weights wG [B,G,4,H,W] and pair
 * weights cG [B,G,2,H,W] (= grr_gtv_pair_weights(wG)); the GLR slab -> wL.  Same values as
 * grr_edge_weights (+ grr_gtv_pair_weights); a single row-wave launch where W <= 256. */
grr_status grr_edge_weights_block(const float* feat, int64_t feat_bstride, int gtv_off, const float* multiM_gtv,
                                  int glr_off, const float* multiM_glr, float* wG, float* cG, float* wL,
                                  int B, int G, int F, int H, int W, void* stream);

/* D — 2x2 mean pool, stride 2 (REF:613, :662-665).  x [B,C,H,W] -> xd [B,C,H/2,W/2]. */
grr_status grr_pool2(const float* x, float* xd, int B, int C, int H, int W, void* stream);

/* Per-module stencil parameters: the four [C] vectors stats_kernel_p01, _p02a,
 * _p02b, _p03 of one GLRFast/GTVFast module (REF:66-118, :177-215). */
typedef struct grr_stencil {
  const float* p01;
  const float* p02a;
  const float* p02b;
  const float* p03;
} grr_stencil;

/* Half-resolution system term (REF:661-675, inside apply_lightweight_transformer):
 *   t = exp(log_mu[g]) * S_L^T (I - W_L) S_L xd  +  exp(log_ro[g]) * G(xd)
 * G = graph-TV C^T C with pair weights cG.  Either term may be disabled by a NULL
 * weight pointer.  xd [B,C,h,w], wL [B,G,4,h,w], cG [B,G,2,h,w] -> t [B,C,h,w]. */
grr_status grr_system_half(const float* xd, const float* wL, const float* cG,
                           grr_stencil sL, grr_stencil sG,
                           const float* log_mu, const float* log_ro,
                           float* t, int B, int G, int F, int h, int w, void* stream);

/* Half-resolution GTV right-hand-side term: t = C^T phi(C xd), unscaled.
 * prox == 0: phi = identity, wG are pair weights [B,G,2,h,w] (rhs A, REF:739-747).
 * prox != 0: phi(t) = eps - (t - eps), eps = soft_threshold(t, exp(log_gamma[g])),
 *            wG are raw edge weights [B,G,4,h,w] (rhs B, REF:758-779; REF:684-704). */
grr_status grr_gtv_rhs_half(const float* xd, const float* wG, grr_stencil sG, int prox,
                            const float* log_gamma, float* t,
                            int B, int G, int F, int h, int w, void* stream);

/* Full-resolution GTV right-hand side (REF:744-749 rhs A, REF:776-781 rhs B):
 *   b = (y + exp(log_ro0[g]) * C^T phi(C x))  +  exp(log_ro1[g]) * U(t_half)
 * U = 2x2 nearest * 0.25 (conv_transpose2d of scaling_kernel01).  t_half may be NULL
 * (single-scale).  If xd_out != NULL also writes D(b).  prox/wG as grr_gtv_rhs_half. */
grr_status grr_gtv_rhs_full(const float* x, const float* y, const float* wG, grr_stencil sG,
                            int prox, const float* log_gamma, const float* log_ro0,
                            const float* t_half, const float* log_ro1,
                            float* b_out, float* xd_out,
                            int B, int G, int F, int H, int W, void* stream);

/* grr_gtv_rhs_full where x and/or y are given un-replicated, [B, F, H, W], standing for their
 * copies over the G graphs (MultiScaleGraphFilter's input, REF13:918-921; x_rep / y_rep != 0):
 * channel g*F + f reads plane f.  b_out / xd_out stay [B, G*F, ...]. */
grr_status grr_gtv_rhs_full_rep(const float* x, int x_rep, const float* y, int y_rep, const float* wG,
                                grr_stencil sG, int prox, const float* log_gamma, const float* log_ro0,
                                const float* t_half, const float* log_ro1, float* b_out, float* xd_out,
                                int B, int G, int F, int H, int W, void* stream);

/* One unrolled CG / heavy-ball stage (REF:751-753, :784-790, extension :797-807):
 *   A x   = ((x + exp(log_mu0) L0 x) + exp(log_ro0) G0 x) + U(t_half)
 *   r     = b - A x
 *   u     = r + beta[g] * u_prev      (u = r when u_prev == NULL or beta == NULL)
 *   x_out = x + alpha[g] * u
 * optional: u_out (u), xd_out (D x_out), and the LocalLowpassFilteringBlock skip
 * x_out <- skip[0] * y_skip + skip[1] * x_out when skip != NULL (REF:985-988).
 * alpha/beta point at row k of alphaCGD/betaCGD ([G]).  t_half from grr_system_half. */
grr_status grr_system_step(const float* x, const float* b, const float* u_prev, const float* t_half,
                           const float* wL, const float* cG, grr_stencil sL, grr_stencil sG,
                           const float* log_mu0, const float* log_ro0,
                           const float* alpha, const float* beta,
                           const float* skip, const float* y_skip,
                           float* x_out, float* u_out, float* xd_out,
                           int B, int G, int F, int H, int W, void* stream);

/* Two consecutive stages k, k+1 of the loop above (REF:784-790 twice) in one pass
 * (temporal blocking; t_k, x_{k+1}, u_{k+1} and t_{k+1} never leave the chip):
 *   half level A:  t_k = exp(log_mu1) L1 xd + exp(log_ro1) G1 xd, xd = D x (the previous pass's
 *                  xd_out; what grr_system_half computes)
 *   stage A (k):   x_{k+1}, u_{k+1} from x, u_prev (beta_a), t_k
 *   half level B:  t_{k+1} = exp(log_mu1) L1 (D x_{k+1}) + exp(log_ro1) G1 (D x_{k+1})
 *   stage B (k+1): x_out = x_{k+2}, u_out = u_{k+2} (beta_b with u_{k+1}), xd_out = D x_{k+2},
 *                  skip applied to x_out as in grr_system_step.
 * Same values as grr_system_half -> grr_system_step(k) -> grr_system_half -> grr_system_step(k+1) up to fp32
 * rounding order.  GLR + GTV pair at both levels; W = 256, or W % 8 == 0 (column strips of 256 lanes
 * owning 224 columns with a 16-column halo), even H; F > 3 runs as groups of <= 3
 * channels (each group reads its graph's weight rows once); outputs must
 * not alias inputs (u_out != u_prev).  Replaces two iterations of the loop body REF:784-790. */
grr_status grr_system_step2(const float* x, const float* b, const float* u_prev, const float* xd,
                            const float* wL0, const float* cG0, grr_stencil sL0, grr_stencil sG0,
                            const float* log_mu0, const float* log_ro0, const float* wL1, const float* cG1,
                            grr_stencil sL1, grr_stencil sG1, const float* log_mu1, const float* log_ro1,
                            const float* alpha_a, const float* beta_a, const float* alpha_b, const float* beta_b,
                            const float* skip, const float* y_skip, float* x_out, float* u_out, float* xd_out,
                            int B, int G, int F, int H, int W, void* stream);
/* Stage 0, right-hand side B and stage 1 in one pass (the first pair of the loop: REF:751-753, :757-781,
 * :784-790 at k = 1; x_1 never leaves the chip):
 *   half level 0:  t_0 = exp(log_mu1) L1 xd_a + exp(log_ro1) G1 xd_a, xd_a = D b_A (grr_gtv_rhs_full's
 *                  xd_out of right-hand side A; what grr_system_half computes)
 *   stage 0:       x_1 = b_A + alpha0 (b_A - A b_A)                       (grr_system_step, x = b = b_A)
 *   rhs B:         b_out = y + exp(log_ro0) C0^T phi(C0 S x_1) + exp(log_ro1) U(C1^T phi(C1 S D x_1)), the
 *                  soft threshold at exp(log_gamma0) / exp(log_gamma1), raw weights wG0 [B,G,4,H,W] /
 *                  wG1 [B,G,4,H/2,W/2]                     (grr_gtv_rhs_half + grr_gtv_rhs_full, prox)
 *   stage 1:       x_out = x_2, u_out = u_2 = b_B - A x_1, xd_out = D x_2  (grr_system_step, no heavy-ball)
 * y: [B,C,H,W], or the [B,F,H,W] image it replicates over the graphs (y_rep != 0).  Same values as
 * grr_system_half -> grr_system_step -> grr_gtv_rhs_half -> grr_gtv_rhs_full -> grr_system_half ->
 * grr_system_step up to fp32 rounding order.  W = 256, even H; F > 3 as groups of <= 3 channels; 16-byte
 * aligned operands; outputs must not alias inputs. */
grr_status grr_system_first_pair(const float* b_a, const float* xd_a, const float* y, int y_rep, const float* wL0,
                                 const float* cG0, const float* wG0, grr_stencil sL0, grr_stencil sG0,
                                 const float* log_mu0, const float* log_ro0, const float* log_gamma0,
                                 const float* wL1, const float* cG1, const float* wG1, grr_stencil sL1,
                                 grr_stencil sG1, const float* log_mu1, const float* log_ro1,
                                 const float* log_gamma1, const float* alpha0, const float* alpha1, float* b_out,
                                 float* x_out, float* u_out, float* xd_out, int B, int G, int F, int H, int W,
                                 void* stream);
/* grr_system_step2 for training: also writes the middle iterate x_{k+1} (x_mid) and its direction
 * u_{k+1} (u_mid) -- the reverse sweep's saved iterates -- besides x_{k+2}, u_{k+2} (u_out required) and
 * D x_{k+2}; no skip.  xd_mid (may be NULL): D x_{k+1}, the pooled middle iterate the kernel's half level
 * already forms, for the reverse sweep's half-level terms (no pool2 of x_{k+1} there).  Same shape
 * limits. */
grr_status grr_system_step2_train(const float* x, const float* b, const float* u_prev, const float* xd,
                                  const float* wL0, const float* cG0, grr_stencil sL0, grr_stencil sG0,
                                  const float* log_mu0, const float* log_ro0, const float* wL1, const float* cG1,
                                  grr_stencil sL1, grr_stencil sG1, const float* log_mu1, const float* log_ro1,
                                  const float* alpha_a, const float* beta_a, const float* alpha_b,
                                  const float* beta_b, float* x_out, float* u_out, float* xd_out, float* x_mid,
                                  float* u_mid, float* xd_mid, int B, int G, int F, int H, int W, void* stream);

/* One unrolled stage of the GLR-only v10 block (exploration/model_multiscale_mixture_GLR/lib/
 * model_GLR_GTV_deep_v10.py:241-335, MixtureGLR): single scale, A x = x + mu[g] L x with mu
 * stored LINEARLY (not as a log, :283-286, :296-305):
 *   r = b - A x;  u = r + beta[g] u_prev (u = r when u_prev == NULL);  x_out = x + alpha[g] u.
 * u_out may be NULL.  With x = b = y and u_prev = NULL this is stage 0 (:316-318). */
grr_status grr_glr_stage(const float* x, const float* b, const float* u_prev, const float* wL, grr_stencil sL,
                         const float* mu, const float* alpha, const float* beta, float* x_out, float* u_out,
                         int B, int G, int F, int H, int W, void* stream);

/* ---- GLRFast / GTVFast sub-API (module methods outside the fused solver) -------------
 * Standalone versions of the reference module methods, for callers of the module API (the
 * solver itself fuses the same arithmetic into the operator kernels above).  Layouts as above;
 * edge signals are [B,G,F,4,H,W] (REF:452-467). */

/* get_neighbors_pixels (REF:128-144): out[b,c,e,p] = x[b,c,clamp(p + delta_e)], out [B,C,4,H,W]. */
grr_status grr_neighbor_gather(const float* x, float* out, int B, int C, int H, int W, void* stream);
/* normalize_and_transform_features (REF:146-157): out[b, g*F + f] = f / max(|f|_2 over F, 1e-12) * multiM[g,f]. */
grr_status grr_normalize_features(const float* f, const float* multiM, float* out, int B, int G, int F, int H, int W,
                                  void* stream);
/* stats_conv (transpose == 0, replicate frame, REF:177-195) / stats_conv_transpose (transpose != 0,
 * conv_transpose2d padding 1 = zero frame, REF:197-215) with the module's stencil. */
grr_status grr_stats_conv(const float* x, grr_stencil s, int transpose, float* out, int B, int G, int F, int H, int W,
                          void* stream);
/* GLRFast.op_L_norm (REF:218-228): out = x - sum_e w_e x(clamp(p + delta_e)); x [B,G,F,H,W], w [B,G,4,H,W]. */
grr_status grr_glr_op_l_norm(const float* x, const float* w, float* out, int B, int G, int F, int H, int W,
                             void* stream);
/* GTVFast.op_C (REF:452-467): edges[b,g,f,e,p] = w_e(p) (S x)(p) - w_e(p) (S x)(clamp(p + delta_e)). */
grr_status grr_gtv_op_c(const float* x, const float* w, grr_stencil s, float* edges, int B, int G, int F, int H, int W,
                        void* stream);
/* GTVFast.op_C_transpose (REF:469-516): z_e = edges_e w_e; o(q) = sum_e z_e(q) - sum_e z_e(q - delta_e) for
 * q - delta_e inside the image (scatters into the pad frame are dropped); out = S^T o.  work [B,G,F,H,W]
 * is caller scratch (o). */
grr_status grr_gtv_op_c_transpose(const float* edges, const float* w, grr_stencil s, float* work, float* out, int B,
                                  int G, int F, int H, int W, void* stream);

/* Reverses of the sub-API methods above (the reference differentiates them with autograd over its
 * ATen ops, REF:128-228, :452-516).  Gradient outputs are overwritten except gM / gtaps, which
 * accumulate (caller zeroes); gtaps is [G*F, 5] in tap order (centre, up, left, right, down) of the
 * stencil p01 k01 + p02a k02a + p02b k02b + p03 k03.  B*C (B*G for per-graph kernels) < 65536. */
/* get_neighbors_pixels reverse: gx [B,C,H,W] from g [B,C,4,H,W] (adjoint of the clamped gather). */
grr_status grr_neighbor_gather_bwd(const float* g, float* gx, int B, int C, int H, int W, void* stream);
/* normalize_and_transform_features reverse: gf [B,G,F,H,W], gM [G,F] += ; F <= 16. */
grr_status grr_normalize_features_bwd(const float* f, const float* multiM, const float* gout, float* gf, float* gM,
                                      int B, int G, int F, int H, int W, void* stream);
/* stats_conv / stats_conv_transpose reverse: gx = S* g (S^T* g), gtaps += d<g, S x>/d taps (gtaps may be NULL). */
grr_status grr_stats_conv_bwd(const float* x, grr_stencil s, int transpose, const float* g, float* gx, float* gtaps,
                              int B, int G, int F, int H, int W, void* stream);
/* GLRFast.op_L_norm reverse: gx [B,G,F,H,W], gw [B,G,4,H,W]. */
grr_status grr_glr_op_l_norm_bwd(const float* x, const float* w, const float* g, float* gx, float* gw, int B, int G,
                                 int F, int H, int W, void* stream);
/* GTVFast.op_C reverse from gE [B,G,F,4,H,W]: gx, gw, gtaps; work [B,G,F,H,W] caller scratch. */
grr_status grr_gtv_op_c_bwd(const float* x, const float* w, grr_stencil s, const float* gE, float* work, float* gx,
                            float* gw, float* gtaps, int B, int G, int F, int H, int W, void* stream);
/* GTVFast.op_C_transpose reverse: gE [B,G,F,4,H,W], gw, gtaps; z = the forward's work buffer (the
 * pre-S^T value o), work2 [B,G,F,H,W] caller scratch. */
grr_status grr_gtv_op_c_transpose_bwd(const float* edges, const float* w, grr_stencil s, const float* z,
                                      const float* g, float* work2, float* gE, float* gw, float* gtaps, int B, int G,
                                      int F, int H, int W, void* stream);

/* ---- feature CNN (MFMA fp32) ------------------------------------------------ */

/* 1x1 convolution, no bias (nn.Conv2d(k=1, groups=1, bias=False); REF:556-566, REF13:623-632):
 * out[b,m,p] = sum_k wt[m,k] * x[b,k,p].  x [B,K,P], wt [M,K], out [B,M,P] (P = H*W). */
grr_status grr_conv1x1(const float* x, const float* wt, float* out, int B, int K, int M, int64_t P,
                       void* stream);

/* The same 1x1 convolution on bf16 MFMA with an exact 3-term split of both fp32 operands
 * (six products, fp32-accurate; see DESIGN.md "x3 GEMM").  K <= 4096 (K > 128: the K-streaming
 * kernel).  workspace: device
 * memory of grr_conv1x1_workspace_bytes(K, M) bytes, 256-B aligned (the split weights). */
int64_t grr_conv1x1_workspace_bytes(int K, int M);
grr_status grr_conv1x1_ws(const float* x, const float* wt, float* out, void* workspace, int B, int K, int M,
                          int64_t P, void* stream);

/* 2x2 stride-2 convolution, no bias (REF:593-602): x [B,K,H,W], wt [M,K,2,2] -> out [B,M,H/2,W/2]. */
grr_status grr_conv2x2s2(const float* x, const float* wt, float* out, int B, int K, int M, int H, int W,
                         void* stream);

/* FeedForward block of the window models' feature CNN (FFBlock, REF7:13-67, nn.Conv2d bias=False):
 * out = skip[0] x + skip[1] W_out (gelu(d1) * d2), [d1; d2] = dwconv3x3_zero(W_in (ln_w * x / sigma)),
 * sigma = sqrt(var_c x (unbiased) + 1e-5).  x, out [B,C,H,W]; ln_w [C]; w_in [2 hid, C]; w_dw [2 hid, 9];
 * w_out [C, hid]; skip [2] (device).  Split-bf16 MFMA GEMMs (fp32-accurate), exact erf gelu.
 * workspace: grr_ffn_workspace_bytes(B, C, hid, H, W) bytes, 256-B aligned. */
int64_t grr_ffn_workspace_bytes(int B, int C, int hid, int H, int W);
grr_status grr_ffn_forward(const float* x, const float* ln_w, const float* w_in, const float* w_dw, const float* w_out,
                           const float* skip, float* out, void* workspace, int B, int C, int hid, int H, int W,
                           void* stream);

/* Weight gradient of a 1x1 / 2x2-s2 convolution or an LNB GEMM (the reverse of REF:556-612,
 * REF13:564-575 under autograd): out[m,k] = sum_b sum_p a[b,m,p] * bop[b,k,p], a [B,M,P], bop [B,K,P],
 * out [M,K]; fp32 MFMA, partial tiles per pixel chunk added in a fixed order (deterministic, no
 * atomics).  Replaces the library GEMM torch.matmul(g, x^T).sum(0) of the reference's autograd.
 * workspace: grr_wgrad_workspace_bytes(B, M, K, P) bytes of device memory; a, bop 16-B aligned. */
int64_t grr_wgrad_workspace_bytes(int B, int M, int K, int64_t P);
/* grr_wgrad's wave tiles: 1 (default) the plan picks 128 x 96, 192 x 64 or 64 x 96 per output shape
 * (least padded MFMA work), 0 the 128 x 96 tile only.  Results are identical up to the fp32 summation
 * order of the pixel chunks.  A/B and test knob. */
grr_status grr_wgrad_set_tiles(int enable);
grr_status grr_wgrad(const float* a, const float* bop, float* out, void* workspace, int B, int M, int K, int64_t P,
                     void* stream);

/* LocalNonLinearBlock forward, nsubnets = 1 (REF:911-964; REF13:564-575):
 *   n   = gamma_c * x / sqrt(var_c(x) + 1e-5)          (CustomLayerNorm, unbiased var over C)
 *   h   = dwconv3x3_replicate(W1 n)                     (C -> 2*hid -> 2*hid)
 *   g   = sigmoid(h_mask) * h_mask * h_value            (hid)
 *   out = skip[0] * x + skip[1] * (W2 g)               (hid -> C)
 * ln_w [C] (norm.weighted_transform), w1 [2hid,C], wdw [2hid,9], w2 [C,hid], skip [2].
 * workspace: grr_lnb_workspace_bytes(B,C,hid,H,W) bytes of device memory. out may not alias x. */
int64_t grr_lnb_workspace_bytes(int B, int C, int hid, int H, int W);
grr_status grr_lnb_forward(const float* x, const float* ln_w, const float* w1, const float* wdw,
                           const float* w2, const float* skip, float* out, void* workspace,
                           int B, int C, int hid, int H, int W, void* stream);

/* The feature CNN's last 1x1 conv and the edge weights of both graph modules of a level in one pass
 * (REF:146-175, :556-612 -- REF13:887-926's patchs_features_extraction[-1] followed by extract_edge_weights
 * for the GTV and the GLR module): feat = wf x (wf [2 G F, C]: rows 0 .. G F - 1 the GTV features, then
 * the GLR features), then grr_edge_weights_block's outputs (wG, cG, wL) from feat -- without feat in memory.
 * x is [B, C, H, W], or the channel-blocked layout of grr_lnb_forward_c8 when x_blocked.  F = 3, G <= 32,
 * C = G F (grr_feature_edges_supported).  The conv runs as fp16 two-term splits of both operands (three
 * products), fp32-class like the fused LocalNonLinearBlock's GEMMs, so the weights agree with the two-pass
 * path to fp32-class rounding, not bitwise.  workspace: grr_feature_edges_workspace_bytes(G), 256-B aligned. */
int grr_feature_edges_supported(int C, int G, int F, int H, int W);
int64_t grr_feature_edges_workspace_bytes(int G);
grr_status grr_feature_edges(const float* x, int x_blocked, const float* wf, const float* multiM_gtv,
                             const float* multiM_glr, float* wG, float* cG, float* wL, void* workspace, int B,
                             int C, int G, int F, int H, int W, void* stream);

/* grr_lnb_forward with either side in the channel-blocked layout [B, ceil(C / 8), H, W, 8] (channel
 * 8 k + j of pixel p at ((b ceil(C / 8) + k) H W + p) 8 + j; pad channels 0): layout bit 0 -- x (read for
 * LN / W1 and the skip term) blocked, bit 1 -- out blocked.  Needs grr_lnb_fused(C, hid); x and out 16-B
 * aligned; workspace as grr_lnb_forward's.  Results equal grr_lnb_forward's bitwise (same arithmetic; the
 * layout only changes the kernel's memory instructions: 16- and 32-byte accesses per lane instead of
 * dwords).  A chain of blocks passes the blocked tensor from one to the next (no reference counterpart:
 * an internal layout of the feature CNN between its LocalNonLinearBlocks, REF13:541-575). */
grr_status grr_lnb_forward_c8(const float* x, const float* ln_w, const float* w1, const float* wdw,
                              const float* w2, const float* skip, float* out, void* workspace, int B, int C,
                              int hid, int H, int W, int layout, void* stream);
/* [B, C, H, W] -> blocked (to_blocked = 1, pads written 0) or back (0). */
grr_status grr_c8_convert(const float* src, float* dst, int B, int C, int H, int W, int to_blocked, void* stream);

/* grr_lnb_forward that also leaves the gated activation g = sigmoid(m) m v [B, hid, H, W] (fp32) at the
 * start of the workspace, for the training reverse's W2 weight gradient (the eager LocalNonLinearBlock
 * forward keeps it instead of recomputing the depthwise + gate).  C <= 128. */
grr_status grr_lnb_forward_keep(const float* x, const float* ln_w, const float* w1, const float* wdw,
                                const float* w2, const float* skip, float* out, void* workspace, int B, int C,
                                int hid, int H, int W, void* stream);
/* 1 when grr_lnb_forward runs the block as one fused pass for these sizes (C <= 96: LN, W1, depthwise,
 * gate and W2 in one kernel, the gated activation kept on chip).  Phase mask 2 of grr_lnb_set_phases then
 * launches the whole block and mask 4 nothing. */
int grr_lnb_fused(int C, int hid);
/* Workspace bytes grr_lnb_forward needs when grr_lnb_fused(C, hid) holds (the fused pass's chunk images
 * only: no gated tensor, no batch or image size), else 0.  grr_lnb_forward_keep still needs
 * grr_lnb_workspace_bytes (g at the workspace's start). */
int64_t grr_lnb_fused_workspace_bytes(int C, int hid);
/* Measurement knob (process-wide): 0 runs C <= 96 blocks on the two-kernel head + mix path instead of
 * the fused pass (same results to fp32 rounding); 1 (default) fused. */
grr_status grr_lnb_set_fused(int enable);
/* grr_lnb_forward for an input x [B, R*Cs, H, W] that is R stacked copies of src [B, Cs, H, W]
 * (the first feature block of MultiScaleGraphFilter, whose input replicates RGB over the graphs,
 * REF13:918-921): LN statistics and W1 are evaluated on src with W1 diag(ln_w) folded over the
 * copies (GEMM1 depth Cs instead of R*Cs); the skip reads x, or src at channel c mod Cs when
 * x == NULL (then no replicated copy needs to exist).  R*Cs <= 128.  workspace:
 * grr_lnb_workspace_bytes(B, R*Cs, hid, H, W). */
grr_status grr_lnb_forward_rep(const float* src, int Cs, int R, const float* x, const float* ln_w, const float* w1,
                               const float* wdw, const float* w2, const float* skip, float* out, void* workspace,
                               int B, int hid, int H, int W, void* stream);
/* 1 when grr_lnb_forward_rep runs the block as one fused pass for these sizes (R > 1, Cs <= 3: the
 * depthwise folded into an im2col GEMM1, gate and W2 in registers, no gated tensor in memory), else 0.
 * Phase mask 2 of grr_lnb_set_phases then launches the whole block and mask 4 nothing. */
int grr_lnb_rep_fused(int Cs, int R, int C, int hid);

/* Channel replication of MultiScaleGraphFilter.forward (REF13:918-921):
 * img [B,Cin,H,W] -> out [B,G*Cin,H,W], out[b, g*Cin + c] = img[b, c]. */
grr_status grr_repeat_graphs(const float* img, float* out, int B, int Cin, int G, int64_t P, void* stream);

/* ---- reverse pass (training, config C4) -------------------------------------
 * Adjoint building blocks of the solver; the host composes them into the reverse of
 * every operator application of MixtureGTVGLR.forward (REF:707-811), the autograd
 * graph the reference gets from PyTorch.  Layouts as above; taps [C,5] are the 3x3
 * cross stencil of one module in the order centre, up, left, right, down (built from
 * stats_kernel_p01/p02a/p02b/p03, REF:178-183).  scale: per-graph [G] multiplier or
 * NULL (=1); "accumulate"/"+=" outputs are read-modify-write, all others overwritten.
 * Reductions (gtaps, gdot, ggamma, gmultiM) are float atomics: run-to-run order may vary. */

/* mode 0: S x (replicate, REF:177-195); 1: S^T x (conv_transpose zero frame, REF:197-215);
 * 2: adjoint of mode 1; 3: adjoint of mode 0.  out = [out +] scale[g] * mode(x). */
grr_status grr_bwd_stencil(const float* x, const float* taps, int mode, const float* scale, int accumulate,
                           float* out, int B, int G, int F, int H, int W, void* stream);
/* x-gradient pass of two operator terms of one level in one sweep: out += scale1[g] P1*(v1) + scale2[g] P2*(v2),
 * P* = the adjoint of the replicate stencil (grr_bwd_stencil mode 3) with each term's taps [C,5].
 * W % 4 == 0, 16-byte aligned planes. */
grr_status grr_bwd_padj2(const float* v1, const float* taps1, const float* scale1, const float* v2, const float* taps2,
                         const float* scale2, float* out, int B, int G, int F, int H, int W, void* stream);
/* gtaps[c,t] += scale[g] * sum u(q) d(mode(z))(q)/dk_t, mode 0 (S) or 1 (S^T). */
grr_status grr_bwd_tapgrad(const float* u, const float* z, int mode, const float* scale, float* gtaps,
                           int B, int G, int F, int H, int W, void* stream);
/* GLR (I - W) reverse (REF:218-237): s = S x, a = adjoint-S^T(g).
 * z_out = (I-W) s, ap_out = (I-W)^T a, gw += scale * d<a,(I-W)s>/dw, gdot[g] += coef * <a, z>. */
grr_status grr_bwd_glr(const float* s, const float* a, const float* w, const float* scale, float coef,
                       float* z_out, float* ap_out, float* gw, float* gdot,
                       int B, int G, int F, int H, int W, void* stream);
/* Pair-Laplacian (linear C^T C, REF:452-523) reverse with pair weights c [B,G,2,H,W]:
 * z_out = K s, ap_out = K a, gc += scale * d<a,Ks>/dc, gdot[g] += coef * <a, z>. */
grr_status grr_bwd_pair(const float* s, const float* a, const float* c, const float* scale, float coef,
                        float* z_out, float* ap_out, float* gc, float* gdot,
                        int B, int G, int F, int H, int W, void* stream);
/* Prox rhs reverse, o = C^T-part(phi(C s)) with phi(t) = 2 soft(t, exp(log_gamma)) - t
 * (REF:684-704, :757-781): o_out, gs_out = d<a,o>/ds, gw += scale * d<a,o>/dw (raw weights),
 * ggamma[g] += scale * d<a,o>/dgamma, gdot[g] += coef * <a, o>. */
grr_status grr_bwd_prox(const float* s, const float* a, const float* w, const float* log_gamma,
                        const float* scale, float coef, float* o_out, float* gs_out, float* gw,
                        float* ggamma, float* gdot, int B, int G, int F, int H, int W, void* stream);
/* Widest image at which grr_bwd_term_acc_supported offers the LDS-ring row kernel with the x-gradient pass
 * inside (default 128; wider levels fold that pass into grr_bwd_cg_glue).  A/B and test knob. */
grr_status grr_bwd_set_term_acc_max_w(int w);
/* Kernel knob for tests and benchmarks (no reference counterpart): 2 (default) runs grr_bwd_term_fused
 * (and _acc) as the LDS-ring row kernel where the shape allows (W % 4 == 0, F <= 7 at 4-column lanes /
 * 12 below, 16-byte aligned planes), else as the register-prefetch row kernel; 1 always the register
 * kernel; 0 the per-pixel kernels.  grr_bwd_edge_weights: row kernel for 1 and 2.
 * Process-wide; results agree to fp32 rounding. */
grr_status grr_bwd_set_term_rows(int enable);
/* Kernel knob for tests and benchmarks (no reference counterpart): 1 (default; env GRR_TERM_TAIL) runs the
 * last column strip of a wide ring-kernel term reverse (W > 64 V, the last strip owning <= 56 columns) as
 * a second, one-column-lane launch; 0 keeps every strip at V columns per lane.  Process-wide; results
 * agree to fp32 rounding (the per-strip wave sums differ). */
grr_status grr_bwd_set_term_tail(int enable);

/* The three reverses above in one pass each, from x and g directly (s = S x and a = adjoint-S^T g
 * recomputed on the fly) with both tap gradients fused: mode 0 GLR (w raw), 1 pair Laplacian
 * (w = pair weights), 2 prox (w raw, log_gamma).  Writes v_out = (I-W)^T a, K a or d<a,o>/ds
 * (x-gradient = adjoint-S of v); gw, ggamma, gdot, gtaps (+=) as the multi-pass path, whose
 * results it reproduces.  GRR_ERR_UNSUPPORTED for F outside {1,2,3,4}. */
grr_status grr_bwd_term_fused(int mode, const float* x, const float* g, const float* taps, const float* w,
                              const float* log_gamma, const float* scale, float coef, float* v_out, float* gw,
                              float* ggamma, float* gdot, float* gtaps, int B, int G, int F, int H, int W,
                              void* stream);
/* grr_bwd_term_fused and the x-gradient pass that consumes its v (grr_bwd_stencil mode 3 with the
 * same taps and scale, accumulating) in one row-streaming pass: gx += scale[g] * adjoint-S(v), v never
 * written; gw, ggamma, gdot, gtaps as grr_bwd_term_fused.  Two calls on one gx (GLR, then pair) equal
 * grr_bwd_padj2 of the two v's.  GRR_ERR_UNSUPPORTED where grr_bwd_term_acc_supported says 0 (the
 * caller keeps the two-pass path) or a plane is not 4V-byte aligned.  The reference computes these
 * gradients by autograd through REF:218-237, :452-523, :684-704. */
int grr_bwd_term_acc_supported(int mode, int F, int H, int W);
grr_status grr_bwd_term_fused_acc(int mode, const float* x, const float* g, const float* taps, const float* w,
                                  const float* log_gamma, const float* scale, float coef, float* gx, float* gw,
                                  float* ggamma, float* gdot, float* gtaps, int B, int G, int F, int H, int W,
                                  void* stream);
/* Reverse of grr_gtv_pair_weights: gw [B,G,4,H,W] += d<gc, c(w)>/dw. */
grr_status grr_bwd_pair_weights(const float* w, const float* gc, float* gw, int B, int G, int H, int W,
                                void* stream);
/* Reverse of grr_edge_weights (REF:146-175): gfeat (slab, overwritten) and gmultiM [G,F] (+=). */
grr_status grr_bwd_edge_weights(const float* feat, int64_t feat_bstride, const float* multiM, const float* w,
                                const float* gw, float* gfeat, int64_t gfeat_bstride, float* gmultiM,
                                int B, int G, int F, int H, int W, void* stream);
/* gdot[g] += coef * sum_{b,f,p} u v  (per-graph inner product; alpha/beta/gamma gradients). */
grr_status grr_bwd_graph_dot(const float* u, const float* v, float coef, float* gdot,
                             int B, int G, int F, int H, int W, void* stream);
/* out = [out +] sa[g] x + sb[g] y  (sa/sb NULL = 1, y NULL = no second term). */
/* One reverse step of the CG / heavy-ball recurrence glue (autograd of REF:784-807 without the
 * operator term): galpha[g] += <gx, u>; gu = alpha[g] gx + beta_next[g] gu_next (gu_next may be
 * NULL); gbeta[g] += <gu, u_prev> (u_prev may be NULL); gbb += gu (gbb may be NULL);
 * gx_out = gx - gu (may alias gx).  Signals [B, G*F, H, W]; alpha, beta_next, galpha, gbeta [G].
 * Two passes of the previous reverse stage may be folded in, gx taken as
 * ((gx + scale1[g] S1*(v1)) + scale2[g] S2*(v2)) + U gx_half:
 * v1, v2 (both or neither; taps [G*F,5], scales [G]): grr_bwd_padj2's operands (W % 4 == 0, 16-byte
 * aligned); gx_half: a half-level x-gradient [B, G*F, H/2, W/2] (grr_bwd_unpool2_acc; H, W even). */
grr_status grr_bwd_cg_glue(const float* gx, const float* gx_half, const float* v1, const float* taps1,
                           const float* scale1, const float* v2, const float* taps2, const float* scale2,
                           const float* u, const float* gu_next, const float* u_prev, const float* alpha,
                           const float* beta_next, float* gu, float* gbb, float* gx_out, float* galpha, float* gbeta,
                           int B, int G, int F, int H, int W, void* stream);
/* grr_bwd_cg_glue that also writes gu_half = D gu [B, G*F, H/2, W/2] (grr_pool2's arithmetic): the
 * half-level operand of the operator reverse that reads gu next, formed in the pass that writes gu
 * (no separate pool of it).  W % 4 == 0, even H, 16-byte aligned planes. */
grr_status grr_bwd_cg_glue_pool(const float* gx, const float* gx_half, const float* v1, const float* taps1,
                                const float* scale1, const float* v2, const float* taps2, const float* scale2,
                                const float* u, const float* gu_next, const float* u_prev, const float* alpha,
                                const float* beta_next, float* gu, float* gbb, float* gx_out, float* gu_half,
                                float* galpha, float* gbeta, int B, int G, int F, int H, int W, void* stream);
grr_status grr_bwd_lincomb(const float* x, const float* sa, const float* y, const float* sb, float* out,
                           int accumulate, int B, int G, int F, int H, int W, void* stream);
/* out [B,C,H,W] += U(xd): 0.25 * xd(q/2) (conv_transpose2d of scaling_kernel01, REF:676-679). */
grr_status grr_bwd_unpool2_acc(const float* xd, float* out, int B, int C, int H, int W, void* stream);
/* gx[b,k,2i+di,2j+dj] = t[b,(2di+dj)K+k,i,j] (t [B,4K,H/2,W/2]): interleaves the four tap planes of
 * the 2x2 stride-2 conv's data gradient (REF:593-602, computed as one 1x1 GEMM with 4K rows).
 * H even, W % 4 == 0. */
grr_status grr_interleave2x2(const float* t, float* gx, int B, int K, int H, int W, void* stream);
/* Data gradient of grr_conv2x2s2: g [B,M,H/2,W/2], wt [M,K,2,2] -> gx [B,K,H,W]. */
grr_status grr_conv2x2s2_bwd_data(const float* g, const float* wt, float* gx, int B, int K, int M, int H, int W,
                                  void* stream);

/* ---- LocalNonLinearBlock reverse (training; REF:911-964) ---------------------------------
 * n = ln_w * x * isd with isd[b,p] = 1/sqrt(var_c x + 1e-5) (unbiased, uncentred x, REF:919-925). */
grr_status grr_lnb_norm(const float* x, const float* ln_w, float* n, float* isd, int B, int C, int64_t P,
                        void* stream);
/* gx [B,C,P] += d<gn, n>/dx;  gln_w [C] += sum gn x isd. */
grr_status grr_lnb_norm_bwd(const float* x, const float* ln_w, const float* isd, const float* gn, float* gx,
                            float* gln_w, int B, int C, int64_t P, void* stream);
/* grr_lnb_norm_bwd with the block's skip term in the same pass (the LocalNonLinearBlock reverse,
 * out = skip[0] x + skip[1] (...), REF13:541-575 under autograd): gx = skip[0] gout + the norm's data
 * gradient (gx written, not accumulated; gx != gout), gskip0[0] += <gout, x>, gln_w += as above. */
grr_status grr_lnb_norm_bwd_skip(const float* x, const float* ln_w, const float* isd, const float* gn,
                                 const float* gout, const float* skip, float* gx, float* gln_w, float* gskip0, int B,
                                 int C, int64_t P, void* stream);
/* depthwise 3x3 with replicate padding (channels_local_linear_op, REF:934-940): wdw [C,9]. */
grr_status grr_dwconv3(const float* h, const float* wdw, float* out, int B, int C, int H, int W, void* stream);
/* its reverse: gh = exact adjoint of the clamped gather applied to g; gwdw [C,9] += weight gradient. */
grr_status grr_dwconv3_bwd(const float* g, const float* h, const float* wdw, float* gh, float* gwdw, int B, int C,
                           int H, int W, void* stream);
/* gate = sigmoid(m) m v of hp = [m; v] [B,2hid,P] (if gate); ghp from ggate (if ggate) (REF:941-947). */
grr_status grr_lnb_gate(const float* hp, const float* ggate, float* gate, float* ghp, int B, int hid, int64_t P,
                        void* stream);
/* the gate's reverse with the skip scale folded in (autograd of REF:941-947, :962-964):
 * ghp = scale[0] * (d gate / d hp) . gq and gdot[0] += <gq, gate>, gq = W2^T gout — so the skip
 * weight's gradient <gout, W2 gate> needs no recomputed W2 gate. */
grr_status grr_lnb_gate_bwd_scaled(const float* hp, const float* gq, const float* scale, float* ghp, float* gdot, int B,
                                   int hid, int64_t P, void* stream);
/* depthwise 3x3 + gate in one row pass: gate [B,hid,H,W] = sigmoid(m) m v of (m, v) = dw3(hh) (the
 * depthwise output itself is not stored).  W <= 256 with W % V == 0, else GRR_ERR_UNSUPPORTED. */
grr_status grr_lnb_dw3_gate(const float* hh, const float* wdw, float* gate, int B, int hid, int H, int W,
                            void* stream);
/* Kernel knob (no reference counterpart): 1 (default) runs grr_lnb_gate_dw3_bwd's recomputing variant (hp NULL)
 * with its operand rows through a per-wave LDS-DMA ring where W % 4 == 0 and the planes are 16-byte aligned
 * (one strip of 8-column lanes for 256 < W <= 512, W % 8 == 0, 32-byte aligned planes), 0 the
 * register-prefetch row kernel.  Process-wide; results agree to fp32 rounding.  A/B and tests. */
grr_status grr_lnb_set_bwd_ring(int enable);
/* Host replay of the gate + depthwise reverse ring kernel's DMA geometry at image width W (W % 4 == 0): GRR_OK
 * when every ring-row DMA of every column strip writes inside its ring row and reads inside its image row
 * (the invariant whose violation faulted round 5's two-DMAs-per-row attempt), else GRR_ERR_SHAPE with the
 * first violation in grr_last_error.  Covers the strip instance of the width (V = 1, 2, 4) and, for
 * 256 < W <= 512 with W % 8 == 0, the one-strip V = 8 instance (two DMAs per 2-KB ring row) that
 * grr_lnb_gate_dw3_bwd runs there.  No device work. */
grr_status grr_dw3_ring_check(int W);
/* grr_lnb_gate_bwd_scaled and grr_dwconv3_bwd in one row pass (ghp stays on chip): hp [B,2hid,H,W]
 * (depthwise output; NULL = recomputed from hh in-kernel), gq [B,hid,H,W], hh [B,2hid,H,W]
 * (depthwise input), wdw [2hid,9] ->
 * gh [B,2hid,H,W]; gwdw [2hid,9] += ; gdot[0] += <gq, gate>.  W <= 256 with W % V == 0
 * (V = 1 / 2 / 4 for W <= 64 / 128 / 256), else GRR_ERR_UNSUPPORTED. */
grr_status grr_lnb_gate_dw3_bwd(const float* hp, const float* gq, const float* scale, const float* hh,
                                const float* wdw, float* gh, float* gwdw, float* gdot, int B, int hid, int H, int W,
                                void* stream);

/* The same two row passes for the window models' FeedForward (REF7:29-48): zero-padded depthwise
 * (nn.Conv2d padding=1) and gate = gelu(d1) d2 (exact erf gelu); the reverse recomputes the depthwise
 * output from hh (no hp operand) and adds <gq, gate> to gdot[0]. */
grr_status grr_ffn_dw3_gate(const float* hh, const float* wdw, float* gate, int B, int hid, int H, int W,
                            void* stream);
grr_status grr_ffn_gate_dw3_bwd(const float* gq, const float* scale, const float* hh, const float* wdw, float* gh,
                                float* gwdw, float* gdot, int B, int hid, int H, int W, void* stream);

/* ---- window graphs (older image-domain models) ------------------------------
 * REF7 = exploration/model_multiscale_mixture_GLR/lib/model_GLR_GTV_deep_v7.py,
 * REF1 = .../lib/model_GLR_GTV_deep_v1.py.  Graphs connect each pixel to the K
 * neighbours of a connection window; delta is a HOST array int32 [K,2] of (dy, dx)
 * offsets in the reference's edge order (itertools.product over the window, REF7:285-296),
 * |dy|, |dx| <= 2, K <= 24.  Signals x [B,G,Fs,H,W] (Fs = signal channels, 3 for RGB);
 * edge weights [B,G,K,H,W]; taps device [5] = (centre, up, left, right, down) of the
 * module's stats stencil (identity (1,0,0,0,0) for REF1, which has none). */

/* Edge weights of a window graph (GLRFast/GTVFast.extract_edge_weights, REF7:418-446):
 * feat channels [g*F, (g+1)*F) of each batch item (batch stride feat_bstride floats),
 * normalised over F, scaled by multiM [G,F], K dot products with the (replicate-clamped)
 * neighbours, softmax over the K edges -> w [B,G,K,H,W]; deg [B,G,H,W] (may be NULL). */
grr_status grr_win_edge_weights(const float* feat, int64_t feat_bstride, const float* multiM, const int32_t* delta,
                                int K, float* w, float* deg, int B, int G, int F, int H, int W, void* stream);

/* One fused pass of MixtureGTV's solver (REF7:892-1004; REF1:558-676), edge tensors never
 * materialised.  mu, ro [G] linear, log_gamma [G] (gamma = exp), alpha/beta [G] = one row.
 *  mode 0, CG step: A x = x + mu S_L^T(S_L x - W_L S_L x) + ro S_G^T C^T C S_G x (REF7:892-911),
 *          u = (y - A x) + beta u_prev (u = y - A x when u_prev == NULL), out = x + alpha u,
 *          u_out = u (may be NULL); y is the right-hand side [B,G,Fs,H,W].
 *  mode 1, rhs:      out = ro S_G^T C^T (C S_G x) + y        (first ADMM rhs, bias 0, REF7:945-949)
 *  mode 2, prox rhs: out = ro S_G^T C^T (2 soft(C S_G x, gamma) - C S_G x) + y
 *                    (one ADMM bias update from 0, REF7:958-967);
 *          modes 1/2: y [B,Fs,H,W] shared by the graphs, x per graph or (x_rep) [B,Fs,H,W].
 *  mode 3, module apply (GLRFast/GTVFast.forward, REF7:503-511, :776-782):
 *          out = mu S_L^T(S_L x - W_L S_L x) [wL != NULL] + ro S_G^T C^T C S_G x [wG != NULL];
 *          mu / ro may be NULL (= 1); y unused.
 * S reads x with a reflect frame (REF7:449-467); L/C neighbours clamp to the frame; S^T and
 * the C^T scatter drop what lands outside (REF7:469-488, :748-774).
 *  modes 4, 5, 7: modes 0, 1, 3 with wG holding the pair weights of grr_win_pair_weights (the
 *          same linear GTV term, K weight loads per position instead of 2 K). */
grr_status grr_win_solver(int mode, const float* x, int x_rep, const float* y, const float* u_prev, const float* wL,
                          const float* wG, const float* tapsL, const float* tapsG, const float* mu, const float* ro,
                          const float* log_gamma, const float* alpha, const float* beta, const int32_t* delta, int K,
                          float* out, float* u_out, int B, int G, int Fs, int H, int W, void* stream);

/* Pair weights of a window graph's linear GTV term: c [B,G,K,H,W] with
 * c_e(q) = w_e(q)^2 + [q + d_e inside] w_e'(q + d_e)^2, e' the edge of offset -d_e, so that
 * C^T C s (q) = sum_e c_e(q) (s(q) - s(clamp(q + d_e))) (the frame-dropped scatter of
 * GTVFast.op_C_transpose, REF7:748-774, paired edge by edge).  GRR_ERR_UNSUPPORTED when an offset
 * has no reverse in delta. */
grr_status grr_win_pair_weights(const float* w, const int32_t* delta, int K, float* c, int B, int G, int H, int W,
                                void* stream);

/* Graph mixture (REF7:1006-1009): out[b,c] = sum_g x[b,g,c] score[b,g] + dc[b,c] (dc may be NULL).
 * x [B,G,Fs,H,W], score [B,G,H,W], dc/out [B,Fs,H,W]. */
grr_status grr_win_mix(const float* x, const float* score, const float* dc, float* out, int B, int G, int Fs, int H,
                       int W, void* stream);

/* ---- window-graph reverse (training): replaces torch autograd through MixtureGTV's solver,
 * edge weights and mixture (REF7:418-446, :449-488, :892-1011 under loss.backward() of the
 * multiblocks training script).  Planes [B,G,Fs,H,W]; per-graph scale vectors [G] may be
 * NULL (= 1); every reduction output (gw, gdot, ggamma, gtaps, gmultiM) ACCUMULATES.
 * H, W >= 2 (the reflect frame). */

/* Stencil of the reverse: mode 0 S x (reflect frame), 1 S^T* g (zero-frame correlation),
 * 2 S* g (adjoint of the reflect-frame stencil).  out = [out +] scale[g] y. */
grr_status grr_win_bwd_stencil(const float* x, const float* taps, int mode, const float* scale, int accumulate,
                               float* out, int B, int G, int Fs, int H, int W, void* stream);
/* gtaps[t] += sum scale[g] u(p) z(src_t(p)); mode 0 src = reflect(p + d_t) (S), 1 src = p - d_t (S^T). */
grr_status grr_win_bwd_tapgrad(const float* u, const float* z, int mode, const float* scale, float* gtaps, int B,
                               int G, int Fs, int H, int W, void* stream);
/* GLR term reverse, pass 1 (s = S x, b = S^T* g): l_out = (I - W) s, gsd = scale b,
 * E [B,G,Fs,K,H,W] = scale b w_e (gathered by grr_win_bwd_gather; may be NULL with
 * grr_win_bwd_gather_fused), gw += -scale b s(n_e),
 * gdot[g] += coef <b, l>. */
grr_status grr_win_bwd_glr(const float* s, const float* b, const float* w, const int32_t* delta, int K,
                           const float* scale, float coef, float* l_out, float* E, float* gsd, float* gw, float* gdot,
                           int B, int G, int Fs, int H, int W, void* stream);
/* GTV term reverse, pass 1 (C^T C, or with prox C^T phi(C .)): gsd, E as above, PW [B,G,Fs,K,H,W] (E, PW
 * may be NULL with grr_win_bwd_gather_fused)
 * = w_e phi(z_e) (the gather rebuilds o = C^T phi from it), gw, gdot[g] += coef <b, o>,
 * ggamma[g] += dL/dgamma (prox). */
grr_status grr_win_bwd_gtv(const float* s, const float* b, const float* w, const int32_t* delta, int K, int prox,
                           const float* log_gamma, const float* scale, float coef, float* PW, float* E, float* gsd,
                           float* gw, float* gdot, float* ggamma, int B, int G, int Fs, int H, int W, void* stream);
/* Pass 2: gs -= sum_e sum_{p: clamp(p + delta_e) = q} E_e(p) (in place); with PW also o_out. */
grr_status grr_win_bwd_gather(const float* E, const float* PW, const int32_t* delta, int K, float* gs, float* o_out,
                              int B, int G, int Fs, int H, int W, void* stream);
/* Pass 2 without the E / PW planes (pass 1 then runs with E = PW = NULL): each E_e(p) / PW_e(p) is
 * recomputed at the pixel that gathers it from s, b, w (gtv = 0: the GLR term's E; gtv = 1: the GTV
 * term's E and, with o_out, o = C^T phi(C s); prox, log_gamma, scale as in pass 1).  Same result as
 * grr_win_bwd_glr / _gtv writing the planes + grr_win_bwd_gather, without 2 Fs K floats per pixel
 * written and read back. */
grr_status grr_win_bwd_gather_fused(const float* s, const float* b, const float* w, const int32_t* delta, int K,
                                    int gtv, int prox, const float* log_gamma, const float* scale, float* gs,
                                    float* o_out, int B, int G, int Fs, int H, int W, void* stream);
/* Edge-weight reverse of grr_win_edge_weights: gw is overwritten (softmax reverse in place);
 * the [G*F] slab of gfeat and gmultiM [G,F] accumulate (the GTV and GLR graphs share features). */
grr_status grr_win_bwd_edge_weights(const float* feat, int64_t feat_bstride, const float* multiM, const float* w,
                                    float* gw, const int32_t* delta, int K, float* gfeat, int64_t gfeat_bstride,
                                    float* gmultiM, int B, int G, int F, int H, int W, void* stream);
/* Mixture reverse: gx[b,g,c] = gout[b,c] score[b,g], gscore[b,g] = sum_c gout[b,c] x[b,g,c]. */
grr_status grr_win_bwd_mix(const float* gout, const float* x, const float* score, float* gx, float* gscore, int B,
                           int G, int Fs, int H, int W, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GRR_H */
