// Host-side check of libgrr's C-ABI argument validation under AddressSanitizer + UBSan
// (built by tests/test_abi_sanitize.py with -fsanitize on the host side only; no GPU needed).
// Every entry point of include/grr.h is called with NULL operands and zero / negative sizes and
// must refuse with a grr_status error and a non-empty thread-local grr_last_error(), without
// touching memory; errors set on two threads at once must stay per-thread.
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

#include "grr.h"

static int g_fail = 0;

#define EXPECT_ERR(call)                                                                        \
  do {                                                                                          \
    grr_status st_ = (call);                                                                    \
    const char* msg_ = grr_last_error();                                                        \
    if (st_ == GRR_OK || !msg_ || !*msg_) {                                                     \
      std::fprintf(stderr, "FAIL %s: status %d msg '%s'\n", #call, (int)st_, msg_ ? msg_ : "(null)"); \
      ++g_fail;                                                                                 \
    }                                                                                           \
  } while (0)

int main() {
  const grr_stencil ns{nullptr, nullptr, nullptr, nullptr};
  float* n = nullptr;
  void* s = nullptr;
  EXPECT_ERR(grr_set_kernel_variant(7));
  EXPECT_ERR(grr_bwd_set_term_rows(5));
  EXPECT_ERR(grr_lnb_set_fused(2));
  EXPECT_ERR(grr_lnb_forward_keep(n, n, n, n, n, n, n, n, 1, 8, 16, 8, 8, s));
  EXPECT_ERR(grr_stream_copy(n, n, 3, s));
  EXPECT_ERR(grr_neighbor_table(nullptr, 0, 4, s));
  EXPECT_ERR(grr_edge_weights(n, 0, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_gtv_pair_weights(n, n, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_edge_weights_block(n, 0, 0, n, 0, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_pool2(n, n, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_system_half(n, n, n, ns, ns, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_gtv_rhs_half(n, n, ns, 0, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_gtv_rhs_full(n, n, n, ns, 0, n, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_gtv_rhs_full_rep(n, 1, n, 1, n, ns, 0, n, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_system_step(n, n, n, n, n, n, ns, ns, n, n, n, n, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_system_step2(n, n, n, n, n, n, ns, ns, n, n, n, n, ns, ns, n, n, n, n, n, n, n, n, n, n, n, 1, 1, 1,
                              8, 256, s));
  EXPECT_ERR(grr_glr_stage(n, n, n, n, ns, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_neighbor_gather(n, n, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_normalize_features(n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_stats_conv(n, ns, 0, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_glr_op_l_norm(n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_gtv_op_c(n, n, ns, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_gtv_op_c_transpose(n, n, ns, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_neighbor_gather_bwd(n, n, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_normalize_features_bwd(n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_stats_conv_bwd(n, ns, 0, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_glr_op_l_norm_bwd(n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_gtv_op_c_bwd(n, n, ns, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_gtv_op_c_transpose_bwd(n, n, ns, n, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_conv1x1(n, n, n, 1, 4, 4, 64, s));
  EXPECT_ERR(grr_conv1x1_ws(n, n, n, n, 1, 4, 4, 64, s));
  EXPECT_ERR(grr_conv2x2s2(n, n, n, 1, 4, 4, 8, 8, s));
  EXPECT_ERR(grr_lnb_forward(n, n, n, n, n, n, n, n, 1, 8, 16, 8, 8, s));
  EXPECT_ERR(grr_lnb_forward_rep(n, 3, 4, n, n, n, n, n, n, n, n, 1, 16, 8, 8, s));
  EXPECT_ERR(grr_repeat_graphs(n, n, 1, 3, 4, 64, s));
  EXPECT_ERR(grr_bwd_stencil(n, n, 0, n, 0, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_tapgrad(n, n, 0, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_padj2(n, n, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_glr(n, n, n, n, 1.f, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_pair(n, n, n, n, 1.f, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_prox(n, n, n, n, n, 1.f, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_term_fused(0, n, n, n, n, n, n, 1.f, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_term_fused_acc(0, n, n, n, n, n, n, 1.f, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_pair_weights(n, n, n, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_edge_weights(n, 0, n, n, n, n, 0, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_graph_dot(n, n, 1.f, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_lincomb(n, n, n, n, n, 0, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_cg_glue(n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_cg_glue_pool(n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_bwd_unpool2_acc(n, n, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_conv2x2s2_bwd_data(n, n, n, 1, 4, 4, 8, 8, s));
  EXPECT_ERR(grr_interleave2x2(n, n, 1, 4, 8, 8, s));
  EXPECT_ERR(grr_lnb_norm(n, n, n, n, 1, 4, 64, s));
  EXPECT_ERR(grr_lnb_norm_bwd(n, n, n, n, n, n, 1, 4, 64, s));
  EXPECT_ERR(grr_lnb_norm_bwd_skip(n, n, n, n, n, n, n, n, n, 1, 4, 64, s));
  EXPECT_ERR(grr_dwconv3(n, n, n, 1, 4, 8, 8, s));
  EXPECT_ERR(grr_dwconv3_bwd(n, n, n, n, n, 1, 4, 8, 8, s));
  EXPECT_ERR(grr_lnb_gate(n, n, n, n, 1, 4, 64, s));
  EXPECT_ERR(grr_lnb_gate_bwd_scaled(n, n, n, n, n, 1, 4, 64, s));
  EXPECT_ERR(grr_lnb_gate_dw3_bwd(n, n, n, n, n, n, n, n, 1, 4, 8, 8, s));
  EXPECT_ERR(grr_lnb_dw3_gate(n, n, n, 1, 4, 8, 8, s));
  EXPECT_ERR(grr_ffn_dw3_gate(n, n, n, 1, 4, 8, 8, s));
  EXPECT_ERR(grr_ffn_gate_dw3_bwd(n, n, n, n, n, n, n, 1, 4, 8, 8, s));
  EXPECT_ERR(grr_ffn_forward(n, n, n, n, n, n, n, n, 1, 8, 16, 8, 8, s));
  EXPECT_ERR(grr_wgrad(n, n, n, n, 1, 8, 8, 64, s));
  EXPECT_ERR(grr_system_step2_train(n, n, n, n, n, n, ns, ns, n, n, n, n, ns, ns, n, n, n, n, n, n, n, n, n, n, n,
                                    n, 1, 2, 3, 8, 256, s));
  const int32_t delta[4] = {-1, 0, 0, -1};
  EXPECT_ERR(grr_win_edge_weights(n, 0, n, delta, 2, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_solver(0, n, 0, n, n, n, n, n, n, n, n, n, n, n, delta, 2, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_mix(n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_pair_weights(n, delta, 2, n, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_bwd_stencil(n, n, 0, n, 0, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_bwd_tapgrad(n, n, 0, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_bwd_glr(n, n, n, delta, 2, n, 1.f, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_bwd_gtv(n, n, n, delta, 2, 1, n, n, 1.f, n, n, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_bwd_gather(n, n, delta, 2, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_bwd_gather_fused(n, n, n, delta, 2, 1, 0, n, n, n, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_bwd_edge_weights(n, 0, n, n, n, delta, 2, n, 0, n, 1, 1, 1, 8, 8, s));
  EXPECT_ERR(grr_win_bwd_mix(n, n, n, n, n, 1, 1, 1, 8, 8, s));
  // non-positive sizes with non-NULL (never dereferenced) pointers
  float dummy[4];
  EXPECT_ERR(grr_pool2(dummy, dummy + 1, 0, 1, 8, 8, s));
  EXPECT_ERR(grr_pool2(dummy, dummy + 1, 1, 1, 7, 8, s));   // odd size at a pooled level -> SHAPE
  EXPECT_ERR(grr_neighbor_gather(dummy, dummy, 1, 1, 8, 8, s));   // aliasing refused
  // thread-local error messages
  std::string a, b;
  std::thread t1([&] { grr_pool2(nullptr, nullptr, 1, 1, 8, 8, nullptr); a = grr_last_error(); });
  std::thread t2([&] { grr_set_kernel_variant(9); b = grr_last_error(); });
  t1.join();
  t2.join();
  if (a.find("grr_pool2") == std::string::npos || b.find("grr_set_kernel_variant") == std::string::npos) {
    std::fprintf(stderr, "FAIL thread-local errors: '%s' / '%s'\n", a.c_str(), b.c_str());
    ++g_fail;
  }
  if (grr_version() < 1) ++g_fail;
  std::printf("abi sanitize check: %d failure(s)\n", g_fail);
  return g_fail ? 1 : 0;
}
