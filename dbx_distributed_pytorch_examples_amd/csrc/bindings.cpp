// pybind11 bindings for the HIP kernels: a thin C ABI (raw device pointers + hipStream_t as
// integers). Deliberately independent of the libtorch C++ API so the extension builds in seconds
// with hipcc and never mixes ABIs with the bundled torch; the Python side (ops/_ext.py) checks
// dtype/shape/contiguity and passes tensor.data_ptr() + the current torch stream.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

namespace py = pybind11;
#include "abi.h"

extern "C" {
int dbx_conv_igemm(int mode, int bm, int bn, const dbx::IGemmArgs* a, int pro, int stats, int accum, int epi,
                   hipStream_t st, int dma);
int dbx_conv_wgrad(int mode, int bm, int bn, const dbx::WgradArgs* a, int pro, hipStream_t st, unsigned lds_pad,
                   int dma);
int dbx_wgrad_reduce_multi_plan(const float* const*, float* const*, const long long*, const int*, const float*,
                                const int*, int, void*, int*, int*);
int dbx_wgrad_reduce_multi_run(const void*, int, int, int, hipStream_t);
int dbx_wgrad_reduce_job_bytes();
int dbx_wgrad_reduce(const float* ws, float* dw, long long n, int nsplit, float scale, int accumulate, hipStream_t st);
int dbx_wgrad_reduce_gather(const float* ws, float* dw, int OC, int R, int S, int IC, int nsplit, float scale,
                            int accumulate, hipStream_t st);
int dbx_wgrad_patch3(const dbx::WgradArgs* a, long long ws_cap, hipStream_t st, int max_wg);
int dbx_conv_dwfused(const dbx::DwFusedArgs* a, long long ws_cap, hipStream_t st, int max_cus);
int dbx_stem_bwd(dbx::StemBwdArgs* a, long long ws_cap, int fused, hipStream_t st);
int dbx_bn_finalize(const double*, int, int, float, const float*, const float*, float, float, float*, float*, float*,
                    float*, float*, float*, hipStream_t);
int dbx_bn_eval_coeff(int, const float*, const float*, float, const float*, const float*, float*, float*, hipStream_t);
int dbx_channel_stats(const bf16*, long long, int, double*, int, hipStream_t);
int dbx_bn_apply(const bf16*, const float*, const float*, const bf16*, const float*, const float*, bf16*, long long, int,
                 int, int, unsigned char*, hipStream_t, const dbx::BnFin*, const dbx::BnFin*);
int dbx_bn_bwd_reduce(const bf16*, const bf16*, const bf16*, const float*, const float*, const float*, const float*,
                      long long, int, double*, int, int, hipStream_t);
int dbx_bn_bwd_coeff(const double*, int, int, float, const float*, const float*, const float*, float*, float*, float*,
                     int, hipStream_t);
int dbx_bn_bwd_apply(const bf16*, const bf16*, const bf16*, const float*, const float*, const float*, bf16*, bf16*,
                     long long, int, int, hipStream_t, const dbx::BnFin*);
int dbx_bn_bwd_apply2(const bf16*, const bf16*, const float*, bf16*, const bf16*, const float*, bf16*, long long, int,
                      hipStream_t, const dbx::BnFin*, const dbx::BnFin*);
int dbx_maxpool_fwd(const bf16*, const float*, const float*, bf16*, unsigned char*, bf16*, int, int, int, int, int,
                    int, int, int, int, int, hipStream_t, const dbx::BnFin*);
int dbx_maxpool_bwd(const bf16*, const unsigned char*, bf16*, int, int, int, int, int, int, int, int, int, hipStream_t);
int dbx_pool_bn_bwd(const bf16*, const unsigned char*, const bf16*, const float*, const float*, const float*,
                    const float*, const float*, bf16*, double*, int, int, int, int, int, int, int, int, int, int, int,
                    hipStream_t);
int dbx_avgpool_fwd(const bf16*, bf16*, int, int, int, hipStream_t);
int dbx_avgpool_bwd(const bf16*, bf16*, int, int, int, hipStream_t);
int dbx_softmax_ce(const void*, int, const long long*, void*, float*, double*, int, int, float, float,
                   const long long*, const float*, hipStream_t);
int dbx_sgd(float*, const float*, float*, bf16*, long long, const float*, float, float, float, float, int, int,
            const float*, float, hipStream_t);
int dbx_adam(float*, const float*, float*, float*, bf16*, long long, const float*, float, float, float, float, float, int,
             float, float, const float*, float, hipStream_t);
int dbx_sumsq(const float*, long long, double*, hipStream_t);
int dbx_lars_scale(const float*, float*, const int*, const int*, const int*, int, int, double*, float, float, float,
                   hipStream_t);
int dbx_clip_factor(const double*, float, float*, hipStream_t);
int dbx_normalize_u8(const unsigned char*, bf16*, const unsigned char*, int, int, int, int, float, float, float, float,
                     float, float, hipStream_t);
int dbx_weight_prep(const float*, bf16*, const void*, int, hipStream_t);
int dbx_weight_prep16(const bf16*, bf16*, const void*, int, hipStream_t);
int dbx_augment_u8(const unsigned char*, bf16*, const float*, const unsigned char*, int, int, int, int, int, int, float,
                   float, float, float, float, float, const int*, const int*, hipStream_t);
int dbx_small_gemm(int, int, int, int, const dbx::GemmArgs*, hipStream_t);
long long dbx_mnist_saved_bytes();
int dbx_mnist_fwd(const float*, const float*, void*, float*, int, unsigned long long, unsigned, int, hipStream_t);
int dbx_mnist_bwd(const float*, const float*, const void*, const float*, float*, float*, int, unsigned long long,
                  unsigned, hipStream_t);
int dbx_colsum(const bf16*, float*, int, int, int, hipStream_t);
int dbx_dropout(const bf16*, bf16*, long long, unsigned long long, unsigned, unsigned, float, const unsigned*,
                hipStream_t);
int dbx_cast_f32_bf16(const float*, bf16*, long long, hipStream_t);
int dbx_cast_bf16_f32(const bf16*, float*, long long, float, int, hipStream_t);
}

template <typename T>
static inline T P(uintptr_t v) { return reinterpret_cast<T>(v); }
static inline hipStream_t S(uintptr_t v) { return reinterpret_cast<hipStream_t>(v); }
static void check(int rc, const char* what) {
  if (rc != 0) {
    std::string msg = std::string("dbx kernel launch failed: ") + what + " rc=" + std::to_string(rc);
    if (rc > 0) msg += std::string(" (") + hipGetErrorString((hipError_t)rc) + ")";
    throw std::runtime_error(msg);
  }
}

void register_runtime(py::module& m);  // csrc/runtime/mds_loader.cpp
void register_comm(py::module& m);     // csrc/runtime/comm.cpp

PYBIND11_MODULE(_C, m) {
  register_runtime(m);
  register_comm(m);
  m.doc() = "dbx_distributed_pytorch_examples_amd native HIP kernels (gfx950)";
  m.def("conv_igemm", [](int mode, int bm, int bn, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t in_scale,
                         uintptr_t in_shift, int relu_in, uintptr_t stats, int nshard, int N, int IH, int IW, int IC,
                         int OH, int OW, int OC, int R, int S_, int stride, int pad, int accum, int nr, int ns, int r0,
                         int s0, int tstep, int dh0, int dw0, int osub, int oph, int opw, int FH, int FW,
                         uintptr_t addsrc, int add_sub, int epi, uintptr_t mbits, uintptr_t ybn, uintptr_t ybn2,
                         uintptr_t bsc, uintptr_t bsh, uintptr_t mean1, uintptr_t inv1, uintptr_t mean2,
                         uintptr_t inv2, uintptr_t bstats1, uintptr_t bstats2, uintptr_t a_out, uintptr_t res,
                         uintptr_t res_scale, uintptr_t res_shift, uintptr_t tail_out, uintptr_t tail_bits,
                         uintptr_t st, int dma, uintptr_t fin1, uintptr_t fin2, int fin_base, int fin_final,
                         uintptr_t fin_in, int ksplit, int kper, uintptr_t skws, uintptr_t skcnt) {
    dbx::IGemmArgs a{P<const bf16*>(x), P<const bf16*>(w), P<bf16*>(y), P<const float*>(in_scale),
                     P<const float*>(in_shift), P<double*>(stats), N, IH, IW, IC, OH, OW, OC, R, S_, stride, pad,
                     N * OH * OW, nshard > 0 ? nshard : 1, relu_in, nr, ns, r0, s0, tstep, dh0, dw0, osub, oph, opw,
                     FH, FW, P<const bf16*>(addsrc), add_sub, P<const unsigned char*>(mbits), P<const bf16*>(ybn),
                     P<const bf16*>(ybn2), P<const float*>(bsc), P<const float*>(bsh), P<const float*>(mean1),
                     P<const float*>(inv1), P<const float*>(mean2), P<const float*>(inv2), P<double*>(bstats1),
                     P<double*>(bstats2), P<bf16*>(a_out), P<const bf16*>(res), P<const float*>(res_scale),
                     P<const float*>(res_shift), P<bf16*>(tail_out), P<unsigned char*>(tail_bits), 0ull, 0ull,
                     P<const dbx::BnFin*>(fin1), P<const dbx::BnFin*>(fin2), fin_base, fin_final,
                     P<const dbx::BnFin*>(fin_in), P<float*>(skws), P<unsigned*>(skcnt), ksplit > 1 ? ksplit : 1,
                     kper};
    if (fin_in && !in_scale) throw std::invalid_argument("conv_igemm: input finalize without a BN prologue");
    if ((fin1 || fin2) && !(stats || bstats1)) throw std::invalid_argument("conv_igemm: BN finalize without statistics");
    if (fin2 && !bstats2) throw std::invalid_argument("conv_igemm: second BN finalize without its statistics");
    {  // magic divisors when exact: m < N*OH*OW, so m * OH*OW < 2^40 suffices
      const unsigned long long two40 = 1ull << 40, ohw = (unsigned long long)OH * OW;
      if (ohw > 0 && (unsigned long long)N * ohw * ohw < two40) {
        a.mag_ohw = (two40 + ohw - 1) / ohw;
        a.mag_ow = (two40 + OW - 1) / OW;
      }
    }
    check(dbx_conv_igemm(mode, bm, bn, &a, in_scale != 0, stats != 0, accum, epi, S(st), dma), "conv_igemm");
  });
  m.def("wgrad_reduce_multi_plan", [](std::vector<uintptr_t> ws, std::vector<uintptr_t> dw, std::vector<long long> n,
                                       std::vector<int> nsplit, std::vector<float> scale, std::vector<int> acc,
                                       uintptr_t table) {
    const size_t nj = ws.size();
    if (dw.size() != nj || n.size() != nj || nsplit.size() != nj || scale.size() != nj || acc.size() != nj)
      throw std::invalid_argument("wgrad_reduce_multi_plan: job lists of different lengths");
    std::vector<const float*> w(nj);
    std::vector<float*> d(nj);
    for (size_t q = 0; q < nj; ++q) { w[q] = P<const float*>(ws[q]); d[q] = P<float*>(dw[q]); }
    int ga = 0, gb = 0;
    check(dbx_wgrad_reduce_multi_plan(w.data(), d.data(), n.data(), nsplit.data(), scale.data(), acc.data(), (int)nj,
                                      P<void*>(table), &ga, &gb),
          "wgrad_reduce_multi_plan");
    return std::make_pair(ga, gb);
  });
  m.def("wgrad_reduce_multi_run", [](uintptr_t table_dev, int nj, int ga, int gb, uintptr_t st) {
    check(dbx_wgrad_reduce_multi_run(P<const void*>(table_dev), nj, ga, gb, S(st)), "wgrad_reduce_multi_run");
  });
  m.def("wgrad_reduce_job_bytes", []() { return dbx_wgrad_reduce_job_bytes(); });
  m.def("conv_wgrad", [](int mode, int bm, int bn, uintptr_t dy, uintptr_t x, uintptr_t ws, uintptr_t in_scale,
                         uintptr_t in_shift, int relu_in, int N, int IH, int IW, int IC, int OH, int OW, int OC, int R,
                         int S_, int stride, int pad, int KTOT, int nsplit, int m_per_split, uintptr_t st,
                         unsigned lds_pad, int dma, uintptr_t dw, uintptr_t cnt, float scale, int accumulate) {
    const unsigned long long two40 = 1ull << 40;
    const unsigned long long ohw = (unsigned long long)OH * OW;
    if ((unsigned long long)N * ohw * ohw >= two40) throw std::runtime_error("conv_wgrad: batch too large for mdiv");
    dbx::WgradArgs a{P<const bf16*>(dy), P<const bf16*>(x), P<float*>(ws), P<const float*>(in_scale),
                     P<const float*>(in_shift), N, IH, IW, IC, OH, OW, OC, R, S_, stride, pad, N * OH * OW, KTOT,
                     nsplit, m_per_split, relu_in, (two40 + OW - 1) / OW, (two40 + ohw - 1) / ohw,
                     P<float*>(dw), P<unsigned*>(cnt), scale, accumulate};
    if (dw && nsplit > 1 && !cnt) throw std::invalid_argument("conv_wgrad: fused split-K reduction needs tile counters");
    check(dbx_conv_wgrad(mode, bm, bn, &a, in_scale != 0, S(st), lds_pad, dma), "conv_wgrad");
  });
  m.def("wgrad_patch3", [](uintptr_t dy, uintptr_t x, uintptr_t ws, long long ws_cap, int N, int IH, int IW, int IC,
                           int OH, int OW, int OC, int R, int S_, int stride, int pad, uintptr_t st, int max_wg) {
    // 3x3 patch weight gradient (conv_patch3.hip): one fp32 slab per workgroup; returns the count
    dbx::WgradArgs a{P<const bf16*>(dy), P<const bf16*>(x), P<float*>(ws), nullptr, nullptr, N, IH, IW, IC, OH, OW,
                     OC, R, S_, stride, pad, N * OH * OW, R * S_ * IC, 0, 0, 0, 0ull, 0ull};
    const int n = dbx_wgrad_patch3(&a, ws_cap, S(st), max_wg);
    if (n <= 0) check(n ? n : -1, "wgrad_patch3");
    return n;
  });
  m.def("conv_dwfused", [](uintptr_t g, uintptr_t y3, uintptr_t coeff, uintptr_t wt, uintptr_t y2, uintptr_t bsc,
                           uintptr_t bsh, uintptr_t mean2, uintptr_t inv2, uintptr_t da, uintptr_t bstats, uintptr_t ws,
                           long long ws_cap, int M, int K, int C, int nshard, uintptr_t st, int max_cus) {
    // fused bottleneck-conv3 backward (conv_dwfused.hip): returns the number of dW partial slabs
    dbx::DwFusedArgs a{P<const bf16*>(g), P<const bf16*>(y3), P<const float*>(coeff), P<const bf16*>(wt),
                       P<const bf16*>(y2), P<const float*>(bsc), P<const float*>(bsh), P<const float*>(mean2),
                       P<const float*>(inv2), P<bf16*>(da), P<double*>(bstats), P<float*>(ws), M, K, C,
                       nshard > 0 ? nshard : 1};
    const int n = dbx_conv_dwfused(&a, ws_cap, S(st), max_cus);
    if (n <= 0) check(n ? n : -1, "conv_dwfused");
    return n;
  });
  m.def("stem_bwd", [](uintptr_t dpool, uintptr_t arg, uintptr_t y, uintptr_t sc, uintptr_t sh, uintptr_t coeff,
                       uintptr_t x4, uintptr_t ws, long long ws_cap, int N, int H, int W, int C, int Pp, int Qq, int PK,
                       int pstride, int ppad, int IH, int IW, int R, int S_, int stride, int pad, int fused,
                       uintptr_t st) {
    // stem backward / stem weight gradient (stem_bwd.hip): returns the number of dW partial slabs
    const unsigned long long two40 = 1ull << 40, hw = (unsigned long long)H * W;
    if ((unsigned long long)N * hw * hw >= two40) throw std::runtime_error("stem_bwd: batch too large for mdiv");
    dbx::StemBwdArgs a{P<const bf16*>(dpool), P<const unsigned char*>(arg), P<const bf16*>(y), P<const float*>(sc),
                       P<const float*>(sh), P<const float*>(coeff), P<const bf16*>(x4), P<float*>(ws), N, H, W, C, Pp, Qq,
                       PK, pstride, ppad, IH, IW, R, S_, stride, pad, N * H * W, 0, 0, (two40 + hw - 1) / hw,
                       (two40 + W - 1) / W};
    const int n = dbx_stem_bwd(&a, ws_cap, fused, S(st));
    if (n <= 0) check(n ? n : -1, "stem_bwd");
    return n;
  });
  m.def("wgrad_reduce_gather", [](uintptr_t ws, uintptr_t dw, int OC, int R, int S_, int IC, int nsplit, float scale,
                                  int acc, uintptr_t st) {
    check(dbx_wgrad_reduce_gather(P<const float*>(ws), P<float*>(dw), OC, R, S_, IC, nsplit, scale, acc, S(st)),
          "wgrad_reduce_gather");
  });
  m.def("wgrad_reduce", [](uintptr_t ws, uintptr_t dw, long long n, int nsplit, float scale, int acc, uintptr_t st) {
    check(dbx_wgrad_reduce(P<const float*>(ws), P<float*>(dw), n, nsplit, scale, acc, S(st)), "wgrad_reduce");
  });
  m.def("bn_finalize", [](uintptr_t stats, int nshard, int C, float count, uintptr_t gamma, uintptr_t beta, float eps,
                          float momentum, uintptr_t rm, uintptr_t rv, uintptr_t scale, uintptr_t shift, uintptr_t smean,
                          uintptr_t sinv, uintptr_t st) {
    check(dbx_bn_finalize(P<const double*>(stats), nshard, C, count, P<const float*>(gamma), P<const float*>(beta), eps,
                          momentum, P<float*>(rm), P<float*>(rv), P<float*>(scale), P<float*>(shift), P<float*>(smean),
                          P<float*>(sinv), S(st)),
          "bn_finalize");
  });
  m.def("bn_eval_coeff", [](int C, uintptr_t gamma, uintptr_t beta, float eps, uintptr_t rm, uintptr_t rv,
                            uintptr_t scale, uintptr_t shift, uintptr_t st) {
    check(dbx_bn_eval_coeff(C, P<const float*>(gamma), P<const float*>(beta), eps, P<const float*>(rm),
                            P<const float*>(rv), P<float*>(scale), P<float*>(shift), S(st)),
          "bn_eval_coeff");
  });
  m.def("channel_stats", [](uintptr_t y, long long M, int C, uintptr_t stats, int nshard, uintptr_t st) {
    check(dbx_channel_stats(P<const bf16*>(y), M, C, P<double*>(stats), nshard, S(st)), "channel_stats");
  });
  m.def("bn_apply", [](uintptr_t y, uintptr_t sc, uintptr_t sh, uintptr_t res, uintptr_t rsc, uintptr_t rsh,
                       uintptr_t out, long long n, int C, int res_mode, int relu, uintptr_t mbits, uintptr_t st,
                       uintptr_t fin, uintptr_t rfin) {
    check(dbx_bn_apply(P<const bf16*>(y), P<const float*>(sc), P<const float*>(sh), P<const bf16*>(res),
                       P<const float*>(rsc), P<const float*>(rsh), P<bf16*>(out), n, C, res_mode, relu,
                       P<unsigned char*>(mbits), S(st), P<const dbx::BnFin*>(fin), P<const dbx::BnFin*>(rfin)),
          "bn_apply");
  });
  m.def("bn_bwd_reduce", [](uintptr_t dout, uintptr_t mref, uintptr_t y, uintptr_t sc, uintptr_t sh, uintptr_t mean,
                            uintptr_t invstd, long long M, int C, uintptr_t stats, int nshard, int mask_mode,
                            uintptr_t st) {
    check(dbx_bn_bwd_reduce(P<const bf16*>(dout), P<const bf16*>(mref), P<const bf16*>(y), P<const float*>(sc),
                            P<const float*>(sh), P<const float*>(mean), P<const float*>(invstd), M, C,
                            P<double*>(stats), nshard, mask_mode, S(st)),
          "bn_bwd_reduce");
  });
  m.def("bn_bwd_coeff", [](uintptr_t stats, int nshard, int C, float count, uintptr_t gamma, uintptr_t mean,
                           uintptr_t invstd, uintptr_t coeff, uintptr_t dgamma, uintptr_t dbeta, int acc, uintptr_t st) {
    check(dbx_bn_bwd_coeff(P<const double*>(stats), nshard, C, count, P<const float*>(gamma), P<const float*>(mean),
                           P<const float*>(invstd), P<float*>(coeff), P<float*>(dgamma), P<float*>(dbeta), acc, S(st)),
          "bn_bwd_coeff");
  });
  m.def("bn_bwd_apply", [](uintptr_t dout, uintptr_t mref, uintptr_t y, uintptr_t sc, uintptr_t sh, uintptr_t coeff,
                           uintptr_t dy, uintptr_t gout, long long n, int C, int mask_mode, uintptr_t st, uintptr_t fin) {
    check(dbx_bn_bwd_apply(P<const bf16*>(dout), P<const bf16*>(mref), P<const bf16*>(y), P<const float*>(sc),
                           P<const float*>(sh), P<const float*>(coeff), P<bf16*>(dy), P<bf16*>(gout), n, C, mask_mode,
                           S(st), P<const dbx::BnFin*>(fin)),
          "bn_bwd_apply");
  });
  m.def("bn_bwd_apply2", [](uintptr_t g, uintptr_t y1, uintptr_t c1, uintptr_t dy1, uintptr_t y2, uintptr_t c2,
                            uintptr_t dy2, long long n, int C, uintptr_t st, uintptr_t fin1, uintptr_t fin2) {
    check(dbx_bn_bwd_apply2(P<const bf16*>(g), P<const bf16*>(y1), P<const float*>(c1), P<bf16*>(dy1),
                            P<const bf16*>(y2), P<const float*>(c2), P<bf16*>(dy2), n, C, S(st),
                            P<const dbx::BnFin*>(fin1), P<const dbx::BnFin*>(fin2)),
          "bn_bwd_apply2");
  });
  m.def("maxpool_fwd", [](uintptr_t x, uintptr_t sc, uintptr_t sh, uintptr_t out, uintptr_t arg, uintptr_t ymax, int N,
                          int H, int W, int C, int Pp, int Q, int K, int stride, int pad, int relu, uintptr_t st,
                          uintptr_t fin) {
    check(dbx_maxpool_fwd(P<const bf16*>(x), P<const float*>(sc), P<const float*>(sh), P<bf16*>(out),
                          P<unsigned char*>(arg), P<bf16*>(ymax), N, H, W, C, Pp, Q, K, stride, pad, relu, S(st),
                          P<const dbx::BnFin*>(fin)),
          "maxpool_fwd");
  });
  m.def("maxpool_bwd", [](uintptr_t dout, uintptr_t arg, uintptr_t dx, int N, int H, int W, int C, int Pp, int Q, int K,
                          int stride, int pad, uintptr_t st) {
    check(dbx_maxpool_bwd(P<const bf16*>(dout), P<const unsigned char*>(arg), P<bf16*>(dx), N, H, W, C, Pp, Q, K,
                          stride, pad, S(st)),
          "maxpool_bwd");
  });
  m.def("pool_bn_bwd", [](uintptr_t dpool, uintptr_t arg, uintptr_t y, uintptr_t sc, uintptr_t sh, uintptr_t c1,
                          uintptr_t c2, uintptr_t c3, uintptr_t dy, uintptr_t stats, int nshard, int N, int H, int W,
                          int C, int Pp, int Q, int K, int stride, int pad, int apply, uintptr_t st) {
    check(dbx_pool_bn_bwd(P<const bf16*>(dpool), P<const unsigned char*>(arg), P<const bf16*>(y), P<const float*>(sc),
                          P<const float*>(sh), P<const float*>(c1), P<const float*>(c2), P<const float*>(c3),
                          P<bf16*>(dy), P<double*>(stats), nshard, N, H, W, C, Pp, Q, K, stride, pad, apply, S(st)),
          "pool_bn_bwd");
  });
  m.def("avgpool_fwd", [](uintptr_t x, uintptr_t out, int N, int HW, int C, uintptr_t st) {
    check(dbx_avgpool_fwd(P<const bf16*>(x), P<bf16*>(out), N, HW, C, S(st)), "avgpool_fwd");
  });
  m.def("avgpool_bwd", [](uintptr_t dout, uintptr_t dx, int N, int HW, int C, uintptr_t st) {
    check(dbx_avgpool_bwd(P<const bf16*>(dout), P<bf16*>(dx), N, HW, C, S(st)), "avgpool_bwd");
  });
  m.def("softmax_ce", [](uintptr_t logits, int is_bf16, uintptr_t labels, uintptr_t dlogits, uintptr_t loss_out,
                         uintptr_t stats, int B, int C, float smoothing, float gscale, uintptr_t labels2, uintptr_t lam,
                         uintptr_t st) {
    check(dbx_softmax_ce(P<const void*>(logits), is_bf16, P<const long long*>(labels), P<void*>(dlogits),
                         P<float*>(loss_out), P<double*>(stats), B, C, smoothing, gscale,
                         P<const long long*>(labels2), P<const float*>(lam), S(st)),
          "softmax_ce");
  });
  m.def("sgd", [](uintptr_t p, uintptr_t g, uintptr_t v, uintptr_t p16, long long n, uintptr_t hyper, float lr,
                  float mom, float damp, float wd, int nesterov, int first, uintptr_t gsp, float gs, uintptr_t st) {
    check(dbx_sgd(P<float*>(p), P<const float*>(g), P<float*>(v), P<bf16*>(p16), n, P<const float*>(hyper), lr, mom,
                  damp, wd, nesterov, first, P<const float*>(gsp), gs, S(st)),
          "sgd");
  });
  m.def("adam", [](uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, uintptr_t p16, long long n, uintptr_t hyper,
                   float lr, float b1, float b2, float eps, float wd, int decoupled, float bc1, float bc2, uintptr_t gsp,
                   float gs, uintptr_t st) {
    check(dbx_adam(P<float*>(p), P<const float*>(g), P<float*>(mm), P<float*>(v), P<bf16*>(p16), n,
                   P<const float*>(hyper), lr, b1, b2, eps, wd, decoupled, bc1, bc2, P<const float*>(gsp), gs, S(st)),
          "adam");
  });
  m.def("lars_scale", [](uintptr_t p, uintptr_t g, uintptr_t off, uintptr_t len, uintptr_t adapt, int nseg, int max_len,
                         uintptr_t norms, float gs, float eta, float wd, uintptr_t st) {
    check(dbx_lars_scale(P<const float*>(p), P<float*>(g), P<const int*>(off), P<const int*>(len),
                         P<const int*>(adapt), nseg, max_len, P<double*>(norms), gs, eta, wd, S(st)),
          "lars_scale");
  });
  m.def("sumsq", [](uintptr_t x, long long n, uintptr_t out, uintptr_t st) {
    check(dbx_sumsq(P<const float*>(x), n, P<double*>(out), S(st)), "sumsq");
  });
  m.def("clip_factor", [](uintptr_t sumsq, float max_norm, uintptr_t out, uintptr_t st) {
    check(dbx_clip_factor(P<const double*>(sumsq), max_norm, P<float*>(out), S(st)), "clip_factor");
  });
  m.def("normalize_u8", [](uintptr_t in, uintptr_t out, uintptr_t flip, int N, int H, int W, int Cin, float m0, float m1,
                           float m2, float s0, float s1, float s2, uintptr_t st) {
    check(dbx_normalize_u8(P<const unsigned char*>(in), P<bf16*>(out), P<const unsigned char*>(flip), N, H, W, Cin, m0,
                           m1, m2, s0, s1, s2, S(st)),
          "normalize_u8");
  });
  m.def("augment_u8", [](uintptr_t in, uintptr_t out, uintptr_t boxes, uintptr_t flip, int N, int Hin, int Win, int Cin,
                         int Ho, int Wo, float m0, float m1, float m2, float s0, float s1, float s2, uintptr_t perm,
                         uintptr_t mixbox, uintptr_t st) {
    check(dbx_augment_u8(P<const unsigned char*>(in), P<bf16*>(out), P<const float*>(boxes),
                         P<const unsigned char*>(flip), N, Hin, Win, Cin, Ho, Wo, m0, m1, m2, s0, s1, s2,
                         P<const int*>(perm), P<const int*>(mixbox), S(st)),
          "augment_u8");
  });
  m.def("small_gemm", [](int ta, int tb, int out_f32, int drop, uintptr_t A, uintptr_t B, uintptr_t C, uintptr_t bias_f,
                         uintptr_t bias_h, int M, int N, int K, int lda, int ldb, int ldc, float alpha, int accumulate,
                         unsigned long long seed, unsigned offset, unsigned thresh, float inv_keep, uintptr_t offset_dev,
                         uintptr_t st, uintptr_t ws, int splitk) {
    // classifier-head GEMM (head_ops.hip); splitk > 1: K split over workgroups, partials in ws
    dbx::GemmArgs g{P<const bf16*>(A), P<const bf16*>(B), P<void*>(C), P<const float*>(bias_f), P<const bf16*>(bias_h),
                    M, N, K, lda, ldb, ldc, alpha, accumulate, seed, offset, thresh, inv_keep,
                    P<const unsigned*>(offset_dev), P<float*>(ws), splitk};
    check(dbx_small_gemm(ta, tb, out_f32, drop, &g, S(st)), "small_gemm");
  }, py::arg("ta"), py::arg("tb"), py::arg("out_f32"), py::arg("drop"), py::arg("A"), py::arg("B"), py::arg("C"),
     py::arg("bias_f"), py::arg("bias_h"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("lda"), py::arg("ldb"),
     py::arg("ldc"), py::arg("alpha"), py::arg("accumulate"), py::arg("seed"), py::arg("offset"), py::arg("thresh"),
     py::arg("inv_keep"), py::arg("offset_dev"), py::arg("st"), py::arg("ws") = 0, py::arg("splitk") = 1);
  m.def("mnist_saved_bytes", []() { return dbx_mnist_saved_bytes(); });
  m.def("mnist_fwd", [](uintptr_t x, uintptr_t params, uintptr_t saved, uintptr_t logp, int N, unsigned long long seed,
                        unsigned offset, int train, uintptr_t st) {
    // fused MNIST Net forward, one workgroup per image (mnist_ops.hip)
    check(dbx_mnist_fwd(P<const float*>(x), P<const float*>(params), P<void*>(saved), P<float*>(logp), N, seed, offset,
                        train, S(st)), "mnist_fwd");
  });
  m.def("mnist_bwd", [](uintptr_t x, uintptr_t params, uintptr_t saved, uintptr_t dlogp, uintptr_t gws, uintptr_t grad,
                        int N, unsigned long long seed, unsigned offset, uintptr_t st) {
    check(dbx_mnist_bwd(P<const float*>(x), P<const float*>(params), P<const void*>(saved), P<const float*>(dlogp),
                        P<float*>(gws), P<float*>(grad), N, seed, offset, S(st)), "mnist_bwd");
  });
  m.def("colsum", [](uintptr_t X, uintptr_t out, int M, int N, int accumulate, uintptr_t st) {
    check(dbx_colsum(P<const bf16*>(X), P<float*>(out), M, N, accumulate, S(st)), "colsum");
  });
  m.def("dropout", [](uintptr_t x, uintptr_t y, long long n, unsigned long long seed, unsigned offset, unsigned thresh,
                      float inv_keep, uintptr_t offset_dev, uintptr_t st) {
    check(dbx_dropout(P<const bf16*>(x), P<bf16*>(y), n, seed, offset, thresh, inv_keep, P<const unsigned*>(offset_dev),
                      S(st)), "dropout");
  });
  m.def("weight_prep16", [](uintptr_t src, uintptr_t wbuf, uintptr_t desc, int nlayers, uintptr_t st) {
    check(dbx_weight_prep16(P<const bf16*>(src), P<bf16*>(wbuf), P<const void*>(desc), nlayers, S(st)),
          "weight_prep16");
  });
  m.def("weight_prep", [](uintptr_t master, uintptr_t wbuf, uintptr_t desc, int nlayers, uintptr_t st) {
    check(dbx_weight_prep(P<const float*>(master), P<bf16*>(wbuf), P<const void*>(desc), nlayers, S(st)),
          "weight_prep");
  });
  m.def("cast_f32_bf16", [](uintptr_t x, uintptr_t y, long long n, uintptr_t st) {
    check(dbx_cast_f32_bf16(P<const float*>(x), P<bf16*>(y), n, S(st)), "cast_f32_bf16");
  });
  m.def("cast_bf16_f32", [](uintptr_t x, uintptr_t y, long long n, float scale, int acc, uintptr_t st) {
    check(dbx_cast_bf16_f32(P<const bf16*>(x), P<float*>(y), n, scale, acc, S(st)), "cast_bf16_f32");
  });
  m.attr("arch") = "gfx950";
}
