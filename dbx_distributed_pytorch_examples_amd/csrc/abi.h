// Argument structs shared by the kernel translation units and the pybind11 bindings.
#pragma once
typedef __bf16 bf16;
namespace dbx {
// BatchNorm finalize descriptor (device-resident, one per BN and direction): what bn_finalize
// (mode 1: sharded sums -> scale / shift / saved mean, invstd / running stats) or bn_bwd_coeff
// (mode 2: -> the backward coefficients [3][C] and dgamma / dbeta) would compute, done instead by the
// last tile of the producing conv that touches each 64-channel group (bn_fin.h bn_fin_tail).
struct BnFin {
  unsigned* cnt;          // [C / 64] arrival counters (zeroed; the finalizing block resets its group's)
  const double* stats;    // [nshard][2][C]
  const float* gamma;     // nullable (1)
  const float* beta;      // nullable (0), mode 1
  float* running_mean;    // mode 1, nullable (no running-stat update)
  float* running_var;
  float* scale;           // mode 1 out
  float* shift;
  float* mean;            // mode 1: out (save_mean, nullable) ; mode 2: in
  float* invstd;          // mode 1: out (save_invstd, nullable) ; mode 2: in
  float* coeff;           // mode 2 out [3][C]
  float* dgamma;          // mode 2 out (nullable)
  float* dbeta;
  int C, nshard, mode, accumulate;
  float count, eps, momentum, pad_;
};
struct IGemmArgs {
  const bf16* x;          // A source, NHWC [N][IH][IW][IC]
  const bf16* w;          // B, [OC][KTOT] with KTOT = R*S*IC (STEM: 8*32)
  bf16* y;                // out, [M][OC]
  const float* in_scale;  // prologue affine per input channel (nullable)
  const float* in_shift;
  double* stats;          // [nshard][2][OC] (sum, sumsq) or null; fp64 so the atomics are order-independent
  int N, IH, IW, IC, OH, OW, OC, R, S, stride, pad;
  int M, nshard, relu_in;
  // tap subset iterated by the K loop: r = r0 + tstep*tr (tr < nr), s = s0 + tstep*ts (ts < ns)
  int nr, ns, r0, s0, tstep;
  // DGRAD: A gather ih = i + dh0 - tr ; output pixel (i*osub + oph, j*osub + opw) of [FH][FW]
  int dh0, dw0, osub, oph, opw, FH, FW;
  // ---- DGRAD epilogue fusions --------------------------------------------------------
  // accumulate: out = acc + addsrc[pixel / add_sub] (only at pixels with h, w % add_sub == 0);
  // addsrc == null -> the output itself
  const bf16* addsrc;
  int add_sub;
  // BN-backward epilogue (EPI 1: mask = bit of mbits, the 1-bit ReLU mask of the block output
  // written by bn_apply; EPI 2: mask = ybn*bsc + bsh > 0):
  // g = mask * out (written instead of out), bstats1 += [sum g, sum g*(ybn-mean1)*inv1],
  // bstats2 += [0, sum g*(ybn2-mean2)*inv2] (second BN fed by the same gradient, nullable)
  const unsigned char* mbits;  // [M][OC/8] bytes, bit j of byte (pix, c/8) = channel c
  const bf16* ybn;
  const bf16* ybn2;
  const float* bsc;
  const float* bsh;
  const float* mean1;
  const float* inv1;
  const float* mean2;
  const float* inv2;
  double* bstats1;  // fp64 [nshard][2][C]
  double* bstats2;
  // DGRAD with the MASK_Y epilogue (EPI 2): also store the BN output relu(ybn*bsc + bsh) it
  // computes for the mask (same shape as the output) -> the input the conv's weight gradient
  // needs, so that wgrad runs without a BN prologue (nullable)
  bf16* a_out;
  // ---- FWD "tail" prologue: the previous block's output computed on the fly ---------------
  // A = relu(x*in_scale + in_shift + r), r = res (identity shortcut) or res*res_scale + res_shift
  // (downsample branch); the first N tile also stores A to tail_out and its 1-bit ReLU mask to
  // tail_bits: the block output and mask a separate bn_apply pass would have written
  const bf16* res;
  const float* res_scale;
  const float* res_shift;
  bf16* tail_out;
  unsigned char* tail_bits;
  // magic divisors (common.h mdiv) for pixel -> (n, oh, ow): ceil(2^40 / (OH*OW)), ceil(2^40 / OW);
  // 0 = not exact for this size (plain division)
  unsigned long long mag_ohw, mag_ow;
  // in-launch BN finalize of the statistics this launch accumulates (stats: fin1; EPI: bstats1 ->
  // fin1, bstats2 -> fin2; nullable). fin_final: this is the producer's last launch, whose arrivals
  // complete the count fin_base (tiles of its earlier launches) + ceil(M / BM)
  const BnFin* fin1;
  const BnFin* fin2;
  int fin_base, fin_final;
  // consumer-side forward finalize of the INPUT's BatchNorm (PRO, forward; nullable): every
  // workgroup derives the prologue scale / shift from that BN's statistics shards itself, and
  // workgroup 0 also stores what bn_finalize would (scale, shift, saved mean / invstd, running
  // stats) -- the separate finalize launch between producer and consumer disappears. TAIL: an array
  // of two when the shortcut has a BN (res_scale set): [0] the block's last BN, [1] the shortcut's
  const BnFin* fin_in;
  // ---- split-K (implicit-GEMM kernel, non-persistent launches) ---------------------------------
  // ksplit > 1: ntile x ksplit workgroups, slice s covering K blocks [s*kper, min(KB, (s+1)*kper));
  // each stores its fp32 partial tile to skws[s][tile] and the workgroup that draws the tile's last
  // ticket from skcnt[tile] (zero; reset by that workgroup) sums the slices in slice order and runs the
  // epilogue -- the same bits whichever slice finishes last
  float* skws;
  unsigned* skcnt;
  int ksplit, kper;
};
struct WgradArgs {
  const bf16* dy;        // [M][OC]
  const bf16* x;         // NHWC input [N][IH][IW][IC] (STEM: IC = 4)
  float* ws;             // [nsplit][OC][KTOT] fp32 partials
  const float* in_scale; // prologue on X (BN-apply of previous layer) or null
  const float* in_shift;
  int N, IH, IW, IC, OH, OW, OC, R, S, stride, pad;
  int M, KTOT, nsplit, m_per_split, relu_in;
  unsigned long long mag_ow, mag_ohw;  // ceil(2^40 / OW), ceil(2^40 / (OH*OW)): pixel -> (n, oh, ow)
  // in-launch split-K reduction (conv_igemm.hip wgrad_store): dw != null -> the block that draws a
  // tile's last ticket from cnt[tile] (zeroed; reset by that block) sums the tile's nsplit slabs in
  // split order and writes dw = scale * sum (+ dw when accumulate); nsplit == 1 writes dw directly
  float* dw;
  unsigned* cnt;
  float scale;
  int accumulate;
};
// Fused backward of a bottleneck conv3 (1x1 stride-1, C -> K channels), conv_dwfused.hip
struct DwFusedArgs {
  const bf16* g;         // [M][K] gradient of the BN3 output (block-output gradient, ReLU-masked)
  const bf16* y3;        // [M][K] BN3 input (conv3 raw output)
  const float* coeff;    // [3][K] BN3-backward apply: dy3 = k1*g + k2*y3 + k3
  const bf16* wt;        // [C][K] dgrad weights (CRSK, 1x1)
  const bf16* y2;        // [M][C] BN2 input (conv2 raw output)
  const float* bsc;      // BN2 forward scale / shift: a2 = relu(y2*bsc + bsh)
  const float* bsh;
  const float* mean2;    // BN2 batch mean / invstd (backward moments)
  const float* inv2;
  bf16* da;              // [M][C] out: relu-masked data gradient of a2
  double* bstats;        // [nshard][2][C] BN2-backward moments (sum g, sum g*xhat)
  float* ws;             // [grid][K][C] fp32 weight-gradient partial slabs
  int M, K, C, nshard;
};
// Fused stem backward (max-pool backward + BN-backward apply + stem weight gradient), stem_bwd.hip
struct StemBwdArgs {
  const bf16* dpool;          // [N][P][Q][C] max-pool output gradient
  const unsigned char* arg;   // [N][P][Q][C] argmax r*PK + s within each pooling window
  const bf16* y;              // [N][H][W][C] stem conv output (the BN input)
  const float* sc;            // stem BN forward scale / shift (the ReLU mask)
  const float* sh;
  const float* coeff;         // [3][C] BN-backward apply: dy = k1*g + k2*y + k3
  const bf16* x4;             // [N][IH][IW][4] NHWC4 input image
  float* ws;                  // [nsplit][C][256] fp32 weight-gradient partial slabs (8 x 8 x 4 taps)
  int N, H, W, C, P, Q, PK, pstride, ppad;  // stem output / max-pool geometry
  int IH, IW, R, S, stride, pad;             // stem conv geometry
  int M, nsplit, m_per_split;
  unsigned long long mag_hw, mag_w;          // ceil(2^40 / (H*W)), ceil(2^40 / W)
};
// classifier-head GEMM (head_ops.hip): C[M][N] = alpha * A(m,k) B(k,n) (+ bias) (+ C), dropout on A or B
struct GemmArgs {
  const bf16* A;
  const bf16* B;
  void* C;               // fp32 or bf16 [M][ldc]
  const float* bias_f;   // [N] fp32 (nullable)
  const bf16* bias_h;    // [N] bf16 (nullable)
  int M, N, K, lda, ldb, ldc;
  float alpha;
  int accumulate;        // C += result
  unsigned long long seed;
  unsigned offset, thresh;  // dropout: keep if the Philox draw < thresh
  float inv_keep;
  const unsigned* offset_dev;  // nullable: the Philox offset read from device memory (graph replays)
  float* ws;             // split-K (splitk > 1): fp32 partials [splitk][M][N], summed in split order
  int splitk;            // K split over blockIdx.z (1: the tile loop writes C itself)
};

}  // namespace dbx
