// Shared definitions for the gfx950 (MI355X / CDNA4) kernels of this framework.
// Wave64 everywhere; MFMA operands are bf16x8 fragments; accumulators f32x4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define DTC_WAVE 64
#define DTC_LDS __attribute__((address_space(3)))

// Mirror of ops/_native.py GemmArgs (keep field order and types identical).
struct GemmArgs {
  int layout;  // 0: C = A.B^T (nt) 1: C = A.B (nn) 2: C = A^T.B (tn)
  int M, N, K;
  const void* A; long lda;
  const void* B; long ldb;
  void* C; long ldc;
  int c_f32;
  int epi;
  const float* bias;
  const void* aux; long ldaux;
  void* aux_out;
  float alpha, beta;
  const int* labels;
  int vocab_start, n_valid;
  float* part;
  float* label_out;
  void* workspace; long ws_bytes;
  int split_k;
  int defer_reduce;  // layout 2 with split-K > 1: leave the fp32 slabs in `workspace` (the caller's
                     // batched reducer sums them later) instead of launching splitk_reduce
  float* colsum;     // layout 2 (register-staged kernel): colsum[z*M + m] = sum over split z's k-range
                     // of A(k, m) — the bias gradient of the same dY, fused into its weight gradient
};

// Grouped weight gradients (csrc/gemm.hip gemm8p_group_kernel, ops/gemm.py wgrad_group): problem i is
// dW_i[M][N] (fp32, row-major) = beta*dW_i + A_i^T B_i with A_i = dY_i [K][M] and B_i = X_i [K][N] (bf16,
// contiguous rows), plus db_i[M] = beta*db_i + sum_k A_i[k][m] when cs != null.  Mirror of ops/gemm.py
// WgEntry / WgBatch (keep field order and types identical).  Passed by value as the kernel argument.
struct WgEntry {
  const bf16* A;
  const bf16* B;
  float* C;
  float* cs;
  int M, N;
  int tile0;  // first logical tile (filled by the host entry point)
  int nfast;  // tile order (host-set): 0 = M-tiles fastest, 1 = N-tiles fastest (see dtc_wgrad_group)
};
constexpr int WG_MAX = 64;
struct WgBatch {
  int n;
  int K;
  float beta;
  int ntiles;
  float* sq;  // optional [ntiles][8]: per-tile, per-wave sums of squares of the final dW (grad-norm partials)
  // tail split (host-set by dtc_wgrad_group when tail_slab is given): the last tail_tiles logical tiles run
  // as tail_split K-pieces into fp32 tile slabs [tail][split][256][256], finished by wg_tail_reduce
  // in: tail_split 0 = off, 1 = auto (CUs / tail, 2..4), >= 2 = that many pieces; tail_cap = slab floats
  int tail_tiles, tail_split;
  float* tail_slab;
  long tail_cap;
  WgEntry e[WG_MAX];
};

// Batched deferred reductions (csrc/norm_reduce.hip reduce_tasks_kernel): one launch finishes
// every split-K slab / partial-slab reduction and grad-norm partial a backward layer queued.
enum { RED_WIDE = 0, RED_TALL = 1, RED_SUMSQ = 2 };
struct RedTask {
  const float* src;  // WIDE/TALL: partial p, column c at src[p*pstride + c]; SUMSQ: data
  float* dst;        // WIDE/TALL: dst[c] = beta*dst[c] + sum_p (p ascending)
  float* part;       // SUMSQ: part[block] = weight * sum x^2 over the block's share
  long C;            // columns (SUMSQ: elements)
  long pstride;
  int P;
  int mode;
  int blk0;          // first block of this task in the launch (tasks sorted by blk0)
  int nblk;
  float beta;
  float weight;
};
constexpr int RED_MAX_TASKS = 48;  // RedBatch is a kernel argument: 8 + 48 x 64 B < 4 KB
struct RedBatch {
  int ntasks;
  int nblocks;
  RedTask t[RED_MAX_TASKS];
};

enum { EPI_STORE = 0, EPI_RESID = 1, EPI_GELU = 2, EPI_DGELU = 3, EPI_LMHEAD = 4,
       EPI_RESID_LN = 5,  // x = resid + acc + bias (fp32 C) and y = LayerNorm(x) (bf16) + row mean/rstd
       EPI_LN_BWD = 6,    // acc = dy: C = dres + LayerNorm'(dy) (fp32) + bf16 copy + dgamma/dbeta/dbias partials
       EPI_NONE = 99 /* microbench: no store */ };

// Mirror of ops/_native.py LnArgs (keep field order and types identical): a layer GEMM with the
// LayerNorm that follows it fused into the epilogue (csrc/gemm.hip dtc_gemm_ln).
struct LnArgs {
  int bwd;                  // 0: EPI_RESID_LN, 1: EPI_LN_BWD
  int M, N, K;
  const void* A; long lda;  // bf16 [M][K]
  const void* B; long ldb;  // bf16 [N][K] (the weight, or the transposed weight of an NT dgrad)
  float* C;                 // fp32 [M][N]: fwd x = resid + A.B^T + bias; bwd dx
  const float* bias;        // fwd
  const float* resid;       // fwd residual / bwd residual gradient dres (may be null in bwd)
  const float* gamma;
  const float* beta;        // fwd
  void* y;                  // bf16 [M][N]: fwd LayerNorm(x); bwd bf16 copy of dx
  float* mean;              // fwd out, bwd in
  float* rstd;              // fwd out, bwd in
  const float* x;           // bwd: the LayerNorm input
  float* part;              // bwd: column partials [M/128][nslab][N] (dgamma, dbeta[, dbias = sum dx])
  int nslab;
  float eps;
  unsigned long long* sync; // dtc_gemm_ln_sync_words(M, N) words, zero-initialised once
  const long long* step;    // device step counter: epoch = step * nsites + site + 1
  int site, nsites;
  unsigned* err;            // set when a row-statistics wait timed out (outputs are NaN then)
};

#define DTC_CHECK_LAUNCH() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)

// Bounds / invariant checks of the debug build (csrc/build.py --debug: -O1 -g -DDTC_DEBUG).  In a
// device function a failed check prints the condition and aborts the kernel (HIP device assert);
// in the release build it compiles to nothing.  DTC_HOST_CHECK validates launch arguments on the
// host (returns hipErrorInvalidValue from the entry point) in both builds where it is used.
#ifdef DTC_DEBUG
#include <cassert>
#define DTC_ASSERT(cond) assert(cond)
#else
#define DTC_ASSERT(cond) ((void)0)
#endif
#define DTC_HOST_CHECK(cond) do { if (!(cond)) return (int)hipErrorInvalidValue; } while (0)

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// gelu (tanh approximation, jax.nn.gelu(approximate=True) = flax nn.gelu default), written with
// h = (1 + tanh(x)) / 2 = 1 / (1 + exp(-2x)),  x = k0 (u + k1 u^3):
//   gelu(u) = u h,   gelu'(u) = h + u h (1 - h) 2 k0 (1 + 3 k1 u^2)
// = one v_exp_f32 + one v_rcp_f32 + ~8 VALU, no clamps (exp2 -> inf gives h = 0, -> 0 gives h = 1).
// The earlier tanh form (IEEE-rounded division: div_scale/div_fmas/div_fixup per element) made
// the fc1 epilogue ~2x longer.  |err| vs fp32 tanh ~1e-6 relative, far below bf16.
__device__ __forceinline__ float gelu_h(float u, float s /* u*u */) {
  constexpr float L2E = 1.4426950408889634f, k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float arg = u * fmaf(s, -2.f * k0 * k1 * L2E, -2.f * k0 * L2E);  // -2x log2(e)
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(arg));
}
__device__ __forceinline__ float gelu_tanh_f(float u) { return u * gelu_h(u, u * u); }
// gelu(u) and gelu'(u) sharing one exp + rcp (the fc1 epilogue stores gelu'(u) for the backward)
__device__ __forceinline__ void gelu_tanh_and_grad_f(float u, float& gv, float& dgv) {
  constexpr float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float s = u * u, h = gelu_h(u, s);
  gv = u * h;
  dgv = fmaf(u * fmaf(s, 6.f * k0 * k1, 2.f * k0), fmaf(-h, h, h), h);
}
__device__ __forceinline__ float gelu_tanh_grad_f(float u) {
  float g, d;
  gelu_tanh_and_grad_f(u, g, d);
  return d;
}

// Cross-entropy backward of 8 consecutive vocab columns v0..v0+7 of one row:
//   g = (softmax - onehot) * scale = exp2(l * log2(e) + cr) - [v == label] * scale,
//   cr = log2(scale) - lse * log2(e)  (ce_row_c, once per row): one fma + one v_exp per element.
// Columns >= n_valid (vocab padding) give 0: the lm_head forward writes -inf logits there and
// exp2(-inf) = 0, so only a chunk that straddles n_valid is masked explicitly.  Shared by the
// ce_bwd kernels and the fused lm_head dgrad (csrc/gemm.hip ce_dgrad256_kernel), so both produce
// bit-identical dlogits.
__device__ __forceinline__ float ce_row_c(float lse, float scale) {
  return __builtin_amdgcn_logf(scale) - lse * 1.4426950408889634f;  // v_log_f32 is log2
}
// fp32 logits version (the fp32 parity path's lm_head backward); the bf16 one below converts and
// calls it, so both give the same bits for the same logit values.
__device__ __forceinline__ void ce_grad8f(const float (&l)[8], int v0, float cr, int lab, int n_valid, float scale,
                                          float (&g)[8]) {
  constexpr float L2E = 1.4426950408889634f;
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = __builtin_amdgcn_exp2f(fmaf(l[e], L2E, cr));
  // the label's chunk / a chunk past n_valid: rare, so a WAVE-uniform branch around the fix-up
  // (a lane-level if gets predicated into compares + selects on every element)
  const bool fix = (unsigned)(lab - v0) < 8u || v0 + 8 > n_valid;
  if (__builtin_amdgcn_ballot_w64(fix)) {
    if (fix) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (v0 + e >= n_valid) g[e] = 0.f;
        if (v0 + e == lab) g[e] -= scale;
      }
    }
  }
}
__device__ __forceinline__ void ce_grad8(const bf16x8& l8, int v0, float cr, int lab, int n_valid, float scale,
                                         float (&g)[8]) {
  float l[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) l[e] = (float)l8[e];
  ce_grad8f(l, v0, cr, lab, n_valid, scale, g);
}

// Bijective XCD-aware remap of a linear block id (cdna_hip_programming.md §5 "XCD swizzle must
// be bijective"): blocks that the dispatcher deals to the same XCD (b % 8) get a contiguous
// range of logical tile ids, so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int NX = 8;
  if (nwg <= NX) return b;
  int q = nwg / NX, r = nwg % NX;
  int x = b % NX, i = b / NX;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}
