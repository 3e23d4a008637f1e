// LayerNorm fwd/bwd and deterministic column reductions (bias grads, dgamma/dbeta).
//
// LayerNorm (flax nn.LayerNorm, eps 1e-6): one wave64 per row, the row held in registers as
// float4 chunks (16-byte loads), two-pass mean/variance in fp32, output in the GEMM operand
// dtype.  Backward fuses the residual-gradient add and writes a bf16 copy of dx for the next
// dgrad/wgrad GEMM; dgamma/dbeta go through per-block partial slabs + an ordered reduce (no
// float atomics -> bitwise reproducible).
#include "common.h"
#include <cstdlib>

namespace {

// RPW rows per wave, every row's loads issued before the first reduction (as the backward): with one
// row per wave a wave had 3 x 16 B in flight per lane and the kernel ran at ~4 TB/s
// resid (optional): the row is x + resid (the residual add of the producing layer, moved here from its
// GEMM epilogue), written to x_out (may alias x) before it is normalised.
// XB: x is bf16 (a bf16 GEMM output; the sum x + resid is fp32 in x_out, which must not alias x)
template <int NV, int RPW, bool XB = false>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const void* x, const float* __restrict__ resid, float* x_out,
                                                     const float* __restrict__ g,
                                                     const float* __restrict__ b, void* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int M, int D, float eps, int out_f32) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= M) return;
  DTC_ASSERT(D % 4 == 0 && D / 4 <= NV * 64);
  const int D4 = D / 4;
  f32x4 v[RPW][NV], gv[NV], bv[NV];
  // gamma/beta are issued with the row loads so their latency hides under the row reductions
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int row = row0 + q;
    if constexpr (XB) {
      const bf16x4* xr = (const bf16x4*)((const bf16*)x + (long)min(row, M - 1) * D);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int c = lane + 64 * i;
        if (c < D4) {
          const bf16x4 t = xr[c];
          v[q][i] = f32x4{(float)t[0], (float)t[1], (float)t[2], (float)t[3]};
        } else {
          v[q][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    } else {
      const f32x4* xr = (const f32x4*)((const float*)x + (long)min(row, M - 1) * D);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int c = lane + 64 * i;
        v[q][i] = c < D4 ? xr[c] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (resid) {
      const f32x4* rr = (const f32x4*)(resid + (long)min(row, M - 1) * D);
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int c = lane + 64 * i;
        if (c < D4) v[q][i] += rr[c];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    int c = lane + 64 * i;
    gv[i] = c < D4 ? ((const f32x4*)g)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
    bv[i] = c < D4 ? ((const f32x4*)b)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int row = row0 + q;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += v[q][i][0] + v[q][i][1] + v[q][i][2] + v[q][i][3];
    const float mean = warp_sum(s) / D;
    float qs = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int c = lane + 64 * i;
      if (c < D4) {
        f32x4 d = v[q][i] - mean;
        qs += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
      }
    }
    const float rstd = rsqrtf(warp_sum(qs) / D + eps);
    if (row >= M) continue;
    if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
    if (x_out) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int c = lane + 64 * i;
        if (c < D4) ((f32x4*)(x_out + (long)row * D))[c] = v[q][i];
      }
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int c = lane + 64 * i;
      if (c < D4) {
        f32x4 o = (v[q][i] - mean) * rstd * gv[i] + bv[i];
        if (out_f32) ((f32x4*)((float*)y + (long)row * D))[c] = o;
        else ((bf16x4*)((bf16*)y + (long)row * D))[c] = bf16x4{f2bf(o[0]), f2bf(o[1]), f2bf(o[2]), f2bf(o[3])};
      }
    }
  }
}

#ifndef DTC_LN_RPW
#define DTC_LN_RPW 2  // rows per wave in the LayerNorm backward (all loaded before the first use)
#endif
constexpr int LN_RPW = DTC_LN_RPW;
constexpr int LN_BWD_ROWS = 4 * LN_RPW;  // rows per block (4 waves): 512 blocks at M=4096 with 2 rows per wave

// LayerNorm backward, 2 rows per wave with all loads issued before the two row reductions (ILP),
// fused residual-gradient add, bf16 copy of dx, and per-block column partials of
//   slab 0: sum dy*xhat (dgamma)   slab 1: sum dy (dbeta)   slab 2: sum dx (the bias grad of the
//   layer whose OUTPUT gradient dx is: out_proj.b / fc2.b — saves a separate colsum pass)
template <int NV>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const void* __restrict__ dy, int dy_f32, const float* __restrict__ x,
                                                     const float* __restrict__ g, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* __restrict__ dres,
                                                     float* __restrict__ dx, bf16* __restrict__ dx_c,
                                                     float* __restrict__ part, int nslab, int M, int D, int iters) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int D4 = D / 4;
  f32x4 ag[NV], ab[NV], ao[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) { ag[i] = f32x4{0.f, 0.f, 0.f, 0.f}; ab[i] = ag[i]; ao[i] = ag[i]; }
  DTC_ASSERT(D % 4 == 0 && D / 4 <= NV * 64 && (long)blockIdx.x * LN_BWD_ROWS * iters < M + LN_BWD_ROWS * iters);
  f32x4 gv[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    gv[i] = c < D4 ? ((const f32x4*)g)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // iters row groups per block (one partial row per block: fewer partials for the column reduction)
  for (int it = 0; it < iters; ++it) {
  const int r0 = (blockIdx.x * iters + it) * LN_BWD_ROWS + wave * LN_RPW;
  f32x4 xh[LN_RPW][NV], d[LN_RPW][NV], rv[LN_RPW][NV];
  float s1[LN_RPW] = {}, s2[LN_RPW] = {}, rsv[LN_RPW] = {};
  // every global load of the row group (x, dy, the residual gradient) is issued before the first
  // use: the residual-gradient read used to sit after the row reductions, fully exposed
#pragma unroll
  for (int q = 0; q < LN_RPW; ++q) {
    const int row = r0 + q;
    const bool ok = row < M;
    const float mu = ok ? mean[row] : 0.f;
    rsv[q] = ok ? rstd[row] : 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      f32x4 xv = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f}, rr = {0.f, 0.f, 0.f, 0.f};
      if (ok && c < D4) {
        xv = ((const f32x4*)(x + (long)row * D))[c];
        if (dy_f32) dv = ((const f32x4*)((const float*)dy + (long)row * D))[c];
        else { bf16x4 t = ((const bf16x4*)((const bf16*)dy + (long)row * D))[c]; dv = f32x4{(float)t[0], (float)t[1], (float)t[2], (float)t[3]}; }
        if (dres) rr = ((const f32x4*)(dres + (long)row * D))[c];
      }
      xh[q][i] = (xv - mu) * rsv[q];
      d[q][i] = dv;
      rv[q][i] = rr;
    }
  }
#pragma unroll
  for (int q = 0; q < LN_RPW; ++q)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      if (c < D4) {
        f32x4 gd = d[q][i] * gv[i];
        s1[q] += gd[0] + gd[1] + gd[2] + gd[3];
        f32x4 t2 = gd * xh[q][i];
        s2[q] += t2[0] + t2[1] + t2[2] + t2[3];
        ag[i] += d[q][i] * xh[q][i];
        ab[i] += d[q][i];
      }
    }
#pragma unroll
  for (int q = 0; q < LN_RPW; ++q) {
    const int row = r0 + q;
    const float c1 = warp_sum(s1[q]) / D, c2 = warp_sum(s2[q]) / D;
    if (row >= M) continue;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = lane + 64 * i;
      if (c < D4) {
        f32x4 gd = d[q][i] * gv[i];
        f32x4 o = (gd - c1 - xh[q][i] * c2) * rsv[q];
        if (dres) o += rv[q][i];
        ((f32x4*)(dx + (long)row * D))[c] = o;
        if (dx_c) ((bf16x4*)(dx_c + (long)row * D))[c] = bf16x4{f2bf(o[0]), f2bf(o[1]), f2bf(o[2]), f2bf(o[3])};
        ao[i] += o;
      }
    }
  }
  }  // row groups
  // block reduce of the column partials over the 4 waves (fixed order); part[block][nslab][D]
  __shared__ __attribute__((aligned(16))) float red[4][3][NV * 256];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    ((f32x4*)red[wave][0])[c] = ag[i];
    ((f32x4*)red[wave][1])[c] = ab[i];
    ((f32x4*)red[wave][2])[c] = ao[i];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      if (s >= nslab) break;
      const float v = (red[0][s][c] + red[1][s][c]) + (red[2][s][c] + red[3][s][c]);
      part[((long)blockIdx.x * nslab + s) * D + c] = v;
    }
  }
}

// out (beta*out +)= sum_p part[p*C + c], c in [0, C), the C columns cut into segments of `seg`
// columns routed to o0 / o1 / o2.  Block = 32 columns x 8 partial groups (whole 128-B row segments; 16
// columns read half lines), LDS tree over the groups — deterministic order, P/8 loads per thread, 8 in
// flight.  The batched TALL reduction (reduce_tasks_kernel) uses the same scheme: both paths stay bitwise
// equal.
constexpr int SR_COLS = 32, SR_GROUPS = 256 / SR_COLS;
__global__ void __launch_bounds__(256) slab_reduce(const float* __restrict__ part, int P, int C, float* __restrict__ o0,
                                                   float* __restrict__ o1, float* __restrict__ o2, int seg, float beta) {
  const int tx = threadIdx.x % SR_COLS, ty = threadIdx.x / SR_COLS;
  const int c = blockIdx.x * SR_COLS + tx;
  DTC_ASSERT(P >= 1 && ty < SR_GROUPS && (long)blockIdx.x * SR_COLS < C);
  float s = 0.f;
  if (c < C) {
#pragma unroll 8
    for (int p = ty; p < P; p += SR_GROUPS) s += part[(long)p * C + c];
  }
  __shared__ float red[SR_GROUPS][SR_COLS];
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int gq = 0; gq < SR_GROUPS; ++gq) t += red[gq][tx];
    const int which = c / seg, col = c % seg;
    float* o = which == 0 ? o0 : (which == 1 ? o1 : o2);
    o[col] = beta != 0.f ? beta * o[col] + t : t;
  }
}

constexpr int CS_ROWS = 32;  // rows per stage-1 slab

// stage 1: part[slab][n] = sum over the slab's rows.  Block = 64 column-threads (4 columns each,
// vector loads) x 4 row groups of CS_ROWS/4 rows, LDS combine of the groups.
__global__ void __launch_bounds__(256) colsum_stage1(const void* __restrict__ dy, int is_f32, int M, int N, long ld,
                                                     float* __restrict__ part) {
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int n = (blockIdx.x * 64 + tx) * 4;
  const int r0 = blockIdx.y * CS_ROWS + ty * (CS_ROWS / 4);
  DTC_ASSERT((long)blockIdx.y * CS_ROWS < M && ld >= N && ld % 4 == 0);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    if (n + 4 <= N) {
#pragma unroll
      for (int i = 0; i < CS_ROWS / 4; ++i) {
        const int r = r0 + i;
        if (r < M) {
          if (is_f32) s += *(const f32x4*)((const float*)dy + (long)r * ld + n);
          else { bf16x4 t = *(const bf16x4*)((const bf16*)dy + (long)r * ld + n); s += f32x4{(float)t[0], (float)t[1], (float)t[2], (float)t[3]}; }
        }
      }
    } else {
      for (int i = 0; i < CS_ROWS / 4; ++i) {
        const int r = r0 + i;
        if (r < M)
          for (int j = 0; j < 4 && n + j < N; ++j)
            s[j] += is_f32 ? ((const float*)dy)[(long)r * ld + n + j] : (float)((const bf16*)dy)[(long)r * ld + n + j];
      }
    }
  }
  __shared__ f32x4 red[4][64];
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && n < N) {
    f32x4 t = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
    float* o = part + (long)blockIdx.y * N + n;
    if (n + 4 <= N) *(f32x4*)o = t;
    else for (int j = 0; j < 4 && n + j < N; ++j) o[j] = t[j];
  }
}

// One launch for a whole backward layer's deferred reductions (split-K weight-gradient slabs,
// LayerNorm dgamma/dbeta partials, bias column partials) and grad-norm partials.  Each per-op
// reduce kernel it replaces is tiny, so its cost was the ~5 us per-launch floor of a replayed
// graph node, paid ~9 times per layer.  Every output element is summed by one thread in a fixed
// partial order (p ascending), so results are bitwise reproducible and equal the per-op path.
//  WIDE  (few partials, many columns; split-K slabs): 1024 columns per block, f32x4 per thread.
//  TALL  (many partials, few columns; LN / colsum partials): 32 columns x 8 partial groups per
//        block, fixed-order LDS combine (the slab_reduce scheme).
//  SUMSQ (grad-norm chunk): part[b] = weight * sum x^2 over a grid-stride share of the range.
__global__ void __launch_bounds__(256) reduce_tasks_kernel(RedBatch batch) {
  // task of this block: binary search over the ascending blk0 (a linear scan cost up to 47 dependent scalar
  // loads of the kernel argument per block: 18 us for a launch of 48 one-block norm chunks)
  int t = 0, hi = batch.ntasks - 1;
  while (t < hi) {
    const int mid = (t + hi + 1) >> 1;
    if ((int)blockIdx.x >= batch.t[mid].blk0) t = mid;
    else hi = mid - 1;
  }
  const RedTask& T = batch.t[t];
  const int b = blockIdx.x - T.blk0;
  DTC_ASSERT(t < batch.ntasks && b >= 0 && b < T.nblk && (int)blockIdx.x < batch.nblocks);
  DTC_ASSERT(T.mode == RED_SUMSQ ? (T.part != nullptr) : (T.dst != nullptr && T.P >= 1));
  const int tid = threadIdx.x;
  if (T.mode == RED_WIDE) {
    const long c = ((long)b * 256 + tid) * 4;
    if (c >= T.C) return;
    if (c + 4 <= T.C) {
      f32x4 s = *(const f32x4*)(T.src + c);
      for (int p = 1; p < T.P; ++p) s += *(const f32x4*)(T.src + (long)p * T.pstride + c);
      f32x4* o = (f32x4*)(T.dst + c);
      if (T.beta != 0.f) s += T.beta * *o;
      *o = s;
    } else {
      for (long cc = c; cc < T.C; ++cc) {
        float s = T.src[cc];
        for (int p = 1; p < T.P; ++p) s += T.src[(long)p * T.pstride + cc];
        T.dst[cc] = T.beta != 0.f ? T.beta * T.dst[cc] + s : s;
      }
    }
  } else if (T.mode == RED_TALL) {
    const int tx = tid % SR_COLS, ty = tid / SR_COLS;
    const long c = (long)b * SR_COLS + tx;
    float s = 0.f;
    if (c < T.C) {
#pragma unroll 8
      for (int p = ty; p < T.P; p += SR_GROUPS) s += T.src[(long)p * T.pstride + c];
    }
    __shared__ float red[SR_GROUPS][SR_COLS];
    red[ty][tx] = s;
    __syncthreads();
    if (ty == 0 && c < T.C) {
      float u = 0.f;
#pragma unroll
      for (int gq = 0; gq < SR_GROUPS; ++gq) u += red[gq][tx];
      T.dst[c] = T.beta != 0.f ? T.beta * T.dst[c] + u : u;
    }
  } else {
    float acc = 0.f;
    const long n4 = T.C / 4, stride = (long)T.nblk * 256;
    const f32x4* x4 = (const f32x4*)T.src;
    long i = (long)b * 256 + tid;
    for (; i + 3 * stride < n4; i += 4 * stride) {  // 4 independent 16-B loads in flight
      f32x4 v0 = x4[i], v1 = x4[i + stride], v2 = x4[i + 2 * stride], v3 = x4[i + 3 * stride];
      f32x4 q = v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;
      acc += (q[0] + q[1]) + (q[2] + q[3]);
    }
    for (; i < n4; i += stride) { f32x4 v = x4[i] * x4[i]; acc += (v[0] + v[1]) + (v[2] + v[3]); }
    if (b == 0)
      for (long i = n4 * 4 + tid; i < T.C; i += 256) acc += T.src[i] * T.src[i];
    acc = warp_sum(acc);
    __shared__ float wred[4];
    if ((tid & 63) == 0) wred[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) T.part[b] = T.weight * ((wred[0] + wred[1]) + (wred[2] + wred[3]));
  }
}

}  // namespace

#define DTC_NV_SWITCH(NV_, ...)                                              \
  switch (NV_) {                                                             \
    case 1: { constexpr int NVC = 1; __VA_ARGS__; } break;                   \
    case 2: { constexpr int NVC = 2; __VA_ARGS__; } break;                   \
    case 3: { constexpr int NVC = 3; __VA_ARGS__; } break;                   \
    case 4: { constexpr int NVC = 4; __VA_ARGS__; } break;                   \
    case 5: case 6: { constexpr int NVC = 6; __VA_ARGS__; } break;           \
    case 7: case 8: { constexpr int NVC = 8; __VA_ARGS__; } break;           \
    default: return 2001;                                                    \
  }

extern "C" {

int dtc_add_layernorm_fwd(const float* x, const float* resid, float* x_out, const float* g, const float* b, void* y,
                          float* mean, float* rstd, int M, int D, float eps, int out_f32, hipStream_t st) {
  if (D % 4) return 2002;
  int nv = (D / 4 + 63) / 64;
  // one row per wave (two rows per wave measured neutral on GPT-2 small, round 3: removed)
  dim3 grid((M + 3) / 4);
  DTC_NV_SWITCH(nv, hipLaunchKernelGGL((ln_fwd_kernel<NVC, 1>), grid, dim3(256), 0, st, x, resid, x_out, g, b, y, mean,
                                       rstd, M, D, eps, out_f32));
  DTC_CHECK_LAUNCH();
  return 0;
}

// x_out = (fp32) d + resid with d bf16 (a bf16 out_proj / fc2 output, DTC_FWD_BF16), then LayerNorm(x_out)
int dtc_add_layernorm_fwd_bf16(const bf16* d, const float* resid, float* x_out, const float* g, const float* b,
                               void* y, float* mean, float* rstd, int M, int D, float eps, int out_f32, hipStream_t st) {
  if (D % 4) return 2002;
  DTC_HOST_CHECK(d && resid && x_out && (const void*)d != (const void*)x_out);
  int nv = (D / 4 + 63) / 64;
  dim3 grid((M + 3) / 4);
  DTC_NV_SWITCH(nv, hipLaunchKernelGGL((ln_fwd_kernel<NVC, 1, true>), grid, dim3(256), 0, st, d, resid, x_out, g, b, y,
                                       mean, rstd, M, D, eps, out_f32));
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_layernorm_fwd(const float* x, const float* g, const float* b, void* y, float* mean, float* rstd, int M, int D,
                      float eps, int out_f32, hipStream_t st) {
  return dtc_add_layernorm_fwd(x, nullptr, nullptr, g, b, y, mean, rstd, M, D, eps, out_f32, st);
}

// DTC_LN_BWD_ITER: row groups of LN_BWD_ROWS per block.  2 (512 blocks at 8192 rows): half the partial
// rows for the batched column reduction -- GPT-2 small step 11.22-11.24 vs 11.31-11.34 ms with 1,
// 11.25-11.29 with 4 (profiles/r4_ab_ln_bwd_iter.log)
static int ln_bwd_iters() {
  static const int v = [] { const char* e = getenv("DTC_LN_BWD_ITER"); return e ? std::max(1, atoi(e)) : 2; }();
  return v;
}

long dtc_layernorm_bwd_workspace_bytes(int M, int D) {
  const int rows = LN_BWD_ROWS * ln_bwd_iters();
  long blocks = (M + rows - 1) / rows;
  return blocks * 3 * D * 4;
}

int dtc_layernorm_bwd(const void* dy, int dy_f32, const float* x, const float* g, const float* mean, const float* rstd,
                      const float* dres, float* dx, bf16* dx_c, float* dg, float* db, float* dbias, int M, int D,
                      int accumulate, float* ws, long ws_bytes, int defer, hipStream_t st) {
  if (D % 4 || D > 1024) return 2002;  // dgamma/dbeta block reduce holds D <= 1024 in LDS
  const int iters = ln_bwd_iters();
  int blocks = (M + LN_BWD_ROWS * iters - 1) / (LN_BWD_ROWS * iters);
  if (ws_bytes < dtc_layernorm_bwd_workspace_bytes(M, D)) return 2003;
  int nv = (D / 4 + 63) / 64;
  const int nslab = dbias ? 3 : 2;
  DTC_NV_SWITCH(nv, hipLaunchKernelGGL(ln_bwd_kernel<NVC>, dim3(blocks), dim3(256), 0, st, dy, dy_f32, x, g, mean, rstd,
                                       dres, dx, dx_c, ws, nslab, M, D, iters));
  DTC_CHECK_LAUNCH();
  if (defer) return 0;  // partials stay in ws: [blocks][nslab][D] (a RED_TALL task per slab)
  hipLaunchKernelGGL(slab_reduce, dim3((nslab * D + SR_COLS - 1) / SR_COLS), dim3(256), 0, st, ws, blocks, nslab * D, dg, db, dbias,
                     D, accumulate ? 1.f : 0.f);
  DTC_CHECK_LAUNCH();
  return 0;
}

long dtc_colsum_workspace_bytes(int M, int N) { return (long)((M + CS_ROWS - 1) / CS_ROWS) * N * 4; }

int dtc_colsum(const void* dy, int is_f32, int M, int N, long ld, float* out, float beta, float* ws, long ws_bytes,
               int defer, hipStream_t st) {
  int P = (M + CS_ROWS - 1) / CS_ROWS;
  if (ws_bytes < dtc_colsum_workspace_bytes(M, N)) return 2004;
  if (ld % 4) return 2005;
  dim3 g1((N + 255) / 256, P);
  hipLaunchKernelGGL(colsum_stage1, g1, dim3(256), 0, st, dy, is_f32, M, N, ld, ws);
  DTC_CHECK_LAUNCH();
  if (defer) return 0;  // partials stay in ws: [P][N]
  hipLaunchKernelGGL(slab_reduce, dim3((N + SR_COLS - 1) / SR_COLS), dim3(256), 0, st, ws, P, N, out, out, out, N, beta);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_red_max_tasks() { return RED_MAX_TASKS; }
int dtc_red_task_bytes() { return (int)sizeof(RedTask); }

int dtc_reduce_tasks(const RedBatch* b, hipStream_t st) {
  if (b->ntasks <= 0) return 0;
  if (b->ntasks > RED_MAX_TASKS) return 2010;
  hipLaunchKernelGGL(reduce_tasks_kernel, dim3(b->nblocks), dim3(256), 0, st, *b);
  DTC_CHECK_LAUNCH();
  return 0;
}

// generic ordered reduction of fp32 partial slabs: out (beta*out +) sum_p part[p][c]
int dtc_slab_reduce(const float* part, int P, int C, float* out, float beta, hipStream_t st) {
  hipLaunchKernelGGL(slab_reduce, dim3((C + SR_COLS - 1) / SR_COLS), dim3(256), 0, st, part, P, C, out, out, out, C, beta);
  DTC_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
