// Causal flash attention for gfx950 (reference: model/CausalSelfAttention.py:34-44).
//
// Layout: qkv [B, T, 3, H, HD] bf16 straight out of the fused QKV GEMM (row stride 3*H*HD),
// o [B, T, H, HD] bf16 (= out_proj input), lse [B, H, T] fp32 (natural log).
//
// All products use v_mfma_f32_16x16x32_bf16 (K = 32 = the reference head_dim).  The trick
// that keeps softmax in registers (cdna_hip_programming.md §3 "accumulator tile as the next
// MFMA's operand", T10): compute the score tile TRANSPOSED so the query sits on the lane:
//     S^T[key][q] = K · Q^T   ->  lane (g, j) holds keys 4g..4g+3 of query j
// Two such 16-key tiles give exactly the 8 k-values (keys 4g+r and 16+4g+r) that the next
// MFMA's B operand needs in the same permuted k order the GEMM uses, so P never leaves
// registers; V (and Q/K/dO in backward) is read k-major from LDS with ds_read_b64_tr_b16.
//
// Backward = 3 kernels, no atomics (bitwise deterministic): delta = rowsum(dO*O); dK/dV with
// one workgroup per 64-key block sweeping the queries; dQ with one workgroup per 64-query
// block sweeping the keys.  P is recomputed from the saved LSE.
#include "common.h"
#include <vector>
#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

template <int HD>
struct AttnLds {
  // row-read image (ds_read_b128 of 8 contiguous hd): 160-B rows (40 dwords) make the 16 rows x
  // 4 lane groups of a fragment read hit 64 distinct banks (80-B rows measured 35% conflicts)
  static constexpr int KLD = 80;
  static_assert(HD <= 64, "KLD sized for head_dim <= 64");
  static constexpr int VLD = HD + 16;  // tr-read image (rows = keys/queries, cols = hd)
};

// A/B fragment from a row-major [row][ld] LDS tile: lane (g, i) gets row r0+i, cols c0+8g..+7
__device__ __forceinline__ bf16x8 row_frag(const bf16* lds, int ld, int r0, int c0, int lane) {
  return *(const bf16x8*)(lds + (r0 + (lane & 15)) * ld + c0 + 8 * (lane >> 4));
}
// transposed fragment: element j of lane (g, i) = tile[row k(j)][col c0+i] with
// k(j) = r0 + 4g + j (j<4), r0 + 16 + 4g + (j-4) (j>=4)   (the permuted k order)
__device__ __forceinline__ bf16x8 tr_frag(const bf16* lds, int ld, int r0, int c0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const bf16* p0 = lds + (r0 + 4 * g + q) * ld + c0 + 4 * p;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0 + 16 * ld));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ bf16x8 pack_p(const f32x4& a, const f32x4& b) {
  return bf16x8{f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3]), f2bf(b[0]), f2bf(b[1]), f2bf(b[2]), f2bf(b[3])};
}
__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// raw v_exp_f32 (softmax arguments are <= 0: no overflow range handling needed; the libm exp2f
// wraps every call in ldexp/compare/select denormal scaffolding)
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
// max / sum of x over the lane pair (l, l ^ 32): one v_permlane32_swap (a VALU op) instead of the
// ds_bpermute round trip + address arithmetic __shfl_xor(x, 32) compiles to
__device__ __forceinline__ float pair_max32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// stage a [rows][HD] tile (rows starting at token t0) of slot `which` (0 q, 1 k, 2 v) into LDS [rows][ld]
template <int HD, int ROWS>
__device__ __forceinline__ void stage_tile(bf16* lds, int ld, const bf16* __restrict__ base, long tok_stride, int t0,
                                           int T, int tid, int nthreads) {
  constexpr int CH = ROWS * HD / 8;
  for (int c = tid; c < CH; c += nthreads) {
    int r = c / (HD / 8), col = (c % (HD / 8)) * 8;
    int t = t0 + r;
    u32x4 v = t < T ? *(const u32x4*)(base + (long)t * tok_stride + col) : u32x4{0, 0, 0, 0};
    *(u32x4*)(lds + r * ld + col) = v;
  }
}

// Register-staged pair of [ROWS][HD] tiles (K&V, Q&dO, ...) for a 2-deep software pipeline:
// tile i+2 is loaded into registers while LDS holds tile i and registers hold tile i+1 (T14).
template <int HD, int ROWS, int NTH = 256>
struct PairStage {
  static constexpr int CH = ROWS * HD / 8;             // 16-B chunks per tile
  static constexpr int CPT = (CH + NTH - 1) / NTH;     // per thread
  u32x4 x[CPT], y[CPT];
  __device__ __forceinline__ void load(const bf16* __restrict__ bx, long sx, const bf16* __restrict__ by, long sy,
                                       int t0, int T, int tid) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + NTH * i;
      const int r = c / (HD / 8), col = (c % (HD / 8)) * 8, t = t0 + r;
      const bool ok = c < CH && t < T;
      x[i] = ok ? *(const u32x4*)(bx + (long)t * sx + col) : u32x4{0, 0, 0, 0};
      y[i] = ok ? *(const u32x4*)(by + (long)t * sy + col) : u32x4{0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void store(bf16* lx, int ldx, bf16* ly, int ldy, int tid) const {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + NTH * i;
      if (c < CH) {
        const int r = c / (HD / 8), col = (c % (HD / 8)) * 8;
        *(u32x4*)(lx + r * ldx + col) = x[i];
        *(u32x4*)(ly + r * ldy + col) = y[i];
      }
    }
  }
};

// Runs body(ldsX, ldsY, it) for it = 0..n-1 over tiles starting at token t0_of(it), with the
// tiles streamed through two LDS stages and two register stages (one barrier per tile).
template <int HD, int ROWS, int NTH = 256, typename T0, typename Body>
__device__ __forceinline__ void pipelined_tiles(int n, T0 t0_of, const bf16* bx, long sx, const bf16* by, long sy,
                                                int T, bf16* lds, int ldx, int ldy, int tid, Body body) {
  if (n <= 0) return;
  bf16* X0 = lds;
  bf16* Y0 = X0 + ROWS * ldx;
  bf16* X1 = Y0 + ROWS * ldy;
  bf16* Y1 = X1 + ROWS * ldx;
  PairStage<HD, ROWS, NTH> p0, p1;
  p0.load(bx, sx, by, sy, t0_of(0), T, tid);
  if (n > 1) p1.load(bx, sx, by, sy, t0_of(1), T, tid);
  p0.store(X0, ldx, Y0, ldy, tid);
  __syncthreads();
  for (int it = 0; it < n; it += 2) {
    if (it + 2 < n) p0.load(bx, sx, by, sy, t0_of(it + 2), T, tid);
    body(X0, Y0, it);
    if (it + 1 < n) p1.store(X1, ldx, Y1, ldy, tid);
    __syncthreads();
    if (it + 1 >= n) break;
    if (it + 3 < n) p1.load(bx, sx, by, sy, t0_of(it + 3), T, tid);
    body(X1, Y1, it + 1);
    if (it + 2 < n) p0.store(X0, ldx, Y0, ldy, tid);
    __syncthreads();
  }
}

// ============================================================================ forward
template <int HD>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ o,
                                                       float* __restrict__ lse, int B, int T, int H, float scale) {
  constexpr int KC = HD / 32;  // k-chunks of the QK^T product
  constexpr int HT = HD / 16;  // 16-wide hd tiles of the output
  using L = AttnLds<HD>;
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * 64 * (L::KLD + L::VLD)];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, j = lane & 15;
  const int nqb = (T + 63) / 64;
  const int qb = nqb - 1 - (int)(blockIdx.x % nqb);  // heavy (late) query blocks first
  const int bh = blockIdx.x / nqb, b = bh / H, h = bh % H;
  const long ts = 3L * H * HD;  // token stride
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const int q = qb * 64 + 16 * w + j;  // this lane's query row
  bf16x8 qf[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc)
    qf[kc] = q < T ? *(const bf16x8*)(Qb + (long)q * ts + kc * 32 + 8 * g) : bf16x8{};
  const float c = scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x4 acc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto body = [&](const bf16* sK, const bf16* sV, int kt) {
    f32x4 s[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      s[st] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) s[st] = mfma(row_frag(sK, L::KLD, st * 16, kc * 32, lane), qf[kc], s[st]);
    }
    float mt = -INFINITY;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = kt * 64 + st * 16 + 4 * g + r;
        float x = s[st][r] * c;
        x = (key <= q && key < T) ? x : -INFINITY;
        s[st][r] = x;
        mt = fmaxf(mt, x);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float alpha = fast_exp2(m - mn);  // m = -inf on the first tile -> 0
    m = mn;
    float ls = 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float pv = fast_exp2(s[st][r] - mn);
        s[st][r] = pv;
        ls += pv;
      }
    l = l * alpha + ls;
#pragma unroll
    for (int t = 0; t < HT; ++t) acc[t] *= alpha;
    bf16x8 pf0 = pack_p(s[0], s[1]), pf1 = pack_p(s[2], s[3]);
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      acc[t] = mfma(tr_frag(sV, L::VLD, 0, t * 16, lane), pf0, acc[t]);
      acc[t] = mfma(tr_frag(sV, L::VLD, 32, t * 16, lane), pf1, acc[t]);
    }
  };
  pipelined_tiles<HD, 64>(qb + 1, [](int it) { return it * 64; }, Kb, ts, Vb, ts, T, lds, L::KLD, L::VLD, tid, body);
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (q < T) {
    const float inv = 1.f / l;
    bf16* orow = o + ((long)b * T + q) * H * HD + h * HD;
#pragma unroll
    for (int t = 0; t < HT; ++t)
      *(bf16x4*)(orow + t * 16 + 4 * g) =
          bf16x4{f2bf(acc[t][0] * inv), f2bf(acc[t][1] * inv), f2bf(acc[t][2] * inv), f2bf(acc[t][3] * inv)};
    if (g == 0) lse[((long)b * H + h) * T + q] = (m + __log2f(l)) * LN2;
  }
}

// ============================================================================ backward
// delta[b,h,t] = sum_d dO*O.  HD/8 lanes per row, 16 B of O and dO each (a wave reads whole 128-B row
// lines, coalesced), rows in (b, h, t) order so the delta stores are contiguous; the partial dot
// products meet by lane shuffles.  (One thread per row striding 128 B per lane: 10.7 us at GPT-2 small.)
template <int HD>
__global__ void __launch_bounds__(256) attn_delta_kernel(const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                                         float* __restrict__ delta, int B, int T, int H) {
  constexpr int LPR = HD / 8;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long i = gid / LPR;  // (b, h, t) row
  const int part = (int)(gid % LPR);
  const bool ok = i < (long)B * T * H;
  float s = 0.f;
  if (ok) {
    const int t = (int)(i % T);
    const long bh = i / T;
    const int h = (int)(bh % H), b = (int)(bh / H);
    DTC_ASSERT(b < B && h < H && part < LPR);
    const long off = (((long)b * T + t) * H + h) * HD + part * 8;
    const bf16x8 a = *(const bf16x8*)(o + off), c = *(const bf16x8*)(dout + off);
#pragma unroll
    for (int r = 0; r < 8; ++r) s += (float)a[r] * (float)c[r];
  }
#pragma unroll
  for (int w = LPR / 2; w >= 1; w >>= 1) s += __shfl_xor(s, w, 64);
  if (ok && part == 0) delta[i] = s;
}

template <int HD>
static void launch_attn_delta(const bf16* o, const bf16* dout, float* delta, int B, int T, int H, hipStream_t st) {
  const long threads = (long)B * T * H * (HD / 8);
  hipLaunchKernelGGL(attn_delta_kernel<HD>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, o, dout, delta,
                     B, T, H);
}

// dK, dV: workgroup = (b, h, 64-key block); wave w owns keys kb*64+16w..+15 (key on the lane).
template <int HD>
__global__ void __launch_bounds__(256) attn_bwd_dkdv_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                            const float* __restrict__ lse, const float* __restrict__ delta,
                                                            bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  constexpr int KC = HD / 32, HT = HD / 16;
  using L = AttnLds<HD>;
  __shared__ __attribute__((aligned(16))) bf16 lds[4 * 64 * L::VLD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, j = lane & 15;
  const int nkb = (T + 63) / 64;
  const int kb = (int)(blockIdx.x % nkb);  // kb 0 (sweeps all queries, heaviest) launches first
  const int bh = blockIdx.x / nkb, b = bh / H, h = bh % H;
  const long ts = 3L * H * HD, dts = (long)H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const bf16* dOb = dout + (long)b * T * dts + h * HD;
  const float* lseb = lse + ((long)b * H + h) * T;
  const float* delb = delta + ((long)b * H + h) * T;
  const int key = kb * 64 + 16 * w + j;
  bf16x8 kf[KC], vf[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    kf[kc] = key < T ? *(const bf16x8*)(Kb + (long)key * ts + kc * 32 + 8 * g) : bf16x8{};
    vf[kc] = key < T ? *(const bf16x8*)(Vb + (long)key * ts + kc * 32 + 8 * g) : bf16x8{};
  }
  const float c = scale * LOG2E;
  f32x4 dk[HT], dv[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) { dk[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[t] = dk[t]; }

  auto body = [&](const bf16* sQ, const bf16* sD, int it) {
    const int q0 = kb * 64 + 64 * it;  // 64 queries per pipeline step (4 MFMA row tiles)
    f32x4 p[4], ds[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        s = mfma(row_frag(sQ, L::VLD, qt * 16, kc * 32, lane), kf[kc], s);    // S[q][key]
        dp = mfma(row_frag(sD, L::VLD, qt * 16, kc * 32, lane), vf[kc], dp);  // dP[q][key]
      }
      const int qr = q0 + qt * 16 + 4 * g;  // rows of this lane's 4 registers
      f32x4 l4 = {0.f, 0.f, 0.f, 0.f}, d4 = {0.f, 0.f, 0.f, 0.f};
      if (qr + 4 <= T) { l4 = *(const f32x4*)(lseb + qr); d4 = *(const f32x4*)(delb + qr); }
      else for (int r = 0; r < 4; ++r) if (qr + r < T) { l4[r] = lseb[qr + r]; d4[r] = delb[qr + r]; }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = qr + r;
        float pv = (key <= qq && qq < T && key < T) ? fast_exp2(s[r] * c - l4[r] * LOG2E) : 0.f;
        p[qt][r] = pv;
        ds[qt][r] = pv * (dp[r] - d4[r]);
      }
    }
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {  // two 32-query k-chunks of the dV / dK products
      const bf16x8 pb = pack_p(p[2 * hq], p[2 * hq + 1]), dsb = pack_p(ds[2 * hq], ds[2 * hq + 1]);
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        dv[t] = mfma(tr_frag(sD, L::VLD, 32 * hq, t * 16, lane), pb, dv[t]);   // dV^T[hd][key] += dO^T P
        dk[t] = mfma(tr_frag(sQ, L::VLD, 32 * hq, t * 16, lane), dsb, dk[t]);  // dK^T[hd][key] += Q^T dS
      }
    }
  };
  const int nq = (T - kb * 64 + 63) / 64;
  pipelined_tiles<HD, 64>(nq, [kb](int it) { return kb * 64 + 64 * it; }, Qb, ts, dOb, dts, T, lds, L::VLD, L::VLD,
                          tid, body);
  if (key < T) {
    bf16* pk = dqkv + ((long)b * T + key) * ts + (1 * H + h) * HD;
    bf16* pv = dqkv + ((long)b * T + key) * ts + (2 * H + h) * HD;
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      *(bf16x4*)(pk + t * 16 + 4 * g) = bf16x4{f2bf(dk[t][0] * scale), f2bf(dk[t][1] * scale), f2bf(dk[t][2] * scale),
                                               f2bf(dk[t][3] * scale)};
      *(bf16x4*)(pv + t * 16 + 4 * g) = bf16x4{f2bf(dv[t][0]), f2bf(dv[t][1]), f2bf(dv[t][2]), f2bf(dv[t][3])};
    }
  }
}

// dQ: workgroup = (b, h, 64-query block); wave w owns queries qb*64+16w..+15 (query on the lane).
template <int HD>
__global__ void __launch_bounds__(256) attn_bwd_dq_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                          const float* __restrict__ lse, const float* __restrict__ delta,
                                                          bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  constexpr int KC = HD / 32, HT = HD / 16;
  using L = AttnLds<HD>;
  __shared__ __attribute__((aligned(16))) bf16 lds[4 * 64 * L::VLD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, j = lane & 15;
  const int nqb = (T + 63) / 64;
  const int qb = nqb - 1 - (int)(blockIdx.x % nqb);
  const int bh = blockIdx.x / nqb, b = bh / H, h = bh % H;
  const long ts = 3L * H * HD, dts = (long)H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const bf16* dOb = dout + (long)b * T * dts + h * HD;
  const int q = qb * 64 + 16 * w + j;
  bf16x8 qf[KC], df[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    qf[kc] = q < T ? *(const bf16x8*)(Qb + (long)q * ts + kc * 32 + 8 * g) : bf16x8{};
    df[kc] = q < T ? *(const bf16x8*)(dOb + (long)q * dts + kc * 32 + 8 * g) : bf16x8{};
  }
  const float lq = q < T ? lse[((long)b * H + h) * T + q] * LOG2E : 0.f;
  const float dq_ = q < T ? delta[((long)b * H + h) * T + q] : 0.f;
  const float c = scale * LOG2E;
  f32x4 acc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kend = min(T, qb * 64 + 64);
  auto body = [&](const bf16* sK, const bf16* sV, int it) {
    const int k0 = 64 * it;  // 64 keys per pipeline step
    f32x4 ds[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        s = mfma(row_frag(sK, L::VLD, kt * 16, kc * 32, lane), qf[kc], s);   // S^T[key][q]
        dp = mfma(row_frag(sV, L::VLD, kt * 16, kc * 32, lane), df[kc], dp); // dP^T[key][q]
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = k0 + kt * 16 + 4 * g + r;
        float pv = (kk <= q && kk < T && q < T) ? fast_exp2(s[r] * c - lq) : 0.f;
        ds[kt][r] = pv * (dp[r] - dq_);
      }
    }
#pragma unroll
    for (int hk = 0; hk < 2; ++hk) {
      const bf16x8 dsb = pack_p(ds[2 * hk], ds[2 * hk + 1]);
#pragma unroll
      for (int t = 0; t < HT; ++t) acc[t] = mfma(tr_frag(sK, L::VLD, 32 * hk, t * 16, lane), dsb, acc[t]);  // dQ^T += K^T dS^T
    }
  };
  pipelined_tiles<HD, 64>((kend + 63) / 64, [](int it) { return 64 * it; }, Kb, ts, Vb, ts, T, lds, L::VLD, L::VLD,
                          tid, body);
  if (q < T) {
    bf16* pq = dqkv + ((long)b * T + q) * ts + (0 * H + h) * HD;
#pragma unroll
    for (int t = 0; t < HT; ++t)
      *(bf16x4*)(pq + t * 16 + 4 * g) = bf16x4{f2bf(acc[t][0] * scale), f2bf(acc[t][1] * scale),
                                               f2bf(acc[t][2] * scale), f2bf(acc[t][3] * scale)};
  }
}


// ============================================================================ resident variants
// For short sequences (T * (hd row + tr image) fits LDS: the reference T = 512, hd = 32) the whole
// (b, h) K/V (forward, dQ) or Q/dO (dK/dV) panel is loaded into LDS ONCE, then every wave walks
// its own 16-row group against it with no further barriers: the tiled kernels above pay a
// global-load + barrier round trip per 64-key tile and are latency-bound on the long causal rows
// (23 us fwd / 60 us bwd at the reference shape).  Two 1024-thread blocks per (b, h), wave w of
// block s owning 16-row group 2w+s, so causal work is balanced across the pair and each SIMD
// interleaves 4 waves.
constexpr int RES_THREADS = 1024;
constexpr int RES_MAXT = 512;  // 16 waves x 2 blocks x 16 rows

// max / sum over the 4 lane groups (lanes j, j+16, j+32, j+48) with the gfx950 row swaps instead
// of ds_bpermute round trips through LDS
__device__ __forceinline__ float group_max(float x) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float group_sum(float x) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Block -> ((b, h), half) for the resident kernels.  Both halves of a (b, h) stage the SAME panels;
// blocks are dealt round-robin over the 8 XCDs (b and b + 8 share one), so the two halves are placed
// 8 ids apart: the second one's panel loads hit the XCD's L2 instead of HBM (staging was ~5-6 us of
// each phase, HBM-bound with every CU staging at once).  Needs B*H % 8 == 0, else the plain map.
#ifndef DTC_ATTN_XCD_PAIR
#define DTC_ATTN_XCD_PAIR 1
#endif
__device__ __forceinline__ void res_block_map(int bid, int nbh, int& half, int& bh) {
  if (DTC_ATTN_XCD_PAIR && nbh % 8 == 0) {
    half = (bid >> 3) & 1;
    bh = ((bid >> 4) << 3) | (bid & 7);
  } else {
    half = bid & 1;
    bh = bid >> 1;
  }
}

// whole-sequence [T][HD] panel -> LDS [T][LD]: every load of the thread in flight before any store
template <int LD, int HD, int MAXT>
__device__ __forceinline__ void stage_rows(bf16* lds, const bf16* __restrict__ base, long tok_stride, int T, int Tp,
                                           int tid) {
  constexpr int CPR = HD / 8, PER = (MAXT * CPR + RES_THREADS - 1) / RES_THREADS;
  u32x4 v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = tid + i * RES_THREADS, r = c / CPR, col = (c % CPR) * 8;
    v[i] = r < T ? *(const u32x4*)(base + (long)r * tok_stride + col) : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = tid + i * RES_THREADS, r = c / CPR, col = (c % CPR) * 8;
    if (r < Tp) *(u32x4*)(lds + r * LD + col) = v[i];  // rows T..Tp-1 zero-filled
  }
}

template <int HD>
__global__ void __launch_bounds__(RES_THREADS) attn_fwd_res_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ o,
                                                                  float* __restrict__ lse, int B, int T, int H,
                                                                  float scale, int zig) {
  constexpr int KC = HD / 32, HT = HD / 16;
  using L = AttnLds<HD>;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop bounds
  int half, bh;
  res_block_map(blockIdx.x, B * H, half, bh);
  const int b = bh / H, h = bh % H;
  const int Tp = (T + 63) / 64 * 64;
  bf16* sK = lds;
  bf16* sV = lds + Tp * L::KLD;
  const long ts = 3L * H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  stage_rows<L::KLD, HD, RES_MAXT>(sK, Kb, ts, T, Tp, tid);  // rows >= T are zero-filled
  stage_rows<L::VLD, HD, RES_MAXT>(sV, Vb, ts, T, Tp, tid);
  __syncthreads();
  // zig: waves w..w+3 of every other row of four take their query groups in reverse, so the four
  // waves sharing a SIMD (w, w+4, w+8, w+12) carry 18 causal tiles each instead of 16 / 20
  const int wk = (zig && (w & 4)) ? (w | 3) - (w & 3) : w;
  const int qg = 2 * wk + half;
  if (qg * 16 >= T) return;  // no barrier below
  const int q = qg * 16 + j;
  bf16x8 qf[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) qf[kc] = q < T ? *(const bf16x8*)(Qb + (long)q * ts + kc * 32 + 8 * g) : bf16x8{};
  const float c = scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x4 acc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntile = (qg * 16 + 16 + 63) / 64;
  for (int kt = 0; kt < ntile; ++kt) {
    const bf16* tK = sK + kt * 64 * L::KLD;
    const bf16* tV = sV + kt * 64 * L::VLD;
    const bool diag = kt == ntile - 1;  // only the last tile reaches past the query
    f32x4 sc[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      sc[st] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) sc[st] = mfma(row_frag(tK, L::KLD, st * 16, kc * 32, lane), qf[kc], sc[st]);
    }
    float mt = -INFINITY;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = sc[st][r] * c;
        if (diag) {
          const int key = kt * 64 + st * 16 + 4 * g + r;
          x = (key <= q && key < T) ? x : -INFINITY;
        }
        sc[st][r] = x;
        mt = fmaxf(mt, x);
      }
    mt = group_max(mt);
    const float mn = fmaxf(m, mt);
    const float alpha = fast_exp2(m - mn);
    m = mn;
    float ls = 0.f;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = fast_exp2(sc[st][r] - mn);
        sc[st][r] = pv;
        ls += pv;
      }
    l = l * alpha + ls;
#pragma unroll
    for (int t = 0; t < HT; ++t) acc[t] *= alpha;
    const bf16x8 pf0 = pack_p(sc[0], sc[1]), pf1 = pack_p(sc[2], sc[3]);
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      acc[t] = mfma(tr_frag(tV, L::VLD, 0, t * 16, lane), pf0, acc[t]);
      acc[t] = mfma(tr_frag(tV, L::VLD, 32, t * 16, lane), pf1, acc[t]);
    }
  }
  l = group_sum(l);
  if (q < T) {
    const float inv = 1.f / l;
    bf16* orow = o + ((long)b * T + q) * H * HD + h * HD;
#pragma unroll
    for (int t = 0; t < HT; ++t)
      *(bf16x4*)(orow + t * 16 + 4 * g) =
          bf16x4{f2bf(acc[t][0] * inv), f2bf(acc[t][1] * inv), f2bf(acc[t][2] * inv), f2bf(acc[t][3] * inv)};
    if (g == 0) lse[((long)b * H + h) * T + q] = (m + __log2f(l)) * LN2;
  }
}

// Chunked forward for sequences the resident kernel cannot hold (T > RES_MAXT, or head_dim 64:
// GPT-2 medium is T 1024 / hd 64).  A 1024-thread block (16 waves x 16 query rows = 256 queries of
// one (b, h)) streams K/V in 128-key chunks through a 2-stage LDS + 2-stage register pipeline:
// one barrier per 128 keys shared by 16 waves (the 256-thread tiled kernel pays a barrier and a
// K/V load per 64 keys per 4 waves, and was latency-bound at ~25 TF/s).  Each wave skips the
// 64-key tiles past its rows and masks only the tiles that cross its diagonal.
constexpr int CH_THREADS = 1024, CH_KEYS = 128, CH_QROWS = 256;
template <int HD>
__host__ __device__ constexpr int ch_lds_fwd() { return 2 * CH_KEYS * (AttnLds<HD>::KLD + AttnLds<HD>::VLD) * 2; }

template <int HD>
__global__ void __launch_bounds__(CH_THREADS) attn_fwd_chunk_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ o,
                                                                   float* __restrict__ lse, int B, int T, int H,
                                                                   float scale) {
  constexpr int KC = HD / 32, HT = HD / 16;
  using L = AttnLds<HD>;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // heavy (late) query blocks first ACROSS the grid: at ~2 blocks per CU a per-(b, h) order leaves
  // CUs with two heavy blocks (1.6x the mean work); grid-wide LPT pairs each heavy block with a
  // light one on the same CU
  const int nqb = (T + CH_QROWS - 1) / CH_QROWS, nbh = B * H;
  const int qblk = nqb - 1 - (int)(blockIdx.x / nbh);
  const int bh = blockIdx.x % nbh, b = bh / H, h = bh % H;
  const long ts = 3L * H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const int qbase = qblk * CH_QROWS + 16 * w;  // this wave's rows qbase .. qbase + 15
  DTC_ASSERT(qblk >= 0 && b < B && qbase < T + CH_QROWS);
  const int q = qbase + j;
  bf16x8 qf[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) qf[kc] = q < T ? *(const bf16x8*)(Qb + (long)q * ts + kc * 32 + 8 * g) : bf16x8{};
  const float c = scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x4 acc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto body = [&](const bf16* sK, const bf16* sV, int it) {
#pragma unroll
    for (int t2 = 0; t2 < CH_KEYS / 64; ++t2) {
      const int kb = it * CH_KEYS + t2 * 64;
      if (kb > qbase + 15 || qbase >= T) continue;  // wave-uniform: tile entirely past this wave's rows
      const bool diag = kb + 63 > qbase;            // crosses the diagonal (or the sequence end)
      const bf16* tK = sK + t2 * 64 * L::KLD;
      const bf16* tV = sV + t2 * 64 * L::VLD;
      f32x4 sc[4];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        sc[st] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) sc[st] = mfma(row_frag(tK, L::KLD, st * 16, kc * 32, lane), qf[kc], sc[st]);
      }
      float mt = -INFINITY;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = sc[st][r];
          if (diag) {
            const int key = kb + st * 16 + 4 * g + r;
            x = (key <= q && key < T) ? x : -INFINITY;
          }
          sc[st][r] = x;
          mt = fmaxf(mt, x);
        }
      mt = group_max(mt) * c;
      const float mn = fmaxf(m, mt);
      const float alpha = fast_exp2(m - mn);
      m = mn;
      float ls = 0.f;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = fast_exp2(fmaf(sc[st][r], c, -mn));
          sc[st][r] = pv;
          ls += pv;
        }
      l = l * alpha + ls;
#pragma unroll
      for (int t = 0; t < HT; ++t) acc[t] *= alpha;
      const bf16x8 pf0 = pack_p(sc[0], sc[1]), pf1 = pack_p(sc[2], sc[3]);
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        acc[t] = mfma(tr_frag(tV, L::VLD, 0, t * 16, lane), pf0, acc[t]);
        acc[t] = mfma(tr_frag(tV, L::VLD, 32, t * 16, lane), pf1, acc[t]);
      }
    }
  };
  const int nch = (min(T, qblk * CH_QROWS + CH_QROWS) + CH_KEYS - 1) / CH_KEYS;
  pipelined_tiles<HD, CH_KEYS, CH_THREADS>(nch, [](int it) { return it * CH_KEYS; }, Kb, ts, Vb, ts, T, lds, L::KLD,
                                           L::VLD, tid, body);
  l = group_sum(l);
  if (q < T) {
    const float inv = 1.f / l;
    bf16* orow = o + ((long)b * T + q) * H * HD + h * HD;
#pragma unroll
    for (int t = 0; t < HT; ++t)
      *(bf16x4*)(orow + t * 16 + 4 * g) =
          bf16x4{f2bf(acc[t][0] * inv), f2bf(acc[t][1] * inv), f2bf(acc[t][2] * inv), f2bf(acc[t][3] * inv)};
    if (g == 0) lse[((long)b * H + h) * T + q] = (m + __log2f(l)) * LN2;
  }
}

// ============================================================================ forward, 32 queries per wave
// v_mfma_f32_32x32x16_bf16 with the score tile computed TRANSPOSED (S^T = K Q^T: 32 keys x 32 queries,
// query on the lane) so softmax is lane-local: lane (r, h) holds 16 keys {(i&3) + 8(i>>2) + 4h} of
// query r per 32-key block, and its partner lane r + 32 the other 16 (one shfl_xor 32 per max).  The
// accumulator is directly the B operand of PV (O^T = V^T P^T: registers 8s..8s+7 = the k-step s
// fragment, keys in the permuted order 16s + 8(j>>2) + 4h + (j&3), cdna_hip_programming.md §3), so P
// never leaves registers; V^T fragments come from a row-major [key][hd] LDS image by
// ds_read_b64_tr_b16.  Per 64-key tile a wave does 16 MFMAs of 32 cycles and reads 8 K fragments + 16
// transposed V halves (2x the queries per K/V byte of the 16-row kernel above, which was LDS-bound at
// 16 rows per wave); the softmax VALU fills the MFMAs' issue gaps across the 3 waves per SIMD.
// Max tracking is deferred (T13): the running max m moves only when a tile's max exceeds it by
// FW_THR (log2 units), so the O / l rescale runs on a few early tiles instead of on every tile; P
// stays <= 2^FW_THR (exact in bf16 range, fp32 sums).  Block = 4 waves = 128 queries of one (b, h);
// K/V stream through 2 LDS + 2 register stages (pipelined_tiles), one barrier per 64 keys; heavy
// (late) query blocks first across the grid.
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
constexpr int FW_THREADS = 256, FW_QROWS = 128, FW_KEYS = 64;
constexpr float FW_THR = 8.f;
template <int HD>
struct FwLds {
  // K image [key][KLD]: ds_read_b128 rows r = lane & 31 at a fixed 16-B chunk; row strides of 36 / 20
  // dwords put the 16 rows of every 16-lane read group on distinct 4-bank windows.  V image [key][VLD]:
  // ds_read_b64_tr_b16 reads 4 rows x 32 lanes; a row stride = 16 (mod 64) dwords makes them disjoint.
  static constexpr int KLD = HD + 8;
  static constexpr int VLD = HD == 32 ? 32 : 96;
  static constexpr int STAGE = FW_KEYS * (KLD + VLD);
};
template <int HD>
__host__ __device__ constexpr int fw_lds_bytes() { return 2 * FwLds<HD>::STAGE * 2; }

// A fragment of V^T (32 hd rows x 16 keys, permuted k order) from the [key][VLD] image: keys
// k0 + 4h + (0..3) and k0 + 8 + 4h + (0..3) of hd column c0 + (lane & 31)
__device__ __forceinline__ bf16x8 vt_frag32(const bf16* sv, int vld, int k0, int c0, int lane) {
  const int G = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
  const bf16* p0 = sv + (k0 + 4 * (G >> 1) + qq) * vld + c0 + 16 * (G & 1) + 4 * p;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0 + 8 * vld));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = f2bf(x[8 * s + e]);
  return r;
}

// One register stage of a [64 rows][HD] tile pair (K & V, Q & dO, ...) read through buffer resources
// (32-bit offsets from a per-(b, h) base: no 64-bit address registers per load), rows >= T read as 0 by
// the hardware range check.  The pipelines below keep ONE register set: tile t+1 is loaded before tile
// t's compute and written to the other LDS buffer after it (T14), one barrier per tile.
template <int HD, int NTH>
struct RegStage {
  static constexpr int CPT = 64 * HD / 8 / NTH;  // 16-B chunks per thread per operand
  u32x4 x[CPT], y[CPT];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rx, long sx, __amdgpu_buffer_rsrc_t ry, long sy, int t0,
                                       int tid) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + NTH * i, r = c / (HD / 8), col = (c % (HD / 8)) * 8;
      x[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(((long)(t0 + r) * sx + col) * 2), 0, 0));
      y[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ry, (int)(((long)(t0 + r) * sy + col) * 2), 0, 0));
    }
  }
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const bf16* base, long stride, int T, int width) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(((long)(T - 1) * stride + width) * 2), 0x00020000);
}

template <int HD>
__global__ void __launch_bounds__(FW_THREADS, 2) attn_fwd32_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ o,
                                                              float* __restrict__ lse, int B, int T, int H,
                                                              float scale) {
  constexpr int HC = HD / 16, HB = HD / 32;
  using L = FwLds<HD>;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nqb = (T + FW_QROWS - 1) / FW_QROWS, nbh = B * H;
  const int qblk = nqb - 1 - (int)(blockIdx.x / nbh);
  const int bh = blockIdx.x % nbh, b = bh / H, h = bh % H;
  DTC_ASSERT(qblk >= 0 && b < B && h < H);
  const long ts = 3L * H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const __amdgpu_buffer_rsrc_t rK = rows_rsrc(qkv + (long)b * T * ts + (1 * H + h) * HD, ts, T, HD);
  const __amdgpu_buffer_rsrc_t rV = rows_rsrc(qkv + (long)b * T * ts + (2 * H + h) * HD, ts, T, HD);
  const int q0 = qblk * FW_QROWS + 32 * w;  // this wave's queries q0 .. q0 + 31
  const int q = q0 + r;
  bf16x8 qf[HC];  // B operand of S^T = K Q^T: lane (r, h) holds Q[q][16c + 8h .. +7]
#pragma unroll
  for (int c = 0; c < HC; ++c) qf[c] = q < T ? *(const bf16x8*)(Qb + (long)q * ts + 16 * c + 8 * hh) : bf16x8{};
  const float cs = scale * LOG2E;
  float m = -1e30f, l = 0.f;  // m: running max of s * cs (finite start: masked scores give exp2(-inf) = 0)
  f32x16 acc[HB];
#pragma unroll
  for (int i = 0; i < HB; ++i) acc[i] = f32x16{};
  const int qlim = min(q, T - 1);  // last key this lane's query may see

  // one 64-key tile; MASK: the tile crosses this wave's diagonal (or the sequence end)
  auto tile = [&](const bf16* sK, const bf16* sV, int kb, auto MASK) {
    f32x16 sc[2];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      sc[k2] = f32x16{};
#pragma unroll
      for (int c = 0; c < HC; ++c)
        sc[k2] = mfma32(*(const bf16x8*)(sK + (k2 * 32 + r) * L::KLD + 16 * c + 8 * hh), qf[c], sc[k2]);
    }
    if constexpr (decltype(MASK)::value) {
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int lim = qlim - (kb + 32 * k2 + 4 * hh);  // keep key offset (i&3) + 8(i>>2) <= lim
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[k2][i] = ((i & 3) + 8 * (i >> 2) <= lim) ? sc[k2][i] : -INFINITY;
      }
    }
    float mt = sc[0][0];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int i = 0; i < 16; ++i) mt = fmaxf(mt, sc[k2][i]);
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * cs;  // the partner lane holds the query's other keys
    // deferred max: rare after the first tiles.  hipcc if-converts it (the 32-value rescale runs on every
    // tile); keeping it a branch with __builtin_expect measured slower (29.3 vs 28.2 us)
    if (__builtin_amdgcn_ballot_w64(mt > m + FW_THR) != 0) {
      const float mn = mt > m + FW_THR ? mt : m;
      const float alpha = fast_exp2(m - mn);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int i = 0; i < HB; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] *= alpha;
    }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = fast_exp2(fmaf(sc[k2][i], cs, -m));
        sc[k2][i] = pv;
        l += pv;
      }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = pack8(sc[k2], s2);
#pragma unroll
        for (int i = 0; i < HB; ++i) acc[i] = mfma32(vt_frag32(sV, L::VLD, 32 * k2 + 16 * s2, 32 * i, lane), pf, acc[i]);
      }
  };
  const int nkt = (min(T, qblk * FW_QROWS + FW_QROWS) + FW_KEYS - 1) / FW_KEYS;
  RegStage<HD, FW_THREADS> rs;
  auto store = [&](int buf) {
    bf16* sK = lds + buf * L::STAGE;
    bf16* sV = sK + FW_KEYS * L::KLD;
#pragma unroll
    for (int i = 0; i < RegStage<HD, FW_THREADS>::CPT; ++i) {
      const int c = tid + FW_THREADS * i, rr = c / (HD / 8), col = (c % (HD / 8)) * 8;
      *(u32x4*)(sK + rr * L::KLD + col) = rs.x[i];
      *(u32x4*)(sV + rr * L::VLD + col) = rs.y[i];
    }
  };
  rs.load(rK, ts, rV, ts, 0, tid);
  store(0);
  __syncthreads();
  for (int it = 0; it < nkt; ++it) {
    if (it + 1 < nkt) rs.load(rK, ts, rV, ts, (it + 1) * FW_KEYS, tid);
    const int kb = it * FW_KEYS;
    const bf16* sK = lds + (it & 1) * L::STAGE;
    if (kb <= q0 + 31 && q0 < T) {  // wave-uniform: else the whole tile lies past this wave's queries
      if (kb + FW_KEYS - 1 > q0) tile(sK, sK + FW_KEYS * L::KLD, kb, std::true_type{});
      else tile(sK, sK + FW_KEYS * L::KLD, kb, std::false_type{});
    }
    if (it + 1 < nkt) store((it + 1) & 1);
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  if (q < T) {
    const float inv = 1.f / l;
    bf16* orow = o + ((long)b * T + q) * H * HD + h * HD;
#pragma unroll
    for (int i = 0; i < HB; ++i)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *(bf16x4*)(orow + 32 * i + 8 * g4 + 4 * hh) =
            bf16x4{f2bf(acc[i][4 * g4] * inv), f2bf(acc[i][4 * g4 + 1] * inv), f2bf(acc[i][4 * g4 + 2] * inv),
                   f2bf(acc[i][4 * g4 + 3] * inv)};
    if (hh == 0) lse[((long)b * H + h) * T + q] = (m + __log2f(l)) * LN2;
  }
}

// ---------------------------------------------------------------------------- forward, round 5 pipeline
// attn_fwd32_kernel's math (transposed score tile, lane-local softmax, deferred max, P straight from the
// accumulators into PV) with a deeper load pipeline and one code path per tile:
//  * TWO register sets alternate (the loop is unrolled by 2, named sets, no runtime-indexed registers), so
//    tile t+2's K/V loads are issued at the top of tile t and have two compute phases + a barrier to land;
//    the loads are unconditional (a load in a branch makes hipcc wait vmcnt(0) at the next LDS write);
//  * all of a tile's V^T fragments (8 x 4 VGPRs) are requested right after the QK^T MFMAs, so they land
//    under the softmax and the 8 PV MFMAs issue back to back;
//  * two running row sums instead of one serial chain of 32 dependent adds;
//  * the diagonal mask under a wave-uniform runtime branch inside ONE tile body: two template
//    instantiations of the whole tile (masked / unmasked) got different register assignments for the O
//    accumulators and ended every tile in ~31 v_mov_b64 copies at the join; one body: 180 instead of 248
//    VGPRs, 12 copies per tile.
// Measured (profiles/r5_attention.md): 26.6-26.9 us per GPT-2-small layer (two instantiations: 27.9-28.2,
// round-4 kernel 28.2-28.5).  At 3 waves / SIMD (168 VGPRs, 48 B spilled): 30.7 us.
// WPS = waves per SIMD (blocks per CU).  3 (default): the V^T fragments of each 32-key half requested just
// before its PV MFMAs instead of all at once after QK^T -- 154 instead of 178 VGPRs, so three 4-wave blocks
// share a CU (768 blocks = one round at GPT-2 small) and the extra wave per SIMD covers the tile's serial
// QK^T -> softmax -> PV chain: 27.21 -> 26.54 us per layer, bitwise identical (profiles/r6_attn_fwd_wps3.log;
// 4 waves/SIMD spills 38 VGPRs).  flags bit 5 = the 2-wave form (A/B).
// CU-balanced block order of a grid that is exactly one round (every block resident from the start): block
// bid runs on XCD bid % 8 as that XCD's k = bid / 8-th block, and blocks k, k + C, k + 2C, ... of an XCD
// (C = CUs per XCD) share a CU.  The host assigns the query blocks to those CU slots by longest-processing-
// time-first (per-CU causal work within 1 unit instead of 17 vs 10 units of the heavy-first order at GPT-2
// small): q[k] = query block, j[k] = which of its (b, h) on this XCD (bh = 8 j + XCD).  n = 0: heavy-first.
constexpr int FW_ORDER_MAX = 256;
struct FwOrder {
  int n;
  unsigned char q[FW_ORDER_MAX], j[FW_ORDER_MAX];
};

template <int HD, int WPS = 3>
__global__ void __launch_bounds__(FW_THREADS, WPS) attn_fwd5_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ o,
                                                               float* __restrict__ lse, int B, int T, int H,
                                                               float scale, FwOrder ord) {
  static_assert(HD == 64, "round-5 forward: head_dim 64");
  constexpr int HC = HD / 16, HB = HD / 32;
  using L = FwLds<HD>;
  using RS = RegStage<HD, FW_THREADS>;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nqb = (T + FW_QROWS - 1) / FW_QROWS, nbh = B * H;
  int qblk, bh;
  if (ord.n) {
    const int k = (int)blockIdx.x >> 3;
    DTC_ASSERT(k < ord.n);
    qblk = ord.q[k];
    bh = 8 * ord.j[k] + ((int)blockIdx.x & 7);
  } else {
    qblk = nqb - 1 - (int)(blockIdx.x / nbh);
    bh = blockIdx.x % nbh;
  }
  const int b = bh / H, h = bh % H;
  DTC_ASSERT(qblk >= 0 && b < B && h < H);
  const long ts = 3L * H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const __amdgpu_buffer_rsrc_t rK = rows_rsrc(qkv + (long)b * T * ts + (1 * H + h) * HD, ts, T, HD);
  const __amdgpu_buffer_rsrc_t rV = rows_rsrc(qkv + (long)b * T * ts + (2 * H + h) * HD, ts, T, HD);
  const int q0 = qblk * FW_QROWS + 32 * w;
  const int q = q0 + r;
  const int nkt = (min(T, qblk * FW_QROWS + FW_QROWS) + FW_KEYS - 1) / FW_KEYS;
  RS ra, rb;  // tile it (even) / it + 1 (odd) register sets
  ra.load(rK, ts, rV, ts, 0, tid);
  bf16x8 qf[HC];
#pragma unroll
  for (int c = 0; c < HC; ++c) qf[c] = q < T ? *(const bf16x8*)(Qb + (long)q * ts + 16 * c + 8 * hh) : bf16x8{};
  rb.load(rK, ts, rV, ts, FW_KEYS, tid);  // younger than Q: the first tile waits for Q only
  const float cs = scale * LOG2E;
  float m = -1e30f, l0 = 0.f, l1 = 0.f;
  f32x16 acc[HB];
#pragma unroll
  for (int i = 0; i < HB; ++i) acc[i] = f32x16{};
  const int qlim = min(q, T - 1);

  auto tile = [&](const bf16* sK, const bf16* sV, int kb, bool diag) {
    bf16x8 kf[2][HC];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int c = 0; c < HC; ++c) kf[k2][c] = *(const bf16x8*)(sK + (k2 * 32 + r) * L::KLD + 16 * c + 8 * hh);
    f32x16 sc[2];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      sc[k2] = f32x16{};
#pragma unroll
      for (int c = 0; c < HC; ++c) sc[k2] = mfma32(kf[k2][c], qf[c], sc[k2]);
    }
    // every V^T fragment of the tile in flight now: they land under the softmax
    bf16x8 vf[2][2][HB];
    if constexpr (WPS == 2) {
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < HB; ++i) vf[k2][s2][i] = vt_frag32(sV, L::VLD, 32 * k2 + 16 * s2, 32 * i, lane);
    }
    if (diag) {  // wave-uniform: only the tiles that cross this wave's diagonal pay for the compares
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int lim = qlim - (kb + 32 * k2 + 4 * hh);
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[k2][i] = ((i & 3) + 8 * (i >> 2) <= lim) ? sc[k2][i] : -INFINITY;
      }
    }
    float mt0 = sc[0][0], mt1 = sc[1][0];
#pragma unroll
    for (int i = 1; i < 16; ++i) {
      mt0 = fmaxf(mt0, sc[0][i]);
      mt1 = fmaxf(mt1, sc[1][i]);
    }
    float mt = fmaxf(mt0, mt1);
    mt = pair_max32(mt) * cs;
    if (__builtin_amdgcn_ballot_w64(mt > m + FW_THR) != 0) {
      const float mn = mt > m + FW_THR ? mt : m;
      const float alpha = fast_exp2(m - mn);
      m = mn;
      l0 *= alpha;
      l1 *= alpha;
#pragma unroll
      for (int i = 0; i < HB; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] *= alpha;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p0 = fast_exp2(fmaf(sc[0][i], cs, -m));
      const float p1 = fast_exp2(fmaf(sc[1][i], cs, -m));
      sc[0][i] = p0;
      sc[1][i] = p1;
      l0 += p0;
      l1 += p1;
    }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      if constexpr (WPS != 2) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < HB; ++i) vf[k2][s2][i] = vt_frag32(sV, L::VLD, 32 * k2 + 16 * s2, 32 * i, lane);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = pack8(sc[k2], s2);
#pragma unroll
        for (int i = 0; i < HB; ++i) acc[i] = mfma32(vf[k2][s2][i], pf, acc[i]);
      }
    }
  };
  auto compute = [&](int it) {
    const int kb = it * FW_KEYS;
    const bf16* sK = lds + (it & 1) * L::STAGE;
    if (kb <= q0 + 31 && q0 < T) tile(sK, sK + FW_KEYS * L::KLD, kb, kb + FW_KEYS - 1 > q0);  // wave-uniform
  };
  auto store = [&](const RS& rs, int buf) {
    bf16* sK = lds + buf * L::STAGE;
    bf16* sV = sK + FW_KEYS * L::KLD;
#pragma unroll
    for (int i = 0; i < RS::CPT; ++i) {
      const int c = tid + FW_THREADS * i, rr = c / (HD / 8), col = (c % (HD / 8)) * 8;
      *(u32x4*)(sK + rr * L::KLD + col) = rs.x[i];
      *(u32x4*)(sV + rr * L::VLD + col) = rs.y[i];
    }
  };
  store(ra, 0);
  __syncthreads();
  // the prefetch loads are unconditional (a tile past the block's last one reads rows that are never used,
  // rows >= T read 0): a load in a branch makes hipcc's wait counting assume it may be missing and wait
  // vmcnt(0) at the next write -- for the younger set too, which is the stall this pipeline removes
  for (int it = 0; it < nkt; it += 2) {
    // even tile: LDS stage 0 holds tile it, rb tile it + 1 (in flight), ra is free
    ra.load(rK, ts, rV, ts, (it + 2) * FW_KEYS, tid);
    compute(it);
    if (it + 1 < nkt) store(rb, 1);
    __syncthreads();
    if (it + 1 >= nkt) break;
    rb.load(rK, ts, rV, ts, (it + 3) * FW_KEYS, tid);
    compute(it + 1);
    if (it + 2 < nkt) store(ra, 0);
    __syncthreads();
  }
  const float l = pair_sum32(l0 + l1);
  if (q < T) {
    const float inv = 1.f / l;
    bf16* orow = o + ((long)b * T + q) * H * HD + h * HD;
#pragma unroll
    for (int i = 0; i < HB; ++i)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *(bf16x4*)(orow + 32 * i + 8 * g4 + 4 * hh) =
            bf16x4{f2bf(acc[i][4 * g4] * inv), f2bf(acc[i][4 * g4 + 1] * inv), f2bf(acc[i][4 * g4 + 2] * inv),
                   f2bf(acc[i][4 * g4 + 3] * inv)};
    if (hh == 0) lse[((long)b * H + h) * T + q] = (m + __log2f(l)) * LN2;
  }
}

// ============================================================================ backward, 32 rows per wave
// The 32x32x16 forms of the two chunked backward kernels (head_dim 64).  Every 64-row tile they read
// both ways -- row fragments (ds_read_b128) for one product and transposed fragments
// (ds_read_b64_tr_b16) for another -- sits in ONE swizzled image: 64 rows x 64 bf16 (128-B rows), 16-B
// chunk c of row r at chunk position c ^ sw8(r), sw8(r) = ((r >> 1) & 1) << 2 | ((r >> 2) & 3).  The row
// reads (rows lane & 31 of one chunk) then hit 16 distinct 4-bank windows per 16-lane read group, and a
// transposed read (4 consecutive rows x 4 chunks per 32 lanes) all 64 banks once.
__device__ __forceinline__ int sw8(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ bf16x8 sw_row(const bf16* t, int row, int ch) {
  return *(const bf16x8*)(t + row * 64 + ((ch ^ sw8(row)) << 3));
}
// A fragment of X^T (32 columns c0.. of the tile as rows, 16 tile rows k0.. as k, permuted order)
__device__ __forceinline__ bf16x8 sw_tr(const bf16* t, int k0, int c0, int lane) {
  const int G = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
  const int r0 = k0 + 4 * (G >> 1) + qq, r1 = r0 + 8, col = c0 + 16 * (G & 1) + 4 * p;
  const bf16* p0 = t + r0 * 64 + (((col >> 3) ^ sw8(r0)) << 3) + (col & 7);
  const bf16* p1 = t + r1 * 64 + (((col >> 3) ^ sw8(r1)) << 3) + (col & 7);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Two [64][64] bf16 tiles (rows t0.., two operands, buffer-resource loads) + optionally two fp32 row vectors
// [64] (lse, delta) for the swizzled images; ONE register set (T14: tile t+1 loaded before tile t's
// compute, written to the other LDS buffer after it), one barrier per tile.
template <int NTH, bool VEC>
struct SwStage {
  static constexpr int CPT = 64 * 8 / NTH;
  u32x4 x[CPT], y[CPT];
  f32x4 v;
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rx, long sx, __amdgpu_buffer_rsrc_t ry, long sy,
                                       const float* __restrict__ va, const float* __restrict__ vb, int t0, int T,
                                       int tid) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + NTH * i, r = c >> 3, ch = c & 7;
      x[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(((long)(t0 + r) * sx + 8 * ch) * 2), 0, 0));
      y[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ry, (int)(((long)(t0 + r) * sy + 8 * ch) * 2), 0, 0));
    }
    if (VEC && tid < 32) {  // va (lse) in log2 units: the consumer's exponent is one fma
      const float* src = tid < 16 ? va : vb;
      const int r = 4 * (tid & 15), t = t0 + r;
      if (t + 4 <= T) v = *(const f32x4*)(src + t);
      else for (int e = 0; e < 4; ++e) v[e] = t + e < T ? src[t + e] : 0.f;
      if (tid < 16) v *= LOG2E;
    }
  }
  __device__ __forceinline__ void store(bf16* lx, bf16* ly, float* lv, int tid) const {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = tid + NTH * i, r = c >> 3, ch = c & 7;
      *(u32x4*)(lx + r * 64 + ((ch ^ sw8(r)) << 3)) = x[i];
      *(u32x4*)(ly + r * 64 + ((ch ^ sw8(r)) << 3)) = y[i];
    }
    if (VEC && tid < 32) *(f32x4*)(lv + (tid < 16 ? 0 : 64) + 4 * (tid & 15)) = v;
  }
};
constexpr int SW_STAGE = 2 * 64 * 64 + 2 * 64 * 2;  // bf16 elements per stage (2 images + 2 fp32 vectors)

// body(sX, sY, sVec, it) over tiles t0_of(it)
template <int NTH, bool VEC, typename T0, typename Body>
__device__ __forceinline__ void sw_pipelined_tiles(int n, T0 t0_of, __amdgpu_buffer_rsrc_t rx, long sx,
                                                   __amdgpu_buffer_rsrc_t ry, long sy, const float* va,
                                                   const float* vb, int T, bf16* lds, int tid, Body body) {
  if (n <= 0) return;
  auto X = [&](int k) { return lds + k * SW_STAGE; };
  auto Y = [&](int k) { return lds + k * SW_STAGE + 64 * 64; };
  auto Vv = [&](int k) { return (float*)(lds + k * SW_STAGE + 2 * 64 * 64); };
  SwStage<NTH, VEC> st;
  st.load(rx, sx, ry, sy, va, vb, t0_of(0), T, tid);
  st.store(X(0), Y(0), Vv(0), tid);
  __syncthreads();
  for (int it = 0; it < n; ++it) {
    if (it + 1 < n) st.load(rx, sx, ry, sy, va, vb, t0_of(it + 1), T, tid);
    body(X(it & 1), Y(it & 1), Vv(it & 1), it);
    if (it + 1 < n) st.store(X((it + 1) & 1), Y((it + 1) & 1), Vv((it + 1) & 1), tid);
    __syncthreads();
  }
}

// dQ (+ delta = rowsum(dO * O) for the dK/dV kernel): block = 4 waves = 128 queries of one (b, h); wave
// = 32 queries on the lane.  Per 32-key block: S^T = K Q^T and dP^T = V dO^T (K / V row fragments, Q /
// dO stationary in registers), dS^T = P^T (dP^T - delta) in registers, dQ^T += K^T dS^T (K transposed
// fragments, dS^T straight from the accumulators).
// DELTA_IN (the merged launch): delta comes precomputed (attn_delta_kernel) instead of from O here.
template <int HD, bool DELTA_IN>
__device__ __forceinline__ void dq32_body(int bid, const bf16* __restrict__ qkv, const bf16* __restrict__ o,
                                          const bf16* __restrict__ dout, const float* __restrict__ lse,
                                          float* __restrict__ delta, bf16* __restrict__ dqkv, int B, int T, int H,
                                          float scale) {
  static_assert(HD == 64, "swizzled 64-wide images");
  constexpr int HC = HD / 16, HB = HD / 32;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nqb = (T + FW_QROWS - 1) / FW_QROWS, nbh = B * H;
  const int qblk = nqb - 1 - (int)(bid / nbh);
  const int bh = bid % nbh, b = bh / H, h = bh % H;
  DTC_ASSERT(qblk >= 0 && b < B && h < H);
  const long ts = 3L * H * HD, dts = (long)H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const bf16* dOb = dout + (long)b * T * dts + h * HD;
  const int q0 = qblk * FW_QROWS + 32 * w, q = q0 + r;
  bf16x8 qf[HC], df[HC];
  float dpart = 0.f;
#pragma unroll
  for (int c = 0; c < HC; ++c) {
    qf[c] = q < T ? *(const bf16x8*)(Qb + (long)q * ts + 16 * c + 8 * hh) : bf16x8{};
    df[c] = q < T ? *(const bf16x8*)(dOb + (long)q * dts + 16 * c + 8 * hh) : bf16x8{};
    if constexpr (!DELTA_IN) {
      const bf16x8 of = q < T ? *(const bf16x8*)(o + ((long)b * T + q) * dts + h * HD + 16 * c + 8 * hh) : bf16x8{};
#pragma unroll
      for (int e = 0; e < 8; ++e) dpart += (float)of[e] * (float)df[c][e];
    }
  }
  float dlt;
  if constexpr (DELTA_IN) {
    dlt = q < T ? delta[((long)b * H + h) * T + q] : 0.f;
  } else {
    dlt = dpart + __shfl_xor(dpart, 32, 64);
    if (hh == 0 && q < T) delta[((long)b * H + h) * T + q] = dlt;
  }
  const float lq = q < T ? lse[((long)b * H + h) * T + q] * LOG2E : 0.f;
  const float cs = scale * LOG2E;
  f32x16 acc[HB];
#pragma unroll
  for (int i = 0; i < HB; ++i) acc[i] = f32x16{};
  // one 32-key block; the causal mask only on the diagonal blocks, under a wave-uniform branch inside ONE
  // body (two instantiations of the whole block joined with 16 v_mov_b64 copies of the dQ accumulators per
  // block: 79.4 -> 78.7 us per merged backward, profiles/r5_attention.md).  Keys >= T only meet queries >= T
  // (key <= q), whose rows are never written, and load as zeros (buffer range): the causal mask suffices.
  auto kblock = [&](const bf16* sK, const bf16* sV, int k2, int ks, bool diag) {
    f32x16 st = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      st = mfma32(sw_row(sK, 32 * k2 + r, 2 * c + hh), qf[c], st);
      dp = mfma32(sw_row(sV, 32 * k2 + r, 2 * c + hh), df[c], dp);
    }
    const int lim = q - (ks + 4 * hh);  // register i holds key ks + 4h + (i & 3) + 8 (i >> 2)
#pragma unroll
    for (int i = 0; i < 16; ++i) st[i] = fast_exp2(fmaf(st[i], cs, -lq));
    if (diag) {
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] = ((i & 3) + 8 * (i >> 2) <= lim) ? st[i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) st[i] *= dp[i] - dlt;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 dsb = pack8(st, s2);
#pragma unroll
      for (int i = 0; i < HB; ++i) acc[i] = mfma32(sw_tr(sK, 32 * k2 + 16 * s2, 32 * i, lane), dsb, acc[i]);
    }
  };
  auto body = [&](const bf16* sK, const bf16* sV, const float*, int it) {
    const int kb = it * 64;
    if (kb > q0 + 31 || q0 >= T) return;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const int ks = kb + 32 * k2;
      if (ks > q0 + 31) break;  // wave-uniform: these 32 keys lie past every query
      kblock(sK, sV, k2, ks, ks + 31 > q0);
    }
  };
  const int nkt = (min(T, qblk * FW_QROWS + FW_QROWS) + 63) / 64;
  sw_pipelined_tiles<FW_THREADS, false>(nkt, [](int it) { return it * 64; }, rows_rsrc(Kb, ts, T, HD), ts,
                                        rows_rsrc(Vb, ts, T, HD), ts, nullptr, nullptr, T, lds, tid, body);
  if (q < T) {
    bf16* pq = dqkv + ((long)b * T + q) * ts + (0 * H + h) * HD;
#pragma unroll
    for (int i = 0; i < HB; ++i)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *(bf16x4*)(pq + 32 * i + 8 * g4 + 4 * hh) =
            bf16x4{f2bf(acc[i][4 * g4] * scale), f2bf(acc[i][4 * g4 + 1] * scale), f2bf(acc[i][4 * g4 + 2] * scale),
                   f2bf(acc[i][4 * g4 + 3] * scale)};
  }
}

template <int HD>
__global__ void __launch_bounds__(FW_THREADS, 2) attn_bwd_dq32_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16* __restrict__ dqkv, int B, int T, int H,
    float scale) {
  dq32_body<HD, false>((int)blockIdx.x, qkv, o, dout, lse, delta, dqkv, B, T, H, scale);
}

// dK, dV: block = 4 waves = 128 keys of one (b, h); wave = 32 keys on the lane.  Per 32-query block:
// S = Q K^T and dP = dO V^T (Q / dO row fragments, K / V stationary), P and dS = P (dP - delta) with the
// key on the lane, dV^T += dO^T P and dK^T += Q^T dS (Q / dO transposed fragments of the same images,
// P / dS straight from the accumulators).  The heaviest key block (0: every query) goes first.
template <int HD>
__device__ __forceinline__ void dkdv32_body(int bid, const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                            const float* __restrict__ lse, const float* __restrict__ delta,
                                            bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  static_assert(HD == 64, "swizzled 64-wide images");
  constexpr int HC = HD / 16, HB = HD / 32;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbh = B * H;
  const int kblk = (int)(bid / nbh);
  const int bh = bid % nbh, b = bh / H, h = bh % H;
  DTC_ASSERT(kblk * FW_QROWS < T && b < B && h < H);
  const long ts = 3L * H * HD, dts = (long)H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const bf16* dOb = dout + (long)b * T * dts + h * HD;
  const float* lseb = lse + ((long)b * H + h) * T;
  const float* delb = delta + ((long)b * H + h) * T;
  const int k0w = kblk * FW_QROWS + 32 * w, key = k0w + r;  // this wave's keys k0w .. k0w + 31
  bf16x8 kf[HC], vf[HC];
#pragma unroll
  for (int c = 0; c < HC; ++c) {
    kf[c] = key < T ? *(const bf16x8*)(Kb + (long)key * ts + 16 * c + 8 * hh) : bf16x8{};
    vf[c] = key < T ? *(const bf16x8*)(Vb + (long)key * ts + 16 * c + 8 * hh) : bf16x8{};
  }
  const float cs = scale * LOG2E;
  f32x16 dk[HB], dv[HB];
#pragma unroll
  for (int i = 0; i < HB; ++i) dk[i] = dv[i] = f32x16{};
  const int qt0 = kblk * FW_QROWS / 64;  // first 64-query tile (queries >= the block's keys)
  // one 32-query block; the causal mask (key <= query) only where the block straddles the wave's keys,
  // under a wave-uniform branch inside ONE body (as the forward / dQ: no second register assignment).
  // Queries >= T need no mask: their Q / dO rows load as zeros (buffer range) and lse / delta as 0, so
  // they add nothing to dK / dV; keys >= T are never written.
  auto qblock = [&](const bf16* sQ, const bf16* sD, const float* sv, int k2, int qs, bool diag) {
    f32x16 sc = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int c = 0; c < HC; ++c) {
      sc = mfma32(sw_row(sQ, 32 * k2 + r, 2 * c + hh), kf[c], sc);
      dp = mfma32(sw_row(sD, 32 * k2 + r, 2 * c + hh), vf[c], dp);
    }
    const int lim = key - (qs + 4 * hh);  // register 4 g4 + e holds query qs + 4h + 8 g4 + e
    f32x16 ds;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int qr = 32 * k2 + 8 * g4 + 4 * hh;  // tile rows of registers 4 g4 .. 4 g4 + 3
      const f32x4 l4 = *(const f32x4*)(sv + qr), d4 = *(const f32x4*)(sv + 64 + qr);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = 4 * g4 + e;
        sc[i] = fast_exp2(fmaf(sc[i], cs, -l4[e]));
        ds[i] = dp[i] - d4[e];
      }
    }
    if (diag) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[i] = ((i & 3) + 8 * (i >> 2) >= lim) ? sc[i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) ds[i] *= sc[i];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pb = pack8(sc, s2), dsb = pack8(ds, s2);
#pragma unroll
      for (int i = 0; i < HB; ++i) {
        dv[i] = mfma32(sw_tr(sD, 32 * k2 + 16 * s2, 32 * i, lane), pb, dv[i]);
        dk[i] = mfma32(sw_tr(sQ, 32 * k2 + 16 * s2, 32 * i, lane), dsb, dk[i]);
      }
    }
  };
  auto body = [&](const bf16* sQ, const bf16* sD, const float* sv, int it) {
    const int qb = (qt0 + it) * 64;
    if (qb + 63 < k0w || k0w >= T) return;  // wave-uniform: every query of the tile before the keys
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const int qs = qb + 32 * k2;
      if (qs + 31 < k0w || qs >= T) continue;  // wave-uniform
      qblock(sQ, sD, sv, k2, qs, qs < k0w + 31);  // wave-uniform: some query of the block precedes a key
    }
  };
  const int nqt = (T - qt0 * 64 + 63) / 64;
  sw_pipelined_tiles<FW_THREADS, true>(nqt, [qt0](int it) { return (qt0 + it) * 64; }, rows_rsrc(Qb, ts, T, HD), ts,
                                       rows_rsrc(dOb, dts, T, HD), dts, lseb, delb, T, lds, tid, body);
  if (key < T) {
    bf16* pk = dqkv + ((long)b * T + key) * ts + (1 * H + h) * HD;
    bf16* pv = dqkv + ((long)b * T + key) * ts + (2 * H + h) * HD;
#pragma unroll
    for (int i = 0; i < HB; ++i)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * i + 8 * g4 + 4 * hh;
        *(bf16x4*)(pk + d0) = bf16x4{f2bf(dk[i][4 * g4] * scale), f2bf(dk[i][4 * g4 + 1] * scale),
                                     f2bf(dk[i][4 * g4 + 2] * scale), f2bf(dk[i][4 * g4 + 3] * scale)};
        *(bf16x4*)(pv + d0) = bf16x4{f2bf(dv[i][4 * g4]), f2bf(dv[i][4 * g4 + 1]), f2bf(dv[i][4 * g4 + 2]),
                                     f2bf(dv[i][4 * g4 + 3])};
      }
  }
}

template <int HD>
__global__ void __launch_bounds__(FW_THREADS, 2) attn_bwd_dkdv32_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  dkdv32_body<HD>((int)blockIdx.x, qkv, dout, lse, delta, dqkv, B, T, H, scale);
}

// dK/dV and dQ blocks in ONE launch (delta precomputed by attn_delta_kernel): the dK/dV blocks first,
// then the dQ blocks, each heaviest first, so the second kernel's blocks fill the first one's tail
// instead of each launch ending in its own partial round (DTC_ATTN_BWD_MERGED).
template <int HD>
__global__ void __launch_bounds__(FW_THREADS, 2) attn_bwd_merged32_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    float* __restrict__ delta, bf16* __restrict__ dqkv, int B, int T, int H, float scale, int nk) {
  const int bid = (int)blockIdx.x;
  if (bid < nk) dkdv32_body<HD>(bid, qkv, dout, lse, delta, dqkv, B, T, H, scale);
  else dq32_body<HD, true>(bid - nk, qkv, nullptr, dout, lse, delta, dqkv, B, T, H, scale);
}

// Chunked backward for T > RES_MAXT / head_dim 64 (the tiled kernels above with 16 waves = 256
// rows per block, 128-row Q/dO or K/V chunks, wave-uniform tile skips, diagonal-only masks and a
// grid-wide heavy-first block order; see attn_fwd_chunk_kernel).
template <int HD>
__host__ __device__ constexpr int ch_lds_bwd() { return 4 * CH_KEYS * AttnLds<HD>::VLD * 2; }

// dK, dV: block = (b, h, NTH/4 keys); wave w owns keys kb0 + 16w .. +15 (key on the lane).  512
// threads: the dk/dv/p/ds accumulators spill at the 128 VGPRs of a 1024-thread block (hd 64)
constexpr int CHB_THREADS = 512, CHB_KROWS = CHB_THREADS / 4;
template <int HD>
__global__ void __launch_bounds__(CHB_THREADS) attn_bwd_dkdv_chunk_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  constexpr int KC = HD / 32, HT = HD / 16;
  using L = AttnLds<HD>;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbh = B * H;
  const int kblk = (int)(blockIdx.x / nbh);  // key block 0 sweeps every query: heaviest, dispatched first
  const int bh = blockIdx.x % nbh, b = bh / H, h = bh % H;
  const long ts = 3L * H * HD, dts = (long)H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const bf16* dOb = dout + (long)b * T * dts + h * HD;
  const float* lseb = lse + ((long)b * H + h) * T;
  const float* delb = delta + ((long)b * H + h) * T;
  const int kb0 = kblk * CHB_KROWS, kmin = kb0 + 16 * w;  // this wave's keys kmin .. kmin + 15
  DTC_ASSERT(b < B && h < H && kb0 < T);
  const int key = kmin + j;
  bf16x8 kf[KC], vf[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    kf[kc] = key < T ? *(const bf16x8*)(Kb + (long)key * ts + kc * 32 + 8 * g) : bf16x8{};
    vf[kc] = key < T ? *(const bf16x8*)(Vb + (long)key * ts + kc * 32 + 8 * g) : bf16x8{};
  }
  const float c = scale * LOG2E;
  f32x4 dk[HT], dv[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) { dk[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[t] = dk[t]; }
  const int cq0 = kb0 / CH_KEYS * CH_KEYS;  // first query chunk (queries >= the block's keys)

  auto body = [&](const bf16* sQ, const bf16* sD, int it) {
#pragma unroll
    for (int t2 = 0; t2 < CH_KEYS / 64; ++t2) {
      const int q0 = cq0 + it * CH_KEYS + t2 * 64;
      if (q0 + 63 < kmin || kmin >= T || q0 >= T) continue;  // wave-uniform: every query before the keys
      const bool diag = q0 < kmin + 15 || q0 + 64 > T;
      const bf16* tQ = sQ + t2 * 64 * L::VLD;
      const bf16* tD = sD + t2 * 64 * L::VLD;
      f32x4 p[4], ds[4];
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          sv = mfma(row_frag(tQ, L::VLD, qt * 16, kc * 32, lane), kf[kc], sv);  // S[q][key]
          dp = mfma(row_frag(tD, L::VLD, qt * 16, kc * 32, lane), vf[kc], dp);  // dP[q][key]
        }
        const int qr = q0 + qt * 16 + 4 * g;
        f32x4 l4 = {0.f, 0.f, 0.f, 0.f}, d4 = {0.f, 0.f, 0.f, 0.f};
        if (qr + 4 <= T) { l4 = *(const f32x4*)(lseb + qr); d4 = *(const f32x4*)(delb + qr); }
        else for (int r = 0; r < 4; ++r) if (qr + r < T) { l4[r] = lseb[qr + r]; d4[r] = delb[qr + r]; }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = qr + r;
          float pv = fast_exp2(fmaf(sv[r], c, -l4[r] * LOG2E));
          if (diag) pv = (key <= qq && qq < T && key < T) ? pv : 0.f;
          p[qt][r] = pv;
          ds[qt][r] = pv * (dp[r] - d4[r]);
        }
      }
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) {
        const bf16x8 pb = pack_p(p[2 * hq], p[2 * hq + 1]), dsb = pack_p(ds[2 * hq], ds[2 * hq + 1]);
#pragma unroll
        for (int t = 0; t < HT; ++t) {
          dv[t] = mfma(tr_frag(tD, L::VLD, 32 * hq, t * 16, lane), pb, dv[t]);
          dk[t] = mfma(tr_frag(tQ, L::VLD, 32 * hq, t * 16, lane), dsb, dk[t]);
        }
      }
    }
  };
  const int nch = (T - cq0 + CH_KEYS - 1) / CH_KEYS;
  pipelined_tiles<HD, CH_KEYS, CHB_THREADS>(nch, [cq0](int it) { return cq0 + it * CH_KEYS; }, Qb, ts, dOb, dts, T, lds,
                                            L::VLD, L::VLD, tid, body);
  if (key < T) {
    bf16* pk = dqkv + ((long)b * T + key) * ts + (1 * H + h) * HD;
    bf16* pv = dqkv + ((long)b * T + key) * ts + (2 * H + h) * HD;
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      *(bf16x4*)(pk + t * 16 + 4 * g) = bf16x4{f2bf(dk[t][0] * scale), f2bf(dk[t][1] * scale), f2bf(dk[t][2] * scale),
                                               f2bf(dk[t][3] * scale)};
      *(bf16x4*)(pv + t * 16 + 4 * g) = bf16x4{f2bf(dv[t][0]), f2bf(dv[t][1]), f2bf(dv[t][2]), f2bf(dv[t][3])};
    }
  }
}

// dQ: block = (b, h, 256 queries); wave w owns queries qb0 + 16w .. +15 (query on the lane).  Also
// computes delta = rowsum(dO * O) of its queries (from the dO / O fragments it holds) and writes
// it for the dK/dV kernel, which runs after it: no separate delta pass.
template <int HD>
__global__ void __launch_bounds__(CH_THREADS) attn_bwd_dq_chunk_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16* __restrict__ dqkv, int B, int T, int H,
    float scale) {
  constexpr int KC = HD / 32, HT = HD / 16;
  using L = AttnLds<HD>;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nqb = (T + CH_QROWS - 1) / CH_QROWS, nbh = B * H;
  const int qblk = nqb - 1 - (int)(blockIdx.x / nbh);  // the last query block sweeps every key: first
  const int bh = blockIdx.x % nbh, b = bh / H, h = bh % H;
  const long ts = 3L * H * HD, dts = (long)H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const bf16* dOb = dout + (long)b * T * dts + h * HD;
  const int qbase = qblk * CH_QROWS + 16 * w;
  const int q = qbase + j;
  DTC_ASSERT(qblk >= 0 && b < B && h < H);
  bf16x8 qf[KC], df[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    qf[kc] = q < T ? *(const bf16x8*)(Qb + (long)q * ts + kc * 32 + 8 * g) : bf16x8{};
    df[kc] = q < T ? *(const bf16x8*)(dOb + (long)q * dts + kc * 32 + 8 * g) : bf16x8{};
  }
  const float lq = q < T ? lse[((long)b * H + h) * T + q] * LOG2E : 0.f;
  float dpart = 0.f;  // this lane's share of rowsum(dO * O): hd columns kc*32 + 8g .. +7
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    const bf16x8 of = q < T ? *(const bf16x8*)(o + ((long)b * T + q) * dts + h * HD + kc * 32 + 8 * g) : bf16x8{};
#pragma unroll
    for (int r = 0; r < 8; ++r) dpart += (float)of[r] * (float)df[kc][r];
  }
  const float dlt = group_sum(dpart);
  if (g == 0 && q < T) delta[((long)b * H + h) * T + q] = dlt;
  const float c = scale * LOG2E;
  f32x4 acc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto body = [&](const bf16* sK, const bf16* sV, int it) {
#pragma unroll
    for (int t2 = 0; t2 < CH_KEYS / 64; ++t2) {
      const int k0 = it * CH_KEYS + t2 * 64;
      if (k0 > qbase + 15 || qbase >= T) continue;  // wave-uniform: keys past every query of the wave
      const bool diag = k0 + 63 > qbase;
      const bf16* tK = sK + t2 * 64 * L::VLD;
      const bf16* tV = sV + t2 * 64 * L::VLD;
      f32x4 ds[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          sv = mfma(row_frag(tK, L::VLD, kt * 16, kc * 32, lane), qf[kc], sv);  // S^T[key][q]
          dp = mfma(row_frag(tV, L::VLD, kt * 16, kc * 32, lane), df[kc], dp);  // dP^T[key][q]
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float pv = fast_exp2(fmaf(sv[r], c, -lq));
          if (diag) {
            const int kk = k0 + kt * 16 + 4 * g + r;
            pv = (kk <= q && kk < T && q < T) ? pv : 0.f;
          }
          ds[kt][r] = pv * (dp[r] - dlt);
        }
      }
#pragma unroll
      for (int hk = 0; hk < 2; ++hk) {
        const bf16x8 dsb = pack_p(ds[2 * hk], ds[2 * hk + 1]);
#pragma unroll
        for (int t = 0; t < HT; ++t) acc[t] = mfma(tr_frag(tK, L::VLD, 32 * hk, t * 16, lane), dsb, acc[t]);
      }
    }
  };
  const int nch = (min(T, qblk * CH_QROWS + CH_QROWS) + CH_KEYS - 1) / CH_KEYS;
  pipelined_tiles<HD, CH_KEYS, CH_THREADS>(nch, [](int it) { return it * CH_KEYS; }, Kb, ts, Vb, ts, T, lds, L::VLD,
                                           L::VLD, tid, body);
  if (q < T) {
    bf16* pq = dqkv + ((long)b * T + q) * ts + (0 * H + h) * HD;
#pragma unroll
    for (int t = 0; t < HT; ++t)
      *(bf16x4*)(pq + t * 16 + 4 * g) = bf16x4{f2bf(acc[t][0] * scale), f2bf(acc[t][1] * scale),
                                               f2bf(acc[t][2] * scale), f2bf(acc[t][3] * scale)};
  }
}

// delta = rowsum(dO * O) of one 8-wide chunk pair, combined over the 4 chunks of a 32-wide head
// row in the order (c0 + c2) + (c1 + c3) — the dQ (group_sum) and dK/dV (xor shuffles) paths
// produce bitwise identical values
__device__ __forceinline__ float dot8(bf16x8 a, bf16x8 c) {
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 8; ++r) s += (float)a[r] * (float)c[r];
  return s;
}

// dO panel -> LDS [Tp][LD] like stage_rows (HD = 32: 4 chunks per row, 4 adjacent threads per
// row), plus delta[r] = rowsum(dO*O) -> sDel[r] (0 for padding rows)
template <int LD, int MAXT>
__device__ __forceinline__ void stage_dout_delta(bf16* lds, float* sDel, const bf16* __restrict__ dOb,
                                                 const bf16* __restrict__ Ob, long tok_stride, int T, int Tp, int tid) {
  constexpr int HD = 32, CPR = HD / 8, PER = (MAXT * CPR + RES_THREADS - 1) / RES_THREADS;
  static_assert(RES_THREADS % CPR == 0, "a row's chunks must sit in adjacent lanes");
  u32x4 v[PER], ov[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = tid + i * RES_THREADS, r = c / CPR, col = (c % CPR) * 8;
    v[i] = r < T ? *(const u32x4*)(dOb + (long)r * tok_stride + col) : u32x4{0, 0, 0, 0};
    ov[i] = r < T ? *(const u32x4*)(Ob + (long)r * tok_stride + col) : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = tid + i * RES_THREADS, r = c / CPR, col = (c % CPR) * 8;
    if (r < Tp) *(u32x4*)(lds + r * LD + col) = v[i];
    float d = dot8(__builtin_bit_cast(bf16x8, v[i]), __builtin_bit_cast(bf16x8, ov[i]));
    d += __shfl_xor(d, 2, 64);
    d += __shfl_xor(d, 1, 64);
    if ((c % CPR) == 0 && r < Tp) sDel[r] = d;
  }
}

// Diagnostic build only (-DDTC_ATTN_STAMPS, scripts/attn_stamps.py): per-block wall-clock stamps
// (s_memrealtime, 100 MHz) at entry, after the panel staging barrier, and at each wave's end.
#ifdef DTC_ATTN_STAMPS
constexpr int STAMP_SLOTS = 18;
__device__ unsigned long long g_attn_stamps[4096 * STAMP_SLOTS];
#define ATTN_STAMP(slot) (g_attn_stamps[(size_t)blockIdx.x * STAMP_SLOTS + (slot)] = __builtin_amdgcn_s_memrealtime())
#else
#define ATTN_STAMP(slot) ((void)0)
#endif

// dK, dV with Q and dO resident: wave owns 16 keys (key on the lane), walks queries >= its keys
template <int HD>
__device__ __forceinline__ void attn_bwd_dkdv_res_body(
    bf16* lds, int bid, const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  constexpr int KC = HD / 32, HT = HD / 16;
  using L = AttnLds<HD>;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop bounds
  int half, bh;
  res_block_map(bid, B * H, half, bh);
  const int b = bh / H, h = bh % H;
  const int Tp = (T + 63) / 64 * 64 + 64;  // + one tile of slack: query tiles start at 16-row offsets
  bf16* sQ = lds;
  bf16* sD = lds + Tp * L::VLD;
  float* sDel = (float*)(sD + Tp * L::VLD);
  float* sLse = sDel + Tp;  // lse (log2 units) of every query row: read per tile from LDS, not L2
  const long ts = 3L * H * HD, dts = (long)H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const bf16* dOb = dout + (long)b * T * dts + h * HD;
  const float* lseb = lse + ((long)b * H + h) * T;
  stage_rows<L::VLD, HD, RES_MAXT + 64>(sQ, Qb, ts, T, Tp, tid);
  stage_dout_delta<L::VLD, RES_MAXT + 64>(sD, sDel, dOb, o + (long)b * T * dts + h * HD, dts, T, Tp, tid);
  for (int r = tid; r < Tp; r += RES_THREADS) sLse[r] = r < T ? lseb[r] * LOG2E : 0.f;
  __syncthreads();
  if (threadIdx.x == 0) ATTN_STAMP(1);
  const int kg = 2 * w + half;
  if (kg * 16 >= T) return;
  const int key = kg * 16 + j;
  bf16x8 kf[KC], vf[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    kf[kc] = key < T ? *(const bf16x8*)(Kb + (long)key * ts + kc * 32 + 8 * g) : bf16x8{};
    vf[kc] = key < T ? *(const bf16x8*)(Vb + (long)key * ts + kc * 32 + 8 * g) : bf16x8{};
  }
  const float c = scale * LOG2E;
  f32x4 dk[HT], dv[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) { dk[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[t] = dk[t]; }
  for (int q0 = kg * 16; q0 < T; q0 += 64) {
    const bf16* tQ = sQ + q0 * L::VLD;
    const bf16* tD = sD + q0 * L::VLD;
    const bool diag = q0 == kg * 16;
    f32x4 p[4], ds[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      f32x4 sc = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        sc = mfma(row_frag(tQ, L::VLD, qt * 16, kc * 32, lane), kf[kc], sc);
        dp = mfma(row_frag(tD, L::VLD, qt * 16, kc * 32, lane), vf[kc], dp);
      }
      const int qr = q0 + qt * 16 + 4 * g;
      // T % 4 == 0 (use_resident): a 4-row group is entirely in or out of range -> selects, no branch
      const int qc = min(qr, T - 4);
      f32x4 l4 = *(const f32x4*)(sLse + qc), d4 = *(const f32x4*)(sDel + qc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = qr + r;
        const bool ok = diag ? (key <= qq && qq < T) : (qq < T);
        const float pv = ok ? fast_exp2(sc[r] * c - l4[r]) : 0.f;  // sLse holds lse * log2(e)
        p[qt][r] = pv;
        ds[qt][r] = pv * (dp[r] - d4[r]);
      }
    }
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
      const bf16x8 pb = pack_p(p[2 * hq], p[2 * hq + 1]), dsb = pack_p(ds[2 * hq], ds[2 * hq + 1]);
#pragma unroll
      for (int t = 0; t < HT; ++t) {
        dv[t] = mfma(tr_frag(tD, L::VLD, 32 * hq, t * 16, lane), pb, dv[t]);
        dk[t] = mfma(tr_frag(tQ, L::VLD, 32 * hq, t * 16, lane), dsb, dk[t]);
      }
    }
  }
  if (key < T) {
    bf16* pk = dqkv + ((long)b * T + key) * ts + (1 * H + h) * HD;
    bf16* pv = dqkv + ((long)b * T + key) * ts + (2 * H + h) * HD;
#pragma unroll
    for (int t = 0; t < HT; ++t) {
      *(bf16x4*)(pk + t * 16 + 4 * g) = bf16x4{f2bf(dk[t][0] * scale), f2bf(dk[t][1] * scale), f2bf(dk[t][2] * scale),
                                               f2bf(dk[t][3] * scale)};
      *(bf16x4*)(pv + t * 16 + 4 * g) = bf16x4{f2bf(dv[t][0]), f2bf(dv[t][1]), f2bf(dv[t][2]), f2bf(dv[t][3])};
    }
  }
}

// dQ with K and V resident: wave owns 16 queries, walks keys <= its queries
template <int HD>
__device__ __forceinline__ void attn_bwd_dq_res_body(
    bf16* lds, int bid, const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  constexpr int KC = HD / 32, HT = HD / 16;
  using L = AttnLds<HD>;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, j = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar loop bounds
  int half, bh;
  res_block_map(bid, B * H, half, bh);
  const int b = bh / H, h = bh % H;
  const int Tp = (T + 63) / 64 * 64;
  bf16* sK = lds;
  bf16* sV = lds + Tp * L::VLD;
  const long ts = 3L * H * HD, dts = (long)H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const bf16* dOb = dout + (long)b * T * dts + h * HD;
  stage_rows<L::VLD, HD, RES_MAXT>(sK, Kb, ts, T, Tp, tid);
  stage_rows<L::VLD, HD, RES_MAXT>(sV, Vb, ts, T, Tp, tid);
  __syncthreads();
  if (threadIdx.x == 0) ATTN_STAMP(1);
  const int qg = 2 * w + half;
  if (qg * 16 >= T) return;
  const int q = qg * 16 + j;
  bf16x8 qf[KC], df[KC], of[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    qf[kc] = q < T ? *(const bf16x8*)(Qb + (long)q * ts + kc * 32 + 8 * g) : bf16x8{};
    df[kc] = q < T ? *(const bf16x8*)(dOb + (long)q * dts + kc * 32 + 8 * g) : bf16x8{};
    of[kc] = q < T ? *(const bf16x8*)(o + ((long)b * T + q) * dts + h * HD + kc * 32 + 8 * g) : bf16x8{};
  }
  const float lq = q < T ? lse[((long)b * H + h) * T + q] * LOG2E : 0.f;
  static_assert(KC == 1, "fused delta assumes head_dim 32");
  const float dq_ = group_sum(dot8(df[0], of[0]));  // delta = rowsum(dO*O) (same order as dK/dV)
  const float c = scale * LOG2E;
  f32x4 acc[HT];
#pragma unroll
  for (int t = 0; t < HT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ntile = (qg * 16 + 16 + 63) / 64;
  for (int kt = 0; kt < ntile; ++kt) {
    const bf16* tK = sK + kt * 64 * L::VLD;
    const bf16* tV = sV + kt * 64 * L::VLD;
    const bool diag = kt == ntile - 1;
    f32x4 ds[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      f32x4 sc = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        sc = mfma(row_frag(tK, L::VLD, st * 16, kc * 32, lane), qf[kc], sc);
        dp = mfma(row_frag(tV, L::VLD, st * 16, kc * 32, lane), df[kc], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = kt * 64 + st * 16 + 4 * g + r;
        const bool ok = diag ? (kk <= q && kk < T && q < T) : (q < T);
        const float pv = ok ? fast_exp2(sc[r] * c - lq) : 0.f;
        ds[st][r] = pv * (dp[r] - dq_);
      }
    }
#pragma unroll
    for (int hk = 0; hk < 2; ++hk) {
      const bf16x8 dsb = pack_p(ds[2 * hk], ds[2 * hk + 1]);
#pragma unroll
      for (int t = 0; t < HT; ++t) acc[t] = mfma(tr_frag(tK, L::VLD, 32 * hk, t * 16, lane), dsb, acc[t]);
    }
  }
  if (q < T) {
    bf16* pq = dqkv + ((long)b * T + q) * ts + (0 * H + h) * HD;
#pragma unroll
    for (int t = 0; t < HT; ++t)
      *(bf16x4*)(pq + t * 16 + 4 * g) = bf16x4{f2bf(acc[t][0] * scale), f2bf(acc[t][1] * scale),
                                               f2bf(acc[t][2] * scale), f2bf(acc[t][3] * scale)};
  }
}

// One launch for the whole resident backward: blocks [0, 2BH) compute dK/dV, [2BH, 4BH) dQ.
// delta = rowsum(dO*O) is computed inside both (no separate delta kernel / launch).
template <int HD>
__global__ void __launch_bounds__(RES_THREADS) attn_bwd_res_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int nkv = 2 * B * H;
  if (threadIdx.x == 0) ATTN_STAMP(0);
  if ((int)blockIdx.x < nkv) attn_bwd_dkdv_res_body<HD>(lds, blockIdx.x, qkv, o, dout, lse, dqkv, B, T, H, scale);
  else attn_bwd_dq_res_body<HD>(lds, blockIdx.x - nkv, qkv, o, dout, lse, dqkv, B, T, H, scale);
  if ((threadIdx.x & 63) == 0) ATTN_STAMP(2 + (threadIdx.x >> 6));
}

// split variant (DTC_ATTN_MERGED=0): the same bodies as two launches
template <int HD>
__global__ void __launch_bounds__(RES_THREADS) attn_bwd_dkdv_res_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  attn_bwd_dkdv_res_body<HD>(lds, blockIdx.x, qkv, o, dout, lse, dqkv, B, T, H, scale);
}
template <int HD>
__global__ void __launch_bounds__(RES_THREADS) attn_bwd_dq_res_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  attn_bwd_dq_res_body<HD>(lds, blockIdx.x, qkv, o, dout, lse, dqkv, B, T, H, scale);
}

// ============================================================================ fused single-round backward
// The merged backward above runs 2*B*H dK/dV blocks and 2*B*H dQ blocks of 16 waves at one block
// per CU: two rounds, each paying its own panel staging and its own causal tail (the wave with the
// most tiles sets the round time).  Here ONE block per (b, h) half holds all four panels (Q, dO,
// K, V) and wave w computes BOTH the dK/dV of key group g = 2w + half (queries >= its keys:
// ~(T - 16g)/64 tiles) and the dQ of query group g (keys <= its queries: ~(16g + 16)/64 tiles), so
// every wave carries the same ~T/64 + 1 tiles and the backward is a single round with one staging.
//
// LDS: unpadded [rows][32] bf16 panels (64-B rows) with the 16-B chunk c of row r stored at
// c ^ fb_swz(r), fb_swz = {0, 2, 3, 1}[(r >> 2) & 3]: the row-fragment ds_read_b128 (16 rows x 4
// chunks) and the transposed ds_read_b64_tr_b16 (8 rows x 32 B per 32-lane half) are both
// bank-conflict-free (tests/test_attn_swizzle_cpu.py simulates the banks).  Q and dO get 64 slack
// rows (dK/dV query tiles start at 16-row offsets) and every row >= T is zero: there p = 2^0 = 1
// but dO = 0 and delta = 0, so dV and dK receive exactly 0 from them — no bounds masks in the loops.
// The causal mask is needed only on the diagonal tile, which is peeled (DIAG template).
constexpr int FB_THREADS = 1024;
constexpr int FB_MAXT_Q = RES_MAXT + 64;  // Q/dO panel rows at T = RES_MAXT

__device__ __forceinline__ int fb_swz(int r) { return (0x1320 >> (((r >> 2) & 3) * 4)) & 3; }

// A/B operand fragment: rows r0 + (lane & 15), hd chunk lane >> 4 (r0 % 16 == 0)
__device__ __forceinline__ bf16x8 fb_row(const bf16* p, int r0, int lane) {
  const int r = r0 + (lane & 15), c = lane >> 4;
  return *(const bf16x8*)(p + r * 32 + ((c ^ fb_swz(r)) << 3));
}
// transposed fragment over the 32 k-rows r0..r0+31 (r0 % 16 == 0), hd columns 16t..16t+15, in the
// permuted k order of tr_frag above
__device__ __forceinline__ bf16x8 fb_tr(const bf16* p, int r0, int t, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int r = r0 + 4 * g + q;
  const int c = 2 * t + (pp >> 1);
  const bf16* p0 = p + r * 32 + ((c ^ fb_swz(r)) << 3) + (pp & 1) * 4;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0 + 16 * 32));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// dK/dV of one 64-query tile (queries q0..q0+63) for this wave's 16 keys
template <bool DIAG>
__device__ __forceinline__ void fb_dkdv_tile(const bf16* sQ, const bf16* sD, const float* sLse, const float* sDel,
                                             int q0, int key, const bf16x8& kf, const bf16x8& vf, float c,
                                             f32x4 (&dk)[2], f32x4 (&dv)[2], int lane) {
  const int g = lane >> 4;
  f32x4 p[4], ds[4];
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    const f32x4 sc = mfma(fb_row(sQ, q0 + qt * 16, lane), kf, z);  // S[q][key]
    const f32x4 dp = mfma(fb_row(sD, q0 + qt * 16, lane), vf, z);  // dP[q][key]
    const int qr = q0 + qt * 16 + 4 * g;
    const f32x4 l4 = *(const f32x4*)(sLse + qr), d4 = *(const f32x4*)(sDel + qr);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float pv = fast_exp2(sc[r] * c - l4[r]);  // sLse holds lse * log2(e)
      if (DIAG) pv = key <= qr + r ? pv : 0.f;
      p[qt][r] = pv;
      ds[qt][r] = pv * (dp[r] - d4[r]);
    }
  }
#pragma unroll
  for (int hq = 0; hq < 2; ++hq) {
    const bf16x8 pb = pack_p(p[2 * hq], p[2 * hq + 1]), dsb = pack_p(ds[2 * hq], ds[2 * hq + 1]);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      dv[t] = mfma(fb_tr(sD, q0 + 32 * hq, t, lane), pb, dv[t]);   // dV^T[hd][key] += dO^T P
      dk[t] = mfma(fb_tr(sQ, q0 + 32 * hq, t, lane), dsb, dk[t]);  // dK^T[hd][key] += Q^T dS
    }
  }
}

// dQ of one 64-key tile (keys k0..k0+63) for this wave's 16 queries
template <bool DIAG>
__device__ __forceinline__ void fb_dq_tile(const bf16* sK, const bf16* sV, int k0, int q, float lq, float dlt,
                                           const bf16x8& qf, const bf16x8& df, float c, f32x4 (&acc)[2], int lane) {
  const int g = lane >> 4;
  f32x4 ds[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    const f32x4 sc = mfma(fb_row(sK, k0 + st * 16, lane), qf, z);
    const f32x4 dp = mfma(fb_row(sV, k0 + st * 16, lane), df, z);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float pv = fast_exp2(sc[r] * c - lq);
      if (DIAG) pv = k0 + st * 16 + 4 * g + r <= q ? pv : 0.f;
      ds[st][r] = pv * (dp[r] - dlt);
    }
  }
#pragma unroll
  for (int hk = 0; hk < 2; ++hk) {
    const bf16x8 dsb = pack_p(ds[2 * hk], ds[2 * hk + 1]);
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[t] = mfma(fb_tr(sK, k0 + 32 * hk, t, lane), dsb, acc[t]);
  }
}

// rows of the Q/dO panels (and lse/delta) the fused backward stages: the dK/dV query tiles of the
// last key group reach row 16*(ngroups-1) + 63
__host__ __device__ inline int fb_rows_q(int T) { return (T + 15) / 16 * 16 + 64; }
__host__ __device__ inline int fb_rows_k(int T) { return (T + 63) / 64 * 64; }

template <int HD>
__global__ void __launch_bounds__(FB_THREADS) attn_bwd_fused_kernel(
    const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
    const float* __restrict__ lse, bf16* __restrict__ dqkv, int B, int T, int H, float scale) {
  static_assert(HD == 32, "fused backward: head_dim 32 (one MFMA K, 64-B panel rows)");
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, g4 = lane >> 4, j = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int half, bh;
  res_block_map(blockIdx.x, B * H, half, bh);
  const int b = bh / H, h = bh % H;
  const int Rq = fb_rows_q(T), Rk = fb_rows_k(T);
  bf16* sQ = lds;
  bf16* sD = sQ + Rq * 32;
  bf16* sK = sD + Rq * 32;
  bf16* sV = sK + Rk * 32;
  float* sLse = (float*)(sV + Rk * 32);
  float* sDel = sLse + Rq;
  const long ts = 3L * H * HD, dts = (long)H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  const bf16* dOb = dout + (long)b * T * dts + h * HD;
  const bf16* Ob = o + (long)b * T * dts + h * HD;
  const float* lseb = lse + ((long)b * H + h) * T;

  // ---- staging: every global load of the thread in flight before the first LDS store
  {
    constexpr int PQ = (FB_MAXT_Q * 4 + FB_THREADS - 1) / FB_THREADS;  // 16-B chunks per thread (Q/dO/O)
    constexpr int PK = (RES_MAXT * 4 + FB_THREADS - 1) / FB_THREADS;   // (K/V)
    u32x4 vq[PQ], vd[PQ], vo[PQ], vk[PK], vv[PK];
#pragma unroll
    for (int i = 0; i < PQ; ++i) {
      const int c = tid + i * FB_THREADS, r = c >> 2, col = (c & 3) * 8;
      const bool ok = r < T;
      vq[i] = ok ? *(const u32x4*)(Qb + (long)r * ts + col) : u32x4{0, 0, 0, 0};
      vd[i] = ok ? *(const u32x4*)(dOb + (long)r * dts + col) : u32x4{0, 0, 0, 0};
      vo[i] = ok ? *(const u32x4*)(Ob + (long)r * dts + col) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < PK; ++i) {
      const int c = tid + i * FB_THREADS, r = c >> 2, col = (c & 3) * 8;
      const bool ok = r < T;
      vk[i] = ok ? *(const u32x4*)(Kb + (long)r * ts + col) : u32x4{0, 0, 0, 0};
      vv[i] = ok ? *(const u32x4*)(Vb + (long)r * ts + col) : u32x4{0, 0, 0, 0};
    }
    float lv[PQ / 4 + 1];
#pragma unroll
    for (int i = 0; i * FB_THREADS < FB_MAXT_Q; ++i) {
      const int r = tid + i * FB_THREADS;
      lv[i] = r < T ? lseb[r] * LOG2E : 0.f;
    }
#pragma unroll
    for (int i = 0; i < PQ; ++i) {
      const int c = tid + i * FB_THREADS, r = c >> 2, ch = c & 3;
      // delta[r] = rowsum(dO * O): the row's 4 chunks sit in 4 adjacent lanes
      float d = dot8(__builtin_bit_cast(bf16x8, vd[i]), __builtin_bit_cast(bf16x8, vo[i]));
      d += __shfl_xor(d, 2, 64);
      d += __shfl_xor(d, 1, 64);
      if (r < Rq) {
        const int off = r * 32 + ((ch ^ fb_swz(r)) << 3);
        *(u32x4*)(sQ + off) = vq[i];
        *(u32x4*)(sD + off) = vd[i];
        if (ch == 0) sDel[r] = d;
      }
    }
#pragma unroll
    for (int i = 0; i < PK; ++i) {
      const int c = tid + i * FB_THREADS, r = c >> 2, ch = c & 3;
      if (r < Rk) {
        const int off = r * 32 + ((ch ^ fb_swz(r)) << 3);
        *(u32x4*)(sK + off) = vk[i];
        *(u32x4*)(sV + off) = vv[i];
      }
    }
#pragma unroll
    for (int i = 0; i * FB_THREADS < FB_MAXT_Q; ++i) {
      const int r = tid + i * FB_THREADS;
      if (r < Rq) sLse[r] = lv[i];
    }
  }
  __syncthreads();
  const int grp = 2 * w + half;
  if (grp * 16 >= T) return;  // no barrier below
  const float c = scale * LOG2E;

  // ---- dK / dV of keys 16*grp .. +15 (queries q0 >= the keys; the first tile is the diagonal)
  {
    const int key = grp * 16 + j;
    const bf16x8 kf = fb_row(sK, grp * 16, lane), vf = fb_row(sV, grp * 16, lane);
    f32x4 dk[2], dv[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) { dk[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[t] = dk[t]; }
    fb_dkdv_tile<true>(sQ, sD, sLse, sDel, grp * 16, key, kf, vf, c, dk, dv, lane);
    for (int q0 = grp * 16 + 64; q0 < T; q0 += 64)
      fb_dkdv_tile<false>(sQ, sD, sLse, sDel, q0, key, kf, vf, c, dk, dv, lane);
    if (key < T) {
      bf16* pk = dqkv + ((long)b * T + key) * ts + (1 * H + h) * HD;
      bf16* pv = dqkv + ((long)b * T + key) * ts + (2 * H + h) * HD;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        *(bf16x4*)(pk + t * 16 + 4 * g4) = bf16x4{f2bf(dk[t][0] * scale), f2bf(dk[t][1] * scale),
                                                  f2bf(dk[t][2] * scale), f2bf(dk[t][3] * scale)};
        *(bf16x4*)(pv + t * 16 + 4 * g4) = bf16x4{f2bf(dv[t][0]), f2bf(dv[t][1]), f2bf(dv[t][2]), f2bf(dv[t][3])};
      }
    }
  }
  // ---- dQ of queries 16*grp .. +15 (keys <= the queries; the last tile is the diagonal)
  {
    const int q = grp * 16 + j;
    const bf16x8 qf = fb_row(sQ, grp * 16, lane), df = fb_row(sD, grp * 16, lane);
    const float lq = sLse[q], dlt = sDel[q];
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const int ntile = (grp * 16 + 16 + 63) / 64;
    for (int kt = 0; kt < ntile - 1; ++kt) fb_dq_tile<false>(sK, sV, kt * 64, q, lq, dlt, qf, df, c, acc, lane);
    fb_dq_tile<true>(sK, sV, (ntile - 1) * 64, q, lq, dlt, qf, df, c, acc, lane);
    if (q < T) {
      bf16* pq = dqkv + ((long)b * T + q) * ts + (0 * H + h) * HD;
#pragma unroll
      for (int t = 0; t < 2; ++t)
        *(bf16x4*)(pq + t * 16 + 4 * g4) = bf16x4{f2bf(acc[t][0] * scale), f2bf(acc[t][1] * scale),
                                                  f2bf(acc[t][2] * scale), f2bf(acc[t][3] * scale)};
    }
  }
}


inline long fb_lds_bytes(int T) {
  return (long)(2 * fb_rows_q(T) + 2 * fb_rows_k(T)) * 32 * 2 + (long)2 * fb_rows_q(T) * 4;
}

// LDS bytes of the resident kernels; 0 if the sequence does not fit (then the tiled kernels run)
inline long res_lds_fwd(int T, int HD) { const long Tp = (T + 63) / 64 * 64; return Tp * (AttnLds<32>::KLD + HD + 16) * 2; }
inline long res_lds_dkdv(int T, int HD) { const long Tp = (T + 63) / 64 * 64 + 64; return 2 * Tp * (HD + 16) * 2 + Tp * 8; }
inline long res_lds_dq(int T, int HD) { const long Tp = (T + 63) / 64 * 64; return 2 * Tp * (HD + 16) * 2; }
constexpr long LDS_MAX = 160 * 1024;

bool use_resident(int T, int HD) {
  static const int enabled = [] { const char* v = getenv("DTC_ATTN_RESIDENT"); return v ? atoi(v) : 1; }();
  return enabled && HD == 32 && T % 4 == 0 && T <= RES_MAXT && res_lds_fwd(T, HD) <= LDS_MAX &&
         res_lds_dkdv(T, HD) <= LDS_MAX && res_lds_dq(T, HD) <= LDS_MAX;
}

// chunked kernels for what the resident ones cannot hold (DTC_ATTN_CHUNK=0: the 256-thread tiled kernels)
bool attn_chunk_enabled() {
  static const int v = [] { const char* e = getenv("DTC_ATTN_CHUNK"); return e ? atoi(e) : 1; }();
  return v != 0;
}

template <typename K>
void allow_lds(K kernel, long bytes) {  // > 64 KB of dynamic LDS must be opted into per kernel
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace

extern "C" {

// copies the diagnostic stamps (DTC_ATTN_STAMPS builds only; returns 4003 otherwise)
int dtc_attn_stamps(unsigned long long* host, long n) {
#ifdef DTC_ATTN_STAMPS
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_attn_stamps), n * sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
#else
  (void)host; (void)n;
  return 4003;
#endif
}

// The CU-balanced order (FwOrder) for nqb query blocks x nbh (b, h) at WPS blocks per CU, or n = 0 when the
// grid is not exactly one round of 8 equal XCDs.  Longest-processing-time-first per XCD: the query blocks,
// heaviest first, each to the least-loaded CU with a free slot; CU c's s-th block becomes k = s * C + c.
static FwOrder fw_order(int nqb, int nbh, int wps) {
  static int cached_key = -1;
  static FwOrder cached;
  const int key = (nqb << 20) | (nbh << 4) | wps;
  if (key == cached_key) return cached;
  FwOrder ord{};
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 0;
  const int C = cus / 8, per_xcd = nbh / 8 * nqb;
  if (cus % 8 == 0 && nbh % 8 == 0 && C > 0 && per_xcd == C * wps && per_xcd <= FW_ORDER_MAX && nqb <= 255 &&
      nbh / 8 <= 255) {
    std::vector<int> load(C, 0), cnt(C, 0), used(nqb, 0);
    for (int q = nqb - 1; q >= 0; --q)
      for (int i = 0; i < nbh / 8; ++i) {
        int c = -1;
        for (int t = 0; t < C; ++t)
          if (cnt[t] < wps && (c < 0 || load[t] < load[c])) c = t;
        const int k = cnt[c] * C + c;
        ord.q[k] = (unsigned char)q;
        ord.j[k] = (unsigned char)used[q]++;
        load[c] += q + 1;
        ++cnt[c];
      }
    ord.n = per_xcd;
  }
  cached_key = key;
  cached = ord;
  return ord;
}

int dtc_attn_fwd(const bf16* qkv, bf16* o, float* lse, int B, int T, int H, int HD, long flags, float scale,
                 hipStream_t st) {
  if (use_resident(T, HD)) {
    allow_lds(attn_fwd_res_kernel<32>, res_lds_fwd(T, HD));
    // flags bit 0: plain wave -> query-group order (A/B of the SIMD-balanced order)
    hipLaunchKernelGGL(attn_fwd_res_kernel<32>, dim3(B * H * 2), dim3(RES_THREADS), res_lds_fwd(T, HD), st, qkv, o,
                       lse, B, T, H, scale, (int)!(flags & 1));
    DTC_CHECK_LAUNCH();
    return 0;
  }
  // default at head_dim 64: the round-5 forward (2-deep K/V prefetch, V^T fragments ahead of the softmax, one
  // code path per tile; 26.6-26.9 vs 28.2-28.5 us per layer, profiles/r5_attention.md); flags bit 4 = the
  // round-4 kernel (A/B),
  // bit 2 = the 16-row chunked kernel
  if (HD == 64 && (flags & 32) && !(flags & 16) && !(flags & 4) && attn_chunk_enabled()) {
    allow_lds(attn_fwd5_kernel<64, 2>, fw_lds_bytes<64>());
    FwOrder ord;
    ord.n = 0;
    hipLaunchKernelGGL((attn_fwd5_kernel<64, 2>), dim3(B * H * ((T + FW_QROWS - 1) / FW_QROWS)), dim3(FW_THREADS),
                       fw_lds_bytes<64>(), st, qkv, o, lse, B, T, H, scale, ord);
    DTC_CHECK_LAUNCH();
    return 0;
  }
  if (HD == 64 && !(flags & 16) && !(flags & 4) && attn_chunk_enabled()) {
    allow_lds(attn_fwd5_kernel<64, 3>, fw_lds_bytes<64>());
    const int nqb = (T + FW_QROWS - 1) / FW_QROWS;
    // CU-balanced block order (default; flags bit 6 = the heavy-first order, A/B): 25.8 -> 24.2-24.5 us per
    // GPT-2-small layer, bitwise identical (profiles/r6_attn_order_ab*.log)
    const FwOrder ord = (flags & 64) ? FwOrder{} : fw_order(nqb, B * H, 3);
    hipLaunchKernelGGL((attn_fwd5_kernel<64, 3>), dim3(B * H * nqb), dim3(FW_THREADS), fw_lds_bytes<64>(), st, qkv, o,
                       lse, B, T, H, scale, ord);
    DTC_CHECK_LAUNCH();
    return 0;
  }
  // flags bit 2: the 16-query-row chunked kernel instead of the 32-row one (A/B)
  if (HD == 64 && !(flags & 4) && attn_chunk_enabled()) {
    allow_lds(attn_fwd32_kernel<64>, fw_lds_bytes<64>());
    hipLaunchKernelGGL(attn_fwd32_kernel<64>, dim3(B * H * ((T + FW_QROWS - 1) / FW_QROWS)), dim3(FW_THREADS),
                       fw_lds_bytes<64>(), st, qkv, o, lse, B, T, H, scale);
    DTC_CHECK_LAUNCH();
    return 0;
  }
  if (attn_chunk_enabled() && (HD == 32 || HD == 64)) {
    const dim3 g(B * H * ((T + CH_QROWS - 1) / CH_QROWS));
    if (HD == 64) {
      allow_lds(attn_fwd_chunk_kernel<64>, ch_lds_fwd<64>());
      hipLaunchKernelGGL(attn_fwd_chunk_kernel<64>, g, dim3(CH_THREADS), ch_lds_fwd<64>(), st, qkv, o, lse, B, T, H, scale);
    } else {
      allow_lds(attn_fwd_chunk_kernel<32>, ch_lds_fwd<32>());
      hipLaunchKernelGGL(attn_fwd_chunk_kernel<32>, g, dim3(CH_THREADS), ch_lds_fwd<32>(), st, qkv, o, lse, B, T, H, scale);
    }
    DTC_CHECK_LAUNCH();
    return 0;
  }
  int nqb = (T + 63) / 64;
  dim3 grid(B * H * nqb);
  if (HD == 32) hipLaunchKernelGGL(attn_fwd_kernel<32>, grid, dim3(256), 0, st, qkv, o, lse, B, T, H, scale);
  else if (HD == 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, st, qkv, o, lse, B, T, H, scale);
  else return 4001;
  DTC_CHECK_LAUNCH();
  return 0;
}

long dtc_attn_bwd_workspace_bytes(int B, int T, int H, int HD) { return (long)B * H * T * 4; }

int dtc_attn_bwd(const bf16* qkv, const bf16* o, const float* lse, const bf16* dout, bf16* dqkv, int flags, int B,
                 int T, int H, int HD, float scale, float* ws, long ws_bytes, hipStream_t st) {
  if (ws_bytes < dtc_attn_bwd_workspace_bytes(B, T, H, HD)) return 4002;
  int nb = (T + 63) / 64;
  dim3 grid(B * H * nb);
  static const int merged = [] { const char* v = getenv("DTC_ATTN_MERGED"); return v ? atoi(v) : 1; }();
  // DTC_ATTN_FUSED=0: the two-round merged/split resident kernels instead of the fused single round
  static const int fused = [] { const char* v = getenv("DTC_ATTN_FUSED"); return v ? atoi(v) : 1; }();
  // flags bit 0: force the two-round kernels (in-process A/B, benchmarks/attn_ab.py)
  if (use_resident(T, HD) && fused && !(flags & 1) && fb_lds_bytes(T) <= LDS_MAX) {
    allow_lds(attn_bwd_fused_kernel<32>, fb_lds_bytes(T));
    hipLaunchKernelGGL(attn_bwd_fused_kernel<32>, dim3(B * H * 2), dim3(FB_THREADS), fb_lds_bytes(T), st, qkv, o, dout,
                       lse, dqkv, B, T, H, scale);
  } else if (use_resident(T, HD) && !merged) {
    allow_lds(attn_bwd_dkdv_res_kernel<32>, res_lds_dkdv(T, HD));
    allow_lds(attn_bwd_dq_res_kernel<32>, res_lds_dq(T, HD));
    hipLaunchKernelGGL(attn_bwd_dkdv_res_kernel<32>, dim3(B * H * 2), dim3(RES_THREADS), res_lds_dkdv(T, HD), st, qkv,
                       o, dout, lse, dqkv, B, T, H, scale);
    hipLaunchKernelGGL(attn_bwd_dq_res_kernel<32>, dim3(B * H * 2), dim3(RES_THREADS), res_lds_dq(T, HD), st, qkv, o,
                       dout, lse, dqkv, B, T, H, scale);
  } else if (use_resident(T, HD)) {
    const long lds_b = std::max(res_lds_dkdv(T, HD), res_lds_dq(T, HD));
    allow_lds(attn_bwd_res_kernel<32>, lds_b);
    hipLaunchKernelGGL(attn_bwd_res_kernel<32>, dim3(B * H * 4), dim3(RES_THREADS), lds_b, st, qkv, o, dout, lse,
                       dqkv, B, T, H, scale);
  } else if (attn_chunk_enabled() && (HD == 32 || HD == 64)) {
    const dim3 g(B * H * ((T + CH_QROWS - 1) / CH_QROWS)), gk(B * H * ((T + CHB_KROWS - 1) / CHB_KROWS));
    if (HD == 64 && !(flags & 4)) {
      // 32x32x16 kernels (flags bit 2: the 16-row chunked ones); dQ first: it writes delta
      constexpr int lb = 2 * SW_STAGE * 2;
      allow_lds(attn_bwd_dq32_kernel<64>, lb);
      allow_lds(attn_bwd_dkdv32_kernel<64>, lb);
      const dim3 g32(B * H * ((T + FW_QROWS - 1) / FW_QROWS));
      // DTC_ATTN_BWD_MERGED (default 1; flags bit 3 forces it): delta pass + one launch of dK/dV and dQ
      // blocks -- 82.9 vs 85.3 us per layer, step 11.35-11.37 vs 11.40-11.42 ms (profiles/r4_attn_merged.log)
      static const int bwd_merged = [] { const char* v = getenv("DTC_ATTN_BWD_MERGED"); return v ? atoi(v) : 1; }();
      if (bwd_merged || (flags & 8)) {
        allow_lds(attn_bwd_merged32_kernel<64>, lb);
        launch_attn_delta<64>(o, dout, ws, B, T, H, st);
        hipLaunchKernelGGL(attn_bwd_merged32_kernel<64>, dim3(2 * g32.x), dim3(FW_THREADS), lb, st, qkv, dout, lse, ws,
                           dqkv, B, T, H, scale, (int)g32.x);
      } else {
        hipLaunchKernelGGL(attn_bwd_dq32_kernel<64>, g32, dim3(FW_THREADS), lb, st, qkv, o, dout, lse, ws, dqkv, B, T,
                           H, scale);
        hipLaunchKernelGGL(attn_bwd_dkdv32_kernel<64>, g32, dim3(FW_THREADS), lb, st, qkv, dout, lse, ws, dqkv, B, T,
                           H, scale);
      }
    } else if (HD == 64) {
      allow_lds(attn_bwd_dkdv_chunk_kernel<64>, ch_lds_bwd<64>());
      allow_lds(attn_bwd_dq_chunk_kernel<64>, ch_lds_bwd<64>());
      // dQ first: it writes delta (ws) for the dK/dV kernel
      hipLaunchKernelGGL(attn_bwd_dq_chunk_kernel<64>, g, dim3(CH_THREADS), ch_lds_bwd<64>(), st, qkv, o, dout, lse,
                         ws, dqkv, B, T, H, scale);
      hipLaunchKernelGGL(attn_bwd_dkdv_chunk_kernel<64>, gk, dim3(CHB_THREADS), ch_lds_bwd<64>(), st, qkv, dout, lse, ws,
                         dqkv, B, T, H, scale);
    } else {
      allow_lds(attn_bwd_dkdv_chunk_kernel<32>, ch_lds_bwd<32>());
      allow_lds(attn_bwd_dq_chunk_kernel<32>, ch_lds_bwd<32>());
      // dQ first: it writes delta (ws) for the dK/dV kernel
      hipLaunchKernelGGL(attn_bwd_dq_chunk_kernel<32>, g, dim3(CH_THREADS), ch_lds_bwd<32>(), st, qkv, o, dout, lse,
                         ws, dqkv, B, T, H, scale);
      hipLaunchKernelGGL(attn_bwd_dkdv_chunk_kernel<32>, gk, dim3(CHB_THREADS), ch_lds_bwd<32>(), st, qkv, dout, lse, ws,
                         dqkv, B, T, H, scale);
    }
  } else if (HD == 32) {
    launch_attn_delta<32>(o, dout, ws, B, T, H, st);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<32>, grid, dim3(256), 0, st, qkv, dout, lse, ws, dqkv, B, T, H, scale);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<32>, grid, dim3(256), 0, st, qkv, dout, lse, ws, dqkv, B, T, H, scale);
  } else if (HD == 64) {
    launch_attn_delta<64>(o, dout, ws, B, T, H, st);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<64>, grid, dim3(256), 0, st, qkv, dout, lse, ws, dqkv, B, T, H, scale);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<64>, grid, dim3(256), 0, st, qkv, dout, lse, ws, dqkv, B, T, H, scale);
  } else {
    return 4001;
  }
  DTC_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
