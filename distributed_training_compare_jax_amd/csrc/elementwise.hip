// Streaming kernels: embedding+dropout fwd/bwd, cross-entropy combine/backward, fused
// clip+AdamW, global-norm reduction, casts.  All memory-bound: 16-byte vector accesses,
// grid-stride, no host sync, stream-ordered (graph-capturable).
#include "common.h"

namespace {

// ---------------------------------------------------------------- Philox4x32-10 (dropout)
// Counter = (group lo, group hi, 0, 0) with group = global_element_index / 4; key = (seed, step).
// Bit-identical to ops/embedding.py:philox4x32 (tested).
__device__ __forceinline__ u32x4 philox(uint64_t group, uint32_t k0, uint32_t k1) {
  uint32_t c0 = (uint32_t)group, c1 = (uint32_t)(group >> 32), c2 = 0, c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
  }
  return u32x4{c0, c1, c2, c3};
}

__device__ __forceinline__ uint32_t drop_threshold(float p) {
  double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// h[tok, d..d+3] = dropout(wte[id] + wpe[t])  — one thread per 4 channels (one Philox call)
// One wave per token row (a block = 4 rows): the id is one wave-uniform load, and each lane keeps all of
// its row's wte / wpe vectors in flight before the dropout and the stores (one thread per 4 channels
// waited on the id load, then on the row load: 17 us for 8192 x 768).  Same Philox element mapping.
__global__ void __launch_bounds__(256) embed_fwd_kernel(const int* __restrict__ ids, const float* __restrict__ wte,
                                                        const float* __restrict__ wpe, float* __restrict__ h, int B,
                                                        int T, int D, float p, uint32_t seed,
                                                        const int64_t* __restrict__ step, long row0) {
  constexpr int VPL = 4;  // f32x4 per lane per pass: rows up to 64 * 4 * 4 = 1024 channels in one pass
  const long tok = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (tok >= (long)B * T) return;
  const int t = (int)(tok % T);
  const int id = __builtin_amdgcn_readfirstlane(ids[tok]);
  const int D4 = D / 4;
  DTC_ASSERT(id >= 0 && t < T);
  const uint32_t thr = drop_threshold(p);
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t st = p > 0.f ? (uint32_t)step[0] : 0u;
  const long gtok = (row0 + tok / T) * T + t;
  for (int c0 = 0; c0 < D4; c0 += 64 * VPL) {
    f32x4 v[VPL];
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int c = c0 + k * 64 + lane;
      if (c < D4) v[k] = *(const f32x4*)(wte + (long)id * D + 4 * c) + *(const f32x4*)(wpe + (long)t * D + 4 * c);
    }
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int c = c0 + k * 64 + lane;
      if (c >= D4) continue;
      if (p > 0.f) {
        const uint64_t grp = ((uint64_t)gtok * D + 4 * c) >> 2;
        const u32x4 u = philox(grp, seed, st);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[k][r] = u[r] >= thr ? v[k][r] * sc : 0.f;
      }
      *(f32x4*)(h + tok * D + 4 * c) = v[k];
    }
  }
}

// ---------------------------------------------------------------- embedding backward
// Deterministic (no float atomics), so every DP rank that rebuilds dwte from the same gathered
// tokens gets bit-identical rows, and two runs give bit-identical grads:
//   1. embed_sort_kernel  (runs early, off the critical path: it only needs the ids)
//      key = id << nb | token  -> one-block bitonic sort in LDS.  Keys are unique, so the sorted
//      order (hence every summation order below) is a pure function of the ids.
//   2. embed_piece_sums   pieces of 16-64 sorted keys: each run of equal ids inside a tile is summed
//      in order into P[first position of the run]
//   3. embed_segment_sum  per id: P[segment start] + P[each tile boundary inside the segment]
//   dwpe: one thread per (t, 4 channels) sums over the batch in order.
constexpr int SORT_MAX = 32768;

__global__ void __launch_bounds__(1024) embed_sort_kernel(const int* __restrict__ ids, int n, int npad, int nb,
                                                          uint32_t* __restrict__ keys) {
  __shared__ uint32_t s[SORT_MAX];
  for (int i = threadIdx.x; i < npad; i += 1024) s[i] = i < n ? ((uint32_t)ids[i] << nb) | (uint32_t)i : 0xFFFFFFFFu;
  __syncthreads();
  for (int k = 2; k <= npad; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < npad; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          uint32_t a = s[i], b = s[l];
          if ((a > b) == ((i & k) == 0)) { s[i] = b; s[l] = a; }
        }
      }
      __syncthreads();
    }
  for (int i = threadIdx.x; i < n; i += 1024) keys[i] = s[i];
}

__device__ __forceinline__ f32x4 dropped_row(const float* __restrict__ dh, long tok, int T, int D, int d, float p,
                                             uint32_t thr, float sc, uint32_t seed, uint32_t step, long row0) {
  f32x4 g = *(const f32x4*)(dh + tok * D + d);
  if (p > 0.f) {
    uint64_t grp = ((uint64_t)(row0 * T + tok) * D + d) >> 2;
    u32x4 u = philox(grp, seed, step);
#pragma unroll
    for (int r = 0; r < 4; ++r) g[r] = u[r] >= thr ? g[r] * sc : 0.f;
  }
  return g;
}

// block (bx, by) of the (pieces, ceil(D/256)) grid, 64 threads x 4 channels
__device__ __forceinline__ void embed_piece_sums(int bx, int by, const uint32_t* __restrict__ keys, int n, int nb,
                                                 int piece, const float* __restrict__ dh, float* __restrict__ P, int T,
                                                 int D, float p, uint32_t seed, const int64_t* __restrict__ step,
                                                 long row0) {
  const int d = (by * 64 + threadIdx.x) * 4;
  if (d >= D) return;
  const int q_beg = bx * piece, q_end = min(n, q_beg + piece);
  DTC_ASSERT(q_beg < n && nb >= 1 && nb < 32 && d + 4 <= D);
  const uint32_t tmask = (1u << nb) - 1;
  const uint32_t thr = drop_threshold(p), stp = (uint32_t)step[0];
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int start = q_beg;
  uint32_t cur = keys[q_beg] >> nb;
  for (int q0 = q_beg; q0 < q_end; q0 += 8) {
    f32x4 g[8];
    uint32_t id[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // 8 independent row loads in flight
      const int q = min(q0 + u, q_end - 1);
      const uint32_t key = keys[q];
      id[u] = key >> nb;
      g[u] = dropped_row(dh, key & tmask, T, D, d, p, thr, sc, seed, stp, row0);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (q0 + u >= q_end) break;
      if (id[u] != cur) {
        *(f32x4*)(P + (long)start * D + d) = acc;
        acc = f32x4{0.f, 0.f, 0.f, 0.f};
        start = q0 + u;
        cur = id[u];
      }
      acc += g[u];
    }
  }
  *(f32x4*)(P + (long)start * D + d) = acc;
}

// grid (n, ceil(D/256)), 64 threads; only the first key of each id does work.  Pieces of one id
// start at its first key and at every piece boundary inside its run; they are fetched 8 at a time
// (membership is monotone along the run) and added in order.
// sq (optional, beta = 0 only): block (s, y) writes sq[s * gridDim.y + y] = its rows' sum of squares of the
// FINAL dwte values (0 for the blocks that do no work), so the gradient norm needs no pass over the table:
// every row no id touches is zero.
__global__ void __launch_bounds__(64) embed_segment_sum(const uint32_t* __restrict__ keys, int n, int nb, int piece,
                                                        const float* __restrict__ P, float* __restrict__ dwte, int D,
                                                        int accumulate, float* __restrict__ sq,
                                                        uint32_t* __restrict__ keys_out) {
  const int s = blockIdx.x;
  const uint32_t id = keys[s] >> nb;
  if (keys_out && blockIdx.y == 0 && threadIdx.x == 0) keys_out[s] = keys[s];  // the next call's prev_keys
  DTC_ASSERT(s < n && piece >= 1 && !(sq && accumulate));
  float* sq_slot = sq ? sq + (long)s * gridDim.y + blockIdx.y : nullptr;
  if (s > 0 && (keys[s - 1] >> nb) == id) {  // not the first occurrence of this id (block-uniform)
    if (sq_slot && threadIdx.x == 0) *sq_slot = 0.f;
    return;
  }
  const int d = (blockIdx.y * 64 + threadIdx.x) * 4;
  float q2 = 0.f;  // this lane's sum of squares of the final values
  if (d < D) {
    f32x4 acc = *(const f32x4*)(P + (long)s * D + d);
    for (int q = (s / piece + 1) * piece; q < n; q += 8 * piece) {
      bool in[8];
      f32x4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int qq = q + u * piece;
        in[u] = qq < n && (keys[min(qq, n - 1)] >> nb) == id;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        t[u] = in[u] ? *(const f32x4*)(P + (long)(q + u * piece) * D + d) : f32x4{0.f, 0.f, 0.f, 0.f};
      bool more = true;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (!in[u]) { more = false; break; }
        acc += t[u];
      }
      if (!more) break;
    }
    float* o = dwte + (long)id * D + d;
    if (accumulate) acc += *(const f32x4*)o;
    *(f32x4*)o = acc;
    q2 = acc[0] * acc[0] + acc[1] * acc[1] + acc[2] * acc[2] + acc[3] * acc[3];
  }
  if (sq_slot) {  // every lane of the (one-wave) block reaches the sum
    const float z = warp_sum(q2);
    if (threadIdx.x == 0) *sq_slot = z;
  }
}

// returns the sum of squares of the dwpe values this thread wrote (0 past the end)
__device__ __forceinline__ float wpe_bwd(long i, const float* __restrict__ dh, float* __restrict__ dwpe, int B, int T,
                                         int D, float p, uint32_t seed, const int64_t* __restrict__ step, long row0,
                                         int accumulate) {
  const int D4 = D / 4;
  if (i >= (long)T * D4) return 0.f;
  int t = (int)(i / D4);
  int d = (int)(i % D4) * 4;
  DTC_ASSERT(D % 4 == 0 && t < T && d + 4 <= D && B >= 1);
  const uint32_t thr = drop_threshold(p), stp = (uint32_t)step[0];
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < B; ++b) acc += dropped_row(dh, (long)b * T + t, T, D, d, p, thr, sc, seed, stp, row0);
  float* o = dwpe + (long)t * D + d;
  if (accumulate) acc += *(f32x4*)o;
  *(f32x4*)o = acc;
  return acc[0] * acc[0] + acc[1] * acc[1] + acc[2] * acc[2] + acc[3] * acc[3];
}

// The embedding backward's first launch: three independent jobs in one grid of 64-thread blocks, so the
// latency-bound piece sums run alongside the bandwidth-bound table zeroing instead of after it:
// [0, nzero) zero the dwte table (EB_ZCH float4 per block; beta = 0 only; with prev_keys: one block per key of
// the previous call, zeroing that id's row once -- the only rows that can be nonzero), then the piece-sum blocks
// (pieces x dblk), then dwpe (one thread per (t, 4 channels)).  Was three launches, 53 us at GPT-2 small;
// 36.8 us in this order (40.9 us with the piece sums first).
constexpr int EB_ZCH = 64 * 32;
__global__ void __launch_bounds__(64) embed_bwd_stage1(const uint32_t* __restrict__ keys, int n, int nb, int piece,
                                                       int npieces, int dblk, const float* __restrict__ dh,
                                                       float* __restrict__ P, float* __restrict__ dwte, long n4zero,
                                                       int nzero, float* __restrict__ dwpe, int B, int T, int D,
                                                       float p, uint32_t seed, const int64_t* __restrict__ step,
                                                       long row0, int accumulate, float* __restrict__ sq_wpe,
                                                       const uint32_t* __restrict__ prev_keys) {
  int b = blockIdx.x;
  if (b < nzero) {
    if (prev_keys) {  // sparse: zero the rows the previous call wrote (every other row is still zero)
      const uint32_t id = prev_keys[b] >> nb;
      if (b > 0 && (prev_keys[b - 1] >> nb) == id) return;  // not the id's first key (block-uniform)
      f32x4* z = (f32x4*)(dwte + (long)id * D);
      for (int e = threadIdx.x; e < D / 4; e += 64) z[e] = f32x4{0.f, 0.f, 0.f, 0.f};
      return;
    }
    f32x4* z = (f32x4*)dwte;
    const long e0 = (long)b * EB_ZCH, e1 = min(n4zero, e0 + EB_ZCH);
    for (long e = e0 + threadIdx.x; e < e1; e += 64) z[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  b -= nzero;
  if (b < npieces * dblk) {
    embed_piece_sums(b % npieces, b / npieces, keys, n, nb, piece, dh, P, T, D, p, seed, step, row0);
    return;
  }
  b -= npieces * dblk;
  const float q = wpe_bwd((long)b * 64 + threadIdx.x, dh, dwpe, B, T, D, p, seed, step, row0, accumulate);
  if (sq_wpe) {  // one sum-of-squares slot per dwpe block (the norm's fused partials, beta = 0 only)
    const float z = warp_sum(q);
    if (threadIdx.x == 0) sq_wpe[b] = z;
  }
}

// ---------------------------------------------------------------- cross-entropy
// per row: (max, sum exp) over P partials (strided), optional lse, rowstat outputs.
// lse[row] = mx + log sum_p s_p * exp(m_p - mx) over P partial (max, sum exp) pairs at
// part[(row*srow + p*spart)*2].  Block = 16 rows x 16 partial lanes with the ROW on the fast lane
// index: for the part-major GEMM partials (srow 1, spart M) lanes 0-15 read 16 consecutive rows'
// pairs (one 128-B line) per partial — the one-wave-per-row mapping read 8 B per line.  Two passes
// (row max, then the rescaled sum), each combined over the 16 lanes in fixed order.
constexpr int CC_ROWS = 16, CC_LANES = 16, CC_REG = 56;
__global__ void __launch_bounds__(256) ce_combine_rows(const float* __restrict__ part, int M, int P, long srow, long spart,
                                                       float* __restrict__ lse_out, float* __restrict__ rowstat) {
  const int r = threadIdx.x % CC_ROWS, pl = threadIdx.x / CC_ROWS;
  const int row = blockIdx.x * CC_ROWS + r;
  DTC_ASSERT(P >= 1 && pl < CC_LANES && (long)blockIdx.x * CC_ROWS < M);
  __shared__ float red[CC_LANES][CC_ROWS];
  __shared__ float rmax[CC_ROWS];
  // P <= CC_LANES * CC_REG (GPT-2 small: 788 = 197 lm_head tiles x 4 wave columns): every partial of the thread
  // is loaded once, all
  // loads in flight together, and the sum pass reads the registers (the two global passes were latency-bound:
  // 21 us for 13 MB).  Same max / sum order as the two-pass form: bitwise identical.
  const bool in_reg = P <= CC_LANES * CC_REG;
  f32x2 qv[CC_REG];
  float mx = -INFINITY;
  if (row < M) {
    if (in_reg) {
#pragma unroll
      for (int k = 0; k < CC_REG; ++k) {
        const int p = pl + k * CC_LANES;
        qv[k] = p < P ? *(const f32x2*)(part + (row * srow + p * spart) * 2) : f32x2{-INFINITY, 0.f};
      }
#pragma unroll
      for (int k = 0; k < CC_REG; ++k) mx = fmaxf(mx, qv[k][0]);
    } else {
#pragma unroll 4
      for (int p = pl; p < P; p += CC_LANES) mx = fmaxf(mx, part[(row * srow + p * spart) * 2]);
    }
  }
  red[pl][r] = mx;
  __syncthreads();
  if (pl == 0) {
    float m = red[0][r];
#pragma unroll
    for (int q = 1; q < CC_LANES; ++q) m = fmaxf(m, red[q][r]);
    rmax[r] = m;
  }
  __syncthreads();
  mx = rmax[r];
  float s = 0.f;
  if (row < M) {
    if (in_reg) {
#pragma unroll
      for (int k = 0; k < CC_REG; ++k)
        if (qv[k][1] > 0.f) s += qv[k][1] * __expf(qv[k][0] - mx);
    } else {
#pragma unroll 4
      for (int p = pl; p < P; p += CC_LANES) {
        const f32x2 q = *(const f32x2*)(part + (row * srow + p * spart) * 2);
        if (q[1] > 0.f) s += q[1] * __expf(q[0] - mx);
      }
    }
  }
  __syncthreads();
  red[pl][r] = s;
  __syncthreads();
  if (pl == 0 && row < M) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < CC_LANES; ++q) t += red[q][r];
    if (lse_out) lse_out[row] = mx + __logf(t);
    if (rowstat) { rowstat[2 * row] = mx; rowstat[2 * row + 1] = t; }
  }
}

// loss = scale * sum_m (lse[m] - label_logit[m])  (one block, fixed reduction order)
__global__ void ce_loss_reduce(const float* __restrict__ lse, const float* __restrict__ lab, int M, float scale,
                               float* __restrict__ loss, int accumulate) {
  __shared__ float red[1024 / 64];
  // 8 independent loads in flight per thread (a one-load-per-iteration chain waited on each load:
  // 4.6 us for 8192 rows); fixed order: deterministic
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int nb = (int)blockDim.x;
  int m = threadIdx.x;
  for (; m + 7 * nb < M; m += 8 * nb) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += lse[m + k * nb] - lab[m + k * nb];
  }
  for (; m < M; m += nb) a[0] += lse[m] - lab[m];
  float s = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    loss[0] = (accumulate ? loss[0] : 0.f) + scale * t;
  }
}

// dlogits = (exp(l - lse) - onehot) * scale (common.h ce_grad8), in place, 8 bf16 per thread
__global__ void ce_bwd_kernel(bf16* __restrict__ logits, long ld, const float* __restrict__ lse,
                              const int* __restrict__ labels, int M, int V, int vstart, int n_valid, float scale) {
  const int V8 = V / 8;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * V8) return;
  int m = (int)(i / V8);
  int n = (int)(i % V8) * 8;
  DTC_ASSERT(m < M && n + 8 <= V && labels[m] >= 0);
  bf16x8* p = (bf16x8*)(logits + (long)m * ld + n);
  const bf16x8 v = *p;
  float g[8];
  ce_grad8(v, n, ce_row_c(lse[m], scale), labels[m] - vstart, n_valid, scale, g);
  bf16x8 o;
#pragma unroll
  for (int r = 0; r < 8; ++r) o[r] = f2bf(g[r]);
  *p = o;
}

// Same, plus per-column partial sums of dlogits (the lm_head bias gradient) over chunks of
// ce_rows() rows: colpart[chunk][V] (fp32, pre-rounding).  Grid (ceil(V/8/256), ceil(M/rows)):
// a thread walks `rows` rows of one 8-column group, so the 412 MB dlogits pass also yields
// db without a second read of it.
// DTC_CE_ROWS (default 128): rows per block of the CE backward = rows per column-partial slab; 128 halves
// the slabs the batched reduction reads (GPT-2 small 11.18-11.22 vs 11.22-11.25 ms with 64,
// profiles/r4_ab_ce_rows.log)
static int ce_rows() {
  static const int v = [] { const char* e = getenv("DTC_CE_ROWS"); return e ? std::max(8, atoi(e)) : 128; }();
  return v;
}
__global__ void __launch_bounds__(256) ce_bwd_colsum_kernel(bf16* __restrict__ logits, long ld,
                                                           const float* __restrict__ lse,
                                                           const int* __restrict__ labels, int M, int V, int vstart,
                                                           int n_valid, float scale, float* __restrict__ colpart,
                                                           int rows) {
  const int n = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (n >= V) return;
  const int m0 = blockIdx.y * rows, m1 = min(M, m0 + rows);
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  DTC_ASSERT(m0 < M && n + 8 <= V);
#pragma unroll 4
  for (int m = m0; m < m1; ++m) {
    bf16x8* p = (bf16x8*)(logits + (long)m * ld + n);
    const bf16x8 v = *p;
    float g[8];
    ce_grad8(v, n, ce_row_c(lse[m], scale), labels[m] - vstart, n_valid, scale, g);
    bf16x8 o;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      cs[r] += g[r];
      o[r] = f2bf(g[r]);
    }
    *p = o;
  }
  float* out = colpart + (long)blockIdx.y * V + n;
  *(f32x4*)out = f32x4{cs[0], cs[1], cs[2], cs[3]};
  *(f32x4*)(out + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
}

// fp32 logits (dtype: fp32 parity mode): dlogits in place + fp32 column partials, same structure
__global__ void __launch_bounds__(256) ce_bwd_colsum_f32_kernel(float* __restrict__ logits, long ld,
                                                               const float* __restrict__ lse,
                                                               const int* __restrict__ labels, int M, int V,
                                                               int vstart, int n_valid, float scale,
                                                               float* __restrict__ colpart, int rows) {
  const int n = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (n >= V) return;
  const int m0 = blockIdx.y * rows, m1 = min(M, m0 + rows);
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int m = m0; m < m1; ++m) {
    float* p = logits + (long)m * ld + n;
    const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
    const float l[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    float g[8];
    ce_grad8f(l, n, ce_row_c(lse[m], scale), labels[m] - vstart, n_valid, scale, g);
#pragma unroll
    for (int r = 0; r < 8; ++r) cs[r] += g[r];
    *(f32x4*)p = f32x4{g[0], g[1], g[2], g[3]};
    *(f32x4*)(p + 4) = f32x4{g[4], g[5], g[6], g[7]};
  }
  if (colpart) {
    float* out = colpart + (long)blockIdx.y * V + n;
    *(f32x4*)out = f32x4{cs[0], cs[1], cs[2], cs[3]};
    *(f32x4*)(out + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
  }
}

// ---------------------------------------------------------------- optimizer
constexpr int SS_BLOCKS = 1024;

// stage 1: per-block partial of sum_s w_s * sum x^2 over the segment table (float64 [S][3])
__global__ void __launch_bounds__(256) sumsq_stage1(const float* __restrict__ x, const double* __restrict__ seg, int S,
                                                    float* __restrict__ part) {
  float acc = 0.f;
  const long stride = (long)gridDim.x * blockDim.x;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (int s = 0; s < S; ++s) {
    const long off = (long)seg[3 * s], len = (long)seg[3 * s + 1];
    const float w = (float)seg[3 * s + 2];
    DTC_ASSERT(off >= 0 && len >= 0 && off % 4 == 0);
    float a = 0.f;
    const long len4 = len >> 2;  // ranges are 64-element aligned: 16-byte loads, 4 in flight
    const f32x4* x4 = (const f32x4*)(x + off);
    long i = tid;
    for (; i + 3 * stride < len4; i += 4 * stride) {
      f32x4 v0 = x4[i], v1 = x4[i + stride], v2 = x4[i + 2 * stride], v3 = x4[i + 3 * stride];
      f32x4 q = v0 * v0 + v1 * v1 + v2 * v2 + v3 * v3;
      a += (q[0] + q[1]) + (q[2] + q[3]);
    }
    for (; i < len4; i += stride) { f32x4 v = x4[i] * x4[i]; a += (v[0] + v[1]) + (v[2] + v[3]); }
    for (long j = (len4 << 2) + tid; j < len; j += stride) { float v = x[off + j]; a += v * v; }
    acc += w * a;
  }
  __shared__ float red[4];
  acc = warp_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void sumsq_stage2(const float* __restrict__ part, int P, float* __restrict__ out, int64_t* __restrict__ step) {
  __shared__ double red[16];
  // 8 independent loads in flight per thread (~16-20k partials: the one-load-per-iteration chain took
  // 10.5 us, on the critical path before the AdamW launch); fixed order: deterministic
  double c[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  const int nb = (int)blockDim.x;
  int i = threadIdx.x;
  for (; i + 7 * nb < P; i += 8 * nb) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = part[i + k * nb];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] += v[k];
  }
  for (; i < P; i += nb) c[0] += part[i];
  double a = ((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7]));
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    out[0] = (float)t;
    if (step) step[0] += 1;
  }
}

// clip-by-global-norm + AdamW (optax semantics), 4 elements per thread per grid-stride step; bf16
// mirror for i < n_mirror.  A full grid (one step) is the fastest standalone pass; a capped grid
// (dtc_adamw max_blocks) leaves most of each CU to concurrent work (the deferred optimizer runs beside
// the next step's forward GEMMs).
#ifndef DTC_ADAMW_CH
#define DTC_ADAMW_CH 2
#endif
template <bool STRIDE, int CH>
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, bf16* __restrict__ mirror, long n, long n_mirror,
                             const int64_t* __restrict__ step, const float* __restrict__ sumsq, float lr, float b1,
                             float b2, float eps, float wd, float max_norm, const float* __restrict__ enable) {
  // CH 4-element groups per thread, 1024 elements apart (the per-thread clip / bias-correction
  // prologue — a sqrt, two powf and a division — amortised over 4*CH elements)
  long i = (long)blockIdx.x * blockDim.x * 4 * CH + threadIdx.x * 4;
  if (!STRIDE && i >= n) return;
  if (enable && enable[0] == 0.f) return;  // deferred update already applied (or none pending)
  const float norm = sqrtf(sumsq[0]);
  const float clip = (max_norm > 0.f && !(norm < max_norm)) ? max_norm / norm : 1.f;
  const float t = (float)step[0];
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const long stride = STRIDE ? (long)gridDim.x * blockDim.x * 4 * CH : n;
  do {
    if (STRIDE && i >= n) break;
    // once-touched stream (2.7 GB per step): non-temporal loads/stores keep it out of L2/MALL
    // (measured 5.42 -> 5.345 ms/step)
    f32x4 pp[CH], gg[CH], mm[CH], vv[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const long j = i + (long)c * blockDim.x * 4;
      if (CH > 1 && j >= n) break;
      DTC_ASSERT(j + 4 <= n && n_mirror <= n);  // n % 4 == 0 (host-checked)
      pp[c] = __builtin_nontemporal_load((f32x4*)(p + j));
      gg[c] = __builtin_nontemporal_load((const f32x4*)(g + j));
      mm[c] = __builtin_nontemporal_load((f32x4*)(m + j));
      vv[c] = __builtin_nontemporal_load((f32x4*)(v + j));
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const long j = i + (long)c * blockDim.x * 4;
      if (CH > 1 && j >= n) break;
      // explicit fmaf: no contraction left to the compiler, so every launch shape (full grid,
      // capped grid, any CH) rounds identically
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gc = gg[c][r] * clip;
        mm[c][r] = fmaf(b1, mm[c][r], (1.f - b1) * gc);
        vv[c][r] = fmaf(b2, vv[c][r], ((1.f - b2) * gc) * gc);
        const float mh = mm[c][r] / bc1, vh = vv[c][r] / bc2;
        pp[c][r] = fmaf(-lr, fmaf(wd, pp[c][r], mh / (sqrtf(vh) + eps)), pp[c][r]);
      }
      __builtin_nontemporal_store(pp[c], (f32x4*)(p + j));
      __builtin_nontemporal_store(mm[c], (f32x4*)(m + j));
      __builtin_nontemporal_store(vv[c], (f32x4*)(v + j));
      if (j < n_mirror) *(bf16x4*)(mirror + j) = bf16x4{f2bf(pp[c][0]), f2bf(pp[c][1]), f2bf(pp[c][2]), f2bf(pp[c][3])};
    }
    i += stride;
  } while (STRIDE);
}

// ---- AdamW with the transposed bf16 mirror written by the update itself (DTC_ADAMW_TR) -------------------
// The weights that keep a transposed compute copy (fc1 / qkv / out_proj / lm_head: their dgrads run NT on
// W^T) are updated in 64 x 64 tiles whose bf16 values go through LDS into W^T as well, so the separate
// transpose pass (re-reading the fresh mirror: 72 us per GPT-2-small step) disappears; every other range of
// the flat buffer takes the element-wise update in one segmented launch.  Same per-element arithmetic as
// adamw_kernel (one shared function): p, m, v, the mirror and W^T are bitwise what the two-pass path writes.
__device__ __forceinline__ void adamw4(f32x4& p, const f32x4& g, f32x4& m, f32x4& v, float clip, float bc1, float bc2,
                                       float lr, float b1, float b2, float eps, float wd) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float gc = g[r] * clip;
    m[r] = fmaf(b1, m[r], (1.f - b1) * gc);
    v[r] = fmaf(b2, v[r], ((1.f - b2) * gc) * gc);
    const float mh = m[r] / bc1, vh = v[r] / bc2;
    p[r] = fmaf(-lr, fmaf(wd, p[r], mh / (sqrtf(vh) + eps)), p[r]);
  }
}

struct AwHyper {
  const int64_t* step;
  const float* sumsq;
  float lr, b1, b2, eps, wd, max_norm;
};
__device__ __forceinline__ void aw_prologue(const AwHyper& h, float& clip, float& bc1, float& bc2) {
  const float norm = sqrtf(h.sumsq[0]);
  clip = (h.max_norm > 0.f && !(norm < h.max_norm)) ? h.max_norm / norm : 1.f;
  const float t = (float)h.step[0];
  bc1 = 1.f - powf(h.b1, t);
  bc2 = 1.f - powf(h.b2, t);
}

constexpr int AW_MAX_SEG = 96;
struct AwSeg {
  long lo, n;   // flat range [lo, lo + n), 4-aligned
  int blk0, pad;
};
struct AwSegs {
  int nseg, nblocks;
  AwSeg s[AW_MAX_SEG];
};
// element-wise update of the segments (the ranges without a transposed copy), 4 x 4 elements per thread
__global__ void __launch_bounds__(256) adamw_seg_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        bf16* __restrict__ mirror, long n_mirror, AwSegs segs,
                                                        AwHyper h) {
  int lo = 0, hi = segs.nseg - 1;  // the segment whose block range holds blockIdx.x
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int)blockIdx.x >= segs.s[mid].blk0) lo = mid; else hi = mid - 1;
  }
  const AwSeg& S = segs.s[lo];
  float clip, bc1, bc2;
  aw_prologue(h, clip, bc1, bc2);
  const long base = S.lo + (long)(blockIdx.x - S.blk0) * 256 * 16;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const long j = base + (long)c * 1024 + threadIdx.x * 4;
    if (j >= S.lo + S.n) break;
    DTC_ASSERT(j + 4 <= S.lo + S.n);
    f32x4 pp = __builtin_nontemporal_load((f32x4*)(p + j)), gg = __builtin_nontemporal_load((const f32x4*)(g + j));
    f32x4 mm = __builtin_nontemporal_load((f32x4*)(m + j)), vv = __builtin_nontemporal_load((f32x4*)(v + j));
    adamw4(pp, gg, mm, vv, clip, bc1, bc2, h.lr, h.b1, h.b2, h.eps, h.wd);
    __builtin_nontemporal_store(pp, (f32x4*)(p + j));
    __builtin_nontemporal_store(mm, (f32x4*)(m + j));
    __builtin_nontemporal_store(vv, (f32x4*)(v + j));
    if (j < n_mirror) *(bf16x4*)(mirror + j) = bf16x4{f2bf(pp[0]), f2bf(pp[1]), f2bf(pp[2]), f2bf(pp[3])};
  }
}

constexpr int AWT_MAX = 64;
struct AwtTask {
  long off;     // flat offset of the [rows][cols] weight (its mirror sits at the same offset)
  bf16* dst;    // W^T [cols][rows]
  int rows, cols, blk0, pad;
};
struct AwtBatch {
  int ntasks, nblocks;
  AwtTask t[AWT_MAX];
};
// 64 x 64 tiles of the transposed-mirror weights: update, mirror, and W^T through an LDS tile
__global__ void __launch_bounds__(256) adamw_tr_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       bf16* __restrict__ mirror, AwtBatch b, AwHyper h) {
  int lo = 0, hi = b.ntasks - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int)blockIdx.x >= b.t[mid].blk0) lo = mid; else hi = mid - 1;
  }
  const AwtTask& T = b.t[lo];
  const int tcols = (T.cols + 63) / 64, bi = blockIdx.x - T.blk0;
  DTC_ASSERT(bi >= 0 && bi < ((T.rows + 63) / 64) * tcols && T.cols % 4 == 0 && T.rows % 8 == 0);
  const int r0 = (bi / tcols) * 64, c0 = (bi % tcols) * 64;
  __shared__ bf16 tile[64][64 + 1];  // row length 65: the column reads below spread over the banks
  float clip, bc1, bc2;
  aw_prologue(h, clip, bc1, bc2);
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // 64 rows x 16 groups of 4 columns: a row is 16 lanes x 16 B
    const int c = tid + 256 * i, r = c >> 4, c4 = (c & 15) * 4;
    bf16x4 o = {};
    if (r0 + r < T.rows && c0 + c4 + 4 <= T.cols) {
      const long j = T.off + (long)(r0 + r) * T.cols + c0 + c4;
      f32x4 pp = __builtin_nontemporal_load((f32x4*)(p + j)), gg = __builtin_nontemporal_load((const f32x4*)(g + j));
      f32x4 mm = __builtin_nontemporal_load((f32x4*)(m + j)), vv = __builtin_nontemporal_load((f32x4*)(v + j));
      adamw4(pp, gg, mm, vv, clip, bc1, bc2, h.lr, h.b1, h.b2, h.eps, h.wd);
      __builtin_nontemporal_store(pp, (f32x4*)(p + j));
      __builtin_nontemporal_store(mm, (f32x4*)(m + j));
      __builtin_nontemporal_store(vv, (f32x4*)(v + j));
      o = bf16x4{f2bf(pp[0]), f2bf(pp[1]), f2bf(pp[2]), f2bf(pp[3])};
      *(bf16x4*)(mirror + j) = o;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[r][c4 + e] = o[e];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // W^T rows = W columns, 8 x 16 B per row
    const int c = tid + i * 256, dr = c >> 3, ch = (c & 7) * 8;
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = tile[ch + e][dr];
    // non-temporal: W^T is read only in the backward (as transpose_batch_kernel's stores)
    if (c0 + dr < T.cols && r0 + ch + 8 <= T.rows)
      __builtin_nontemporal_store(o, (bf16x8*)(T.dst + (long)(c0 + dr) * T.rows + r0 + ch));
  }
}

__global__ void cast_kernel(const float* __restrict__ x, bf16* __restrict__ y, long n) {
  long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 4 <= n) {
    f32x4 v = *(const f32x4*)(x + i);
    *(bf16x4*)(y + i) = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
  } else {
    for (long j = i; j < n; ++j) y[j] = f2bf(x[j]);
  }
}

__global__ void zero4_kernel(f32x4* __restrict__ x, long n4) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) x[i] = f32x4{0.f, 0.f, 0.f, 0.f};
}

__global__ void fill_kernel(float* __restrict__ x, float v, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = v;
}

inline int blocks_for(long n, int per_block) { return (int)((n + per_block - 1) / per_block); }

// Batched bf16 transpose of weight matrices (the transposed compute mirror: the fc1 / qkv dgrads
// run as NT GEMMs on W^T, both operands K-major).  64x64 tiles through LDS: rows of the source and
// of the destination are read / written as 16-byte vectors.  Task t: src [rows][cols] -> dst
// [cols][rows], blocks [blk0, blk0 + ceil(rows/64) * ceil(cols/64)).
constexpr int TR_MAX_TASKS = 32;
struct TrTask {
  const bf16* src;
  bf16* dst;
  int rows, cols, blk0, pad;
};
struct TrBatch {
  int ntasks, nblocks;
  TrTask t[TR_MAX_TASKS];
};

__global__ void __launch_bounds__(256) transpose_batch_kernel(TrBatch batch) {
  int t = 0, hi = batch.ntasks - 1;  // binary search over the ascending blk0
  while (t < hi) {
    const int mid = (t + hi + 1) >> 1;
    if ((int)blockIdx.x >= batch.t[mid].blk0) t = mid;
    else hi = mid - 1;
  }
  const TrTask& T = batch.t[t];
  const int b = blockIdx.x - T.blk0;
  const int tcols = (T.cols + 63) / 64;
  DTC_ASSERT(b >= 0 && b < ((T.rows + 63) / 64) * tcols && (int)blockIdx.x < batch.nblocks);
  const int r0 = (b / tcols) * 64, c0 = (b % tcols) * 64;
  // row length 65: a column read (8 lanes per row group, rows 8 apart) lands rows 4 banks apart -> the 64
  // lanes cover 32 distinct banks (+8 padding: ~6 bank conflicts per LDS instruction under PMC).  Time-neutral
  // (18.6 vs 18.5-20.0 us per call): the kernel is bound by its 86 MB read + 86 MB write, not by LDS
  __shared__ bf16 tile[64][64 + 1];
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // 64 rows x 8 chunks of 8
    const int c = tid + i * 256, r = c >> 3, ch = (c & 7) * 8;
    bf16x8 v{};
    if (r0 + r < T.rows && c0 + ch + 8 <= T.cols) v = *(const bf16x8*)(T.src + (long)(r0 + r) * T.cols + c0 + ch);
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[r][ch + e] = v[e];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // destination rows = source columns
    const int c = tid + i * 256, dr = c >> 3, ch = (c & 7) * 8;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[ch + e][dr];
    // non-temporal: the transposed mirror is read only in the backward (cached stores measured slower,
    // profiles/r2_ab_nt_transpose.log)
    if (c0 + dr < T.cols && r0 + ch + 8 <= T.rows)
      __builtin_nontemporal_store(v, (bf16x8*)(T.dst + (long)(c0 + dr) * T.rows + r0 + ch));
  }
}

}  // namespace

extern "C" {

int dtc_version() { return 1; }

int dtc_embed_fwd(const int* ids, const float* wte, const float* wpe, float* h, int B, int T, int D, int V, float p,
                  long seed, const int64_t* step, long row0, hipStream_t st) {
  if (D % 4) return 3001;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(blocks_for((long)B * T, 4)), dim3(256), 0, st, ids, wte, wpe, h, B, T, D,
                     p, (uint32_t)seed, step, row0);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_embed_sort_bits(int n) {
  int nb = 1;
  while ((1 << nb) < n) ++nb;
  return nb;
}

// keys[n] (uint32) = sorted (id << nb | token); n <= 32768 and V <= 2^(32-nb)
int dtc_embed_sort(const int* ids, int n, int V, uint32_t* keys, hipStream_t st) {
  if (n <= 0 || n > SORT_MAX) return 3003;
  const int nb = dtc_embed_sort_bits(n);
  if (nb < 32 && (long)V > (1L << (32 - nb))) return 3004;
  int npad = 2;
  while (npad < n) npad <<= 1;
  hipLaunchKernelGGL(embed_sort_kernel, dim3(1), dim3(1024), 0, st, ids, n, npad, nb, keys);
  DTC_CHECK_LAUNCH();
  return 0;
}

// dwte (+)= scatter(ids, dropout'(dh)), dwpe (+)= sum_b dropout'(dh); keys from dtc_embed_sort,
// P = n*D fp32 scratch.  Bitwise deterministic.
// sq (optional; accumulate == 0): dtc_embed_sq_slots(B, T, D) sum-of-squares partials of the final dwte / dwpe
// values -- the gradient norm's share of the two tables without a pass over them (FusedAdamW fused partials)
long dtc_embed_sq_slots(int B, int T, int D) {
  const long dblk = (D / 4 + 63) / 64, nwpe = ((long)T * (D / 4) + 63) / 64;
  return (long)B * T * dblk + nwpe;
}

// prev_keys (optional, n entries, accumulate == 0 only): the keys of the previous call into this same dwte,
// whose rows are the only nonzero ones -- zeroed sparsely instead of the whole V x D table (GPT-2 small: at
// most 25 of 154 MB); prev_valid = 0 on the first call (full zeroing).  The call stores its own keys there.
int dtc_embed_bwd(const uint32_t* keys, const float* dh, float* dwte, float* dwpe, float* P, int B, int T, int D, int V,
                  float p, long seed, const int64_t* step, long row0, int accumulate, float* sq, uint32_t* prev_keys,
                  int prev_valid, hipStream_t st) {
  if (D % 4) return 3001;
  if ((sq || prev_keys) && accumulate) return 3005;
  const int n = B * T;
  if (n > SORT_MAX) return 3003;
  const int nb = dtc_embed_sort_bits(n);
  // piece length trades the sequential in-piece sum against the per-id walk over pieces
  const int piece = n <= 4096 ? 16 : (n <= 16384 ? 32 : 64);
  const int dblk = (D / 4 + 63) / 64;
  const int npieces = (n + piece - 1) / piece;
  // zero the table (beta = 0) with kernel blocks (not a memset node) in the same launch as the piece sums
  const long n4 = accumulate ? 0 : (long)V * D / 4;
  const bool sparse = prev_keys && prev_valid;
  const long nzero = sparse ? n : (n4 + EB_ZCH - 1) / EB_ZCH;
  const long nwpe = ((long)T * (D / 4) + 63) / 64;
  const long nblk = nzero + (long)npieces * dblk + nwpe;
  if (nblk > 0x7fffffffL) return 3004;
  hipLaunchKernelGGL(embed_bwd_stage1, dim3((unsigned)nblk), dim3(64), 0, st, keys, n, nb, piece, npieces, dblk, dh, P,
                     dwte, n4, (int)nzero, dwpe, B, T, D, p, (uint32_t)seed, step, row0, accumulate,
                     sq ? sq + (long)n * dblk : nullptr, sparse ? prev_keys : nullptr);
  DTC_CHECK_LAUNCH();
  hipLaunchKernelGGL(embed_segment_sum, dim3(n, dblk), dim3(64), 0, st, keys, n, nb, piece, P, dwte, D, accumulate, sq,
                     prev_keys);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_ce_combine(const float* part, int M, int P, long srow, long spart, const float* label_logit, float* lse_out,
                   float* rowstat_out, float loss_scale, float* loss_out, int accumulate, hipStream_t st) {
  float* lse = lse_out;
  if (loss_out && !lse) return 3002;
  hipLaunchKernelGGL(ce_combine_rows, dim3((M + CC_ROWS - 1) / CC_ROWS), dim3(256), 0, st, part, M, P, srow, spart, lse,
                     rowstat_out);
  DTC_CHECK_LAUNCH();
  if (loss_out) {
    hipLaunchKernelGGL(ce_loss_reduce, dim3(1), dim3(1024), 0, st, lse, label_logit, M, loss_scale, loss_out, accumulate);
    DTC_CHECK_LAUNCH();
  }
  return 0;
}

int dtc_ce_colsum_rows() { return ce_rows(); }

// colpart (optional): [ceil(M/ce_rows())][V] fp32 column partial sums of dlogits
int dtc_ce_bwd(bf16* logits, long ld, const float* lse, const int* labels, int M, int V, int vstart, int n_valid,
               float scale, float* colpart, hipStream_t st) {
  if (V % 8 || ld % 8) return 3003;
  if (colpart) {
    dim3 grid((V / 8 + 255) / 256, (M + ce_rows() - 1) / ce_rows());
    hipLaunchKernelGGL(ce_bwd_colsum_kernel, grid, dim3(256), 0, st, logits, ld, lse, labels, M, V, vstart, n_valid,
                       scale, colpart, ce_rows());
    DTC_CHECK_LAUNCH();
    return 0;
  }
  long n = (long)M * (V / 8);
  hipLaunchKernelGGL(ce_bwd_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, st, logits, ld, lse, labels, M, V, vstart,
                     n_valid, scale);
  DTC_CHECK_LAUNCH();
  return 0;
}

// fp32 logits: colpart (optional) [ceil(M/ce_rows())][V]
int dtc_ce_bwd_f32(float* logits, long ld, const float* lse, const int* labels, int M, int V, int vstart, int n_valid,
                   float scale, float* colpart, hipStream_t st) {
  if (V % 8 || ld % 4) return 3003;
  dim3 grid((V / 8 + 255) / 256, (M + ce_rows() - 1) / ce_rows());
  hipLaunchKernelGGL(ce_bwd_colsum_f32_kernel, grid, dim3(256), 0, st, logits, ld, lse, labels, M, V, vstart, n_valid,
                     scale, colpart, ce_rows());
  DTC_CHECK_LAUNCH();
  return 0;
}

long dtc_sumsq_workspace_bytes() { return SS_BLOCKS * 4; }

int dtc_sumsq_segments(const float* x, const double* seg, int S, float* out, int64_t* step, float* ws, long ws_bytes,
                       hipStream_t st) {
  if (ws_bytes < SS_BLOCKS * 4) return 3004;
  hipLaunchKernelGGL(sumsq_stage1, dim3(SS_BLOCKS), dim3(256), 0, st, x, seg, S, ws);
  DTC_CHECK_LAUNCH();
  hipLaunchKernelGGL(sumsq_stage2, dim3(1), dim3(1024), 0, st, ws, SS_BLOCKS, out, step);
  DTC_CHECK_LAUNCH();
  return 0;
}

// Incremental global norm: chunk i of the grads is reduced into part[0:nblocks] as soon as it
// is final (overlapping backward); dtc_sum_finish sums all chunk partials in a fixed order.
int dtc_sumsq_partial(const float* x, const double* seg, int S, float* part, int nblocks, hipStream_t st) {
  if (nblocks <= 0) return 3006;
  hipLaunchKernelGGL(sumsq_stage1, dim3(nblocks), dim3(256), 0, st, x, seg, S, part);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_sum_finish(const float* part, int P, float* out, int64_t* step, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_stage2, dim3(1), dim3(1024), 0, st, part, P, out, step);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_adamw(float* p, const float* g, float* m, float* v, bf16* mirror, long n, long n_mirror, const int64_t* step,
              const float* sumsq, float lr, float b1, float b2, float eps, float wd, float max_norm,
              const float* enable, int max_blocks, hipStream_t st) {
  if (n % 4 || n_mirror % 4) return 3005;
  const long blocks = blocks_for(n / 4, 256 * DTC_ADAMW_CH);
  if (max_blocks > 0 && blocks > max_blocks)  // capped grid, grid-stride over the rest
    hipLaunchKernelGGL((adamw_kernel<true, DTC_ADAMW_CH>), dim3(max_blocks), dim3(256), 0, st, p, g, m, v, mirror, n, n_mirror,
                       step, sumsq, lr, b1, b2, eps, wd, max_norm, enable);
  else  // DTC_ADAMW_CH 4-element groups per thread, one grid step
    hipLaunchKernelGGL((adamw_kernel<false, DTC_ADAMW_CH>), dim3(blocks), dim3(256), 0, st, p, g, m, v, mirror, n, n_mirror, step, sumsq, lr, b1, b2, eps, wd, max_norm, enable);
  DTC_CHECK_LAUNCH();
  return 0;
}

// fused AdamW + transposed mirror: segments (element-wise) and tiles (with W^T); the host builds both lists
int dtc_aw_max_seg() { return AW_MAX_SEG; }
int dtc_aw_max_tasks() { return AWT_MAX; }
int dtc_aw_seg_bytes() { return (int)sizeof(AwSeg); }
int dtc_aw_task_bytes() { return (int)sizeof(AwtTask); }
int dtc_adamw_tr(float* p, const float* g, float* m, float* v, bf16* mirror, long n_mirror, const AwSegs* segs,
                 const AwtBatch* tasks, const int64_t* step, const float* sumsq, float lr, float b1, float b2, float eps,
                 float wd, float max_norm, hipStream_t st) {
  if (segs->nseg > AW_MAX_SEG || tasks->ntasks > AWT_MAX || n_mirror % 4) return 3005;
  for (int i = 0; i < segs->nseg; ++i)
    if (segs->s[i].lo % 4 || segs->s[i].n % 4) return 3005;
  for (int i = 0; i < tasks->ntasks; ++i)
    if (tasks->t[i].rows % 8 || tasks->t[i].cols % 4 || tasks->t[i].off % 4) return 3011;
  const AwHyper h{step, sumsq, lr, b1, b2, eps, wd, max_norm};
  if (segs->nseg > 0 && segs->nblocks > 0) {
    hipLaunchKernelGGL(adamw_seg_kernel, dim3(segs->nblocks), dim3(256), 0, st, p, g, m, v, mirror, n_mirror, *segs, h);
    DTC_CHECK_LAUNCH();
  }
  if (tasks->ntasks > 0 && tasks->nblocks > 0) {
    hipLaunchKernelGGL(adamw_tr_kernel, dim3(tasks->nblocks), dim3(256), 0, st, p, g, m, v, mirror, *tasks, h);
    DTC_CHECK_LAUNCH();
  }
  return 0;
}

int dtc_tr_max_tasks() { return TR_MAX_TASKS; }
int dtc_tr_task_bytes() { return (int)sizeof(TrTask); }

// rows and cols must be multiples of 8 (16-byte vectors)
int dtc_transpose_batch(const TrBatch* b, hipStream_t st) {
  if (b->ntasks <= 0) return 0;
  if (b->ntasks > TR_MAX_TASKS) return 3010;
  for (int i = 0; i < b->ntasks; ++i)
    if (b->t[i].rows % 8 || b->t[i].cols % 8) return 3011;
  hipLaunchKernelGGL(transpose_batch_kernel, dim3(b->nblocks), dim3(256), 0, st, *b);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_cast_f32_bf16(const float* x, bf16* y, long n, hipStream_t st) {
  hipLaunchKernelGGL(cast_kernel, dim3(blocks_for((n + 3) / 4, 256)), dim3(256), 0, st, x, y, n);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_fill_f32(float* x, float v, long n, hipStream_t st) {
  hipLaunchKernelGGL(fill_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, st, x, v, n);
  DTC_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
