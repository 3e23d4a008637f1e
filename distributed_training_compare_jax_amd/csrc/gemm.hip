// bf16 MFMA GEMM for gfx950 with fused epilogues — every Dense of the GPT, fwd and bwd.
//
//   C[m,n] = epi( sum_k A(m,k) * B(n,k) )      fp32 accumulation
//   layout 0 (nt): A[m*lda+k], B[n*ldb+k]        forward   y  = x W^T       (W stored [out,in])
//   layout 1 (nn): A[m*lda+k], B[k*ldb+n]        dgrad     dX = dY W
//   layout 2 (tn): A[k*lda+m], B[k*ldb+n]        wgrad     dW = dY^T X
//
// CDNA4 design (see cdna_hip_programming.md §3, §5, T10, T14):
//  * 256 threads = 4 waves (2x2); each wave owns a (BM/2)x(BN/2) sub-tile of 16x16 MFMA tiles
//    (v_mfma_f32_16x16x32_bf16: measured ~1.15x the FLOP/s of 32x32x16 on random data).
//  * The MFMA's A operand is the GEMM's B side and vice versa, so the accumulator puts the
//    GEMM's m on the lane (lane&15) and 4 CONSECUTIVE n in a lane's 4 registers: epilogue
//    stores are 8-byte (bf16x4) / 16-byte (f32x4) vectors, bias is one float4.
//  * Register-staged, double-buffered LDS (T14: issue the global loads of tile k+1 before the
//    MFMAs of tile k, write LDS after them, one barrier per k-tile).
//  * K-contiguous operands: LDS rows padded to BK+8 (144 B rows) and read with two
//    ds_read_b64 per fragment (conflict-free: 144/4 = 36 spreads the 16 rows over all banks).
//  * M/N-contiguous operands (dgrad's W, wgrad's dY and X): stored k-major in LDS
//    ([BK][R+16], 288 B rows) and read with ds_read_b64_tr_b16, the gfx950 hardware
//    transpose read — no transposed copies of any tensor exist anywhere.
//  * Both operands use the same permuted k order inside an MFMA (element j of lane group g
//    holds k = 4g+j for j<4, 16+4g+(j-4) for j>=4), which makes both read kinds conflict-free.
//  * XCD-aware block remap (each XCD gets a contiguous run of tiles; M-tiles fastest so the
//    blocks sharing a weight panel share an L2).
//  * Split-K (fp32 slabs + deterministic reduce) for the small wgrad grids.
#include "common.h"
#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace {

constexpr int NT = 256;

template <int R, int BK, bool KMAJ>
struct Tile {
  // LDS row length (elements).  K-major: 160-B rows (40 dwords): a ds_read_b128 fragment read by 16
  // rows x 4 lane groups covers all 64 banks exactly once per 16-lane group (conflict-free).
  // MN-major: 288-B rows for R=128 / 160-B for R=64 (rows 8 apart stay 32 B apart in bank space,
  // conflict-free for ds_read_b64_tr_b16).
  static constexpr int LD = KMAJ ? (BK + 16) : (R + 16);
  static constexpr int ROWS = KMAJ ? R : BK;
  static constexpr int ELEMS = ROWS * LD;
  static constexpr int CHUNKS = R * BK / 8;  // 16-byte chunks in the tile
  static constexpr int PER_THREAD = CHUNKS / NT;
  static_assert(CHUNKS % NT == 0, "tile too small for 256 threads");

  // global -> registers through a buffer resource: branch-free, and any byte past the operand's
  // extent (rows/cols beyond M or N at a ragged edge) reads as 0 by the hardware range check.
  // Columns beyond the extent INSIDE a row (MN-major operand) only feed output rows/cols that
  // the epilogue never stores.
  __device__ __forceinline__ static void load(u32x4 (&reg)[PER_THREAD], __amdgpu_buffer_rsrc_t rs, long ld, int r0,
                                              int k0, int tid) {
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      int c = tid + i * NT;
      long off;
      if (KMAJ) {
        int row = c / (BK / 8), col = (c % (BK / 8)) * 8;
        off = ((long)(r0 + row) * ld + k0 + col) * 2;
      } else {
        int krow = c / (R / 8), col = (c % (R / 8)) * 8;
        off = ((long)(k0 + krow) * ld + r0 + col) * 2;
      }
      reg[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
    }
  }
  __device__ __forceinline__ static void store(const u32x4 (&reg)[PER_THREAD], bf16* lds, int tid) {
#pragma unroll
    for (int i = 0; i < PER_THREAD; ++i) {
      int c = tid + i * NT;
      if (KMAJ) {
        // k-permuted image: inside each 32-k group, the 8-byte segment a = k/4 (k = 4a..4a+3)
        // lands at element 8*(a&3) + 4*(a>>2), so lane group g's 8 fragment elements
        // (k = 4g..4g+3 and 16+4g..16+4g+3) are contiguous -> ONE ds_read_b128 per fragment
        int row = c / (BK / 8), col = (c % (BK / 8)) * 8;
        int grp = col & ~31, a0 = (col & 31) >> 2;  // a0 even: segments a0, a0+1
        bf16* rp = lds + row * LD + grp;
        // the a0 segments of every row fill one bank-pair set (mod 32) and the a0+1 segments the
        // other, and a ds_write_b64 lane group spans two rows: odd rows store their segments in
        // the opposite order, so each group of 16 lanes hits 16 distinct bank pairs (was 2-way)
        bf16* p0 = rp + 8 * (a0 & 3) + 4 * (a0 >> 2);
        bf16* p1 = rp + 8 * ((a0 + 1) & 3) + 4 * ((a0 + 1) >> 2);
        const u32x2 v0 = u32x2{reg[i][0], reg[i][1]}, v1 = u32x2{reg[i][2], reg[i][3]};
        const bool odd = row & 1;
        *(u32x2*)(odd ? p1 : p0) = odd ? v1 : v0;
        *(u32x2*)(odd ? p0 : p1) = odd ? v0 : v1;
      } else {
        int krow = c / (R / 8), col = (c % (R / 8)) * 8;
        *(u32x4*)(lds + krow * LD + col) = reg[i];
      }
    }
  }
  // MFMA fragment of 16-row tile t at k-chunk kk (32 k) in the permuted k order.
  __device__ __forceinline__ static bf16x8 frag(const bf16* lds, int t, int kk, int lane) {
    const int g = lane >> 4;
    if (KMAJ) {
      return *(const bf16x8*)(lds + (t * 16 + (lane & 15)) * LD + kk * 32 + 8 * g);
    } else {
      const int li = lane & 15, q = li >> 2, pp = li & 3;
      const bf16* p0 = lds + (kk * 32 + 4 * g + q) * LD + t * 16 + 4 * pp;
      const bf16* p1 = p0 + 16 * LD;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p1));
      return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  }
};

// Column sums of an MN-major operand tile held in registers (Tile::load layout): chunk
// c = tid + i*NT covers row c / (R/8) and the 8 columns 8*(c % (R/8)).., the same 8 columns for
// every i, so a thread accumulates 8 running sums (fused bias gradient of a wgrad GEMM).
template <int R, int PT>
__device__ __forceinline__ void colsum_acc(float (&cs)[8], const u32x4 (&reg)[PT]) {
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const bf16x8 v = __builtin_bit_cast(bf16x8, reg[i]);
#pragma unroll
    for (int j = 0; j < 8; ++j) cs[j] += (float)v[j];
  }
}

// Fixed-order block combine of colsum_acc sums -> out[0..R) (rows >= mlim skipped).  `red` is
// scratch LDS of (NT/(R/8)) * R floats; must be called by all threads after the main loop.
template <int R>
__device__ __forceinline__ void colsum_store(const float (&cs)[8], float* red, float* out, int mlim, int tid) {
  constexpr int CPR = R / 8, G = 256 / CPR;
  const int grp = tid / CPR, col = (tid % CPR) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[grp * R + col + j] = cs[j];
  __syncthreads();
  if (tid < R && tid < mlim) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) s += red[g * R + tid];
    out[tid] = s;
  }
}

// LayerNorm fused into a layer GEMM's epilogue (EPI_RESID_LN / EPI_LN_BWD; see ln_fwd_epilogue)
struct LnEpi {
  const float* gamma; const float* beta;
  bf16* y; float* mean; float* rstd;
  const float* x; float* part; int nslab;
  float eps;
  unsigned long long* sync; const long long* step; int site, nsites;
  unsigned* err;
};

struct Epi {
  int M, N;
  void* C; long ldc;
  const float* bias;
  const void* aux; long ldaux;
  void* aux_out;
  float alpha, beta;
  const int* labels; int vocab_start, n_valid;
  float* part; int nparts;
  float* label_out;
  float* colsum;
  int cs_accum;  // colsum IS the bias gradient: colsum[m] = beta*colsum[m] + sum (split == 1 only)
  float* sq;     // gemm8p_tile, fp32 store: per-wave sums of squares of the stored values (8 slots)
  int slab_tile; // gemm8p_tile split-K: slab = [split][BIG][64 CB] tile-local slabs instead of [split][M][N]
  LnEpi ln;
};

// Output stores of the GEMM epilogues: cached (every layer-GEMM output non-temporal measured slower for
// the outputs the next kernel reads, profiles/r2_ab_nt_stores.log; the few streamed outputs say so)
#define DTC_OUT_STORE(ptr, val) (*(ptr) = (val))

template <int EPI, bool OUTF32>
__device__ __forceinline__ float epilogue_store(const Epi& e, int m, int n, f32x4 v) {  // returns sum o^2 of fp32 stores
  DTC_ASSERT(m >= 0 && m < e.M && n >= 0 && n < e.N);
  const bool full = (n + 4 <= e.N);
  float b[4] = {0.f, 0.f, 0.f, 0.f};
  if (e.bias) {
    if (full) { f32x4 bb = *(const f32x4*)(e.bias + n); b[0] = bb[0]; b[1] = bb[1]; b[2] = bb[2]; b[3] = bb[3]; }
    else { for (int r = 0; r < 4; ++r) if (n + r < e.N) b[r] = e.bias[n + r]; }
  }
  float o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = e.alpha * v[r] + b[r];
  if (EPI == EPI_RESID) {
    const float* res = (const float*)e.aux + (long)m * e.ldaux + n;
    if (full) { f32x4 rr = *(const f32x4*)res; for (int r = 0; r < 4; ++r) o[r] += rr[r]; }
    else { for (int r = 0; r < 4; ++r) if (n + r < e.N) o[r] += res[r]; }
  }
  if (EPI == EPI_DGELU) {  // aux = gelu'(u), stored by the forward's EPI_GELU epilogue
    const bf16* u = (const bf16*)e.aux + (long)m * e.ldaux + n;
    if (full) { bf16x4 uu = *(const bf16x4*)u; for (int r = 0; r < 4; ++r) o[r] *= (float)uu[r]; }
    else { for (int r = 0; r < 4; ++r) if (n + r < e.N) o[r] *= (float)u[r]; }
  }
  if (EPI == EPI_STORE && OUTF32 && e.beta != 0.f) {
    const float* c = (const float*)e.C + (long)m * e.ldc + n;
    for (int r = 0; r < 4; ++r) if (n + r < e.N) o[r] += e.beta * c[r];
  }
  if (OUTF32) {
    float* c = (float*)e.C + (long)m * e.ldc + n;
    if (full) {
      DTC_OUT_STORE((f32x4*)c, (f32x4{o[0], o[1], o[2], o[3]}));
      return o[0] * o[0] + o[1] * o[1] + o[2] * o[2] + o[3] * o[3];
    }
    float ss = 0.f;
    for (int r = 0; r < 4; ++r)
      if (n + r < e.N) { c[r] = o[r]; ss += o[r] * o[r]; }
    return ss;
  } else {
    bf16* c = (bf16*)e.C + (long)m * e.ldc + n;
    bf16x4 gb;
    if (EPI == EPI_GELU) {  // C = gelu'(u) (the backward's dGELU factor), aux_out = gelu(u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float gv, dgv;
        gelu_tanh_and_grad_f(o[r], gv, dgv);
        o[r] = dgv;
        gb[r] = f2bf(gv);
      }
    }
    bf16x4 ob = {f2bf(o[0]), f2bf(o[1]), f2bf(o[2]), f2bf(o[3])};
    if (full) DTC_OUT_STORE((bf16x4*)c, ob);
    else for (int r = 0; r < 4; ++r) if (n + r < e.N) c[r] = ob[r];
    if (EPI == EPI_GELU) {
      bf16* g = (bf16*)e.aux_out + (long)m * e.ldc + n;
      if (full) DTC_OUT_STORE((bf16x4*)g, gb);
      else for (int r = 0; r < 4; ++r) if (n + r < e.N) g[r] = gb[r];
    }
  }
  return 0.f;
}


// Per-wave LDS staging of a bf16 (TM*16) x 64 output tile, so global stores go out as full
// 128-B rows (8 rows per instruction) instead of 16 rows x 32 B.  8-byte chunk c of row R sits
// at chunk c ^ (R & 15): fragment writes and row reads are both bank-conflict-free.
__device__ __forceinline__ void stage_put(bf16* st, int row, int chunk, bf16x4 v) {
  *(bf16x4*)(st + row * 64 + ((chunk ^ (row & 15)) << 2)) = v;
}

// NT: non-temporal stores (streamed past L2/MALL) for outputs no kernel reads soon: the 412 MB of
// logits, gelu'(u) (read in the backward).  Measured per kernel in the step: those gain (lm_head
// forward -19 us, and the CE backward reading after it -17 us), while outputs the NEXT kernel
// reads (qkv -> attention, dgrads -> LayerNorm backward) lose as much as their producer gains.
template <int ROWS, bool NT = false>
__device__ __forceinline__ void stage_out(const bf16* st, bf16* C, long ldc, int m_base, int n_base, int M, int N,
                                          int lane) {
  if (m_base + ROWS <= M && n_base + 64 <= N) {  // interior tile (wave-uniform): no per-row checks
#pragma unroll 4
    for (int it = 0; it < ROWS / 8; ++it) {
      const int row = it * 8 + (lane >> 3), p = lane & 7;
      u32x4 v = *(const u32x4*)(st + row * 64 + ((p ^ ((row >> 1) & 7)) << 3));
      if (row & 1) v = u32x4{v[2], v[3], v[0], v[1]};
      u32x4* dst = (u32x4*)(C + (long)(m_base + row) * ldc + n_base + p * 8);
      if (NT) __builtin_nontemporal_store(v, dst);
      else DTC_OUT_STORE(dst, v);
    }
    return;
  }
#pragma unroll 4
  for (int it = 0; it < ROWS / 8; ++it) {
    const int row = it * 8 + (lane >> 3), p = lane & 7;
    u32x4 v = *(const u32x4*)(st + row * 64 + ((p ^ ((row >> 1) & 7)) << 3));
    if (row & 1) v = u32x4{v[2], v[3], v[0], v[1]};
    const int m = m_base + row, n = n_base + p * 8;
    if (m >= M) continue;
    bf16* c = C + (long)m * ldc + n;
    if (n + 8 <= N) {
      if (NT) __builtin_nontemporal_store(v, (u32x4*)c);
      else DTC_OUT_STORE((u32x4*)c, v);
    } else {
      const bf16x8 b = __builtin_bit_cast(bf16x8, v);
      for (int r = 0; r < 8; ++r) if (n + r < N) c[r] = b[r];
    }
  }
}

// stage_out for a wave tile COLS (16, 32 or 64) columns wide in the same [ROWS][64] stage image: LPR = COLS/8
// lanes per row, 64/LPR rows per store instruction
// EDGE = false: the caller guarantees the tile lies inside M x N (no bounds code at all)
template <int ROWS, int COLS, bool NT = false, bool EDGE = true>
__device__ __forceinline__ void stage_out_w(const bf16* st, bf16* C, long ldc, int m_base, int n_base, int M, int N,
                                            int lane) {
  static_assert(COLS % 16 == 0 && COLS <= 64, "16-B pieces of a 64-column stage row");
  if constexpr (COLS == 64 && EDGE) {
    stage_out<ROWS, NT>(st, C, ldc, m_base, n_base, M, N, lane);
    return;
  }
  constexpr int LPR = COLS / 8, RPI = 64 / LPR;
  const bool interior = !EDGE || (m_base + ROWS <= M && n_base + COLS <= N);  // wave-uniform
#pragma unroll 4
  for (int it = 0; it < ROWS / RPI; ++it) {
    const int row = it * RPI + lane / LPR, p = lane % LPR;
    u32x4 v = *(const u32x4*)(st + row * 64 + ((p ^ ((row >> 1) & 7)) << 3));
    if (row & 1) v = u32x4{v[2], v[3], v[0], v[1]};
    const int m = m_base + row, n = n_base + p * 8;
    bf16* c = C + (long)m * ldc + n;
    if (interior || (m < M && n + 8 <= N)) {
      if (NT) __builtin_nontemporal_store(v, (u32x4*)c);
      else DTC_OUT_STORE((u32x4*)c, v);
    } else if (m < M) {
      const bf16x8 b = __builtin_bit_cast(bf16x8, v);
      for (int r = 0; r < 8; ++r) if (n + r < N) c[r] = b[r];
    }
  }
}

// the inverse: rows [m_base, +ROWS) x columns [n_base, +COLS) of a bf16 matrix into the stage image (zeros
// outside M x N), so fragment-order reads (stage_get) see it in the accumulator layout
template <int ROWS, int COLS, bool EDGE = true>
__device__ __forceinline__ void stage_in(const bf16* __restrict__ src, long ld, bf16* st, int m_base, int n_base,
                                         int M, int N, int lane) {
  constexpr int LPR = COLS / 8, RPI = 64 / LPR, NIT = ROWS / RPI, G = NIT < 4 ? NIT : 4;
  // groups of 4 rows-passes (4 x 16 B in flight per lane): the accumulators are live around this call
#pragma unroll 1
  for (int it0 = 0; it0 < NIT; it0 += G)
#pragma unroll
  for (int it = it0; it < it0 + G; ++it) {
    const int row = it * RPI + lane / LPR, p = lane % LPR;
    const int m = m_base + row, n = n_base + p * 8;
    u32x4 v = u32x4{0u, 0u, 0u, 0u};
    if (!EDGE || (m < M && n + 8 <= N)) {
      v = *(const u32x4*)(src + (long)m * ld + n);
    } else if (m < M) {
      bf16x8 b = {};
      for (int r = 0; r < 8; ++r) if (n + r < N) b[r] = src[(long)m * ld + n + r];
      v = __builtin_bit_cast(u32x4, b);
    }
    if (row & 1) v = u32x4{v[2], v[3], v[0], v[1]};
    *(u32x4*)(st + row * 64 + ((p ^ ((row >> 1) & 7)) << 3)) = v;
  }
}

// the 4 values of fragment (row, 8-byte chunk) as stage_put wrote them
__device__ __forceinline__ bf16x4 stage_get(const bf16* st, int row, int chunk) {
  return *(const bf16x4*)(st + row * 64 + ((chunk ^ (row & 15)) << 2));
}

// fp32 per-wave stage [ROWS][COLS] (COLS = 32 or 64): 16-B chunk c of row r at c ^ (r % (COLS/4)),
// conflict-free for the fragment writes (8 rows per lane group) and the row reads.  stage_out_f32
// writes whole rows (128/256 B per row, 8/4 rows per instruction) and adds the fp32 residual
// (`res`) or beta*C on the way out, in the same order as epilogue_store.
template <int COLS>
__device__ __forceinline__ void stage_put_f32(float* st, int row, int chunk, f32x4 v) {
  constexpr int CPR = COLS / 4;
  *(f32x4*)(st + row * COLS + ((chunk ^ (row & (CPR - 1))) << 2)) = v;
}

template <int ROWS, int COLS>
__device__ __forceinline__ void stage_out_f32(const float* st, float* C, long ldc, int m_base, int n_base, int M, int N,
                                              int lane, const float* res, long ldres, float beta) {
  constexpr int CPR = COLS / 4, RPI = 64 / CPR;
#pragma unroll 4
  for (int it = 0; it < ROWS / RPI; ++it) {
    const int row = it * RPI + lane / CPR, p = lane % CPR;
    f32x4 v = *(const f32x4*)(st + row * COLS + ((p ^ (row & (CPR - 1))) << 2));
    const int m = m_base + row, n = n_base + p * 4;
    if (m >= M || n >= N) continue;
    float* c = C + (long)m * ldc + n;
    if (n + 4 <= N) {
      if (res) v += *(const f32x4*)(res + (long)m * ldres + n);
      if (beta != 0.f) v += beta * *(const f32x4*)c;
      *(f32x4*)c = v;
    } else {
      for (int r = 0; r < 4; ++r)
        if (n + r < N) {
          float o = v[r];
          if (res) o += res[(long)m * ldres + n + r];
          if (beta != 0.f) o += beta * c[r];
          c[r] = o;
        }
    }
  }
}

// acc fragments (+ alpha/bias when `bias_on`) -> per-wave fp32 stage -> whole-row stores
template <int TN, int TM, int WM, int WN>
__device__ __forceinline__ void staged_f32_epilogue(const f32x4 (&acc)[TN][TM], float* stg, float* C, long ldc, int mb,
                                                    int nb, int M, int N, int lane, bool bias_on, float alpha,
                                                    const f32x4 (&bb)[TN], const float* res, long ldres, float beta) {
#pragma unroll
  for (int j = 0; j < TM; ++j)
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      f32x4 v = acc[i][j];
      if (bias_on) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = alpha * v[r] + bb[i][r];
      }
      stage_put_f32<WN>(stg, j * 16 + (lane & 15), i * 4 + (lane >> 4), v);
    }
  stage_out_f32<WM, WN>(stg, C, ldc, mb, nb, M, N, lane, res, ldres, beta);
}

// ---- LayerNorm fused into the layer GEMM epilogue (tp = pp = 1) ---------------------------------
// The GEMM that writes the fp32 residual stream x (out_proj / fc2 forward) also emits y = LN(x) in
// bf16 with the row mean / rstd, and the NT dgrad that produces a LayerNorm's output gradient dy
// (fc1 / qkv backward) finishes the LayerNorm backward itself (dy is never stored): one launch and
// one full [M, D] pass less per LayerNorm.  A row of D columns is spread over D/64 blocks (2 waves
// of 32 columns each), so the row statistics are exchanged INSIDE the launch
// (cdna_hip_programming.md Guideline 16, R1): every wave stores one packed pair of partials per
// (row, 32-column chunk) with write-through `sc1` stores (agent-scope relaxed atomics) and drains
// them (vmcnt(0)); after a block barrier one lane raises the block's flag = epoch; wave 0 of every
// block polls its row group's D/64 flags (one per lane, relaxed), and after a barrier every wave
// reads the partials with `sc1` loads only (no acquire fence needed).  The fp32 output stores are
// issued between publishing and waiting, so they drain while the row group catches up.
// epoch = step * nsites + site + 1 (device step counter, so it advances under hipGraph replay; sites
// numbered in execution order, so two consecutive uses of the shared buffer never carry the same tag).
// Liveness: the fused launches map blocks so that each XCD's dispatch order visits a row group's
// D/64 tiles consecutively, so a group only waits on blocks dispatched before any later group's;
// every spin is bounded (LN_SPIN_MAX): on a timeout the rows' statistics become NaN (so does the
// loss) and `err` is set, never a hang.
// Forward statistics: per-chunk mean and M2 = sum (x - mean_c)^2, combined with Chan's formula in a
// fixed order (bitwise reproducible, two-pass accuracy).
// sync layout (u64 words): partials [M][D/32] (lo = first, hi = second float), flags [M/128][D/64].
#ifndef LN_SPIN_MAX
#define LN_SPIN_MAX (1u << 17)
#endif
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) unsigned gu32_t;

__device__ __forceinline__ void pay_store(unsigned long long* p, float a, float b) {
  __hip_atomic_store((gu64_t*)p, ((unsigned long long)__float_as_uint(b) << 32) | __float_as_uint(a), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ f32x2 pay_load(const unsigned long long* p) {
  const unsigned long long u = __hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return f32x2{__uint_as_float((unsigned)u), __uint_as_float((unsigned)(u >> 32))};
}

// every wave's sc1 partial stores drained, then ONE lane raises this block's flag
__device__ __forceinline__ void ln_publish(unsigned long long* flag, unsigned epoch, int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_store((gu64_t*)flag, (unsigned long long)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 polls the row group's `n` flags (lane k <- flag k), the result is broadcast through LDS
__device__ __forceinline__ bool ln_wait_group(const unsigned long long* flags, int n, unsigned epoch, int* lds_ok,
                                              int wave, int lane) {
  if (wave == 0) {
    bool ok = false;
    for (unsigned spins = 0;; ++spins) {
      bool mine = true;
      if (lane < n)
        mine = (unsigned)__hip_atomic_load((gu64_t*)(flags + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      if (__all(mine)) {
        ok = true;
        break;
      }
      if (spins >= LN_SPIN_MAX) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0) *lds_ok = ok ? 1 : 0;
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below the poll
  return *lds_ok != 0;
}

__device__ __forceinline__ float sum8(float v) {  // over the 8 lanes of a row (xor butterfly: same in all 8)
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

__device__ __forceinline__ void ln_flag_error(const LnEpi& L, int lane) {
  if (lane == 0) __hip_atomic_store((gu32_t*)L.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// EPI_RESID_LN.  Wave tile WM x 32 (TM x 2 fragments).  Row pass as stage_out_f32: lane handles row
// it*8 + lane/8, columns 4*(lane%8) .. +3 of the wave's 32.
template <int TN, int TM, int WM, int WN, int WGM, int WGN>
__device__ __forceinline__ void ln_fwd_epilogue(const f32x4 (&acc)[TN][TM], float* stg, int* lds_ok, const Epi& e,
                                                int m0, int n0, int wm, int wn, int wave, int lane, int tid,
                                                const f32x4 (&bb)[TN]) {
  static_assert(WN == 32 && WM % 8 == 0, "LN epilogue: 32-column wave tiles");
  constexpr int IT = WM / 8;
  const LnEpi& L = e.ln;
  const int mb = m0 + wm * WM, nb = n0 + wn * WN;
  const int N = e.N, nch = N / 32, nq = nch / 8, chunk = nb / 32, tiles_n = N / (WN * WGN);
  const int rr = lane >> 3, p = lane & 7, n = nb + p * 4;
  const f32x4 gv = *(const f32x4*)(L.gamma + n), bv = *(const f32x4*)(L.beta + n);
  const unsigned epoch = (unsigned)(*L.step) * (unsigned)L.nsites + (unsigned)L.site + 1u;
  unsigned long long* pay = L.sync;
  unsigned long long* flags = L.sync + (long)e.M * nch + (long)(m0 / (WM * WGM)) * tiles_n;
#pragma unroll
  for (int j = 0; j < TM; ++j)
#pragma unroll
    for (int i = 0; i < TN; ++i) stage_put_f32<WN>(stg, j * 16 + (lane & 15), i * 4 + (lane >> 4), acc[i][j] + bb[i]);
  f32x4 xv[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int row = it * 8 + rr, m = mb + row;
    f32x4 v = *(const f32x4*)(stg + row * WN + ((p ^ (row & 7)) << 2));
    v += *(const f32x4*)((const float*)e.aux + (long)m * e.ldaux + n);
    xv[it] = v;
    const float mc = sum8((v[0] + v[1]) + (v[2] + v[3])) * (1.f / 32.f);
    const f32x4 d = v - mc;
    const float m2 = sum8((d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]));
    if (p == 0) pay_store(pay + (long)m * nch + chunk, mc, m2);
  }
  ln_publish(flags + n0 / (WN * WGN), epoch, tid);
#pragma unroll
  for (int it = 0; it < IT; ++it)  // the residual stream itself drains while the row group catches up
    *(f32x4*)((float*)e.C + (long)(mb + it * 8 + rr) * e.ldc + n) = xv[it];
  const bool ok = ln_wait_group(flags, tiles_n, epoch, lds_ok, wave, lane);
  if (!ok) ln_flag_error(L, lane);
  const float inv_nch = 1.f / (float)nch, inv_n = 1.f / (float)N;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int m = mb + it * 8 + rr;
    f32x2 pv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) pv[q] = q < nq ? pay_load(pay + (long)m * nch + p + 8 * q) : f32x2{0.f, 0.f};
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) if (q < nq) s += pv[q][0];
    const float mean = sum8(s) * inv_nch;
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < nq) {
        const float d = pv[q][0] - mean;
        t += fmaf(32.f * d, d, pv[q][1]);
      }
    float rstd = rsqrtf(sum8(t) * inv_n + L.eps);
    const float mu = ok ? mean : __builtin_nanf("");
    if (!ok) rstd = __builtin_nanf("");
    const f32x4 o = (xv[it] - mu) * rstd * gv + bv;
    *(bf16x4*)(L.y + (long)m * N + n) = __builtin_convertvector(o, bf16x4);
    if (chunk == 0 && p == 0) {
      L.mean[m] = mu;
      L.rstd[m] = rstd;
    }
  }
}

// EPI_LN_BWD: acc = dy (the LayerNorm's output gradient, never stored).  C = dres + LN'(dy) (fp32),
// ln.y = bf16 copy, and this block's column partials over its BM rows of dgamma = sum dy*xhat,
// dbeta = sum dy (and dbias = sum dx when nslab == 3) -> part[m0/BM][s][n].  `red`: LDS scratch of
// NW*3*32 floats past the per-wave stages.
template <int TN, int TM, int WM, int WN, int WGM, int WGN>
__device__ __forceinline__ void ln_bwd_epilogue(const f32x4 (&acc)[TN][TM], float* stg, float* red, int* lds_ok,
                                                const Epi& e, int m0, int n0, int wm, int wn, int wave, int lane,
                                                int tid) {
  static_assert(WN == 32 && WM % 8 == 0, "LN epilogue: 32-column wave tiles");
  constexpr int IT = WM / 8;
  const LnEpi& L = e.ln;
  const int mb = m0 + wm * WM, nb = n0 + wn * WN;
  const int N = e.N, nch = N / 32, nq = nch / 8, chunk = nb / 32, tiles_n = N / (WN * WGN);
  const int rr = lane >> 3, p = lane & 7, n = nb + p * 4;
  const f32x4 gv = *(const f32x4*)(L.gamma + n);
  const unsigned epoch = (unsigned)(*L.step) * (unsigned)L.nsites + (unsigned)L.site + 1u;
  unsigned long long* pay = L.sync;
  unsigned long long* flags = L.sync + (long)e.M * nch + (long)(m0 / (WM * WGM)) * tiles_n;
#pragma unroll
  for (int j = 0; j < TM; ++j)
#pragma unroll
    for (int i = 0; i < TN; ++i) stage_put_f32<WN>(stg, j * 16 + (lane & 15), i * 4 + (lane >> 4), acc[i][j]);
  f32x4 gd[IT], xh[IT];
  float rs[IT];
  f32x4 cg = {0.f, 0.f, 0.f, 0.f}, cb = cg, co = cg;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int row = it * 8 + rr, m = mb + row;
    const f32x4 dy = *(const f32x4*)(stg + row * WN + ((p ^ (row & 7)) << 2));
    const f32x4 xv = *(const f32x4*)(L.x + (long)m * N + n);
    rs[it] = L.rstd[m];
    xh[it] = (xv - L.mean[m]) * rs[it];
    gd[it] = dy * gv;
    cg += dy * xh[it];
    cb += dy;
    const float s1 = sum8((gd[it][0] + gd[it][1]) + (gd[it][2] + gd[it][3]));
    const f32x4 t2 = gd[it] * xh[it];
    const float s2 = sum8((t2[0] + t2[1]) + (t2[2] + t2[3]));
    if (p == 0) pay_store(pay + (long)m * nch + chunk, s1, s2);
  }
  ln_publish(flags + n0 / (WN * WGN), epoch, tid);
  const float* dres = (const float*)e.aux;
  f32x4 rv[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it)  // residual-gradient loads in flight while the row group catches up
    rv[it] = dres ? *(const f32x4*)(dres + (long)(mb + it * 8 + rr) * e.ldaux + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  const bool ok = ln_wait_group(flags, tiles_n, epoch, lds_ok, wave, lane);
  if (!ok) ln_flag_error(L, lane);
  const float inv_n = 1.f / (float)N;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int m = mb + it * 8 + rr;
    f32x2 pv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) pv[q] = q < nq ? pay_load(pay + (long)m * nch + p + 8 * q) : f32x2{0.f, 0.f};
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (q < nq) {
        a += pv[q][0];
        b += pv[q][1];
      }
    float c1 = sum8(a) * inv_n;
    const float c2 = sum8(b) * inv_n;
    if (!ok) c1 = __builtin_nanf("");
    const f32x4 o = (gd[it] - c1 - xh[it] * c2) * rs[it] + rv[it];
    *(f32x4*)((float*)e.C + (long)m * e.ldc + n) = o;
    *(bf16x4*)(L.y + (long)m * N + n) = __builtin_convertvector(o, bf16x4);
    co += o;
  }
  // column partials: over the wave's 4 row groups of 8 lanes (same p), then over the WGM waves along M
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      cg[r] += __shfl_xor(cg[r], o, 64);
      cb[r] += __shfl_xor(cb[r], o, 64);
      co[r] += __shfl_xor(co[r], o, 64);
    }
  }
  const int w = wm * WGN + wn;
  if (rr == 0) {
    *(f32x4*)(red + (w * 3 + 0) * 32 + p * 4) = cg;
    *(f32x4*)(red + (w * 3 + 1) * 32 + p * 4) = cb;
    *(f32x4*)(red + (w * 3 + 2) * 32 + p * 4) = co;
  }
  __syncthreads();
  const int nslab = L.nslab;
  if (tid < nslab * WGN * 32) {
    const int s = tid / (WGN * 32), c = tid % (WGN * 32), cw = c / 32, cc = c % 32;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < WGM; ++k) v += red[((k * WGN + cw) * 3 + s) * 32 + cc];
    L.part[((long)(m0 / (WM * WGM)) * nslab + s) * N + n0 + c] = v;
  }
}

// lm_head epilogue: logits (bf16) + per-row partial (max, sum exp) over this wave's TN*16 columns +
// the label logit.  acc[i][j]: lane holds C[m_base + 16j + (lane&15)][n_base + 16i + 4(lane>>4) + r].
// Epilogue operands loaded up front (all loads in flight together, ideally before the main loop
// ends): one bias vector per column group and one label per fragment row.
template <int TN, int TM>
struct EpiPre {
  f32x4 bb[TN];
  int lab[TM];                   // label of fragment row j*16 + (lane & 15)   (register epilogue)
  int labr[(TM * 16 + 63) / 64];  // label of wave row q*64 + lane               (LDS-staged epilogue)
};

template <int TN, int TM>
__device__ __forceinline__ void epi_prefetch(const Epi& e, int m_base, int n_base, int lane, bool labels,
                                             EpiPre<TN, TM>& pre) {
  const int g4 = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n_base + i * 16 + g4;
    pre.bb[i] = (e.bias && n + 4 <= e.N) ? *(const f32x4*)(e.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int m = m_base + j * 16 + (lane & 15);
    pre.lab[j] = (labels && m < e.M) ? e.labels[m] - e.vocab_start : -1;
  }
#pragma unroll
  for (int q = 0; q < (TM * 16 + 63) / 64; ++q) {
    const int m = m_base + q * 64 + lane;
    pre.labr[q] = (labels && m < e.M) ? e.labels[m] - e.vocab_start : -1;
  }
}

// Per-row (max, sum exp) of this wave's TN*16 logits + bf16 logits.  FULL: every column of the
// wave is a real vocab entry (all tiles but the last), so no per-element validity selects.  The
// staged form reads the label logit back from the LDS stage (one read per row) instead of
// comparing every element against the label, and folds (v - max)*log2(e) into one fma.
template <int TN, int TM, bool FULL, bool STAGED, bool ACCB>
__device__ __forceinline__ void lmhead_rows(const f32x4 (&acc)[TN][TM], const Epi& e, int m_base, int n_base,
                                            int part_idx, int lane, const EpiPre<TN, TM>& pre, bf16* stage) {
  constexpr float L2E = 1.4426950408889634f;
  const int g4 = 4 * (lane >> 4);
  bool okv[TN][4];
#pragma unroll
  for (int i = 0; i < TN; ++i) {  // validity: once per column group, shared by all TM rows
    const int n = n_base + i * 16 + g4;
#pragma unroll
    for (int r = 0; r < 4; ++r) okv[i][r] = FULL || ((n + r) < e.n_valid && (n + r) < e.N);
  }
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int m = m_base + j * 16 + (lane & 15);
    const bool mvalid = m < e.M;
    float v[TN][4];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = n_base + i * 16 + g4;
      bf16x4 ob = __builtin_convertvector(ACCB ? acc[i][j] : acc[i][j] + pre.bb[i], bf16x4);  // 2 cvt_pk
      const u32x2 pk = __builtin_bit_cast(u32x2, ob);  // the rounded logits back as f32: 1 op each
      const float rv[4] = {__uint_as_float(pk[0] << 16), __uint_as_float(pk[0] & 0xffff0000u),
                           __uint_as_float(pk[1] << 16), __uint_as_float(pk[1] & 0xffff0000u)};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[i][r] = okv[i][r] ? rv[r] : -INFINITY;
        mx = fmaxf(mx, v[i][r]);
      }
      if (!FULL) {
#pragma unroll
        for (int r = 0; r < 4; ++r) if (!okv[i][r]) ob[r] = f2bf(-INFINITY);
      }
      if (STAGED) {
        stage_put(stage, j * 16 + (lane & 15), i * 4 + (lane >> 4), ob);
      } else {
        if (mvalid && n + 4 <= e.N) *(bf16x4*)((bf16*)e.C + (long)m * e.ldc + n) = ob;
        const int lab = pre.lab[j];
        if (lab >= n && lab < n + 4 && lab < e.n_valid) e.label_out[m] = v[i][lab - n];
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
    if (FULL || mx != -INFINITY) {
      const float mxl = mx * L2E;
      sum = __builtin_amdgcn_exp2f(fmaf(v[0][0], L2E, -mxl));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int r = (i == 0); r < 4; ++r) sum += __builtin_amdgcn_exp2f(fmaf(v[i][r], L2E, -mxl));
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    // part-major [nparts][M]: the 16 rows of a fragment write one contiguous 128-B line
    if (mvalid && lane < 16) *(f32x2*)(e.part + ((long)part_idx * e.M + m) * 2) = f32x2{mx, sum};
  }
  if (STAGED) {
    // label logit: row q*64 + lane, if its label falls in this wave's columns (same wave wrote the
    // stage: LDS ops of one wave complete in order)
#pragma unroll
    for (int q = 0; q < (TM * 16 + 63) / 64; ++q) {
      const int row = q * 64 + lane, m = m_base + row, d = pre.labr[q] - n_base;
      if (row < TM * 16 && m < e.M && d >= 0 && d < TN * 16 && pre.labr[q] < e.n_valid)
        e.label_out[m] = (float)stage[row * 64 + ((((d >> 2) ^ (row & 15))) << 2) + (d & 3)];
    }
    stage_out<TM * 16, true>(stage, (bf16*)e.C, e.ldc, m_base, n_base, e.M, e.N, lane);  // logits: NT
  }
}

// lm_head epilogue: logits (bf16) + per-row partial (max, sum exp) over this wave's TN*16 columns +
// the label logit.  acc[i][j]: lane holds C[m_base + 16j + (lane&15)][n_base + 16i + 4(lane>>4) + r].
// Epilogue operands loaded up front (all loads in flight together, ideally before the main loop
// ends): one bias vector per column group and one label per fragment row.  ACCB: the accumulators
// started from the bias (the main loop added onto it), so no bias add here.
template <int TN, int TM, bool STAGED = false, bool ACCB = false>
__device__ __forceinline__ void lmhead_epilogue(const f32x4 (&acc)[TN][TM], const Epi& e, int m_base, int n_base,
                                                int part_idx, int lane, const EpiPre<TN, TM>& pre,
                                                bf16* stage = nullptr) {
  const bool full = n_base + TN * 16 <= min(e.n_valid, e.N);  // wave-uniform
  if (full) lmhead_rows<TN, TM, true, STAGED, ACCB>(acc, e, m_base, n_base, part_idx, lane, pre, stage);
  else lmhead_rows<TN, TM, false, STAGED, ACCB>(acc, e, m_base, n_base, part_idx, lane, pre, stage);
}

// LDS elements of the register-staged kernel (two stages of A and B tiles)
template <int BM, int BN, int BK, bool AK, bool BKM>
constexpr int gemm_smem_elems() { return 2 * (Tile<BM, BK, AK>::ELEMS + Tile<BN, BK, BKM>::ELEMS); }

// The register-staged GEMM tile program; `bid` is the block's id within ITS problem (so two
// problems can share one launch: gemm_pair_kernel) and `smem` its LDS.
template <int BM, int BN, int BK, bool AK, bool BKM, int EPI, bool OUTF32>
__device__ __forceinline__ void gemm_body(bf16* smem, int bid, const bf16* __restrict__ A, long lda, int a_bytes,
                                          const bf16* __restrict__ B, long ldb, int b_bytes, int M, int N, int K,
                                          int tiles_m, int tiles_n, int gm, int split, int k_per_split,
                                          float* __restrict__ slab, const Epi& e) {
  using TA = Tile<BM, BK, AK>;
  using TB = Tile<BN, BK, BKM>;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  constexpr int BUF = TA::ELEMS + TB::ELEMS;  // one stage: A tile then B tile

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = tiles_m * tiles_n;
  const int lid = xcd_remap(bid, ntiles * split);
  const int tile = lid % ntiles, z = lid / ntiles;
  // grouped tile order: groups of `gm` M-tiles sweep all N-tiles, so the run of tiles one XCD
  // receives touches few A rows AND few B columns (per-XCD L2 footprint; gm = tiles_m -> M fastest)
  const int grp = tile / (gm * tiles_n), in_g = tile % (gm * tiles_n);
  const int gm_eff = min(gm, tiles_m - grp * gm);
  const int tm_idx = grp * gm + in_g % gm_eff, tn_idx = in_g / gm_eff;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;
  DTC_ASSERT(tm_idx >= 0 && tn_idx >= 0 && z >= 0 && m0 < M && n0 < N);
  const int kbeg = z * k_per_split;
  const int nk = min(k_per_split, K - kbeg) / BK;

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, b_bytes, 0x00020000);
  auto compute = [&](const bf16* sAc) {
    const bf16* sBc = sAc + TA::ELEMS;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int j = 0; j < TM; ++j) fa[j] = TA::frag(sAc, wm * TM + j, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i) fb[i] = TB::frag(sBc, wn * TN + i, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
  };
  bf16* const s0 = smem;
  bf16* const s1 = smem + BUF;
  // dGELU epilogue operand u (bf16, the fragment layout): loaded before the main loop so its
  // latency hides under the MFMAs instead of stalling the epilogue (measured +8.6 us at fc2 dgrad)
  constexpr bool PRE_U = (EPI == EPI_DGELU) && (WN == 64);
  bf16x4 upre[PRE_U ? TN : 1][PRE_U ? TM : 1];
  if constexpr (PRE_U) {
    const int g4p = 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wm * WM + j * 16 + (lane & 15), n = n0 + wn * WN + i * 16 + g4p;
        upre[i][j] = (m < M && n + 4 <= N) ? *(const bf16x4*)((const bf16*)e.aux + (long)m * e.ldaux + n)
                                           : bf16x4{};
      }
  }
  // bias of the LDS-staged epilogues, loaded before the main loop for the same reason
#ifndef DTC_STAGE_STORE
#define DTC_STAGE_STORE 1  // plain bf16 stores through the LDS stage too
#endif
  constexpr bool STAGED = (EPI == EPI_GELU || EPI == EPI_DGELU || (DTC_STAGE_STORE && EPI == EPI_STORE)) && !OUTF32 &&
                          WN == 64;
#ifndef DTC_STAGE_F32
#define DTC_STAGE_F32 1  // fp32 outputs and split-K slabs through an fp32 LDS stage
#endif
  constexpr bool FIT32 = DTC_STAGE_F32 && (WN == 64 || WN == 32) &&
                         4 * WM * WN * 4 <= gemm_smem_elems<BM, BN, BK, AK, BKM>() * 2;  // stage fits the LDS
  constexpr bool STAGED32 = FIT32 && OUTF32 && (EPI == EPI_STORE || EPI == EPI_RESID);
  f32x4 bpre[(STAGED || STAGED32) ? TN : 1];
  if constexpr (STAGED || STAGED32) {
    const int g4p = 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = n0 + wn * WN + i * 16 + g4p;
      bpre[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (e.bias) {
        if (n + 4 <= N) bpre[i] = *(const f32x4*)(e.bias + n);
        else for (int r = 0; r < 4; ++r) if (n + r < N) bpre[i][r] = e.bias[n + r];
      }
    }
  }
  // fused bias gradient (wgrad only: MN-major A = dY, first N-tile column of blocks)
  const bool do_cs = !AK && e.colsum != nullptr && tn_idx == 0;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#ifndef DTC_DEEP_PREFETCH_MAX
#define DTC_DEEP_PREFETCH_MAX (64 * 64)  // 2-deep register prefetch for 128^2 tiles measured 5.99 vs 5.66 ms/step
#endif
  if constexpr (BM * BN <= DTC_DEEP_PREFETCH_MAX) {
    // small tiles (few MFMAs per k-step): 2-deep register prefetch.  While the MFMAs consume LDS
    // stage kt, tile kt+1's loads are a full k-step old and tile kt+2's are being issued (two
    // named register sets, no runtime-indexed register arrays -> no scratch; guide §5.4 rule 20).
    u32x4 ra0[TA::PER_THREAD], rb0[TB::PER_THREAD], ra1[TA::PER_THREAD], rb1[TB::PER_THREAD];
    TA::load(ra0, rsA, lda, m0, kbeg, tid);
    TB::load(rb0, rsB, ldb, n0, kbeg, tid);
    if (nk > 1) {
      TA::load(ra1, rsA, lda, m0, kbeg + BK, tid);
      TB::load(rb1, rsB, ldb, n0, kbeg + BK, tid);
    }
    TA::store(ra0, s0, tid);
    TB::store(rb0, s0 + TA::ELEMS, tid);
    if (do_cs) colsum_acc<BM, TA::PER_THREAD>(cs, ra0);
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      if (kt + 2 < nk) {
        TA::load(ra0, rsA, lda, m0, kbeg + (kt + 2) * BK, tid);
        TB::load(rb0, rsB, ldb, n0, kbeg + (kt + 2) * BK, tid);
      }
      compute(s0);
      if (kt + 1 < nk) {
        TA::store(ra1, s1, tid);
        TB::store(rb1, s1 + TA::ELEMS, tid);
        if (do_cs) colsum_acc<BM, TA::PER_THREAD>(cs, ra1);
      }
      __syncthreads();
      if (kt + 1 >= nk) break;
      if (kt + 3 < nk) {
        TA::load(ra1, rsA, lda, m0, kbeg + (kt + 3) * BK, tid);
        TB::load(rb1, rsB, ldb, n0, kbeg + (kt + 3) * BK, tid);
      }
      compute(s1);
      if (kt + 2 < nk) {
        TA::store(ra0, s0, tid);
        TB::store(rb0, s0 + TA::ELEMS, tid);
        if (do_cs) colsum_acc<BM, TA::PER_THREAD>(cs, ra0);
      }
      __syncthreads();
    }
  } else {
    // large tiles: one register set (T14: issue tile kt+1 before the MFMAs of tile kt, write it
    // to the other LDS stage after them; the co-resident block's MFMAs cover the rest)
    u32x4 ra[TA::PER_THREAD], rb[TB::PER_THREAD];
    TA::load(ra, rsA, lda, m0, kbeg, tid);
    TB::load(rb, rsB, ldb, n0, kbeg, tid);
    TA::store(ra, s0, tid);
    TB::store(rb, s0 + TA::ELEMS, tid);
    if (do_cs) colsum_acc<BM, TA::PER_THREAD>(cs, ra);
    // write-after-barrier (guide T14 as G15 writes it): tile kt+1, loaded one iteration ago, is
    // written at the top of iteration kt (its buffer was last read before the previous barrier)
    // and tile kt+2's loads go out right behind it, so each load has a whole compute phase AND a
    // barrier to land instead of the compute phase alone
    if (nk > 1) {
      TA::load(ra, rsA, lda, m0, kbeg + BK, tid);
      TB::load(rb, rsB, ldb, n0, kbeg + BK, tid);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      bf16* cur = (kt & 1) ? s1 : s0;
      bf16* nxt = (kt & 1) ? s0 : s1;
      if (kt + 1 < nk) {
        TA::store(ra, nxt, tid);
        TB::store(rb, nxt + TA::ELEMS, tid);
        if (do_cs) colsum_acc<BM, TA::PER_THREAD>(cs, ra);
        if (kt + 2 < nk) {
          TA::load(ra, rsA, lda, m0, kbeg + (kt + 2) * BK, tid);
          TB::load(rb, rsB, ldb, n0, kbeg + (kt + 2) * BK, tid);
        }
      }
      compute(cur);
      __syncthreads();
    }
  }
  if constexpr (!AK) {
    // do_cs is block-uniform, so the combine's barrier is reached by every thread of the block;
    // LDS is free after the main loop's final barrier
    if (do_cs) colsum_store<BM>(cs, (float*)smem, e.colsum + (long)z * M + m0, M - m0, tid);
  }

  // ---------------- epilogue: lane holds C[m = .. + (lane&15)][n = .. + 4*(lane>>4) + r]
  const int g4 = 4 * (lane >> 4);
  if (split > 1) {
    float* s = slab + (long)z * M * N;
    if constexpr (FIT32) {
      if (do_cs) __syncthreads();  // colsum_store's reads of LDS are done before it is reused
      const f32x4 nob[TN] = {};
      staged_f32_epilogue<TN, TM, WM, WN>(acc, (float*)smem + wave * (WM * WN), s, N, m0 + wm * WM, n0 + wn * WN, M, N,
                                          lane, false, 1.f, nob, nullptr, 0, 0.f);
      return;
    }
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        int m = m0 + wm * WM + j * 16 + (lane & 15);
        int n = n0 + wn * WN + i * 16 + g4;
        if (m < M) {
          float* c = s + (long)m * N + n;
          if (n + 4 <= N) *(f32x4*)c = acc[i][j];
          else for (int r = 0; r < 4; ++r) if (n + r < N) c[r] = acc[i][j][r];
        }
      }
    return;
  }
  if constexpr (STAGED32) {
    if (do_cs) __syncthreads();
    staged_f32_epilogue<TN, TM, WM, WN>(acc, (float*)smem + wave * (WM * WN), (float*)e.C, e.ldc, m0 + wm * WM,
                                        n0 + wn * WN, M, N, lane, true, e.alpha, bpre,
                                        EPI == EPI_RESID ? (const float*)e.aux : nullptr, e.ldaux,
                                        EPI == EPI_STORE ? e.beta : 0.f);
    return;
  }
  if (EPI == EPI_LMHEAD) {
    EpiPre<TN, TM> pre;
    epi_prefetch<TN, TM>(e, m0 + wm * WM, n0 + wn * WN, lane, true, pre);
    lmhead_epilogue<TN, TM>(acc, e, m0 + wm * WM, n0 + wn * WN, tn_idx * 2 + wn, lane, pre);
    return;
  }
  if constexpr (EPI == EPI_NONE) {  // microbenchmark: main loop only (keep the accumulators live)
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  if constexpr (STAGED) {
    // bf16 outputs through a per-wave LDS stage so global stores leave as full 128-B rows (the
    // fragment layout writes 16 rows x 32 B per instruction); LDS is free after the last barrier
    bf16* stg = smem + wave * (WM * 64);
    const int mb = m0 + wm * WM, nb = n0 + wn * WN;
    const f32x4(&bb)[TN] = bpre;
#pragma unroll
    for (int pass = 0; pass < (EPI == EPI_GELU ? 2 : 1); ++pass) {
#pragma unroll
      for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          bf16x4 ob;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = e.alpha * acc[i][j][r] + bb[i][r];
            if constexpr (EPI == EPI_GELU) {  // pass 0: C = gelu'(u), pass 1: aux_out = gelu(u)
              float gv, dgv;
              gelu_tanh_and_grad_f(v, gv, dgv);
              v = pass == 1 ? gv : dgv;
            }
            if constexpr (EPI == EPI_DGELU) v *= (float)upre[PRE_U ? i : 0][PRE_U ? j : 0][r];
            ob[r] = f2bf(v);
          }
          stage_put(stg, j * 16 + (lane & 15), i * 4 + (lane >> 4), ob);
        }
      // GELU pass 0 = gelu'(u), read only in the backward: non-temporal
      if (EPI == EPI_GELU && pass == 0) stage_out<WM, true>(stg, (bf16*)e.C, e.ldc, mb, nb, M, N, lane);
      else stage_out<WM>(stg, (bf16*)(pass == 0 ? e.C : e.aux_out), e.ldc, mb, nb, M, N, lane);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      int m = m0 + wm * WM + j * 16 + (lane & 15);
      int n = n0 + wn * WN + i * 16 + g4;
      if (m < M && n < N) epilogue_store<EPI, OUTF32>(e, m, n, acc[i][j]);
    }
}

template <int BM, int BN, int BK, bool AK, bool BKM, int EPI, bool OUTF32>
__global__ void __launch_bounds__(NT, 2)
gemm_kernel(const bf16* __restrict__ A, long lda, int a_bytes, const bf16* __restrict__ B, long ldb, int b_bytes, int M,
            int N, int K, int tiles_m, int tiles_n, int gm, int split, int k_per_split, float* __restrict__ slab, Epi e) {
  __shared__ __attribute__((aligned(16))) bf16 smem[gemm_smem_elems<BM, BN, BK, AK, BKM>()];
  gemm_body<BM, BN, BK, AK, BKM, EPI, OUTF32>(smem, blockIdx.x, A, lda, a_bytes, B, ldb, b_bytes, M, N, K, tiles_m,
                                               tiles_n, gm, split, k_per_split, slab, e);
}

// One register-staged problem, fully planned (operands, grid geometry, epilogue).
struct GemmLaunch {
  const bf16* A; long lda; int a_bytes;
  const bf16* B; long ldb; int b_bytes;
  int M, N, K, tiles_m, tiles_n, gm, split, kps, nblocks;
  float* slab;
  Epi e{};
};

template <int BM, int BN, int BK, bool AK, bool BKM, int EPI, bool OUTF32>
struct GemmCfg {
  static constexpr int SMEM = gemm_smem_elems<BM, BN, BK, AK, BKM>();
  __device__ __forceinline__ static void run(bf16* smem, int bid, const GemmLaunch& g) {
    gemm_body<BM, BN, BK, AK, BKM, EPI, OUTF32>(smem, bid, g.A, g.lda, g.a_bytes, g.B, g.ldb, g.b_bytes, g.M, g.N, g.K,
                                                 g.tiles_m, g.tiles_n, g.gm, g.split, g.kps, g.slab, g.e);
  }
};

// Two independent GEMMs in ONE launch (a layer's dgrad and weight gradient read the same dY):
// blocks [0, nb1) run problem 1, the rest problem 2.  Saves a dependent kernel boundary and lets
// the second problem's blocks fill the CUs the first one's last wave leaves idle.  nb1 % 8 == 0
// keeps both problems' XCD-aware tile maps (blockIdx % 8) intact.  `second_first`: problem 2's
// blocks take the low block ids instead (dispatched first), so the long split-K weight-gradient
// blocks start in the first round and the short whole-K dgrad tiles back-fill behind them.
template <class C1, class C2>
__global__ void __launch_bounds__(NT, 2) gemm_pair_kernel(GemmLaunch g1, GemmLaunch g2, int second_first) {
  __shared__ __attribute__((aligned(16))) bf16 smem[C1::SMEM > C2::SMEM ? C1::SMEM : C2::SMEM];
  const int b = blockIdx.x;
  if (second_first) {
    if (b < g2.nblocks) C2::run(smem, b, g2);
    else C1::run(smem, b - g2.nblocks, g1);
  } else {
    if (b < g1.nblocks) C1::run(smem, b, g1);
    else C2::run(smem, b - g1.nblocks, g2);
  }
}


// ============================================================================================
// 256x256 tile, 8 waves (2 along M x 4 along N, 128x64 per wave), for the lm_head-sized GEMMs
// (fwd [4096 x 50304 x 512], wgrad [50304 x 512 x 4096], dgrad [4096 x 512 x 50304]).  Why a
// second kernel: at 128^2 / 64x64-per-wave the LDS->VGPR traffic equals the MFMA rate
// (1/64+1/64 B per FLOP) and the L2->LDS traffic is 64 FLOP/B, so those tiles cap near ~40 % of
// peak; 128x64 per wave cuts LDS bytes/FLOP by 25 % and the 256^2 block halves L2 bytes/FLOP
// (measured main loop 1.0-1.3 PF/s).  1 block/CU (128 KB LDS), so staging is direct
// global->LDS DMA (global_load_lds_dwordx4, no staging VGPRs, cdna_hip_programming.md §5):
// tile k+1 streams into the other LDS buffer while the MFMAs consume tile k.
//  * K-major operand image: [256 rows][64 k] bf16 (128-B rows); 16-B chunk c of row r stored at
//    c ^ ((r>>1)&7).  MN-major image: [64 k][256 rows] (512-B rows); chunk c of k-row r stored at
//    c ^ mn_swz(r).  The DMA destination is lane-linear per wave, so the swizzle is applied on the
//    per-lane SOURCE address; every fragment read below is bank-conflict-free.
//  * Both operand kinds deliver the natural k order (K-major: one ds_read_b128 per fragment;
//    MN-major: two ds_read_b64_tr_b16 over k-rows 8g..8g+3 / 8g+4..8g+7), so any pairing works.
//  * Out-of-range rows/cols (ragged edges) are clamped to valid addresses: they only feed outputs
//    the epilogue never stores.  K (per split) must be a multiple of 64; MN-major extents % 8 == 0.
constexpr int NT2 = 512;
constexpr int BIG = 256;
constexpr int IMG = BIG * 64;  // elements per operand image

typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* glb_vptr;

// MN-major image swizzle: 16-B chunk c of k-row r lives at c ^ mn_swz(r).  The 8 k-rows one
// ds_read_b64_tr_b16 pass touches ({0-3, 8-11} + 16u, or +4) get 8 distinct 32-B bank windows.
__device__ __forceinline__ int mn_swz(int r) { return 2 * ((r & 3) | ((r >> 1) & 4)); }

template <bool KMAJ>
__device__ __forceinline__ void dma_tile(const bf16* __restrict__ X, long ldx, int r0, int rmax, int k0, bf16* img,
                                         int wave, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int blk = q * 8 + wave;  // one 1-KB DMA instruction per wave
    if (KMAJ) {                    // 8 rows x 128 B
      const int row = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      const int grow = min(r0 + row, rmax - 1);
      __builtin_amdgcn_global_load_lds((glb_vptr)(X + (long)grow * ldx + k0 + c * 8), (lds_vptr)(img + blk * 512), 16,
                                       0, 0);
    } else {                       // 2 k-rows x 512 B
      const int kr = blk * 2 + (lane >> 5);
      const int c = (lane & 31) ^ mn_swz(kr);
      const int col = min(r0 + c * 8, rmax - 8);
      __builtin_amdgcn_global_load_lds((glb_vptr)(X + (long)(k0 + kr) * ldx + col), (lds_vptr)(img + blk * 512), 16,
                                       0, 0);
    }
  }
}

// MFMA fragment of 16-row group t (0..15) at k-chunk kk (32 k), natural k order (lane group g
// holds k = 8g..8g+7): K-major = one ds_read_b128; MN-major = two ds_read_b64_tr_b16 over the
// k-rows 8g..8g+3 and 8g+4..8g+7 (the transpose hands lane i column i of the 4 rows).
template <bool KMAJ>
__device__ __forceinline__ bf16x8 big_frag(const bf16* img, int t, int kk, int lane) {
  const int g = lane >> 4, li = lane & 15;
  if (KMAJ) {
    const int row = t * 16 + li;
    return *(const bf16x8*)(img + row * 64 + (((kk * 4 + g) ^ ((row >> 1) & 7)) << 3));
  } else {
    const int q = li >> 2, pp = li & 3;
    const int k0 = kk * 32 + 8 * g + q, k1 = k0 + 4;
    const int c = 2 * t + (pp >> 1), w = (pp & 1) * 4;
    const bf16* p0 = img + k0 * 256 + ((c ^ mn_swz(k0)) << 3) + w;
    const bf16* p1 = img + k1 * 256 + ((c ^ mn_swz(k1)) << 3) + w;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p1));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  }
}

// ============================================================================================
// 256x256 tile, phase-interleaved ("ping-pong") main loop: the same tile, waves and epilogues as
// a plain 2-buffer 256^2 loop (the round-2 gemm256_kernel), with the staging pipeline rebuilt for ~1 block per CU
// (cdna_hip_programming.md §5 "The 256² 8-phase template", T3-T5):
//  * each K-step (64 k) is 4 phases; in phase p a wave ds-reads its A fragments of output rows
//    32p..32p+31 (+ all its B fragments at p = 0), issues 2 LDS-DMA instructions of the pipeline,
//    raw s_barrier, then 16 MFMAs between s_setprio(1)/(0), raw s_barrier.  The waves of the second
//    M half (waves 4-7, the other wave of each SIMD) run one barrier behind, so on every SIMD one
//    wave's MFMAs cover the other's LDS reads and DMA issue.
//  * operand images are 4 chunks of 64 contiguous rows (m or n) x 64 k: wave group wr reads A chunks
//    2wr (phases 0-1) and 2wr+1 (phases 2-3), wave column q reads B chunk q.  Contiguous chunks keep
//    every DMA source run a whole 128-B line for both operand kinds.
//    K-major chunk: [64 rows][64 k] (128-B rows, 16-B k-piece c of image row r at c ^ ((r>>1)&7),
//    the gemm256 image); MN-major chunk: [64 k][64 rows] (128-B k-rows, 16-B piece c of k-row r at
//    c ^ mn8_swz(r)).  Fragment reads of both kinds are bank-conflict-free.
//  * DMA schedule (2 per thread per phase): p0 A chunks 0,2 of K-step t+1, p1 A chunks 1,3 of t+1,
//    p2 B chunks 0,1 of t+2, p3 B chunks 2,3 of t+2.  Every region is re-staged >= 2 phases after its
//    last read (WAR: A chunks 0,2 are last read in phase 1, 1,3 in phase 3, B in phase 0).  Counted
//    waits (never vmcnt(0) in steady state) at the end of p0 (vmcnt 6: A chunks 1,3 of t landed) and
//    p2 (vmcnt 4: B and A chunks 0,2 of t+1): each retires data two phases before its first read,
//    which covers the half-phase stagger of the two wave groups.
constexpr int P8_CHUNK = 64 * 64;  // elements per operand chunk

__device__ __forceinline__ int mn8_swz(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

// one LDS-DMA instruction per wave: chunk q (rows 64q..64q+63) of an operand at k-step k0 -> img
template <bool KMAJ>
__device__ __forceinline__ void p8_dma(const bf16* __restrict__ X, long ldx, int r0, int rmax, int k0, bf16* img,
                                       int q, int wave, int lane) {
  if (KMAJ) {  // 8 image rows x 128 B
    const int r = wave * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int g = min(r0 + 64 * q + r, rmax - 1);
    __builtin_amdgcn_global_load_lds((glb_vptr)(X + (long)g * ldx + k0 + c * 8),
                                     (lds_vptr)(img + q * P8_CHUNK + wave * 512), 16, 0, 0);
  } else {  // 8 k-rows x 128 B
    const int kr = wave * 8 + (lane >> 3);
    const int pc = (lane & 7) ^ mn8_swz(kr);
    const int col = min(r0 + 64 * q + 8 * pc, rmax - 8);
    __builtin_amdgcn_global_load_lds((glb_vptr)(X + (long)(k0 + kr) * ldx + col),
                                     (lds_vptr)(img + q * P8_CHUNK + wave * 512), 16, 0, 0);
  }
}

// the per-lane source address p8_dma uses for chunk q at k0 = 0 (a K-step adds k0, or k0 * ldx
// for an MN-major operand): kernels that keep it in registers pay one add per DMA instruction
template <bool KMAJ>
__device__ __forceinline__ const bf16* p8_src(const bf16* __restrict__ X, long ldx, int r0, int rmax, int q, int wave,
                                              int lane) {
  if (KMAJ) {
    const int r = wave * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    return X + (long)min(r0 + 64 * q + r, rmax - 1) * ldx + c * 8;
  }
  const int kr = wave * 8 + (lane >> 3);
  const int pc = (lane & 7) ^ mn8_swz(kr);
  return X + (long)kr * ldx + min(r0 + 64 * q + 8 * pc, rmax - 8);
}

__device__ __forceinline__ void p8_dma_at(const bf16* src, bf16* img, int q, int wave) {
  __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(img + q * P8_CHUNK + wave * 512), 16, 0, 0);
}

// ds_read_b64_tr_b16 as inline asm: hipcc puts an s_waitcnt vmcnt(0) in front of every builtin
// transpose read while an LDS-DMA is in flight (it does not for ds_read_b128), which drained the
// whole DMA pipeline each phase of the MN-major kernels.  The compiler does not count these reads:
// their consumers sit behind p8_lgkm_wait, which waits lgkmcnt(0) and ties the fragment registers.
__device__ __forceinline__ s16x4 ds_tr16_asm(const bf16* p) {
  s16x4 r;
  const unsigned a = (unsigned)(unsigned long)(DTC_LDS void*)(p);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}

// fragment of 16-row group t (0..15: chunk t>>2, rows 16(t&3)..) at k-chunk kk, natural k order
template <bool KMAJ>
__device__ __forceinline__ bf16x8 p8_frag(const bf16* img, int t, int kk, int lane) {
  if (KMAJ) return big_frag<true>(img, t, kk, lane);
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const bf16* base = img + (t >> 2) * P8_CHUNK;
  const int k0 = kk * 32 + 8 * g + q, k1 = k0 + 4;
  const int pc = 2 * (t & 3) + (pp >> 1), w = (pp & 1) * 4;
  const bf16* p0 = base + k0 * 64 + ((pc ^ mn8_swz(k0)) << 3) + w;
  const bf16* p1 = base + k1 * 64 + ((pc ^ mn8_swz(k1)) << 3) + w;
  const s16x4 lo = ds_tr16_asm(p0), hi = ds_tr16_asm(p1);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// every LDS read of the phase has landed; the fragments are tied in so no consumer moves above it
__device__ __forceinline__ void p8_lgkm_wait(bf16x8 (&fa)[2][2], bf16x8 (&fb)[4][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fb[0][0]), "+v"(fb[0][1]),
                 "+v"(fb[1][0]), "+v"(fb[1][1]), "+v"(fb[2][0]), "+v"(fb[2][1]), "+v"(fb[3][0]), "+v"(fb[3][1])
               :
               : "memory");
}
__device__ __forceinline__ void p8_lgkm_wait(bf16x8 (&fa)[2][2], bf16x8 (&fb)[3][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fb[0][0]), "+v"(fb[0][1]),
                 "+v"(fb[1][0]), "+v"(fb[1][1]), "+v"(fb[2][0]), "+v"(fb[2][1])
               :
               : "memory");
}
__device__ __forceinline__ void p8_lgkm_wait(bf16x8 (&fa)[2][2], bf16x8 (&fb)[2][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fb[0][0]), "+v"(fb[0][1]),
                 "+v"(fb[1][0]), "+v"(fb[1][1])
               :
               : "memory");
}
__device__ __forceinline__ void p8_lgkm_wait(bf16x8 (&fa)[2][2], bf16x8 (&fb)[1][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fb[0][0]), "+v"(fb[0][1])
               :
               : "memory");
}

#define P8_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

template <int N>  // s_waitcnt vmcnt(N), N a compile-time count
__device__ __forceinline__ void vmcnt_c() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// CB = B chunks of 64 columns: 4 = the 256^2 tile; 3 = 256 x 192 (128 x 48 per wave) for the layer GEMMs
// whose N = 3072 makes exactly 2 rounds of 256 x 192 tiles (GPT-2 small fc1 forward / fc2 dgrad)
// One 256 x 64*CB output tile (tm_idx, tn_idx) of split z: the body of gemm8p_kernel and of the
// grouped weight-gradient kernel (gemm8p_group_kernel).  All LDS is the one array below.
// smem: the kernel's ONE LDS array, >= 2 * (4 + CB) * P8_CHUNK elements ([buf][A img | B img]); a kernel
// that runs tiles of two widths (gemm8r_kernel) passes the same array to both
template <bool AK, bool BKM, int EPI, bool OUTF32, int CB, bool EDGE = true>
__device__ __forceinline__ void gemm8p_tile_s(bf16* smem, const bf16* __restrict__ A, long lda,
                                              const bf16* __restrict__ B, long ldb, int M, int N, int K, int tm_idx,
                                              int tn_idx, int z, int split, int k_per_split, float* __restrict__ slab,
                                              const Epi& e) {
  constexpr int TM = 8, TN = CB;  // 16x16 fragments per wave: 128 (m) x 16*CB (n)
  constexpr int WN = 16 * CB;     // columns per wave
  static_assert(CB == 4 || (EPI != EPI_LMHEAD), "the CE epilogue assumes 64-column waves");
  static_assert(CB >= 1 && CB <= 4, "1..4 column chunks of 64");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;  // M half (= wave group), 64-column slice
  const int m0 = tm_idx * BIG, n0 = tn_idx * (64 * CB);
  DTC_ASSERT(tm_idx >= 0 && tn_idx >= 0 && z >= 0 && z < split && m0 < M && n0 < N);
  const int kbeg = z * k_per_split;
  const int nk = min(k_per_split, K - kbeg) / 64;
  DTC_ASSERT(nk >= 1);

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto imgA = [&](int t) { return smem + (t & 1) * (4 + CB) * P8_CHUNK; };
  auto imgB = [&](int t) { return smem + (t & 1) * (4 + CB) * P8_CHUNK + IMG; };
  auto dmaA = [&](int t, int q) { p8_dma<AK>(A, lda, m0, M, kbeg + t * 64, imgA(t), q, wave, lane); };
  auto dmaB = [&](int t, int q) { p8_dma<BKM>(B, ldb, n0, N, kbeg + t * 64, imgB(t), q, wave, lane); };

  // the 256^2 kernels (EDGE) prefetch the bias of a plain store with the LM-head operands; gemm8r's tiles load
  // it in the epilogue (16 fewer registers live through the main loop)
  constexpr bool PRE_BIAS = EDGE && CB == 4 && EPI == EPI_STORE && !OUTF32;
  EpiPre<TN, TM> pre;  // epilogue operands: loaded ahead of every DMA, retired by the prologue wait
  if (split == 1 && (EPI == EPI_LMHEAD || PRE_BIAS))
    epi_prefetch<TN, TM>(e, m0 + wr * 128, n0 + wc * WN, lane, EPI == EPI_LMHEAD, pre);
  // prologue: B(0), A(0), B(1) in flight; wait for the first two
#pragma unroll
  for (int q = 0; q < CB; ++q) dmaB(0, q);
#pragma unroll
  for (int q = 0; q < 4; ++q) dmaA(0, q);
  if (nk > 1) {
#pragma unroll
    for (int q = 0; q < CB; ++q) dmaB(1, q);
    vmcnt_c<CB>();
  } else {
    P8_VMCNT(0);
  }
  if (EPI == EPI_LMHEAD && split == 1) {  // the bias is the accumulators' starting value
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = pre.bb[i];
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // second wave group: one barrier behind

  // fused bias gradient of a weight-gradient GEMM (layout TN, e.colsum): column sums over K (tokens) of
  // the A operand = sum_k A(m, k) * 1, one MFMA of a ones B fragment per A fragment.  Only the n-tile-0
  // blocks; wave column wc takes the A fragments of phase p = wc (4 MFMAs per K-step per wave, +6 %), so
  // no wave lags the barriers.  Per split z: colsum[z * M + m] (summed in order by the caller's reducer).
  const bool do_cs = !AK && EPI == EPI_STORE && OUTF32 && e.colsum != nullptr && tn_idx == 0;
  const bf16x8 ones = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  f32x4 csacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  bf16x8 fb[TN][2], fa[2][2];
  for (int t = 0; t < nk; ++t) {
    const bf16* sA = imgA(t);
    const bf16* sB = imgB(t);
    const bool more1 = t + 1 < nk, more2 = t + 2 < nk;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // ---- load slot: fragments of this phase + 2 DMA instructions of the pipeline
      if (p == 0) {
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) fb[i][kk] = p8_frag<BKM>(sB, CB * wc + i, kk, lane);
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fa[jj][kk] = p8_frag<AK>(sA, 8 * wr + 2 * p + jj, kk, lane);
      if (p < 2) {
        if (more1) { dmaA(t + 1, p); dmaA(t + 1, p + 2); }
      } else {
        if (more2) {
          if (2 * p - 4 < CB) dmaB(t + 2, 2 * p - 4);
          if (2 * p - 3 < CB) dmaB(t + 2, 2 * p - 3);
        }
      }
      __builtin_amdgcn_s_barrier();
      p8_lgkm_wait(fa, fb);
      // ---- MFMA slot: output rows 32p..32p+31 of this wave's 128 x all 64 columns, K = 64
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            acc[i][2 * p + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i][kk], fa[jj][kk], acc[i][2 * p + jj], 0, 0, 0);
      if (do_cs && p == wc) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) csacc[jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, fa[jj][kk], csacc[jj], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      if (p == 0) {
        if (more1) vmcnt_c<CB + 2>(); else P8_VMCNT(0);  // A chunks 1,3 of t landed (B(t+1), A(t+1) 0,2 younger)
      } else if (p == 2) {
        // younger than A(t+1) chunks 0,2 and B(t+1): A(t+1) 1,3 + the B(t+2) chunks issued in phase 2
        if (more2) vmcnt_c<2 + (CB < 2 ? CB : 2)>(); else if (more1) P8_VMCNT(2); else P8_VMCNT(0);
      }
      __builtin_amdgcn_s_barrier();
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // balance the second group's extra barrier: LDS free after it

  const int g4 = 4 * (lane >> 4);
  if (do_cs && lane < 16) {  // every lane group holds the same sums (the ones operand)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int m = m0 + wr * 128 + (2 * wc + jj) * 16 + lane;
      if (m < M) {
        float v = csacc[jj][0];
        if (e.cs_accum && e.beta != 0.f) v += e.beta * e.colsum[m];  // grouped weight gradients: db itself
        e.colsum[(long)z * M + m] = v;
      }
    }
  }
  if (split > 1) {  // fp32 slab z; splitk_reduce (or wg_tail_reduce) sums the slabs in a fixed order
    if (e.slab_tile) {  // tile-local [split][BIG][64 CB] slab (grouped weight gradients' tail split)
      float* sl = slab + (long)z * BIG * (64 * CB);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int r = wr * 128 + j * 16 + (lane & 15), c = wc * WN + i * 16 + g4;
          if (m0 + r < M && n0 + c < N) *(f32x4*)(sl + (long)r * (64 * CB) + c) = acc[i][j];
        }
      return;
    }
    float* sl = slab + (long)z * M * N;
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wr * 128 + j * 16 + (lane & 15);
        const int n = n0 + wc * WN + i * 16 + g4;
        if (m < M && n < N) *(f32x4*)(sl + (long)m * N + n) = acc[i][j];  // N % 4 == 0 (checked by host)
      }
    return;
  }
  bf16* stage = smem + wave * (128 * 64);
  if constexpr (CB == 4 && EPI == EPI_LMHEAD) {
    lmhead_epilogue<TN, TM, true, true>(acc, e, m0 + wr * 128, n0 + wc * 64, tn_idx * 4 + wc, lane, pre, stage);
    return;
  }
  // staged bf16 epilogue: the 256^2 kernels' plain stores, gemm8r's plain, GELU-pair and dGELU stores
  constexpr bool STAGED = !OUTF32 && ((EPI == EPI_STORE && (CB == 4 || !EDGE)) ||
                                      (!EDGE && (EPI == EPI_DGELU || EPI == EPI_GELU)));
  if constexpr (STAGED) {
    // bf16 outputs through the wave's LDS stage (128 rows x 64 columns, WN of them used): whole-row
    // 16-B stores instead of 16 rows x 8 B per fragment store.  GELU: two passes (C = gelu'(u), then
    // aux_out = gelu(u)).  DGELU: the wave's u tile is staged first (row loads, fragment-order LDS reads)
    const int mb = m0 + wr * 128, nb = n0 + wc * WN;
    f32x4 bb[TN];
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = nb + i * 16 + g4;
      bb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (PRE_BIAS) {
        bb[i] = pre.bb[i];
        if (e.bias && n < N && n + 4 > N)
          for (int r = 0; r < 4; ++r) bb[i][r] = n + r < N ? e.bias[n + r] : 0.f;
      } else if (e.bias) {
        if (!EDGE || n + 4 <= N) bb[i] = *(const f32x4*)(e.bias + n);
        else for (int r = 0; r < 4; ++r) bb[i][r] = n + r < N ? e.bias[n + r] : 0.f;
      }
    }
    if constexpr (EPI == EPI_DGELU) {
      // the wave's u tile into its own stage (LDS ops of one wave complete in order: no barrier); each
      // fragment below reads its u values from the very slot its result then overwrites
      stage_in<128, WN, EDGE>((const bf16*)e.aux, e.ldaux, stage, mb, nb, M, N, lane);
    }
    if constexpr (EPI == EPI_GELU) {
      // two halves of 64 rows: the pair (gelu'(u), gelu(u)) of each fragment computed once and staged as
      // stage rows [0, 64) and [64, 128), then both 64-row slabs stored (two full passes over the 128
      // accumulators spilled: the compiler kept the first pass's GELU values for the second)
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
        for (int jj = 0; jj < TM / 2; ++jj)
#pragma unroll
          for (int i = 0; i < TN; ++i) {
            const int j = hf * (TM / 2) + jj;
            bf16x4 od, og;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float gv, dgv;
              gelu_tanh_and_grad_f(e.alpha * acc[i][j][r] + bb[i][r], gv, dgv);
              od[r] = f2bf(dgv);
              og[r] = f2bf(gv);
            }
            stage_put(stage, jj * 16 + (lane & 15), i * 4 + (lane >> 4), od);
            stage_put(stage, 64 + jj * 16 + (lane & 15), i * 4 + (lane >> 4), og);
            __builtin_amdgcn_sched_barrier(0);
          }
        // gelu'(u) is read only in the backward: non-temporal
        stage_out_w<64, WN, true, EDGE>(stage, (bf16*)e.C, e.ldc, mb + hf * 64, nb, M, N, lane);
        stage_out_w<64, WN, false, EDGE>(stage + 64 * 64, (bf16*)e.aux_out, e.ldc, mb + hf * 64, nb, M, N, lane);
      }
      return;
    }
#pragma unroll
    for (int pass = 0; pass < 1; ++pass) {
#pragma unroll
      for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          bf16x4 ob, uf = {};
          if constexpr (EPI == EPI_DGELU) uf = stage_get(stage, j * 16 + (lane & 15), i * 4 + (lane >> 4));
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = e.alpha * acc[i][j][r] + bb[i][r];
            if constexpr (EPI == EPI_GELU) {
              float gv, dgv;
              gelu_tanh_and_grad_f(v, gv, dgv);
              v = pass == 1 ? gv : dgv;
            }
            if constexpr (EPI == EPI_DGELU) v *= (float)uf[r];
            ob[r] = f2bf(v);
          }
          stage_put(stage, j * 16 + (lane & 15), i * 4 + (lane >> 4), ob);
          // GELU / dGELU: one fragment at a time (the scheduler otherwise interleaves all 32 fragments' GELU
          // temporaries or u reads next to the 128 accumulator registers and spills)
          if constexpr (EPI == EPI_DGELU || EPI == EPI_GELU) __builtin_amdgcn_sched_barrier(0);
        }
      if (EPI == EPI_GELU && pass == 0) stage_out_w<128, WN, true, EDGE>(stage, (bf16*)e.C, e.ldc, mb, nb, M, N, lane);
      else stage_out_w<128, WN, false, EDGE>(stage, (bf16*)(pass == 0 ? e.C : e.aux_out), e.ldc, mb, nb, M, N, lane);
    }
    return;
  }
  if (EPI == EPI_NONE) {  // microbenchmark: main loop only (keep the accumulators live)
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      int m = m0 + wr * 128 + j * 16 + (lane & 15);
      int n = n0 + wc * WN + i * 16 + g4;
      if (m < M && n < N) ss += epilogue_store<EPI, OUTF32>(e, m, n, acc[i][j]);
    }
  if (OUTF32 && e.sq) {  // grad-norm partial of this wave's part of the tile: one slot per wave, no barrier
    ss = warp_sum(ss);     // (a block-wide sum needed a __syncthreads that waited for every store: +70 us)
    if (lane == 0) e.sq[wave] = ss;
  }
}

template <bool AK, bool BKM, int EPI, bool OUTF32, int CB>
__device__ __forceinline__ void gemm8p_tile(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb,
                                            int M, int N, int K, int tm_idx, int tn_idx, int z, int split,
                                            int k_per_split, float* __restrict__ slab, const Epi& e) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (4 + CB) * P8_CHUNK];  // the only LDS object
  gemm8p_tile_s<AK, BKM, EPI, OUTF32, CB>(smem, A, lda, B, ldb, M, N, K, tm_idx, tn_idx, z, split, k_per_split, slab,
                                          e);
}

template <bool AK, bool BKM, int EPI, bool OUTF32, int CB = 4>
__global__ void __launch_bounds__(NT2, 1)
gemm8p_kernel(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, int M, int N, int K,
              int tiles_m, int tiles_n, int gm, int split, int k_per_split, float* __restrict__ slab, Epi e) {
  const int ntiles = tiles_m * tiles_n;
  const int lid = xcd_remap(blockIdx.x, ntiles * split);
  const int tile = lid % ntiles, z = lid / ntiles;
  const int grp = tile / (gm * tiles_n), in_g = tile % (gm * tiles_n);
  const int gm_eff = min(gm, tiles_m - grp * gm);
  const int tm_idx = grp * gm + in_g % gm_eff, tn_idx = in_g / gm_eff;
  gemm8p_tile<AK, BKM, EPI, OUTF32, CB>(A, lda, B, ldb, M, N, K, tm_idx, tn_idx, z, split, k_per_split, slab, e);
}

// ============================================================================================
// gemm8r: the 256-row tiles of gemm8p_kernel in ONE launch of two column widths, for the layer GEMMs
// whose 256^2 grid is a full round plus a remainder (GPT-2 small at 8192 tokens: qkv forward 288 tiles =
// 1.125 rounds, fc1 forward / fc2 NT dgrad 384 = 1.5 rounds) or less than a round (N = 768: 96 tiles):
// columns [0, n_split) run as 256 x 256 tiles (whole rounds of 256 blocks), columns [n_split, N) as
// 256 x 64*CB2 tiles, sized so the remainder is at most one round of narrower tiles.  The remainder
// blocks take the higher block ids: the hardware dispatches them as the CUs of the first round free up.
// No cross-block exchange (no split-K slabs): every output element is summed in one block in K order.
// One LDS array for both widths (the 256^2 tile's 128 KB).
struct R8Args {
  const bf16* A; long lda;
  const bf16* B; long ldb;
  int M, N, K, n_split;
  int tm, tn1, gm1, nb1;  // part 1: tiles_m x tn1 tiles of 256 x 256 (nb1 blocks)
  int tn2, gm2;           // part 2: tiles_m x tn2 tiles of 256 x 64*CB2
  int ilv;                // 1: interleaved block order (below)
};

// Block -> (part, logical tile).  ilv = 0: all 256^2 tiles, then the narrow ones.  ilv = 1 (DTC_R8_ILV):
// [first half of the 256^2 tiles | first half of the narrow ones | second half of each]: the first
// dispatch round then holds both widths, the CUs that drew a narrow tile go on to a 256^2 one and the
// others to a narrow one, so the CUs end their tiles at staggered times and each epilogue's store burst
// overlaps other CUs' main loops instead of the whole chip storing at once.
__device__ __forceinline__ void r8_block(const R8Args& a, int b, int nb2, bool& big, int& lid) {
  if (!a.ilv) {
    big = b < a.nb1;
    lid = big ? xcd_remap(b, a.nb1) : xcd_remap(b - a.nb1, nb2);
    return;
  }
  const int h1 = a.nb1 / 2, h2 = nb2 / 2;
  if (b < h1) { big = true; lid = xcd_remap(b, h1); return; }
  b -= h1;
  if (b < h2) { big = false; lid = xcd_remap(b, h2); return; }
  b -= h2;
  if (b < a.nb1 - h1) { big = true; lid = h1 + xcd_remap(b, a.nb1 - h1); return; }
  b -= a.nb1 - h1;
  big = false;
  lid = h2 + xcd_remap(b, nb2 - h2);
}

template <bool AK, bool BKM, int EPI, bool OUTF32, int CB2>
__global__ void __launch_bounds__(NT2, 1) gemm8r_kernel(R8Args a, Epi e) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * (4 + 4) * P8_CHUNK];  // the only LDS object
  const int b = (int)blockIdx.x;
  auto order = [](int lid, int tm, int tn, int gm, int& tm_idx, int& tn_idx) {
    const int grp = lid / (gm * tn), in_g = lid % (gm * tn);
    const int gm_eff = min(gm, tm - grp * gm);
    tm_idx = grp * gm + in_g % gm_eff;
    tn_idx = in_g / gm_eff;
  };
  int tm_idx, tn_idx;
  const int nb2 = a.tm * a.tn2;
  bool big;
  int lid;
  r8_block(a, b, nb2, big, lid);
  if (big) {
    order(lid, a.tm, a.tn1, a.gm1, tm_idx, tn_idx);
    Epi e1 = e;
    e1.N = a.n_split;
    gemm8p_tile_s<AK, BKM, EPI, OUTF32, 4, false>(smem, a.A, a.lda, a.B, a.ldb, a.M, a.n_split, a.K, tm_idx, tn_idx,
                                                   0, 1, a.K, nullptr, e1);
    return;
  }
  order(lid, a.tm, a.tn2, a.gm2, tm_idx, tn_idx);
  // part 2 as its own problem: columns n_split.. of B / C / bias / aux
  const int ns = a.n_split;
  Epi e2 = e;
  e2.N = a.N - ns;
  e2.C = OUTF32 ? (void*)((float*)e.C + ns) : (void*)((bf16*)e.C + ns);
  if (e.bias) e2.bias = e.bias + ns;
  if (e.aux) e2.aux = (const void*)((const bf16*)e.aux + ns);
  if (e.aux_out) e2.aux_out = (void*)((bf16*)e.aux_out + ns);
  const bf16* B2 = BKM ? a.B + (long)ns * a.ldb : a.B + ns;
  gemm8p_tile_s<AK, BKM, EPI, OUTF32, CB2, false>(smem, a.A, a.lda, B2, a.ldb, a.M, a.N - ns, a.K, tm_idx, tn_idx, 0,
                                                   1, a.K, nullptr, e2);
}

// Grouped weight gradients: dW_i = beta*dW_i + dY_i^T X_i (+ db_i = beta*db_i + colsum(dY_i)) for up to
// WG_MAX problems that share K (the tokens) in ONE launch of whole 256^2 tiles (no split-K, no fp32
// slabs, no reduction pass).  The backward defers every layer's four weight gradients to here: at
// K = 8192 tokens a layer's four GEMMs are only 108 tiles, which used to need split-K x 7 across the
// CUs plus a 400 MB/layer slab reduction (profiles/r3_gpt2_small_profile_final.md: 3.6 ms of a
// 13.2 ms step); twelve layers together are 1296 whole tiles, ~5 rounds of 256 CUs.
// Block -> (problem, tile): XCD-remapped logical id, problems back to back, M-tiles fastest (the
// blocks an XCD runs together share the X panel of one N-tile).
// Tail split (b.tail_tiles > 0): the grid's last blocks are K-pieces of the last tail_tiles logical tiles,
// so the final, partly filled round of whole tiles (GPT-2 small: 1887 tiles = 7 rounds + 95) becomes
// tail_split times as many blocks of 1/tail_split the length; wg_tail_reduce finishes those tiles.
// entry of logical tile lid: binary search over the ascending tile0 (a linear scan was up to ~50 dependent
// scalar loads of the kernel argument at every block's start)
__device__ __forceinline__ const WgEntry& wg_entry(const WgBatch& b, int lid) {
  int lo = 0, hi = b.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (lid >= b.e[mid].tile0) lo = mid;
    else hi = mid - 1;
  }
  return b.e[lo];
}

__global__ void __launch_bounds__(NT2, 1) gemm8p_group_kernel(WgBatch b) {
  const int nmain = b.ntiles - b.tail_tiles;
  int lid, z = 0;
  if ((int)blockIdx.x < nmain) {
    lid = xcd_remap(blockIdx.x, nmain);
  } else {
    const int u = blockIdx.x - nmain;
    lid = nmain + u / b.tail_split;
    z = u % b.tail_split;
  }
  DTC_ASSERT(lid < b.ntiles);
  const WgEntry& w = wg_entry(b, lid);
  const int t = lid - w.tile0;
  const int tiles_m = (w.M + BIG - 1) / BIG, tiles_n = (w.N + BIG - 1) / BIG;
  const int tm_idx = w.nfast ? t / tiles_n : t % tiles_m, tn_idx = w.nfast ? t % tiles_n : t / tiles_m;
  DTC_ASSERT(tn_idx * BIG < w.N && tm_idx * BIG < w.M);
  Epi e{};
  e.M = w.M; e.N = w.N; e.C = w.C; e.ldc = w.N; e.alpha = 1.f; e.beta = b.beta;
  if (lid >= nmain) {  // K-piece z of a tail tile (no bias column sums there: host-checked)
    DTC_ASSERT(w.cs == nullptr && b.tail_slab != nullptr);
    e.slab_tile = 1;
    const int kps = b.K / b.tail_split;
    gemm8p_tile<false, false, EPI_STORE, true, 4>(w.A, w.M, w.B, w.N, w.M, w.N, b.K, tm_idx, tn_idx, z, b.tail_split,
                                                   kps, b.tail_slab + (long)(lid - nmain) * b.tail_split * BIG * BIG, e);
    return;
  }
  e.colsum = w.cs; e.cs_accum = 1;
  e.sq = b.sq ? b.sq + (long)lid * (NT2 / 64) : nullptr;  // NT2 / 64 wave slots per tile
  gemm8p_tile<false, false, EPI_STORE, true, 4>(w.A, w.M, w.B, w.N, w.M, w.N, b.K, tm_idx, tn_idx, 0, 1, b.K,
                                                 nullptr, e);
}

// Finish the tail tiles: dW = beta*dW + sum_z slab[z] (z ascending), and their grad-norm partials (block
// (tail tile, row group q) of 32 rows writes sq slot q of its tile, the slots the whole tile's waves
// fill in the main kernel).  Grid (tail_tiles * 8), 256 threads: 32 rows x 64 float4 columns, 8 float4 per
// thread, every load of a thread issued before its first add (1024-thread blocks of 2 float4 each ran 1.5
// rounds of short-lived waves: 33 us for 75 MB at GPT-2 small).
constexpr int WGT_THREADS = 256;
__global__ void __launch_bounds__(WGT_THREADS) wg_tail_reduce(WgBatch b) {
  const int nmain = b.ntiles - b.tail_tiles;
  const int tt = blockIdx.x / 8, q = blockIdx.x % 8;
  const int lid = nmain + tt;
  const WgEntry& w = wg_entry(b, lid);
  const int t = lid - w.tile0;
  const int tiles_m = (w.M + BIG - 1) / BIG, tiles_n = (w.N + BIG - 1) / BIG;
  const int m0 = (w.nfast ? t / tiles_n : t % tiles_m) * BIG, n0 = (w.nfast ? t % tiles_n : t / tiles_m) * BIG;
  const float* slab = b.tail_slab + (long)tt * b.tail_split * BIG * BIG;
  float ss = 0.f;
  constexpr int IT = 32 * 64 / WGT_THREADS;  // float4 per thread, all loads of a slab issued before any add
  bool ok[IT];
  long so[IT], co[IT];
  f32x4 v[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int k = threadIdx.x + WGT_THREADS * i;
    const int r = q * 32 + k / 64, c = (k % 64) * 4;
    ok[i] = m0 + r < w.M && n0 + c < w.N;
    so[i] = (long)r * BIG + c;
    co[i] = (long)(m0 + r) * w.N + n0 + c;
    v[i] = ok[i] ? *(const f32x4*)(slab + so[i]) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int z = 1; z < b.tail_split; ++z) {
    f32x4 u[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) u[i] = ok[i] ? *(const f32x4*)(slab + (long)z * BIG * BIG + so[i]) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < IT; ++i) v[i] += u[i];
  }
  if (b.beta != 0.f) {
    f32x4 u[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) u[i] = ok[i] ? *(const f32x4*)(w.C + co[i]) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < IT; ++i) v[i] += b.beta * u[i];
  }
#pragma unroll
  for (int i = 0; i < IT; ++i)
    if (ok[i]) {
      *(f32x4*)(w.C + co[i]) = v[i];
      ss += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
    }
  if (!b.sq) return;
  __shared__ float red[WGT_THREADS / 64];
  ss = warp_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int w = 0; w < WGT_THREADS / 64; ++w) tot += red[w];
    b.sq[(long)lid * (NT2 / 64) + q] = tot;
  }
}

// ============================================================================================
// 128 x (64*CB) tile, 8 waves (2 along M x 4 along N, 64 x 16*CB per wave), NS-stage LDS-DMA ring,
// phase-interleaved like gemm8p_kernel -- for the layer GEMMs.  Their shapes quantise badly on
// 128^2 / 256^2 tiles (GPT-2 small: M = 8192 tokens, N = 768 / 2304 / 3072 = 4 / 12 / 16 x 192;
// GPT-2 medium: N = 1024 / 3072 / 4096 = 4 x 256, 16 x 192, 16 x 256) but make EXACTLY 1, 3 or 4
// rounds of 256 tiles here, one block per CU, and the 64 x 48 (CB = 3) / 64 x 64 (CB = 4) wave tile
// keeps LDS reads at 0.58 / 0.5 ds_read_b128 per MFMA (one per MFMA is the CU's limit).
//  * K-step = 64 k, 2 phases: phase p reads the wave's A fragments of rows 32p..32p+31 (+ all its B
//    fragments at p = 0), issues its share of the ring's DMA, raw s_barrier, 12 (CB = 3) / 16 (CB = 4) MFMAs between
//    s_setprio(1)/(0), raw s_barrier; waves 4-7 run one barrier behind (as gemm8p).
//  * Ring of NS stages (A image = 2 chunks, B image = CB chunks of [64 rows][64 k] -- the gemm8p
//    chunk images and swizzles).  Stage s is loaded D = NS-1 K-steps ahead: its B chunks in phase 0
//    of step s-D, its A chunks in phase 1 (each region re-staged 2 phases after its last read: B is
//    last read in phase 0, A in phase 1 of the slot's previous step).  Stage t+1
//    is retired by a counted vmcnt at the end of phase 0 of step t, one full phase before its first
//    read (the staggered wave group reads it one barrier later).  Never vmcnt(0) in steady state.
//  * NS = 4 for CB = 3 (160 KB: the whole LDS), 3 for CB = 4 (144 KB).
__device__ __forceinline__ void n8_vmcnt(int n) {  // s_waitcnt vmcnt(n), n a runtime value <= 18
  switch (n) {
    case 0: P8_VMCNT(0); break;
    case 2: P8_VMCNT(2); break;
    case 3: P8_VMCNT(3); break;
    case 4: P8_VMCNT(4); break;
    case 5: P8_VMCNT(5); break;
    case 6: P8_VMCNT(6); break;
    case 8: P8_VMCNT(8); break;
    case 9: P8_VMCNT(9); break;
    case 10: P8_VMCNT(10); break;
    case 11: P8_VMCNT(11); break;
    case 12: P8_VMCNT(12); break;
    case 15: P8_VMCNT(15); break;
    case 16: P8_VMCNT(16); break;
    case 18: P8_VMCNT(18); break;
    default: P8_VMCNT(0); break;  // over-waiting is always safe
  }
}

// compile-time loop: f(integral_constant<I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// One accumulator fragment (row m, columns n..n+3) of the overlapped epilogue: bias and the dGELU
// factor come from registers, so the only memory operations are the stores.
template <int EPI, bool OUTF32>
__device__ __forceinline__ void n8_frag_out(const Epi& e, int m, int n, f32x4 v, f32x4 bias, bf16x4 aux) {
  float o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = v[r] + bias[r];
  if (EPI == EPI_DGELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] *= (float)aux[r];
  }
  if (OUTF32) {
    *(f32x4*)((float*)e.C + (long)m * e.ldc + n) = f32x4{o[0], o[1], o[2], o[3]};
    return;
  }
  bf16x4 ob, gb;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (EPI == EPI_GELU) {  // C = gelu'(u), aux_out = gelu(u) (as epilogue_store)
      float gv, dgv;
      gelu_tanh_and_grad_f(o[r], gv, dgv);
      ob[r] = f2bf(dgv);
      gb[r] = f2bf(gv);
    } else {
      ob[r] = f2bf(o[r]);
    }
  }
  *(bf16x4*)((bf16*)e.C + (long)m * e.ldc + n) = ob;
  if (EPI == EPI_GELU) *(bf16x4*)((bf16*)e.aux_out + (long)m * e.ldc + n) = gb;
}

template <int CB, int NS, bool AK, bool BKM, int EPI, bool OUTF32>
__global__ void __launch_bounds__(NT2, 1)
gemm8n_kernel(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, int M, int N, int K,
              int tiles_m, int tiles_n, int gm, Epi e) {
  static_assert(NS >= 3, "stage t+1 must be issued before the phase-0 wait of step t");
  constexpr int CA = 2, TM = 4, TN = CB, BN = 64 * CB, D = NS - 1, PIECES = CA + CB;
  constexpr int SIMG = PIECES * P8_CHUNK;
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * SIMG];  // the only LDS object
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int ntiles = tiles_m * tiles_n;
  // persistent: block b runs tiles bl, bl + G, ... (round r of the grid = tiles [rG, rG + G), the
  // same XCD-grouped order a one-tile-per-block launch would use); its K-steps form ONE stream, so
  // the next tile's first stages load under the current tile's last K-steps and its epilogue stores
  // drain under the next tile's MFMAs
  const int G = gridDim.x;
  const int bl = xcd_remap(blockIdx.x, G);
  const int nk = K / 64;
  DTC_ASSERT(nk >= 1);
  const int nr = bl < ntiles ? (ntiles - bl + G - 1) / G : 0;
  const int S = nr * nk;
  if (S == 0) return;
  auto origin = [&](int r, int& m0, int& n0) {
    const int tile = bl + r * G;
    const int grp = tile / (gm * tiles_n), in_g = tile % (gm * tiles_n);
    const int gm_eff = min(gm, tiles_m - grp * gm);
    m0 = (grp * gm + in_g % gm_eff) * 128;
    n0 = (in_g / gm_eff) * BN;
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Overlapped epilogue (bf16 / fp32 stores and the GELU pair: epilogues with no operand to read
  // but the bias): a finished tile's accumulators move to pacc and are stored two fragments per phase
  // during the NEXT tile's first NPEEL K-steps, between the MFMA clusters (the staggered wave group
  // runs its MFMAs meanwhile), instead of stalling all 8 waves at the tile boundary -- at one block
  // per CU nothing else would hide it.  Those K-steps are peeled (compile-time fragment indices: the
  // accumulator arrays stay in registers).  The stores are extra younger vector-memory ops for the
  // counted waits (stricter, never early); the bias is loaded once per tile.  Epilogues that read a
  // residual / dGELU factor per element keep the immediate form: a load in the loop would make its
  // use wait for every older in-flight DMA stage.
  constexpr bool OVL = EPI == EPI_STORE || EPI == EPI_GELU;
  constexpr int NFRAG = TN * TM, NPEEL = OVL ? NFRAG / 4 : 0;  // 2 fragments per phase, 2 phases per step
  f32x4 pacc[TN][TM], pbias[TN];
  bool pend = false;
  int em0 = 0, en0 = 0;
  const int g4e = 4 * (lane >> 4);
  auto epi_frag = [&](auto F) {
    constexpr int f = decltype(F)::value, i = f / TM, j = f % TM;
    const int m = em0 + wr * 64 + j * 16 + (lane & 15);
    const int n = en0 + wc * 16 * TN + i * 16 + g4e;
    if (m < M) n8_frag_out<EPI, OUTF32>(e, m, n, pacc[i][j], pbias[i], bf16x4{});
  };
  int cm0, cn0;  // origin of the tile being computed
  origin(0, cm0, cn0);
  DTC_ASSERT(nk >= NPEEL);

  auto imgA = [&](int s) { return smem + (s % NS) * SIMG; };  // NS constant: no division
  auto imgB = [&](int s) { return smem + (s % NS) * SIMG + CA * P8_CHUNK; };
  // stage s = (round s / nk, K-step s % nk).  The issue side walks the stream with its own counters
  // (round pr, K-step pk, tile origin pm0 / pn0): no runtime integer division in the loop
  // per-lane DMA source pointers of the issue side's tile (recomputed only at tile boundaries) plus
  // the running K offset: one 64-bit add per DMA instruction in the loop
  int pr = 0, pk = 0;
  const bf16* srcA[CA];
  const bf16* srcB[CB];
  long offA = 0, offB = 0;
  const long stepA = AK ? 64 : 64 * lda, stepB = BKM ? 64 : 64 * ldb;
  auto set_src = [&](int r) {
    int m0, n0;
    origin(r, m0, n0);
#pragma unroll
    for (int q = 0; q < CA; ++q) srcA[q] = p8_src<AK>(A, lda, m0, M, q, wave, lane);
#pragma unroll
    for (int q = 0; q < CB; ++q) srcB[q] = p8_src<BKM>(B, ldb, n0, N, q, wave, lane);
    offA = offB = 0;
  };
  set_src(0);
  auto advance = [&]() {
    offA += stepA;
    offB += stepB;
    if (++pk == nk) {
      pk = 0;
      ++pr;
      if (pr < nr) set_src(pr);
    }
  };
  auto dmaA = [&](int s, int q) { p8_dma_at(srcA[q] + offA, imgA(s), q, wave); };
  auto dmaB = [&](int s, int q) { p8_dma_at(srcB[q] + offB, imgB(s), q, wave); };

  // prologue: stages 0..D-1 (B then A each), wait for stage 0
  const int npro = min(D, S);
  for (int s = 0; s < npro; ++s) {
#pragma unroll
    for (int q = 0; q < CB; ++q) dmaB(s, q);
#pragma unroll
    for (int q = 0; q < CA; ++q) dmaA(s, q);
    advance();
  }
  n8_vmcnt((npro - 1) * PIECES);
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // second wave group: one barrier behind

  int t = 0;  // consume side: K-step of the stream
  bf16x8 fb[TN][2], fa[2][2];
  // one K-step; SL >= 0: also store fragments 4 SL .. 4 SL + 3 of the pending tile
  auto kstep = [&](auto SLc) {
    constexpr int SL = decltype(SLc)::value;
    const bf16* sA = imgA(t);
    const bf16* sB = imgB(t);
    const bool issue = t + D < S;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if (p == 0) {
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) fb[i][kk] = p8_frag<BKM>(sB, TN * wc + i, kk, lane);
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fa[jj][kk] = p8_frag<AK>(sA, 4 * wr + 2 * p + jj, kk, lane);
      if (issue) {
        if (p == 0) {
#pragma unroll
          for (int q = 0; q < CB; ++q) dmaB(t + D, q);
        } else {
#pragma unroll
          for (int q = 0; q < CA; ++q) dmaA(t + D, q);
          advance();
        }
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int jj = 0; jj < 2; ++jj)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) asm volatile("" : "+v"(fa[jj][kk]));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) asm volatile("" : "+v"(fb[i][kk]));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            acc[i][2 * p + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i][kk], fa[jj][kk], acc[i][2 * p + jj], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (SL >= 0) {
        if (pend) {
          if (p == 0) {
            epi_frag(std::integral_constant<int, 4 * SL>{});
            epi_frag(std::integral_constant<int, 4 * SL + 1>{});
          } else {
            epi_frag(std::integral_constant<int, 4 * SL + 2>{});
            epi_frag(std::integral_constant<int, 4 * SL + 3>{});
          }
        }
      }
      if (p == 0 && t + 1 < S) {
        // retire stage t+1: younger than its A pieces are the stages t+2 .. t+D-1 that exist, and
        // B(t+D) when it was issued this phase.  Epilogue loads / stores issued since are extra
        // younger operations: they only make this wait stricter (never early)
        if (t + D < S) {
          vmcnt_c<(D - 2) * PIECES + CB>();  // steady state: one s_waitcnt, no branch
        } else {
          const int full = max(0, min(t + D - 1, S - 1) - (t + 1));
          n8_vmcnt(full * PIECES);
        }
      }
      __builtin_amdgcn_s_barrier();
    }
    ++t;
  };
  for (int cr = 0; cr < nr; ++cr) {
    static_for<0, NPEEL>([&](auto sl) { kstep(sl); });
    for (int k = NPEEL; k < nk; ++k) kstep(std::integral_constant<int, -1>{});
    // the tile's last K-step is done: its epilogue (from registers, no LDS), then restart
    const int m0 = cm0, n0 = cn0;
    if (cr + 1 < nr) origin(cr + 1, cm0, cn0);
    const int g4 = 4 * (lane >> 4);
    if constexpr (OVL) {  // stored during the next tile's first K-steps (after the loop for the last)
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        pbias[i] = e.bias ? *(const f32x4*)(e.bias + n0 + wc * 16 * TN + i * 16 + g4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < TM; ++j) pacc[i][j] = acc[i][j];
      }
      em0 = m0;
      en0 = n0;
      pend = true;
    } else if constexpr (EPI == EPI_NONE) {  // microbenchmark: main loop only (keep the accumulators live)
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) asm volatile("" ::"v"(acc[i][j]));
    } else {
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int m = m0 + wr * 64 + j * 16 + (lane & 15);
          const int n = n0 + wc * 16 * TN + i * 16 + g4;
          if (m < M && n < N) epilogue_store<EPI, OUTF32>(e, m, n, acc[i][j]);
        }
    }
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr (OVL) static_for<0, NFRAG>([&](auto f) { epi_frag(f); });  // the block's last tile
  if (wr == 0) __builtin_amdgcn_s_barrier();  // balance the second group's extra barrier
}

// ============================================================================================
// lm_head backward with the cross-entropy backward fused into the dgrad's A operand.
//   dlogits[t][v] = (exp(logit[t][v] - lse[t]) - [v == label[t]]) * scale   (pad columns 0)
//   dX[t][:]      = sum_v dlogits[t][v] * W[v][:]    (NT split-K on W^T, as the unfused dgrad)
//   colpart       = column sums of dlogits (the lm_head bias gradient's partials)
// The logits tile is register-staged (not DMA'd) so each element is transformed once per block on
// its way into the LDS image — the K-major image layout of dma_tile<true> — and the unfused
// ce_bwd pass (read 412 MB + write 412 MB) disappears: n-tile-0 blocks store the bf16 dlogits (the
// weight gradient's input) and the column sums, the latter as MFMAs of a ones operand with
// transposed reads of the A image (any k order sums the same), 16 columns per wave and k-step.
// Each thread stages the SAME 16-B vocab chunk of 4 rows (the swizzle term (row>>1)&7 does not
// depend on the 64-row step), so its label / lse values stay in registers for the whole block.
__device__ __forceinline__ bf16x8 ce_colsum_frag(const bf16* img, int r0, int vt, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int row = r0 + 4 * g + q;  // rows r0 + {4g+q} and +16: every row of r0..r0+31 once
  const int ch = 2 * vt + (pp >> 1);
  const bf16* p0 = img + row * 64 + ((ch ^ ((row >> 1) & 7)) << 3) + (pp & 1) * 4;
  // asm reads (ds_tr16_asm): the builtin made hipcc drain the in-flight W^T DMA before every column-sum
  // k-step; the caller waits lgkmcnt(0) with the fragments tied in
  const s16x4 lo = ds_tr16_asm(p0), hi = ds_tr16_asm(p0 + 16 * 64);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

struct CeDgradArgs {
  const bf16* logits; long ldl;
  const float* lse; const int* labels; int vocab_start, n_valid; float scale;
  const bf16* wt; long ldw;        // W^T [N = d][K = vocab] bf16, K-major
  bf16* dlogits; long ldd;         // [M][K] bf16 out (n-tile 0 blocks)
  float* colpart;                  // [2 * tiles_m][K] fp32 out (n-tile 0 blocks)
  float* slab;                     // split-K fp32 slabs [split][M][N]
  int M, N, K, tiles_m, tiles_n, gm, split, kps;
};

__global__ void __launch_bounds__(NT2, 1) ce_dgrad256_kernel(CeDgradArgs a) {
  constexpr int TM = 8, TN = 4;
  __shared__ __attribute__((aligned(16))) bf16 smem[4 * IMG];  // [buf][A img | B img], 128 KB
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = a.tiles_m * a.tiles_n;
  const int lid = xcd_remap(blockIdx.x, ntiles * a.split);
  const int tile = lid % ntiles, z = lid / ntiles;
  const int grp = tile / (a.gm * a.tiles_n), in_g = tile % (a.gm * a.tiles_n);
  const int gm_eff = min(a.gm, a.tiles_m - grp * a.gm);
  const int tm_idx = grp * a.gm + in_g % gm_eff, tn_idx = in_g / gm_eff;
  const int m0 = tm_idx * BIG, n0 = tn_idx * BIG;
  DTC_ASSERT(tm_idx >= 0 && tn_idx >= 0 && z >= 0 && m0 < a.M && n0 < a.N);
  const int kbeg = z * a.kps;
  const int nk = min(a.kps, a.K - kbeg) / 64;
  // the dlogits stores + column sums of k-step kt go to n-tile kt % 2 (the two n-tiles share them)
  // no dlogits output requested: nothing to own
  const int nown = a.dlogits ? min(a.tiles_n, 2) : 0;
  auto owns = [&](int kt) { return tn_idx < nown && kt % nown == tn_idx; };

  // staging coordinates: rows q*64 + srow (q = 0..3), 16-B chunk schunk of the 64-wide k-step,
  // stored at LDS chunk position lane & 7 (the dma_tile<true> image)
  const int srow = wave * 8 + (lane >> 3), spos = lane & 7, schunk = spos ^ ((srow >> 1) & 7);
  float cr_r[4];
  int lab_r[4];
  bool ok_r[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = m0 + q * 64 + srow;
    ok_r[q] = m < a.M;
    cr_r[q] = ok_r[q] ? ce_row_c(a.lse[m], a.scale) : -INFINITY;  // rows past M: exp2(-inf) = 0
    lab_r[q] = ok_r[q] ? a.labels[m] - a.vocab_start : -1;
  }
  u32x4 R[4];
  auto load_a = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = min(m0 + q * 64 + srow, a.M - 1);
      R[q] = *(const u32x4*)(a.logits + (long)m * a.ldl + k0 + schunk * 8);
    }
  };
  // transform the staged logits into dlogits: LDS image + (lead) global dlogits
  auto put_a = [&](int k0, bf16* img, bool lead) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bf16x8 l8 = __builtin_bit_cast(bf16x8, R[q]);
      const int v0 = k0 + schunk * 8;
      float gv[8];
      ce_grad8(l8, v0, cr_r[q], lab_r[q], a.n_valid, a.scale, gv);  // as ce_bwd: identical dlogits bits
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(gv[e]);
      const int row = q * 64 + srow;
      *(bf16x8*)(img + row * 64 + spos * 8) = o;
      // non-temporal: 412 MB that would otherwise push the last layers' saved activations out of
      // the Infinity Cache right before their backward (measured -12..-29 us/step)
      if (lead && ok_r[q]) __builtin_nontemporal_store(o, (bf16x8*)(a.dlogits + (long)(m0 + row) * a.ldd + v0));
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16x8 ones = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
  const int cs_vt = wave & 3, cs_half = wave >> 2;

  // prologue: k-step 0 staged, the logits of k-step 1 already in registers
  dma_tile<true>(a.wt, a.ldw, n0, a.N, kbeg, smem + IMG, wave, lane);
  if (nk > 0) {
    load_a(kbeg);
    put_a(kbeg, smem, owns(0));
  }
  if (nk > 1) load_a(kbeg + 64);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // iteration kt: B(kt+1) DMA; A(kt+1) (registers, loaded one iteration ago) transformed into the
  // other buffer; A(kt+2) loads issued; then the MFMAs of k-step kt, under which those loads land.
  // The barrier waits only for the DMA: every vector-memory op issued after it (dlogits stores,
  // the A(kt+2) loads, the column-sum store) may stay in flight (vmcnt counts in issue order).
  for (int kt = 0; kt < nk; ++kt) {
    const bf16* sA = smem + (kt & 1) * 2 * IMG;
    const bf16* sB = sA + IMG;
    bf16* nA = smem + ((kt + 1) & 1) * 2 * IMG;
    const bool more = kt + 1 < nk, more2 = kt + 2 < nk;
    const int k1 = kbeg + (kt + 1) * 64;
    if (more) dma_tile<true>(a.wt, a.ldw, n0, a.N, k1, nA + IMG, wave, lane);
    const bool st1 = more && owns(kt + 1);
    if (more) put_a(k1, nA, st1);
    if (more2) load_a(k1 + 64);
    const bool cs_own = owns(kt);
    if (cs_own) {  // column sums of this k-step's dlogits tile: 4 MFMAs per wave
      f32x4 cs = {0.f, 0.f, 0.f, 0.f};
      bf16x8 cf[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) cf[s4] = ce_colsum_frag(sA, cs_half * 128 + 32 * s4, cs_vt, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cf[0]), "+v"(cf[1]), "+v"(cf[2]), "+v"(cf[3]) : : "memory");
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) cs = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, cf[s4], cs, 0, 0, 0);
      if (lane < 16) a.colpart[(long)(2 * tm_idx + cs_half) * a.K + kbeg + kt * 64 + cs_vt * 16 + lane] = cs[0];
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int j = 0; j < TM; ++j) fa[j] = big_frag<true>(sA, wm * 8 + j, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i) fb[i] = big_frag<true>(sB, wn * 4 + i, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
    // ops issued after the DMA: 4 stores (every staged row valid), 4 loads, 1 column-sum store
    const int after = ((st1 && m0 + BIG <= a.M) ? 4 : 0) + (more2 ? 4 : 0) + (cs_own ? 1 : 0);
    if (after >= 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else if (after >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after >= 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if (after >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (after >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  const int g4 = 4 * (lane >> 4);
  float* sl = a.slab + (long)z * a.M * a.N;  // split-K slab z (splitk_reduce sums them in order)
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * 128 + j * 16 + (lane & 15);
      const int n = n0 + wn * 64 + i * 16 + g4;
      if (m < a.M && n < a.N) *(f32x4*)(sl + (long)m * a.N + n) = acc[i][j];
    }
}

// C = beta*C + sum_z slab[z]   (fp32, deterministic order)
__global__ void splitk_reduce(const float* __restrict__ slab, int split, long MN, float* __restrict__ C, long ldc,
                              int N, float beta) {
  long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= MN) return;
  DTC_ASSERT(N % 4 == 0 && i4 + 4 <= MN);
  long m = i4 / N;
  int n = (int)(i4 % N);
  f32x4 s = *(const f32x4*)(slab + i4);
  for (int z = 1; z < split; ++z) {
    f32x4 t = *(const f32x4*)(slab + z * MN + i4);
    s += t;
  }
  float* c = C + m * ldc + n;
  if (beta != 0.f) {
    f32x4 old = *(const f32x4*)c;
    s += beta * old;
  }
  *(f32x4*)c = s;
}

// ============================================================================================
// DMA-pipelined layer GEMM (64x64 or 128x128 tiles, 4 waves, NSTAGE-deep LDS ring).
// The layer GEMMs ([4096 x 512..2048 x 512..4096]) give each CU only 1-2 tiles, so they are bound
// by how many operand bytes a CU keeps in flight from L2, not by MFMA rate: the register-staged
// kernel above holds 1-2 K-tiles per block.  Here operands stream global->LDS by
// global_load_lds (no staging VGPRs) into an NSTAGE ring with NSTAGE-1 K-tiles in flight: each
// K-step waits only for the OLDEST tile with a counted s_waitcnt vmcnt(N) and a raw s_barrier
// (cdna_hip_programming.md §5 "Pipelining across barriers": __syncthreads would drain every
// DMA), then refills the slot the previous step just finished reading.
//  * K-major image [R][64 k] (128-B rows, chunk swizzle c ^ ((r>>1)&7)), MN-major image
//    [64 k][R] (R*2-B rows, swizzle dimg_mn_swz) — DMA destination lane-linear, swizzle on the
//    source address, conflict-free ds_read_b128 / ds_read_b64_tr_b16 fragment reads, natural
//    k order for both (any layout pairing).
//  * Ragged edges: rows/cols clamped to valid addresses (only feed unstored outputs).
template <int R>
__device__ __forceinline__ int dimg_mn_swz(int r) {
  if (R == 64) return 2 * (((r >> 1) & 1) | ((r >> 2) & 2));  // 128-B rows: 4 windows per bank row
  return 2 * ((r & 3) | ((r >> 1) & 4));                      // >= 256-B rows: 8 windows
}

template <int R, bool KMAJ, int NW = 4>
struct DImg {
  static constexpr int ELEMS = R * 64;
  static constexpr int NI = ELEMS * 2 / 1024 / NW;  // 1-KB DMA instructions per wave (NW waves)
  static_assert(NI >= 1, "operand image smaller than one DMA instruction per wave");
  __device__ __forceinline__ static void dma(const bf16* __restrict__ X, long ldx, int r0, int rmax, int k0, bf16* img,
                                             int wave, int lane) {
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int blk = q * NW + wave;
      const bf16* src;
      if (KMAJ) {
        const int row = blk * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((row >> 1) & 7);
        src = X + (long)min(r0 + row, rmax - 1) * ldx + k0 + c * 8;
      } else {
        constexpr int LPR = R / 8;  // lanes per k-row
        const int kr = blk * (64 / LPR) + lane / LPR;
        const int c = (lane % LPR) ^ dimg_mn_swz<R>(kr);
        src = X + (long)(k0 + kr) * ldx + min(r0 + c * 8, rmax - 8);
      }
      __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(img + blk * 512), 16, 0, 0);
    }
  }
  __device__ __forceinline__ static bf16x8 frag(const bf16* img, int t, int kk, int lane) {
    const int g = lane >> 4, li = lane & 15;
    if (KMAJ) {
      const int row = t * 16 + li;
      return *(const bf16x8*)(img + row * 64 + (((kk * 4 + g) ^ ((row >> 1) & 7)) << 3));
    } else {
      const int q = li >> 2, pp = li & 3;
      const int k0 = kk * 32 + 8 * g + q, k1 = k0 + 4;
      const int c = 2 * t + (pp >> 1), w = (pp & 1) * 4;
      const bf16* p0 = img + k0 * R + ((c ^ dimg_mn_swz<R>(k0)) << 3) + w;
      const bf16* p1 = img + k1 * R + ((c ^ dimg_mn_swz<R>(k1)) << 3) + w;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p0));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DTC_LDS s16x4*)(DTC_LDS void*)(p1));
      return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  }
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `ahead` K-tiles' DMAs (G instructions each) are still in flight
template <int G, int MAXAHEAD>
__device__ __forceinline__ void wait_tiles(int ahead) {
  if (MAXAHEAD >= 3 && ahead >= 3) wait_vmcnt<3 * G>();
  else if (MAXAHEAD >= 2 && ahead >= 2) wait_vmcnt<2 * G>();
  else if (ahead >= 1) wait_vmcnt<G>();
  else wait_vmcnt<0>();
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BM, int BN, int NSTAGE, bool AK, bool BKM, int EPI, bool OUTF32>
__global__ void __launch_bounds__(NT, (BM * BN <= 64 * 64) ? 2 : 1)
gemm_dma_kernel(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, int M, int N, int K,
                int tiles_m, int tiles_n, int gm, int split, int k_per_split, float* __restrict__ slab, Epi e) {
  using IA = DImg<BM, AK>;
  using IB = DImg<BN, BKM>;
  constexpr int STAGE = IA::ELEMS + IB::ELEMS;
  constexpr int G = IA::NI + IB::NI;  // DMA instructions per thread per K-tile
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) bf16 smem[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = tiles_m * tiles_n;
  const int lid = xcd_remap(blockIdx.x, ntiles * split);
  const int tile = lid % ntiles, z = lid / ntiles;
  const int grp = tile / (gm * tiles_n), in_g = tile % (gm * tiles_n);
  const int gm_eff = min(gm, tiles_m - grp * gm);
  const int tm_idx = grp * gm + in_g % gm_eff, tn_idx = in_g / gm_eff;
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;
  DTC_ASSERT(tm_idx >= 0 && tn_idx >= 0 && z >= 0 && m0 < M && n0 < N);
  const int kbeg = z * k_per_split;
  const int nk = min(k_per_split, K - kbeg) / 64;

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) {
      IA::dma(A, lda, m0, M, kbeg + s * 64, smem + s * STAGE, wave, lane);
      IB::dma(B, ldb, n0, N, kbeg + s * 64, smem + s * STAGE + IA::ELEMS, wave, lane);
    }
  for (int kt = 0; kt < nk; ++kt) {
    wait_tiles<G, NSTAGE - 2>(min(NSTAGE - 2, nk - 1 - kt));  // tile kt landed (this wave)
    raw_barrier();                                            // ... for every wave; slot kt-1 free
    const int nt = kt + NSTAGE - 1;
    if (nt < nk) {
      bf16* sl = smem + (nt % NSTAGE) * STAGE;
      IA::dma(A, lda, m0, M, kbeg + nt * 64, sl, wave, lane);
      IB::dma(B, ldb, n0, N, kbeg + nt * 64, sl + IA::ELEMS, wave, lane);
    }
    const bf16* sA = smem + (kt % NSTAGE) * STAGE;
    const bf16* sB = sA + IA::ELEMS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int j = 0; j < TM; ++j) fa[j] = IA::frag(sA, wm * TM + j, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i) fb[i] = IB::frag(sB, wn * TN + i, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
  }

  const int g4 = 4 * (lane >> 4);
  constexpr bool ST32 = DTC_STAGE_F32 && 4 * WM * WN * 4 <= NSTAGE * STAGE * 2;
  if constexpr (ST32) {
    if (split > 1 || (OUTF32 && (EPI == EPI_STORE || EPI == EPI_RESID))) {
      raw_barrier();  // every wave's last fragment reads are done: the ring is free for the stage
      const bool sp = split > 1;
      f32x4 bb[TN];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int n = n0 + wn * WN + i * 16 + g4;
        bb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (!sp && e.bias) {
          if (n + 4 <= N) bb[i] = *(const f32x4*)(e.bias + n);
          else for (int r = 0; r < 4; ++r) if (n + r < N) bb[i][r] = e.bias[n + r];
        }
      }
      staged_f32_epilogue<TN, TM, WM, WN>(acc, (float*)smem + wave * (WM * WN),
                                          sp ? slab + (long)z * M * N : (float*)e.C, sp ? N : e.ldc, m0 + wm * WM,
                                          n0 + wn * WN, M, N, lane, !sp, e.alpha, bb,
                                          (!sp && EPI == EPI_RESID) ? (const float*)e.aux : nullptr, e.ldaux,
                                          (!sp && EPI == EPI_STORE) ? e.beta : 0.f);
      return;
    }
  }
  if (split > 1) {
    float* sl = slab + (long)z * M * N;
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wm * WM + j * 16 + (lane & 15);
        const int n = n0 + wn * WN + i * 16 + g4;
        if (m < M) {
          float* c = sl + (long)m * N + n;
          if (n + 4 <= N) *(f32x4*)c = acc[i][j];
          else for (int r = 0; r < 4; ++r) if (n + r < N) c[r] = acc[i][j][r];
        }
      }
    return;
  }
  if (EPI == EPI_LMHEAD) {
    EpiPre<TN, TM> pre;
    epi_prefetch<TN, TM>(e, m0 + wm * WM, n0 + wn * WN, lane, true, pre);
    lmhead_epilogue<TN, TM>(acc, e, m0 + wm * WM, n0 + wn * WN, tn_idx * 2 + wn, lane, pre);
    return;
  }
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + (lane & 15);
      const int n = n0 + wn * WN + i * 16 + g4;
      if (m < M && n < N) epilogue_store<EPI, OUTF32>(e, m, n, acc[i][j]);
    }
}

// ============================================================================================
// 8-wave DMA-ring layer GEMM (512 threads, WGM x WGN waves, one block per CU).  The 4-wave kernels
// above run at 2 blocks/CU (register-staged) or 1 block/CU with one wave per SIMD (DMA): their main
// loops fill LDS at ~45 GB/s per CU, which bounds every layer GEMM of the reference step at its 1-2
// tiles per CU.  Two waves per SIMD over an NSTAGE global_load_lds ring keep more bytes in flight
// and give each SIMD a second wave to issue under the first one's LDS reads: at the reference shapes
// the main loops run 20-40 % faster (benchmarks/gemm_dma8_micro.hip).  Same operand images,
// swizzles, counted-vmcnt/raw-barrier ring and epilogues as gemm_dma_kernel; the bf16 epilogues go
// through a per-wave LDS stage when the wave tile is 64 columns wide (full 128-B output rows).
template <int BM, int BN, int NSTAGE, int WGM, int WGN, bool AK, bool BKM, int EPI, bool OUTF32>
__global__ void __launch_bounds__(64 * WGM * WGN, 1)
gemm_dmaw_kernel(const bf16* __restrict__ A, long lda, const bf16* __restrict__ B, long ldb, int M, int N, int K,
                 int tiles_m, int tiles_n, int gm, int split, int k_per_split, float* __restrict__ slab, Epi e) {
  constexpr int NW = WGM * WGN;
  using IA = DImg<BM, AK, NW>;
  using IB = DImg<BN, BKM, NW>;
  constexpr int STAGE = IA::ELEMS + IB::ELEMS;
  constexpr int G = IA::NI + IB::NI;  // DMA instructions per thread per K-tile
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  constexpr int LDS_BYTES = NSTAGE * STAGE * 2;
  __shared__ __attribute__((aligned(16))) bf16 smem[NSTAGE * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WGM, wn = wave / WGM;
  const int ntiles = tiles_m * tiles_n;
  const int lid = xcd_remap(blockIdx.x, ntiles * split);
  const int tile = lid % ntiles, z = lid / ntiles;
  const int grp = tile / (gm * tiles_n), in_g = tile % (gm * tiles_n);
  const int gm_eff = min(gm, tiles_m - grp * gm);
  // LayerNorm epilogues: N fastest, so a row group's tiles are consecutive in each XCD's dispatch order
  constexpr bool LNE = EPI == EPI_RESID_LN || EPI == EPI_LN_BWD;
  const int m0 = LNE ? (tile / tiles_n) * BM : (grp * gm + in_g % gm_eff) * BM;
  const int n0 = LNE ? (tile % tiles_n) * BN : (in_g / gm_eff) * BN;
  const int kbeg = z * k_per_split;
  const int nk = min(k_per_split, K - kbeg) / 64;
  const int g4 = 4 * (lane >> 4);
  const int mb = m0 + wm * WM, nb = n0 + wn * WN;

  // epilogue operands issued ahead of the main loop (their latency hides under it)
  constexpr bool STAGED16 = !OUTF32 && WN == 64 && (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_DGELU) &&
                            NW * WM * 64 * 2 <= LDS_BYTES;
  constexpr bool ST32 = DTC_STAGE_F32 && (WN == 64 || WN == 32) && BM * BN * 4 <= LDS_BYTES;
  f32x4 bpre[TN];
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = nb + i * 16 + g4;
    bpre[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (split == 1 && e.bias) {
      if (n + 4 <= N) bpre[i] = *(const f32x4*)(e.bias + n);
      else for (int r = 0; r < 4; ++r) if (n + r < N) bpre[i][r] = e.bias[n + r];
    }
  }
  constexpr bool PRE_U = EPI == EPI_DGELU;
  bf16x4 upre[PRE_U ? TN : 1][PRE_U ? TM : 1];
  if constexpr (PRE_U) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = mb + j * 16 + (lane & 15), n = nb + i * 16 + g4;
        upre[i][j] = (m < M && n + 4 <= N) ? *(const bf16x4*)((const bf16*)e.aux + (long)m * e.ldaux + n) : bf16x4{};
      }
  }

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < NSTAGE - 1; ++st)
    if (st < nk) {
      IA::dma(A, lda, m0, M, kbeg + st * 64, smem + st * STAGE, wave, lane);
      IB::dma(B, ldb, n0, N, kbeg + st * 64, smem + st * STAGE + IA::ELEMS, wave, lane);
    }
  // the epilogue operand loads above sit in the VM queue AHEAD of the ring's DMAs: the first counted
  // wait covers them too (they have landed long before the first K-tile is needed)
  for (int kt = 0; kt < nk; ++kt) {
    wait_tiles<G, NSTAGE - 2>(min(NSTAGE - 2, nk - 1 - kt));  // tile kt landed (this wave)
    raw_barrier();                                            // ... for every wave; slot kt-1 free
    const int nt = kt + NSTAGE - 1;
    if (nt < nk) {
      bf16* sl = smem + (nt % NSTAGE) * STAGE;
      IA::dma(A, lda, m0, M, kbeg + nt * 64, sl, wave, lane);
      IB::dma(B, ldb, n0, N, kbeg + nt * 64, sl + IA::ELEMS, wave, lane);
    }
    const bf16* sA = smem + (kt % NSTAGE) * STAGE;
    const bf16* sB = sA + IA::ELEMS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int j = 0; j < TM; ++j) fa[j] = IA::frag(sA, wm * TM + j, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i) fb[i] = IB::frag(sB, wn * TN + i, kk, lane);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[i], fa[j], acc[i][j], 0, 0, 0);
    }
  }
  if constexpr (EPI == EPI_NONE) {  // microbenchmark: main loop only (keep the accumulators live)
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  if (nk > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  raw_barrier();  // every wave's last fragment reads are done: the ring is free for the stages
  if constexpr (EPI == EPI_RESID_LN) {
    static_assert(OUTF32 && (NW * WM * WN + 1) * 4 <= LDS_BYTES, "LN epilogue stage");
    ln_fwd_epilogue<TN, TM, WM, WN, WGM, WGN>(acc, (float*)smem + wave * (WM * WN), (int*)((float*)smem + NW * WM * WN),
                                              e, m0, n0, wm, wn, wave, lane, tid, bpre);
    return;
  }
  if constexpr (EPI == EPI_LN_BWD) {
    static_assert(OUTF32 && (NW * WM * WN + NW * 3 * 32 + 1) * 4 <= LDS_BYTES, "LN epilogue stage");
    float* const red = (float*)smem + NW * WM * WN;
    ln_bwd_epilogue<TN, TM, WM, WN, WGM, WGN>(acc, (float*)smem + wave * (WM * WN), red, (int*)(red + NW * 3 * 32), e, m0,
                                              n0, wm, wn, wave, lane, tid);
    return;
  }
  if constexpr (ST32) {
    if (split > 1 || (OUTF32 && (EPI == EPI_STORE || EPI == EPI_RESID))) {
      const bool sp = split > 1;
      staged_f32_epilogue<TN, TM, WM, WN>(acc, (float*)smem + wave * (WM * WN), sp ? slab + (long)z * M * N : (float*)e.C,
                                          sp ? N : e.ldc, mb, nb, M, N, lane, !sp, e.alpha, bpre,
                                          (!sp && EPI == EPI_RESID) ? (const float*)e.aux : nullptr, e.ldaux,
                                          (!sp && EPI == EPI_STORE) ? e.beta : 0.f);
      return;
    }
  }
  if (split > 1) {  // slab without the LDS stage
    float* sl = slab + (long)z * M * N;
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = mb + j * 16 + (lane & 15), n = nb + i * 16 + g4;
        if (m < M) {
          float* c = sl + (long)m * N + n;
          if (n + 4 <= N) *(f32x4*)c = acc[i][j];
          else for (int r = 0; r < 4; ++r) if (n + r < N) c[r] = acc[i][j][r];
        }
      }
    return;
  }
  if constexpr (STAGED16) {
    bf16* stg = smem + wave * (WM * 64);
#pragma unroll
    for (int pass = 0; pass < (EPI == EPI_GELU ? 2 : 1); ++pass) {
#pragma unroll
      for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          bf16x4 ob;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = e.alpha * acc[i][j][r] + bpre[i][r];
            if constexpr (EPI == EPI_GELU) {  // pass 0: C = gelu'(u), pass 1: aux_out = gelu(u)
              float gv, dgv;
              gelu_tanh_and_grad_f(v, gv, dgv);
              v = pass == 1 ? gv : dgv;
            }
            if constexpr (EPI == EPI_DGELU) v *= (float)upre[PRE_U ? i : 0][PRE_U ? j : 0][r];
            ob[r] = f2bf(v);
          }
          stage_put(stg, j * 16 + (lane & 15), i * 4 + (lane >> 4), ob);
        }
      // GELU pass 0 = gelu'(u), read only in the backward: non-temporal
      if (EPI == EPI_GELU && pass == 0) stage_out<WM, true>(stg, (bf16*)e.C, e.ldc, mb, nb, M, N, lane);
      else stage_out<WM>(stg, (bf16*)(pass == 0 ? e.C : e.aux_out), e.ldc, mb, nb, M, N, lane);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = mb + j * 16 + (lane & 15), n = nb + i * 16 + g4;
      if (m < M && n < N) epilogue_store<EPI, OUTF32>(e, m, n, acc[i][j]);
    }
}

struct Plan {
  int bm, bn, bk, split;
};

// LDS-DMA variant of the 64x64 forward-layout tiles (measured fc2/out_proj fwd 22 -> 18.6 us; the
// dgrad / wgrad layouts and the 128x128 tiles measured slower or equal on it and stay register-staged).
// DTC_GEMM_DMA=0: register-staged everywhere (diagnostic)
inline bool gemm_dma_fwd64() {
  static const bool m = [] { const char* v = getenv("DTC_GEMM_DMA"); return v ? atoi(v) != 0 : true; }();
  return m;
}

// allow_split: 1 = small-grid split (wgrad), 2 = huge-K only (dgrad through the lm_head)
Plan make_plan(int M, int N, int K, int allow_split) {
  Plan p{128, 128, 64, 1};
  if (K % 64) {  // K a multiple of 32 only (e.g. a TP shard of d_model=768): BK=32, small tiles
    p.bm = p.bn = 64;
    p.bk = 32;
    return p;
  }
  const int nk = K / 64;
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
  if (allow_split && K >= 8192 && t128 >= 32) {  // e.g. dH = dlogits . W_lm (K = vocab)
    p.split = (int)std::max(1L, std::min((long)nk / 64, (512 + t128 - 1) / t128));
    return p;
  }
  // weight gradients: 128^2 tiles + split-K (A/B: 5.99 vs 6.05 ms on 64^2 tiles)
  if (allow_split == 1 && t128 < 256) {
    static const int target = [] { const char* v = getenv("DTC_WGRAD_BLOCKS"); return v ? atoi(v) : 256; }();
    while (t128 * p.split < target && nk / (p.split * 2) >= 8) p.split *= 2;
    return p;
  }
  if (t128 >= 256) return p;
  {
    p.bm = p.bn = 64;
    const long t64 = (long)((M + 63) / 64) * ((N + 63) / 64);
    if (allow_split == 1)
    {
      // weight gradients run on the backward side stream next to the dgrad chain: a grid that
      // fills every CU starves the critical path, so their split-K targets DTC_WGRAD_BLOCKS blocks
      static const int target = [] { const char* v = getenv("DTC_WGRAD_BLOCKS"); return v ? atoi(v) : 512; }();
      while (t64 * p.split < target && nk / (p.split * 2) >= 4) p.split *= 2;
    }
  }
  return p;
}

// Tile-group height for grids with many N-tiles (> 16): groups of gm M-tiles sweep the N-tiles, so the
// blocks an XCD runs at once share gm A panels (L2-resident) and stream the B panels.  Was gm = tiles_m
// (every M-tile of one N-tile in a row): an XCD then re-fetched all of A for each N-tile -- the GPT-2
// small fc1 forward / fc2 dgrad (24 N-tiles of 128) pulled 408 MB per call through L2 and the lm_head
// forward 3.5 GB (rocprofv3 FETCH_SIZE, profiles/r3_gpt2_small_pmc_final.md).  DTC_WIDE_GM: the height
// (0 = the old tiles_m).
inline int wide_gm(int tiles_m) {
  static const int g = [] { const char* v = getenv("DTC_WIDE_GM"); return v ? atoi(v) : 3; }();
  return g > 0 ? std::min(tiles_m, g) : tiles_m;
}

// exact byte extent of an operand (rows x K if K-major, K x rows if MN-major) for the buffer range check
inline int operand_bytes(bool kmajor, int rows, int K, long ld) {
  long n = kmajor ? ((long)(rows - 1) * ld + K) : ((long)(K - 1) * ld + rows);
  return (int)std::min(n * 2, (long)0x7FFFFFF0);
}

// Plan a register-staged launch of problem `a` with tile BMxBN (grid geometry, operand extents,
// epilogue) — shared by the single and the paired launch paths.
template <int BM, int BN, bool AK, bool BKM>
GemmLaunch make_launch(const GemmArgs& a, const Plan& p) {
  GemmLaunch g;
  Epi& e = g.e;
  e = Epi{};
  e.M = a.M; e.N = a.N; e.C = a.C; e.ldc = a.ldc; e.bias = a.bias; e.aux = a.aux; e.ldaux = a.ldaux;
  e.aux_out = a.aux_out; e.alpha = a.alpha; e.beta = a.beta; e.labels = a.labels; e.vocab_start = a.vocab_start;
  e.n_valid = a.n_valid; e.part = a.part; e.label_out = a.label_out;
  e.colsum = a.colsum;
  g.tiles_m = (a.M + BM - 1) / BM;
  g.tiles_n = (a.N + BN - 1) / BN;
  e.nparts = g.tiles_n * 2;
  const int nk = a.K / p.bk;
  g.kps = ((nk + p.split - 1) / p.split) * p.bk;
  const int ntiles = g.tiles_m * g.tiles_n;
  g.gm = wide_gm(g.tiles_m);
  if (g.tiles_n <= 16) g.gm = std::max(1, std::min(g.tiles_m, (ntiles / 8 + g.tiles_n - 1) / g.tiles_n));
  g.split = p.split;
  g.nblocks = ntiles * p.split;
  g.A = (const bf16*)a.A; g.lda = a.lda; g.a_bytes = operand_bytes(AK, a.M, a.K, a.lda);
  g.B = (const bf16*)a.B; g.ldb = a.ldb; g.b_bytes = operand_bytes(BKM, a.N, a.K, a.ldb);
  g.M = a.M; g.N = a.N; g.K = a.K;
  g.slab = (float*)a.workspace;
  return g;
}

template <int BM, int BN, bool AK, bool BKM, int EPI, bool OUTF32>
int launch_t(const GemmArgs& a, const Plan& p, hipStream_t st) {
  Epi e{};
  e.M = a.M; e.N = a.N; e.C = a.C; e.ldc = a.ldc; e.bias = a.bias; e.aux = a.aux; e.ldaux = a.ldaux;
  e.aux_out = a.aux_out; e.alpha = a.alpha; e.beta = a.beta; e.labels = a.labels; e.vocab_start = a.vocab_start;
  e.n_valid = a.n_valid; e.part = a.part; e.label_out = a.label_out;
  e.colsum = a.colsum;
  int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  e.nparts = tiles_n * 2;
  const int nk = a.K / p.bk;
  const int kps = ((nk + p.split - 1) / p.split) * p.bk;
  const int ntiles = tiles_m * tiles_n;
  // per-XCD share of tiles = ntiles*split/8: with few N-tiles make each XCD own whole M-row groups
  int gm = wide_gm(tiles_m);
  if (tiles_n <= 16) gm = std::max(1, std::min(tiles_m, (ntiles / 8 + tiles_n - 1) / tiles_n));
  dim3 grid(ntiles * p.split);
  const int ab = operand_bytes(AK, a.M, a.K, a.lda), bb = operand_bytes(BKM, a.N, a.K, a.ldb);
  if constexpr (BM == 64 && AK && BKM) {
    if (p.bk == 64 && gemm_dma_fwd64()) {
      hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, 4, AK, BKM, EPI, OUTF32>), grid, dim3(NT), 0, st, (const bf16*)a.A,
                         a.lda, (const bf16*)a.B, a.ldb, a.M, a.N, a.K, tiles_m, tiles_n, gm, p.split, kps,
                         (float*)a.workspace, e);
      DTC_CHECK_LAUNCH();
      if (p.split > 1 && !a.defer_reduce) {
        long MN = (long)a.M * a.N;
        int blocks = (int)((MN / 4 + 255) / 256);
        hipLaunchKernelGGL(splitk_reduce, dim3(blocks), dim3(256), 0, st, (const float*)a.workspace, p.split, MN,
                           (float*)a.C, a.ldc, a.N, a.beta);
        DTC_CHECK_LAUNCH();
      }
      return 0;
    }
  }
  if (p.bk == 32)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, 32, AK, BKM, EPI, OUTF32>), grid, dim3(NT), 0, st, (const bf16*)a.A, a.lda,
                       ab, (const bf16*)a.B, a.ldb, bb, a.M, a.N, a.K, tiles_m, tiles_n, gm, p.split, kps,
                       (float*)a.workspace, e);
  else if (p.bk == 64)
    hipLaunchKernelGGL((gemm_kernel<BM, BN, 64, AK, BKM, EPI, OUTF32>), grid, dim3(NT), 0, st, (const bf16*)a.A, a.lda,
                       ab, (const bf16*)a.B, a.ldb, bb, a.M, a.N, a.K, tiles_m, tiles_n, gm, p.split, kps,
                       (float*)a.workspace, e);
  else
    return 1007;
  DTC_CHECK_LAUNCH();
  if (p.split > 1 && !a.defer_reduce) {
    long MN = (long)a.M * a.N;
    int blocks = (int)((MN / 4 + 255) / 256);
    hipLaunchKernelGGL(splitk_reduce, dim3(blocks), dim3(256), 0, st, (const float*)a.workspace, p.split, MN,
                       (float*)a.C, a.ldc, a.N, a.beta);
    DTC_CHECK_LAUNCH();
  }
  return 0;
}

template <bool AK, bool BKM, int EPI, bool OUTF32>
int launch_sz(const GemmArgs& a, const Plan& p, hipStream_t st) {
  if (p.bm == 128) return launch_t<128, 128, AK, BKM, EPI, OUTF32>(a, p, st);
  return launch_t<64, 64, AK, BKM, EPI, OUTF32>(a, p, st);
}


// The 256^2 kernel pays on lm_head-sized problems.  Returns the split-K factor (0 = use the
// 128/64 kernels).  layout 0 (fwd): whole tiles; layout 1 (dgrad through the lm_head, K = vocab):
// split so ~256 blocks run (so does layout 0 at K >= 16384: the same dgrad as an NT GEMM on a
// transposed lm_head weight, ~25% faster main loop with both operands K-major); layout 2 (wgrad): no split (a 103 MB fp32 output; extra slab passes
// cost more than the last partial wave of tiles).
// DTC_WGRAD_CS256=0: bias gradients of the split-K 256^2 weight gradients as a separate column sum
static int g_wgrad_cs256 = [] { const char* v = getenv("DTC_WGRAD_CS256"); return v ? atoi(v) : 1; }();
static int g_wgrad256 = [] { const char* v = getenv("DTC_WGRAD256"); return v ? atoi(v) : 1; }();

int big_split(int layout, int M, int N, int K) {
  // DTC_GEMM256: bit mask of layouts allowed to use it (1 fwd, 2 dgrad, 4 wgrad; default all)
  static const int enabled = [] { const char* v = getenv("DTC_GEMM256"); return v ? atoi(v) : 7; }();
  if (!(enabled & (1 << layout)) || K % 64) return 0;
  if (layout != 0 && N % 8) return 0;              // MN-major B extent (dgrad / wgrad)
  if (layout == 2 && M % 8) return 0;              // MN-major A extent (wgrad)
  static const int min_tiles = [] { const char* v = getenv("DTC_BIG_MIN_TILES"); return v ? atoi(v) : 512; }();
  const long t = (long)((M + BIG - 1) / BIG) * ((N + BIG - 1) / BIG);
  if (layout == 2) {
    if (t >= 256 && K >= 1024) return 1;
    // DTC_WGRAD256=1 (default; in-step 14.30 -> 14.23 ms): layer weight gradients (K = tokens, a few dozen 256^2 tiles) split-K across
    // ~256 blocks of >= 8 K-steps on this kernel, fp32 slabs summed by the caller's reducer
    // K >= 8192 tokens: at the reference model's 4096 the split pieces are 4-8 K-steps and the grid half
    // empty (whole step 4.65 -> 5.04 ms with it, profiles/r3_ab_ref_regress.log)
    if (!g_wgrad256 || t < 8 || K < 8192) return 0;
    int split = (int)std::max(1L, 256 / t);
    while (split > 1 && (K / 64) / split < 8) --split;
    // fp32 slabs of one problem <= 96 MB (a layer's four weight gradients share the reducer's window)
    while (split > 1 && (long)split * M * N * 4 > (96L << 20)) --split;
    return split > 1 ? split : 0;
  }
  // ordinary K: whole tiles, when there are enough of them, or when the last round of 256^2 tiles is
  // nearly empty anyway (GPT-2 small qkv forward: 288 tiles = 1.125 rounds, 54.7 -> 47.7 us;
  // fc1's 384 = 1.5 rounds stays on the 128^2 kernel: 76 vs 85 us, profiles/r3_gemm_bench_gpt2s*.log)
  static const int tail_ok = [] { const char* v = getenv("DTC_BIG_TAIL"); return v ? atoi(v) : 64; }();
  if (K < 16384) return (t >= min_tiles || (layout == 0 && t >= 256 && t % 256 <= tail_ok)) ? 1 : 0;
  if (t > 256) return 0;                           // dgrad through the vocab (NN, or NT on W^T): split-K
  int split = (int)std::max(1L, 256 / t);
  while (split > 1 && (K / 64) / split < 8) --split;
  return split;
}

inline int big_kps(int K, int split) { return ((K / 64 + split - 1) / split) * 64; }

// compute units of the current device (one-block-per-CU persistent grids)
static int cu_count() {
  static const int n = [] {
    int d = 0, v = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess) v = 0;
    return v > 0 ? v : 256;
  }();
  return n;
}

// default on: GPT-2 small lm_head dgrad 553 -> 502 us, step 11.01-11.04 vs 11.04-11.09 ms
// (profiles/r4_ab_big_cb3.log)
static int g_big_cb3 = [] { const char* v = getenv("DTC_BIG_CB3"); return v ? atoi(v) : 1; }();
template <bool AK, bool BKM, int EPI, bool OUTF32>
int launch_big(const GemmArgs& a, int split, hipStream_t st) {
  Epi e{};
  e.M = a.M; e.N = a.N; e.C = a.C; e.ldc = a.ldc; e.bias = a.bias; e.aux = a.aux; e.ldaux = a.ldaux;
  e.aux_out = a.aux_out; e.alpha = a.alpha; e.beta = a.beta; e.labels = a.labels; e.vocab_start = a.vocab_start;
  e.n_valid = a.n_valid; e.part = a.part; e.label_out = a.label_out;
  e.colsum = a.colsum;  // fused bias gradient (gemm8p_kernel, layout TN only)
  const int tiles_m = (a.M + BIG - 1) / BIG, tiles_n = (a.N + BIG - 1) / BIG;
  e.nparts = tiles_n * 4;
  const int ntiles = tiles_m * tiles_n;
  // tile order: groups of gm M-tiles sweep all N-tiles.  With few N-tiles a group is sized to the
  // ~32 blocks an XCD runs at once, so the N-tiles sharing an A panel run together on one L2 (a group
  // spanning a whole XCD run -- 74 tiles of the lm_head weight gradient -- left 2 of its 3 N-tiles
  // re-fetching their A panel from HBM: 2x FETCH_SIZE, profiles/r3_gemm8p.md)
  int gm = wide_gm(tiles_m);
  if (tiles_n <= 16) gm = std::max(1, std::min(tiles_m, 32 / tiles_n));
  const int kps = big_kps(a.K, split);
  if (split > 1 && (a.ws_bytes < (long)split * a.M * a.N * 4 || a.N % 4)) return 1005;
  // DTC_BIG_CB3: split-K problems whose 256^2 grid leaves CUs idle (the GPT-2 small lm_head dgrad: 96 tiles
  // x split 2 = 192 blocks) run 256 x 192 tiles when that grid is exactly one block per CU (128 x 2 = 256)
  const int cb3 = g_big_cb3;
  bool done = false;
  if constexpr (EPI == EPI_STORE && OUTF32) {
    const int tn3 = a.N / 192;
    if (cb3 && split > 1 && a.N % 192 == 0 && ntiles * split < cu_count() && tiles_m * tn3 * split == cu_count()) {
      const int gm3 = std::max(1, std::min(tiles_m, 32 / tn3));
      hipLaunchKernelGGL((gemm8p_kernel<AK, BKM, EPI, OUTF32, 3>), dim3(tiles_m * tn3 * split), dim3(NT2), 0, st,
                         (const bf16*)a.A, a.lda, (const bf16*)a.B, a.ldb, a.M, a.N, a.K, tiles_m, tn3, gm3, split,
                         kps, (float*)a.workspace, e);
      DTC_CHECK_LAUNCH();
      done = true;
    }
  }
  if (!done) {
    hipLaunchKernelGGL((gemm8p_kernel<AK, BKM, EPI, OUTF32>), dim3(ntiles * split), dim3(NT2), 0, st,
                       (const bf16*)a.A, a.lda, (const bf16*)a.B, a.ldb, a.M, a.N, a.K, tiles_m, tiles_n, gm, split,
                       kps, (float*)a.workspace, e);
    DTC_CHECK_LAUNCH();
  }
  if (split > 1 && !a.defer_reduce) {
    long MN = (long)a.M * a.N;
    int blocks = (int)((MN / 4 + 255) / 256);
    hipLaunchKernelGGL(splitk_reduce, dim3(blocks), dim3(256), 0, st, (const float*)a.workspace, split, MN,
                       (float*)a.C, a.ldc, a.N, a.beta);
    DTC_CHECK_LAUNCH();
  }
  return 0;
}

// ---- gemm8r plans (layer GEMMs on 256-row tiles of two widths, one launch) ---------------------------
// DTC_GEMM8R: 1 (default) = use the plan for NT problems (forwards, dgrads on transposed weights) with a bf16
// staged epilogue (plain + bias, GELU pair, dGELU) whose 256^2 grid is not whole rounds; 2 = also fp32
// outputs (measured slower: out_proj f32 21 -> 29 us); 4 = also NN problems (dgrads on the row-major weight:
// the fc2 dgrad + dGELU); 0 = off.  HBM-cold, GPT-2 small (profiles/r5_gemm8r.md):
// qkv fwd 44.5 -> 41.6 us, fc1 fwd + GELU 67.3 -> 54.9, fc2 NT dgrad + dGELU 73.7 -> 61.3; step 10.89 -> 10.74 ms
// NN added (default 5): fc2 dgrad + dGELU on the row-major weight 74.3 -> 62.3 us cold, step 10.84 -> 10.74 ms
// (profiles/r5_gemm8r.md), level with the NT form on a transposed copy (DTC_DGRAD_NT_FC2=1: 10.76 ms)
static int g_r8_mask = [] { const char* v = getenv("DTC_GEMM8R"); return v ? atoi(v) : 5; }();
// DTC_R8_ILV: interleaved gemm8r block order (r8_block); A/B switch, set at run time by dtc_gemm_set_r8_ilv
static int g_r8_ilv = [] { const char* v = getenv("DTC_R8_ILV"); return v ? atoi(v) : 1; }();

struct R8Plan {
  int n_split = -1, cb2 = 0;
};

static R8Plan r8_plan(int layout, int M, int N, int K, int epi, bool f32) {
  R8Plan r;
  if (!g_r8_mask || !(layout == 0 || (layout == 1 && (g_r8_mask & 4))) || M % BIG || N % 64 || K % 64 || K < 256 ||
      K > 4096 || N > 16384)
    return r;
  if (!(epi == EPI_STORE || epi == EPI_GELU || epi == EPI_DGELU)) return r;
  if (f32 && (epi != EPI_STORE || !(g_r8_mask & 2))) return r;
  const int tm = M / BIG, q = N / BIG, cus = cu_count();
  if ((long)tm * q % cus == 0 && q > 0 && N % BIG == 0) return r;  // whole rounds of 256^2 tiles: launch_big
  int c1 = q;
  while (c1 > 0 && ((long)tm * c1) % cus) --c1;  // whole rounds of 256^2 tiles
  const int u = (N - BIG * c1) / 64;
  int best = 0;
  long best_cost = 0;
  for (int cb : {4, 2, 1}) {
    if (u % cb) continue;
    const long blocks = (long)tm * (u / cb);
    const long cost = ((blocks + cus - 1) / cus) * cb;  // rounds x tile width
    if (!best || cost < best_cost) {
      best = cb;
      best_cost = cost;
    }
  }
  if (!best) return r;
  r.n_split = BIG * c1;
  r.cb2 = best;
  return r;
}

template <bool AK, bool BKM, int EPI, bool OUTF32, int CB2>
int launch_r8_cb(const GemmArgs& a, const R8Plan& pl, hipStream_t st) {
  Epi e{};
  e.M = a.M; e.N = a.N; e.C = a.C; e.ldc = a.ldc; e.bias = a.bias; e.aux = a.aux; e.ldaux = a.ldaux;
  e.aux_out = a.aux_out; e.alpha = a.alpha; e.beta = a.beta;
  R8Args r;
  r.A = (const bf16*)a.A; r.lda = a.lda; r.B = (const bf16*)a.B; r.ldb = a.ldb;
  r.M = a.M; r.N = a.N; r.K = a.K; r.n_split = pl.n_split;
  r.tm = a.M / BIG;
  r.tn1 = pl.n_split / BIG;
  r.nb1 = r.tm * r.tn1;
  r.gm1 = r.tn1 > 0 ? std::max(1, std::min(r.tm, 32 / r.tn1)) : 1;
  r.tn2 = (a.N - pl.n_split) / (64 * CB2);
  r.gm2 = std::max(1, std::min(r.tm, 32 / std::max(1, r.tn2)));
  r.ilv = g_r8_ilv && r.nb1 >= 2 && r.tm * r.tn2 >= 2;
  const int grid = r.nb1 + r.tm * r.tn2;
  hipLaunchKernelGGL((gemm8r_kernel<AK, BKM, EPI, OUTF32, CB2>), dim3(grid), dim3(NT2), 0, st, r, e);
  DTC_CHECK_LAUNCH();
  return 0;
}

template <int EPI, bool OUTF32, bool BKM = true>
int launch_r8(const GemmArgs& a, const R8Plan& pl, hipStream_t st) {
  if (pl.cb2 == 4) return launch_r8_cb<true, BKM, EPI, OUTF32, 4>(a, pl, st);
  if (pl.cb2 == 2) return launch_r8_cb<true, BKM, EPI, OUTF32, 2>(a, pl, st);
  return launch_r8_cb<true, BKM, EPI, OUTF32, 1>(a, pl, st);
}

// ---- gemm8n_kernel plans (layer GEMMs, 128 x 64*CB tiles) ----------------------------------------
// DTC_GEMM8N bit mask: 1 = forwards and NT dgrads (layout 0), 2 = NN dgrads (layout 1), 4 = also
// multi-round problems.  A problem takes it when its tile count on 128x192 (CB 3) or 128x256 (CB 4)
// tiles is exactly one round of 256 (the d_model-wide outputs of GPT-2 small / medium at 8192 tokens:
// out_proj / fc2 forwards, qkv / fc1 / out_proj dgrads).  Measured (profiles/r3_gemm8n.md): one round
// wins (fc1 NT dgrad 60.8 -> 44.9 us, fc2 forward 63.5 -> 49.5 us); 3-4 rounds lose to the 128^2 /
// 256^2 kernels (fc1 forward 75.6 -> 85.6 us: each round pays its own prologue fill and epilogue at
// one block per CU), and so does a vocab-sized K (the lm_head dgrad keeps its split-K 256^2 kernel).
static int g_n8_mask = [] { const char* v = getenv("DTC_GEMM8N"); return v ? atoi(v) : 3; }();
// DTC_N8_CB: only this tile width (3 = 128 x 192, 4 = 128 x 256) for gemm8n plans (0 = 3 then 4; A/B)
static int g_n8_cb = [] { const char* v = getenv("DTC_N8_CB"); return v ? atoi(v) : 0; }();

// DTC_N8_MINK: smallest K of a one-round gemm8n problem (default 1024; 768 = also the out_proj forward /
// dgrad, whose plain stores take the overlapped epilogue since the residual add moved to the LayerNorm)
static int g_n8_mink = [] { const char* v = getenv("DTC_N8_MINK"); return v ? atoi(v) : 1024; }();

static int n8_cb(int layout, int M, int N, int K, int epi) {
  // K >= 1024: at K = 768 (out_proj forward, 12 K-steps) the one-block-per-CU epilogue (fp32 residual
  // in + out, nothing to hide it under) costs more than the main loop gains (29.2 vs 26.6 us)
  if (layout > 1 || !(g_n8_mask & (1 << layout)) || K % 64 || K < 768 || K > 8192 || M < 128) return 0;
  if (epi != EPI_STORE && epi != EPI_RESID && epi != EPI_GELU && epi != EPI_DGELU) return 0;
  const long tm = (M + 127) / 128;
  for (int cb : {3, 4}) {
    if (g_n8_cb && cb != g_n8_cb) continue;
    const int bn = 64 * cb;
    if (N % bn) continue;
    const long t = tm * (N / bn);
    if ((t == 256 && K >= g_n8_mink) || ((g_n8_mask & 4) && t > 256 && t % 256 == 0)) return cb;
  }
  return 0;
}

template <int CB, bool AK, bool BKM, int EPI, bool OUTF32>
int launch_n8(const GemmArgs& a, hipStream_t st) {
  Epi e{};
  e.M = a.M; e.N = a.N; e.C = a.C; e.ldc = a.ldc; e.bias = a.bias; e.aux = a.aux; e.ldaux = a.ldaux;
  e.aux_out = a.aux_out; e.alpha = a.alpha; e.beta = a.beta;
  const int tiles_m = (a.M + 127) / 128, tiles_n = a.N / (64 * CB);
  // an XCD's ~32 concurrent tiles = 8 M-tiles x 4 N-tiles (A panel and B panel both shared)
  const int gm = tiles_n <= 4 ? std::max(1, std::min(tiles_m, 32 / tiles_n)) : std::min(tiles_m, 8);
  constexpr int NS = CB == 3 ? 4 : 3;
  const int grid = std::min(tiles_m * tiles_n, cu_count());  // persistent: one block per CU
  hipLaunchKernelGGL((gemm8n_kernel<CB, NS, AK, BKM, EPI, OUTF32>), dim3(grid), dim3(NT2), 0, st,
                     (const bf16*)a.A, a.lda, (const bf16*)a.B, a.ldb, a.M, a.N, a.K, tiles_m, tiles_n, gm, e);
  DTC_CHECK_LAUNCH();
  return 0;
}

template <bool AK, bool BKM, int EPI, bool OUTF32>
int launch_n8cb(const GemmArgs& a, int cb, hipStream_t st) {
  return cb == 3 ? launch_n8<3, AK, BKM, EPI, OUTF32>(a, st) : launch_n8<4, AK, BKM, EPI, OUTF32>(a, st);
}

// the (layout, epilogue, output) combinations the layer GEMMs use; -1 = not instantiated
int launch_n8_any(const GemmArgs& a, int cb, hipStream_t st) {
  const int epi = a.epi;
  const bool f32 = a.c_f32 != 0;
  if (a.layout == 0) {
    if (epi == EPI_STORE) return f32 ? launch_n8cb<true, true, EPI_STORE, true>(a, cb, st)
                                     : launch_n8cb<true, true, EPI_STORE, false>(a, cb, st);
    if (epi == EPI_RESID && f32) return launch_n8cb<true, true, EPI_RESID, true>(a, cb, st);
    if (epi == EPI_GELU && !f32) return launch_n8cb<true, true, EPI_GELU, false>(a, cb, st);
    if (epi == EPI_DGELU && !f32) return launch_n8cb<true, true, EPI_DGELU, false>(a, cb, st);
  } else if (a.layout == 1 && a.N % 8 == 0) {
    if (epi == EPI_STORE) return f32 ? launch_n8cb<true, false, EPI_STORE, true>(a, cb, st)
                                     : launch_n8cb<true, false, EPI_STORE, false>(a, cb, st);
    if (epi == EPI_DGELU && !f32) return launch_n8cb<true, false, EPI_DGELU, false>(a, cb, st);
  }
  return -1;
}

// Paired launch: a1 = dgrad (layout 1, whole-K tiles), a2 = weight gradient (layout 2, split-K slabs
// left for the caller's batched reducer when split > 1).  Only register-staged, BK = 64 plans pair.
template <class C1, class C2, int BM1, int BM2, bool BKM1 = false>
int launch_pair_t(const GemmArgs& a1, const Plan& p1, const GemmArgs& a2, const Plan& p2, hipStream_t st) {
  const GemmLaunch g1 = make_launch<BM1, BM1, true, BKM1>(a1, p1);
  const GemmLaunch g2 = make_launch<BM2, BM2, false, false>(a2, p2);
  if (g1.nblocks % 8 && g2.nblocks % 8) return 1100;  // XCD maps would disagree: not pairable
  // the dgrad blocks dispatch first unless only the weight-gradient count keeps the XCD maps aligned
  // (weight gradients first measured slower: 5.348 vs 5.284 ms/step, round 2)
  const int second_first = g1.nblocks % 8 ? 1 : 0;
  hipLaunchKernelGGL((gemm_pair_kernel<C1, C2>), dim3(g1.nblocks + g2.nblocks), dim3(NT), 0, st, g1, g2,
                     second_first);
  DTC_CHECK_LAUNCH();
  return 0;
}

template <int EPI1, bool F1>
int launch_pair_w(const GemmArgs& a1, const Plan& p1, const GemmArgs& a2, const Plan& p2, hipStream_t st) {
  using W128 = GemmCfg<128, 128, 64, false, false, EPI_STORE, true>;
  using W64 = GemmCfg<64, 64, 64, false, false, EPI_STORE, true>;
  if (a1.layout == 0) {  // dgrad as NT on the transposed weight (both operands K-major)
    if (p1.bm != 128 || p2.bm != 128) return 1100;
    using D = GemmCfg<128, 128, 64, true, true, EPI1, F1>;
    return launch_pair_t<D, W128, 128, 128, true>(a1, p1, a2, p2, st);
  }
  if (p1.bm == 128) {
    using D = GemmCfg<128, 128, 64, true, false, EPI1, F1>;
    return p2.bm == 128 ? launch_pair_t<D, W128, 128, 128>(a1, p1, a2, p2, st)
                        : launch_pair_t<D, W64, 128, 64>(a1, p1, a2, p2, st);
  }
  using D = GemmCfg<64, 64, 64, true, false, EPI1, F1>;
  return p2.bm == 128 ? launch_pair_t<D, W128, 64, 128>(a1, p1, a2, p2, st)
                      : launch_pair_t<D, W64, 64, 64>(a1, p1, a2, p2, st);
}

// ---- 8-wave DMA plans (gemm_dmaw_kernel) for the layer-GEMM shapes ------------------------------
// Main loop only, L2-hot and back to back (benchmarks/gemm_dma8_micro.hip) the 8-wave configs beat the
// 4-wave kernels on every layer shape (e.g. fc1 fwd 10.9 -> 8.8 us, fc1 dgrad 26 -> 18 us), but in the
// step (rocprofv3, profiles/r2_gemm_w8_instep.md) only two keep a gain once their epilogues and
// in-step operand traffic are counted: the fp32 residual forwards (out_proj, fc2: 128x64 tiles, 16.1
// -> 14.4 us per call) and the bias-free small weight gradient (out_proj: 64x128, split 8, 11.4 ->
// 10.8 us).  The 256x128 bf16 forwards tie (14.4 vs 14.7, 22.9 vs 22.6 us: the all-CU epilogue
// dominates), the dgrads lose (fc1 dgrad 26.5 -> 34-36 us) and unpairing the fc2 / qkv
// dgrad+weight-gradient launches loses (37.9 -> 49.6, 36.1 -> 43.4 us).  Those configs stay
// selectable for experiments (DTC_GEMM_W8=2) but are off in the default plan.
enum { W_NONE = -1, W_256x128 = 0, W_128x64 = 1, W_64x128 = 2, W_128x128 = 3 };

inline int gemm_w8_mode() {  // DTC_GEMM_W8 bits: 1 = measured winners (default), 2 = every config, 4 = 128x64 fp32 dgrads
  static const int v = [] { const char* s = getenv("DTC_GEMM_W8"); return s ? atoi(s) : 1; }();
  return v;
}

struct WPlan {
  int cfg, split;
};

// The 8-wave config (and split-K) of a problem, or W_NONE.  Layer-sized problems only (the lm_head
// GEMMs keep the 256^2 kernel); weight gradients that fuse their bias column sums (has_colsum) stay
// on the register-staged kernel, which reads dY through registers.
WPlan dmaw_plan(int layout, int M, int N, int K, int epi, bool f32, bool has_colsum) {
  WPlan w{W_NONE, 1};
  const int mode = gemm_w8_mode();
  if (!(mode & 7) || K % 64 || M % 8 || N % 8) return w;
  const bool all = (mode & 2) != 0;
  auto tiles = [&](int bm, int bn) { return (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (layout == 0) {
    if (all && !f32 && (epi == EPI_STORE || epi == EPI_GELU) && K <= 1024 && tiles(256, 128) >= 128 &&
        tiles(256, 128) <= 512)
      w.cfg = W_256x128;
    else if ((f32 ? (epi == EPI_RESID || epi == EPI_STORE) : epi == EPI_STORE) && K <= 4096 && tiles(128, 64) >= 192 &&
             tiles(128, 64) <= 512)
      w.cfg = W_128x64;
  } else if (layout == 1) {
    if (all && !f32 && epi == EPI_DGELU && K <= 1024 && tiles(256, 128) >= 128 && tiles(256, 128) <= 512)
      w.cfg = W_256x128;
    else if (all && epi == EPI_STORE && K <= 4096 && tiles(64, 128) >= 192 && tiles(64, 128) <= 512)
      w.cfg = W_64x128;
    else if ((mode & 4) && epi == EPI_STORE && f32 && K <= 4096 && tiles(128, 64) >= 192 && tiles(128, 64) <= 512)
      w.cfg = W_128x64;
  } else if (layout == 2 && epi == EPI_STORE && f32 && !has_colsum && tiles(128, 128) <= 256 &&
             (all || tiles(128, 128) <= 48)) {
    // (<= 48 tiles: also GPT-2's [768 x 768] out_proj weight gradient, 53.4 -> 38.3 us)
    // weight gradient (K = tokens): split-K towards 256 blocks of >= 8 k-steps
    const int nk = K / 64;
    const int cfg = tiles(128, 128) >= 32 ? W_128x128 : W_64x128;
    const long t = cfg == W_128x128 ? tiles(128, 128) : tiles(64, 128);
    int split = 1;
    while (t * split * 2 <= 256 && nk / (split * 2) >= 8) split *= 2;
    w.cfg = cfg;
    w.split = split;
  }
  return w;
}

template <int BM, int BN, int NS, int WGM, int WGN, bool AK, bool BKM, int EPI, bool OUTF32>
int launch_w(const GemmArgs& a, int split, hipStream_t st) {
  Epi e{};
  e.M = a.M; e.N = a.N; e.C = a.C; e.ldc = a.ldc; e.bias = a.bias; e.aux = a.aux; e.ldaux = a.ldaux;
  e.aux_out = a.aux_out; e.alpha = a.alpha; e.beta = a.beta; e.labels = a.labels; e.vocab_start = a.vocab_start;
  e.n_valid = a.n_valid; e.part = a.part; e.label_out = a.label_out; e.colsum = nullptr;
  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  e.nparts = tiles_n * WGN;
  const int ntiles = tiles_m * tiles_n;
  int gm = wide_gm(tiles_m);
  if (tiles_n <= 16) gm = std::max(1, std::min(tiles_m, (ntiles / 8 + tiles_n - 1) / tiles_n));
  const int nk = a.K / 64;
  const int kps = ((nk + split - 1) / split) * 64;
  if (split > 1 && a.ws_bytes < (long)split * a.M * a.N * 4) return 1005;
  hipLaunchKernelGGL((gemm_dmaw_kernel<BM, BN, NS, WGM, WGN, AK, BKM, EPI, OUTF32>), dim3(ntiles * split),
                     dim3(64 * WGM * WGN), 0, st, (const bf16*)a.A, a.lda, (const bf16*)a.B, a.ldb, a.M, a.N, a.K, tiles_m,
                     tiles_n, gm, split, kps, (float*)a.workspace, e);
  DTC_CHECK_LAUNCH();
  if (split > 1 && !a.defer_reduce) {
    long MN = (long)a.M * a.N;
    hipLaunchKernelGGL(splitk_reduce, dim3((int)((MN / 4 + 255) / 256)), dim3(256), 0, st, (const float*)a.workspace, split,
                       MN, (float*)a.C, a.ldc, a.N, a.beta);
    DTC_CHECK_LAUNCH();
  }
  return 0;
}

// only the (config, layout, epilogue) combinations dmaw_plan can return are instantiated
template <bool AK, bool BKM, int EPI, bool OUTF32>
int launch_wcfg(const GemmArgs& a, const WPlan& w, hipStream_t st) {
  if constexpr (!OUTF32 && (EPI == EPI_STORE || EPI == EPI_GELU || EPI == EPI_DGELU) && (AK && (BKM || EPI == EPI_DGELU)))
    if (w.cfg == W_256x128) return launch_w<256, 128, 2, 4, 2, AK, BKM, EPI, OUTF32>(a, w.split, st);
  if constexpr (AK && ((OUTF32 && (EPI == EPI_STORE || (BKM && EPI == EPI_RESID))) || (BKM && !OUTF32 && EPI == EPI_STORE)))
    if (w.cfg == W_128x64) return launch_w<128, 64, 4, 4, 2, AK, BKM, EPI, OUTF32>(a, w.split, st);
  if constexpr (EPI == EPI_STORE && ((AK && !BKM) || (!AK && !BKM && OUTF32)))
    if (w.cfg == W_64x128) return launch_w<64, 128, 4, 2, 4, AK, BKM, EPI, OUTF32>(a, w.split, st);
  if constexpr (!AK && !BKM && OUTF32 && EPI == EPI_STORE)
    if (w.cfg == W_128x128) return launch_w<128, 128, 4, 4, 2, AK, BKM, EPI, OUTF32>(a, w.split, st);
  return 1101;  // not instantiated (dmaw_plan and this table disagree)
}

}  // namespace

extern "C" {

// dgrad (a1: layout 1, epi STORE or DGELU) and weight gradient (a2: layout 2, fp32, defer_reduce
// when split) of one Dense in one launch.  Returns 1100 when the pair cannot share a launch (the
// caller then issues the two GEMMs separately).
int dtc_gemm_pair(const GemmArgs* a1, const GemmArgs* a2, hipStream_t st) {
  if ((a1->layout != 1 && a1->layout != 0) || a2->layout != 2) return 1100;
  if (a1->K % 64 || a2->K % 64 || a1->N % 8 || a2->M % 8 || a2->N % 8) return 1100;
  if (a1->lda % 8 || a1->ldb % 8 || a1->ldc % 4 || a2->lda % 8 || a2->ldb % 8 || a2->ldc % 4) return 1100;
  if (a1->M <= 0 || a1->N <= 0 || a2->M <= 0 || a2->N <= 0) return 1100;
  if (a2->epi != EPI_STORE || !a2->c_f32 || a2->bias) return 1100;
  if (big_split(a1->layout, a1->M, a1->N, a1->K) || big_split(2, a2->M, a2->N, a2->K)) return 1100;
  if (n8_cb(a1->layout, a1->M, a1->N, a1->K, a1->epi)) return 1100;  // dgrad on gemm8n_kernel: own launch
  if (a1->alpha == 1.f && a1->beta == 0.f && !a1->colsum &&
      r8_plan(a1->layout, a1->M, a1->N, a1->K, a1->epi, a1->c_f32 != 0).cb2)
    return 1100;  // dgrad on gemm8r_kernel: own launch (the same plan dtc_gemm picks for it alone)
  if (dmaw_plan(a1->layout, a1->M, a1->N, a1->K, a1->epi, a1->c_f32 != 0, false).cfg != W_NONE ||
      dmaw_plan(2, a2->M, a2->N, a2->K, a2->epi, a2->c_f32 != 0, a2->colsum != nullptr).cfg != W_NONE)
    return 1100;  // the 8-wave kernels run these as two launches
  const Plan p1 = make_plan(a1->M, a1->N, a1->K, (a1->layout == 1 && a1->epi == EPI_STORE && a1->c_f32) ? 2 : 0);
  const Plan p2 = make_plan(a2->M, a2->N, a2->K, 1);
  if (p1.split != 1 || p1.bk != 64 || p2.bk != 64) return 1100;
  if (p2.split > 1 && (!a2->defer_reduce || a2->ws_bytes < (long)p2.split * a2->M * a2->N * 4)) return 1100;
  if (a1->epi == EPI_DGELU && !a1->c_f32) return launch_pair_w<EPI_DGELU, false>(*a1, p1, *a2, p2, st);
  if (a1->epi == EPI_STORE && a1->c_f32) return launch_pair_w<EPI_STORE, true>(*a1, p1, *a2, p2, st);
  if (a1->epi == EPI_STORE && !a1->c_f32) return launch_pair_w<EPI_STORE, false>(*a1, p1, *a2, p2, st);
  return 1100;
}

// Fused lm_head backward (ce_dgrad256_kernel): dX [M][N] fp32 (= sum of the split-K slabs, written
// by splitk_reduce), dlogits [M][K] bf16, colpart [2*ceil(M/256)][K] fp32.  K % 64 == 0, N % 8 == 0.
// split-K of the fused lm_head dgrad: the big_split plan (forced 4 / 5 / 8 measured within noise)
static int ce_split(int M, int N, int K) { return std::max(1, big_split(1, M, N, K)); }

long dtc_ce_dgrad_workspace_bytes(int M, int N, int K) {
  const int split = ce_split(M, N, K);
  return split > 1 ? (long)split * M * N * 4 : (long)M * N * 4;
}
int dtc_ce_dgrad_colpart_rows(int M) { return 2 * ((M + BIG - 1) / BIG); }

int dtc_ce_dgrad(const bf16* logits, long ldl, const float* lse, const int* labels, int vocab_start, int n_valid,
                 float scale, const bf16* wt, long ldw, bf16* dlogits, long ldd, float* colpart, float* dx, int M, int N,
                 int K, float* ws, long ws_bytes, hipStream_t st) {
  if (K % 64 || N % 8 || ldl % 8 || ldw % 8 || ldd % 8) return 1300;
  const int split = ce_split(M, N, K);
  if (ws_bytes < (long)split * M * N * 4) return 1301;
  CeDgradArgs a;
  a.logits = logits; a.ldl = ldl; a.lse = lse; a.labels = labels; a.vocab_start = vocab_start; a.n_valid = n_valid;
  a.scale = scale; a.wt = wt; a.ldw = ldw; a.dlogits = dlogits; a.ldd = ldd; a.colpart = colpart; a.slab = ws;
  a.M = M; a.N = N; a.K = K;
  a.tiles_m = (M + BIG - 1) / BIG;
  a.tiles_n = (N + BIG - 1) / BIG;
  const int ntiles = a.tiles_m * a.tiles_n;
  a.gm = a.tiles_m;
  if (a.tiles_n <= 16) a.gm = std::max(1, std::min(a.tiles_m, (ntiles * split / 8 + a.tiles_n - 1) / a.tiles_n));
  a.split = split;
  a.kps = big_kps(K, split);
  hipLaunchKernelGGL(ce_dgrad256_kernel, dim3(ntiles * split), dim3(NT2), 0, st, a);
  DTC_CHECK_LAUNCH();
  const long MN = (long)M * N;
  hipLaunchKernelGGL(splitk_reduce, dim3((int)((MN / 4 + 255) / 256)), dim3(256), 0, st, (const float*)ws, split, MN,
                     dx, (long)N, N, 0.f);
  DTC_CHECK_LAUNCH();
  return 0;
}

int dtc_gemm_ln(const LnArgs* a, hipStream_t st) {
  if (a->M <= 0 || a->M % 128 || a->N % 256 || a->N > 1024 || a->K <= 0 || a->K % 64) return 1400;
  if (a->lda % 8 || a->ldb % 8) return 1400;
  if (!a->sync || !a->step || !a->gamma || !a->err || !a->C || !a->y || !a->mean || !a->rstd) return 1401;
  if (a->bwd ? (!a->x || !a->part || a->nslab < 2 || a->nslab > 3) : (!a->resid || !a->beta)) return 1402;
  Epi e{};
  e.M = a->M; e.N = a->N; e.C = a->C; e.ldc = a->N; e.bias = a->bwd ? nullptr : a->bias;
  e.aux = a->resid; e.ldaux = a->N; e.alpha = 1.f;
  e.ln.gamma = a->gamma; e.ln.beta = a->beta; e.ln.y = (bf16*)a->y; e.ln.mean = a->mean; e.ln.rstd = a->rstd;
  e.ln.x = a->x; e.ln.part = a->part; e.ln.nslab = a->nslab; e.ln.eps = a->eps;
  e.ln.sync = a->sync; e.ln.step = a->step; e.ln.site = a->site; e.ln.nsites = a->nsites; e.ln.err = a->err;
  const int tiles_m = a->M / 128, tiles_n = a->N / 64;
  const dim3 grid(tiles_m * tiles_n), block(512);
  if (a->bwd)
    hipLaunchKernelGGL((gemm_dmaw_kernel<128, 64, 4, 4, 2, true, true, EPI_LN_BWD, true>), grid, block, 0, st,
                       (const bf16*)a->A, a->lda, (const bf16*)a->B, a->ldb, a->M, a->N, a->K, tiles_m, tiles_n, tiles_m,
                       1, a->K, nullptr, e);
  else
    hipLaunchKernelGGL((gemm_dmaw_kernel<128, 64, 4, 4, 2, true, true, EPI_RESID_LN, true>), grid, block, 0, st,
                       (const bf16*)a->A, a->lda, (const bf16*)a->B, a->ldb, a->M, a->N, a->K, tiles_m, tiles_n, tiles_m,
                       1, a->K, nullptr, e);
  DTC_CHECK_LAUNCH();
  return 0;
}

long dtc_gemm_ln_sync_words(int M, int N) { return (long)M * (N / 32) + (long)(M / 128) * (N / 64); }

int dtc_lmhead_nparts(int M, int N, int K) { return big_split(0, M, N, K) ? ((N + 255) / 256) * 4 : ((N + 127) / 128) * 2; }

// split-K factor dtc_gemm will use for a weight-gradient (layout 2) problem (1 = none); has_db: the
// caller wants the bias gradient fused (GemmArgs.colsum), which pins the register-staged kernel
int dtc_gemm_wgrad_split(int M, int N, int K, int has_db) {
  if (const int bs = big_split(2, M, N, K)) return bs;
  if (!has_db) {
    const WPlan w = dmaw_plan(2, M, N, K, EPI_STORE, true, false);
    if (w.cfg != W_NONE) return w.split;
  }
  return make_plan(M, N, K, 1).split;
}

// 1 if the weight-gradient GEMM runs on the register-staged kernel, which can fuse the bias
// gradient (GemmArgs.colsum); the 256^2 and DMA kernels cannot
int dtc_gemm_wgrad_fuses_colsum(int M, int N, int K) {
  if (big_split(2, M, N, K)) return g_wgrad_cs256 ? 1 : 0;  // gemm8p_kernel sums it with MFMAs
  return 1;  // the register-staged 64^2 / 128^2 weight-gradient plans (never the DMA variant)
}

long dtc_gemm_workspace_bytes(int layout, int M, int N, int K) {
  Plan p = make_plan(M, N, K, layout == 2 ? 1 : (layout == 1 ? 2 : 0));
  const int bs = big_split(layout, M, N, K);
  int split = bs ? bs : p.split;
  if (layout == 2 && !bs) split = std::max(split, dmaw_plan(2, M, N, K, EPI_STORE, true, false).split);
  return split > 1 ? (long)split * M * N * 4 : 0;
}

// weight gradients split-K on the 256^2 kernel (DTC_WGRAD256 at load time); returns the previous value
int dtc_gemm_set_wgrad256(int on) {
  const int old = g_wgrad256;
  g_wgrad256 = on;
  return old;
}

// gemm8n layout mask (DTC_GEMM8N at load time); returns the previous mask (tests / A/B)
int dtc_gemm_set_n8(int mask) {
  const int old = g_n8_mask;
  g_n8_mask = mask;
  return old;
}

// 256 x 192 split-K plan of launch_big (DTC_BIG_CB3 at load time); returns the previous value
int dtc_gemm_set_big_cb3(int on) {
  const int old = g_big_cb3;
  g_big_cb3 = on;
  return old;
}

int dtc_gemm_set_n8_mink(int k) {
  const int old = g_n8_mink;
  g_n8_mink = k;
  return old;
}

int dtc_gemm_set_n8_cb(int cb) {
  const int old = g_n8_cb;
  g_n8_cb = cb;
  return old;
}

int dtc_wg_entry_bytes() { return (int)sizeof(WgEntry); }
int dtc_wg_max() { return WG_MAX; }
int dtc_wg_batch_bytes() { return (int)sizeof(WgBatch); }

// Grouped weight gradients (gemm8p_group_kernel).  Host-side checks: K a positive multiple of 64,
// M and N multiples of 8 (MN-major operand extents), 16-B aligned operands.
int dtc_wgrad_group(const WgBatch* in, hipStream_t st) {
  DTC_HOST_CHECK(in && in->n >= 1 && in->n <= WG_MAX && in->K >= 64 && in->K % 64 == 0);
  WgBatch b = *in;
  int t = 0;
  for (int i = 0; i < b.n; ++i) {
    WgEntry& w = b.e[i];
    DTC_HOST_CHECK(w.A && w.B && w.C && w.M >= 8 && w.N >= 8 && w.M % 8 == 0 && w.N % 8 == 0);
    DTC_HOST_CHECK(((unsigned long)w.A % 16) == 0 && ((unsigned long)w.B % 16) == 0 && ((unsigned long)w.C % 16) == 0);
    w.tile0 = t;
    t += ((w.M + BIG - 1) / BIG) * ((w.N + BIG - 1) / BIG);
    // tile order.  M-tiles fastest: the blocks an XCD runs together share one N-panel of X and each
    // streams its own dY panel, so a problem's dY is read once per N-tile -- for the lm_head (dY 824 MB,
    // 3 N-tiles) 3 times from HBM.  N-tiles fastest co-schedules an M-block's N-tiles on one XCD, so the
    // larger operand dY is read once and the smaller X panels are the re-read ones: used when M >= 2N
    // (the lm_head: -60 us/step, profiles/r5_wg_nfast_ab.log; also qkv / fc1: a further -15 us,
    // r5_wg_nfast2_ab.log).  DTC_WG_NFAST=0 keeps M-fastest everywhere.
    static const bool nfast_on = [] { const char* v = getenv("DTC_WG_NFAST"); return !v || atoi(v) != 0; }();
    w.nfast = nfast_on && w.M >= 2 * w.N;
  }
  b.ntiles = t;
  // tail split: the last (t mod CUs) tiles as K-pieces when every one of them belongs to a problem without
  // bias column sums, K divides into 64-multiples, and the caller gave a slab big enough
  int tail = 0, split = 0;
  const int cus = cu_count();
  if (in->tail_slab && in->tail_split > 0 && cus > 0 && t > cus) {
    tail = t % cus;
    split = in->tail_split > 1 ? in->tail_split : std::max(2, std::min(4, tail > 0 ? cus / tail : 0));
    bool ok = tail > 0 && b.K % (64 * split) == 0 && (long)tail * split <= 2L * cus &&
              (long)tail * split * BIG * BIG <= in->tail_cap;
    for (int i = 0; ok && i < b.n; ++i) {
      const WgEntry& w = b.e[i];
      const int end = w.tile0 + ((w.M + BIG - 1) / BIG) * ((w.N + BIG - 1) / BIG);
      if (end > t - tail && w.cs) ok = false;
    }
    if (!ok) tail = split = 0;
  }
  b.tail_tiles = tail;
  b.tail_split = split > 1 ? split : 1;
  if (!tail) b.tail_slab = nullptr;
  hipLaunchKernelGGL(gemm8p_group_kernel, dim3(t - tail + tail * b.tail_split), dim3(NT2), 0, st, b);
  DTC_CHECK_LAUNCH();
  if (tail) {
    hipLaunchKernelGGL(wg_tail_reduce, dim3(tail * 8), dim3(WGT_THREADS), 0, st, b);
    DTC_CHECK_LAUNCH();
  }
  return 0;
}

// gemm8r plan mask (DTC_GEMM8R at load time); returns the previous value (tests / A/B)
int dtc_gemm_set_r8(int mask) {
  const int old = g_r8_mask;
  g_r8_mask = mask;
  return old;
}

int dtc_gemm_set_r8_ilv(int on) {
  const int old = g_r8_ilv;
  g_r8_ilv = on;
  return old;
}

int dtc_gemm(const GemmArgs* a, hipStream_t st) {
  if (a->K % 32 != 0) return 1001;               // K must be a multiple of 32 (BK = 64, or 32)
  if (a->lda % 8 || a->ldb % 8 || a->ldc % 4) return 1002;  // 16-B row alignment
  if (a->M <= 0 || a->N <= 0) return 0;
  const int epi = a->epi;
  const bool f32 = a->c_f32 != 0;
  if (a->layout <= 1 && !a->colsum && a->alpha == 1.f && a->beta == 0.f &&
      !n8_cb(a->layout, a->M, a->N, a->K, epi)) {
    const R8Plan pl = r8_plan(a->layout, a->M, a->N, a->K, epi, f32);
    if (pl.cb2 && a->layout == 0) {
      if (epi == EPI_STORE) return f32 ? launch_r8<EPI_STORE, true>(*a, pl, st) : launch_r8<EPI_STORE, false>(*a, pl, st);
      if (epi == EPI_GELU) return launch_r8<EPI_GELU, false>(*a, pl, st);
      if (epi == EPI_DGELU) return launch_r8<EPI_DGELU, false>(*a, pl, st);
    } else if (pl.cb2 && !f32) {  // NN (W MN-major): the fc2 dgrad + dGELU, bf16 dgrads
      if (epi == EPI_DGELU) return launch_r8<EPI_DGELU, false, false>(*a, pl, st);
      if (epi == EPI_STORE) return launch_r8<EPI_STORE, false, false>(*a, pl, st);
    }
  }
  if (a->layout <= 1 && !a->colsum && a->alpha == 1.f && a->beta == 0.f) {
    const int cb = n8_cb(a->layout, a->M, a->N, a->K, epi);
    if (cb) {
      const int r = launch_n8_any(*a, cb, st);
      if (r >= 0) return r;
    }
  }
  if (a->layout <= 2 && !(a->layout == 2 && (a->bias || big_split(2, a->M, a->N, a->K)))) {
    const WPlan w = dmaw_plan(a->layout, a->M, a->N, a->K, epi, f32, a->colsum != nullptr);
    if (w.cfg != W_NONE) {
      if (a->layout == 0) {
        if (epi == EPI_STORE) return f32 ? launch_wcfg<true, true, EPI_STORE, true>(*a, w, st)
                                         : launch_wcfg<true, true, EPI_STORE, false>(*a, w, st);
        if (epi == EPI_GELU && !f32) return launch_wcfg<true, true, EPI_GELU, false>(*a, w, st);
        if (epi == EPI_RESID && f32) return launch_wcfg<true, true, EPI_RESID, true>(*a, w, st);
      } else if (a->layout == 1) {
        if (epi == EPI_DGELU && !f32) return launch_wcfg<true, false, EPI_DGELU, false>(*a, w, st);
        if (epi == EPI_STORE) return f32 ? launch_wcfg<true, false, EPI_STORE, true>(*a, w, st)
                                         : launch_wcfg<true, false, EPI_STORE, false>(*a, w, st);
      } else if (epi == EPI_STORE && f32) {
        return launch_wcfg<false, false, EPI_STORE, true>(*a, w, st);
      }
    }
  }
  if (a->layout == 0) {
    Plan p = make_plan(a->M, a->N, a->K, 0);
    const int bs0 = big_split(0, a->M, a->N, a->K);
    if (bs0 > 1 && epi == EPI_STORE && f32) return launch_big<true, true, EPI_STORE, true>(*a, bs0, st);
    if (bs0 == 1) {
      if (epi == EPI_LMHEAD) return launch_big<true, true, EPI_LMHEAD, false>(*a, 1, st);
      if (epi == EPI_GELU) return launch_big<true, true, EPI_GELU, false>(*a, 1, st);
      if (epi == EPI_DGELU && !f32) return launch_big<true, true, EPI_DGELU, false>(*a, 1, st);
      if (epi == EPI_RESID) return launch_big<true, true, EPI_RESID, true>(*a, 1, st);
      if (epi == EPI_STORE)
        return f32 ? launch_big<true, true, EPI_STORE, true>(*a, 1, st) : launch_big<true, true, EPI_STORE, false>(*a, 1, st);
      return 1003;
    }
    if (epi == EPI_LMHEAD) {
      if (p.bk != 64) return 1008;
      p.bm = p.bn = 128;
      return launch_t<128, 128, true, true, EPI_LMHEAD, false>(*a, p, st); }
    if (epi == EPI_GELU) return launch_sz<true, true, EPI_GELU, false>(*a, p, st);
    if (epi == EPI_DGELU && !f32) return launch_sz<true, true, EPI_DGELU, false>(*a, p, st);  // NT dgrad (W^T)
    if (epi == EPI_RESID) return launch_sz<true, true, EPI_RESID, true>(*a, p, st);
    if (epi == EPI_STORE) return f32 ? launch_sz<true, true, EPI_STORE, true>(*a, p, st)
                                     : launch_sz<true, true, EPI_STORE, false>(*a, p, st);
    return 1003;
  }
  if (a->layout == 1) {
    if (a->N % 8) return 1004;
    {
      const int bs = big_split(1, a->M, a->N, a->K);
      if (bs > 1 && epi == EPI_STORE && f32) return launch_big<true, false, EPI_STORE, true>(*a, bs, st);
      if (bs == 1 && a->K < 16384) {
        if (epi == EPI_DGELU) return launch_big<true, false, EPI_DGELU, false>(*a, 1, st);
        if (epi == EPI_STORE)
          return f32 ? launch_big<true, false, EPI_STORE, true>(*a, 1, st) : launch_big<true, false, EPI_STORE, false>(*a, 1, st);
      }
    }
    Plan p = make_plan(a->M, a->N, a->K, (epi == EPI_STORE && f32) ? 2 : 0);
    if (p.split > 1 && a->ws_bytes < (long)p.split * a->M * a->N * 4) return 1005;
    if (epi == EPI_DGELU) return launch_sz<true, false, EPI_DGELU, false>(*a, p, st);
    if (epi == EPI_STORE) return f32 ? launch_sz<true, false, EPI_STORE, true>(*a, p, st)
                                     : launch_sz<true, false, EPI_STORE, false>(*a, p, st);
    return 1003;
  }
  if (a->layout == 2) {
    if (a->M % 8 || a->N % 8) return 1004;
    if (epi != EPI_STORE || !f32 || a->bias) return 1003;
    if (a->colsum && !dtc_gemm_wgrad_fuses_colsum(a->M, a->N, a->K)) return 1009;
    if (const int bs = big_split(2, a->M, a->N, a->K)) return launch_big<false, false, EPI_STORE, true>(*a, bs, st);
    Plan p = make_plan(a->M, a->N, a->K, 1);
    if (p.split > 1 && a->ws_bytes < (long)p.split * a->M * a->N * 4) return 1005;
    return launch_sz<false, false, EPI_STORE, true>(*a, p, st);
  }
  return 1006;
}

}  // extern "C"
