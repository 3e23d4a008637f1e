// Exact-fp32 MFMA GEMM for gfx950 — the reference's own precision (dtype: fp32 parity mode).
//
// The reference computes every Dense in fp32 (flax Dense, model/MLP.py:13-20,
// model/CausalSelfAttention.py:18-20,46, model/GPTModel.py:72).  gfx950 has no reduced-precision
// (xf32/TF32) matrix path; it has an EXACT f32-input MFMA, v_mfma_f32_32x32x2_f32: one f32 per
// lane per operand, 16 f32 accumulators, 64 cycles per instruction and a 64-cycle dependent
// latency (cdna_hip_programming.md §3 "FP32-input MFMA"), i.e. 64 FLOP/clk/SIMD = ~157 TF/s dense
// for the chip, each product rounded once into a k-ordered fma chain (no wider internal sum).
//
//   C[m,n] = epi( sum_k A(m,k) * B(k,n) )      (same GemmArgs / layouts / epilogue ids as gemm.hip)
//   layout 0 (nt): A[m*lda+k], B[n*ldb+k]     forward    y  = x W^T        (W stored [out,in])
//   layout 1 (nn): A[m*lda+k], B[k*ldb+n]     dgrad      dX = dY W
//   layout 2 (tn): A[k*lda+m], B[k*ldb+n]     wgrad      dW = dY^T X
//
// Design (MI355X-first, not a bf16 kernel recompiled):
//  * At 1/16 of the bf16 MFMA rate the kernel is matrix-core bound with almost any staging, so the
//    structure optimises for MFMA issue: 256 threads = 2x2 waves, each wave TMxTN tiles of 32x32
//    (one independent accumulator chain per tile; a single 32x32x2 chain already issues back to
//    back because its dependent latency equals its issue interval), 2 blocks per CU.
//  * Both operands are staged into LDS in ONE image layout, [k][row] (row = m for A, n for B), so
//    every MFMA operand read is one ds_read_b32 of 32 consecutive floats per half-wave (the two
//    halves read k and k+1): conflict-free whatever the global layout.  K-contiguous operands are
//    transposed on the register -> LDS write (4 ds_write_b32; row pitch R+2 floats makes the 32
//    lanes of a half-wave hit 32 distinct banks), M/N-contiguous ones are written as float4.
//  * Register-staged, double-buffered LDS (the loads of k-tile t+1 are in flight under the MFMAs
//    of tile t, written after them, one barrier per 16-deep k-tile = 8 MFMA k-steps per barrier).
//  * Buffer-resource loads: rows past M/N read 0 by the hardware range check (ragged edges are
//    branch-free); a ragged last k-tile is zero-filled by a select (K % 4 == 0, host-checked).
//  * Accumulator layout (32x32 C/D map: col = lane&31, row = (r&3)+8(r>>2)+4(lane>>5)) puts n on the
//    lane: each store instruction writes two 128-B row segments; bias is one load per lane.
//  * Split-K (fp32 slabs + fixed-order reduce) for the long-K / small-MN shapes (weight gradients,
//    the lm_head dgrad over K = vocab).
//  * XCD-aware bijective block remap (common.h xcd_remap), M-tiles fastest.
#include "common.h"
#include <algorithm>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NTF = 256;  // threads per block
constexpr int BKF = 16;   // K granularity (every plan's k-tile is a multiple)

// k per LDS stage: the MFMAs between two barriers are (BK/2) * TM * TN per wave; 16 for the 128x128
// tile (32 MFMAs = 2048 cycles per barrier), 32 for the smaller tiles so they get as many
template <int TM, int TN>
constexpr int bk_of() { return TM * TN >= 4 ? 16 : 32; }

template <int R, bool KMAJ, int BK>
struct FTile {
  // LDS image [BK][LD] floats: element (k, r) at k*LD + r.  K-major tiles are written transposed,
  // 4 ds_write_b32 per float4: a half-wave covers 32/(BK/4) rows x BK/4 k-quads, bank
  // (4*kq*LD + j*LD + row) % 32, distinct over the 32 lanes when 4*LD = 32/(BK/4) (mod 32): LD = R+2
  // for BK 16, R+1 for BK 32.  M/N-major tiles are written as float4 (16-B aligned rows: R+4).
  static constexpr int LD = KMAJ ? (BK == 16 ? R + 2 : R + 1) : R + 4;
  static constexpr int ELEMS = BK * LD;
  static constexpr int CHUNKS = R * BK / 4;  // float4 chunks per tile
  static constexpr int PT = CHUNKS / NTF;
  static_assert(CHUNKS % NTF == 0, "tile too small for 256 threads");

  // rs: resource whose base is the operand's first row of this tile (KMAJ: row r0; else k-row k0)
  // k indices >= klim (the split's end, in the resource's k coordinates) read as 0: a K that is not
  // a multiple of BK (any K % 4 == 0 works) and split boundaries inside a k-tile
  __device__ __forceinline__ static void load(f32x4 (&reg)[PT], __amdgpu_buffer_rsrc_t rs, long ld, int kofs, int rofs,
                                              int klim, int tid) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int c = tid + i * NTF;
      long off;
      bool ok;
      if (KMAJ) {
        const int row = c / (BK / 4), kq = c % (BK / 4);
        off = ((long)row * ld + kofs + 4 * kq) * 4;
        ok = kofs + 4 * kq < klim;
      } else {
        const int krow = c / (R / 4), col = (c % (R / 4)) * 4;
        off = ((long)(kofs + krow) * ld + rofs + col) * 4;
        ok = kofs + krow < klim;
      }
      const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
      reg[i] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ static void store(const f32x4 (&reg)[PT], float* lds, int tid) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int c = tid + i * NTF;
      if (KMAJ) {
        const int row = c / (BK / 4), kq = c % (BK / 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) lds[(4 * kq + j) * LD + row] = reg[i][j];
      } else {
        const int krow = c / (R / 4), col = (c % (R / 4)) * 4;
        *(f32x4*)(lds + krow * LD + col) = reg[i];
      }
    }
  }
};

struct GemmF {
  const float* A; long lda; long a_elems;
  const float* B; long ldb; long b_elems;
  int M, N, K;
  int tiles_m, tiles_n, split, kps;
  float* slab;  // split > 1: fp32 slabs [split][M][N]
  // epilogue
  float* C; long ldc;
  const float* bias;
  const float* aux; long ldaux;
  float* aux_out;
  float alpha, beta;
  const int* labels; int vocab_start, n_valid;
  float* part; float* label_out;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_from(const float* base, long elems_left) {
  long bytes = elems_left * 4;
  if (bytes > 0x7fffffffL) bytes = 0x7fffffffL;
  if (bytes < 0) bytes = 0;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

// Exact (libm-quality) exp for the fp32 parity path's softmax statistics.
__device__ __forceinline__ float exp_f32(float x) { return expf(x); }

template <int TM, int TN, bool AK, bool BKM, int EPI>
__global__ void __launch_bounds__(NTF, 2) gemm_f32_kernel(GemmF g) {
  constexpr int BM = 64 * TM, BN = 64 * TN, BK = bk_of<TM, TN>();
  using TA = FTile<BM, AK, BK>;
  using TB = FTile<BN, BKM, BK>;
  constexpr int BUF = TA::ELEMS + TB::ELEMS;
  __shared__ __attribute__((aligned(16))) float smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntiles = g.tiles_m * g.tiles_n;
  const int lid = xcd_remap(blockIdx.x, ntiles * g.split);
  const int tile = lid % ntiles, z = lid / ntiles;
  const int tm_idx = tile % g.tiles_m, tn_idx = tile / g.tiles_m;  // M-tiles fastest: blocks of one
  const int m0 = tm_idx * BM, n0 = tn_idx * BN;                    // XCD share the B (weight) panel
  const int kbeg = z * g.kps;
  const int klen = min(g.kps, g.K - kbeg);
  const int nk = (klen + BK - 1) / BK;  // a ragged last k-tile is zero-filled by the loads

  // resources: K-major operands start at the tile's first row, M/N-major at the split's first k-row
  const long a_base = AK ? (long)m0 * g.lda : (long)kbeg * g.lda;
  const long b_base = BKM ? (long)n0 * g.ldb : (long)kbeg * g.ldb;
  const __amdgpu_buffer_rsrc_t rsA = rsrc_from(g.A + a_base, g.a_elems - a_base);
  const __amdgpu_buffer_rsrc_t rsB = rsrc_from(g.B + b_base, g.b_elems - b_base);
  // k offset inside the resource: K-major -> kbeg + t*BK (column), M/N-major -> t*BK (row)
  auto kofs = [&](int t) { return t * BK; };
  const int ak0 = AK ? kbeg : 0, bk0 = BKM ? kbeg : 0;
  const int alim = ak0 + klen, blim = bk0 + klen;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  f32x4 ra[TA::PT], rb[TB::PT];
  if (nk > 0) {
    TA::load(ra, rsA, g.lda, ak0 + kofs(0), m0, alim, tid);
    TB::load(rb, rsB, g.ldb, bk0 + kofs(0), n0, blim, tid);
    TA::store(ra, smem, tid);
    TB::store(rb, smem + TA::ELEMS, tid);
  }
  __syncthreads();
  const int half = lane >> 5, l32 = lane & 31;
  for (int t = 0; t < nk; ++t) {
    const float* sA = smem + (t & 1) * BUF;
    const float* sB = sA + TA::ELEMS;
    const bool more = t + 1 < nk;
    if (more) {
      TA::load(ra, rsA, g.lda, ak0 + kofs(t + 1), m0, alim, tid);
      TB::load(rb, rsB, g.ldb, bk0 + kofs(t + 1), n0, blim, tid);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int k = 2 * kk + half;
      float fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = sA[k * TA::LD + wm * 32 * TM + i * 32 + l32];
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = sB[k * TB::LD + wn * 32 * TN + j * 32 + l32];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      float* nA = smem + ((t + 1) & 1) * BUF;
      TA::store(ra, nA, tid);
      TB::store(rb, nA + TA::ELEMS, tid);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  const int mw = m0 + wm * 32 * TM, nw = n0 + wn * 32 * TN;
  if (g.split > 1) {  // raw partial sums -> slab z (splitk_reduce_f32 applies beta and the sum order)
    float* sl = g.slab + (long)z * g.M * g.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = nw + j * 32 + l32;
        if (n >= g.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
          if (m < g.M) sl[(long)m * g.N + n] = acc[i][j][r];
        }
      }
    return;
  }
  if (EPI == EPI_LMHEAD) {
    // logits = acc + bias (pad columns -inf), stored if C; per (row, wave column slice) partial
    // (max, sum exp) -> part[p][m] with p = tn_idx*2 + wn; the label's logit -> label_out[m]
    const int p = tn_idx * 2 + wn;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float lg[TN][16];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = nw + j * 32 + l32;
        const float b = (n < g.N && g.bias) ? g.bias[n] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float o = acc[i][j][r] + b;
          if (n >= g.n_valid) o = -INFINITY;
          lg[j][r] = o;
          const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
          if (m < g.M && n < g.N) {
            if (g.C) g.C[(long)m * g.ldc + n] = o;
            if (g.labels[m] - g.vocab_start == n) g.label_out[m] = o;
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float mx = lg[0][r];
#pragma unroll
        for (int j = 1; j < TN; ++j) mx = fmaxf(mx, lg[j][r]);
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        float s = 0.f;
        if (mx > -INFINITY) {
#pragma unroll
          for (int j = 0; j < TN; ++j) s += exp_f32(lg[j][r] - mx);
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (l32 == 0 && m < g.M) *(f32x2*)(g.part + ((long)p * g.M + m) * 2) = f32x2{mx, s};
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = nw + j * 32 + l32;
      if (n >= g.N) continue;
      const float b = g.bias ? g.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mw + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (m >= g.M) continue;
        DTC_ASSERT(m < g.M && n < g.N);
        float o = g.alpha * acc[i][j][r] + b;
        float* c = g.C + (long)m * g.ldc + n;
        if (EPI == EPI_RESID) o += g.aux[(long)m * g.ldaux + n];
        if (EPI == EPI_DGELU) o *= g.aux[(long)m * g.ldaux + n];
        if (EPI == EPI_STORE && g.beta != 0.f) o += g.beta * *c;
        if (EPI == EPI_GELU) {  // C = gelu'(u) (the backward's dGELU factor), aux_out = gelu(u)
          // precise tanh (this is the parity path; the bf16 kernels use the exp2/rcp form)
          constexpr float k0 = 0.7978845608028654f, k1 = 0.044715f;
          const float u2 = o * o, th = tanhf(k0 * (o + k1 * o * u2));
          g.aux_out[(long)m * g.ldc + n] = 0.5f * o * (1.f + th);
          o = 0.5f * (1.f + th) + 0.5f * o * (1.f - th * th) * k0 * (1.f + 3.f * k1 * u2);
        }
        *c = o;
      }
    }
}

// C = beta*C + sum_z slab[z]   (fixed z order: deterministic)
__global__ void splitk_reduce_f32(const float* __restrict__ slab, int split, int M, int N, float* __restrict__ C,
                                  long ldc, float beta) {
  const long MN = (long)M * N;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= MN) return;
  DTC_ASSERT(split >= 1 && ldc >= N);
  float s = slab[i];
  for (int z = 1; z < split; ++z) s += slab[z * MN + i];
  const long m = i / N, n = i % N;
  float* c = C + m * ldc + n;
  if (beta != 0.f) s += beta * *c;
  *c = s;
}

struct PlanF {
  int tm, tn, split, kps, tiles_m, tiles_n;
};

// Tile / split-K choice: the biggest tile that still gives >= 2 blocks per CU (512), then smaller
// tiles, then split-K over the largest tile for long-K problems that cannot fill the chip.  Every
// split's k range is a multiple of the variant's BK (a K that is not falls back to the BK-16 tile).
PlanF plan_f32(int M, int N, int K) {
  static const int cands[3][2] = {{2, 2}, {2, 1}, {1, 1}};
  const int target = 512;
  for (auto& c : cands) {
    const int tm = (M + 64 * c[0] - 1) / (64 * c[0]), tn = (N + 64 * c[1] - 1) / (64 * c[1]);
    if ((long)tm * tn >= target) return PlanF{c[0], c[1], 1, K, tm, tn};
  }
  // split-K: 128x128 if K is long, else 64x64; slices of >= 256 k
  const int ct = K >= 4096 ? 2 : 1;
  const int bk = ct == 2 ? 16 : 32;
  const int tm = (M + 64 * ct - 1) / (64 * ct), tn = (N + 64 * ct - 1) / (64 * ct);
  const long tiles = (long)tm * tn;
  int split = (int)std::max<long>(1, (target + tiles - 1) / tiles);
  split = std::min(split, std::max(1, K / 256));
  int kps = (K + split - 1) / split;
  kps = (kps + bk - 1) / bk * bk;
  split = (K + kps - 1) / kps;
  return PlanF{ct, ct, split, kps, tm, tn};
}

template <int TM, int TN, bool AK, bool BKM, int EPI>
int launch_f32(const GemmF& g, hipStream_t st) {
  const int blocks = g.tiles_m * g.tiles_n * g.split;
  hipLaunchKernelGGL((gemm_f32_kernel<TM, TN, AK, BKM, EPI>), dim3(blocks), dim3(NTF), 0, st, g);
  DTC_CHECK_LAUNCH();
  return 0;
}

template <bool AK, bool BKM, int EPI>
int launch_tiles(const GemmF& g, const PlanF& p, hipStream_t st) {
  if (p.tm == 2 && p.tn == 2) return launch_f32<2, 2, AK, BKM, EPI>(g, st);
  if (p.tm == 2 && p.tn == 1) return launch_f32<2, 1, AK, BKM, EPI>(g, st);
  return launch_f32<1, 1, AK, BKM, EPI>(g, st);
}

template <bool AK, bool BKM>
int launch_epi(const GemmF& g, const PlanF& p, int epi, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return launch_tiles<AK, BKM, EPI_STORE>(g, p, st);
    case EPI_RESID: return launch_tiles<AK, BKM, EPI_RESID>(g, p, st);
    case EPI_GELU: return launch_tiles<AK, BKM, EPI_GELU>(g, p, st);
    case EPI_DGELU: return launch_tiles<AK, BKM, EPI_DGELU>(g, p, st);
    case EPI_LMHEAD: return launch_tiles<AK, BKM, EPI_LMHEAD>(g, p, st);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

extern "C" {

long dtc_gemm_f32_workspace_bytes(int layout, int M, int N, int K) {
  (void)layout;
  const PlanF p = plan_f32(M, N, K);
  return p.split > 1 ? (long)p.split * M * N * 4 : 0;
}

// LM-head partial count of the fp32 kernel: one (max, sumexp) pair per row per 64-wide... per wave
// column slice (2 per 128-column N-tile, or per 64-column tile when the plan picks TN = 1).
int dtc_lmhead_nparts_f32(int M, int N, int K) {
  const PlanF p = plan_f32(M, N, K);
  return p.tiles_n * 2;
}

int dtc_gemm_f32(const GemmArgs* a, hipStream_t st) {
  DTC_HOST_CHECK(a->layout >= 0 && a->layout <= 2);
  DTC_HOST_CHECK(a->c_f32 == 1);
  DTC_HOST_CHECK(a->K > 0 && a->M > 0 && a->N > 0);
  DTC_HOST_CHECK(a->layout == 2 || a->K % 4 == 0);  // float4 loads along k of a K-major operand
  DTC_HOST_CHECK(a->lda % 4 == 0 && a->ldb % 4 == 0);
  DTC_HOST_CHECK(((uintptr_t)a->A & 15) == 0 && ((uintptr_t)a->B & 15) == 0);
  const bool AK = a->layout != 2, BKM = a->layout == 0;
  PlanF p = plan_f32(a->M, a->N, a->K);
  GemmF g{};
  g.A = (const float*)a->A; g.lda = a->lda;
  g.a_elems = AK ? (long)a->M * a->lda : (long)a->K * a->lda;
  g.B = (const float*)a->B; g.ldb = a->ldb;
  g.b_elems = BKM ? (long)a->N * a->ldb : (long)a->K * a->ldb;
  g.M = a->M; g.N = a->N; g.K = a->K;
  g.C = (float*)a->C; g.ldc = a->ldc;
  g.bias = a->bias; g.aux = (const float*)a->aux; g.ldaux = a->ldaux; g.aux_out = (float*)a->aux_out;
  g.alpha = a->alpha; g.beta = a->beta;
  g.labels = a->labels; g.vocab_start = a->vocab_start; g.n_valid = a->n_valid;
  g.part = a->part; g.label_out = a->label_out;
  // buffer offsets are 32-bit: the K-major operand spans BM rows per block, the M/N-major one the
  // split's k range
  auto fits = [](long elems) { return elems * 4 < 0x7fffffffL; };
  const bool splittable = a->epi == EPI_STORE && a->bias == nullptr && a->alpha == 1.f;
  if (p.split > 1 && !splittable) {  // epilogues that need the full sum in registers: no split-K
    p.split = 1;
    p.kps = a->K;
  }
  if (p.split > 1 && (long)p.split * a->M * a->N * 4 > a->ws_bytes) return 1101;  // workspace too small
  g.tiles_m = p.tiles_m; g.tiles_n = p.tiles_n; g.split = p.split; g.kps = p.kps;
  DTC_HOST_CHECK(AK ? fits(128L * a->lda) : fits((long)(p.kps + 32) * a->lda));
  DTC_HOST_CHECK(BKM ? fits(128L * a->ldb) : fits((long)(p.kps + 32) * a->ldb));
  g.slab = (float*)a->workspace;
  if (a->epi == EPI_LMHEAD && a->layout != 0) return (int)hipErrorInvalidValue;
  int rc;
  if (a->layout == 0) rc = launch_epi<true, true>(g, p, a->epi, st);
  else if (a->layout == 1) rc = launch_epi<true, false>(g, p, a->epi, st);
  else rc = launch_epi<false, false>(g, p, a->epi, st);
  if (rc) return rc;
  if (p.split > 1) {
    const long MN = (long)a->M * a->N;
    hipLaunchKernelGGL(splitk_reduce_f32, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, st, g.slab, p.split, a->M,
                       a->N, g.C, a->ldc, a->beta);
    DTC_CHECK_LAUNCH();
  }
  return 0;
}

}  // extern "C"
