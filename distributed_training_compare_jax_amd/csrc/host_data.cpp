// Host-side data pipeline (native): the synthetic FineWeb-shaped token stream of data/synthetic.py,
// bit-identical to its numpy path (tests/test_aux_cpu.py checks equality).
//
// Why native: under the DP embedding gather every rank materialises the WHOLE global batch each
// step (the token ids rebuild the embedding-table gradient), so at dp8 the host produces
// 64 x 513 tokens per step; the vectorised numpy path costs ~160 ns/token there (5.3 ms, as long
// as the GPU step itself), this loop ~10-20 ns/token.  The reference's loader is a host Python
// generator (data/fineweb_edu.py:15-39); this is its runtime-side equivalent for synthetic data.
//
// Token at global position p (a pure function of (seed, p), so any rank can produce any rows):
//   z(p)   = rank_to_id[ searchsorted_right(cdf, U1(p)) ]              (Zipf-like unigram)
//   tok(p) = U2(p) < p_bigram ? succ[z(p-1)] : z(p)                     (learnable bigram)
// with U_k(p) = (splitmix64(uint64(p) ^ key_k) >> 11) * 2^-53.  The searchsorted is exact: a
// guide table over 2^gbits equal u-buckets bounds the binary search to one bucket's cdf range.
#include <algorithm>
#include <cstdint>

namespace {

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

inline double uniform(uint64_t key, int64_t pos) {
  const uint64_t h = splitmix64(static_cast<uint64_t>(pos) ^ key);
  return static_cast<double>(h >> 11) * (1.0 / 9007199254740992.0);
}

}  // namespace

extern "C" {

// guide[b] = searchsorted_right(cdf, b / 2^gbits) for b in [0, 2^gbits]; out: int32 [count]
int dtc_synth_tokens(uint64_t key1, uint64_t key2, const double* cdf, int vocab, const int32_t* guide, int gbits,
                     const int64_t* rank_to_id, const int64_t* succ, double p_bigram, int64_t start, int64_t count,
                     int32_t* out) {
  if (vocab <= 0 || gbits < 1 || gbits > 24 || count < 0) return 1;
  const double G = static_cast<double>(1 << gbits);
  auto z_at = [&](int64_t pos) -> int64_t {
    const double u = uniform(key1, pos);
    const int b = static_cast<int>(u * G);  // exact (power-of-two scale), b < 2^gbits since u < 1
    const double* lo = cdf + guide[b];
    const double* hi = cdf + guide[b + 1];
    int64_t idx = std::upper_bound(lo, hi, u) - cdf;
    if (idx > vocab - 1) idx = vocab - 1;
    return rank_to_id[idx];
  };
  int64_t prev = z_at(start - 1);
  for (int64_t i = 0; i < count; ++i) {
    const int64_t pos = start + i;
    const int64_t z = z_at(pos);
    out[i] = static_cast<int32_t>(uniform(key2, pos) < p_bigram ? succ[prev] : z);
    prev = z;
  }
  return 0;
}

int dtc_host_abi_version() { return 1; }

}  // extern "C"
