/*
 * ORACLE -- plain-C restatement of the reference's negative-sample index draws.
 * TEST INFRASTRUCTURE ONLY: loaded by tests/ (ctypes) as the checker for the HIP sampler kernels.
 *
 * The reference draws negatives with numpy's legacy global RandomState:
 *   - catalogue sampler  np.random.choice(nonitems, N)      datasets/dcuedataset.py:219
 *   - in-batch sampler   np.random.choice(indexes)          nn/dcue.py:703-707 (commented spec)
 *   - random_seed mode   np.random.seed(S) before each sample  datasets/dcuedataset.py:167-168
 * numpy (2.2, third-party, absent from /root/reference) implements these as:
 *   seed(int)  -> init_genrand(seed)                              (MT19937, Matsumoto & Nishimura)
 *   choice(a, size) -> randint(0, len(a), size) -> for 0 < rng=len-1 <= 0xFFFFFFFF:
 *       mask = smallest 2^k-1 >= rng; repeat v = genrand_int32() & mask until v <= rng
 *       (rng == 0 consumes no draw and returns 0).
 * Pinned against numpy itself and the golden vectors in tests/golden/{inbatch_draws,catalogue}.npz.
 */
#include <stdint.h>
#include <string.h>

#define MT_N 624
#define MT_M 397

typedef struct {
  uint32_t key[MT_N];
  int pos;
} mt_state;

void mt_seed(mt_state* s, uint32_t seed) {
  s->key[0] = seed;
  for (int i = 1; i < MT_N; ++i)
    s->key[i] = 1812433253u * (s->key[i - 1] ^ (s->key[i - 1] >> 30)) + (uint32_t)i;
  s->pos = MT_N;
}

static void mt_twist(mt_state* s) {
  for (int i = 0; i < MT_N; ++i) {
    uint32_t y = (s->key[i] & 0x80000000u) | (s->key[(i + 1) % MT_N] & 0x7fffffffu);
    s->key[i] = s->key[(i + MT_M) % MT_N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  s->pos = 0;
}

uint32_t mt_next(mt_state* s) {
  if (s->pos >= MT_N) mt_twist(s);
  uint32_t y = s->key[s->pos++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

static uint32_t mask_for(uint32_t rng) {
  uint32_t m = rng;
  m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
  return m;
}

/* one legacy bounded draw in [0, rng] */
uint32_t mt_bounded(mt_state* s, uint32_t rng) {
  if (rng == 0) return 0;
  uint32_t m = mask_for(rng), v;
  while ((v = (mt_next(s) & m)) > rng) {
  }
  return v;
}

/* raw tempered outputs (for checking the GPU twist/temper) */
void oracle_mt_stream(uint32_t seed, int n, uint32_t* out) {
  mt_state s;
  mt_seed(&s, seed);
  for (int i = 0; i < n; ++i) out[i] = mt_next(&s);
}

/* in-batch: r[i][j] = draw over B-1 others, mapped past i; global stream, row-major */
int oracle_inbatch(uint32_t seed, int B, int N, int64_t* out) {
  if (B < 2) return -1;
  mt_state s;
  mt_seed(&s, seed);
  for (int i = 0; i < B; ++i)
    for (int j = 0; j < N; ++j) {
      uint32_t r = mt_bounded(&s, (uint32_t)(B - 2));
      out[(int64_t)i * N + j] = (int64_t)(r < (uint32_t)i ? r : r + 1);
    }
  return 0;
}

/*
 * catalogue: for each sample b, nonitems = split_items \ user_items(user b) (sorted), N draws.
 * split_items sorted ascending; user items given as CSR (indptr over users, indices = item ids,
 * any order).  reseed != 0 -> fresh stream per sample from `seed` (random_seed mode), else one
 * stream for all samples.  Writes item ids.  Returns -2 if a user has no candidates.
 */
int oracle_catalogue(uint32_t seed, int reseed, const int64_t* split_items, int n_split,
                     const int64_t* indptr, const int64_t* indices, const int64_t* users,
                     int n_samples, int N, int64_t* out) {
  mt_state s;
  mt_seed(&s, seed);
  for (int b = 0; b < n_samples; ++b) {
    if (reseed) mt_seed(&s, seed);
    int64_t u = users[b];
    /* excluded[q] marks split_items[q] as one of the user's items */
    int excluded_count = 0;
    static unsigned char excl[1 << 20];
    if (n_split > (1 << 20)) return -3;
    memset(excl, 0, (size_t)n_split);
    for (int64_t e = indptr[u]; e < indptr[u + 1]; ++e) {
      int64_t item = indices[e];
      int lo = 0, hi = n_split;
      while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (split_items[mid] < item) lo = mid + 1; else hi = mid;
      }
      if (lo < n_split && split_items[lo] == item && !excl[lo]) {
        excl[lo] = 1;
        ++excluded_count;
      }
    }
    int n_cand = n_split - excluded_count;
    if (n_cand <= 0) return -2;
    for (int j = 0; j < N; ++j) {
      uint32_t r = mt_bounded(&s, (uint32_t)(n_cand - 1));
      int seen = -1, q = 0;
      for (q = 0; q < n_split; ++q)
        if (!excl[q] && ++seen == (int)r) break;
      out[(int64_t)b * N + j] = split_items[q];
    }
  }
  return 0;
}
