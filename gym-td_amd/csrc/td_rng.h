// td_rng.h -- the two MT19937 streams gym-TD draws from, usable on host and device.
//
//  * CPython ``random`` (built-in opponents, TDGymBasic.py:84-86,98-100,113-117,
//    137-191): init_by_array seeding of ``random.seed(int)``, getrandbits(k<=32) =
//    genrand >> (32-k), randbelow by rejection on getrandbits(bit_length(n)),
//    random() = 53-bit (a>>5, b>>6) double, shuffle = Fisher-Yates over randbelow.
//  * numpy legacy ``RandomState`` (road generation, TDRoadGen.py:10-181, and
//    ``num_roads`` TDGymBasic.py:42): init_genrand seeding, randint(lo, hi) =
//    masked rejection on 32-bit outputs (no draw when hi-lo == 1).
//
// Both use the same MT19937 core; state = 624 words + position.
#pragma once
#include <stdint.h>

#ifndef TD_HD
#if defined(__HIPCC__)
#define TD_HD __host__ __device__
#else
#define TD_HD
#endif
#endif

namespace td {

constexpr int MT_N = 624;
constexpr int MT_M = 397;

TD_HD inline void mt_init_genrand(uint32_t* mt, uint32_t s) {
  mt[0] = s;
  for (int i = 1; i < MT_N; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
}

// CPython random.seed(int) with 0 <= seed < 2**32: key = [seed] (init_by_array, len 1).
TD_HD inline void mt_init_by_array(uint32_t* mt, const uint32_t* key, int klen) {
  mt_init_genrand(mt, 19650218u);
  int i = 1, j = 0;
  for (int k = (MT_N > klen ? MT_N : klen); k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    ++i; ++j;
    if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
    if (j >= klen) j = 0;
  }
  for (int k = MT_N - 1; k; --k) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= MT_N) { mt[0] = mt[MT_N - 1]; i = 1; }
  }
  mt[0] = 0x80000000u;
}

TD_HD inline void mt_twist(uint32_t* mt) {
  for (int i = 0; i < MT_N; ++i) {
    uint32_t y = (mt[i] & 0x80000000u) | (mt[(i + 1) % MT_N] & 0x7fffffffu);
    mt[i] = mt[(i + MT_M) % MT_N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
}

TD_HD inline uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// A stream over caller-owned storage: words[0..623] state, words[624] position.
struct MtRef {
  uint32_t* w;
  TD_HD uint32_t next() {
    uint32_t p = w[MT_N];
    if (p >= (uint32_t)MT_N) { mt_twist(w); p = 0; }
    uint32_t y = w[p];
    w[MT_N] = p + 1;
    return mt_temper(y);
  }
  // ---- CPython random ----
  TD_HD uint32_t getrandbits(int k) { return next() >> (32 - k); }
  TD_HD int64_t randbelow(int64_t n) {  // n >= 1, n < 2**32
    if (n <= 0) return 0;
    int k = 0;
    for (uint64_t v = (uint64_t)n; v; v >>= 1) ++k;
    uint32_t r = getrandbits(k);
    while ((int64_t)r >= n) r = getrandbits(k);
    return r;
  }
  TD_HD int64_t py_randint(int64_t a, int64_t b) { return a + randbelow(b - a + 1); }
  TD_HD double py_random() {
    uint32_t a = next() >> 5, b = next() >> 6;
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
  }
  // ---- numpy legacy RandomState ----
  TD_HD int64_t np_randint(int64_t lo, int64_t hi) {  // requires hi > lo
    if (hi <= lo) return lo;  // numpy raises here; callers check first
    uint64_t rng = (uint64_t)(hi - lo - 1);
    if (rng == 0) return lo;
    uint64_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (next() & (uint32_t)mask)) > rng) {}
    return lo + (int64_t)v;
  }
};

// Lazy-twist form used on the device (td_step.hip WaveMt): w[625] = tw, words
// [tw, 624) of the current block are not yet twisted.  Complete them in place,
// giving CPython's ``getstate()`` form (624 words + position).
TD_HD inline void mt_finish_lazy(uint32_t* w) {
  for (uint32_t p = w[625]; p < (uint32_t)MT_N; ++p) {
    uint32_t y = (w[p] & 0x80000000u) | (w[(p + 1) % MT_N] & 0x7fffffffu);
    w[p] = w[(p + MT_M) % MT_N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
  }
  w[625] = MT_N;
}

// MT19937 over 626 words with a lazy twist (see mt_finish_lazy): the next block's
// word p is computed when drawn.  Draws are bit-identical to MtRef; the 624-word
// twist loop never runs on the critical path.  pos / tw live in registers while
// drawing; load() / store() move them from / to w[624], w[625].
struct LazyMt {
  uint32_t* w;
  uint32_t pos, tw;
  TD_HD void load() { pos = w[MT_N]; tw = w[MT_N + 1]; }
  TD_HD void store() { w[MT_N] = pos; w[MT_N + 1] = tw; }
  TD_HD uint32_t next() {
    if (pos >= (uint32_t)MT_N) { pos = 0; tw = 0; }
    uint32_t y;
    if (pos >= tw) {
      const uint32_t a = w[pos];
      const uint32_t nb = w[pos == MT_N - 1 ? 0u : pos + 1u];
      const uint32_t far = w[pos < (uint32_t)(MT_N - MT_M) ? pos + MT_M : pos - (MT_N - MT_M)];
      const uint32_t yy = (a & 0x80000000u) | (nb & 0x7fffffffu);
      y = far ^ (yy >> 1) ^ ((yy & 1u) ? 0x9908b0dfu : 0u);
      w[pos] = y;
      tw = pos + 1;
    } else {
      y = w[pos];
    }
    ++pos;
    return mt_temper(y);
  }
  TD_HD int64_t np_randint(int64_t lo, int64_t hi) {  // numpy legacy masked rejection
    if (hi <= lo) return lo;
    uint64_t rng = (uint64_t)(hi - lo - 1);
    if (rng == 0) return lo;
    uint64_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (next() & (uint32_t)mask)) > rng) {}
    return lo + (int64_t)v;
  }
};

TD_HD inline void py_seed(uint32_t* w, uint32_t seed) {
  uint32_t key[1] = {seed};
  mt_init_by_array(w, key, 1);
  w[MT_N] = MT_N;
}

TD_HD inline void np_seed(uint32_t* w, uint32_t seed) {
  mt_init_genrand(w, seed);
  w[MT_N] = MT_N;
}

}  // namespace td
