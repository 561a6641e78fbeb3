// CPU check of kcount.h (the Kendall engine's per-window pair counting and cross-range
// fix-up) against brute force. Built and run by tests/test_kcount.py.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <algorithm>
#include <vector>

#include "kcount.h"

using namespace vr;

static uint64_t brute_pairs(uint64_t o, uint64_t z) {
  uint64_t r = 0;
  for (int i = 0; i < 64; ++i)
    for (int j = i + 1; j < 64; ++j) r += ((o >> i) & 1) && ((z >> j) & 1);
  return r;
}

// stream of L positions: kind[p] in {0: excluded, 1: one, 2: zero}, start[p]
template <bool TIE>
static int check_stream(std::mt19937_64& g, int nwin, double pstart, int nranges) {
  const int L = nwin * 64;
  std::vector<int> kind(L);
  std::vector<int> st(L);
  for (int p = 0; p < L; ++p) {
    const int u = (int)(g() % 8);
    kind[p] = u < 2 ? 0 : (TIE ? 1 : (u < 5 ? 1 : 2));
    st[p] = (p == 0) || (std::uniform_real_distribution<double>(0, 1)(g) < pstart);
  }
  // brute force: sum over zeros j of ones i < j in the same segment (TIE: members both)
  uint64_t want = 0;
  int seg0 = 0;
  for (int j = 0; j < L; ++j) {
    if (st[j]) seg0 = j;
    const bool zj = TIE ? kind[j] == 1 : kind[j] == 2;
    if (!zj) continue;
    for (int i = seg0; i < j; ++i) want += kind[i] == 1;
  }
  // ranges of windows, each from a zero state, then fix-up in order
  std::vector<int> cuts{0, nwin};
  for (int r = 1; r < nranges; ++r) cuts.push_back((int)(g() % (nwin + 1)));
  std::sort(cuts.begin(), cuts.end());
  uint64_t got = 0;
  KFix F = kfix_identity();
  for (size_t r = 0; r + 1 < cuts.size(); ++r) {
    KSeg a{0, 0, 0};
    bool seen = false;
    for (int w = cuts[r]; w < cuts[r + 1]; ++w) {
      uint64_t o = 0, z = 0, S = 0;
      for (int b = 0; b < 64; ++b) {
        const int p = w * 64 + b;
        if (kind[p] == 1) o |= 1ull << b;
        if (kind[p] == 2) z |= 1ull << b;
        if (st[p]) S |= 1ull << b;
      }
      if (TIE) z = o;
      if (!TIE && kc_pairs64(o, z) != brute_pairs(o, z)) {
        printf("pairs64 mismatch\n");
        return 1;
      }
      kseg_window<TIE>(o, z, S, a, seen);
    }
    got += a.acc;
    kfix_push(F, a.zlead, a.c, seen);
  }
  got += F.f0;  // carry into the stream start is 0
  if (got != want) {
    printf("%s mismatch: got %llu want %llu (nwin %d pstart %g ranges %d)\n", TIE ? "tie" : "inv",
           (unsigned long long)got, (unsigned long long)want, nwin, pstart, nranges);
    return 1;
  }
  return 0;
}

int main() {
  std::mt19937_64 g(12345);
  // pairs32 exhaustive-ish on structured words
  for (int t = 0; t < 200000; ++t) {
    uint64_t o = g(), z = g() & ~o;
    if (t % 3 == 0) o &= g();
    if (kc_pairs64(o, z) != brute_pairs(o, z)) {
      printf("pairs64 mismatch %llx %llx\n", (unsigned long long)o, (unsigned long long)z);
      return 1;
    }
  }
  int bad = 0;
  const double ps[] = {0.0, 0.002, 0.02, 0.2, 0.6, 1.0};
  for (int rep = 0; rep < 40; ++rep)
    for (double p : ps) {
      const int nwin = 1 + (int)(g() % 12);
      const int nr = 1 + (int)(g() % 6);
      bad |= check_stream<false>(g, nwin, p, nr);
      bad |= check_stream<true>(g, nwin, p, nr);
    }
  if (!bad) printf("kcount ok\n");
  return bad;
}
