// Bit-parallel pair counting for the Kendall engine (kendall.hip), host- and
// device-compilable so tests/test_kcount.py can check it against brute force on the CPU.
//
// A window is 64 consecutive positions of a sorted stream; for one subset (one lane) the
// included positions are split into "ones" o and "zeros" z (disjoint 64-bit sets), and
// uniform segment starts S cut the stream into segments (tie groups / radix buckets).
// The engine needs, per segment, the number of (one, zero) pairs with the one first:
//   sum over zeros j of #{ones i < j in the same segment}.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define VR_HD __host__ __device__
#else
#define VR_HD
#endif

namespace vr {

VR_HD inline uint32_t kc_popc32(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
VR_HD inline uint32_t kc_popc64(uint64_t x) { return (uint32_t)__builtin_popcountll(x); }
VR_HD inline uint32_t kc_ctz64(uint64_t x) { return (uint32_t)__builtin_ctzll(x); }
VR_HD inline uint64_t kc_lowmask(uint32_t b) { return b >= 64 ? ~0ull : ((1ull << b) - 1ull); }

// sum of the four byte products (v_dot4_u32_u8 on the device)
VR_HD inline uint32_t kc_dot4(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_udot4(a, b, 0u, false);
#else
  return (a & 255u) * (b & 255u) + ((a >> 8) & 255u) * ((b >> 8) & 255u) +
         ((a >> 16) & 255u) * ((b >> 16) & 255u) + (a >> 24) * (b >> 24);
#endif
}

// #{(i, j): i < j, bit i of o, bit j of z} for 32-bit words, by field level: pairs inside
// 2-bit fields, then across the halves of each nibble, of each byte, and across bytes
// (SWAR field counts; the cross-half products are byte dot products).
VR_HD inline uint32_t kc_pairs32(uint32_t o, uint32_t z) {
  uint32_t r = kc_popc32(o & (z >> 1) & 0x55555555u);
  const uint32_t o2 = o - ((o >> 1) & 0x55555555u);  // 2-bit field counts
  const uint32_t z2 = z - ((z >> 1) & 0x55555555u);
  r += kc_dot4(o2 & 0x03030303u, (z2 >> 2) & 0x03030303u);         // even nibbles
  r += kc_dot4((o2 >> 4) & 0x03030303u, (z2 >> 6) & 0x03030303u);  // odd nibbles
  const uint32_t o4 = (o2 & 0x33333333u) + ((o2 >> 2) & 0x33333333u);  // nibble counts
  const uint32_t z4 = (z2 & 0x33333333u) + ((z2 >> 2) & 0x33333333u);
  r += kc_dot4(o4 & 0x0F0F0F0Fu, (z4 >> 4) & 0x0F0F0F0Fu);           // nibble halves of bytes
  const uint32_t o8 = (o4 + (o4 >> 4)) & 0x0F0F0F0Fu;                 // byte counts
  const uint32_t z8 = (z4 + (z4 >> 4)) & 0x0F0F0F0Fu;
  r += kc_dot4((o8 * 0x01010101u) << 8, z8);                          // across bytes
  return r;
}

VR_HD inline uint64_t kc_pairs64(uint64_t o, uint64_t z) {
  const uint32_t ol = (uint32_t)o, oh = (uint32_t)(o >> 32);
  const uint32_t zl = (uint32_t)z, zh = (uint32_t)(z >> 32);
  return (uint64_t)kc_pairs32(ol, zl) + kc_pairs32(oh, zh) + (uint64_t)kc_popc32(ol) * kc_popc32(zh);
}

// Running state of one lane over a contiguous range of windows.
//   acc    sum over zeros j of #{ones before j in j's segment, inside the range}
//   c      ones since the last segment start (since the range start if none yet)
//   zlead  zeros before the first segment start of the range (they also pair with ones
//          of the same segment that precede the range: fixed up across ranges)
struct KSeg {
  uint64_t acc;
  uint32_t c;
  uint32_t zlead;
};

// One window. TIE: o == z == the included members of multi-element tie groups, and the
// count is sum over groups of C(k, 2). `seen` (uniform) = a segment start was met.
// sum over zeros j of the ones before j in the window (segments ignored)
template <bool TIE>
VR_HD inline uint64_t kseg_inner(uint64_t o, uint64_t z) {
  if (TIE) {
    const uint32_t p = kc_popc64(z);
    return (uint64_t)p * (p - 1u) / 2u;
  }
  return kc_pairs64(o, z);
}

// One window given its kseg_inner (callers can compute several windows' inner counts first).
template <bool TIE>
VR_HD inline void kseg_window_inner(uint64_t o, uint64_t z, uint64_t S, uint64_t inner, KSeg& a, bool& seen) {
  const uint32_t pz = kc_popc64(z);
  const uint32_t po = TIE ? pz : kc_popc64(o);
  if (S == 0) {
    a.acc += (uint64_t)a.c * pz + inner;
    if (!seen) a.zlead += pz;
    a.c += po;
    return;
  }
  // zeros of the lead part also pair with the carried ones; zeros of the part starting at
  // s_k must not count the ones before s_k: subtract |z in part k| * P(s_k)
  uint64_t mk = kc_lowmask(kc_ctz64(S));
  uint32_t Zp = kc_popc64(z & mk);
  uint32_t Pp = TIE ? Zp : kc_popc64(o & mk);
  a.acc += (uint64_t)a.c * Zp + inner;
  if (!seen) a.zlead += Zp;
  seen = true;
  uint32_t sub = 0;  // <= 64 x 64 inside one window
  for (uint64_t r = S & (S - 1); r; r &= r - 1) {
    mk = kc_lowmask(kc_ctz64(r));
    const uint32_t Zs = kc_popc64(z & mk);
    const uint32_t Ps = TIE ? Zs : kc_popc64(o & mk);
    sub += (Zs - Zp) * Pp;
    Zp = Zs;
    Pp = Ps;
  }
  sub += (pz - Zp) * Pp;
  a.acc -= sub;
  a.c = po - Pp;
}

template <bool TIE>
VR_HD inline void kseg_window(uint64_t o, uint64_t z, uint64_t S, KSeg& a, bool& seen) {
  kseg_window_inner<TIE>(o, z, S, kseg_inner<TIE>(o, z), a, seen);
}

// Cross-range fix-up, applied to ranges in stream order: range r's lead zeros pair with
// the ones carried into it, carry_in(r) = c(r-1) + (seen(r-1) ? 0 : carry_in(r-1)).
// As an affine map of an unknown carry C: fix = f0 + g C, carry_out = a + b C.
struct KFix {
  uint64_t f0, g, a;
  uint32_t b;
};
VR_HD inline KFix kfix_identity() { return {0ull, 0ull, 0ull, 1u}; }
VR_HD inline void kfix_push(KFix& F, uint32_t zlead, uint32_t c, bool seen) {
  F.f0 += (uint64_t)zlead * F.a;
  F.g += F.b ? (uint64_t)zlead : 0ull;
  if (seen) {
    F.a = c;
    F.b = 0;
  } else {
    F.a += c;
  }
}

}  // namespace vr
