// Fq inversion by optimized binary GCD (T. Pornin, "Optimized Binary GCD for
// Modular Inversion", 2020), for one lane.
//
// The reference inverts with a variable-time binary extended Euclid
// (src/bls12_381/fq.rs:849-902); the inverse is unique, so any correct
// algorithm gives the same bits.  Fermat (a^(q-2), tower.h) costs ~570
// sequential Montgomery products -- the latency floor of every kernel that
// normalizes points one chunk per lane.  This routine replaces it with
// 26 outer steps of:
//   * 30 inner binary-GCD steps on 62-bit approximations of (a, b) (the low 30
//     bits and the top 32 bits), branch-free, accumulating the update matrix
//     (f0 g0; f1 g1) with |f| + |g| <= 2^30 in int32;
//   * one exact update (a, b) <- ((a f0 + b g0), (a f1 + b g1)) / 2^30 and
//     (u, v) <- the same combination divided by 2^30 mod q (one Montgomery
//     digit), keeping a = u y and b = v y (mod q).
// 26 x 30 = 780 >= 2 len(q) - 1 = 761 inner steps, enough for b to reach
// gcd = 1 (Pornin, Theorem 1); then v = y^-1.
//
// Plain 32-bit-word C++ with fully unrolled limb loops (no dynamically indexed
// register arrays), usable from host code for the CPU test
// (tests/test_bgcd.py compiles it with g++) and from device code.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PA_HD __host__ __device__ __forceinline__
#else
#define PA_HD static inline
#endif

namespace pa {
namespace bgcd {

constexpr int kS = 30;      // bits divided out per outer step = inner steps
constexpr int kOuter = 26;  // ceil((2 * 381 - 1) / 30)
constexpr uint32_t kMask = (1u << kS) - 1;
constexpr uint32_t kQInv = 0x3ffcfffdu;  // -q^-1 mod 2^30

PA_HD uint32_t qw(int i) {
    constexpr uint32_t q[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                                0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
    return q[i];
}

PA_HD int clz32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __clz(x);
#else
    return x ? __builtin_clz(x) : 32;
#endif
}

PA_HD int bitlen(const uint32_t* x) {
    int n = 0;
#pragma unroll
    for (int i = 0; i < 12; i++)
        if (x[i]) n = 32 * i + 32 - clz32(x[i]);
    return n;
}

// floor(x / 2^p) mod 2^32 for 30 <= p <= 352 (selects, no dynamic indexing)
PA_HD uint32_t bits32(const uint32_t* x, int p) {
    const int wi = p >> 5, sh = p & 31;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        if (i == wi) lo = x[i];
        if (i == wi + 1) hi = x[i];
    }
    const uint64_t v = ((uint64_t)hi << 32) | lo;
    return (uint32_t)(v >> sh);
}

// c = (x f + y g) / 2^30, exact; returns true if c < 0 (then c holds |c|)
PA_HD bool comb_shift(uint32_t* c, const uint32_t* x, const uint32_t* y, int32_t f, int32_t g) {
    uint32_t t[13];
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        acc += (int64_t)(uint64_t)x[i] * f + (int64_t)(uint64_t)y[i] * g;
        t[i] = (uint32_t)acc;
        acc >>= 32;
    }
    t[12] = (uint32_t)acc;
    const bool negv = (int32_t)t[12] < 0;
    // shift right by 30 (low 30 bits are zero by construction)
#pragma unroll
    for (int i = 0; i < 12; i++) c[i] = (t[i] >> kS) | (t[i + 1] << (32 - kS));
    if (negv) {
        uint64_t b = 1;
#pragma unroll
        for (int i = 0; i < 12; i++) {
            b += (uint32_t)~c[i];
            c[i] = (uint32_t)b;
            b >>= 32;
        }
    }
    return negv;
}

// c = (x f + y g) / 2^30 mod q, for x, y in [0, q), |f| + |g| <= 2^30
PA_HD void comb_mod(uint32_t* c, const uint32_t* x, const uint32_t* y, int32_t f, int32_t g) {
    uint32_t t[13];
    int64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        acc += (int64_t)(uint64_t)x[i] * f + (int64_t)(uint64_t)y[i] * g;
        t[i] = (uint32_t)acc;
        acc >>= 32;
    }
    t[12] = (uint32_t)acc;
    // t += k q with k = -t q^-1 mod 2^30: the low 30 bits become zero
    const uint32_t k = (t[0] * kQInv) & kMask;
    uint64_t cy = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        cy += (uint64_t)t[i] + (uint64_t)k * qw(i);
        t[i] = (uint32_t)cy;
        cy >>= 32;
    }
    t[12] += (uint32_t)cy;  // two's complement top word absorbs the carry
    // s = t / 2^30 in [-q, 2q)
    uint32_t s[12];
#pragma unroll
    for (int i = 0; i < 12; i++) s[i] = (t[i] >> kS) | (t[i + 1] << (32 - kS));
    const uint32_t top = (uint32_t)((int32_t)t[12] >> kS);  // 0 or all-ones (sign)
    // negative: add q
    {
        const uint32_t m = top;  // all-ones iff negative
        uint64_t b = 0;
#pragma unroll
        for (int i = 0; i < 12; i++) {
            b += (uint64_t)s[i] + (qw(i) & m);
            s[i] = (uint32_t)b;
            b >>= 32;
        }
    }
    // >= q: subtract q
    uint32_t d[12];
    int64_t br = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
        br += (int64_t)s[i] - (int64_t)qw(i);
        d[i] = (uint32_t)br;
        br >>= 32;
    }
    const bool ge = br == 0;  // no borrow: s >= q
#pragma unroll
    for (int i = 0; i < 12; i++) c[i] = ge ? d[i] : s[i];
}

// out = y^-1 mod q (plain integers, y < q); false iff y == 0
PA_HD bool inverse(uint32_t* out, const uint32_t* y) {
    uint32_t a[12], b[12], u[12], v[12];
#pragma unroll
    for (int i = 0; i < 12; i++) {
        a[i] = y[i];
        b[i] = qw(i);
        u[i] = i == 0;
        v[i] = 0;
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll 1
#endif
    for (int it = 0; it < kOuter; it++) {
        int n = bitlen(a);
        const int nb = bitlen(b);
        n = n > nb ? n : nb;
        n = n > 62 ? n : 62;
        uint64_t xa = ((uint64_t)bits32(a, n - 32) << kS) | (a[0] & kMask);
        uint64_t xb = ((uint64_t)bits32(b, n - 32) << kS) | (b[0] & kMask);
        int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll
        for (int j = 0; j < kS; j++) {
            const bool odd = xa & 1;
            const bool sw = odd && xa < xb;
            const uint64_t na = sw ? xb : xa, nb2 = sw ? xa : xb;
            const int32_t nf0 = sw ? f1 : f0, ng0 = sw ? g1 : g0;
            const int32_t nf1 = sw ? f0 : f1, ng1 = sw ? g0 : g1;
            xa = (odd ? na - nb2 : na) >> 1;
            xb = nb2;
            f0 = odd ? nf0 - nf1 : nf0;
            g0 = odd ? ng0 - ng1 : ng0;
            f1 = nf1 << 1;
            g1 = ng1 << 1;
        }
        uint32_t na[12], nbv[12];
        if (comb_shift(na, a, b, f0, g0)) {
            f0 = -f0;
            g0 = -g0;
        }
        if (comb_shift(nbv, a, b, f1, g1)) {
            f1 = -f1;
            g1 = -g1;
        }
        uint32_t nu[12], nv[12];
        comb_mod(nu, u, v, f0, g0);
        comb_mod(nv, u, v, f1, g1);
#pragma unroll
        for (int i = 0; i < 12; i++) {
            a[i] = na[i];
            b[i] = nbv[i];
            u[i] = nu[i];
            v[i] = nv[i];
        }
    }
    uint32_t one = b[0] ^ 1u;
#pragma unroll
    for (int i = 1; i < 12; i++) one |= b[i];
#pragma unroll
    for (int i = 0; i < 12; i++) out[i] = v[i];
    return one == 0;
}

}  // namespace bgcd
}  // namespace pa
