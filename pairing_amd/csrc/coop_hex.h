// Sixteen-lane base-field product (experiment, round 4; not on a product
// path yet): one Fq value per 16-lane DPP row, lane k = lane & 15 holding limb
// k of the lazy 14 x 28-bit representation (fl.h), lanes 14 and 15 zero.  The
// latency-shaped paths (decode, MSM Horner, comb base chains, the verifier VM)
// run their products on lane quads (coop_quad.h): four limbs per lane, ~30
// instructions per CIOS row for a lone wave to issue.  Here a row is ~12:
//   t_k += a_i b_k;  m = (t_0 (-q^-1)) mod 2^28 broadcast from lane 0 (DPP
//   row_newbcast);  t_k += m q_k;  t_k <- t_(k+1) (DPP row_shl, the 64-bit
//   accumulator in two moves), lane 0 adding the dropped limb's carry.
// The result is the exact base-2^28 digits of (T + m q) / 2^392 -- the
// leaves' output (fl_gen.h), bit for bit, as the quad form's.
#pragma once
#include "fl.h"

namespace pa {
namespace hex {

constexpr int kShl1 = 0x101;   // row_shl:1: lane k reads lane k+1 of its row (lane 15: 0)
constexpr int kShr1 = 0x111;   // row_shr:1: lane k reads lane k-1 (lane 0: 0)

template <int C>
PA_DEV uint32_t dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, C, 0xf, 0xf, false);
}
template <int L>
PA_DEV uint32_t bcast(uint32_t x) {   // row_newbcast:L -- lane L of the row to all 16
    return dpp<0x150 + L>(x);
}
PA_DEV uint64_t mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

struct Ctx {
    int k;        // limb index = lane & 15
    uint32_t q;   // limb k of q (0 for the pads)
};
PA_DEV Ctx ctx(int lane) {
    Ctx c;
    c.k = lane & 15;
    c.q = c.k < 14 ? FL_Q[c.k] : 0u;
    return c;
}

// the whole value in every lane of the row from the spread limbs
template <int L = 0>
PA_DEV void gather(uint32_t* full, uint32_t v) {
    full[L] = bcast<L>(v);
    if constexpr (L + 1 < 14) gather<L + 1>(full, v);
}

// exact base-2^28 digits of sum t_k 2^(28 k) over the row (value < 2^392,
// t_k < 2^64): carries move one lane up per round until none is left
PA_DEV uint32_t norm(uint64_t t) {
    uint32_t d = (uint32_t)t & FL_MASK;
    uint64_t cy = t >> 28;
#pragma unroll 1
    for (int r = 0; r < 15; r++) {
        const uint32_t lo = dpp<kShr1>((uint32_t)cy), hi = dpp<kShr1>((uint32_t)(cy >> 32));
        const uint64_t v = (uint64_t)d + ((uint64_t)hi << 32 | lo);
        d = (uint32_t)v & FL_MASK;
        cy = v >> 28;
        if (!__any(cy != 0)) break;
    }
    return d;
}

// a b (+ c d) R'^-1, R' = 2^392: a, c whole (14 limbs), b, d this lane's limb;
// returns this lane's limb of the leaves' output
template <bool TWO>
PA_DEV uint32_t mont(const uint32_t* a, uint32_t b, const uint32_t* cc, uint32_t d, const Ctx& c) {
    uint64_t t = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
        t = mad(a[i], b, t);
        if (TWO) t = mad(cc[i], d, t);
        const uint32_t m = bcast<0>(((uint32_t)t * FL_QINV) & FL_MASK);
        t = mad(m, c.q, t);
        // lane 0's t is now 0 mod 2^28: its carry joins lane 1's accumulator,
        // which becomes lane 0's
        const uint64_t cy = t >> 28;
        const uint32_t lo = dpp<kShl1>((uint32_t)t), hi = dpp<kShl1>((uint32_t)(t >> 32));
        t = ((uint64_t)hi << 32 | lo) + (c.k == 0 ? cy : 0ull);
    }
    return norm(t);
}

}  // namespace hex
}  // namespace pa
