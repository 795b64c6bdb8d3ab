// Test-only code object (built into pairing_amd/lib/test/coop_quad_unit.hsaco,
// never loaded by the product): the quad-cooperative field operations of
// coop_quad.h side by side with the one-lane code they must reproduce bit for
// bit (fl_gen.h leaves, fl.h red).  One case per quad of lanes:
//   in  [case][4][16] u32: operands a, b, c, d as 14 limbs + 2 zero pads
//   out [case][2][16] u32: quad result, one-lane result
//   op 0 = a*b (P1), 1 = a*b + c*d (P2), 2 = a^2 (SQ), 3 = red(a),
//   4 = gather(a) then a*b with a spread (the prologue path)
#include "../../pairing_amd/csrc/coop_quad.h"

using namespace pa;

extern "C" __global__ void __launch_bounds__(256) coop_quad_unit(const uint32_t* __restrict__ in,
                                                                 uint32_t* __restrict__ out, uint32_t n,
                                                                 uint32_t op) {
    const int tid = threadIdx.x;
    const uint32_t item = blockIdx.x * 64 + (tid >> 2);
    const quad::Ctx c = quad::ctx(tid);
    if (item >= n) return;   // whole quads leave together
    const uint32_t* x = in + (size_t)item * 64;
    uint32_t af[14], cf[14], b[4], d[4], a[4], o[4];
    for (int i = 0; i < 14; i++) {
        af[i] = x[i];
        cf[i] = x[32 + i];
    }
    for (int j = 0; j < 4; j++) {
        a[j] = x[4 * c.r + j];
        b[j] = x[16 + 4 * c.r + j];
        d[j] = x[48 + 4 * c.r + j];
    }
    if (op == 0) {
        quad::mont<false>(o, af, b, af, b, c);
    } else if (op == 1) {
        quad::mont<true>(o, af, b, cf, d, c);
    } else if (op == 2) {
        quad::mont<false>(o, af, a, af, a, c);
    } else if (op == 3) {
        for (int j = 0; j < 4; j++) o[j] = a[j];
        quad::red(o, c);
    } else {
        uint32_t g[14];
        quad::gather(g, a);
        quad::mont<false>(o, g, b, g, b, c);
    }
    uint32_t* y = out + (size_t)item * 32;
    for (int j = 0; j < 4; j++) y[4 * c.r + j] = o[j];
    if (c.lead) {
        uint32_t r[14], bf[14], df[14];
        for (int i = 0; i < 14; i++) {
            bf[i] = x[16 + i];
            df[i] = x[48 + i];
        }
        if (op == 0 || op == 4) {
            fl_mul_leaf(r, af, bf);
        } else if (op == 1) {
            fl_sop2_leaf(r, af, bf, cf, df);
        } else if (op == 2) {
            fl_sqr_leaf(r, af);
        } else {
            F<16> v;
            for (int i = 0; i < 14; i++) v.w[i] = af[i];
            const F<1> t = red(v);
            for (int i = 0; i < 14; i++) r[i] = t.w[i];
        }
        for (int i = 0; i < 14; i++) y[16 + i] = r[i];
        y[30] = y[31] = 0;
    }
}

// ---- sixteen-lane products (coop_hex.h): one case per 16-lane row ----
//   op 0 = a*b, 1 = a*b + c*d, 2 = a^2, 4 = gather(a) then a*b with a spread
#include "../../pairing_amd/csrc/coop_hex.h"

extern "C" __global__ void __launch_bounds__(256) coop_hex_unit(const uint32_t* __restrict__ in,
                                                                uint32_t* __restrict__ out, uint32_t n,
                                                                uint32_t op) {
    const int tid = threadIdx.x;
    const uint32_t item = blockIdx.x * 16 + (tid >> 4);
    const hex::Ctx c = hex::ctx(tid);
    if (item >= n) return;   // whole rows leave together
    const uint32_t* x = in + (size_t)item * 64;
    uint32_t af[14], cf[14];
    for (int i = 0; i < 14; i++) {
        af[i] = x[i];
        cf[i] = x[32 + i];
    }
    const uint32_t a = x[c.k], b = x[16 + c.k], d = x[48 + c.k];
    uint32_t o;
    if (op == 0) {
        o = hex::mont<false>(af, b, af, b, c);
    } else if (op == 1) {
        o = hex::mont<true>(af, b, cf, d, c);
    } else if (op == 2) {
        o = hex::mont<false>(af, a, af, a, c);
    } else {
        uint32_t g[14];
        hex::gather(g, a);
        o = hex::mont<false>(g, b, g, b, c);
    }
    uint32_t* y = out + (size_t)item * 32;
    y[c.k] = o;
    if (c.k == 0) {
        uint32_t r[14], bf[14], df[14];
        for (int i = 0; i < 14; i++) {
            bf[i] = x[16 + i];
            df[i] = x[48 + i];
        }
        if (op == 0 || op == 4) fl_mul_leaf(r, af, bf);
        else if (op == 1) fl_sop2_leaf(r, af, bf, cf, df);
        else fl_sqr_leaf(r, af);
        for (int i = 0; i < 14; i++) y[16 + i] = r[i];
        y[30] = y[31] = 0;
    }
}

// Latency probe: ONE wave runs `iters` dependent squarings x <- x^2 R'^-1 of
// the values it holds -- mode 0 on lane quads (16 values), mode 1 on 16-lane
// rows (4 values); out[0..1] = wall-clock ticks (100 MHz) and shader cycles
// of the chain, out[2 + ...] the final limbs (so the chain is not dead code)
extern "C" __global__ void __launch_bounds__(64) coop_chain_probe(uint32_t* __restrict__ out, uint32_t mode,
                                                                  uint32_t iters) {
    const int tid = threadIdx.x;
    uint32_t res = 0;
    const uint64_t w0 = wall_clock64(), c0 = clock64();
    if (mode == 0) {
        const quad::Ctx c = quad::ctx(tid);
        uint32_t v[4];
        for (int j = 0; j < 4; j++) v[j] = (4 * c.r + j < 13) ? (0x1234567u + 77u * tid + j) & FL_MASK : 0u;
#pragma unroll 1
        for (uint32_t it = 0; it < iters; it++) {
            uint32_t g[14], o[4];
            quad::gather(g, v);
            quad::mont<false>(o, g, v, g, v, c);
            for (int j = 0; j < 4; j++) v[j] = o[j];
        }
        res = v[0] ^ v[1] ^ v[2] ^ v[3];
    } else {
        const hex::Ctx c = hex::ctx(tid);
        uint32_t v = c.k < 13 ? (0x1234567u + 77u * tid) & FL_MASK : 0u;
#pragma unroll 1
        for (uint32_t it = 0; it < iters; it++) {
            uint32_t g[14];
            hex::gather(g, v);
            v = hex::mont<false>(g, v, g, v, c);
        }
        res = v;
    }
    const uint64_t w1 = wall_clock64(), c1 = clock64();
    if (tid == 0) {
        out[0] = (uint32_t)(w1 - w0);
        out[1] = (uint32_t)(c1 - c0);
    }
    out[2 + tid] = res;
}
