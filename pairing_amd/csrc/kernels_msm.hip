// Variable-base scalar multiplication and multi-scalar multiplication (MSM)
// for G1 and G2 (SURVEY.md §8 f, rank 3).
//
// Per-lane scalar multiplication, bit-exact Jacobian output:
//   CurveAffine::mul (ec.rs:174-177 -> mul_bits ec.rs:88-95): for every one of
//     the 256 scalar bits, MSB first: double, then add_assign_mixed(base) if set.
//   CurveProjective::mul_assign (ec.rs:534-553): double-and-add with full
//     add_assign(self), doubling only after the first set bit.
// Both replay the reference's exact formula sequence (curve.h), so the X, Y, Z
// words equal the reference's, not just the point.
//
// MSM  sum_i s_i * P_i  (affine bases, FrRepr scalars: the shape of the
// downstream provers' multiexp over `CurveAffine::mul` + `add_assign`).  The
// result is equal *as a point* to the reference's sum (PartialEq, ec.rs:45-85);
// Jacobian words differ because the addition chain is Pippenger's:
//   1. k_msm_digits: signed c-bit digits per window (|d| <= 2^(c-1)); item
//      (window, |d|) -> sort key, (i | sign<<31) -> value.   c*W >= 257 so any
//      256-bit FrRepr (also >= r, as the reference's BitIterator allows) fits.
//   2. a stable LSD counting sort of the items by bucket, 8 bits per pass
//      (k_sort_hist / k_sort_scan / k_sort_scatter, ceil((c-1)/8) passes):
//      each bucket's points become contiguous in term order, windows stay
//      apart, zero digits are dropped.  Same order as a stable sort of the
//      (w*B + |d|-1) keys, so the result is deterministic.
//   3. k_msm_bucket_bounds: [start, end) per bucket from the sorted keys.
//   4. k_msm_chunk_acc: one lane per 64 sorted items, mixed additions
//      (madd-2007-bl) of the affine bases gathered from HBM (y negated for
//      negative digits), run by run; k_msm_bucket_fix folds the pieces of
//      buckets that span chunks and zeroes empty buckets.
//   5. k_msm_segments: per window, sum_m m*B_m by running sums over segments of
//      L buckets (T += B_m; S += T, top down), plus a*T for the segment offset.
//   6. k_msm_group_sum (repeated): segment results -> one sum per window.
//   7. k_msm_horner_q: one group of lane quads, sum_w 2^(c*w) S_w.
// Steps 4-7 run per part of the windows (top windows first, msm_run): a part's
// reduction (4's fix-up, 5, 6) and its Horner leg run on side streams while
// the next part accumulates, so only the last part's tail is exposed.
// Work: n*W mixed additions + ~2*W*2^(c-1) additions + ~256 doublings.

#include <vector>

#include "curve_fl.h"
#include "curve_fl2.h"
#include "dec_quad.h"
#include "launch_msm.h"

#include <cstdlib>
#include <mutex>
#include <utility>

namespace pa {

template <int G> struct Grp;
template <> struct Grp<1> {
    using F = Fq;
    static constexpr int AW = 13;  // u64 words per affine record (pa_g1_affine)
    static constexpr int JW = 18;  // u64 words per Jacobian record (pa_g1)
};
template <> struct Grp<2> {
    using F = Fq2;
    static constexpr int AW = 25;
    static constexpr int JW = 36;
};

// ---------------- per-lane scalar multiplication ----------------
template <int G>
__global__ void __launch_bounds__(64) k_affine_mul(const uint64_t* __restrict__ p, const uint64_t* __restrict__ s,
                                                   uint64_t* __restrict__ out, size_t n) {
    using F = typename Grp<G>::F;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<F> a;
    load_aff(a, p + (size_t)Grp<G>::AW * i);
    uint64_t k[4];
#pragma unroll
    for (int w = 0; w < 4; w++) k[w] = s[4 * i + w];
    Jac<F> acc;
    jac_zero(acc);
#pragma unroll 1
    for (int bit = 255; bit >= 0; bit--) {  // mul_bits, ec.rs:88-95
        jac_double(acc);
        if ((k[bit >> 6] >> (bit & 63)) & 1) jac_add_mixed(acc, a);
    }
    store_jac(out + (size_t)Grp<G>::JW * i, acc);
}

template <int G>
__global__ void __launch_bounds__(64) k_proj_mul(const uint64_t* __restrict__ p, const uint64_t* __restrict__ s,
                                                 uint64_t* __restrict__ out, size_t n) {
    using F = typename Grp<G>::F;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Jac<F> base, acc;
    load_jac(base, p + (size_t)Grp<G>::JW * i);
    uint64_t k[4];
#pragma unroll
    for (int w = 0; w < 4; w++) k[w] = s[4 * i + w];
    jac_zero(acc);
    bool found_one = false;
#pragma unroll 1
    for (int bit = 255; bit >= 0; bit--) {  // mul_assign, ec.rs:534-553
        const bool b = (k[bit >> 6] >> (bit & 63)) & 1;
        if (found_one) jac_double(acc);
        else found_one = b;
        if (b) jac_add(acc, base);
    }
    store_jac(out + (size_t)Grp<G>::JW * i, acc);
}

// ---------------- MSM ----------------
struct MsmPlan {
    uint32_t c, W, B, L;        // window bits, windows, buckets per window, segment length
    uint32_t passes;            // counting-sort passes over the c-1 magnitude bits
    uint32_t T;                 // items per lane of the bucket accumulation
    uint32_t tpw;               // sort tiles per window
    size_t items;               // W * n
    size_t off_keys_in, off_keys_out, off_vals_in, off_vals_out, off_start, off_end;
    size_t off_buckets, off_segs, off_tmp, off_hist, off_wtot, off_cont, off_basefl, off_hacc, off_long;
    size_t total;
};

static inline uint32_t msm_window_bits(size_t n) {
    int lg = 0;
    while (lg < 40 && ((size_t)1 << (lg + 1)) <= n) lg++;
    int c = lg - 3;
    static const int cmax = [] {   // A/B knob: PA_MSM_CMAX (default 16)
        const char* v = getenv("PA_MSM_CMAX");
        const int k = v ? atoi(v) : 16;
        return k < 4 ? 4 : (k > 20 ? 20 : k);
    }();
    if (c < 4) c = 4;
    if (c > cmax) c = cmax;
    return (uint32_t)c;
}

// items (sorted (bucket, term) pairs) per lane of the bucket accumulation
// (PA_MSM_CHUNK to A/B, 8..512): 32 / 48 / 64 / 96 / 128 measured 167 / 162 /
// 170 / 159 / 171 M terms/s at 2^20 with one part, 64 with two parts 175-177
// (profiles/r04_msm_parts.txt)
constexpr uint32_t kMsmChunk = 64;
// Below 64 items per lane the chunk shrinks until a part's accumulation has
// one lane for each of the chip's 256 CUs x 4 SIMDs x 64 (G2 at 2^16: 20 x 2^16
// items, 320 waves at 64 per lane)
constexpr size_t kMsmFillLanes = 65536;
static uint32_t msm_chunk(size_t items, uint32_t parts) {
    static const int env = [] {
        const char* v = getenv("PA_MSM_CHUNK");
        return v ? atoi(v) : 0;
    }();
    if (env) return (uint32_t)(env < 8 ? 8 : (env > 512 ? 512 : env));
    const size_t t = (items + kMsmFillLanes * parts - 1) / (kMsmFillLanes * parts);
    return (uint32_t)(t < 8 ? 8 : (t > kMsmChunk ? kMsmChunk : t));
}
// window parts (msm_run): at most this many, each with a Horner accumulator slot
constexpr uint32_t kMsmMaxParts = 8;
// a bucket whose items span more chunks than this has its continuation pieces
// summed by a block (k_msm_long_fix), not serially by one lane of
// k_msm_bucket_fix.  A block costs ~span/256 + 8 additions per bucket with at
// most kMsmLongBlocks buckets at a time, a lane `span` additions with every
// bucket at once: above 128 chunks the block is never the slower choice, even
// when every bucket of every window is that long (at most ~2 100 of them at
// 2^20 terms)
constexpr size_t kMsmLongSpan = 128;
constexpr unsigned kMsmLongBlocks = 256;
// counting sort: a tile is 16 rounds of one item per thread of a 256-thread block
constexpr uint32_t kSortIpt = 16;
constexpr uint32_t kSortTile = 256 * kSortIpt;

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// window parts of one MSM (PA_MSM_PARTS, default 2; 1 = every kernel on the
// caller's stream in order; 3 and 4 measured slower: the tails compete with the
// next part's accumulation for SIMDs, profiles/r04_msm_parts.txt)
static uint32_t msm_parts(uint32_t W) {
    static const uint32_t parts = [] {
        const char* v = getenv("PA_MSM_PARTS");
        const int k = v ? atoi(v) : 2;
        return (uint32_t)(k < 1 ? 1 : (k > (int)kMsmMaxParts ? (int)kMsmMaxParts : k));
    }();
    return parts < W ? parts : W;
}

static hipError_t msm_plan(MsmPlan& p, int group, size_t n) {
    p.c = msm_window_bits(n);
    p.W = (257 + p.c - 1) / p.c;
    p.B = 1u << (p.c - 1);
    // A/B knob: PA_MSM_SEG; default 8 buckets per segment for G1, 4 for G2 (G2
    // at 2^16 / 2^18: 5.91 / 9.13 ms with 8, 5.73 / 8.90 with 4; G1 at 2^20: 173
    // vs 163 M terms/s; profiles/r04_msm_g2_lazy.txt)
    static const int seg_env = [] {
        const char* v = getenv("PA_MSM_SEG");
        const int k = v ? atoi(v) : 0;
        return k == 2 || k == 4 || k == 8 || k == 16 || k == 32 ? k : 0;
    }();
    const uint32_t seg = seg_env ? (uint32_t)seg_env : (group == 1 ? 8u : 4u);
    p.L = p.B < seg ? p.B : seg;  // short segments: the running sums are a latency chain per lane
    p.items = (size_t)p.W * n;
    p.passes = (p.c - 1 + 7) / 8;
    p.tpw = (uint32_t)((n + kSortTile - 1) / kSortTile);
    const size_t jw = 8 * (size_t)(group == 1 ? Grp<1>::JW : Grp<2>::JW);
    const size_t nb = (size_t)p.W * p.B;
    const size_t nseg = (size_t)p.W * (p.B / p.L);
    size_t off = 0;
    p.off_keys_in = off; off = align256(off + 4 * p.items);
    p.off_keys_out = off; off = align256(off + 4 * p.items);
    p.off_vals_in = off; off = align256(off + 4 * p.items);
    p.off_vals_out = off; off = align256(off + 4 * p.items);
    p.off_start = off; off = align256(off + 4 * nb);
    p.off_end = off; off = align256(off + 4 * nb);
    p.off_buckets = off; off = align256(off + jw * nb);
    p.off_segs = off; off = align256(off + jw * nseg);
    p.off_tmp = off; off = align256(off + jw * nseg);
    p.T = msm_chunk(p.items, msm_parts(p.W));
    p.off_cont = off; off = align256(off + jw * ((p.items + p.T - 1) / p.T + 1));
    p.off_basefl = off; off = align256(off + 4 * (group == 1 ? 28 : 56) * n);
    p.off_hist = off; off = align256(off + 4 * (size_t)p.W * 256 * p.tpw);
    p.off_wtot = off; off = align256(off + 4 * (size_t)p.W);
    p.off_hacc = off; off = align256(off + jw * kMsmMaxParts);
    p.off_long = off; off = align256(off + 4 * (nb + kMsmMaxParts));   // long-bucket lists + counts
    p.total = off;
    return hipSuccess;
}

__global__ void __launch_bounds__(256) k_msm_digits(const uint64_t* __restrict__ scalars, size_t n, uint32_t c,
                                                    uint32_t W, uint32_t B, uint32_t* __restrict__ keys,
                                                    uint32_t* __restrict__ vals) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k[4];
#pragma unroll
    for (int w = 0; w < 4; w++) k[w] = scalars[4 * i + w];
    const uint32_t sentinel = W * B;
    const uint32_t mask = (1u << c) - 1;
    uint32_t carry = 0;
    for (uint32_t w = 0; w < W; w++) {
        const uint32_t bit = w * c;
        uint32_t raw = 0;
        if (bit < 256) {
            const uint32_t word = bit >> 6, sh = bit & 63;
            uint64_t v = k[word] >> sh;
            if (sh + c > 64 && word < 3) v |= k[word + 1] << (64 - sh);
            raw = (uint32_t)v & mask;
        }
        raw += carry;
        int d;
        if (raw > B) {
            d = (int)raw - (int)(1u << c);
            carry = 1;
        } else {
            d = (int)raw;
            carry = 0;
        }
        const size_t at = (size_t)w * n + i;
        if (d == 0) {
            keys[at] = sentinel;
            vals[at] = (uint32_t)i;
        } else {
            const uint32_t mag = (uint32_t)(d < 0 ? -d : d);
            keys[at] = w * B + (mag - 1);
            vals[at] = (uint32_t)i | (d < 0 ? 0x80000000u : 0u);
        }
    }
}

__global__ void __launch_bounds__(256) k_msm_bucket_bounds(const uint32_t* __restrict__ keys, size_t items,
                                                           uint32_t sentinel, uint32_t* __restrict__ start,
                                                           uint32_t* __restrict__ end) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= items) return;
    const uint32_t k = keys[j];
    if (k >= sentinel) return;
    if (j == 0 || keys[j - 1] != k) start[k] = (uint32_t)j;
    if (j + 1 == items || keys[j + 1] != k) end[k] = (uint32_t)(j + 1);
}

// ---- the bucketing sort (step 2) ----
// Items are (key, value) = (w*B + |d|-1, term | sign<<31).  Pass k orders the
// items of each window by the 8-bit digit ((key & (B-1)) >> 8k), stably; the
// first pass reads the window-major digit output (window w at [w*n, w*n + n),
// zero digits carry key >= sentinel and are skipped), every pass writes the
// windows compacted (window w at [wbase(w), wbase(w) + wtot[w])).  A window's
// source range is cut in tiles of kSortTile items; hist[w][digit][tile] holds
// the tile's digit counts, and after k_sort_scan the exclusive prefix over
// (digit, tile) in that order -- where the tile's run of each digit starts.

// window w's first item in the compacted layout
PA_DEV uint32_t sort_wbase(const uint32_t* __restrict__ wtot, uint32_t w) {
    uint32_t b = 0;
    for (uint32_t k = 0; k < w; k++) b += wtot[k];
    return b;
}

struct SortPass {
    uint32_t shift, bmask, sentinel, tpw, first;
    size_t n;
};

// window w's source range [base, base + count); tile t is its items
// [t kSortTile, (t + 1) kSortTile) clipped to count
PA_DEV void sort_window(const SortPass& sp, const uint32_t* __restrict__ wtot, uint32_t w, size_t& base,
                        uint32_t& count) {
    if (sp.first) {
        base = (size_t)w * sp.n;
        count = (uint32_t)sp.n;
    } else {
        base = sort_wbase(wtot, w);
        count = wtot[w];
    }
}

__global__ void __launch_bounds__(256) k_sort_hist(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ wtot,
                                                   SortPass sp, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    const uint32_t tid = threadIdx.x, w = blockIdx.x / sp.tpw, t = blockIdx.x % sp.tpw;
    h[tid] = 0;
    __syncthreads();
    size_t base;
    uint32_t count;
    sort_window(sp, wtot, w, base, count);
    const uint32_t lo = t * kSortTile;
    uint32_t key[kSortIpt];  // the whole tile's loads in flight at once
#pragma unroll
    for (uint32_t r = 0; r < kSortIpt; r++) {
        const uint32_t k = lo + r * 256 + tid;
        key[r] = k < count ? keys[base + k] : 0xffffffffu;
    }
#pragma unroll
    for (uint32_t r = 0; r < kSortIpt; r++)
        if (key[r] < sp.sentinel) atomicAdd(&h[((key[r] & sp.bmask) >> sp.shift) & 0xff], 1u);
    __syncthreads();
    hist[((size_t)w * 256 + tid) * sp.tpw + t] = h[tid];
}

// exclusive prefix over one window's 256 x tpw counts (digit-major), in place;
// the window's item count into wtot[w].  One 1024-thread block per window,
// segments of 1024 x 64 counters: each thread's 64 as 16 uint4 loads in
// flight, a block scan of the 1024 thread sums, then the prefixed writes.
__global__ void __launch_bounds__(1024) k_sort_scan(uint32_t* __restrict__ hist, uint32_t tpw,
                                                    uint32_t* __restrict__ wtot) {
    __shared__ uint32_t s[2][1024];
    const uint32_t tid = threadIdx.x;
    uint32_t* a = hist + (size_t)blockIdx.x * 256 * tpw;
    const uint32_t len = 256 * tpw;  // a multiple of 4
    uint32_t carry = 0;
    for (uint32_t seg = 0; seg < len; seg += 1024 * 64) {
        const uint32_t b0 = seg + tid * 64;
        uint4 v[16];
#pragma unroll
        for (int q = 0; q < 16; q++)
            v[q] = b0 + 4 * q < len ? *reinterpret_cast<const uint4*>(a + b0 + 4 * q) : make_uint4(0, 0, 0, 0);
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < 16; q++) sum += v[q].x + v[q].y + v[q].z + v[q].w;
        s[0][tid] = sum;
        __syncthreads();
        int cur = 0;
        for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan
            s[cur ^ 1][tid] = s[cur][tid] + (tid >= d ? s[cur][tid - d] : 0u);
            cur ^= 1;
            __syncthreads();
        }
        uint32_t run = carry + s[cur][tid] - sum;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            uint4 o;
            o.x = run;
            o.y = (run += v[q].x);
            o.z = (run += v[q].y);
            o.w = (run += v[q].z);
            run += v[q].w;
            if (b0 + 4 * q < len) *reinterpret_cast<uint4*>(a + b0 + 4 * q) = o;
        }
        carry += s[cur][1023];
        __syncthreads();  // s is rewritten by the next segment
    }
    if (tid == 0) wtot[blockIdx.x] = carry;
}

// One block per tile: rank the tile's items by digit, stably, stage them
// digit-sorted in LDS, then write each digit's run to its place --
// consecutive threads write consecutive addresses of a few runs instead of
// one scattered word each.  Wave q owns the tile's items [q 1024, (q+1) 1024),
// 64 consecutive ones per round, and counts digits in its own LDS row, so the
// ranking needs no block barrier: source order = (wave, round, lane).
__global__ void __launch_bounds__(256) k_sort_scatter(const uint32_t* __restrict__ keys_in,
                                                      const uint32_t* __restrict__ vals_in,
                                                      const uint32_t* __restrict__ hist,
                                                      const uint32_t* __restrict__ wtot, SortPass sp,
                                                      uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out) {
    __shared__ uint32_t gbase[256], loff[256], wcnt[4][256], scan[2][256];
    __shared__ uint32_t sk[kSortTile], sv[kSortTile];
    __shared__ uint32_t wb_s;
    const uint32_t tid = threadIdx.x, w = blockIdx.x / sp.tpw, t = blockIdx.x % sp.tpw;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    size_t base;
    uint32_t count;
    sort_window(sp, wtot, w, base, count);
    const uint32_t lo = t * kSortTile + wave * (64 * kSortIpt);
    uint32_t keyr[kSortIpt], valr[kSortIpt];  // the wave's loads in flight at once
#pragma unroll
    for (uint32_t r = 0; r < kSortIpt; r++) {
        const uint32_t k = lo + r * 64 + lane;
        keyr[r] = 0xffffffffu;
        valr[r] = 0;
        if (k < count) {
            keyr[r] = keys_in[base + k];
            valr[r] = vals_in[base + k];
        }
    }
    if (tid == 0) wb_s = sort_wbase(wtot, w);
    // this tile's digit counts from the prefix: next entry (digit-major) minus this one
    const size_t flat = (size_t)tid * sp.tpw + t, len = (size_t)256 * sp.tpw;
    const uint32_t* hw = hist + (size_t)w * len;
    const uint32_t off = hw[flat];
    const uint32_t cnt = (flat + 1 < len ? hw[flat + 1] : wtot[w]) - off;
    scan[0][tid] = cnt;
#pragma unroll
    for (int q = 0; q < 4; q++) wcnt[q][tid] = 0;
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1;
    uint32_t slot[kSortIpt];  // rank among the wave's items of the same digit
#pragma unroll
    for (uint32_t r = 0; r < kSortIpt; r++) {
        const bool valid = keyr[r] < sp.sentinel;
        const uint32_t d = valid ? ((keyr[r] & sp.bmask) >> sp.shift) & 0xff : 0;
        // lanes of this wave holding the same digit (8 ballots)
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint64_t m = __ballot((d >> b) & 1);
            peers &= ((d >> b) & 1) ? m : ~m;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        const uint32_t before = valid ? wcnt[wave][d] : 0;  // read by all peers before the leader's write
        slot[r] = before + rank;
        if (valid && rank == 0) wcnt[wave][d] = before + (uint32_t)__popcll(peers);
    }
    int cur = 0;
    for (uint32_t d = 1; d < 256; d <<= 1) {  // tile-local digit starts (the barrier also publishes wcnt)
        scan[cur ^ 1][tid] = scan[cur][tid] + (tid >= d ? scan[cur][tid - d] : 0u);
        cur ^= 1;
        __syncthreads();
    }
    const uint32_t tile_items = scan[cur][255];
    loff[tid] = scan[cur][tid] - cnt;
    gbase[tid] = wb_s + off;
    {  // wave q's run of digit d starts after waves < q's
        uint32_t run = scan[cur][tid] - cnt;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t c = wcnt[q][tid];  // column tid is this thread's alone here
            wcnt[q][tid] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kSortIpt; r++) {
        if (keyr[r] < sp.sentinel) {
            const uint32_t d = ((keyr[r] & sp.bmask) >> sp.shift) & 0xff;
            const uint32_t pos = wcnt[wave][d] + slot[r];
            sk[pos] = keyr[r];
            sv[pos] = valr[r];
        }
    }
    __syncthreads();
    for (uint32_t k = tid; k < tile_items; k += 256) {
        const uint32_t key = sk[k];
        const uint32_t d = ((key & sp.bmask) >> sp.shift) & 0xff;
        const size_t pos = (size_t)gbase[d] + (k - loff[d]);
        keys_out[pos] = key;
        vals_out[pos] = sv[k];
    }
}

// Bucket accumulation, load-balanced: lane k owns the sorted items
// [k T, (k+1) T) (T = MsmPlan::T) and adds their bases run by run.  A run whose
// bucket starts inside the chunk is written to the bucket; the chunk's first
// run, when its bucket started in an earlier chunk, goes to cont[k] and is
// folded in by k_msm_bucket_fix.  Every lane does at most T mixed additions
// whatever the digit distribution (a window whose digits crowd into few
// buckets -- the top window of scalars < r -- no longer makes a few lanes
// walk hundreds of terms).
#ifndef PA_MSM_ACC_ATTR
#define PA_MSM_ACC_ATTR
#endif
// chunk k0 + i of the window part [w0, w1): its items [k T, (k+1) T) clipped to
// the part's items [jlo, jhi) of the sorted (window-compacted) array, k0 =
// floor(jlo / T).  A window's items start with a new bucket, so a chunk
// straddling two parts is split cleanly (its second piece never writes cont[k]).
PA_DEV bool chunk_range(size_t i, const uint32_t* __restrict__ wtot, uint32_t w0, uint32_t w1, uint32_t T,
                        size_t& k, size_t& j0, size_t& j1) {
    const size_t jlo = sort_wbase(wtot, w0), jhi = sort_wbase(wtot, w1);
    k = jlo / T + i;
    j0 = k * T;
    j1 = j0 + T;
    if (j0 < jlo) j0 = jlo;
    if (j1 > jhi) j1 = jhi;
    return j0 < j1;
}

template <int G>
PA_DEV void msm_flush(uint32_t key, const Jac<typename Grp<G>::F>& acc, size_t j0, size_t k,
                      const uint32_t* __restrict__ start, uint64_t* __restrict__ buckets,
                      uint64_t* __restrict__ cont) {
    constexpr int JW = Grp<G>::JW;
    if (start[key] >= j0) store_jac(buckets + (size_t)JW * key, acc);
    else store_jac(cont + (size_t)JW * k, acc);
}

template <int G>
__global__ void __launch_bounds__(64) k_msm_chunk_acc(const uint64_t* __restrict__ bases,
                                                      const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ vals,
                                                      const uint32_t* __restrict__ start,
                                                      const uint32_t* __restrict__ wtot, uint32_t w0, uint32_t w1,
                                                      uint32_t T, uint32_t sentinel, uint64_t* __restrict__ buckets,
                                                      uint64_t* __restrict__ cont) {
    using F = typename Grp<G>::F;
    size_t k, j0, j1;
    if (!chunk_range((size_t)blockIdx.x * blockDim.x + threadIdx.x, wtot, w0, w1, T, k, j0, j1)) return;
    uint32_t cur = keys[j0];
    if (cur >= sentinel) return;  // zero digits sort last
    Jac<F> acc;
    jac_zero(acc);
#pragma unroll 1
    for (size_t j = j0; j < j1; j++) {
        const uint32_t key = keys[j];
        if (key >= sentinel) break;
        if (key != cur) {
            msm_flush<G>(cur, acc, j0, k, start, buckets, cont);
            jac_zero(acc);
            cur = key;
        }
        const uint32_t v = vals[j];
        Aff<F> p;
        load_aff(p, bases + (size_t)Grp<G>::AW * (v & 0x7fffffffu));
        if (v >> 31) neg(p.y, p.y);
        jac_add_mixed(acc, p);
    }
    msm_flush<G>(cur, acc, j0, k, start, buckets, cont);
}

// G1 on the lazy 28-bit core: the affine bases converted once per MSM
// (x, y -> 28 u32; the infinity flag in bit 31 of x's top limb, which is
// below 2^18, so a bucket item gathers ONE 112-byte record) ...
__global__ void __launch_bounds__(256) k_msm_bases_fl(const uint64_t* __restrict__ bases, size_t n,
                                                      uint32_t* __restrict__ fl) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<Fq> a;
    load_aff(a, bases + (size_t)Grp<1>::AW * i);
    const F<1> x = fl_from_abi(a.x), y = fl_from_abi(a.y);
    uint32_t* d = fl + 28 * i;
#pragma unroll
    for (int k = 0; k < 14; k++) {
        d[k] = x.w[k] | (k == 13 && a.inf ? 0x80000000u : 0u);
        d[14 + k] = y.w[k];
    }
}

PA_DEV void msm_flush_fl(uint32_t key, const FlJac& acc, bool untouched, size_t j0, size_t k,
                         const uint32_t* __restrict__ start, uint64_t* __restrict__ buckets,
                         uint64_t* __restrict__ cont) {
    constexpr int JW = Grp<1>::JW;
    uint64_t* o = start[key] >= j0 ? buckets + (size_t)JW * key : cont + (size_t)JW * k;
    if (untouched) {
        Jac<Fq> z;
        jac_zero(z);
        store_jac(o, z);
    } else {
        fl_store(o, acc.x);
        fl_store(o + 6, acc.y);
        fl_store(o + 12, acc.z);
    }
}

// ... and k_msm_chunk_acc<1> with the lazy mixed addition (curve_fl.h);
// bucket pieces leave in the ABI form the later phases read.  PREFETCH: the
// next item's base is gathered while the current addition runs (the one-wave
// kernel's latency hiding); without it the two-wave kernel's other wave hides
// the gathers and the 28 registers go to the addition.
template <bool PREFETCH>
PA_DEV void chunk_acc_fl_body(const uint32_t* __restrict__ basefl, const uint32_t* __restrict__ keys,
                                              const uint32_t* __restrict__ vals, const uint32_t* __restrict__ start,
                                              const uint32_t* __restrict__ wtot, uint32_t w0, uint32_t w1,
                                              uint32_t T, uint32_t sentinel, uint64_t* __restrict__ buckets,
                                              uint64_t* __restrict__ cont) {
    size_t k, j0, j1;
    if (!chunk_range((size_t)blockIdx.x * blockDim.x + threadIdx.x, wtot, w0, w1, T, k, j0, j1)) return;
    uint32_t cur = keys[j0];
    if (cur >= sentinel) return;
    FlJac acc;
    acc.x = fl_zero();
    acc.y = fl_one();
    acc.z = fl_zero();
    bool untouched = true;
    // software pipeline: the (key, value) pair two items ahead and the base
    // of the next item are in flight while the current mixed addition runs
    // (the bucket phase is bound by these dependent random gathers)
    auto fetch = [&](size_t jj, uint32_t& kk, uint32_t& vv) {
        kk = sentinel;
        vv = 0;
        if (jj < j1) {
            kk = keys[jj];
            vv = vals[jj];
        }
    };
    auto gather = [&](uint32_t kk, uint32_t vv, F<1>& x, F<1>& y, bool& inf) {
        inf = true;
        if (kk < sentinel) {
            const uint32_t idx = vv & 0x7fffffffu;
            const uint2* src = reinterpret_cast<const uint2*>(basefl + 28 * (size_t)idx);
#pragma unroll
            for (int q = 0; q < 7; q++) {
                const uint2 a = src[q], b = src[7 + q];
                x.w[2 * q] = a.x;
                x.w[2 * q + 1] = a.y;
                y.w[2 * q] = b.x;
                y.w[2 * q + 1] = b.y;
            }
            inf = (x.w[13] >> 31) != 0;
            x.w[13] &= 0x7fffffffu;
        }
    };
    uint32_t key0, v0, key1, v1;
    fetch(j0, key0, v0);
    fetch(j0 + 1, key1, v1);
    F<1> tx, ty;
    bool inf;
    if (PREFETCH) gather(key0, v0, tx, ty, inf);
#pragma unroll 1
    for (size_t j = j0; j < j1; j++) {
        if (key0 >= sentinel) break;
        uint32_t key2, v2;
        fetch(j + 2, key2, v2);
        F<1> nx, ny;
        bool ninf;
        if (PREFETCH) gather(key1, v1, nx, ny, ninf);
        else gather(key0, v0, tx, ty, inf);
        if (key0 != cur) {
            msm_flush_fl(cur, acc, untouched, j0, k, start, buckets, cont);
            untouched = true;
            cur = key0;
        }
        if (!inf) {  // an infinity base is add_assign_mixed's no-op
            const F<2> oy = (v0 >> 31) ? neg(ty) : relax<2>(ty);
            fl_jac_add_mixed(acc, untouched, tx, oy);
        }
        key0 = key1;
        v0 = v1;
        key1 = key2;
        v1 = v2;
        if (PREFETCH) {
            tx = nx;
            ty = ny;
            inf = ninf;
        }
    }
    msm_flush_fl(cur, acc, untouched, j0, k, start, buckets, cont);
}
#define PA_CHUNK_ACC_FL_ARGS                                                                                   \
    const uint32_t *__restrict__ basefl, const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals, \
        const uint32_t *__restrict__ start, const uint32_t *__restrict__ wtot, uint32_t w0, uint32_t w1,      \
        uint32_t T, uint32_t sentinel, uint64_t *__restrict__ buckets, uint64_t *__restrict__ cont
// one wave per SIMD (256 VGPRs + 75 AGPRs), the base prefetched
__global__ void __launch_bounds__(64) PA_MSM_ACC_ATTR k_msm_chunk_acc_fl(PA_CHUNK_ACC_FL_ARGS) {
    chunk_acc_fl_body<true>(basefl, keys, vals, start, wtot, w0, w1, T, sentinel, buckets, cont);
}
// two waves per SIMD (256 registers), the gathers hidden by the other wave
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_msm_chunk_acc_fl_2w(PA_CHUNK_ACC_FL_ARGS) {
    chunk_acc_fl_body<false>(basefl, keys, vals, start, wtot, w0, w1, T, sentinel, buckets, cont);
}
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_msm_chunk_acc_fl_2wp(PA_CHUNK_ACC_FL_ARGS) {
    chunk_acc_fl_body<true>(basefl, keys, vals, start, wtot, w0, w1, T, sentinel, buckets, cont);
}


// One lane per bucket: empty buckets become the identity; a bucket spanning
// several chunks adds the continuation pieces of the chunks after its first.
template <int G, bool LAZY>
__global__ void __launch_bounds__(64) k_msm_bucket_fix(const uint32_t* __restrict__ start,
                                                       const uint32_t* __restrict__ end, size_t b0, size_t b1,
                                                       uint32_t T, const uint64_t* __restrict__ cont,
                                                       uint64_t* __restrict__ buckets,
                                                       uint32_t* __restrict__ long_list,
                                                       uint32_t* __restrict__ long_count) {
    using F = typename Grp<G>::F;
    constexpr int JW = Grp<G>::JW;
    const size_t b = b0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= b1) return;
    const uint32_t s = start[b], e = end[b];
    if (s == e) {
        Jac<F> z;
        jac_zero(z);
        store_jac(buckets + (size_t)JW * b, z);
        return;
    }
    const size_t first = s / T, last = (e - 1) / T;
    if (first == last) return;
    if (long_list && last - first > kMsmLongSpan) {   // k_msm_long_fix folds it, a block per bucket
        long_list[atomicAdd(long_count, 1u)] = (uint32_t)b;
        return;
    }
    if constexpr (G == 1) {  // lazy core, same formulas and values
        FlJac acc = fl_load_jac(buckets + (size_t)JW * b);
#pragma unroll 1
        for (size_t k = first + 1; k <= last; k++) fl_jac_add(acc, fl_load_jac(cont + (size_t)JW * k));
        fl_store_jac(buckets + (size_t)JW * b, acc);
        return;
    } else if constexpr (LAZY) {
        FlJac2 acc = fl2_load_jac(buckets + (size_t)JW * b);
#pragma unroll 1
        for (size_t k = first + 1; k <= last; k++) fl2_jac_add(acc, fl2_load_jac(cont + (size_t)JW * k));
        fl2_store_jac(buckets + (size_t)JW * b, acc);
        return;
    }
    Jac<F> acc;
    load_jac(acc, buckets + (size_t)JW * b);
#pragma unroll 1
    for (size_t k = first + 1; k <= last; k++) {
        Jac<F> x;
        load_jac(x, cont + (size_t)JW * k);
        jac_add(acc, x);
    }
    store_jac(buckets + (size_t)JW * b, acc);
}

// One lane per segment of L buckets of one window: sum_m m * B_m over the segment.
template <int G>
__global__ void __launch_bounds__(64) k_msm_segments(const uint64_t* __restrict__ buckets, uint32_t B, uint32_t L,
                                                     size_t t0, size_t t1, uint64_t* __restrict__ segs) {
    using F = typename Grp<G>::F;
    constexpr int JW = Grp<G>::JW;
    const size_t t = t0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= t1) return;
    const uint32_t spw = B / L;
    const size_t w = t / spw;
    const uint32_t j = (uint32_t)(t % spw);
    const uint64_t* bw = buckets + (size_t)JW * (w * B);
    Jac<F> T, S;
    jac_zero(T);
    jac_zero(S);
#pragma unroll 1
    for (uint32_t m = (j + 1) * L; m > j * L; m--) {  // magnitudes (j*L, (j+1)*L], top down
        Jac<F> bk;
        load_jac(bk, bw + (size_t)JW * (m - 1));
        jac_add(T, bk);
        jac_add(S, T);
    }
    const uint32_t a = j * L;  // S = sum (m - a) B_m; add a * T
    if (a && !jac_is_zero(T)) {
        Jac<F> aT;
        jac_zero(aT);
#pragma unroll 1
        for (int bit = 31; bit >= 0; bit--) {
            jac_double(aT);
            if ((a >> bit) & 1) jac_add(aT, T);
        }
        jac_add(S, aT);
    }
    store_jac(segs + (size_t)JW * t, S);
}

// out[w*stride + g] = sum_{k<G} in[w*stride + g*G + k]  (indices < count), windows
// [w0, w1); the fixed per-window stride keeps the window parts' levels apart
template <int G>
__global__ void __launch_bounds__(64) k_msm_group_sum(const uint64_t* __restrict__ in, uint32_t count,
                                                      uint32_t group, uint32_t gpw, uint32_t w0, uint32_t w1,
                                                      uint32_t stride, uint64_t* __restrict__ out) {
    using F = typename Grp<G>::F;
    constexpr int JW = Grp<G>::JW;
    const size_t t = (size_t)w0 * gpw + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)w1 * gpw) return;
    const size_t w = t / gpw;
    const uint32_t g = (uint32_t)(t % gpw);
    Jac<F> acc;
    jac_zero(acc);
#pragma unroll 1
    for (uint32_t k = 0; k < group; k++) {
        const uint32_t idx = g * group + k;
        if (idx >= count) break;
        Jac<F> x;
        load_jac(x, in + (size_t)JW * (w * stride + idx));
        jac_add(acc, x);
    }
    store_jac(out + (size_t)JW * (w * stride + g), acc);
}

// k_msm_group_sum<1> on the lazy core, one quad per output (fl_jac_add_q)
__global__ void __launch_bounds__(64) k_msm_group_sum_fl(const uint64_t* __restrict__ in, uint32_t count,
                                                         uint32_t group, uint32_t gpw, uint32_t w0, uint32_t w1,
                                                         uint32_t stride, uint64_t* __restrict__ out) {
    constexpr int JW = Grp<1>::JW;
    const size_t t = (size_t)w0 * gpw + (((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2);
    const int q = threadIdx.x & 3;
    if (t >= (size_t)w1 * gpw) return;
    const size_t w = t / gpw;
    const uint32_t g = (uint32_t)(t % gpw);
    FlJac acc;
    acc.x = fl_zero();
    acc.y = fl_one();
    acc.z = fl_zero();
#pragma unroll 1
    for (uint32_t k = 0; k < group; k++) {
        const uint32_t idx = g * group + k;
        if (idx >= count) break;
        fl_jac_add_q(acc, fl_load_jac(in + (size_t)JW * (w * stride + idx)), q);
    }
    if (q == 0) fl_store_jac(out + (size_t)JW * (w * stride + g), acc);
}

template <int G>
__global__ void __launch_bounds__(64) k_msm_horner(const uint64_t* __restrict__ wsum, uint32_t stride, uint32_t W,
                                                   uint32_t c, uint64_t* __restrict__ out) {
    using F = typename Grp<G>::F;
    constexpr int JW = Grp<G>::JW;
    // one wave; the doublings use three lanes (jac_double_3lane), every lane
    // holds the same accumulator
    if (blockIdx.x != 0) return;
    const int lane = threadIdx.x;
    Jac<F> acc;
    load_jac(acc, wsum + (size_t)JW * stride * (W - 1));
#pragma unroll 1
    for (int w = (int)W - 2; w >= 0; w--) {
#pragma unroll 1
        for (uint32_t k = 0; k < c; k++) jac_double_3lane(acc, lane);
        Jac<F> x;
        load_jac(x, wsum + (size_t)JW * stride * w);
        jac_add(acc, x);
    }
    if (lane == 0) store_jac(out, acc);
}

// G1 Horner entirely on the lazy core: doublings over three lanes
// (fl_jac_double_3lane), window sums added with fl_jac_add.  #E(Fq) is odd,
// so a nonzero accumulator never doubles to zero and a zero one is skipped.
__global__ void __launch_bounds__(64) k_msm_horner_fl(const uint64_t* __restrict__ wsum, uint32_t stride, uint32_t W,
                                                      uint32_t c, uint64_t* __restrict__ out) {
    constexpr int JW = Grp<1>::JW;
    if (blockIdx.x != 0) return;
    const int lane = threadIdx.x;
    FlJac acc = fl_load_jac(wsum + (size_t)JW * stride * (W - 1));
#pragma unroll 1
    for (int w = (int)W - 2; w >= 0; w--) {
        if (!fl_is_zero(acc.z)) {
#pragma unroll 1
            for (uint32_t k = 0; k < c; k++) fl_jac_double_3lane(acc, lane);
        }
        fl_jac_add(acc, fl_load_jac(wsum + (size_t)JW * stride * w));
    }
    if (lane == 0) fl_store_jac(out, acc);
}

// Horner on a group of lane quads (dec_quad.h; G1: 4 quads, G2: 8 quads): each
// doubling is three levels of side-by-side products (one per quad, G2 one
// Fq2 coordinate per quad) instead of the three-lane doubling's chain, and a
// quad product is ~2.5x shorter than a one-lane leaf: the 256 doublings of the
// top window are the MSM's longest dependent chain.  Same sum as a point.
PA_DEV void load_jac_q(dq::Jq<dq::Q>& r, const uint64_t* p, const dq::Lc& l) {
    Fq x, y, z;
    fq_load(x, p);
    fq_load(y, p + 6);
    fq_load(z, p + 12);
    r = {dq::from_abi(x, l), dq::from_abi(y, l), dq::from_abi(z, l)};
}
PA_DEV void load_jac_q(dq::Jq<dq::Q2>& r, const uint64_t* p, const dq::Lc& l) {
    Fq v[6];
#pragma unroll
    for (int k = 0; k < 6; k++) fq_load(v[k], p + 6 * k);
    r.x = {dq::from_abi(v[0], l), dq::from_abi(v[1], l)};
    r.y = {dq::from_abi(v[2], l), dq::from_abi(v[3], l)};
    r.z = {dq::from_abi(v[4], l), dq::from_abi(v[5], l)};
}
PA_DEV void store_jac_q(uint64_t* p, const dq::Jq<dq::Q>& a, bool lead) {
    const Fq x = dq::to_abi(a.x), y = dq::to_abi(a.y), z = dq::to_abi(a.z);
    if (lead) {
        fq_store(p, x);
        fq_store(p + 6, y);
        fq_store(p + 12, z);
    }
}
PA_DEV void store_jac_q(uint64_t* p, const dq::Jq<dq::Q2>& a, bool lead) {
    const Fq v[6] = {dq::to_abi(a.x.c0), dq::to_abi(a.x.c1), dq::to_abi(a.y.c0),
                     dq::to_abi(a.y.c1), dq::to_abi(a.z.c0), dq::to_abi(a.z.c1)};
    if (lead)
#pragma unroll
        for (int k = 0; k < 6; k++) fq_store(p + 6 * k, v[k]);
}
// Windows [wlo, whi) top down: from acc_in (the part above, doubled c times
// first) or, without one, from S_(whi-1).
template <int G>
__global__ void __launch_bounds__(64) k_msm_horner_q(const uint64_t* __restrict__ wsum, uint32_t stride, int whi,
                                                     int wlo, uint32_t c, const uint64_t* __restrict__ acc_in,
                                                     uint64_t* __restrict__ out) {
    constexpr int NQ = G == 1 ? 4 : 8;
    constexpr int JW = Grp<G>::JW;
    using E = typename std::conditional<G == 1, dq::Jq<dq::Q>, dq::Jq<dq::Q2>>::type;
    const int lane = threadIdx.x;
    if (blockIdx.x != 0 || lane >= 4 * NQ) return;   // one group
    const dq::Lc l = dq::lctx(lane, NQ);
    E acc;
    int w = whi - 1;
    if (acc_in) {
        load_jac_q(acc, acc_in, l);
    } else {
        load_jac_q(acc, wsum + (size_t)JW * stride * w, l);
        w--;
    }
#pragma unroll 1
    for (; w >= wlo; w--) {
        if (!dq::is_zero(acc.z)) {
#pragma unroll 1
            for (uint32_t k = 0; k < c; k++) dq::jdbl<NQ>(acc, l);
        }
        E x;
        load_jac_q(x, wsum + (size_t)JW * stride * w, l);
        if (!dq::is_zero(x.z)) dq::jadd<NQ>(acc, dq::make_fixed<NQ>(x, l), l);
    }
    store_jac_q(out, acc, lane == 0);
}

// k_msm_segments<1> on the lazy core (same sums, same formulas)
__global__ void __launch_bounds__(64) k_msm_segments_fl(const uint64_t* __restrict__ buckets, uint32_t B, uint32_t L,
                                                        size_t t0, size_t t1, uint64_t* __restrict__ segs) {
    // one lane per segment: the kernel is throughput bound (4 k waves); a quad
    // per segment (fl_jac_add_q) measured 0.57 -> 1.29 ms (profiles/r03_msm_quad_ab.txt)
    constexpr int JW = Grp<1>::JW;
    const size_t t = t0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= t1) return;
    const uint32_t spw = B / L;
    const size_t w = t / spw;
    const uint32_t j = (uint32_t)(t % spw);
    const uint64_t* bw = buckets + (size_t)JW * (w * B);
    FlJac T, S;
    T.x = fl_zero();
    T.y = fl_one();
    T.z = fl_zero();
    S = T;
#pragma unroll 1
    for (uint32_t m = (j + 1) * L; m > j * L; m--) {  // magnitudes (j*L, (j+1)*L], top down
        fl_jac_add(T, fl_load_jac(bw + (size_t)JW * (m - 1)));
        fl_jac_add(S, T);
    }
    const uint32_t a = j * L;  // S = sum (m - a) B_m; add a * T
    if (a && !fl_is_zero(T.z)) {
        FlJac aT = T;  // top set bit of a
        const int top = 31 - __clz(a);
#pragma unroll 1
        for (int bit = top - 1; bit >= 0; bit--) {
            fl_jac_double(aT);
            if ((a >> bit) & 1) fl_jac_add(aT, T);
        }
        fl_jac_add(S, aT);
    }
    fl_store_jac(segs + (size_t)JW * t, S);
}


// ---- G2 bucket phases on the lazy core's Fq2 (curve_fl2.h; round 4) ----
// The affine bases converted once per MSM (x.c0, x.c1, y.c0, y.c1 -> 56 u32;
// the infinity flag in bit 31 of x.c0's top limb, below 2^18 for F<1>) ...
__global__ void __launch_bounds__(256) k_msm_bases_fl2(const uint64_t* __restrict__ bases, size_t n,
                                                       uint32_t* __restrict__ fl) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Aff<Fq2> a;
    load_aff(a, bases + (size_t)Grp<2>::AW * i);
    const F<1> v[4] = {fl_from_abi(a.x.c0), fl_from_abi(a.x.c1), fl_from_abi(a.y.c0), fl_from_abi(a.y.c1)};
    uint32_t* d = fl + 56 * i;
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int k = 0; k < 14; k++) d[14 * c + k] = v[c].w[k] | (c == 0 && k == 13 && a.inf ? 0x80000000u : 0u);
}

PA_DEV void msm_flush_fl2(uint32_t key, const FlJac2& acc, bool untouched, size_t j0, size_t k,
                          const uint32_t* __restrict__ start, uint64_t* __restrict__ buckets,
                          uint64_t* __restrict__ cont) {
    constexpr int JW = Grp<2>::JW;
    uint64_t* o = start[key] >= j0 ? buckets + (size_t)JW * key : cont + (size_t)JW * k;
    if (untouched) {
        Jac<Fq2> z;
        jac_zero(z);
        store_jac(o, z);
    } else {
        fl2_store_jac(o, acc);
    }
}

// ... k_msm_chunk_acc<2> with the lazy mixed addition; the (key, value) pair
// of the next item in flight while the current addition runs (a prefetched
// 224-byte base would not fit beside the Fq2 temporaries)
__global__ void __launch_bounds__(64) k_msm_chunk_acc_fl2(const uint32_t* __restrict__ basefl,
                                                          const uint32_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ vals,
                                                          const uint32_t* __restrict__ start,
                                                          const uint32_t* __restrict__ wtot, uint32_t w0, uint32_t w1,
                                                          uint32_t T, uint32_t sentinel,
                                                          uint64_t* __restrict__ buckets, uint64_t* __restrict__ cont) {
    size_t k, j0, j1;
    if (!chunk_range((size_t)blockIdx.x * blockDim.x + threadIdx.x, wtot, w0, w1, T, k, j0, j1)) return;
    uint32_t cur = keys[j0];
    if (cur >= sentinel) return;
    FlJac2 acc = fl2_jac_zero();
    bool untouched = true;
    uint32_t key = cur, v = vals[j0];
#pragma unroll 1
    for (size_t j = j0; j < j1; j++) {
        if (key >= sentinel) break;
        uint32_t nkey = sentinel, nv = 0;
        if (j + 1 < j1) {
            nkey = keys[j + 1];
            nv = vals[j + 1];
        }
        if (key != cur) {
            msm_flush_fl2(cur, acc, untouched, j0, k, start, buckets, cont);
            untouched = true;
            cur = key;
        }
        const uint2* src = reinterpret_cast<const uint2*>(basefl + 56 * (size_t)(v & 0x7fffffffu));
        F<1> c[4];
#pragma unroll
        for (int q = 0; q < 28; q++) {
            const uint2 t = src[q];
            c[q / 7].w[2 * (q % 7)] = t.x;
            c[q / 7].w[2 * (q % 7) + 1] = t.y;
        }
        const bool inf = (c[0].w[13] >> 31) != 0;
        c[0].w[13] &= 0x7fffffffu;
        if (!inf) {  // an infinity base is add_assign_mixed's no-op
            const F2<1> y = {c[2], c[3]};
            const F2<2> oy = (v >> 31) ? neg(y) : relax<2>(y);
            fl2_jac_add_mixed(acc, untouched, F2<1>{c[0], c[1]}, oy);
        }
        key = nkey;
        v = nv;
    }
    msm_flush_fl2(cur, acc, untouched, j0, k, start, buckets, cont);
}

// k_msm_segments<2> on the lazy core (same sums, same formulas)
__global__ void __launch_bounds__(64) k_msm_segments_fl2(const uint64_t* __restrict__ buckets, uint32_t B, uint32_t L,
                                                         size_t t0, size_t t1, uint64_t* __restrict__ segs) {
    constexpr int JW = Grp<2>::JW;
    const size_t t = t0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= t1) return;
    const uint32_t spw = B / L;
    const size_t w = t / spw;
    const uint32_t j = (uint32_t)(t % spw);
    const uint64_t* bw = buckets + (size_t)JW * (w * B);
    FlJac2 T = fl2_jac_zero(), S = T;
#pragma unroll 1
    for (uint32_t m = (j + 1) * L; m > j * L; m--) {  // magnitudes (j*L, (j+1)*L], top down
        fl2_jac_add(T, fl2_load_jac(bw + (size_t)JW * (m - 1)));
        fl2_jac_add(S, T);
    }
    const uint32_t a = j * L;  // S = sum (m - a) B_m; add a * T
    if (a && !f2_is_zero(T.z)) {
        FlJac2 aT = T;  // top set bit of a
        const int top = 31 - __clz(a);
#pragma unroll 1
        for (int bit = top - 1; bit >= 0; bit--) {
            fl2_jac_double(aT);
            if ((a >> bit) & 1) fl2_jac_add(aT, T);
        }
        fl2_jac_add(S, aT);
    }
    fl2_store_jac(segs + (size_t)JW * t, S);
}

// k_msm_group_sum<2> on the lazy core, one lane per output
__global__ void __launch_bounds__(64) k_msm_group_sum_fl2(const uint64_t* __restrict__ in, uint32_t count,
                                                          uint32_t group, uint32_t gpw, uint32_t w0, uint32_t w1,
                                                          uint32_t stride, uint64_t* __restrict__ out) {
    constexpr int JW = Grp<2>::JW;
    const size_t t = (size_t)w0 * gpw + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)w1 * gpw) return;
    const size_t w = t / gpw;
    const uint32_t g = (uint32_t)(t % gpw);
    FlJac2 acc = fl2_jac_zero();
#pragma unroll 1
    for (uint32_t k = 0; k < group; k++) {
        const uint32_t idx = g * group + k;
        if (idx >= count) break;
        fl2_jac_add(acc, fl2_load_jac(in + (size_t)JW * (w * stride + idx)));
    }
    fl2_store_jac(out + (size_t)JW * (w * stride + g), acc);
}

// Buckets spanning more than kMsmLongSpan chunks (crowded digits: equal
// scalars, the carry-only top window of c-bit windows above bit 255): one
// block per bucket, each thread summing a strided share of the continuation
// pieces, then a tree through LDS; the bucket's own piece is added last.  The
// list comes from k_msm_bucket_fix; without long buckets the blocks exit at
// once.  Without it one lane walked every piece (G2 at 2^18: 46 ms).
template <int G> struct LazyJac;
template <> struct LazyJac<1> {
    using P = FlJac;
    static constexpr int NT = 256;
    static PA_DEV P zero() { return {fl_zero(), fl_one(), fl_zero()}; }
    static PA_DEV void add(P& a, const P& b) { fl_jac_add(a, b); }
    static PA_DEV P load(const uint64_t* p) { return fl_load_jac(p); }
    static PA_DEV void store(uint64_t* p, const P& a) { fl_store_jac(p, a); }
};
template <> struct LazyJac<2> {
    using P = FlJac2;
    static constexpr int NT = 128;
    static PA_DEV P zero() { return fl2_jac_zero(); }
    static PA_DEV void add(P& a, const P& b) { fl2_jac_add(a, b); }
    static PA_DEV P load(const uint64_t* p) { return fl2_load_jac(p); }
    static PA_DEV void store(uint64_t* p, const P& a) { fl2_store_jac(p, a); }
};
template <int G>
__global__ void __launch_bounds__(LazyJac<G>::NT) k_msm_long_fix(const uint32_t* __restrict__ start,
                                                                 const uint32_t* __restrict__ end, uint32_t T,
                                                                 const uint64_t* __restrict__ cont,
                                                                 uint64_t* __restrict__ buckets,
                                                                 const uint32_t* __restrict__ long_list,
                                                                 const uint32_t* __restrict__ long_count) {
    using L = LazyJac<G>;
    using P = typename L::P;
    constexpr int NT = L::NT, JW = Grp<G>::JW, PW = sizeof(P) / 4;
    __shared__ uint32_t sh[(NT / 2) * PW];
    const int t = threadIdx.x;
    const uint32_t count = *long_count;
#pragma unroll 1
    for (uint32_t idx = blockIdx.x; idx < count; idx += gridDim.x) {
        const uint32_t b = long_list[idx];
        const size_t first = start[b] / T, last = (end[b] - 1) / T;
        P acc = L::zero();
#pragma unroll 1
        for (size_t k = first + 1 + t; k <= last; k += NT) L::add(acc, L::load(cont + (size_t)JW * k));
#pragma unroll 1
        for (int h = NT / 2; h >= 1; h >>= 1) {
            if (t >= h && t < 2 * h) {
                const uint32_t* src = reinterpret_cast<const uint32_t*>(&acc);
#pragma unroll
                for (int q = 0; q < PW; q++) sh[(t - h) * PW + q] = src[q];
            }
            __syncthreads();
            if (t < h) {
                P o;
                uint32_t* dst = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
                for (int q = 0; q < PW; q++) dst[q] = sh[t * PW + q];
                L::add(acc, o);
            }
            __syncthreads();
        }
        if (t == 0) {
            P bk = L::load(buckets + (size_t)JW * b);
            L::add(bk, acc);
            L::store(buckets + (size_t)JW * b, bk);
        }
    }
}

template <int G>
__global__ void __launch_bounds__(64) k_jac_zero_out(uint64_t* __restrict__ out) {
    using F = typename Grp<G>::F;
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    Jac<F> z;
    jac_zero(z);
    store_jac(out, z);
}

static inline unsigned msm_blocks(size_t n, unsigned bs) { return (unsigned)((n + bs - 1) / bs); }

size_t msm_workspace_bytes(int group, size_t n) {
    if (n == 0) return 0;
    MsmPlan p;
    if (msm_plan(p, group, n) != hipSuccess) return 0;
    return p.total;
}

// two non-blocking side streams per device (bucket reduction, Horner legs),
// created on the device of the caller's stream.  They are shared by every
// caller on that device, so MSMs issued concurrently from several host threads
// serialize their window-part tails through them (results are unaffected: each
// call orders its own work with events).
static hipError_t msm_side_streams(hipStream_t caller, hipStream_t out[2]) {
    int dev = 0;
    hipError_t e = hipStreamGetDevice(caller, &dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    static std::mutex mu;
    static hipStream_t side[64][2] = {};
    std::lock_guard<std::mutex> g(mu);
    // the side streams at the highest priority: a part's reduction waves are
    // dispatched as the next part's accumulation frees SIMDs (PA_MSM_PRIO=0: default priority)
    static const bool prio = !getenv("PA_MSM_PRIO") || atoi(getenv("PA_MSM_PRIO")) != 0;
    int lo = 0, hi = 0;
    if (prio && (e = hipDeviceGetStreamPriorityRange(&lo, &hi)) != hipSuccess) return e;
    if (!side[dev][0] || !side[dev][1]) {
        // streams belong to the current device: create them on the caller's
        int cur = 0;
        if ((e = hipGetDevice(&cur)) != hipSuccess) return e;
        if (cur != dev && (e = hipSetDevice(dev)) != hipSuccess) return e;
        for (int k = 0; k < 2 && e == hipSuccess; k++)
            if (!side[dev][k]) e = hipStreamCreateWithPriority(&side[dev][k], hipStreamNonBlocking, prio ? hi : lo);
        if (cur != dev) (void)hipSetDevice(cur);
        if (e != hipSuccess) return e;
    }
    out[0] = side[dev][0];
    out[1] = side[dev][1];
    return hipSuccess;
}

template <int G>
static hipError_t msm_run(const uint64_t* bases, const uint64_t* scalars, size_t n, uint64_t* out, void* ws,
                          size_t ws_bytes, hipStream_t s) {
    constexpr int JW = Grp<G>::JW;
    if (n == 0) {
        hipLaunchKernelGGL(k_jac_zero_out<G>, dim3(1), dim3(64), 0, s, out);
        return hipGetLastError();
    }
    MsmPlan p;
    hipError_t e = msm_plan(p, G, n);
    if (e != hipSuccess) return e;
    if (ws_bytes < p.total || !ws) return hipErrorInvalidValue;
    if (p.items > 0xffffffffull) return hipErrorInvalidValue;  // 32-bit item positions
    char* base = static_cast<char*>(ws);
    uint32_t* keys_in = reinterpret_cast<uint32_t*>(base + p.off_keys_in);
    uint32_t* keys_out = reinterpret_cast<uint32_t*>(base + p.off_keys_out);
    uint32_t* vals_in = reinterpret_cast<uint32_t*>(base + p.off_vals_in);
    uint32_t* vals_out = reinterpret_cast<uint32_t*>(base + p.off_vals_out);
    uint32_t* start = reinterpret_cast<uint32_t*>(base + p.off_start);
    uint32_t* end = reinterpret_cast<uint32_t*>(base + p.off_end);
    uint64_t* buckets = reinterpret_cast<uint64_t*>(base + p.off_buckets);
    uint64_t* segs = reinterpret_cast<uint64_t*>(base + p.off_segs);
    uint64_t* tmp = reinterpret_cast<uint64_t*>(base + p.off_tmp);
    const size_t nb = (size_t)p.W * p.B;

    hipLaunchKernelGGL(k_msm_digits, dim3(msm_blocks(n, 256)), dim3(256), 0, s, scalars, n, p.c, p.W, p.B, keys_in,
                       vals_in);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // the bucketing sort: ping-pong between the _in and _out arrays; the last
    // destination's tail past the nonzero items is set to sentinel keys first
    uint32_t* hist = reinterpret_cast<uint32_t*>(base + p.off_hist);
    uint32_t* wtot = reinterpret_cast<uint32_t*>(base + p.off_wtot);
    uint32_t *ksrc = keys_in, *vsrc = vals_in, *kdst = keys_out, *vdst = vals_out;
    const unsigned tiles = p.W * p.tpw;
    for (uint32_t pass = 0; pass < p.passes; pass++) {
        const SortPass sp{8 * pass, p.B - 1, p.W * p.B, p.tpw, pass == 0 ? 1u : 0u, n};
        hipLaunchKernelGGL(k_sort_hist, dim3(tiles), dim3(256), 0, s, ksrc, wtot, sp, hist);
        hipLaunchKernelGGL(k_sort_scan, dim3(p.W), dim3(1024), 0, s, hist, p.tpw, wtot);
        if (pass + 1 == p.passes && (e = hipMemsetAsync(kdst, 0xff, 4 * p.items, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_sort_scatter, dim3(tiles), dim3(256), 0, s, ksrc, vsrc, hist, wtot, sp, kdst, vdst);
        std::swap(ksrc, kdst);
        std::swap(vsrc, vdst);
    }
    keys_out = ksrc;  // the last pass's output
    vals_out = vsrc;
    if ((e = hipMemsetAsync(start, 0, 4 * nb, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(end, 0, 4 * nb, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_msm_bucket_bounds, dim3(msm_blocks(p.items, 256)), dim3(256), 0, s, keys_out, p.items,
                       p.W * p.B, start, end);
    uint64_t* cont = reinterpret_cast<uint64_t*>(base + p.off_cont);
    uint64_t* hacc = reinterpret_cast<uint64_t*>(base + p.off_hacc);
    const uint32_t* basefl = reinterpret_cast<const uint32_t*>(base + p.off_basefl);
    // G2 on the lazy core's Fq2 (round 4); PA_MSM_G2_LAZY=0: the 12-word kernels (A/B)
    static const bool g2_lazy_env = !getenv("PA_MSM_G2_LAZY") || atoi(getenv("PA_MSM_G2_LAZY")) != 0;
    const bool g2_lazy = G == 2 && g2_lazy_env;
    if constexpr (G == 1)
        hipLaunchKernelGGL(k_msm_bases_fl, dim3(msm_blocks(n, 256)), dim3(256), 0, s, bases, n,
                           reinterpret_cast<uint32_t*>(base + p.off_basefl));
    else if (g2_lazy)
        hipLaunchKernelGGL(k_msm_bases_fl2, dim3(msm_blocks(n, 256)), dim3(256), 0, s, bases, n,
                           reinterpret_cast<uint32_t*>(base + p.off_basefl));
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint32_t spw = p.B / p.L;
    // segment sums -> one per window, `group` at a time (ping-pong segs <-> tmp);
    // every part takes the same number of levels, so the window sums of all of
    // them land in the same buffer
    // shallow chains: 2 additions per level, 2 / 3 / 4 / 8 measured 141.6 / 140.2 / 138.1 / 133.5 M
    // terms/s at 2^20 (profiles/r02_msm_tuning.txt); PA_MSM_GROUP to A/B
    static const uint32_t group = [] {
        const char* v = getenv("PA_MSM_GROUP");
        const int g = v ? atoi(v) : 2;
        return (uint32_t)(g < 2 ? 2 : (g > 16 ? 16 : g));
    }();
    uint64_t* wsum = segs;
    for (uint32_t count = spw; count > 1; count = (count + group - 1) / group) wsum = wsum == segs ? tmp : segs;

    // the windows' throughput kernels of one part (windows [w0, w1))
    // (the part's item range is on the device, wtot: lanes for the most it can hold)
    // the G1 bucket accumulation's kernel: PA_MSM_ACC=0 one wave per SIMD with
    // the base prefetch, 1 two waves without it, 2 two waves with it (A/B)
    static const int acc_kind = [] {
        const char* e = getenv("PA_MSM_ACC");
        return e ? atoi(e) : 0;
    }();
    auto accumulate = [&](uint32_t w0, uint32_t w1, hipStream_t st) {
        const size_t chunks = ((size_t)(w1 - w0) * n + p.T - 1) / p.T + 1;
        if constexpr (G == 1)
            hipLaunchKernelGGL(acc_kind == 1 ? k_msm_chunk_acc_fl_2w
                                             : (acc_kind == 2 ? k_msm_chunk_acc_fl_2wp : k_msm_chunk_acc_fl),
                               dim3(msm_blocks(chunks, 64)), dim3(64), 0, st, basefl, keys_out, vals_out, start, wtot,
                               w0, w1, p.T, p.W * p.B, buckets, cont);
        else if (g2_lazy)
            hipLaunchKernelGGL(k_msm_chunk_acc_fl2, dim3(msm_blocks(chunks, 64)), dim3(64), 0, st, basefl, keys_out,
                               vals_out, start, wtot, w0, w1, p.T, p.W * p.B, buckets, cont);
        else
            hipLaunchKernelGGL(k_msm_chunk_acc<G>, dim3(msm_blocks(chunks, 64)), dim3(64), 0, st, bases, keys_out,
                               vals_out, start, wtot, w0, w1, p.T, p.W * p.B, buckets, cont);
        return hipGetLastError();
    };
    // ... and its bucket -> window-sum reduction
    // (part q: long-bucket list at long_list + b0, its count at long_count[q])
    uint32_t* long_list = reinterpret_cast<uint32_t*>(base + p.off_long);
    uint32_t* long_count = long_list + nb;
    const bool lazy = G == 1 || g2_lazy;
    // segment sums -> one per window, `group` at a time, windows [w0, w1)
    auto group_levels = [&](uint32_t w0, uint32_t w1, hipStream_t st) {
        uint64_t *src = segs, *dst = tmp;
        for (uint32_t count = spw; count > 1;) {
            const uint32_t gpw = (count + group - 1) / group;
            const size_t outs = (size_t)(w1 - w0) * gpw;
            if constexpr (G == 1)
                hipLaunchKernelGGL(k_msm_group_sum_fl, dim3(msm_blocks(4 * outs, 64)), dim3(64), 0, st, src, count,
                                   group, gpw, w0, w1, spw, dst);
            else if (g2_lazy)
                hipLaunchKernelGGL(k_msm_group_sum_fl2, dim3(msm_blocks(outs, 64)), dim3(64), 0, st, src, count,
                                   group, gpw, w0, w1, spw, dst);
            else
                hipLaunchKernelGGL(k_msm_group_sum<G>, dim3(msm_blocks(outs, 64)), dim3(64), 0, st, src, count, group,
                                   gpw, w0, w1, spw, dst);
            count = gpw;
            std::swap(src, dst);
        }
        return hipGetLastError();
    };
    auto reduce = [&](uint32_t w0, uint32_t w1, uint32_t q, hipStream_t st) {
        const size_t b0 = (size_t)w0 * p.B, b1 = (size_t)w1 * p.B;
        hipError_t r;
        if (lazy && (r = hipMemsetAsync(long_count + q, 0, 4, st)) != hipSuccess) return r;
        if (lazy)
            hipLaunchKernelGGL((k_msm_bucket_fix<G, true>), dim3(msm_blocks(b1 - b0, 64)), dim3(64), 0, st, start, end,
                               b0, b1, p.T, cont, buckets, long_list + b0, long_count + q);
        else
            hipLaunchKernelGGL((k_msm_bucket_fix<G, false>), dim3(msm_blocks(b1 - b0, 64)), dim3(64), 0, st, start,
                               end, b0, b1, p.T, cont, buckets, nullptr, long_count + q);
        if (lazy)
            hipLaunchKernelGGL(k_msm_long_fix<G>, dim3(kMsmLongBlocks), dim3(LazyJac<G>::NT), 0, st, start, end, p.T,
                               cont, buckets, long_list + b0, long_count + q);
        const size_t t0 = (size_t)w0 * spw, t1 = (size_t)w1 * spw;
        if constexpr (G == 1)
            hipLaunchKernelGGL(k_msm_segments_fl, dim3(msm_blocks(t1 - t0, 64)), dim3(64), 0, st, buckets, p.B, p.L,
                               t0, t1, segs);
        else if (g2_lazy)
            hipLaunchKernelGGL(k_msm_segments_fl2, dim3(msm_blocks(t1 - t0, 64)), dim3(64), 0, st, buckets, p.B,
                               p.L, t0, t1, segs);
        else
            hipLaunchKernelGGL(k_msm_segments<G>, dim3(msm_blocks(t1 - t0, 64)), dim3(64), 0, st, buckets, p.B, p.L,
                               t0, t1, segs);
        return group_levels(w0, w1, st);
    };

    // the round-3 one-wave Horner kernels (PA_MSM_HORNER=1: three-lane
    // doublings, G1 on the lazy core) run the whole MSM as one part
    static const bool horner_wave = getenv("PA_MSM_HORNER") && atoi(getenv("PA_MSM_HORNER")) == 1;
    const uint32_t parts = horner_wave ? 1 : msm_parts(p.W);
    if (parts == 1) {
        if ((e = accumulate(0, p.W, s)) != hipSuccess || (e = reduce(0, p.W, 0, s)) != hipSuccess) return e;
        if (!horner_wave)
            hipLaunchKernelGGL(k_msm_horner_q<G>, dim3(1), dim3(64), 0, s, wsum, spw, (int)p.W, 0, p.c, nullptr, out);
        else if constexpr (G == 1)
            hipLaunchKernelGGL(k_msm_horner_fl, dim3(1), dim3(64), 0, s, wsum, spw, p.W, p.c, out);
        else
            hipLaunchKernelGGL(k_msm_horner<G>, dim3(1), dim3(64), 0, s, wsum, spw, p.W, p.c, out);
        return hipGetLastError();
    }
    // Window parts, top windows first.  The caller's stream runs every part's
    // bucket accumulation back to back; part q's reduction runs on a side
    // stream behind it and its Horner leg (windows [w0, w1), continuing the
    // part above) on a third, so the latency-bound tails (segment-sum levels,
    // the 16 doublings per window of the Horner chain) of the upper parts
    // hide under the next parts' accumulation.  Only the last part's reduction
    // and Horner leg are exposed.  Same window sums, same Horner: same point.
    hipStream_t side[2];
    if ((e = msm_side_streams(s, side)) != hipSuccess) return e;
    hipStream_t red_s = side[0], hor_s = side[1];
    static const bool serial = getenv("PA_MSM_SERIAL") && atoi(getenv("PA_MSM_SERIAL")) != 0;
    if (serial) red_s = hor_s = s;   // measurement / debugging: the parts in order on the caller's stream
    hipEvent_t ev[2 * kMsmMaxParts + 1] = {};
    int made = 0;
    hipError_t err = hipSuccess;
    auto ck = [&](hipError_t x) {
        if (err == hipSuccess) err = x;
        return err == hipSuccess;
    };
    const int nev = 2 * (int)parts + 1;
    for (; made < nev; made++)
        if (!ck(hipEventCreateWithFlags(&ev[made], hipEventDisableTiming))) break;
    // ev[2q]: part q accumulated; ev[2q + 1]: part q reduced; ev[2 parts]: the upper Horner legs done
    // part q covers windows [wlo(q), wlo(q - 1)); PA_MSM_WLO="b0,b1,..." (descending
    // lower bounds, A/B of unequal parts) overrides the even split
    static const std::vector<uint32_t> wlo_env = [] {
        std::vector<uint32_t> v;
        if (const char* e = getenv("PA_MSM_WLO"))
            for (const char* c = e; *c;) {
                v.push_back((uint32_t)strtoul(c, const_cast<char**>(&c), 10));
                if (*c == ',') c++;
                else break;
            }
        return v;
    }();
    // the override is taken whole or not at all: exactly parts - 1 bounds, strictly
    // descending, each in (0, W) -- otherwise windows would be summed twice or skipped
    bool use_env = wlo_env.size() + 1 == parts;
    for (size_t k = 0; use_env && k < wlo_env.size(); k++)
        use_env = wlo_env[k] > 0 && wlo_env[k] < p.W && (k == 0 || wlo_env[k] < wlo_env[k - 1]);
    auto wlo = [&](uint32_t q) {
        if (use_env && q + 1 < parts) return wlo_env[q];
        return q + 1 == parts ? 0u : (uint32_t)(((uint64_t)p.W * (parts - 1 - q)) / parts);
    };
    for (uint32_t q = 0; q < parts && err == hipSuccess; q++) {
        const uint32_t w1 = q == 0 ? p.W : wlo(q - 1), w0 = wlo(q);
        if (!ck(accumulate(w0, w1, s))) break;
        uint64_t* leg_out = q + 1 == parts ? out : hacc + (size_t)JW * q;
        const uint64_t* leg_in = q == 0 ? nullptr : hacc + (size_t)JW * (q - 1);
        if (q + 1 == parts) {
            if (!ck(reduce(w0, w1, q, s)) || !ck(hipStreamWaitEvent(s, ev[2 * parts], 0))) break;
            hipLaunchKernelGGL(k_msm_horner_q<G>, dim3(1), dim3(64), 0, s, wsum, spw, (int)w1, (int)w0, p.c, leg_in,
                               leg_out);
            ck(hipGetLastError());
            break;
        }
        if (!ck(hipEventRecord(ev[2 * q], s)) || !ck(hipStreamWaitEvent(red_s, ev[2 * q], 0)) ||
            !ck(reduce(w0, w1, q, red_s)) || !ck(hipEventRecord(ev[2 * q + 1], red_s)) ||
            !ck(hipStreamWaitEvent(hor_s, ev[2 * q + 1], 0)))
            break;
        hipLaunchKernelGGL(k_msm_horner_q<G>, dim3(1), dim3(64), 0, hor_s, wsum, spw, (int)w1, (int)w0, p.c, leg_in,
                           leg_out);
        if (!ck(hipGetLastError())) break;
        if (q + 2 == parts) ck(hipEventRecord(ev[2 * parts], hor_s));
    }
    if (err != hipSuccess) {
        // a failed launch sequence: let this call's work already queued on the
        // side streams drain before the caller may release the workspace (an
        // event recorded now waits for that work only, not for what other
        // callers queue on the shared side streams later)
        for (hipStream_t x : {red_s, hor_s}) {
            hipEvent_t done = nullptr;
            if (hipEventCreateWithFlags(&done, hipEventDisableTiming) == hipSuccess &&
                hipEventRecord(done, x) == hipSuccess)
                (void)hipEventSynchronize(done);
            else
                (void)hipStreamSynchronize(x);
            if (done) (void)hipEventDestroy(done);
        }
    }
    for (int k = 0; k < made; k++) (void)hipEventDestroy(ev[k]);
    (void)JW;
    return err;
}

hipError_t launch_msm(int group, const uint64_t* bases, const uint64_t* scalars, size_t n, uint64_t* out, void* ws,
                      size_t ws_bytes, hipStream_t stream) {
    if (n >= 0x80000000ull) return hipErrorInvalidValue;
    return group == 1 ? msm_run<1>(bases, scalars, n, out, ws, ws_bytes, stream)
                      : msm_run<2>(bases, scalars, n, out, ws, ws_bytes, stream);
}

hipError_t launch_scalar_mul(int group, int projective, const uint64_t* p, const uint64_t* scalars, size_t n,
                             uint64_t* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 g(msm_blocks(n, 64)), b(64);
    if (group == 1) {
        if (projective) hipLaunchKernelGGL(k_proj_mul<1>, g, b, 0, stream, p, scalars, out, n);
        else hipLaunchKernelGGL(k_affine_mul<1>, g, b, 0, stream, p, scalars, out, n);
    } else {
        if (projective) hipLaunchKernelGGL(k_proj_mul<2>, g, b, 0, stream, p, scalars, out, n);
        else hipLaunchKernelGGL(k_affine_mul<2>, g, b, 0, stream, p, scalars, out, n);
    }
    return hipGetLastError();
}

}  // namespace pa
