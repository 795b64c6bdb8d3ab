// pairing_amd.hpp -- C++17 host mirror of the reference crate's trait surface
// for the BLS12-381 hot path, on top of the C ABI of pairing_amd.h.
//
// The reference (`pairing` v0.14.2, Rust) exposes the path as traits:
//   Engine::{miller_loop, final_exponentiation, pairing}   src/lib.rs:34-110
//   CurveAffine::{prepare, pairing_with, into_compressed, ...} lib.rs:185-234
//   CurveProjective::{double, add_assign, add_assign_mixed, negate,
//     sub_assign, mul_assign, into_affine, batch_normalization,
//     recommended_wnaf_*}                                    lib.rs:114-181
//   EncodedPoint::{into_affine, into_affine_unchecked, from_affine} lib.rs:236-264
//   CurveAffine::{mul, negate, into_projective}             lib.rs:185-234
//   Field / SqrtField::{add_assign, sub_assign, double, negate, mul_assign,
//     square, inverse, frobenius_map, pow, sqrt}            lib.rs:267-345
//     on Fq, Fq2, Fq6, Fq12 (+ Fq12::conjugate)
//   Wnaf::new().base(g, n).scalar(s), Wnaf::new().scalar(s).base(g),
//     shared()                                              wnaf.rs:73-179
// The classes below keep those names, argument meanings and error behaviour
// (Option -> std::optional, Result<_, GroupDecodingError> -> a thrown
// GroupDecodingError), so code written against the crate reads the same.
// Every operation runs on the GPU through the C ABI; batched forms (the point
// of this library) take std::vector and make one ABI call.  A negative ABI
// status throws pairing_amd::Error with pa_last_error().
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "pairing_amd.h"

namespace pairing_amd {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& what) : std::runtime_error(what), code(code) {}
    int code;
};

inline void check(int rc, const char* what) {
    if (rc != PA_OK) throw Error(rc, std::string(what) + ": " + pa_last_error());
}

// ---------------- fields (fq.rs, fq2.rs, fq12.rs) ----------------
namespace detail {
// R = 2^384 mod q, Fq::one() (fq.rs:23-30, 803-805)
constexpr uint64_t kR[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL,
                            0x77ce585370525745ULL, 0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};
template <class T>
bool bytes_equal(const T& a, const T& b) { return std::memcmp(&a, &b, sizeof(T)) == 0; }
template <class T>
bool bytes_zero(const T& a) {
    T z;
    std::memset(&z, 0, sizeof z);
    return bytes_equal(a, z);
}

// Componentwise add / sub / negate of a tower element as a batch of its
// Fq coordinates (each Fq coordinate of Fq2/Fq6/Fq12 adds independently,
// fq2.rs:103-121, fq6.rs:111-155, fq12.rs:50-88).
template <class T>
void fq_add_n(const T& a, const T& b, T& out) {
    check(pa_fq_add_batch(reinterpret_cast<const pa_fq*>(&a), reinterpret_cast<const pa_fq*>(&b),
                          reinterpret_cast<pa_fq*>(&out), sizeof(T) / sizeof(pa_fq)),
          "add_assign");
}
template <class T>
void fq_sub_n(const T& a, const T& b, T& out) {
    check(pa_fq_sub_batch(reinterpret_cast<const pa_fq*>(&a), reinterpret_cast<const pa_fq*>(&b),
                          reinterpret_cast<pa_fq*>(&out), sizeof(T) / sizeof(pa_fq)),
          "sub_assign");
}
// Field::pow (lib.rs:306-324) by square-and-multiply over the trait's own
// square / mul_assign, for the types without a pow entry point
template <class F>
F pow_generic(const F& x, const std::vector<uint64_t>& exp) {
    F r = F::one();
    for (size_t w = exp.size(); w-- > 0;)
        for (int bit = 63; bit >= 0; bit--) {
            r.square();
            if ((exp[w] >> bit) & 1) r.mul_assign(x);
        }
    return r;
}
}  // namespace detail

// The Field trait (lib.rs:267-325) on each type: zero, one, is_zero, square,
// double, negate, add_assign, sub_assign, mul_assign, inverse,
// frobenius_map, pow; SqrtField::sqrt where the reference has it.
#define PA_FIELD_COMMON(T)                                                     \
    bool is_zero() const { return detail::bytes_zero(v); }                     \
    bool operator==(const T& o) const { return detail::bytes_equal(v, o.v); }  \
    bool operator!=(const T& o) const { return !(*this == o); }                \
    void add_assign(const T& o) { detail::fq_add_n(v, o.v, v); }               \
    void sub_assign(const T& o) { detail::fq_sub_n(v, o.v, v); }               \
    void double_() { add_assign(*this); }                                      \
    void negate() {                                                            \
        T z;                                                                   \
        z.sub_assign(*this);                                                   \
        *this = z;                                                             \
    }

class Fq {
public:
    pa_fq v{};
    static Fq zero() { return Fq(); }
    static Fq one() {
        Fq r;
        std::memcpy(r.v.l, detail::kR, sizeof r.v.l);
        return r;
    }
    PA_FIELD_COMMON(Fq)
    void mul_assign(const Fq& o) { check(pa_fq_mul_batch(&v, &o.v, &v, 1), "Fq::mul_assign"); }
    void square() { check(pa_fq_square_batch(&v, &v, 1), "Fq::square"); }
    void frobenius_map(size_t) {}  // fq.rs:905-907: no effect in a prime field
    std::optional<Fq> inverse() const {
        Fq r;
        uint8_t ok = 0;
        check(pa_fq_inverse_batch(&v, &r.v, &ok, 1), "Fq::inverse");
        return ok ? std::optional<Fq>(r) : std::nullopt;
    }
    Fq pow(const std::vector<uint64_t>& exp) const {
        Fq r;
        check(pa_fq_pow_batch(&v, exp.empty() ? nullptr : exp.data(), exp.size(), &r.v, 1), "Fq::pow");
        return r;
    }
    std::optional<Fq> sqrt() const {
        Fq r;
        uint8_t ok = 0;
        check(pa_fq_sqrt_batch(&v, &r.v, &ok, 1), "Fq::sqrt");
        return ok ? std::optional<Fq>(r) : std::nullopt;
    }
};

class Fq2 {
public:
    pa_fq2 v{};
    static Fq2 zero() { return Fq2(); }
    static Fq2 one() {
        Fq2 r;
        r.v.c0 = Fq::one().v;
        return r;
    }
    PA_FIELD_COMMON(Fq2)
    void mul_assign(const Fq2& o) { check(pa_fq2_mul_batch(&v, &o.v, &v, 1), "Fq2::mul_assign"); }
    void square() { check(pa_fq2_square_batch(&v, &v, 1), "Fq2::square"); }
    void frobenius_map(size_t power) { check(pa_fq2_frobenius_map_batch(&v, &v, 1, power), "Fq2::frobenius_map"); }
    std::optional<Fq2> inverse() const {
        Fq2 r;
        uint8_t ok = 0;
        check(pa_fq2_inverse_batch(&v, &r.v, &ok, 1), "Fq2::inverse");
        return ok ? std::optional<Fq2>(r) : std::nullopt;
    }
    Fq2 pow(const std::vector<uint64_t>& exp) const { return detail::pow_generic(*this, exp); }
    std::optional<Fq2> sqrt() const {
        Fq2 r;
        uint8_t ok = 0;
        check(pa_fq2_sqrt_batch(&v, &r.v, &ok, 1), "Fq2::sqrt");
        return ok ? std::optional<Fq2>(r) : std::nullopt;
    }
};

class Fq6 {
public:
    pa_fq6 v{};
    static Fq6 zero() { return Fq6(); }
    static Fq6 one() {
        Fq6 r;
        r.v.c0 = Fq2::one().v;
        return r;
    }
    PA_FIELD_COMMON(Fq6)
    void mul_assign(const Fq6& o) { check(pa_fq6_mul_batch(&v, &o.v, &v, 1), "Fq6::mul_assign"); }
    void square() { check(pa_fq6_square_batch(&v, &v, 1), "Fq6::square"); }
    void frobenius_map(size_t power) { check(pa_fq6_frobenius_map_batch(&v, &v, 1, power), "Fq6::frobenius_map"); }
    std::optional<Fq6> inverse() const {
        Fq6 r;
        uint8_t ok = 0;
        check(pa_fq6_inverse_batch(&v, &r.v, &ok, 1), "Fq6::inverse");
        return ok ? std::optional<Fq6>(r) : std::nullopt;
    }
    Fq6 pow(const std::vector<uint64_t>& exp) const { return detail::pow_generic(*this, exp); }
};

class Fq12 {
public:
    pa_fq12 v{};
    static Fq12 zero() { return Fq12(); }
    static Fq12 one() {
        Fq12 r;
        r.v.c0.c0.c0 = Fq::one().v;
        return r;
    }
    PA_FIELD_COMMON(Fq12)
    void mul_assign(const Fq12& o) { check(pa_fq12_mul_batch(&v, &o.v, &v, 1), "Fq12::mul_assign"); }
    void square() { check(pa_fq12_square_batch(&v, &v, 1), "Fq12::square"); }
    void conjugate() {  // fq12.rs:30-32
        Fq6 c1{v.c1};
        c1.negate();
        v.c1 = c1.v;
    }
    void frobenius_map(size_t power) {
        check(pa_fq12_frobenius_map_batch(&v, &v, 1, power), "Fq12::frobenius_map");
    }
    std::optional<Fq12> inverse() const {
        Fq12 r;
        uint8_t ok = 0;
        check(pa_fq12_inverse_batch(&v, &r.v, &ok, 1), "Fq12::inverse");
        return ok ? std::optional<Fq12>(r) : std::nullopt;
    }
    Fq12 pow(const std::vector<uint64_t>& exp) const {
        Fq12 r;
        check(pa_fq12_pow_batch(&v, exp.empty() ? nullptr : exp.data(), exp.size(), &r.v, 1), "Fq12::pow");
        return r;
    }
};
#undef PA_FIELD_COMMON

// FrRepr: 4 x u64 little-endian canonical scalar (fr.rs:58)
struct FrRepr {
    pa_fr_repr v{};
    FrRepr() = default;
    explicit FrRepr(uint64_t x) { v.l[0] = x; }
    FrRepr(uint64_t l0, uint64_t l1, uint64_t l2, uint64_t l3) : v{{l0, l1, l2, l3}} {}
};

// ---------------- point encodings (lib.rs:236-264, 469-481) ----------------
class GroupDecodingError : public std::runtime_error {
public:
    enum Kind {
        NotOnCurve = PA_DECODE_NOT_ON_CURVE,
        NotInSubgroup = PA_DECODE_NOT_IN_SUBGROUP,
        CoordinateDecodingError = PA_DECODE_COORDINATE_X_C0,  // any coordinate; see coordinate()
        UnexpectedCompressionMode = PA_DECODE_UNEXPECTED_COMPRESSION_MODE,
        UnexpectedInformation = PA_DECODE_UNEXPECTED_INFORMATION,
    };
    GroupDecodingError(int status, int group)
        : std::runtime_error(describe(status, group)), status_(status), group_(group) {}
    Kind kind() const {
        if (status_ >= PA_DECODE_COORDINATE_X_C0 && status_ <= PA_DECODE_COORDINATE_Y_C1) return CoordinateDecodingError;
        return static_cast<Kind>(status_);
    }
    int status() const { return status_; }
    // the &'static str of CoordinateDecodingError (ec.rs:720-731, 1380-1395)
    const char* coordinate() const { return coordinate_name(status_, group_); }

    static const char* coordinate_name(int status, int group) {
        switch (status) {
            case PA_DECODE_COORDINATE_X_C0: return group == 1 ? "x coordinate" : "x coordinate (c0)";
            case PA_DECODE_COORDINATE_X_C1: return "x coordinate (c1)";
            case PA_DECODE_COORDINATE_Y_C0: return group == 1 ? "y coordinate" : "y coordinate (c0)";
            case PA_DECODE_COORDINATE_Y_C1: return "y coordinate (c1)";
            default: return "";
        }
    }
    static std::string describe(int status, int group) {  // lib.rs:483-500
        switch (status) {
            case PA_DECODE_NOT_ON_CURVE: return "coordinate(s) do not lie on the curve";
            case PA_DECODE_NOT_IN_SUBGROUP: return "the element is not part of an r-order subgroup";
            case PA_DECODE_UNEXPECTED_COMPRESSION_MODE: return "encoding has unexpected compression mode";
            case PA_DECODE_UNEXPECTED_INFORMATION: return "encoding has unexpected information";
            default: return std::string("coordinate(s) could not be decoded: ") + coordinate_name(status, group);
        }
    }

private:
    int status_, group_;
};

class G1Affine;
class G2Affine;

// EncodedPoint for one wire format; `Affine` is G1Affine or G2Affine
template <class Affine, int Group, bool Compressed>
class Encoded {
public:
    static constexpr size_t kSize = (Group == 1 ? 48 : 96) * (Compressed ? 1 : 2);
    std::array<uint8_t, kSize> bytes{};

    static Encoded empty() { return Encoded(); }
    static size_t size() { return kSize; }
    const uint8_t* as_ref() const { return bytes.data(); }
    uint8_t* as_mut() { return bytes.data(); }

    Affine into_affine() const { return decode(true); }
    Affine into_affine_unchecked() const { return decode(false); }
    static Encoded from_affine(const Affine& a) {
        Encoded e;
        encode_batch(&a, 1, &e);
        return e;
    }

    // batched forms: one ABI call; statuses per record (0 = Ok)
    static std::vector<Affine> into_affine_batch(const std::vector<Encoded>& enc, std::vector<uint8_t>& status,
                                                 bool checked = true) {
        std::vector<Affine> out(enc.size());
        status.assign(enc.size(), 0);
        decode_batch(enc.data(), enc.size(), checked, out.data(), status.data());
        return out;
    }
    static std::vector<Encoded> from_affine_batch(const std::vector<Affine>& pts) {
        std::vector<Encoded> out(pts.size());
        encode_batch(pts.data(), pts.size(), out.data());
        return out;
    }

private:
    Affine decode(bool checked) const {
        Affine a;
        uint8_t st = 0;
        decode_batch(this, 1, checked, &a, &st);
        if (st != PA_DECODE_OK) throw GroupDecodingError(st, Group);
        return a;
    }
    static void decode_batch(const Encoded* enc, size_t n, bool checked, Affine* out, uint8_t* st);
    static void encode_batch(const Affine* a, size_t n, Encoded* out);
};

// ---------------- curve points (ec.rs) ----------------
class G1Prepared;
class G2Prepared;
template <int G> class Projective;
using G1 = Projective<1>;   // Jacobian, zero iff z == 0 (ec.rs:224-240)
using G2 = Projective<2>;

// The affine half of the curve_impl! macro (ec.rs:13-29, 97-189) for either group.
#define PA_AFFINE_COMMON(A, RAW, PROJ, BASE, G)                                                     \
    RAW v{};                                                                                       \
    static A zero() { /* ec.rs:158-164 */                                                          \
        A r;                                                                                       \
        r.v.y = BASE::one().v;                                                                     \
        r.v.infinity = 1;                                                                          \
        return r;                                                                                  \
    }                                                                                              \
    bool is_zero() const { return v.infinity != 0; }                                               \
    bool operator==(const A& o) const {                                                            \
        return v.infinity == o.v.infinity &&                                                       \
               (v.infinity || (detail::bytes_equal(v.x, o.v.x) && detail::bytes_equal(v.y, o.v.y))); \
    }                                                                                              \
    bool operator!=(const A& o) const { return !(*this == o); }                                    \
    /* CurveAffine::negate, ec.rs:166-172 */                                                       \
    void negate() {                                                                                \
        if (!is_zero()) {                                                                          \
            BASE y{v.y};                                                                           \
            y.negate();                                                                            \
            v.y = y.v;                                                                             \
        }                                                                                          \
    }                                                                                              \
    /* CurveAffine::into_projective, ec.rs:570-582 */                                              \
    inline PROJ into_projective() const;                                                           \
    /* is_in_correct_subgroup_assuming_on_curve, ec.rs:142-144 (the endomorphism test) */          \
    bool is_in_correct_subgroup_assuming_on_curve() const {                                        \
        uint8_t ok = 0;                                                                            \
        check(pa_g##G##_subgroup_check_batch(&v, 1, &ok), "is_in_correct_subgroup_assuming_on_curve"); \
        return ok != 0;                                                                            \
    }                                                                                              \
    /* CurveAffine::mul, ec.rs:174-177: the reference's double-and-add, bit-exact Jacobian words */ \
    inline PROJ mul(const FrRepr& s) const;                                                        \
    static inline std::vector<PROJ> mul_batch(const std::vector<A>& p, const std::vector<FrRepr>& s);

class G1Affine {
public:
    PA_AFFINE_COMMON(G1Affine, pa_g1_affine, G1, Fq, 1)
    static G1Affine one() {  // ec.rs:877-883 (fq.rs generator words)
        G1Affine r;
        const uint64_t x[6] = {0x5cb38790fd530c16ULL, 0x7817fc679976fff5ULL, 0x154f95c7143ba1c1ULL,
                               0xf0ae6acdf3d0e747ULL, 0xedce6ecc21dbf440ULL, 0x120177419e0bfb75ULL};
        const uint64_t y[6] = {0xbaac93d50ce72271ULL, 0x8c22631a7918fd8eULL, 0xdd595f13570725ceULL,
                               0x51ac582950405194ULL, 0x0e1c8c3fad0059c0ULL, 0x0bbc3efc5008a26aULL};
        std::memcpy(r.v.x.l, x, 48);
        std::memcpy(r.v.y.l, y, 48);
        return r;
    }
    G1Prepared prepare() const;
    Fq12 pairing_with(const G2Affine& other) const;
    Encoded<G1Affine, 1, false> into_uncompressed() const { return Encoded<G1Affine, 1, false>::from_affine(*this); }
    Encoded<G1Affine, 1, true> into_compressed() const { return Encoded<G1Affine, 1, true>::from_affine(*this); }
};

class G2Affine {
public:
    PA_AFFINE_COMMON(G2Affine, pa_g2_affine, G2, Fq2, 2)
    static G2Affine one() {  // ec.rs:1543-1555
        G2Affine r;
        const uint64_t xc0[6] = {0xf5f28fa202940a10ULL, 0xb3f5fb2687b4961aULL, 0xa1a893b53e2ae580ULL,
                                 0x9894999d1a3caee9ULL, 0x6f67b7631863366bULL, 0x058191924350bcd7ULL};
        const uint64_t xc1[6] = {0xa5a9c0759e23f606ULL, 0xaaa0c59dbccd60c3ULL, 0x3bb17e18e2867806ULL,
                                 0x1b1ab6cc8541b367ULL, 0xc2b6ed0ef2158547ULL, 0x11922a097360edf3ULL};
        const uint64_t yc0[6] = {0x4c730af860494c4aULL, 0x597cfa1f5e369c5aULL, 0xe7e6856caa0a635aULL,
                                 0xbbefb5e96e0d495fULL, 0x07d3a975f0ef25a2ULL, 0x0083fd8e7e80dae5ULL};
        const uint64_t yc1[6] = {0xadc0fc92df64b05dULL, 0x18aa270a2b1461dcULL, 0x86adac6a3be4eba0ULL,
                                 0x79495c4ec93da33aULL, 0xe7175850a43ccaedULL, 0x0b2bc2a163de1bf2ULL};
        std::memcpy(r.v.x.c0.l, xc0, 48);
        std::memcpy(r.v.x.c1.l, xc1, 48);
        std::memcpy(r.v.y.c0.l, yc0, 48);
        std::memcpy(r.v.y.c1.l, yc1, 48);
        return r;
    }
    G2Prepared prepare() const;
    Fq12 pairing_with(const G1Affine& other) const;
    Encoded<G2Affine, 2, false> into_uncompressed() const { return Encoded<G2Affine, 2, false>::from_affine(*this); }
    Encoded<G2Affine, 2, true> into_compressed() const { return Encoded<G2Affine, 2, true>::from_affine(*this); }
};
#undef PA_AFFINE_COMMON

// The C ABI of each group, for the Projective template
template <int G> struct GroupAbi;
template <> struct GroupAbi<1> {
    using Raw = pa_g1;
    using RawAffine = pa_g1_affine;
    using Affine = G1Affine;
    using Base = Fq;
    static constexpr auto dbl = &pa_g1_double_batch;
    static constexpr auto add = &pa_g1_add_batch;
    static constexpr auto add_mixed = &pa_g1_add_mixed_batch;
    static constexpr auto neg = &pa_g1_negate_batch;
    static constexpr auto sub = &pa_g1_sub_batch;
    static constexpr auto to_affine = &pa_g1_into_affine_batch;
    static constexpr auto from_affine = &pa_g1_into_projective_batch;
    static constexpr auto eq = &pa_g1_eq_batch;
    static constexpr auto normalize = &pa_g1_batch_normalization;
    static constexpr auto mul_assign = &pa_g1_mul_assign_batch;
    static constexpr auto affine_mul = &pa_g1_affine_mul_batch;
    static constexpr auto fixed_base = &pa_g1_wnaf_fixed_base_window;
    static constexpr auto fixed_base_exact = &pa_g1_wnaf_fixed_base_exact;
    static constexpr auto fixed_scalar_exact = &pa_g1_wnaf_fixed_scalar_exact;
    static constexpr auto window_for_scalar = &pa_g1_recommended_wnaf_for_scalar;
    static constexpr auto window_for_count = &pa_g1_recommended_wnaf_for_num_scalars;
    static constexpr auto multiexp = &pa_g1_multiexp;
};
template <> struct GroupAbi<2> {
    using Raw = pa_g2;
    using RawAffine = pa_g2_affine;
    using Affine = G2Affine;
    using Base = Fq2;
    static constexpr auto dbl = &pa_g2_double_batch;
    static constexpr auto add = &pa_g2_add_batch;
    static constexpr auto add_mixed = &pa_g2_add_mixed_batch;
    static constexpr auto neg = &pa_g2_negate_batch;
    static constexpr auto sub = &pa_g2_sub_batch;
    static constexpr auto to_affine = &pa_g2_into_affine_batch;
    static constexpr auto from_affine = &pa_g2_into_projective_batch;
    static constexpr auto eq = &pa_g2_eq_batch;
    static constexpr auto normalize = &pa_g2_batch_normalization;
    static constexpr auto mul_assign = &pa_g2_mul_assign_batch;
    static constexpr auto affine_mul = &pa_g2_affine_mul_batch;
    static constexpr auto fixed_base = &pa_g2_wnaf_fixed_base_window;
    static constexpr auto fixed_base_exact = &pa_g2_wnaf_fixed_base_exact;
    static constexpr auto fixed_scalar_exact = &pa_g2_wnaf_fixed_scalar_exact;
    static constexpr auto window_for_scalar = &pa_g2_recommended_wnaf_for_scalar;
    static constexpr auto window_for_count = &pa_g2_recommended_wnaf_for_num_scalars;
    static constexpr auto multiexp = &pa_g2_multiexp;
};

// CurveProjective (lib.rs:114-181) for G1 / G2: every operation is the
// reference's formula sequence on the GPU (bit-exact Jacobian words);
// operator== is the reference's representation-independent PartialEq
// (ec.rs:45-85).  The *_batch statics make one ABI call for a whole vector.
template <int G>
class Projective {
public:
    using Abi = GroupAbi<G>;
    using Affine = typename Abi::Affine;
    using Base = typename Abi::Base;
    typename Abi::Raw v{};

    static Projective zero() {  // ec.rs:224-230
        Projective r;
        r.v.y = Base::one().v;
        return r;
    }
    static Projective one() { return Affine::one().into_projective(); }  // ec.rs:232-234
    bool is_zero() const { return Base{v.z}.is_zero(); }
    bool is_normalized() const { return is_zero() || Base{v.z} == Base::one(); }  // ec.rs:242-244

    void double_() { check(Abi::dbl(&v, &v, 1), "CurveProjective::double"); }
    void add_assign(const Projective& o) { check(Abi::add(&v, &o.v, &v, 1), "CurveProjective::add_assign"); }
    void add_assign_mixed(const Affine& o) {
        check(Abi::add_mixed(&v, &o.v, &v, 1), "CurveProjective::add_assign_mixed");
    }
    void negate() { check(Abi::neg(&v, &v, 1), "CurveProjective::negate"); }
    void sub_assign(const Projective& o) { check(Abi::sub(&v, &o.v, &v, 1), "CurveProjective::sub_assign"); }
    void mul_assign(const FrRepr& s) { check(Abi::mul_assign(&v, &s.v, &v, 1), "CurveProjective::mul_assign"); }
    Affine into_affine() const {
        Affine a;
        check(Abi::to_affine(&v, &a.v, 1), "CurveProjective::into_affine");
        return a;
    }
    bool operator==(const Projective& o) const {
        uint8_t r = 0;
        check(Abi::eq(&v, &o.v, &r, 1), "PartialEq");
        return r != 0;
    }
    bool operator!=(const Projective& o) const { return !(*this == o); }

    static size_t recommended_wnaf_for_scalar(const FrRepr& s) { return (size_t)Abi::window_for_scalar(&s.v); }
    static size_t recommended_wnaf_for_num_scalars(size_t n) { return (size_t)Abi::window_for_count(n); }

    // CurveProjective::batch_normalization (ec.rs:246-294), in place
    static void batch_normalization(std::vector<Projective>& v) {
        check(Abi::normalize(v.empty() ? nullptr : &v[0].v, v.size()), "CurveProjective::batch_normalization");
    }
    // ---- batched forms: out[i] = op(a[i], b[i]) in one ABI call ----
    static std::vector<Projective> double_batch(const std::vector<Projective>& a) {
        std::vector<Projective> out(a.size());
        if (!a.empty()) check(Abi::dbl(&a[0].v, &out[0].v, a.size()), "double_batch");
        return out;
    }
    // PartialEq per item (ec.rs:45-85) in one ABI call
    static std::vector<bool> eq_batch(const std::vector<Projective>& a, const std::vector<Projective>& b) {
        if (a.size() != b.size()) throw std::invalid_argument("eq_batch: operand lengths differ");
        std::vector<uint8_t> r(a.size());
        if (!a.empty()) check(Abi::eq(&a[0].v, &b[0].v, r.data(), a.size()), "eq_batch");
        return std::vector<bool>(r.begin(), r.end());
    }
    static std::vector<Projective> add_batch(const std::vector<Projective>& a, const std::vector<Projective>& b) {
        same_size(a.size(), b.size());
        std::vector<Projective> out(a.size());
        if (!a.empty()) check(Abi::add(&a[0].v, &b[0].v, &out[0].v, a.size()), "add_batch");
        return out;
    }
    static std::vector<Projective> add_mixed_batch(const std::vector<Projective>& a, const std::vector<Affine>& b) {
        same_size(a.size(), b.size());
        std::vector<Projective> out(a.size());
        if (!a.empty()) check(Abi::add_mixed(&a[0].v, &b[0].v, &out[0].v, a.size()), "add_mixed_batch");
        return out;
    }
    static std::vector<Affine> into_affine_batch(const std::vector<Projective>& a) {
        std::vector<Affine> out(a.size());
        if (!a.empty()) check(Abi::to_affine(&a[0].v, &out[0].v, a.size()), "into_affine_batch");
        return out;
    }
    static std::vector<Projective> mul_assign_batch(const std::vector<Projective>& a, const std::vector<FrRepr>& s) {
        same_size(a.size(), s.size());
        std::vector<Projective> out(a.size());
        if (!a.empty()) check(Abi::mul_assign(&a[0].v, &s[0].v, &out[0].v, a.size()), "mul_assign_batch");
        return out;
    }
    // sum_i s_i * bases_i (the prover's multiexp; Pippenger on the device),
    // equal as a point to the sum of CurveAffine::mul results
    static Projective multiexp(const std::vector<Affine>& bases, const std::vector<FrRepr>& s) {
        same_size(bases.size(), s.size());
        Projective r;
        check(Abi::multiexp(bases.empty() ? nullptr : &bases[0].v, s.empty() ? nullptr : &s[0].v, bases.size(), &r.v),
              "multiexp");
        return r;
    }

private:
    static void same_size(size_t a, size_t b) {
        if (a != b) throw Error(PA_ERR_INVALID_ARGUMENT, "batch operands differ in length");
    }
};

#define PA_AFFINE_DEFS(A, PROJ, G)                                                                   \
    inline PROJ A::into_projective() const {                                                         \
        PROJ r;                                                                                      \
        check(GroupAbi<G>::from_affine(&v, &r.v, 1), "CurveAffine::into_projective");                \
        return r;                                                                                    \
    }                                                                                                \
    inline PROJ A::mul(const FrRepr& s) const {                                                      \
        PROJ r;                                                                                      \
        check(GroupAbi<G>::affine_mul(&v, &s.v, &r.v, 1), "CurveAffine::mul");                       \
        return r;                                                                                    \
    }                                                                                                \
    inline std::vector<PROJ> A::mul_batch(const std::vector<A>& p, const std::vector<FrRepr>& s) {   \
        if (p.size() != s.size()) throw Error(PA_ERR_INVALID_ARGUMENT, "mul_batch: length mismatch"); \
        std::vector<PROJ> out(p.size());                                                             \
        if (!p.empty()) check(GroupAbi<G>::affine_mul(&p[0].v, &s[0].v, &out[0].v, p.size()), "mul_batch"); \
        return out;                                                                                  \
    }
PA_AFFINE_DEFS(G1Affine, G1, 1)
PA_AFFINE_DEFS(G2Affine, G2, 2)
#undef PA_AFFINE_DEFS

using G1Uncompressed = Encoded<G1Affine, 1, false>;
using G1Compressed = Encoded<G1Affine, 1, true>;
using G2Uncompressed = Encoded<G2Affine, 2, false>;
using G2Compressed = Encoded<G2Affine, 2, true>;

template <class Affine, int Group, bool Compressed>
void Encoded<Affine, Group, Compressed>::decode_batch(const Encoded* enc, size_t n, bool checked, Affine* out,
                                                      uint8_t* st) {
    static_assert(sizeof(Encoded) == kSize, "packed records");
    static_assert(sizeof(Affine) == (Group == 1 ? sizeof(pa_g1_affine) : sizeof(pa_g2_affine)), "ABI layout");
    int rc;
    if constexpr (Group == 1)
        rc = pa_g1_decode_batch(reinterpret_cast<const uint8_t*>(enc), n, Compressed, checked,
                                reinterpret_cast<pa_g1_affine*>(out), st);
    else
        rc = pa_g2_decode_batch(reinterpret_cast<const uint8_t*>(enc), n, Compressed, checked,
                                reinterpret_cast<pa_g2_affine*>(out), st);
    check(rc, "EncodedPoint::into_affine");
}
template <class Affine, int Group, bool Compressed>
void Encoded<Affine, Group, Compressed>::encode_batch(const Affine* a, size_t n, Encoded* out) {
    int rc;
    if constexpr (Group == 1)
        rc = pa_g1_encode_batch(reinterpret_cast<const pa_g1_affine*>(a), n, Compressed,
                                reinterpret_cast<uint8_t*>(out));
    else
        rc = pa_g2_encode_batch(reinterpret_cast<const pa_g2_affine*>(a), n, Compressed,
                                reinterpret_cast<uint8_t*>(out));
    check(rc, "EncodedPoint::from_affine");
}

// G1Prepared is a newtype over G1Affine (ec.rs:924-935)
class G1Prepared {
public:
    G1Affine p;
    bool is_zero() const { return p.is_zero(); }
};
// G2Prepared: 68 line coefficients (ec.rs:1615-1619, mod.rs:168-358), 19.6 KB
class G2Prepared {
public:
    std::shared_ptr<pa_g2_prepared> v = std::make_shared<pa_g2_prepared>();
    bool is_zero() const { return v->infinity != 0; }
    static std::vector<G2Prepared> from_affine_batch(const std::vector<G2Affine>& q) {
        std::vector<pa_g2_prepared> raw(q.size());
        check(pa_g2_prepare_batch(q.empty() ? nullptr : &q[0].v, raw.empty() ? nullptr : raw.data(), q.size()),
              "G2Prepared::from_affine");
        std::vector<G2Prepared> out(q.size());
        for (size_t i = 0; i < q.size(); i++) *out[i].v = raw[i];
        return out;
    }
};

inline G1Prepared G1Affine::prepare() const { return G1Prepared{*this}; }
inline G2Prepared G2Affine::prepare() const { return G2Prepared::from_affine_batch({*this})[0]; }

// ---------------- Engine for Bls12 (mod.rs:30-161, lib.rs:34-110) ----------------
struct Bls12 {
    // Engine::miller_loop: product over the pairs (mod.rs:40-102)
    static Fq12 miller_loop(const std::vector<std::pair<const G1Prepared*, const G2Prepared*>>& pairs) {
        std::vector<pa_g1_affine> p(pairs.size());
        std::vector<pa_g2_prepared> q(pairs.size());
        for (size_t i = 0; i < pairs.size(); i++) {
            p[i] = pairs[i].first->p.v;
            q[i] = *pairs[i].second->v;
        }
        Fq12 r;
        check(pa_multi_miller_loop(p.empty() ? nullptr : p.data(), q.empty() ? nullptr : q.data(), pairs.size(), &r.v),
              "Bls12::miller_loop");
        return r;
    }
    // Engine::miller_loop([(p_i, q)]) for every i with ONE prepared q (the same
    // &G2Prepared in each pair, lib.rs:88-96): a verifying key's prepared gamma /
    // delta against many points; q's lines are staged once per call
    static std::vector<Fq12> miller_loop_shared(const std::vector<G1Prepared>& p, const G2Prepared& q) {
        std::vector<pa_g1_affine> pp(p.size());
        for (size_t i = 0; i < p.size(); i++) pp[i] = p[i].p.v;
        std::vector<Fq12> out(p.size());
        if (!p.empty())
            check(pa_miller_loop_shared_prepared(pp.data(), pp.size(), q.v.get(), &out[0].v),
                  "Bls12::miller_loop_shared");
        return out;
    }
    // Engine::final_exponentiation (mod.rs:104-160): None iff f == 0
    static std::optional<Fq12> final_exponentiation(const Fq12& f) {
        Fq12 r;
        uint8_t ok = 0;
        check(pa_final_exponentiation_batch(&f.v, &r.v, &ok, 1), "Bls12::final_exponentiation");
        return ok ? std::optional<Fq12>(r) : std::nullopt;
    }
    // Engine::pairing (lib.rs:101-109)
    static Fq12 pairing(const G1Affine& p, const G2Affine& q) {
        Fq12 r;
        check(pa_pairing_batch(&p.v, &q.v, &r.v, 1), "Bls12::pairing");
        return r;
    }

    // ---- batched forms (the reason this library exists) ----
    static std::vector<Fq12> pairing_batch(const std::vector<G1Affine>& p, const std::vector<G2Affine>& q) {
        if (p.size() != q.size()) throw Error(PA_ERR_INVALID_ARGUMENT, "pairing_batch: length mismatch");
        std::vector<Fq12> out(p.size());
        if (!p.empty()) check(pa_pairing_batch(&p[0].v, &q[0].v, &out[0].v, p.size()), "Bls12::pairing_batch");
        return out;
    }
    // final_exponentiation(miller_loop(pairs)) with affine inputs: the batch
    // verification product; None iff the Miller value is zero
    static std::optional<Fq12> multi_pairing(const std::vector<G1Affine>& p, const std::vector<G2Affine>& q) {
        if (p.size() != q.size()) throw Error(PA_ERR_INVALID_ARGUMENT, "multi_pairing: length mismatch");
        Fq12 r;
        uint8_t ok = 0;
        check(pa_multi_pairing(p.empty() ? nullptr : &p[0].v, q.empty() ? nullptr : &q[0].v, p.size(), &r.v, &ok),
              "Bls12::multi_pairing");
        return ok ? std::optional<Fq12>(r) : std::nullopt;
    }
};

inline Fq12 G1Affine::pairing_with(const G2Affine& other) const { return Bls12::pairing(*this, other); }
inline Fq12 G2Affine::pairing_with(const G1Affine& other) const { return Bls12::pairing(other, *this); }

// ---------------- Wnaf (wnaf.rs:73-179), G1 and G2 ----------------
// Wnaf::new_().base(g, num_scalars).scalar(s): fixed base (wnaf.rs:93-107,
// 169-178); Wnaf::new_().scalar(s).base(g): fixed scalar (wnaf.rs:111-128,
// 156-166); shared() hands a copy to another thread (wnaf.rs:131-154).  The
// window is the reference's recommended_wnaf_* choice (window()).
//   * fixed scalar: the reference's own table chain, wnaf_form and wnaf_exp on
//     the GPU (pa_g{1,2}_wnaf_fixed_scalar_exact): Jacobian words identical;
//   * fixed base: scalars() multiplies with the signed base-256 comb, so the
//     POINTS equal the reference's (PartialEq, ec.rs:45-85) while Jacobian words
//     may differ; scalars_exact() runs the reference's chain instead
//     (pa_g{1,2}_wnaf_fixed_base_exact, bit-identical words, slower).
// Both include the reference's wnaf_form wrap (add_nocarry, wnaf.rs:30-35):
// for an odd repr whose bits window..255 are all ones its digits spell
// s - 2^256, and so does the product here.
//
// wnaf_wraps(s, w): whether wnaf_form(s, w) wraps; t = 2^256 - s then.
inline bool wnaf_wraps(const FrRepr& s, size_t window, FrRepr* t) {
    if (window < 1 || window > 62 || !(s.v.l[0] & 1)) return false;
    if ((s.v.l[0] | ((1ull << window) - 1)) != ~0ull || (s.v.l[1] & s.v.l[2] & s.v.l[3]) != ~0ull) return false;
    uint64_t c = 1;
    for (int k = 0; k < 4; k++) {
        const uint64_t v = ~s.v.l[k] + c;
        c = (c && v == 0) ? 1 : 0;
        t->v.l[k] = v;
    }
    return true;
}
template <class P>
class WnafBase {
public:
    WnafBase(const P& g, size_t num_scalars) : base_(g), window_(P::recommended_wnaf_for_num_scalars(num_scalars)) {}
    size_t window() const { return window_; }
    WnafBase shared() const { return *this; }
    std::vector<P> scalars(const std::vector<FrRepr>& s) const {
        std::vector<P> out(s.size());
        if (!s.empty()) check(P::Abi::fixed_base(&base_.v, &s[0].v, s.size(), (int)window_, &out[0].v), "Wnaf::scalar");
        return out;
    }
    P scalar(const FrRepr& s) const { return scalars({s})[0]; }
    // bit-identical Jacobian words (window <= 20)
    std::vector<P> scalars_exact(const std::vector<FrRepr>& s) const {
        std::vector<P> out(s.size());
        if (!s.empty())
            check(P::Abi::fixed_base_exact(&base_.v, &s[0].v, s.size(), (int)window_, &out[0].v),
                  "Wnaf::scalar (exact)");
        return out;
    }

private:
    P base_;
    size_t window_;
};

class WnafScalar {
public:
    explicit WnafScalar(const FrRepr& s) : s_(s) {}
    template <class P>
    P base(const P& g) const {
        return bases(std::vector<P>{g})[0];
    }
    template <class P>
    std::vector<P> bases(const std::vector<P>& g) const {
        std::vector<P> out(g.size());
        if (!g.empty())
            check(P::Abi::fixed_scalar_exact(&g[0].v, g.size(), &s_.v, (int)window_for<P>(s_), &out[0].v),
                  "Wnaf::base");
        return out;
    }
    template <class P>
    static size_t window_for(const FrRepr& s) { return P::recommended_wnaf_for_scalar(s); }

private:
    FrRepr s_;
};

class Wnaf {
public:
    static Wnaf new_() { return Wnaf(); }
    template <class P>
    WnafBase<P> base(const P& g, size_t num_scalars) const { return WnafBase<P>(g, num_scalars); }
    WnafScalar scalar(const FrRepr& s) const { return WnafScalar(s); }
};

}  // namespace pairing_amd
