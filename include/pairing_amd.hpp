// pairing_amd.hpp -- C++17 host mirror of the reference crate's trait surface
// for the BLS12-381 hot path, on top of the C ABI of pairing_amd.h.
//
// The reference (`pairing` v0.14.2, Rust) exposes the path as traits:
//   Engine::{miller_loop, final_exponentiation, pairing}   src/lib.rs:34-110
//   CurveAffine::{prepare, pairing_with, into_compressed, ...} lib.rs:185-234
//   CurveProjective::batch_normalization                    lib.rs:114-181
//   EncodedPoint::{into_affine, into_affine_unchecked, from_affine} lib.rs:236-264
//   Field / SqrtField::{mul_assign, square, inverse, sqrt}  lib.rs:267-345
//   Wnaf::new().base(g, n).scalar(s)                         wnaf.rs:73-179
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
}  // namespace detail

class Fq {
public:
    pa_fq v{};
    static Fq zero() { return Fq(); }
    static Fq one() {
        Fq r;
        std::memcpy(r.v.l, detail::kR, sizeof r.v.l);
        return r;
    }
    bool is_zero() const { return detail::bytes_zero(v); }
    bool operator==(const Fq& o) const { return detail::bytes_equal(v, o.v); }
    bool operator!=(const Fq& o) const { return !(*this == o); }
    void mul_assign(const Fq& o) { check(pa_fq_mul_batch(&v, &o.v, &v, 1), "Fq::mul_assign"); }
    void square() { check(pa_fq_square_batch(&v, &v, 1), "Fq::square"); }
    void add_assign(const Fq& o) { check(pa_fq_add_batch(&v, &o.v, &v, 1), "Fq::add_assign"); }
    void sub_assign(const Fq& o) { check(pa_fq_sub_batch(&v, &o.v, &v, 1), "Fq::sub_assign"); }
    void double_() { add_assign(*this); }
    void negate() {
        Fq z;
        z.sub_assign(*this);
        *this = z;
    }
    std::optional<Fq> inverse() const {
        Fq r;
        uint8_t ok = 0;
        check(pa_fq_inverse_batch(&v, &r.v, &ok, 1), "Fq::inverse");
        return ok ? std::optional<Fq>(r) : std::nullopt;
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
    bool is_zero() const { return detail::bytes_zero(v); }
    bool operator==(const Fq2& o) const { return detail::bytes_equal(v, o.v); }
    bool operator!=(const Fq2& o) const { return !(*this == o); }
    void mul_assign(const Fq2& o) { check(pa_fq2_mul_batch(&v, &o.v, &v, 1), "Fq2::mul_assign"); }
    void square() { check(pa_fq2_square_batch(&v, &v, 1), "Fq2::square"); }
    std::optional<Fq2> sqrt() const {
        Fq2 r;
        uint8_t ok = 0;
        check(pa_fq2_sqrt_batch(&v, &r.v, &ok, 1), "Fq2::sqrt");
        return ok ? std::optional<Fq2>(r) : std::nullopt;
    }
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
    bool is_zero() const { return detail::bytes_zero(v); }
    bool operator==(const Fq12& o) const { return detail::bytes_equal(v, o.v); }
    bool operator!=(const Fq12& o) const { return !(*this == o); }
    void mul_assign(const Fq12& o) { check(pa_fq12_mul_batch(&v, &o.v, &v, 1), "Fq12::mul_assign"); }
    void square() { check(pa_fq12_square_batch(&v, &v, 1), "Fq12::square"); }
    void frobenius_map(size_t power) {
        check(pa_fq12_frobenius_map_batch(&v, &v, 1, power), "Fq12::frobenius_map");
    }
    std::optional<Fq12> inverse() const {
        Fq12 r;
        uint8_t ok = 0;
        check(pa_fq12_inverse_batch(&v, &r.v, &ok, 1), "Fq12::inverse");
        return ok ? std::optional<Fq12>(r) : std::nullopt;
    }
};

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
class G1 {  // Jacobian, zero iff z == 0 (ec.rs:224-240)
public:
    pa_g1 v{};
    static G1 zero() {
        G1 r;
        r.v.y = Fq::one().v;
        return r;
    }
    bool is_zero() const { return Fq{v.z}.is_zero(); }
    // CurveProjective::batch_normalization (ec.rs:246-294)
    static void batch_normalization(std::vector<G1>& v) {
        check(pa_g1_batch_normalization(v.empty() ? nullptr : &v[0].v, v.size()), "G1::batch_normalization");
    }
    inline class G1Affine into_affine() const;   // ec.rs:586-619
};

class G1Prepared;
class G2Prepared;

class G1Affine {
public:
    pa_g1_affine v{};
    static G1Affine zero() {  // ec.rs:158-164
        G1Affine r;
        r.v.y = Fq::one().v;
        r.v.infinity = 1;
        return r;
    }
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
    bool is_zero() const { return v.infinity != 0; }
    bool operator==(const G1Affine& o) const {
        return v.infinity == o.v.infinity && (v.infinity || (detail::bytes_equal(v.x, o.v.x) && detail::bytes_equal(v.y, o.v.y)));
    }
    G1 into_projective() const {
        if (is_zero()) return G1::zero();
        G1 r;
        r.v.x = v.x;
        r.v.y = v.y;
        r.v.z = Fq::one().v;
        return r;
    }
    G1Prepared prepare() const;
    Fq12 pairing_with(const G2Affine& other) const;
    Encoded<G1Affine, 1, false> into_uncompressed() const { return Encoded<G1Affine, 1, false>::from_affine(*this); }
    Encoded<G1Affine, 1, true> into_compressed() const { return Encoded<G1Affine, 1, true>::from_affine(*this); }
};

class G2Affine {
public:
    pa_g2_affine v{};
    static G2Affine zero() {
        G2Affine r;
        r.v.y.c0 = Fq::one().v;
        r.v.infinity = 1;
        return r;
    }
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
    bool is_zero() const { return v.infinity != 0; }
    bool operator==(const G2Affine& o) const {
        return v.infinity == o.v.infinity && (v.infinity || (detail::bytes_equal(v.x, o.v.x) && detail::bytes_equal(v.y, o.v.y)));
    }
    G2Prepared prepare() const;
    Fq12 pairing_with(const G1Affine& other) const;
    Encoded<G2Affine, 2, false> into_uncompressed() const { return Encoded<G2Affine, 2, false>::from_affine(*this); }
    Encoded<G2Affine, 2, true> into_compressed() const { return Encoded<G2Affine, 2, true>::from_affine(*this); }
};

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

inline G1Affine G1::into_affine() const {
    if (is_zero()) return G1Affine::zero();
    std::vector<G1> t{*this};
    if (!(Fq{v.z} == Fq::one())) batch_normalization(t);   // z -> 1 on the GPU
    G1Affine a;
    a.v.x = t[0].v.x;
    a.v.y = t[0].v.y;
    return a;
}

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

// ---------------- Wnaf fixed-base path (wnaf.rs:73-179), G1 ----------------
// Wnaf::new().base(g, num_scalars) then .scalar(s): the GPU uses a fixed-base
// comb, so only the resulting points (not the wNAF digits) match the
// reference -- equality is representation-independent (ec.rs:45-85).
class Wnaf {
public:
    static Wnaf new_() { return Wnaf(); }
    Wnaf& base(const G1& g, size_t /*num_scalars*/) {
        base_ = g;
        return *this;
    }
    std::vector<G1> scalars(const std::vector<FrRepr>& s) const {
        std::vector<G1> out(s.size());
        if (!s.empty()) check(pa_g1_wnaf_fixed_base(&base_.v, &s[0].v, s.size(), &out[0].v), "Wnaf::scalar");
        return out;
    }
    G1 scalar(const FrRepr& s) const { return scalars({s})[0]; }

private:
    G1 base_ = G1::zero();
};

}  // namespace pairing_amd
