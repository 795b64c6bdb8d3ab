// The reference's engine / encoding tests, written against the C++ mirror of
// its trait surface (include/pairing_amd.hpp) so they read like the originals:
//   bls12_381/tests/mod.rs:23-52     test_pairing_result_against_relic
//   src/tests/engine.rs:50-126       random_miller_loop_tests, random_bilinearity_tests
//   bls12_381/tests/mod.rs:98-560    invalid-encoding suites (a representative subset)
//   src/tests/curve.rs:68-179, 357-387  wNAF / batch_normalization agreement
// Inputs that need a scalar multiplication on G2 (which the product does not
// expose) come from a data file written by tests/test_cpp_mirror.py with the
// C oracle: n, RELIC Fq12, then n records each of a*G1, b*G2, (ab)*G1,
// e(aP, bQ) and the scalars a.
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "pairing_amd.hpp"

using namespace pairing_amd;

static int g_failures = 0;
#define EXPECT(cond)                                                          \
    do {                                                                      \
        if (!(cond)) {                                                        \
            std::fprintf(stderr, "  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            g_failures++;                                                     \
        }                                                                     \
    } while (0)

struct Data {
    size_t n = 0;
    Fq12 relic;
    std::vector<G1Affine> a_p, ab_p;
    std::vector<G2Affine> b_q;
    std::vector<Fq12> e_ab;
    std::vector<FrRepr> a;
};

template <class T>
static void read_vec(FILE* f, std::vector<T>& v, size_t n) {
    v.resize(n);
    if (n && std::fread(v.data(), sizeof(T), n, f) != n) throw std::runtime_error("short data file");
}

static Data load(const char* path) {
    Data d;
    FILE* f = std::fopen(path, "rb");
    if (!f) throw std::runtime_error("cannot open data file");
    uint64_t n = 0;
    if (std::fread(&n, 8, 1, f) != 1 || std::fread(&d.relic, sizeof(Fq12), 1, f) != 1)
        throw std::runtime_error("short data file");
    d.n = n;
    read_vec(f, d.a_p, n);
    read_vec(f, d.b_q, n);
    read_vec(f, d.ab_p, n);
    read_vec(f, d.e_ab, n);
    read_vec(f, d.a, n);
    std::fclose(f);
    return d;
}

// tests/mod.rs:23-52
static void test_pairing_result_against_relic(const Data& d) {
    EXPECT(Bls12::pairing(G1Affine::one(), G2Affine::one()) == d.relic);
    EXPECT(G1Affine::one().pairing_with(G2Affine::one()) == d.relic);
    EXPECT(G2Affine::one().pairing_with(G1Affine::one()) == d.relic);
}

// engine.rs:93-126: e(aP, bQ) == e(abP, Q), batched and per pair
static void random_bilinearity_tests(const Data& d) {
    std::vector<G2Affine> g2(d.n, G2Affine::one());
    auto e1 = Bls12::pairing_batch(d.a_p, d.b_q);
    auto e2 = Bls12::pairing_batch(d.ab_p, g2);
    for (size_t i = 0; i < d.n; i++) {
        EXPECT(e1[i] == d.e_ab[i]);
        EXPECT(e2[i] == d.e_ab[i]);
    }
    EXPECT(Bls12::pairing(d.a_p[0], d.b_q[0]) == d.e_ab[0]);
}

// engine.rs:50-91: miller_loop over two pairs == product of single pairings
static void random_miller_loop_tests(const Data& d) {
    for (size_t i = 0; i + 1 < d.n && i < 6; i += 2) {
        const G1Prepared p1 = d.a_p[i].prepare(), p2 = d.a_p[i + 1].prepare();
        const G2Prepared q1 = d.b_q[i].prepare(), q2 = d.b_q[i + 1].prepare();
        Fq12 abcd = Bls12::final_exponentiation(Bls12::miller_loop({{&p1, &q1}, {&p2, &q2}})).value();
        Fq12 ab = Bls12::pairing(d.a_p[i], d.b_q[i]);
        ab.mul_assign(Bls12::pairing(d.a_p[i + 1], d.b_q[i + 1]));
        EXPECT(abcd == ab);
        auto mp = Bls12::multi_pairing({d.a_p[i], d.a_p[i + 1]}, {d.b_q[i], d.b_q[i + 1]});
        EXPECT(mp.has_value() && *mp == ab);
    }
    // pairs with an infinity side are skipped (mod.rs:50-54): the empty product is one
    const G1Prepared z1 = G1Affine::zero().prepare(), o1 = G1Affine::one().prepare();
    const G2Prepared z2 = G2Affine::zero().prepare(), o2 = G2Affine::one().prepare();
    EXPECT(Bls12::miller_loop({{&z1, &o2}, {&o1, &z2}}) == Fq12::one());
    EXPECT(Bls12::miller_loop({}) == Fq12::one());
    // final_exponentiation(0) is None (mod.rs:108, 157-158)
    EXPECT(!Bls12::final_exponentiation(Fq12::zero()).has_value());
    // e(P, Q)^r == 1 via e(aP, Q) * e(-aP, Q)... use Fq12 inverse: e * e^-1 == 1
    Fq12 e = d.e_ab[0];
    Fq12 inv = e.inverse().value();
    e.mul_assign(inv);
    EXPECT(e == Fq12::one());
}

template <class Fn>
static int decode_error(Fn fn, const char** coordinate = nullptr) {
    try {
        fn();
    } catch (const GroupDecodingError& err) {
        if (coordinate) *coordinate = err.coordinate();
        return err.kind();
    }
    return -1;
}

// tests/mod.rs:98-560 (representative cases) and round trips
static void encoding_tests(const Data& d) {
    EXPECT(G1Affine::one().into_compressed().into_affine() == G1Affine::one());
    EXPECT(G1Affine::one().into_uncompressed().into_affine() == G1Affine::one());
    EXPECT(G2Affine::one().into_compressed().into_affine() == G2Affine::one());
    EXPECT(G2Affine::one().into_uncompressed().into_affine() == G2Affine::one());
    EXPECT(G1Affine::zero().into_compressed().into_affine() == G1Affine::zero());

    auto c = G1Affine::one().into_compressed();
    c.as_mut()[0] &= 0x7f;
    EXPECT(decode_error([&] { c.into_affine(); }) == GroupDecodingError::UnexpectedCompressionMode);
    auto z = G2Affine::zero().into_uncompressed();
    z.as_mut()[100] |= 1;
    EXPECT(decode_error([&] { z.into_affine(); }) == GroupDecodingError::UnexpectedInformation);
    // Fq::char() written over y.c1 of G2Affine::one() (tests/mod.rs:300-309)
    static const uint8_t q_be[48] = {0x1a, 0x01, 0x11, 0xea, 0x39, 0x7f, 0xe6, 0x9a, 0x4b, 0x1b, 0xa7, 0xb6,
                                     0x43, 0x4b, 0xac, 0xd7, 0x64, 0x77, 0x4b, 0x84, 0xf3, 0x85, 0x12, 0xbf,
                                     0x67, 0x30, 0xd2, 0xa0, 0xf6, 0xb0, 0xf6, 0x24, 0x1e, 0xab, 0xff, 0xfe,
                                     0xb1, 0x53, 0xff, 0xff, 0xb9, 0xfe, 0xff, 0xff, 0xff, 0xff, 0xaa, 0xab};
    auto o = G2Affine::one().into_uncompressed();
    std::memcpy(o.as_mut() + 96, q_be, 48);
    const char* coord = "";
    EXPECT(decode_error([&] { o.into_affine(); }, &coord) == GroupDecodingError::CoordinateDecodingError);
    EXPECT(std::string(coord) == "y coordinate (c1)");
    // x = 0 is not on the curve (tests/mod.rs:168-179)
    auto u = G1Affine::one().into_uncompressed();
    std::memset(u.as_mut(), 0, 48);
    EXPECT(decode_error([&] { u.into_affine(); }) == GroupDecodingError::NotOnCurve);
    EXPECT(u.into_affine_unchecked().v.infinity == 0);   // unchecked skips the curve check

    // batched: the aP encode and decode back
    auto enc = G1Compressed::from_affine_batch(d.a_p);
    std::vector<uint8_t> st;
    auto back = G1Compressed::into_affine_batch(enc, st);
    for (size_t i = 0; i < d.n; i++) {
        EXPECT(st[i] == PA_DECODE_OK);
        EXPECT(back[i] == d.a_p[i]);
    }
    auto enc2 = G2Uncompressed::from_affine_batch(d.b_q);
    auto back2 = G2Uncompressed::into_affine_batch(enc2, st);
    for (size_t i = 0; i < d.n; i++) EXPECT(back2[i] == d.b_q[i]);
}

// curve.rs:68-179, 357-387: Wnaf fixed-base + batch_normalization == a*G
static void wnaf_batch_normalization_tests(const Data& d) {
    auto v = Wnaf::new_().base(G1Affine::one().into_projective(), d.n).scalars(d.a);
    G1::batch_normalization(v);
    for (size_t i = 0; i < d.n; i++) EXPECT(v[i].into_affine() == d.a_p[i]);
}

// SqrtField (fq.rs:1147-1170)
static void sqrt_tests() {
    Fq one = Fq::one();
    auto r = one.sqrt();
    EXPECT(r.has_value());
    Fq s = *r;
    s.square();
    EXPECT(s == one);
    Fq m1 = one;
    m1.negate();
    EXPECT(!m1.sqrt().has_value());   // q = 3 mod 4: -1 is a non-residue
    EXPECT(Fq::zero().sqrt().value().is_zero());
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s DATA_FILE\n", argv[0]);
        return 2;
    }
    try {
        const Data d = load(argv[1]);
        const std::vector<std::pair<const char*, std::function<void()>>> tests = {
            {"test_pairing_result_against_relic", [&] { test_pairing_result_against_relic(d); }},
            {"random_bilinearity_tests", [&] { random_bilinearity_tests(d); }},
            {"random_miller_loop_tests", [&] { random_miller_loop_tests(d); }},
            {"encoding_tests", [&] { encoding_tests(d); }},
            {"wnaf_batch_normalization_tests", [&] { wnaf_batch_normalization_tests(d); }},
            {"sqrt_tests", [&] { sqrt_tests(); }},
        };
        for (const auto& t : tests) {
            const int before = g_failures;
            t.second();
            std::printf("%s %s\n", g_failures == before ? "ok  " : "FAIL", t.first);
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 3;
    }
    return g_failures ? 1 : 0;
}
