#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box).  It extracts DATA -- the limb vectors of the
reference's own known-answer tests and digests of its `.dat` vector files --
and writes them as JSON.  No reference source text is stored.

  kat_limbs.json   -- the hex limb arrays of the reference's KAT tests, by
                      test name, in the order they appear in the test body:
                        fr.rs   test_fr_add_assign / sub_assign / mul_assign /
                                squaring / from_into_repr / legendre
                                                         (fr.rs:911-1505, FrRepr arrays)
                        fq.rs   test_fq_mul_assign       (fq.rs:2558-2584)
                        fq.rs   test_fq_squaring         (fq.rs:2630-2651)
                        fq2.rs  test_fq2_squaring        (fq2.rs:272-345)
                        fq2.rs  test_fq2_mul             (fq2.rs:346-409)
                        fq2.rs  test_fq2_inverse         (fq2.rs:411-458)
                        ec.rs   test_g1_addition_correctness / test_g1_doubling_correctness
                        ec.rs   test_g2_addition_correctness / test_g2_doubling_correctness
                      plus the RELIC pairing KAT (bls12_381/tests/mod.rs:23-52)
                      as 12 decimal integers.
  dat_vectors.json -- for each of the four k*G `.dat` files
                      (bls12_381/tests/mod.rs:55-97): size, SHA-256, and the
                      first 8 records in hex.
"""
import hashlib
import json
import os
import re

REF = "/root/reference/src/bls12_381"
HERE = os.path.dirname(os.path.abspath(__file__))


def test_body(src, name):
    m = re.search(r"fn %s\(\)\s*\{" % re.escape(name), src)
    if not m:
        raise KeyError(name)
    i = m.end()
    depth = 1
    while depth:
        c = src[i]
        depth += c == "{"
        depth -= c == "}"
        i += 1
    return src[m.end():i]


def repr_arrays(body):
    out = []
    for arr in re.findall(r"FqRepr\(\[(.*?)\]\)", body, re.S):
        words = [w.strip() for w in arr.split(",") if w.strip()]
        if len(words) == 6:
            out.append([int(w, 16) for w in words])
    return out


def fr_repr_arrays(body):
    out = []
    for arr in re.findall(r"FrRepr\(\[(.*?)\]\)", body, re.S):
        words = [w.strip() for w in arr.split(",") if w.strip()]
        if len(words) == 4:
            out.append([int(w, 16) for w in words])
    return out


def main():
    kats = {}
    src = open(os.path.join(REF, "fr.rs")).read()
    for t in ("test_fr_add_assign", "test_fr_sub_assign", "test_fr_mul_assign", "test_fr_squaring",
              "test_fr_from_into_repr", "test_fr_legendre"):
        kats[t] = [["%016x" % w for w in a] for a in fr_repr_arrays(test_body(src, t))]
    for fname, tests in (
        ("fq.rs", ["test_fq_mul_assign", "test_fq_squaring"]),
        ("fq2.rs", ["test_fq2_squaring", "test_fq2_mul", "test_fq2_inverse"]),
        ("ec.rs", ["test_g1_addition_correctness", "test_g1_doubling_correctness",
                   "test_g2_addition_correctness", "test_g2_doubling_correctness"]),
    ):
        src = open(os.path.join(REF, fname)).read()
        for t in tests:
            arrs = repr_arrays(test_body(src, t))
            kats[t] = [["%016x" % w for w in a] for a in arrs]
    src = open(os.path.join(REF, "tests", "mod.rs")).read()
    body = test_body(src, "test_pairing_result_against_relic")
    kats["relic_pairing_g1_g2"] = re.findall(r'from_str\("(\d+)"\)', body)
    assert len(kats["relic_pairing_g1_g2"]) == 12
    with open(os.path.join(HERE, "kat_limbs.json"), "w") as f:
        json.dump(kats, f, indent=1)

    dat = {}
    for fn, size in (("g1_uncompressed_valid_test_vectors.dat", 96),
                     ("g1_compressed_valid_test_vectors.dat", 48),
                     ("g2_uncompressed_valid_test_vectors.dat", 192),
                     ("g2_compressed_valid_test_vectors.dat", 96)):
        b = open(os.path.join(REF, "tests", fn), "rb").read()
        dat[fn] = {
            "record_size": size,
            "records": len(b) // size,
            "sha256": hashlib.sha256(b).hexdigest(),
            "first_records_hex": [b[k * size:(k + 1) * size].hex() for k in range(8)],
        }
    with open(os.path.join(HERE, "dat_vectors.json"), "w") as f:
        json.dump(dat, f, indent=1)
    print("wrote", sorted(kats), sorted(dat))


if __name__ == "__main__":
    main()
