#!/usr/bin/env python3
"""HBM bytes per launch of the pairing kernels from a `gpu_session.sh pmccsv`
run (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, CSV):
bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (FETCH_SIZE counts half of
wide coalesced reads on gfx950, MI355X_MICROARCH.md section HBM).  Prints the
per-kernel table and, with --update, writes the entries bench.py reads into
profiles/pmc_traffic.json.

  python tools/pmc_traffic.py gpurun_out [--update NOTE]"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"pa_gen_final_exp": "final_exponentiation", "pa_gen_miller_loop": "miller_loop_fused",
        "pa_gen_final_exp2": "final_exponentiation_lane_pairs", "pa_gen_miller_loop2": "miller_loop_fused_lane_pairs",
        "pa_gen_miller_loop2p": "miller_loop_fused_lane_pairs_pairing_only"}


def load(path, counter):
    acc = collections.defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r.get("Counter_Name") == counter:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d = sys.argv[1]
    f = load(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w = load(os.path.join(d, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {}
    for k in sorted(f):
        b = (2 * f[k] + w.get(k, 0.0)) * 1024
        out[k] = b
        print("%-34s fetch %12.0f KB  write %12.0f KB  -> %10.1f MB per launch" % (k[:34], f[k], w.get(k, 0), b / 1e6))
    if "--update" in sys.argv:
        note = sys.argv[sys.argv.index("--update") + 1]
        path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        with open(path) as fh:
            j = json.load(fh)
        for kern, key in KEYS.items():
            if kern in out:
                j[key] = round(out[kern], 1)
        j["_source"] = note
        with open(path, "w") as fh:
            json.dump(j, fh, indent=1)
        print("updated", path)


if __name__ == "__main__":
    main()
