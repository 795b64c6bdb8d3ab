#!/usr/bin/env python3
"""VALU instruction counts per launch from a `gpu_session.sh pmcdec` / `pmcmsm`
run (rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... --output-format csv).
SQ_INSTS_VALU counts wave-instructions summed over the launch's waves, so
SQ_INSTS_VALU / SQ_WAVES is the VALU instructions one wave (one lane's record,
for the one-record-per-lane decode kernels) issues.  With --update the entries
bench.py reads go into profiles/pmc_valu.json.

  python tools/pmc_valu.py gpurun_out/pmc_dec [--update NOTE]"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"k_decode<2, true>": "g2_decode_compressed", "k_decode<1, true>": "g1_decode_compressed",
        "k_msm_chunk_acc_fl": "g1_msm_chunk_acc", "k_msm_horner_fl": "g1_msm_horner"}


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(os.path.join(d, "run_counter_collection.csv")) as fh:
        for r in csv.DictReader(fh):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for kern, cs in acc.items():
        c = {k: sum(v) / len(v) for k, v in cs.items()}
        if "SQ_INSTS_VALU" not in c or not c.get("SQ_WAVES"):
            continue
        ipw = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        busy = c.get("SQ_WAVE_CYCLES", 0.0)
        print("%-60s waves %8.0f  VALU/wave %12.0f  wait %5.1f%%" % (
            kern[:60], c["SQ_WAVES"], ipw, 100.0 * c.get("SQ_WAIT_ANY", 0.0) / busy if busy else 0.0))
        for pat, key in KEYS.items():
            if pat in kern:
                out[key] = {"valu_instructions_per_wave": round(ipw, 1), "waves": c["SQ_WAVES"],
                            "salu_instructions_per_wave": round(c.get("SQ_INSTS_SALU", 0.0) / c["SQ_WAVES"], 1)}
    if "--update" in sys.argv:
        note = sys.argv[sys.argv.index("--update") + 1]
        path = os.path.join(ROOT, "profiles", "pmc_valu.json")
        j = {}
        if os.path.exists(path):
            with open(path) as fh:
                j = json.load(fh)
        j.update(out)
        j["_source"] = note
        with open(path, "w") as fh:
            json.dump(j, fh, indent=1)
        print("updated", path)


if __name__ == "__main__":
    main()
