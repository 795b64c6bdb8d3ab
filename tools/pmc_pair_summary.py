#!/usr/bin/env python3
"""Summarize the r05 co-residency counter passes (tools/gpu_session.sh pmcpair):
per configuration (variant, n) and per kernel, the LAST dispatch's counters of
each pass (the warm-up dispatch comes first), plus derived ratios; for the
leaf probe (tools/icache_probe) the K=1 / K=16 loops at 1 and 2 waves per SIMD.
Usage: tools/pmc_pair_summary.py [gpurun_out/pmcpair]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcpair"


def load(d):
    """dispatch id -> (kernel, grid, {counter: summed value})"""
    out = collections.OrderedDict()
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                did = int(r["Dispatch_Id"])
                k = out.setdefault(did, [r["Kernel_Name"], int(r["Grid_Size"]), {}])
                # duplicated rows (one per counter instance after reduction) are identical: keep one
                k[2][r["Counter_Name"]] = float(r["Counter_Value"])
    return out


def merged(cfg):
    """kernel name -> counters of its last dispatch, merged over the passes"""
    res = collections.OrderedDict()
    for p in sorted(glob.glob(os.path.join(root, cfg + "_p*"))):
        for did, (name, grid, ctr) in load(p).items():
            if "pa_gen" not in name:
                continue
            res.setdefault(name, {}).update(ctr)
    return res


def derived(c):
    d = {}
    w = c.get("SQ_WAVES")
    if w:
        d["wave_cycles_per_wave(quad)"] = c["SQ_WAVE_CYCLES"] / w
        d["valu_per_wave"] = c["SQ_INSTS_VALU"] / w
        d["busy_cycles"] = c.get("SQ_BUSY_CYCLES")
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_VMEM",
                  "SQ_WAIT_INST_LDS", "SQ_INST_CYCLES_VALU", "SQ_ACTIVE_INST_VALU2"):
            if k in c:
                d[k + "/WAVE_CYCLES"] = c[k] / wc
    if c.get("SQC_ICACHE_REQ"):
        d["icache_hit_rate"] = c.get("SQC_ICACHE_HITS", 0) / c["SQC_ICACHE_REQ"]
    return d


def main():
    cfgs = sorted({os.path.basename(p).rsplit("_p", 1)[0] for p in glob.glob(os.path.join(root, "v*_p*"))})
    for cfg in cfgs:
        for name, c in merged(cfg).items():
            print("== %s  %s" % (cfg, name))
            for k in sorted(c):
                print("   %-32s %18.1f" % (k, c[k]))
            for k, v in derived(c).items():
                print("   %-44s %12.4f" % (k, v) if isinstance(v, float) else "   %-44s %s" % (k, v))
    # the leaf probe: dispatch order is (W in 1, 2) x (K in 1,4,8,16,32,64) x (warm-up, timed)
    ks = [1, 4, 8, 16, 32, 64]
    per = collections.defaultdict(dict)
    for p in sorted(glob.glob(os.path.join(root, "probe_p*"))):
        ds = [v for v in load(p).values() if v[0].startswith("k")]
        for idx, (name, grid, ctr) in enumerate(ds):
            W = 1 + idx // (2 * len(ks))
            K = ks[(idx // 2) % len(ks)]
            if idx % 2 == 1:
                per[(W, K)].update(ctr)
    for (W, K), c in sorted(per.items()):
        if K not in (1, 16):
            continue
        print("== probe waves/SIMD=%d K=%d" % (W, K))
        for k in sorted(c):
            print("   %-32s %18.1f" % (k, c[k]))
        for k, v in derived(c).items():
            print("   %-44s %12.4f" % (k, v) if isinstance(v, float) else "   %-44s %s" % (k, v))


if __name__ == "__main__":
    main()
