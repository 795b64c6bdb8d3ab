#!/usr/bin/env python3
"""Benchmark: BLS12-381 pairings/sec at batch 2^16 per GPU (BASELINE.json).

  python bench.py --gpus N --steps K --warmup W
  (N > 1: one rank per GPU over RCCL.  Under torch.distributed.run the ranks
  come from WORLD_SIZE/RANK/LOCAL_RANK; run directly with N > 1, bench.py
  first checks that N devices are visible and then starts the N ranks itself
  as a torch.distributed.run child, before anything touches the GPU.)

A step = one batch of 2^16 independent pairings e(P_i, Q_i) per GPU, inputs
(G1Affine, G2Affine records) already resident in HBM: the fused
prepare+Miller-loop kernel, then the final-exponentiation kernel, then (N > 1)
one RCCL gather of every rank's 2^16 Fq12 results to rank 0 -- the shard is
independent work (weak scaling), the gather is the path's only exchange.

Rank 0 prints one JSON line with the driver's fields plus
  roofline      -- the dominant kernel's algorithmic HBM bytes per launch over
                   its HIP-event-measured average duration, vs 8 TB/s;
                   `traffic` = PMC-measured HBM bytes per launch from
                   profiles/ when that summary exists.
  cpu_baseline  -- the C restatement of the reference (oracle/, the CPU path
                   of the reference's algorithms) timed on this host's cores
                   over a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# v_mad_u64_u32 issue ceiling, measured at 1, 2, 4 and 8 waves per SIMD
# (tools/valu_peak.hip, profiles/r03_valu_peak.txt): the best sustained rate,
# 8 waves per SIMD, 8 independent chains -> limb multiply-accumulates per
# second.  The pairing kernels run ONE wave per SIMD at batch 2^16 (2^16 lanes
# = 1024 waves = the chip's 1024 SIMDs), whose own ceiling is VALU_MAC_1WAVE_T.
VALU_MAC_PEAK_T = 35.96
VALU_MAC_1WAVE_T = 21.32
# two waves per SIMD (the lane-pair kernels at 2^16), same probe
# (profiles/r03_valu_peak.txt)
VALU_MAC_2WAVE_T = 29.12
# issue ceiling of the one-wave-per-SIMD pairing kernels: one wave issues at most
# one instruction per 4 clk (SQ: one ACTIVE_INST quad-cycle per instruction), at
# the 2.33 GHz the chip holds under them (GRBM_GUI_ACTIVE, profiles/r02_cyc_probe.txt)
ISSUE_PEAK_T = 1024 * 64 / 4 * 2.33e9 / 1e12
# the same at the ~2.15 GHz two dense waves per SIMD leave (GRBM_GUI_ACTIVE per
# dispatch, profiles/r05_coresidency.md): the lane-pair kernels' practical ceiling
ISSUE_2WAVE_T = 1024 * 64 / 4 * 2.15e9 / 1e12
FQ12_BYTES = 576
G1A_BYTES, G2A_BYTES = 104, 200  # ABI records (coordinates + infinity flag + pad)
# algorithmic HBM bytes per pairing, per kernel (DESIGN.md "Roofline")
ML_BYTES = 96 + 192 + 2 + FQ12_BYTES   # P, Q coordinates + flags in, f out
FE_BYTES = FQ12_BYTES + FQ12_BYTES     # f in, e(P,Q) out
G2P_BYTES = 68 * 3 * 96 + 8            # G2Prepared record: 68 (Fq2, Fq2, Fq2) lines + infinity word
ML_PREP_BYTES = G1A_BYTES + G2P_BYTES + FQ12_BYTES
# one prepared Q for the batch: per pairing only P in and the Fq12 out (the
# 22.9 KB line table is read from L2 by every wave, once per call from HBM)
ML_SHARED_BYTES = G1A_BYTES + FQ12_BYTES


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1 << 16, help="pairings per GPU per step")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="a fixed global batch split over the ranks (contiguous shards, every workload but "
                         "verify; "
                         "pairing_amd/shard.py) instead of --batch per GPU; BASELINE config 5 is "
                         "--gpus 8 --global-batch 1048576")
    ap.add_argument("--stub-echo", action="store_true",
                    help="with --cpu-stub: each rank echoes its shard instead of computing pairings "
                         "(plumbing test of large shapes)")
    ap.add_argument("--workload", choices=["pairing", "prepared", "prepared_shared", "fq_mul", "fr_mul", "wnaf", "decode", "msm", "verify"],
                    default="pairing")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="target CPU-work seconds for cpu_baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--decode", action="store_true",
                    help="verify: start from the pairs' compressed encodings and decode them (checked: "
                         "on-curve + subgroup, ec.rs:785-837, 1448-1509) before the multi_pairing")
    ap.add_argument("--layout", choices=["aos", "soa"], default="aos",
                    help="fq_mul: device layout of the operands (SURVEY.md 8(d) config 2 names SoA)")
    ap.add_argument("--cpu-stub", action="store_true",
                    help="launcher test only: gloo ranks on the CPU, the oracle as the per-rank compute "
                         "(tests/test_bench_launcher.py); not a measurement")
    return ap.parse_args()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """--gpus N > 1 without a torch.distributed.run environment: start the N
    ranks as a child torch.distributed.run (one process per GPU, rendezvous on
    127.0.0.1) and return its exit code.  Nothing here touches the GPU:
    torch.cuda.device_count() does not initialise it on this image.  Returns
    None when this process is itself a rank (or N == 1)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    if not args.cpu_stub:
        import torch
        visible = torch.cuda.device_count()
        if visible < args.gpus:
            print("bench.py: --gpus %d but only %d device(s) visible" % (args.gpus, visible), file=sys.stderr)
            return 2
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    return subprocess.call(cmd)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def make_pairs(n, rank, seed=0, span=None):
    """2^16 pairs tiled from a pool of 256 x 256 distinct point combinations,
    1/128 of them with an infinity side (mod.rs:50-54).  Rows rank*n ..
    rank*n + n of the global sequence, or rows span = (start, stop) (a rank's
    shard of a --global-batch): each rank builds only its own rows."""
    d = np.load(os.path.join(ROOT, "tests", "golden", "bench_points.npz"))
    g1, g2 = d["g1"], d["g2"]
    if span is not None:
        idx = np.arange(span[0], span[1], dtype=np.int64) + seed
    else:
        idx = np.arange(n, dtype=np.int64) + rank * n + seed
    p = g1[idx % 256].copy()
    q = g2[(idx // 256 + idx * 7) % 256].copy()
    inf = np.nonzero(idx % 128 == 5)[0]
    p[inf, :] = 0
    one = [0x760900000002fffd, 0xebf4000bc40c0002, 0x5f48985753c758ba,
           0x77ce585370525745, 0x5c071a97a256ec6d, 0x15f65ec3fa80e493]
    p[inf, 6:12] = np.array(one, dtype=np.uint64)
    p[inf, 12] = 1
    return p, q


def kernel_variant_label(n):
    """the pairing kernels a batch of n per GPU runs on (capi.hip: PA_PAIRING_KERNEL 0 = by
    batch size: (PA_PQ_MIN, PA_PQ_MAX] lane groups, <= PA_COOP_MAX cooperative quad VM,
    <= PA_PAIR_MAX generated lane pairs, <= PA_PAIR_MAX + PA_TAIL_MAX lane pairs for the head
    and the tail on the quad VM (<= 832 tail pairs, PA_TAIL_KIND) or the lane groups, <= PA_ONE_MAX
    generated one lane, else lane pairs again; 1 lane pairs, 2 quad VM, 3 one lane, 4 one-wave VM,
    5 lane groups)"""
    env = lambda k, d: int(os.environ.get(k, d))
    v = env("PA_PAIRING_KERNEL", "0")
    if v == 0:
        if env("PA_PQ_MIN", "768") < n <= env("PA_PQ_MAX", "4096"):
            return "lane_groups"
        if n <= env("PA_COOP_MAX", "2304"):
            return "coop"
        pair_max = env("PA_PAIR_MAX", "32768")
        if pair_max < n <= pair_max + env("PA_TAIL_MAX", "2048"):
            kind = os.environ.get("PA_TAIL_KIND", "")
            pq = kind == "pq" or (kind != "coop" and n - pair_max > 832)
            return "gen2+%s_tail" % ("lane_group" if pq else "coop")
        one = pair_max < n <= env("PA_ONE_MAX", "34048")
        return "gen" if one else "gen2"
    return {1: "gen2", 2: "coop", 3: "gen", 4: "coop1", 5: "lane_groups"}.get(v, "variant%d" % v)


def host_threads():
    """(host cores this process may run on, threads the CPU baseline uses):
    the affinity mask, capped by OMP_NUM_THREADS when the environment sets it
    (the GPU box sets 16, its CPU share per GPU)."""
    try:
        host = len(os.sched_getaffinity(0))
    except AttributeError:
        host = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(host, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else host
    return host, max(1, threads)


def _timed_pairings(oracle, p, q, threads, seconds):
    """pairings/s of the oracle on `threads` threads over a prefix of (p, q)
    sized from a calibration run to about `seconds` of wall time"""
    k = min(len(p), max(threads, 2 * threads))
    t0 = time.perf_counter()
    oracle.pairing(p[:k], q[:k], threads)
    per = max(time.perf_counter() - t0, 1e-4) / k           # wall per pairing at this thread count
    n = int(max(k, min(len(p), seconds / per)))
    t0 = time.perf_counter()
    oracle.pairing(p[:n], q[:n], threads)
    wall = time.perf_counter() - t0
    return n / wall, n, wall


def cpu_baseline_pairing(p, q, seconds):
    """The oracle (C restatement of the reference's pairing, OpenMP over
    pairs) on this host: one core, then every thread the host gives us."""
    from oracle import binding as oracle
    host, threads = host_threads()
    v1, n1, w1 = _timed_pairings(oracle, p, q, 1, max(5.0, seconds / 2))
    vt, nt, wt = (v1, n1, w1) if threads == 1 else _timed_pairings(oracle, p, q, threads, max(5.0, seconds / 2))
    # every core of the affinity mask at the measured one-core rate: an upper
    # bound (perfect scaling), reported beside the measured figures.  Not run:
    # the GPU box gives one GPU's job a 16-thread CPU share (OMP_NUM_THREADS)
    return {"value": vt, "unit": "pairings/s", "cores": threads, "kind": "port", "host_cores": host,
            "value_1core": v1, "value_all_host_cores_linear_bound": v1 * host,
            "sample": "C restatement of the reference (oracle/) over a prefix of the same synthetic batch: "
                      "%d pairings on 1 core in %.1f s; %d pairings on %d threads (OpenMP over pairs) in %.1f s; "
                      "host affinity %d cores%s; value_all_host_cores_linear_bound = value_1core x %d "
                      "(not measured: the box's CPU share per GPU job is %d threads)"
                      % (n1, w1, nt, threads, wt, host,
                         ", OMP_NUM_THREADS=%s" % os.environ["OMP_NUM_THREADS"] if os.environ.get("OMP_NUM_THREADS")
                         else "", host, threads)}


def cpu_baseline_prepared(p, q, seconds):
    """The oracle's miller_loop over materialized G2Prepared + final
    exponentiation (the prepare itself outside the timing, as on the GPU),
    one core then every thread, over a prefix of the same batch"""
    from oracle import binding as oracle
    host, threads = host_threads()
    res = []
    for th in sorted({1, threads}):
        k = 2 * th
        t0 = time.perf_counter()
        oracle.final_exponentiation(oracle.miller_loop_batch(p[:k], oracle.g2_prepare(q[:k], th), th), th)
        per = max(time.perf_counter() - t0, 1e-4) / k
        m = int(max(k, min(len(p), max(5.0, seconds / 2) / per)))
        prep = oracle.g2_prepare(q[:m], th)
        t0 = time.perf_counter()
        oracle.final_exponentiation(oracle.miller_loop_batch(p[:m], prep, th), th)
        wall = time.perf_counter() - t0
        res.append((th, m / wall, m, wall))
    v1 = res[0][1]
    th, vt, mt, wt = res[-1]
    return {"value": vt, "unit": "pairings/s", "cores": th, "kind": "port", "host_cores": host, "value_1core": v1,
            "sample": "C restatement of the reference (oracle/): miller_loop_batch over prepared records + "
                      "final_exponentiation, %d pairs on 1 core in %.1f s; %d pairs on %d threads in %.1f s"
                      % (res[0][2], res[0][3], mt, th, wt)}


def cpu_baseline_prepared_shared(p, prep1, seconds):
    """The oracle's miller_loop of every P_i against ONE prepared Q (the record
    repeated per pair, as the reference's &G2Prepared in each pair) + final
    exponentiation, one core then every thread, over a prefix of the batch"""
    from oracle import binding as oracle
    host, threads = host_threads()

    def run(m, th):
        for k in range(0, m, 4096):
            pc = p[k:min(m, k + 4096)]
            oracle.final_exponentiation(oracle.miller_loop_batch(pc, np.repeat(prep1, len(pc), axis=0), th), th)
    res = []
    for th in sorted({1, threads}):
        k = 2 * th
        t0 = time.perf_counter()
        run(k, th)
        per = max(time.perf_counter() - t0, 1e-4) / k
        m = int(max(k, min(len(p), max(5.0, seconds / 2) / per)))
        t0 = time.perf_counter()
        run(m, th)
        wall = time.perf_counter() - t0
        res.append((th, m / wall, m, wall))
    v1 = res[0][1]
    th, vt, mt, wt = res[-1]
    return {"value": vt, "unit": "pairings/s", "cores": th, "kind": "port", "host_cores": host, "value_1core": v1,
            "sample": "C restatement of the reference (oracle/): miller_loop_batch of P_i against one prepared Q "
                      "+ final_exponentiation, %d pairs on 1 core in %.1f s; %d pairs on %d threads in %.1f s"
                      % (res[0][2], res[0][3], mt, th, wt)}


def cpu_baseline_decode(enc1, enc2, seconds):
    """The reference's into_affine for compressed G2 + G1 records, restated in C (OpenMP over records)."""
    from oracle import binding as oracle
    _, threads = host_threads()
    t0 = time.perf_counter()
    oracle.decode(2, enc2[:threads], True, True, threads)
    oracle.decode(1, enc1[:threads], True, True, threads)
    per = max(time.perf_counter() - t0, 1e-4)
    n = int(max(threads, min(len(enc1), threads * seconds / per)))
    t0 = time.perf_counter()
    oracle.decode(2, enc2[:n], True, True, threads)
    oracle.decode(1, enc1[:n], True, True, threads)
    wall = time.perf_counter() - t0
    return {"value": n / wall, "unit": "point pairs/s", "cores": threads, "kind": "port",
            "sample": "%d G2+G1 compressed records of the same batch, C restatement of the reference "
                      "(oracle/), OpenMP over records, %.1f s wall" % (n, wall)}


def cpu_baseline_wnaf(base, scalars, seconds):
    """The reference's Wnaf (window 16 at 2^18 scalars) + batch_normalization, restated in C."""
    from oracle import binding as oracle
    _, threads = host_threads()
    n = min(len(scalars), 131072)
    t0 = time.perf_counter()
    out = oracle.g1_wnaf_fixed_base(base, np.ascontiguousarray(scalars[:n]), threads)
    oracle.g1_batch_normalization(out)
    wall = time.perf_counter() - t0
    return {"value": n / wall, "unit": "points/s", "cores": threads, "kind": "port",
            "sample": "%d scalars, reference wNAF (window for that count) + batch_normalization, C "
                      "restatement, OpenMP over scalars, %.1f s wall" % (n, wall)}


def _check_work_json(work_path):
    """The VALU roofline's MAC count comes from pa_gen_work.json, written by
    tools/pgen/build_gen.py next to the code objects it counts.  A missing file
    or one older than those code objects would price the kernels with stale
    counts, so fail loudly instead of reporting a roofline."""
    if not os.path.exists(work_path):
        raise SystemExit("bench.py: %s is missing (run `make -C pairing_amd`)" % work_path)
    lib = os.path.dirname(work_path)
    t = os.path.getmtime(work_path)
    for co in ("pa_gen_miller_loop.hsaco", "pa_gen_final_exp.hsaco"):
        cp = os.path.join(lib, co)
        # code objects are written first, the work file right after them
        if os.path.exists(cp) and os.path.getmtime(cp) > t + 60:
            raise SystemExit("bench.py: %s is older than %s (rebuild with `make -C pairing_amd`)"
                             % (work_path, cp))


def measure_copy_gbs(nbytes, dev, stream, reps=20):
    """Device-to-device copy of nbytes/2 (nbytes moved: half read, half
    written) timed with HIP events: the achievable streaming rate on this box."""
    import torch
    half = max(1, nbytes // 2 // 8)
    src = torch.empty(half, dtype=torch.int64, device=dev)
    dst = torch.empty_like(src)
    src.fill_(1)
    dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        dst.copy_(src)
    e1.record(stream)
    torch.cuda.synchronize()
    return 2 * half * 8 * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9


def cpu_baseline_fq_mul(a, b, seconds):
    from oracle import binding as oracle
    n = min(len(a), 1 << 20)
    t0 = time.perf_counter()
    oracle.fq_mul(a[:n], b[:n])
    wall = time.perf_counter() - t0
    return {"value": n / wall, "unit": "muls/s", "cores": 1, "kind": "port",
            "sample": "%d Fq::mul_assign, C restatement (oracle/), 1 thread" % n}


def cpu_baseline_fr_mul(a, b):
    from oracle import binding as oracle
    n = min(len(a), 1 << 20)
    t0 = time.perf_counter()
    oracle.fr_mul(np.ascontiguousarray(a[:n]), np.ascontiguousarray(b[:n]))
    wall = time.perf_counter() - t0
    return {"value": n / wall, "unit": "muls/s", "cores": 1, "kind": "port",
            "sample": "%d Fr::mul_assign, C restatement (oracle/), 1 thread" % n}


def cpu_baseline_msm(base, k, s, seconds):
    """The reference-style sum of CurveAffine::mul terms (C restatement), OpenMP over terms,
    on a bounded prefix of the same bases (k_i * G, made by the oracle)."""
    from oracle import binding as oracle
    _, threads = host_threads()
    m = 64 * threads
    pts = oracle.g1_mul_generator(np.ascontiguousarray(k[:m]), threads)
    t0 = time.perf_counter()
    oracle.g1_multiexp(pts, np.ascontiguousarray(s[:m]), threads)
    per = max(time.perf_counter() - t0, 1e-4) / m
    m2 = int(max(m, min(len(k), 0.5 * seconds / per)))
    if m2 > m:
        pts = oracle.g1_mul_generator(np.ascontiguousarray(k[:m2]), threads)
        m = m2
    t0 = time.perf_counter()
    oracle.g1_multiexp(pts, np.ascontiguousarray(s[:m]), threads)
    wall = time.perf_counter() - t0
    return {"value": m / wall, "unit": "terms/s", "cores": threads, "kind": "port",
            "sample": "%d terms: CurveAffine::mul per term + add_assign, C restatement (oracle/), "
                      "OpenMP over terms, %.1f s wall" % (m, wall)}


def main_cpu_stub(args, ws, rank):
    """Launcher test: the same rank/shard/gather/timing structure on gloo with
    the oracle as each rank's compute (no GPU).  Not a measurement."""
    import torch
    import torch.distributed as dist
    from oracle import binding as oracle
    from pairing_amd.shard import gather_rows_to_root
    from pairing_amd.shard import shard_range
    if ws > 1:
        dist.init_process_group("gloo")
    if args.global_batch:
        span = shard_range(args.global_batch, ws, rank)
        n, n_global = span[1] - span[0], args.global_batch
    else:
        span, n, n_global = None, args.batch, args.batch * ws
    p_np, q_np = make_pairs(n, rank, span=span)

    def step():
        if args.stub_echo:
            out = torch.zeros((n, 72), dtype=torch.int64)
            out[:, :13] = torch.from_numpy(p_np.view(np.int64))
        else:
            out = torch.from_numpy(oracle.pairing(p_np, q_np, 1).view(np.int64))
        if ws > 1:
            res = gather_rows_to_root(out, n_global)
            if rank == 0 and res.shape[0] != n_global:
                raise RuntimeError("gathered %d rows, global batch %d" % (res.shape[0], n_global))

    for _ in range(args.warmup):
        step()
    if ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if ws > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if ws > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "launcher test (cpu stub)", "value": n_global * args.steps / elapsed,
                          "unit": "pairings/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": None, "dtype": "u64", "data": "cpu stub: oracle per rank, gloo gather",
                          "config": {"workload": "cpu stub", "batch_per_gpu": n, "global_batch": n_global,
                                     "parallelism": "shard%d+gather" % ws if ws > 1 else "single"}}), flush=True)
    if ws > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    rc = launch_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    ws, rank, local = dist_env()
    # under torch.distributed.run (WORLD_SIZE set) every rank joins the RCCL
    # group and gathers, even at one rank: `torch.distributed.run
    # --nproc-per-node 1 bench.py` runs the sharded path on a one-GPU box
    dist_on = ws > 1 or "WORLD_SIZE" in os.environ
    if ws != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d; timing %d ranks" % (ws, args.gpus, ws), file=sys.stderr)
    if args.cpu_stub:
        return main_cpu_stub(args, ws, rank)
    import torch
    import torch.distributed as dist
    import pairing_amd
    import pairing_amd.device as pdev

    torch.cuda.set_device(local)
    pairing_amd.set_device(local)
    if os.environ.get("PA_PAIRING_KERNEL"):
        pairing_amd.set_pairing_kernel(int(os.environ["PA_PAIRING_KERNEL"]))
    dev = torch.device("cuda", local)
    if dist_on:
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()

    def drain():
        """wait for outstanding asynchronous gathers (the pairing workload
        redefines it when it runs them)"""

    stream = torch.cuda.current_stream()
    n = args.batch
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    k_ms = {"a": [], "b": [], "c": []}

    n_global = n * ws
    from pairing_amd.shard import gather_rows_to_root, shard_range

    def shard(per_rank):
        """(n, n_global, rows of the global sequence this rank owns): weak
        scaling (per_rank rows per rank) or, with --global-batch, the rank's
        contiguous shard of the fixed global batch -- each rank builds and
        stages only its own rows"""
        if args.global_batch:
            a, b = shard_range(args.global_batch, ws, rank)
            return b - a, args.global_batch, np.arange(a, b, dtype=np.int64)
        return per_rank, per_rank * ws, np.arange(rank * per_rank, (rank + 1) * per_rank, dtype=np.int64)

    if args.workload == "pairing":
        span = None
        if args.global_batch:
            # config 5 shape: a fixed global batch in contiguous shards, each
            # rank building and staging only its own rows
            span = shard_range(args.global_batch, ws, rank)
            n, n_global = span[1] - span[0], args.global_batch
        p_np, q_np = make_pairs(n, rank, span=span)
        p = torch.from_numpy(p_np.view(np.int64)).to(dev)
        q = torch.from_numpy(q_np.view(np.int64)).to(dev)
        outs = [pdev.empty_records(n, 72, dev) for _ in range(2 if dist_on else 1)]
        scratch = pdev.empty_records(n, 72, dev)
        if dist_on:
            from pairing_amd.shard import RowGatherer
            gatherer = RowGatherer(n_global, 72, outs[0])
        works = [None, None]
        nstep = [0]

        def step(timed):
            # multi-GPU: results double-buffered, each batch's gather to rank 0
            # (the path's one exchange, RCCL over xGMI) runs while the next
            # batch computes; a buffer is rewritten only after its gather is done
            slot = nstep[0] % len(outs)
            nstep[0] += 1
            out = outs[slot]
            if timed:
                ev[0].record(stream)
            # pa_pairing_batch_device's two stages, timed apart
            pdev.pairing_miller_loop(p, q, scratch, stream)
            if timed:
                ev[1].record(stream)
            if works[slot] is not None:
                works[slot].wait()
                works[slot] = None
            pdev.final_exponentiation(scratch, out, None, stream)
            if timed:
                ev[2].record(stream)
            if dist_on:
                works[slot] = gatherer.gather(out, slot)

        def drain():
            for k, w in enumerate(works):
                if w is not None:
                    w.wait()
                    works[k] = None
    elif args.workload == "prepared":
        # the north-star's own call shape: Bls12::miller_loop over (G1Affine,
        # G2Prepared) pairs + final_exponentiation, the G2Prepared records (68
        # line coefficients each, 19 592 B) materialized in HBM once before the
        # timed region (G2Affine::prepare, timed separately below)
        from pairing_amd._native import W_G2P
        span = shard_range(args.global_batch, ws, rank) if args.global_batch else None
        if span:
            n, n_global = span[1] - span[0], args.global_batch
        p_np, q_np = make_pairs(n, rank, span=span)
        p = torch.from_numpy(p_np.view(np.int64)).to(dev)
        q = torch.from_numpy(q_np.view(np.int64)).to(dev)
        qp = pdev.empty_records(n, W_G2P, dev)
        out = pdev.empty_records(n, 72, dev)
        scratch = pdev.empty_records(n, 72, dev)
        prep_ms = []
        for _ in range(3):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record(stream)
            pdev.g2_prepare(q, qp, stream)
            e[1].record(stream)
            torch.cuda.synchronize()
            prep_ms.append(e[0].elapsed_time(e[1]))

        def step(timed):
            if timed:
                ev[0].record(stream)
            pdev.miller_loop_prepared(p, qp, scratch, stream)
            if timed:
                ev[1].record(stream)
            pdev.final_exponentiation(scratch, out, None, stream)
            if timed:
                ev[2].record(stream)
            if dist_on:
                gather_rows_to_root(out, n_global)
    elif args.workload == "prepared_shared":
        # the verifier's fixed-key shape: every P_i against ONE prepared Q
        # (Engine::miller_loop with the same &G2Prepared in each pair,
        # lib.rs:88-96); the record is prepared once before the timed region
        from pairing_amd._native import W_G2P
        span = shard_range(args.global_batch, ws, rank) if args.global_batch else None
        if span:
            n, n_global = span[1] - span[0], args.global_batch
        p_np, q_np = make_pairs(n, rank, span=span)
        q1_np = q_np[[i for i in range(len(q_np)) if not q_np[i, 24] & 0xff][:1]]
        p = torch.from_numpy(p_np.view(np.int64)).to(dev)
        qp = pdev.empty_records(1, W_G2P, dev)
        pdev.g2_prepare(torch.from_numpy(q1_np.view(np.int64)).to(dev), qp, stream)
        torch.cuda.synchronize()
        prep1_np = qp.cpu().numpy().view(np.uint64)
        out = pdev.empty_records(n, 72, dev)
        scratch = pdev.empty_records(n, 72, dev)

        def step(timed):
            if timed:
                ev[0].record(stream)
            pdev.miller_loop_shared_prepared(p, qp, scratch, stream)
            if timed:
                ev[1].record(stream)
            pdev.final_exponentiation(scratch, out, None, stream)
            if timed:
                ev[2].record(stream)
            if dist_on:
                gather_rows_to_root(out, n_global)
    elif args.workload == "wnaf":
        # config 3: Wnaf::new().base(g, 2^18).scalar(s_i) + G1::batch_normalization
        n, n_global, idx = shard(args.batch if args.batch != (1 << 16) else (1 << 18))
        d = np.load(os.path.join(ROOT, "tests", "golden", "bench_points.npz"))
        base_np = np.zeros((1, 18), np.uint64)
        base_np[0, :12] = d["g1"][0, :12]
        base_np[0, 12:18] = np.array([0x760900000002fffd, 0xebf4000bc40c0002, 0x5f48985753c758ba,
                                      0x77ce585370525745, 0x5c071a97a256ec6d, 0x15f65ec3fa80e493], np.uint64)
        # scalars split over the ranks, every rank its own table (Wnaf::shared(), wnaf.rs:131-154)
        s_np = np.ascontiguousarray(d["s1"][idx % 256])
        s_np[:, 0] ^= idx.astype(np.uint64) << np.uint64(8)
        base = torch.from_numpy(base_np.view(np.int64)).to(dev)
        scal = torch.from_numpy(s_np.view(np.int64)).to(dev)
        out = pdev.empty_records(n, 18, dev)
        fb_table, fb_ws = pdev.fixed_base_buffers(dev)

        def step(timed):
            # one Wnaf::base(g, n).scalar(s_i) call: table build overlapped with
            # the multiply (pa_g1_wnaf_fixed_base_device), then normalization
            if timed:
                ev[0].record(stream)
            pdev.g1_wnaf_fixed_base(base, scal, out, fb_table, fb_ws, stream)
            if timed:
                ev[1].record(stream)
            pdev.g1_batch_normalization(out, stream)
            if timed:
                ev[2].record(stream)
            if dist_on:
                gather_rows_to_root(out, n_global)

        def comb_parts_ms(reps=3):
            """the GLV table build and the GLV comb multiply as separate
            stream-ordered launches (untimed region): the dominant kernel's own
            duration for the roofline"""
            t_ms, m_ms = [], []
            table, ws = pdev.fixed_base_buffers(dev)
            for _ in range(reps):
                e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                e[0].record(stream)
                pdev.g1_fixed_base_glv_table(base, table, ws, stream)
                e[1].record(stream)
                pdev.g1_fixed_base_glv_mul(base, table, ws, scal, out, stream)
                e[2].record(stream)
                torch.cuda.synchronize()
                t_ms.append(e[0].elapsed_time(e[1]))
                m_ms.append(e[1].elapsed_time(e[2]))
            return float(np.mean(t_ms)), float(np.mean(m_ms))

        def exact_ms(reps=3):
            """the bit-exact form (the reference's table chain, wnaf_form and
            wnaf_exp: pa_g1_wnaf_fixed_base_exact_device) on the same scalars,
            untimed region, for comparison with the comb"""
            w = int(pdev._lib.pa_g1_recommended_wnaf_for_num_scalars(n))
            ws_x = pdev.wnaf_exact_workspace(1, n, w, False, dev)
            out_x = pdev.empty_records(n, 18, dev)
            t = []
            for _ in range(reps):
                e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                e[0].record(stream)
                pdev.wnaf_fixed_base_exact(1, base, scal, out_x, w, ws_x, stream)
                e[1].record(stream)
                torch.cuda.synchronize()
                t.append(e[0].elapsed_time(e[1]))
            del ws_x, out_x
            return float(np.median(t))
    elif args.workload == "decode":
        # SURVEY.md §8 f rank 1: the verifier's front end -- compressed G1 and G2
        # records decoded with the on-curve (square root) and subgroup (r*P) checks
        n, n_global, idx = shard(n)
        p_np, q_np = make_pairs(n, rank, span=(int(idx[0]), int(idx[-1]) + 1) if n else (0, 0))
        enc1_np = pairing_amd.g1_encode(p_np, True)
        enc2_np = pairing_amd.g2_encode(q_np, True)
        enc1 = torch.from_numpy(enc1_np).to(dev)
        enc2 = torch.from_numpy(enc2_np).to(dev)
        out1 = pdev.empty_records(n, 13, dev)
        out2 = pdev.empty_records(n, 25, dev)
        st1 = torch.empty(n, dtype=torch.uint8, device=dev)
        st2 = torch.empty(n, dtype=torch.uint8, device=dev)

        def step(timed):
            if timed:
                ev[0].record(stream)
            pdev.decode(2, enc2, True, True, out2, st2, stream)
            if timed:
                ev[1].record(stream)
            pdev.decode(1, enc1, True, True, out1, st1, stream)
            if timed:
                ev[2].record(stream)
            if dist_on:
                gather_rows_to_root(out2, n_global)
                gather_rows_to_root(out1, n_global)
    elif args.workload == "msm":
        # SURVEY.md §8 f rank 3: one G1 multi-scalar multiplication of 2^20 terms
        # (the prover's multiexp).  Distinct bases k_i*G made on the device
        # (fixed-base comb + batch_normalization), random 255-bit scalars.
        # one MSM over n_global terms: each rank sums its shard's terms, the
        # root adds one partial sum per rank (shard.sharded_reduce's shape)
        n, n_global, idx = shard(args.batch if args.batch != (1 << 16) else (1 << 20))
        d = np.load(os.path.join(ROOT, "tests", "golden", "bench_points.npz"))
        base_np = np.zeros((1, 18), np.uint64)
        base_np[0, :12] = d["g1"][0, :12]
        base_np[0, 12:18] = np.array([0x760900000002fffd, 0xebf4000bc40c0002, 0x5f48985753c758ba,
                                      0x77ce585370525745, 0x5c071a97a256ec6d, 0x15f65ec3fa80e493], np.uint64)
        g = np.random.default_rng(1234 + (0 if args.global_batch else rank))
        k_np = g.integers(0, 1 << 63, size=(n, 4), dtype=np.uint64)
        s_np = g.integers(0, 1 << 63, size=(n, 4), dtype=np.uint64)
        k_np[:, 0] ^= idx.astype(np.uint64)                    # distinct k_i
        k_np[:, 3] &= np.uint64(0x0fffffffffffffff)            # < r
        s_np[:, 3] &= np.uint64(0x0fffffffffffffff)
        base = torch.from_numpy(base_np.view(np.int64)).to(dev)
        kk = torch.from_numpy(k_np.view(np.int64)).to(dev)
        jac = pdev.empty_records(n, 18, dev)
        table, _ = pdev.g1_fixed_base_table(base, stream)
        pdev.g1_fixed_base_mul(table, kk, jac, stream)
        pdev.g1_batch_normalization(jac, stream)
        bases = torch.zeros((n, 13), dtype=torch.int64, device=dev)
        bases[:, :12] = jac[:, :12]
        del jac, table
        scal = torch.from_numpy(s_np.view(np.int64)).to(dev)
        msm_out = pdev.empty_records(1, 18, dev)
        msm_ws = pdev.multiexp_workspace(1, n, dev)
        if dist_on:
            parts = pdev.empty_records(ws, 18, dev) if rank == 0 else None
            total = pdev.empty_records(1, 18, dev)
        torch.cuda.synchronize()

        def step(timed):
            if timed:
                ev[0].record(stream)
            pdev.multiexp(1, bases, scal, msm_out, msm_ws, stream)
            if timed:
                ev[1].record(stream)
            if dist_on:
                # the exchange: one Jacobian partial sum (144 B) per rank to the root
                dist.gather(msm_out, list(parts.split(1)) if rank == 0 else None, dst=0)
                if rank == 0:
                    total.copy_(parts[0:1])
                    for r in range(1, ws):
                        pdev.group_add(1, total, parts[r:r + 1], total, stream)
    elif args.workload == "verify":
        # SURVEY.md §8 f rank 2, the verifier shape: one multi_pairing over a few
        # pairs (Engine::miller_loop product + final_exponentiation, mod.rs:40-160)
        # -- a latency, on the cooperative kernels (quad VM: four waves per pairing)
        n = args.batch if args.batch != (1 << 16) else 2
        p_np, q_np = make_pairs(n, rank, seed=3)
        p = torch.from_numpy(p_np.view(np.int64)).to(dev)
        q = torch.from_numpy(q_np.view(np.int64)).to(dev)
        out = pdev.empty_records(1, 72, dev)
        okb = torch.empty(1, dtype=torch.uint8, device=dev)
        work = pdev.empty_records(n, 72, dev)
        if args.decode:
            # the verifier's front end: the proof's points arrive compressed;
            # G1 decodes on a side stream beside G2, the pairing waits for both
            enc1_np = pairing_amd.g1_encode(p_np, True)
            enc2_np = pairing_amd.g2_encode(q_np, True)
            enc1 = torch.from_numpy(np.ascontiguousarray(enc1_np)).to(dev)
            enc2 = torch.from_numpy(np.ascontiguousarray(enc2_np)).to(dev)
            st1 = torch.empty(n, dtype=torch.uint8, device=dev)
            st2 = torch.empty(n, dtype=torch.uint8, device=dev)
            in1 = torch.empty(n, dtype=torch.uint8, device=dev)
            in2 = torch.empty(n, dtype=torch.uint8, device=dev)
            side, side2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
            fork, join, dec1, dec2, join2 = (torch.cuda.Event() for _ in range(5))
            # into_affine = into_affine_unchecked + the subgroup check (ec.rs:786-793,
            # 1449-1457): the pairing starts on the unchecked points and the checks run
            # beside it (pa_g{1,2}_subgroup_check_batch_device); the step ends when both
            # are done, and the statuses say whether its result stands.  PA_VERIFY_SPLIT=0:
            # checked decodes, then the pairing (A/B)
            split = os.environ.get("PA_VERIFY_SPLIT", "1") != "0"

        def step(timed):
            if timed:
                ev[0].record(stream)
            if args.decode:
                fork.record(stream)
                side.wait_event(fork)
                pdev.decode(1, enc1, True, not split, p, st1, side)
                dec1.record(side)
                if split:
                    pdev.subgroup_check(1, p, in1, side)
                pdev.decode(2, enc2, True, not split, q, st2, stream)
                if split:
                    dec2.record(stream)
                    side2.wait_event(dec2)
                    pdev.subgroup_check(2, q, in2, side2)
                stream.wait_event(dec1)
                if timed:
                    ev[2].record(stream)
            pdev.multi_pairing(p, q, out, okb, work, stream)
            if args.decode and split:
                join.record(side)
                join2.record(side2)
                stream.wait_event(join)
                stream.wait_event(join2)
            if timed:
                ev[1].record(stream)
    elif args.workload == "fr_mul":
        g = np.random.default_rng(0 if args.global_batch else rank)
        n, n_global, idx = shard(args.batch if args.batch != (1 << 16) else (1 << 20))
        a_np = g.integers(0, 1 << 63, size=(4096, 4), dtype=np.uint64)[idx % 4096]
        b_np = g.integers(0, 1 << 63, size=(4096, 4), dtype=np.uint64)[(idx * 7 + 3) % 4096]
        a_np[:, 3] &= np.uint64(0x0fffffffffffffff)
        b_np[:, 3] &= np.uint64(0x0fffffffffffffff)
        a = torch.from_numpy(np.ascontiguousarray(a_np).view(np.int64)).to(dev)
        b = torch.from_numpy(np.ascontiguousarray(b_np).view(np.int64)).to(dev)
        out = pdev.empty_records(n, 4, dev)

        def step(timed):
            if timed:
                ev[0].record(stream)
            pdev.fr_mul(a, b, out, stream)
            if timed:
                ev[1].record(stream)
            if dist_on:
                gather_rows_to_root(out, n_global)
    else:
        g = np.random.default_rng(0 if args.global_batch else rank)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from helpers import random_fq
        n, n_global, idx = shard(args.batch if args.batch != (1 << 16) else (1 << 20))
        a_np = random_fq(g, 4096)[idx % 4096]
        b_np = random_fq(g, 4096)[(idx * 7 + 3) % 4096]
        if args.layout == "soa":
            a = torch.from_numpy(np.ascontiguousarray(a_np.T).view(np.int64)).to(dev)
            b = torch.from_numpy(np.ascontiguousarray(b_np.T).view(np.int64)).to(dev)
            out = torch.empty((6, n), dtype=torch.int64, device=dev)
            mul = pdev.fq_mul_soa
        else:
            a = torch.from_numpy(a_np.view(np.int64)).to(dev)
            b = torch.from_numpy(b_np.view(np.int64)).to(dev)
            out = pdev.empty_records(n, 6, dev)
            mul = pdev.fq_mul

        def step(timed):
            if timed:
                ev[0].record(stream)
            mul(a, b, out, stream)
            if timed:
                ev[1].record(stream)
            if dist_on and args.layout != "soa":
                gather_rows_to_root(out, n_global)

    for _ in range(args.warmup):
        step(False)
    drain()
    barrier()
    t0 = time.perf_counter()
    # per-kernel durations from HIP events on the launch stream: one event set
    # per step, read after the closing synchronize (no host sync between steps)
    step_ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    for s in range(args.steps):
        ev[:] = step_ev[s]
        step(True)
    drain()      # the last batches' gathers belong to the timed region
    barrier()
    elapsed = time.perf_counter() - t0
    for e in step_ev:
        k_ms["a"].append(e[0].elapsed_time(e[1]))
        if args.workload in ("pairing", "prepared", "prepared_shared", "wnaf", "decode"):
            k_ms["b"].append(e[1].elapsed_time(e[2]))
        if args.workload == "verify" and args.decode:
            k_ms["b"].append(e[0].elapsed_time(e[2]))   # the decodes

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps

    if rank == 0:
        if args.workload == "pairing":
            ml = float(np.mean(k_ms["a"]))
            fe = float(np.mean(k_ms["b"]))
            dom_name, dom_ms, dom_bytes = ("final_exponentiation", fe, FE_BYTES) if fe >= ml else \
                ("miller_loop_fused", ml, ML_BYTES)
            value = n_global * args.steps / elapsed
            metric, unit = "BLS12-381 pairings/sec at batch 2^16", "pairings/s"
            wl = "bls12_381 e(P_i,Q_i) batch (fused G2 prepare + Miller loop + final exp)"
            if args.global_batch:
                wl += "; fixed global batch %d in %d contiguous shards (BASELINE config 5 at 2^20 over 8)" % (
                    n_global, ws)
            config = {"workload": wl,
                      "kernel_variant": kernel_variant_label(n),
                      "batch_per_gpu": n, "global_batch": n_global,
                      "parallelism": "shard%d+rccl_gather(overlapped)" % ws if dist_on else "single", "kernel_ms": {"miller_loop_fused": round(ml, 3),
                                                             "final_exponentiation": round(fe, 3)}}
        elif args.workload == "prepared":
            ml = float(np.mean(k_ms["a"]))
            fe = float(np.mean(k_ms["b"]))
            dom_name, dom_ms, dom_bytes = ("final_exponentiation", fe, FE_BYTES) if fe >= ml else \
                ("miller_loop_prepared", ml, ML_PREP_BYTES)
            value = n_global * args.steps / elapsed
            metric, unit = "BLS12-381 miller_loop(G1Affine, G2Prepared) + final_exponentiation per second " \
                           "at batch 2^16", "pairings/s"
            config = {"workload": "bls12_381 final_exponentiation(miller_loop([(P_i, Q_i.prepare())])) batch, "
                                  "G2Prepared materialized in HBM (19 592 B per pair)",
                      "batch_per_gpu": n, "global_batch": n_global,
                      "parallelism": "shard%d+rccl_gather" % ws if dist_on else "single",
                      "kernel_ms": {"miller_loop_prepared": round(ml, 3), "final_exponentiation": round(fe, 3),
                                    "untimed: g2_prepare": round(float(np.median(prep_ms)), 3)}}
        elif args.workload == "prepared_shared":
            ml = float(np.mean(k_ms["a"]))
            fe = float(np.mean(k_ms["b"]))
            dom_name, dom_ms, dom_bytes = ("final_exponentiation", fe, FE_BYTES) if fe >= ml else \
                ("miller_loop_shared", ml, ML_SHARED_BYTES)
            value = n_global * args.steps / elapsed
            metric, unit = "BLS12-381 miller_loop(G1Affine_i, one G2Prepared) + final_exponentiation per second " \
                           "at batch 2^16", "pairings/s"
            config = {"workload": "bls12_381 final_exponentiation(miller_loop([(P_i, Q)])) batch against ONE "
                                  "prepared Q (lines staged once per call, no G2 arithmetic per pair)",
                      "batch_per_gpu": n, "global_batch": n_global,
                      "parallelism": "shard%d+rccl_gather" % ws if dist_on else "single",
                      "kernel_ms": {"miller_loop_shared": round(ml, 3), "final_exponentiation": round(fe, 3)}}
        elif args.workload == "wnaf":
            tot_ms, norm_ms = float(np.mean(k_ms["a"])), float(np.mean(k_ms["b"]))
            table_ms, mul_ms = comb_parts_ms()
            x_ms = exact_ms()
            dom_name, dom_ms, dom_bytes = ("g1_glv_comb_mul", mul_ms, 32 + 144) if mul_ms >= norm_ms else \
                ("g1_batch_normalize", norm_ms, 144 + 144)
            value = n_global * args.steps / elapsed
            metric, unit = "G1 fixed-base scalar mults + batch_normalization per second at batch 2^18", "points/s"
            config = {"workload": "Wnaf::base(g, 2^18).scalar(s_i) then G1::batch_normalization",
                      "batch_per_gpu": n, "global_batch": n_global,
                      "kernel_ms": {"table+fixed_base_mul (overlapped)": round(tot_ms, 3),
                                    "batch_normalize": round(norm_ms, 3),
                                    "separately: glv table": round(table_ms, 3), "separately: glv mul": round(mul_ms, 3),
                                    "separately: bit-exact wnaf (reference chain, same scalars)": round(x_ms, 3)}}
        elif args.workload == "decode":
            g2_ms, g1_ms = float(np.mean(k_ms["a"])), float(np.mean(k_ms["b"]))
            dom_name, dom_ms, dom_bytes = ("g2_decode_compressed", g2_ms, 96 + 200 + 1) if g2_ms >= g1_ms else \
                ("g1_decode_compressed", g1_ms, 48 + 104 + 1)
            value = n_global * args.steps / elapsed
            metric, unit = "compressed G1+G2 point pairs decoded (checked) per second at batch 2^16", "point pairs/s"
            config = {"workload": "G2Compressed + G1Compressed ::into_affine (sqrt + on-curve + r*P subgroup check)",
                      "batch_per_gpu": n, "global_batch": n_global,
                      "kernel_ms": {"g2_decode": round(g2_ms, 3), "g1_decode": round(g1_ms, 3)}}
        elif args.workload == "msm":
            dom_name, dom_ms = "g1_multiexp", float(np.mean(k_ms["a"]))
            # per term: W = ceil(257/16) = 17 windows x (104 B base gather + 8 B sort key/value)
            # + 32 B scalar read; the buckets' own traffic is per bucket, not per term
            dom_bytes = 17 * (104 + 8) + 32
            value = n_global * args.steps / elapsed
            metric, unit = "G1 multi-scalar multiplication terms per second at n = 2^20", "terms/s"
            config = {"workload": "one G1 MSM sum_i s_i P_i over 2^20 distinct affine bases (Pippenger, c = 16)",
                      "batch_per_gpu": n, "global_batch": n_global, "kernel_ms": {"multiexp": round(dom_ms, 3)}}
        elif args.workload == "verify":
            dom_name, dom_ms, dom_bytes = "multi_pairing", float(np.mean(k_ms["a"])), 304 * n + 577
            value = dom_ms
            metric, unit = "multi_pairing latency, %d pairs (verifier shape)" % n, "ms"
            config = {"workload": "final_exponentiation(miller_loop([(P_i, Q_i)])) over %d pairs, inputs in HBM, "
                                  "cooperative kernels (quad VM: four waves per pairing, four lanes per Fq value)" % n,
                      "batch_per_gpu": n, "global_batch": n * ws, "kernel_ms": {"multi_pairing": round(dom_ms, 3)}}
            if args.decode:
                dec_ms = float(np.mean(k_ms["b"]))
                metric = "decode + multi_pairing latency, %d pairs (verifier shape from compressed points)" % n
                if split:
                    config["workload"] = ("G1Compressed / G2Compressed into_affine (checked) of %d + %d points as "
                                          "into_affine_unchecked (G1 beside G2 on two streams) + the subgroup checks, "
                                          "which run beside the pairing: " % (n, n)) + config["workload"]
                    config["kernel_ms"] = {"decode_unchecked": round(dec_ms, 3),
                                           "multi_pairing_and_checks": round(dom_ms - dec_ms, 3)}
                    for name, st, inn in (("G1", st1, in1), ("G2", st2, in2)):
                        if not (st.cpu().numpy() == 0).all() or not (inn.cpu().numpy() == 1).all():
                            raise SystemExit("verify: %s inputs did not decode as valid points" % name)
                else:
                    config["workload"] = ("G1Compressed / G2Compressed into_affine (checked) of %d + %d points, G1 "
                                          "beside G2 on two streams, then " % (n, n)) + config["workload"]
                    config["kernel_ms"] = {"decode": round(dec_ms, 3), "multi_pairing": round(dom_ms - dec_ms, 3)}
        elif args.workload == "fr_mul":
            dom_name, dom_ms, dom_bytes = "fr_mul_batch", float(np.mean(k_ms["a"])), 96
            value = n_global * args.steps / elapsed
            metric, unit = "Fr::mul_assign per second at batch 2^20", "muls/s"
            config = {"workload": "2^20 Fr Montgomery multiplications (AoS 4x u64)", "batch_per_gpu": n,
                      "global_batch": n_global}
        else:
            dom_name, dom_ms, dom_bytes = "fq_mul_batch", float(np.mean(k_ms["a"])), 144
            value = n_global * args.steps / elapsed
            metric, unit = "Fq::mul_assign per second at batch 2^20", "muls/s"
            config = {"workload": "2^20 Fq Montgomery multiplications (%s 6x u64)" % args.layout.upper(), "batch_per_gpu": n,
                      "global_batch": n_global}
        if dist_on and args.workload not in ("pairing", "prepared", "prepared_shared"):
            config["parallelism"] = ("shard%d+partial_sums_to_root" if args.workload == "msm" else
                                     "replicas%d" if args.workload == "verify" else "shard%d+rccl_gather") % ws
        achieved = dom_bytes * n / (dom_ms * 1e-3) / 1e9
        traffic, traffic_all = None, {}
        tr_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tr_path):
            with open(tr_path) as f:
                traffic_all = json.load(f)
            traffic = traffic_all.get(dom_name)
        roof = {"kernel": dom_name, "bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "bytes_per_unit": dom_bytes, "avg_launch_ms": round(dom_ms, 4)}
        if args.workload in ("fq_mul", "fr_mul"):
            # what a plain device copy of the same byte count reaches on this
            # box (read a,b / write out = 2 reads + 1 write; the copy moves
            # 1 read + 1 write per byte pair), for context next to the spec peak
            copy_gbs = measure_copy_gbs(dom_bytes * n, dev, stream)
            roof["copy_GBs"] = round(copy_gbs, 1)
            roof["frac_of_copy"] = achieved / copy_gbs
        work_path = os.path.join(ROOT, "pairing_amd", "lib", "pa_gen_work.json")
        if args.workload == "pairing" or (args.workload in ("prepared", "prepared_shared") and
                                          dom_name in ("final_exponentiation", "miller_loop_shared",
                                                       "miller_loop_prepared")):
            _check_work_json(work_path)
            # the pairing kernels are VALU-issue bound (multiply-accumulate
            # chains), not HBM bound: report that roofline, with the HBM view
            # kept alongside
            with open(work_path) as f:
                work = json.load(f)
            # the final exponentiation step is one generated kernel (round 3:
            # in-kernel binary-GCD inversions, compressed squarings).  The
            # binary GCD's instructions are counted, its 64-bit approximation
            # steps are not limb MACs.
            # which code objects ran: the lane-pair kernels' work per pairing (two
            # lanes) differs from the one-lane kernels'
            # (the prepared workloads' final exponentiation follows the same
            # selection, pairing_amd/csrc/capi.hip fe_launch; their Miller loops
            # are other kernels)
            lp = kernel_variant_label(n) == "gen2" and (args.workload == "pairing" or
                                                        dom_name == "final_exponentiation")
            wk = work["final_exp_lane_pairs" if lp else "final_exp"] if dom_name == "final_exponentiation" else \
                work[dom_name] if dom_name in ("miller_loop_shared", "miller_loop_prepared") else \
                work[("miller_loop_lane_pairs_pairing_only" if args.workload == "pairing" else
                      "miller_loop_lane_pairs") if lp else "miller_loop"]
            if lp:
                roof_kernel = {"final_exponentiation": "pa_gen_final_exp2",
                               "miller_loop_fused": "pa_gen_miller_loop2p"}.get(dom_name, dom_name)
                # the headline's Miller loop is the pairing-only code object (its own PMC entry)
                traffic = traffic_all.get(dom_name + "_lane_pairs" + (
                    "_pairing_only" if dom_name == "miller_loop_fused" and args.workload == "pairing" else ""))
            macs = wk["limb_macs"]
            mac_rate = macs * n / (dom_ms * 1e-3) / 1e12
            roof = {"kernel": dom_name, "bound": "valu", "achieved": round(mac_rate, 3),
                    "peak": round(VALU_MAC_PEAK_T, 3), "unit": "T limb-MAC/s (28x28-bit v_mad_u64_u32)",
                    "frac": mac_rate / VALU_MAC_PEAK_T, "traffic": traffic, "macs_per_unit": macs,
                    "avg_launch_ms": round(dom_ms, 4),
                    "hbm": {"achieved_GBs": round(achieved, 3), "peak_GBs": HBM_PEAK_GBS,
                            "bytes_per_unit": dom_bytes}}
            if lp:
                # the lane-pair code objects, two lanes per pairing, two waves per SIMD at 2^16
                roof["code_object"] = roof_kernel
                if args.workload == "pairing":
                    # PMC bytes per launch of both kernels of the step (profiles/pmc_traffic.json)
                    roof["traffic_by_kernel"] = {
                        "pa_gen_miller_loop2p": traffic_all.get("miller_loop_fused_lane_pairs_pairing_only"),
                        "pa_gen_final_exp2": traffic_all.get("final_exponentiation_lane_pairs")}
                roof["peak_two_waves_per_simd"] = VALU_MAC_2WAVE_T
                roof["frac_two_waves"] = mac_rate / VALU_MAC_2WAVE_T
            else:
                roof["peak_one_wave_per_simd"] = VALU_MAC_1WAVE_T
                roof["frac_one_wave"] = mac_rate / VALU_MAC_1WAVE_T
            instr = wk.get("instructions")
            if instr and not lp:
                rate = instr * n / (dom_ms * 1e-3) / 1e12
                roof["issue"] = {"achieved": round(rate, 3), "peak": round(ISSUE_PEAK_T, 3),
                                 "unit": "T lane-instructions/s (one wave per SIMD)", "frac": rate / ISSUE_PEAK_T,
                                 "instructions_per_unit": instr}
            elif instr:
                # lane pairs: instructions of both lanes per pairing; the issue
                # ceiling is the same one instruction per 4 clk per SIMD, but two
                # dense waves per SIMD hold the clock at ~2.15 GHz instead of
                # 2.33 (power cap, profiles/r05_coresidency.md)
                rate = instr * n / (dom_ms * 1e-3) / 1e12
                roof["issue"] = {"achieved": round(rate, 3), "peak": round(ISSUE_PEAK_T, 3),
                                 "unit": "T lane-instructions/s (any waves per SIMD, at 2.33 GHz)",
                                 "frac": rate / ISSUE_PEAK_T, "instructions_per_unit": instr,
                                 "peak_at_two_wave_clock": round(ISSUE_2WAVE_T, 3),
                                 "frac_at_two_wave_clock": rate / ISSUE_2WAVE_T}
        if args.workload == "wnaf" and dom_name == "g1_glv_comb_mul":
            # VALU bound: each mixed addition (madd-2007-bl, ec.rs:446-526) is
            # 7 products + 4 squarings on the lazy 28-bit core (fl_gen.h
            # leaves: 392 / 301 v_mad_u64_u32); a scalar takes
            # GLV split s = q x^2 + rem: 32.77 nonzero signed base-256 digits of
            # rem and q together on average for s uniform below r (simulated
            # over 2e4 scalars with kernels_curve.hip glv_split's arithmetic;
            # the plain 33-window comb: 31.88)
            macs = 32.77 * (7 * 392 + 4 * 301)
            mac_rate = macs * n / (dom_ms * 1e-3) / 1e12
            roof = {"kernel": dom_name, "bound": "valu", "achieved": round(mac_rate, 3),
                    "peak": round(VALU_MAC_PEAK_T, 3), "unit": "T limb-MAC/s (28x28-bit v_mad_u64_u32)",
                    "frac": mac_rate / VALU_MAC_PEAK_T, "traffic": traffic, "macs_per_unit": round(macs),
                    "avg_launch_ms": round(dom_ms, 4),
                    "hbm": {"achieved_GBs": round(achieved, 3), "peak_GBs": HBM_PEAK_GBS,
                            "bytes_per_unit": dom_bytes}}
        valu_path = os.path.join(ROOT, "profiles", "pmc_valu.json")
        if args.workload == "decode" and os.path.exists(valu_path):
            # VALU-issue bound (square roots = Fq exponentiations, the r*P check =
            # 63/126 doublings): one record per lane, so the wave's VALU
            # instruction count (SQ_INSTS_VALU / SQ_WAVES, profiles/pmc_valu.json,
            # a fixed function of the seeded batch) is the lane-instructions per
            # record; timed live here
            with open(valu_path) as f:
                ipr = json.load(f).get(dom_name, {}).get("valu_instructions_per_wave")
            if ipr:
                rate = ipr * n / (dom_ms * 1e-3) / 1e12
                roof = {"kernel": dom_name, "bound": "valu_issue", "achieved": round(rate, 3),
                        "peak": round(ISSUE_PEAK_T, 3), "unit": "T lane-instructions/s (VALU, 1 per 4 clk per SIMD)",
                        "frac": rate / ISSUE_PEAK_T, "traffic": traffic, "instructions_per_unit": ipr,
                        "avg_launch_ms": round(dom_ms, 4),
                        "hbm": {"achieved_GBs": round(achieved, 3), "peak_GBs": HBM_PEAK_GBS,
                                "bytes_per_unit": dom_bytes}}
        if args.workload == "msm":
            # VALU view: every term enters W = 17 windows; each entry is one mixed
            # addition into a bucket (madd-2007-bl on the lazy core: 7 products + 4
            # squarings, 7 x 392 + 4 x 301 limb MACs); the bucket sums and Horner
            # steps are < 3 % on top and not counted
            macs = 17 * (7 * 392 + 4 * 301)
            mac_rate = macs * n / (dom_ms * 1e-3) / 1e12
            roof = {"kernel": "g1_multiexp (all its kernels)", "bound": "valu", "achieved": round(mac_rate, 3),
                    "peak": round(VALU_MAC_PEAK_T, 3), "unit": "T limb-MAC/s (28x28-bit v_mad_u64_u32)",
                    "frac": mac_rate / VALU_MAC_PEAK_T, "traffic": traffic, "macs_per_unit": macs,
                    "avg_launch_ms": round(dom_ms, 4),
                    "hbm": {"achieved_GBs": round(achieved, 3), "peak_GBs": HBM_PEAK_GBS, "bytes_per_unit": dom_bytes}}
        if args.workload == "verify":
            roof = {"kernel": "multi_pairing", "bound": "latency", "achieved": round(dom_ms, 4), "peak": None,
                    "unit": "ms", "frac": None, "traffic": None,
                    "note": "dependent product / linear-combination steps of the quad VM (DESIGN.md section 4, cooperative kernels)"}
        cpu = None
        if not args.no_cpu_baseline and ws == 1:
            if args.workload == "pairing":
                cpu = cpu_baseline_pairing(p_np, q_np, args.cpu_seconds)
            elif args.workload == "prepared":
                cpu = cpu_baseline_prepared(p_np, q_np, args.cpu_seconds)
            elif args.workload == "prepared_shared":
                cpu = cpu_baseline_prepared_shared(p_np, prep1_np, args.cpu_seconds)
            elif args.workload == "wnaf":
                cpu = cpu_baseline_wnaf(base_np, s_np, args.cpu_seconds)
            elif args.workload == "decode":
                cpu = cpu_baseline_decode(enc1_np, enc2_np, args.cpu_seconds)
            elif args.workload == "msm":
                cpu = cpu_baseline_msm(base_np, k_np, s_np, args.cpu_seconds)
            elif args.workload == "fr_mul":
                cpu = cpu_baseline_fr_mul(a_np, b_np)
            elif args.workload == "verify":
                from oracle import binding as oracle
                t0 = time.perf_counter()
                reps = 20
                for _ in range(reps):
                    pp, qq = p_np, q_np
                    if args.decode:
                        pp, _ = oracle.decode(1, enc1_np, True, True, 1)
                        qq, _ = oracle.decode(2, enc2_np, True, True, 1)
                    f = oracle.miller_loop(pp, oracle.g2_prepare(qq))
                    oracle.final_exponentiation(f[None, :].copy())
                cpu = {"value": (time.perf_counter() - t0) / reps * 1e3, "unit": "ms", "cores": 1, "kind": "port",
                       "sample": "%d x %smulti_pairing of the same %d pairs, C restatement (oracle/), 1 thread"
                                 % (reps, "decode (checked) + " if args.decode else "", n)}
            else:
                cpu = cpu_baseline_fq_mul(a_np, b_np, args.cpu_seconds)
        line = {"metric": metric, "value": value, "unit": unit, "n_gpus": ws, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": args.workload != "verify",
                "scaling": "strong" if args.global_batch else "weak", "vs_baseline": None,
                "dtype": "u32 (14 x 28-bit lazy Montgomery limbs)"
                if args.workload in ("pairing", "prepared", "prepared_shared", "verify", "fq_mul")
                else "u32 (256-bit Montgomery, 8 x u32 limbs)" if args.workload == "fr_mul"
                else "u32 (14 x 28-bit lazy Montgomery limbs; 12 x u32 normalize)" if args.workload == "wnaf"
                else "u32 (384-bit Montgomery, 12 x u32 limbs)",
                "data": "synthetic (seeded random points k*G)", "config": config,
                "roofline": roof, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
