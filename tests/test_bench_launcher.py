"""bench.py --gpus N run directly (no WORLD_SIZE): it must start N ranks
itself through torch.distributed.run and report n_gpus = N with the shard +
gather parallelism.  Exercised on the CPU with --cpu-stub (gloo ranks, the
oracle as each rank's compute); the GPU path shares launch_ranks, dist_env
and the rank/shard/gather structure."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_bench_gpus2_launches_two_ranks():
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "6", "--cpu-stub"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout          # rank 0 prints one line
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == "shard2+gather"
    assert line["config"]["global_batch"] == 12
    assert line["value"] > 0 and line["steps"] == 2


def test_bench_gpus1_runs_in_process():
    r = _run(["--gpus", "1", "--steps", "1", "--warmup", "0", "--batch", "4", "--cpu-stub"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_lines(r.stdout)[0]
    assert line["n_gpus"] == 1 and line["config"]["parallelism"] == "single"


def test_bench_fails_when_fewer_devices_than_gpus():
    import torch
    n = torch.cuda.device_count() + 1
    r = _run(["--gpus", str(max(n, 2)), "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2
    assert "visible" in r.stderr


def test_bench_config5_shape_global_batch():
    """BASELINE config 5 (2^20 pairings over 8 GPUs) as the launcher runs it:
    `bench.py --gpus 8 --global-batch 1048576` starts 8 ranks, each builds
    only its 2^17-row shard (make_pairs(span=...)), and the root gathers all
    2^20 result rows (checked inside the stub).  Here with gloo ranks that echo
    their shard instead of computing pairings (plumbing only)."""
    r = _run(["--gpus", "8", "--steps", "1", "--warmup", "0", "--global-batch", str(1 << 20),
              "--cpu-stub", "--stub-echo"], timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_lines(r.stdout)[0]
    assert line["n_gpus"] == 8
    assert line["config"]["global_batch"] == 1 << 20
    assert line["config"]["batch_per_gpu"] == 1 << 17
    assert line["config"]["parallelism"] == "shard8+gather"


def test_bench_global_batch_ragged_shards():
    """a global batch that does not divide: shards differ by one row, the
    root still gathers exactly the global batch (oracle compute, 2 ranks)"""
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--global-batch", "7", "--cpu-stub"])
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_lines(r.stdout)[0]
    assert line["config"]["global_batch"] == 7 and line["config"]["batch_per_gpu"] == 4


def test_kernel_variant_label_follows_the_default_selection(monkeypatch):
    """bench.kernel_variant_label mirrors capi.hip's default selection (lane groups
    in (768, 4096], the quad VM below, lane pairs, split batches up to 34816 with
    the quad VM tail up to 832 tail pairs and the lane groups above) and the
    PA_PAIRING_KERNEL / PA_TAIL_KIND overrides"""
    sys.path.insert(0, ROOT)
    import bench
    for k in ("PA_PAIRING_KERNEL", "PA_PQ_MIN", "PA_PQ_MAX", "PA_COOP_MAX", "PA_PAIR_MAX",
              "PA_TAIL_MAX", "PA_TAIL_KIND", "PA_ONE_MAX"):
        monkeypatch.delenv(k, raising=False)
    want = {1: "coop", 768: "coop", 769: "lane_groups", 4096: "lane_groups", 4097: "gen2",
            32768: "gen2", 32769: "gen2+coop_tail", 33600: "gen2+coop_tail",
            33601: "gen2+lane_group_tail", 34816: "gen2+lane_group_tail", 34817: "gen2", 65536: "gen2"}
    assert {n: bench.kernel_variant_label(n) for n in want} == want
    monkeypatch.setenv("PA_TAIL_KIND", "pq")
    assert bench.kernel_variant_label(32769) == "gen2+lane_group_tail"
    monkeypatch.setenv("PA_PAIRING_KERNEL", "5")
    assert bench.kernel_variant_label(65536) == "lane_groups"
