"""The multi-rank path (pairing_amd/shard.py) with world_size 2 on CPU (gloo):
sharded batch == unsharded batch, sharded multi-pair product == single
product, ragged shards handled.  The per-rank compute is the oracle here
(CPU); on MI355X the same code runs with RCCL and the HIP kernels
(bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pairing_amd.shard import shard_range


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 64, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    from oracle import binding as oracle
    from pairing_amd.shard import sharded_batch, sharded_product

    d = np.load(os.path.join(root, "tests", "golden", "bench_points.npz"))
    p = torch.from_numpy(d["g1"][:n].view(np.int64).copy())
    q = torch.from_numpy(d["g2"][:n].view(np.int64).copy())

    def compute(ps, qs):
        out = oracle.pairing(ps.numpy().view(np.uint64), qs.numpy().view(np.uint64), 2)
        return torch.from_numpy(out.view(np.int64))

    def local_product(ps, qs):
        prep = oracle.g2_prepare(qs.numpy().view(np.uint64))
        f = oracle.miller_loop(ps.numpy().view(np.uint64).copy(), prep)
        return torch.from_numpy(f.reshape(1, 72).view(np.int64).copy())

    def combine(rows):
        acc = rows[0:1].numpy().view(np.uint64)
        for r in range(1, rows.shape[0]):
            acc = oracle.fq12_mul(acc, rows[r:r + 1].numpy().view(np.uint64).copy())
        return torch.from_numpy(acc.view(np.int64))

    out = sharded_batch(p, q, compute)
    prod = sharded_product(p, q, local_product, combine)
    if rank == 0:
        np.savez(result_path, out=out.numpy(), prod=prod.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [8, 11])  # even and ragged shards
def test_sharded_pairing_world2_gloo(tmp_path, oracle, n):
    world = 2
    path = str(tmp_path / "res.npz")
    mp.spawn(_worker, args=(world, _free_port(), n, path), nprocs=world, join=True)
    res = np.load(path)
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "bench_points.npz"))
    p, q = d["g1"][:n].copy(), d["g2"][:n].copy()
    np.testing.assert_array_equal(res["out"].view(np.uint64), oracle.pairing(p, q, 4))
    single = oracle.miller_loop(p, oracle.g2_prepare(q))
    np.testing.assert_array_equal(res["prod"].view(np.uint64)[0], single)


def _hip_worker(rank, world, port, n, result_path):
    """Per-rank compute through the HIP C ABI (pairing_amd): each rank pairs its
    shard and reduces its shard's Miller loops to one Fq12 on the GPU; the
    exchange is gloo here (both ranks share the box's one GPU; RCCL needs a
    device per rank, bench.py --gpus N uses it)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import pairing_amd
    from pairing_amd.shard import sharded_batch, sharded_product

    pairing_amd.set_device(0)
    d = np.load(os.path.join(root, "tests", "golden", "bench_points.npz"))
    p = torch.from_numpy(d["g1"][:n].view(np.int64).copy())
    q = torch.from_numpy(d["g2"][:n].view(np.int64).copy())

    def compute(ps, qs):
        out = pairing_amd.pairing(ps.numpy().view(np.uint64), qs.numpy().view(np.uint64))
        return torch.from_numpy(out.view(np.int64))

    def local_product(ps, qs):
        f = pairing_amd.multi_miller_loop_affine(ps.numpy().view(np.uint64), qs.numpy().view(np.uint64))
        return torch.from_numpy(f.reshape(1, 72).view(np.int64).copy())

    def combine(rows):
        acc = rows[0:1].numpy().view(np.uint64).copy()
        for r in range(1, rows.shape[0]):
            acc = pairing_amd.fq12_mul(acc, rows[r:r + 1].numpy().view(np.uint64).copy())
        fe, ok = pairing_amd.final_exponentiation(acc)
        assert ok[0]
        return torch.from_numpy(np.concatenate([acc, fe], axis=0).view(np.int64))

    out = sharded_batch(p, q, compute)
    prod = sharded_product(p, q, local_product, combine)
    if rank == 0:
        np.savez(result_path, out=out.numpy(), prod=prod.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [64, 1000])  # even / ragged shards; the product runs on the cooperative path (<= 2304)
def test_sharded_pairing_world2_hip(tmp_path, oracle, n):
    # the parent never touches the GPU (the ranks do; a rank without a device raises)
    world = 2
    path = str(tmp_path / "res.npz")
    mp.spawn(_hip_worker, args=(world, _free_port(), n, path), nprocs=world, join=True)
    res = np.load(path)
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "bench_points.npz"))
    p, q = d["g1"][:n].copy(), d["g2"][:n].copy()
    np.testing.assert_array_equal(res["out"].view(np.uint64), oracle.pairing(p, q, 8))
    prod = res["prod"].view(np.uint64)
    single = oracle.miller_loop(p, oracle.g2_prepare(q))
    np.testing.assert_array_equal(prod[0], single)
    fe, ok = oracle.final_exponentiation(single.reshape(1, 72).copy())
    assert ok[0] == 1
    np.testing.assert_array_equal(prod[1], fe[0])


def _shard_from_worker(rank, world, path, n, out_path):
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(path[1]))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pairing_amd.shard import sharded_batch_from
    seen = []

    def load(a, b):        # each rank materializes only rows a..b
        seen.append((a, b))
        rows = np.arange(a, b, dtype=np.int64)[:, None] * np.ones((1, 3), np.int64)
        return torch.from_numpy(rows), torch.from_numpy(rows + 1)
    out = sharded_batch_from(load, n, lambda p, q: p + q)
    if rank == 0:
        np.save(out_path, out.numpy())
    dist.destroy_process_group()
    assert len(seen) == 1


def test_sharded_batch_from_stages_only_the_shard(tmp_path):
    """pairing_amd.shard.sharded_batch_from: every rank loads only its own
    contiguous rows (ragged world-3 split) and the root gathers all n"""
    import numpy as np
    import socket
    import torch.multiprocessing as mp
    sck = socket.socket()
    sck.bind(("127.0.0.1", 0))
    port = sck.getsockname()[1]
    sck.close()
    n = 11
    out_path = str(tmp_path / "out.npy")
    mp.spawn(_shard_from_worker, args=(3, ("x", port), n, out_path), nprocs=3, join=True)
    got = np.load(out_path)
    want = (2 * np.arange(n) + 1)[:, None] * np.ones((1, 3), np.int64)
    np.testing.assert_array_equal(got, want)


def _worker_other(rank, world, port, n, result_path):
    """Fq multiply batch, fixed-base scalar batch (scalars split, every rank
    its own table) and one multi-scalar multiplication (per-rank partial sums
    folded on the root) over a gloo group, oracle compute per rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    from oracle import binding as oracle
    from helpers import random_fq, random_scalars
    from pairing_amd.shard import sharded_batch_from, sharded_reduce

    g = np.random.default_rng(5)            # the same global batch on every rank
    a, b = random_fq(g, n), random_fq(g, n)
    s = random_scalars(g, n)
    bases = oracle.g1_mul_generator(random_scalars(g, n))
    base = oracle.g1_mul_generator_jacobian(random_scalars(g, 1))
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.int64))      # noqa: E731
    u = lambda x: np.ascontiguousarray(x.numpy()).view(np.uint64)               # noqa: E731

    fq = sharded_batch_from(lambda i, j: (a[i:j], b[i:j]), n, lambda x, y: t(oracle.fq_mul(x, y)))
    wnaf = sharded_batch_from(lambda i, j: (s[i:j],), n, lambda x: t(oracle.g1_wnaf_fixed_base(base, x)))

    def fold(rows):
        acc = u(rows[0:1])
        for r in range(1, rows.shape[0]):
            acc = oracle.g1_add(acc, u(rows[r:r + 1]))
        return t(acc)
    msm = sharded_reduce(lambda i, j: (bases[i:j], s[i:j]), n, lambda p, x: t(oracle.g1_multiexp(p, x)), fold)
    if rank == 0:
        np.savez(result_path, fq=fq.numpy(), wnaf=wnaf.numpy(), msm=msm.numpy(), a=a, b=b, s=s, bases=bases,
                 base=base)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [6, 9])  # even and ragged shards
def test_sharded_other_batches_world2_gloo(tmp_path, oracle, n):
    world = 2
    path = str(tmp_path / "other.npz")
    mp.spawn(_worker_other, args=(world, _free_port(), n, path), nprocs=world, join=True)
    r = np.load(path)
    u = lambda x: np.ascontiguousarray(x).view(np.uint64)                       # noqa: E731
    np.testing.assert_array_equal(u(r["fq"]), oracle.fq_mul(r["a"], r["b"]))
    # Wnaf::base(g, count) picks its window from the count (ec.rs:895-921), so a
    # shard's Jacobian words may differ from the whole batch's: equal as points
    assert oracle.g1_eq(u(r["wnaf"]), oracle.g1_wnaf_fixed_base(r["base"], r["s"])).all()
    assert oracle.g1_eq(u(r["msm"]), oracle.g1_multiexp(r["bases"], r["s"])).all()


def _gather_worker(rank, world, port, n_global, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pairing_amd.shard import RowGatherer
    a, b = shard_range(n_global, world, rank)
    outs = [torch.empty((b - a, 5), dtype=torch.int64) for _ in range(2)]
    g = RowGatherer(n_global, 5, outs[0])
    works, got = [None, None], []
    # the bench's pattern: batch k in slot k % 2, its gather asynchronous, the
    # slot rewritten only after its gather finished
    for k in range(5):
        slot = k % 2
        if works[slot] is not None:
            works[slot].wait()
            if rank == 0:
                got.append(g.result(slot).clone())
        outs[slot].copy_(torch.arange(a, b, dtype=torch.int64).view(-1, 1) * 10 + k)
        works[slot] = g.gather(outs[slot], slot)
    for slot in (1, 0):      # batches 3 and 4 still outstanding: 3 sits in slot 1
        works[slot].wait()
        if rank == 0:
            got.append(g.result(slot).clone())
    if rank == 0:
        torch.save(torch.stack(got), result_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_global", [8, 7])
def test_row_gatherer_async_double_buffered(tmp_path, n_global):
    """bench.py's multi-GPU pairing step: double-buffered results, each batch's
    gather to rank 0 asynchronous (RowGatherer), ragged shards padded"""
    out = str(tmp_path / "g.pt")
    mp.spawn(_gather_worker, args=(2, _free_port(), n_global, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    rows = torch.arange(n_global, dtype=torch.int64).view(-1, 1) * 10
    for k in range(5):
        assert torch.equal(got[k], (rows + k).expand(-1, 5)), k
