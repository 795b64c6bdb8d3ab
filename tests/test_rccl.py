"""The sharded path of SURVEY.md section 8(e) on the GPU: pairing_amd/shard.py
over an RCCL ("nccl") process group with the HIP pairing kernels as the
per-rank compute.  The boxes this build gets have one MI355X, so the group
has one rank; the collective (dist.gather to the root) and the shard
arithmetic are the same code the 8-GPU bench runs.  tests/test_distributed.py
covers world size 2 with gloo on the CPU."""
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_sharded_batch_over_rccl_matches_oracle(gpu, oracle):
    import torch
    import torch.distributed as dist
    import bench
    import pairing_amd.device as pdev
    from pairing_amd.shard import sharded_batch

    n = 2048 + 5
    p_np, q_np = bench.make_pairs(n, 0, seed=23)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(),
                            rank=0, world_size=1, device_id=dev)
    try:
        p = torch.from_numpy(p_np.view(np.int64)).to(dev)
        q = torch.from_numpy(q_np.view(np.int64)).to(dev)

        def compute(ps, qs):
            out = pdev.empty_records(ps.shape[0], 72, dev)
            scratch = pdev.empty_records(ps.shape[0], 72, dev)
            pdev.pairing(ps.contiguous(), qs.contiguous(), out, scratch)
            return out

        got = sharded_batch(p, q, compute)
        torch.cuda.synchronize()
        assert dist.get_backend() == "nccl"
    finally:
        dist.destroy_process_group()
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint64), oracle.pairing(p_np, q_np, 8))
