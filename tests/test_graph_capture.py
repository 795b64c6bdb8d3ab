"""pa_pairing_batch_device captured into a HIP graph (torch.cuda.CUDAGraph on
a side stream, relaxed capture mode) and replayed on new inputs written into
the captured buffers: the replay's pairings equal the oracle's (lib.rs:101-109)
for each default regime -- the quad VM, the lane groups, the split range
(capture runs it without the forked tail: capi.hip split_head) and lane pairs.
The first call runs outside the capture so the generated kernels' workspace
exists before it (gen_launch.hip acquire); a code object first loaded inside
the capture reads its workspace symbol on the library's own non-blocking
stream (gen_launch.hip load), which leaves the capture intact."""
import numpy as np
import pytest

from test_bench_sizes import _dev, _host, _threads

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [64, 2048, 32769, 65536])
def test_pairing_batch_replays_from_a_graph(gpu, oracle, n):
    import torch
    import bench
    import pairing_amd.device as pdev
    p1, q1 = bench.make_pairs(n, 0, seed=51)
    p2, q2 = bench.make_pairs(n, 0, seed=52)
    P, Qd = _dev(p1), _dev(q1)
    out = pdev.empty_records(n, 72, "cuda:0")
    scratch = pdev.empty_records(n, 72, "cuda:0")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        pdev.pairing(P, Qd, out, scratch)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
        pdev.pairing(P, Qd, out, scratch)
    torch.cuda.synchronize()
    P.copy_(_dev(p2))
    Qd.copy_(_dev(q2))
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), oracle.pairing(p2, q2, _threads()))
    # and the library keeps working outside the graph (the workspace pool's events)
    P.copy_(_dev(p1))
    Qd.copy_(_dev(q1))
    pdev.pairing(P, Qd, out, scratch)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(out), oracle.pairing(p1, q1, _threads()))
