"""Verifier shape (2-pair multi_pairing, device-resident) issued directly vs
replayed from a HIP graph (relaxed capture): per-call latency with HIP events
around each call, synchronized every iteration.  Checks the replay's result
against the direct call's.  Usage: python tools/graph_verify.py [n_pairs] [iters]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import pairing_amd.device as pdev  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda:0")
    p_np, q_np = bench.make_pairs(n, 0, seed=3)
    p = torch.from_numpy(p_np.view(np.int64)).to(dev)
    q = torch.from_numpy(q_np.view(np.int64)).to(dev)
    out = pdev.empty_records(1, 72, dev)
    ok = torch.empty(1, dtype=torch.uint8, device=dev)
    work = pdev.empty_records(n, 72, dev)
    s = torch.cuda.Stream(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        ts = []
        for i in range(iters + 10):
            a.record(s)
            fn()
            b.record(s)
            b.synchronize()
            if i >= 10:
                ts.append(a.elapsed_time(b))
        return float(np.median(ts)), float(np.min(ts))

    call = lambda: pdev.multi_pairing(p, q, out, ok, work, s)
    med_d, min_d = timed(call)
    want = out.cpu().numpy().copy()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
        call()
    torch.cuda.synchronize()
    out.zero_()
    with torch.cuda.stream(s):
        med_g, min_g = timed(g.replay)
    same = np.array_equal(out.cpu().numpy(), want) and int(ok.item()) == 1
    print("multi_pairing n=%d: direct median %.3f ms (min %.3f); graph replay median %.3f ms (min %.3f); "
          "replay result == direct: %s" % (n, med_d, min_d, med_g, min_g, same))


if __name__ == "__main__":
    main()
